"""ORACLE — test infrastructure only, never the product path.

A plain-PyTorch fp32 CPU restatement of the reference's ResNet50-LSTM
(`resnet50-2d-lstm/src/models/model.py:5-60`, `VideoResNet50LSTM(hidden_size=256,
num_layers=2, dropout=0.5)`), eval mode:

  per frame: torchvision ResNet-50 v1.5 without fc (conv1 7x7/2 -> BN -> ReLU -> MaxPool 3x3/2,
    layer1..4 of Bottlenecks (stride on the 3x3 conv, downsample 1x1 + BN on each layer's
    first block), AdaptiveAvgPool2d(1)) -> 2048 features;
  nn.LSTM(2048, 256, num_layers=2, batch_first=True) over the T frames (torch's own module:
    the reference's arithmetic), last step -> Linear(256,64) -> ReLU -> Dropout -> Linear(64,1).

PARITY: the ResNet-50 part is UNPINNED (torchvision absent: restated from its published
`torchvision/models/resnet.py`); the LSTM and classifier run torch's own modules.

Allowed importers: tests/, __graft_entry__.smoke(), bench.py's cpu_baseline leg.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def _bn(x, p, pre, eps=1e-5):
    return F.batch_norm(x, p[pre + ".running_mean"], p[pre + ".running_var"], p[pre + ".weight"], p[pre + ".bias"],
                        training=False, eps=eps)


def resnet50_features(p: dict, x: torch.Tensor) -> torch.Tensor:
    """x [N, 3, H, W] -> [N, 2048] (torchvision resnet50 minus fc, keys 'resnet50.<child>...')."""
    x = F.conv2d(x, p["resnet50.0.weight"], stride=2, padding=3)
    x = F.relu(_bn(x, p, "resnet50.1"))
    x = F.max_pool2d(x, 3, 2, 1)
    for li, depth in enumerate((3, 4, 6, 3)):
        for i in range(depth):
            pre = f"resnet50.{li + 4}.{i}."
            stride = 2 if (i == 0 and li > 0) else 1
            idt = x
            if pre + "downsample.0.weight" in p:
                idt = _bn(F.conv2d(x, p[pre + "downsample.0.weight"], stride=stride), p, pre + "downsample.1")
            y = F.relu(_bn(F.conv2d(x, p[pre + "conv1.weight"]), p, pre + "bn1"))
            y = F.relu(_bn(F.conv2d(y, p[pre + "conv2.weight"], stride=stride, padding=1), p, pre + "bn2"))
            y = _bn(F.conv2d(y, p[pre + "conv3.weight"]), p, pre + "bn3")
            x = F.relu(y + idt)
    return x.mean(dim=(2, 3))


def lstm_forward(p: dict, video: torch.Tensor, hidden: int = 256, layers: int = 2, return_features: bool = False):
    """video [B, 3, T, H, W] -> logits [B, 1] (VideoResNet50LSTM.forward, model.py:36-60)."""
    B, C, T, H, W = video.shape
    x = video.permute(0, 2, 1, 3, 4).reshape(B * T, C, H, W)
    feats = resnet50_features(p, x).reshape(B, T, -1)
    lstm = torch.nn.LSTM(2048, hidden, num_layers=layers, batch_first=True)
    lstm.load_state_dict({k[len("lstm."):]: v for k, v in p.items() if k.startswith("lstm.")})
    lstm.eval()
    y, _ = lstm(feats)
    y = y[:, -1, :]
    y = F.relu(y @ p["classifier.0.weight"].T + p["classifier.0.bias"])
    logits = y @ p["classifier.3.weight"].T + p["classifier.3.bias"]
    if return_features:
        return logits, feats
    return logits
