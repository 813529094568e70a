"""ORACLE — test infrastructure only, never the product path.

A plain-PyTorch fp32 CPU restatement of the reference's 3D ResNet-50
(`resnet50-3d-video/video_classifier/models/resnet3d.py:4-48`: pytorchvideo
`create_resnet(model_depth=50, model_num_class=2, dropout_rate=0.5, stem (3,7,7)/(1,2,2),
MaxPool3d (1,3,3)/(1,2,2), conv_a kernels ((1,1,1),(1,1,1),(3,1,1),(3,1,1)), conv_b (1,3,3),
spatial strides (1,2,2,2), head AvgPool3d (4,7,7) + global average)`), in eval mode
(BatchNorm with running statistics, dropout off) or, with `training=True`, in training mode
(BatchNorm with batch statistics, the running statistics updated in place with momentum 0.1,
as nn.BatchNorm3d.train(); the head's Dropout as an explicit keep-scale mask `head_keep`
[B, T_pooled, C], None = dropout off).

PARITY UNPINNED: pytorchvideo is not installed in this image and its source is nowhere on
disk; the reference does not pin its version.  This follows pytorchvideo's
published `pytorchvideo/models/resnet.py` / `stem.py` / `head.py`:

  stem: Conv3d(3, 64, (3,7,7), stride (1,2,2), padding (1,3,3), bias=False) -> BN -> ReLU ->
        MaxPool3d((1,3,3), stride (1,2,2), padding (0,1,1))
  stages (3,4,6,3) of bottleneck ResBlocks, dim_inner = dim_out / 4, dim_out 256..2048:
        branch2: conv_a (kernel, padding k//2) -> BN -> ReLU -> conv_b (1,3,3), stride
        (1,s,s) on the stage's first block, padding (0,1,1) -> BN -> ReLU -> conv_c 1x1x1 -> BN;
        branch1 (first block, dim_in != dim_out): Conv3d 1x1x1 with stride (1,s,s) -> BN;
        out = ReLU(branch1(x) + branch2(x));
  head: AvgPool3d((4,7,7), stride 1) -> Dropout (eval: identity) -> Linear over channels at
        every pooled position -> AdaptiveAvgPool3d(1) -> flatten.
BatchNorm eps 1e-5.  Parameter names follow pytorchvideo's `Net` (blocks.0.conv / .norm,
blocks.{1..4}.res_blocks.{i}.branch1_conv / branch1_norm / branch2.conv_{a,b,c} / norm_{a,b,c},
blocks.5.proj).

Allowed importers: tests/, __graft_entry__.smoke(), bench.py's cpu_baseline leg.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

RESNET3D_50 = dict(depths=(3, 4, 6, 3), stem_dim=64, conv_a_kernels=((1, 1, 1), (1, 1, 1), (3, 1, 1), (3, 1, 1)),
                   spatial_strides=(1, 2, 2, 2), head_pool=(4, 7, 7), num_classes=2, bn_eps=1e-5)


def _bn(x, p, pre, eps, training=False):
    return F.batch_norm(x, p[pre + ".running_mean"], p[pre + ".running_var"], p[pre + ".weight"], p[pre + ".bias"],
                        training=training, momentum=0.1, eps=eps)


def resnet3d_forward(p: dict, cfg: dict, video: torch.Tensor, return_stages: bool = False, training: bool = False,
                     head_keep=None, rounding=None):
    """p: pytorchvideo-named fp32 tensors; video [B, 3, T, H, W] -> logits [B, num_classes].

    `rounding` (tests only): optional dict of callables {"act", "weight", "conv_out"} applied to
    every stored activation, every conv weight and every conv output, so a test can restate the
    storage precisions of a bf16 implementation on this same graph (identity when None)."""
    eps = cfg.get("bn_eps", 1e-5)
    ident = lambda t: t  # noqa: E731
    r = rounding or {}
    ra, rw, ro = r.get("act", ident), r.get("weight", ident), r.get("conv_out", ident)
    bnf = lambda x, p, pre, eps: _bn(x, p, pre, eps, training)  # noqa: E731

    def conv(x, name, **kw):
        return ro(F.conv3d(x, rw(p[name]), **kw))

    x = conv(ra(video), "blocks.0.conv.weight", stride=(1, 2, 2), padding=(1, 3, 3))
    x = ra(F.relu(bnf(x, p, "blocks.0.norm", eps)))
    x = F.max_pool3d(x, kernel_size=(1, 3, 3), stride=(1, 2, 2), padding=(0, 1, 1))
    stages = [x]
    for s, depth in enumerate(cfg["depths"]):
        ka = cfg["conv_a_kernels"][s]
        ss = cfg["spatial_strides"][s]
        for i in range(depth):
            pre = f"blocks.{s + 1}.res_blocks.{i}."
            stride = (1, ss, ss) if i == 0 else (1, 1, 1)
            if pre + "branch1_conv.weight" in p:
                sc = ra(bnf(conv(x, pre + "branch1_conv.weight", stride=stride), p, pre + "branch1_norm", eps))
            else:
                sc = x
            y = conv(x, pre + "branch2.conv_a.weight", padding=tuple(k // 2 for k in ka))
            y = ra(F.relu(bnf(y, p, pre + "branch2.norm_a", eps)))
            y = conv(y, pre + "branch2.conv_b.weight", stride=stride, padding=(0, 1, 1))
            y = ra(F.relu(bnf(y, p, pre + "branch2.norm_b", eps)))
            y = bnf(conv(y, pre + "branch2.conv_c.weight"), p, pre + "branch2.norm_c", eps)
            x = ra(F.relu(sc + y))
        stages.append(x)
    x = F.avg_pool3d(x, kernel_size=cfg["head_pool"], stride=1)
    if head_keep is not None:  # Dropout: keep-scale per (clip, pooled position, channel)
        x = x * head_keep.permute(0, 2, 1).reshape(x.shape[0], x.shape[1], x.shape[2], 1, 1)
    x = x.permute(0, 2, 3, 4, 1) @ p["blocks.5.proj.weight"].T + p["blocks.5.proj.bias"]
    logits = x.mean(dim=(1, 2, 3))
    if return_stages:
        return logits, stages
    return logits
