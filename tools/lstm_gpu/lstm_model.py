"""[tools experiment, not the product library] ResNet50-LSTM video classifier on the libvclip.so kernels
plus the recurrence kernels of tools/lstm_gpu/liblstm.so (tools/lstm_gpu/build.py) — drop-in for
`VideoResNet50LSTM(hidden_size=256, num_layers=2, dropout=0.5)` of
resnet50-2d-lstm/src/models/model.py:5-60 (BASELINE configs[0] runs this on the CPU; here it
runs on the GPU): `model(f32[B, 3, T, H, W])` -> `f32[B, 1]`.

Per frame, torchvision's ResNet-50 (v1.5, fc removed) runs on the shared conv path
(resnet3d.ResNet3d with kt = 1 kernels, BatchNorm folded, channels-last bf16), then the
global average pool gives [B*T, 2048] bf16 features.  Each LSTM layer is one MFMA GEMM for
the input projections of all T steps (bias = b_ih + b_hh, f32 out) followed by the fp32
recurrence kernel; the last step's h goes through the 256 -> 64 -> 1 head.
State dict keys are the reference's (resnet50.<child>..., lstm.*, classifier.*).
"""
from __future__ import annotations

from collections import OrderedDict

import numpy as np
import torch

import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import vclip_amd  # noqa: E402,F401
from vclip_amd import ops  # noqa: E402
from vclip_amd.ops import _dev, _need, _p, _stream  # noqa: E402
from vclip_amd.resnet3d import ResNet3d, _ru  # noqa: E402
from vclip_amd.weights import RESNET50_2D, blocks_to_torchvision_resnet50, resnet50_lstm_param_shapes, \
    torchvision_resnet50_to_blocks


_LIB = None
LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "liblstm.so")


def _call(name, *args):
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: python tools/lstm_gpu/build.py")
        from vclip_amd import _lib
        _lib.load()  # the HIP runtime libvclip binds, first
        _LIB = ctypes.CDLL(LIB_PATH)
        _LIB.lstm_last_error.restype = ctypes.c_char_p
    args = [a if isinstance(a, (ctypes.c_void_p, ctypes.c_int64)) else ctypes.c_int64(a) if isinstance(a, int)
            else a for a in args]
    rc = getattr(_LIB, name)(*args)
    if rc != 0:
        raise RuntimeError(f"{name}: {_LIB.lstm_last_error().decode()}")


def global_avgpool(x: torch.Tensor, N: int, P: int, C: int, out: torch.Tensor) -> torch.Tensor:
    """out[n] = mean of rows n*P .. n*P+P-1 of x (bf16 channels-last) -> bf16."""
    _dev(x, out)
    _need(x.dtype == torch.bfloat16 and out.dtype == torch.bfloat16 and x.shape[0] >= N * P and x.shape[1] >= C and
          out.shape[0] >= N and out.shape[1] >= C and x.stride(1) == 1 and out.stride(1) == 1, "global_avgpool shapes")
    _call("vc_global_avgpool", _p(x), x.stride(0), N, P, C, _p(out), out.stride(0), _stream(x))
    return out


def lstm_recurrence(pre: torch.Tensor, B: int, T: int, hidden: int, w_hh: torch.Tensor, h_out: torch.Tensor,
                    h_last: torch.Tensor) -> torch.Tensor:
    _dev(pre, w_hh, h_out, h_last)
    _need(pre.dtype == torch.float32 and pre.shape[0] >= B * T and pre.shape[1] >= 4 * hidden and pre.stride(1) == 1,
          "lstm pre")
    _need(w_hh.dtype == torch.float32 and w_hh.is_contiguous() and tuple(w_hh.shape) == (4 * hidden, hidden), "lstm W_hh")
    _need(h_out.dtype == torch.bfloat16 and h_out.shape[0] >= B * T and h_out.shape[1] >= hidden, "lstm h_out")
    _need(h_last.dtype == torch.float32 and h_last.is_contiguous() and h_last.numel() >= B * hidden, "lstm h_last")
    _call("vc_lstm_recurrence", _p(pre), pre.stride(0), B, T, hidden, _p(w_hh), _p(h_out), h_out.stride(0),
              _p(h_last), _stream(pre))
    return h_last


def mlp_head(h: torch.Tensor, B: int, w1, b1, w2, b2, out: torch.Tensor) -> torch.Tensor:
    _dev(h, w1, b1, w2, b2, out)
    _need(all(t.dtype == torch.float32 and t.is_contiguous() for t in (h, w1, b1, w2, b2, out)), "mlp_head f32")
    _call("vc_mlp_head", _p(h), B, w1.shape[1], _p(w1), _p(b1), w1.shape[0], _p(w2), _p(b2), w2.shape[0], _p(out),
              _stream(h))
    return out



class VideoResNet50LSTM(torch.nn.Module):
    def __init__(self, hidden_size: int = 256, num_layers: int = 2, dropout: float = 0.5):
        super().__init__()
        self.hidden, self.layers = hidden_size, num_layers
        self.backbone = ResNet3d(RESNET50_2D)
        shapes = resnet50_lstm_param_shapes(hidden_size, num_layers)
        self._names = [n for n in shapes if not n.startswith("resnet50.")]
        self.params = torch.nn.ParameterDict()
        for n in self._names:
            self.params[n.replace(".", "__")] = torch.nn.Parameter(torch.zeros(shapes[n]), requires_grad=False)
        self._packed = None
        self._ws = {}

    def state_dict(self, *a, **k):
        out = OrderedDict()
        for n, v in self.backbone.state_dict().items():
            tv = blocks_to_torchvision_resnet50(n)
            out[tv] = v.squeeze(2) if v.dim() == 5 else v
        for n in self._names:
            out[n] = self.params[n.replace(".", "__")].detach()
        return out

    def load_state_dict(self, sd, strict: bool = True):
        sd = {k[len("module."):] if k.startswith("module.") else k: v for k, v in sd.items()}
        bb, rest = {}, {}
        for k, v in sd.items():
            if k.endswith("num_batches_tracked"):
                continue
            b = torchvision_resnet50_to_blocks(k)
            if b is not None:
                v = torch.as_tensor(np.asarray(v)) if not isinstance(v, torch.Tensor) else v
                bb[b] = v.unsqueeze(2) if v.dim() == 4 else v
            else:
                rest[k] = v
        m1, u1 = self.backbone.load_state_dict(bb, strict=strict)
        missing = [n for n in self._names if n not in rest]
        unexpected = [k for k in rest if k not in self._names]
        if strict and (missing or unexpected):
            raise KeyError(f"load_state_dict: missing={missing[:5]} unexpected={unexpected[:5]}")
        with torch.no_grad():
            for n in self._names:
                if n in rest:
                    v = rest[n]
                    v = torch.as_tensor(np.asarray(v)) if not isinstance(v, torch.Tensor) else v
                    self.params[n.replace(".", "__")].copy_(v.reshape(self.params[n.replace(".", "__")].shape))
        self._packed = None
        return m1 + missing, u1 + unexpected

    def _pack(self, device):
        if self._packed is not None and self._packed["device"] == device:
            return self._packed
        P = lambda n: self.params[n.replace(".", "__")].detach().to(device=device, dtype=torch.float32)  # noqa: E731
        pk = {"device": device, "layers": []}
        for l in range(self.layers):
            pk["layers"].append(dict(
                w_ih=P(f"lstm.weight_ih_l{l}").to(torch.bfloat16).contiguous(),
                b=(P(f"lstm.bias_ih_l{l}") + P(f"lstm.bias_hh_l{l}")).contiguous(),
                w_hh=P(f"lstm.weight_hh_l{l}").contiguous()))
        pk["head"] = [P(n).contiguous() for n in ("classifier.0.weight", "classifier.0.bias", "classifier.3.weight",
                                                   "classifier.3.bias")]
        self._packed = pk
        return pk

    @torch.no_grad()
    def forward(self, video: torch.Tensor) -> torch.Tensor:
        if video.device.type != "cuda":
            raise RuntimeError("VideoResNet50LSTM (vclip_amd) runs on the GPU only")
        x = video.contiguous().float() if video.dtype != torch.float32 else video.contiguous()
        return self.forward_logits(x)

    def forward_logits(self, video: torch.Tensor) -> torch.Tensor:
        B, C, T, H, W = video.shape
        pk = self._pack(video.device)
        x, _, (t, h, w), Cf, _ = self.backbone.forward_features(video)
        key = (B, T, str(video.device))
        if key not in self._ws:
            M = _ru(B * T, 256)
            dev = video.device
            self._ws = {key: dict(feat=torch.zeros(M, Cf, dtype=torch.bfloat16, device=dev),
                                  pre=torch.zeros(M, 4 * self.hidden, dtype=torch.float32, device=dev),
                                  hseq=torch.zeros(M, self.hidden, dtype=torch.bfloat16, device=dev),
                                  hlast=torch.zeros(B, self.hidden, dtype=torch.float32, device=dev),
                                  logits=torch.zeros(B, 1, dtype=torch.float32, device=dev))}
        ws = self._ws[key]
        # per-frame AdaptiveAvgPool2d(1): rows are ((b*T + t)*h + y)*w + x
        global_avgpool(x, B * T, h * w, Cf, ws["feat"])
        inp = ws["feat"]
        for L in pk["layers"]:
            ops.gemm(inp, L["w_ih"], L["b"], "bias_f32", ws["pre"])
            lstm_recurrence(ws["pre"], B, T, self.hidden, L["w_hh"], ws["hseq"], ws["hlast"])
            inp = ws["hseq"]
        w1, b1, w2, b2 = pk["head"]
        return mlp_head(ws["hlast"], B, w1, b1, w2, b2, ws["logits"])


def create_model(hidden_size=256, num_layers=2, dropout=0.5, device="cuda", weights_seed: int = 0):
    """VideoResNet50LSTM with seeded synthetic weights (the reference loads torchvision's
    IMAGENET1K_V1 ResNet-50, unavailable offline)."""
    from vclip_amd.weights import make_resnet50_lstm_weights
    m = VideoResNet50LSTM(hidden_size, num_layers, dropout)
    m.load_state_dict(make_resnet50_lstm_weights(seed=weights_seed, hidden=hidden_size))
    return m.to(device) if device else m
