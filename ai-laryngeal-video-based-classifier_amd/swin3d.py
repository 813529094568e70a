"""Video Swin Transformer (torchvision `swin3d_t/s/b` as the reference builds it) on the
libvclip.so kernels — drop-in for `create_model(logger, model_size, pretrained, num_classes)`
of videoswintransformer/swin_video_classifier/models/swin3d.py:7-53, which returns the
torchvision model with `head` replaced by `Linear(768, num_classes)` and is called as
`model(f32[B, 3, T, H, W])` -> `f32[B, num_classes]` (trainer.py:116, inference.py).

Device data layout per stage s (C_s = 96 * 2^s channels, heads_s = C_s / 32):
  tokens in torchvision's channels-last order rows ((b*T + t)*H + h)*W + w, padded to a
  multiple of 256 rows; feature columns padded to a multiple of 128 (Cp) with zero weights,
  so padded columns stay exactly 0 through every GEMM (the GEMM tiles need N % 128, K % 64);
  residual X f32 [M, Cp]; LN output / attention output bf16 [M, Cp]; fused q|k|v bf16;
  MLP hidden bf16 [M, roundup(4C, 128)].
Per block: LN1 -> qkv GEMM (q pre-scaled by d^-1/2 * log2 e) -> shifted-window attention
(gather/scatter by index: no roll / partition copies; bias + shift mask inside) -> proj
GEMM + residual -> LN2 -> fc1 + exact GELU -> fc2 + residual.  Between stages: fused
PatchMerging gather + LN(4C), then the reduction GEMM into the next stage's residual.
Relative-position bias tables are expanded once per (block, window) into the attention
kernel's accumulator fragment order (f32, log2 e scaled, -inf on padded keys).

Parity unpinned against torchvision itself (not installed here): checked against
oracle/swin3d_ref.py, the restatement of torchvision's algorithm.
"""
from __future__ import annotations

import math
from collections import OrderedDict

import numpy as np
import torch

from . import ops, streams
from .weights import swin3d_param_shapes

LOG2E = ops.LOG2E

SWIN3D_CONFIGS = {
    # stochastic_depth_prob (train-time only): torchvision models/video/swin_transformer.py builds
    # swin3d_t, swin3d_s and swin3d_b each with stochastic_depth_prob=0.1 (the 2-D swin_t/s/b use
    # 0.2/0.3/0.5); torchvision is absent from this image, so the value is parity-unpinned
    "tiny": dict(patch_size=(2, 4, 4), embed_dim=96, depths=(2, 2, 6, 2), num_heads=(3, 6, 12, 24),
                 window_size=(8, 7, 7), mlp_ratio=4.0, layer_norm_eps=1e-5, stochastic_depth_prob=0.1),
    "small": dict(patch_size=(2, 4, 4), embed_dim=96, depths=(2, 2, 18, 2), num_heads=(3, 6, 12, 24),
                  window_size=(8, 7, 7), mlp_ratio=4.0, layer_norm_eps=1e-5, stochastic_depth_prob=0.1),
    "base": dict(patch_size=(2, 4, 4), embed_dim=128, depths=(2, 2, 18, 2), num_heads=(4, 8, 16, 32),
                 window_size=(8, 7, 7), mlp_ratio=4.0, layer_norm_eps=1e-5, stochastic_depth_prob=0.1),
}
SWIN3D_CONFIGS["base_in22k"] = SWIN3D_CONFIGS["base"]


def _ru(x, m):
    return (x + m - 1) // m * m


def relative_position_index(window_size):
    """torchvision ShiftedWindowAttention3d.define_relative_position_index."""
    wt, wh, ww = window_size
    coords = torch.stack(torch.meshgrid(torch.arange(wt), torch.arange(wh), torch.arange(ww), indexing="ij"))
    cf = torch.flatten(coords, 1)
    rel = (cf[:, :, None] - cf[:, None, :]).permute(1, 2, 0).contiguous()
    rel[:, :, 0] += wt - 1
    rel[:, :, 1] += wh - 1
    rel[:, :, 2] += ww - 1
    rel[:, :, 0] *= (2 * wh - 1) * (2 * ww - 1)
    rel[:, :, 1] *= 2 * ww - 1
    return rel.sum(-1)


def window_and_shift(size_thw, window_size, shift_size):
    """torchvision _get_window_and_shift_size: clamp the window to the feature size (shift 0 there)."""
    w, s = list(window_size), list(shift_size)
    for i in range(3):
        if size_thw[i] <= w[i]:
            w[i] = size_thw[i]
            s[i] = 0
    return w, s


_BIAS_INDEX = {}


def _bias_gather_index(full_window, window, device):
    """Flat gather index of expand_bias's fragment order into the table extended by two rows:
    ntab (-inf: padded keys) and ntab + 1 (0: padded queries).  Built once per geometry."""
    key = (tuple(full_window), tuple(window), str(device))
    idx = _BIAS_INDEX.get(key)
    if idx is not None:
        return idx
    vol = window[0] * window[1] * window[2]
    npad = _ru(vol, 64)
    ntab = (2 * full_window[0] - 1) * (2 * full_window[1] - 1) * (2 * full_window[2] - 1)
    rel = relative_position_index(full_window)[:vol, :vol]  # [q, k]
    full = torch.full((npad, npad), ntab, dtype=torch.int64)  # [k, q]: padded keys -> -inf
    full[:, vol:] = ntab + 1                                  # padded queries -> 0
    full[:vol, :vol] = rel.t()
    ar = torch.arange
    qb, t, kb, lane, e = torch.meshgrid(ar(npad // 32), ar(npad // 64), ar(2), ar(64), ar(16), indexing="ij")
    k = t * 64 + kb * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5)
    q = qb * 32 + (lane & 31)
    idx = full[k, q].reshape(-1).to(device)
    _BIAS_INDEX[key] = idx
    return idx


def expand_bias(table, full_window, window, device):
    """Relative-position bias of one block in the kernel's fragment order.

    bias[h][q][k] = table[index_full[:vol,:vol]][q][k][h] (torchvision _get_relative_position_bias:
    the FULL window's index, sliced when the window shrinks), scaled by log2 e; -inf on padded
    keys k >= vol, 0 on padded queries.  Returned as f32 [heads, np/32, np/64, 2, 64, 16]:
    [h][qb][t][kb][lane][e] = bias[h][q = 32qb + lane%32][k = 64t + 32kb + (e&3) + 8(e>>2) + 4(lane//32)],
    i.e. each lane's 16 accumulator-layout values of a 32x32 S^T block are contiguous.  One gather
    per call from the table extended by a -inf and a 0 row (the index is built once per geometry)."""
    vol = window[0] * window[1] * window[2]
    npad = _ru(vol, 64)
    tab = table.to(device=device, dtype=torch.float32)
    heads = tab.shape[1]
    ext = torch.cat([tab * LOG2E, torch.tensor([[float("-inf")] * heads, [0.0] * heads], device=device)])
    g = ext.index_select(0, _bias_gather_index(full_window, window, device))  # [slots, heads]
    return g.t().contiguous().view(heads, npad // 32, npad // 64, 2, 64, 16)


_BIAS_MB_INDEX = {}
MB_MASKED = -16384.0  # padded keys in the matrix-pipe bias (exp2 -> 0; finite, as the identity MFMA needs)


def _bias_mb_gather_index(full_window, window, device):
    """Flat gather index of expand_bias_mb's operand-fragment order into the table extended by two
    rows: ntab (padded keys) and ntab + 1 (padded queries).  Built once per geometry."""
    key = (tuple(full_window), tuple(window), str(device))
    idx = _BIAS_MB_INDEX.get(key)
    if idx is not None:
        return idx
    vol = window[0] * window[1] * window[2]
    npad = _ru(vol, 64)
    ntab = (2 * full_window[0] - 1) * (2 * full_window[1] - 1) * (2 * full_window[2] - 1)
    rel = relative_position_index(full_window)[:vol, :vol]  # [q, k]
    full = torch.full((npad, npad), ntab, dtype=torch.int64)  # [k, q]: padded keys
    full[:, vol:] = ntab + 1                                  # padded queries
    full[:vol, :vol] = rel.t()
    ar = torch.arange
    qb, t, kb, s, lane, m = torch.meshgrid(ar(npad // 32), ar(npad // 64), ar(2), ar(2), ar(64), ar(8), indexing="ij")
    k = t * 64 + kb * 32 + s * 16 + 8 * (lane >> 5) + m
    q = qb * 32 + (lane & 31)
    idx = full[k, q].reshape(-1).to(device)
    _BIAS_MB_INDEX[key] = idx
    return idx


def expand_bias_mb(table, full_window, window, device):
    """Relative-position bias of one block as the fp16 B operand of the matrix-pipe bias
    (vc_window_attention3d_mb): [heads, np/32, np/64, 2, 2, 64, 8], element [h][qb][t][kb][s][lane][m]
    = log2 e * bias[h][q = 32qb + lane%32][k = 64t + 32kb + 16s + 8(lane//32) + m] (the same
    torchvision bias as expand_bias), MB_MASKED on padded keys, 0 on padded queries."""
    vol = window[0] * window[1] * window[2]
    npad = _ru(vol, 64)
    tab = table.to(device=device, dtype=torch.float32)
    heads = tab.shape[1]
    ext = torch.cat([tab * LOG2E, torch.tensor([[MB_MASKED] * heads, [0.0] * heads], device=device)])
    g = ext.index_select(0, _bias_mb_gather_index(full_window, window, device))  # [slots, heads]
    # fp16 (2^-12 relative; bf16 would round trained tables by ~1e-2 log2 units)
    return g.t().to(torch.float16).contiguous().view(heads, npad // 32, npad // 64, 2, 2, 64, 8)


class Swin3d(torch.nn.Module):
    """fp32 master parameters in torchvision naming; bf16 / fp32 packed device copies."""

    def __init__(self, cfg: dict, num_classes: int = 2):
        super().__init__()
        self.cfg = dict(cfg, num_classes=num_classes)
        self.num_classes = num_classes
        for h, C in zip(cfg["num_heads"], (cfg["embed_dim"] * 2 ** s for s in range(len(cfg["depths"])))):
            if C // h != 32:
                raise ValueError("libvclip window attention supports head_dim 32 only")
        shapes = swin3d_param_shapes(self.cfg)
        self._names = list(shapes.keys())
        self.params = torch.nn.ParameterDict()
        for n, s in shapes.items():
            self.params[n.replace(".", "__")] = torch.nn.Parameter(torch.zeros(s))
        self._packed = None
        self._bias_cache = {}
        self._ws = {}
        self._ws_used = []
        self.kernel_events = None  # list: HIP events around each window-attention launch (bench.py)
        self.concurrent_streams = None  # n > 1: the inference batch split over n HIP streams
        self.split_sizes = None  # clips per stream part (streams.run_split); None = as even as possible
        self._streams = None
        self._split_out = {}
        # True: the inference forward is captured once per input / configuration into a hipGraph and
        # replayed (streams.GraphReplay); bit-identical logits
        self.graph_replay = False
        self._graphs = None
        self.stochastic_depth = True  # train step: torchvision's StochasticDepth on the residual branches

    def state_dict(self, *a, **k):
        return OrderedDict((n, self.params[n.replace(".", "__")].detach()) for n in self._names)

    def load_state_dict(self, sd, strict: bool = True):
        sd = {k[len("module."):] if k.startswith("module.") else k: v for k, v in sd.items()}
        sd = {k: v for k, v in sd.items() if not k.endswith("relative_position_index")}  # buffers, rebuilt
        missing = [n for n in self._names if n not in sd]
        unexpected = [k for k in sd if k not in self._names]
        if strict and (missing or unexpected):
            raise KeyError(f"load_state_dict: missing={missing[:5]} unexpected={unexpected[:5]}")
        with torch.no_grad():
            for n in self._names:
                if n in sd:
                    v = sd[n]
                    v = torch.as_tensor(np.asarray(v)) if not isinstance(v, torch.Tensor) else v
                    dst = self.params[n.replace(".", "__")]
                    dst.copy_(v.reshape(dst.shape))
        self._packed = None
        self._bias_cache = {}
        return missing, unexpected

    # ---- packing -------------------------------------------------------------------
    def P(self, name):
        return self.params[name.replace(".", "__")]

    def _weights_version(self):
        from . import vivit_train
        return (vivit_train.MASTER_EPOCH[0], sum(p._version for p in self.params.values()))

    def _pack(self, device):
        ver = self._weights_version()  # the fused AdamW updates in place without bumping _version
        if self._packed is not None and self._packed["device"] == device and self._packed["version"] == ver:
            return self._packed
        self._bias_cache = {}
        c = self.cfg
        bf, f32 = torch.bfloat16, torch.float32
        P = lambda n: self.params[n.replace(".", "__")].detach().to(device=device, dtype=f32)  # noqa: E731

        def padw(w, n_p, k_p, dt=bf):
            out = torch.zeros((n_p, k_p), dtype=f32, device=device)
            out[:w.shape[0], :w.shape[1]] = w
            return out.to(dt).contiguous()

        def padb(b, n_p):
            out = torch.zeros(n_p, dtype=f32, device=device)
            if b is not None:
                out[:b.numel()] = b
            return out

        pk = {"device": device, "version": ver}
        C0 = c["embed_dim"]
        pt, ph, pw = c["patch_size"]
        K0 = 3 * pt * ph * pw
        pk["K0p"] = _ru(K0, 64)
        pk["w_emb"] = padw(P("patch_embed.proj.weight").reshape(C0, K0), _ru(C0, 128), pk["K0p"])
        pk["b_emb"] = padb(P("patch_embed.proj.bias"), _ru(C0, 128))
        pk["ln_emb"] = (P("patch_embed.norm.weight").contiguous(), P("patch_embed.norm.bias").contiguous())
        stages = []
        for s, depth in enumerate(c["depths"]):
            C = C0 * 2 ** s
            Cp, hid = _ru(C, 128), int(C * c["mlp_ratio"])
            hp = _ru(hid, 128)
            qs = 32 ** -0.5 * LOG2E
            blocks = []
            for i in range(depth):
                p = f"features.{2 * s}.{i}."
                wq = P(p + "attn.qkv.weight").clone()
                bq = P(p + "attn.qkv.bias").clone()
                wq[:C] *= qs
                bq[:C] *= qs
                blocks.append(dict(
                    ln1=(P(p + "norm1.weight").contiguous(), P(p + "norm1.bias").contiguous()),
                    ln2=(P(p + "norm2.weight").contiguous(), P(p + "norm2.bias").contiguous()),
                    w_qkv=padw(wq, _ru(3 * C, 128), Cp), b_qkv=padb(bq, _ru(3 * C, 128)),
                    w_proj=padw(P(p + "attn.proj.weight"), Cp, Cp), b_proj=padb(P(p + "attn.proj.bias"), Cp),
                    w_1=padw(P(p + "mlp.0.weight"), hp, Cp), b_1=padb(P(p + "mlp.0.bias"), hp),
                    w_2=padw(P(p + "mlp.3.weight"), Cp, hp), b_2=padb(P(p + "mlp.3.bias"), Cp),
                    table=P(p + "attn.relative_position_bias_table").contiguous()))
            st = dict(C=C, Cp=Cp, hid=hid, hp=hp, heads=c["num_heads"][s], blocks=blocks)
            if s < len(c["depths"]) - 1:
                p = f"features.{2 * s + 1}."
                st["merge_ln"] = (P(p + "norm.weight").contiguous(), P(p + "norm.bias").contiguous())
                st["w_red"] = padw(P(p + "reduction.weight"), _ru(2 * C, 128), 4 * C)
                st["b_red"] = padb(None, _ru(2 * C, 128))
            stages.append(st)
        pk["stages"] = stages
        pk["norm"] = (P("norm.weight").contiguous(), P("norm.bias").contiguous())
        pk["w_head"] = P("head.weight").contiguous()
        pk["b_head"] = P("head.bias").contiguous()
        self._packed = pk
        return pk

    def _biasT(self, s, i, window, device):
        """Block (s, i)'s relative-position bias in the inference kernel's layout (expand_bias_mb:
        fp16 operand fragments of vc_window_attention3d_mb), built once per packed weights."""
        key = (s, i, tuple(window), str(device))
        if key not in self._bias_cache:
            tab = self._packed["stages"][s]["blocks"][i]["table"]
            self._bias_cache[key] = expand_bias_mb(tab, self.cfg["window_size"], window, device)
        return self._bias_cache[key]

    def geometry(self, B, T, H, W):
        c = self.cfg
        pt, ph, pw = c["patch_size"]
        if T % pt or H % ph or W % pw:
            raise ValueError("input T/H/W must be multiples of the patch size (2, 4, 4)")
        g = [(T // pt, H // ph, W // pw)]
        for _ in range(len(c["depths"]) - 1):
            t, h, w = g[-1]
            g.append((t, (h + 1) // 2, (w + 1) // 2))
        return g

    def _workspace(self, B, grids, device, part: int = 0):
        key = (B, tuple(grids), str(device), part)
        if key in self._ws:
            ws = self._ws[key]
            if not any(w is ws for w in self._ws_used):
                self._ws_used.append(ws)
            return ws
        if len(self._ws) >= 8:
            self._ws = {}
        c = self.cfg
        bf, f32 = torch.bfloat16, torch.float32
        z = lambda r, cols, dt=bf: torch.zeros((r, cols), dtype=dt, device=device)  # noqa: E731
        ws = {"stages": []}
        t0, h0, w0 = grids[0]
        M0 = _ru(B * t0 * h0 * w0, 256)
        ws["A_emb"] = z(M0, _ru(3 * 2 * 4 * 4, 64))
        ws["E"] = z(M0, _ru(c["embed_dim"], 128), f32)
        for s, (t, h, w) in enumerate(grids):
            C = c["embed_dim"] * 2 ** s
            Cp, hp = _ru(C, 128), _ru(int(C * c["mlp_ratio"]), 128)
            M = _ru(B * t * h * w, 256)
            st = dict(M=M, X=z(M, Cp, f32), Y=z(M, Cp), QKV=z(M, _ru(3 * C, 128)), O=z(M, Cp), Hd=z(M, hp))
            if s < len(grids) - 1:
                t2, h2, w2 = grids[s + 1]
                st["Mg"] = z(_ru(B * t2 * h2 * w2, 256), 4 * C)
            ws["stages"].append(st)
        ws["logits"] = torch.zeros((B, self.num_classes), dtype=f32, device=device)
        ws["pool_work"] = torch.zeros(B * 64 * c["embed_dim"] * 2 ** (len(grids) - 1), dtype=f32, device=device)
        self._ws[key] = ws
        self._ws_used.append(ws)
        return ws

    # ---- forward -------------------------------------------------------------------
    def forward(self, video: torch.Tensor) -> torch.Tensor:
        """`model(clips)` -> logits.  In training mode with autograd enabled (the reference's train
        loop, videoswintransformer/swin_video_classifier/trainers/trainer.py:105-122) the logits carry
        the graph of the HIP train step (_forward_train); otherwise the fused inference path runs."""
        if video.device.type != "cuda":
            raise RuntimeError("Swin3d (vclip_amd) runs on the GPU only: move the clip batch to cuda")
        x = video.contiguous().float() if video.dtype != torch.float32 else video.contiguous()
        if self.training and torch.is_grad_enabled():
            return self._forward_train(x)
        with torch.no_grad():
            return self.forward_logits(x).clone()  # the workspace buffer is reused by the next call

    def _forward_train(self, video: torch.Tensor) -> torch.Tensor:
        """torchvision's SwinTransformer3d forward (oracle/swin3d_ref.py) as autograd ops over the HIP
        kernels (vclip_amd/autograd_ops.py): bf16 MFMA GEMMs with fp32 accumulation on the fp32
        master weights, fp32 residual stream, exact GELU, the shifted-window attention with its
        relative-position bias table differentiable, the fused pool head; the token layout
        [B][T][H][W] rows throughout, PatchMerging's neighbour gather and the residual adds as torch
        layout glue.  Stochastic depth as torchvision's StochasticDepth(p_k, "row") on both residual
        branches of block k (p_k = stochastic_depth_prob * k / (blocks - 1); a per-clip keep mask
        from torch's RNG, scaled by 1 / (1 - p_k)); `self.stochastic_depth = False` turns it off."""
        from . import autograd_ops as A
        c = self.cfg
        B, Cin, T, H, W = video.shape
        if Cin != 3:
            raise ValueError("video must be [B, 3, T, H, W]")
        eps = c["layer_norm_eps"]
        pt, ph, pw = c["patch_size"]
        grids = self.geometry(B, T, H, W)
        t0, h0, w0 = grids[0]
        C0 = c["embed_dim"]
        M0 = B * t0 * h0 * w0
        K0 = 3 * pt * ph * pw
        a_emb = torch.zeros(_ru(M0, 256), _ru(K0, 64), dtype=torch.bfloat16, device=video.device)
        ops.tubelet_im2col(video, (pt, ph, pw), a_emb, layout="bcthw")
        e = A.linear(a_emb[:M0, :K0], self.P("patch_embed.proj.weight").reshape(C0, K0), self.P("patch_embed.proj.bias"),
                     out_f32=True)
        x = A.layer_norm(e, self.P("patch_embed.norm.weight"), self.P("patch_embed.norm.bias"), eps, out_bf16=False)
        full = tuple(c["window_size"])
        nblocks, k = sum(c["depths"]), 0
        sd = c.get("stochastic_depth_prob", 0.0) if self.stochastic_depth else 0.0

        def drop_path(y, prob):  # torchvision StochasticDepth(prob, "row") on a [B * ntok, C] branch output
            if prob <= 0.0:
                return y
            keep = torch.empty(B, 1, 1, device=y.device).bernoulli_(1.0 - prob).div_(1.0 - prob)
            return (y.reshape(B, -1, y.shape[-1]) * keep).reshape(y.shape)

        for s, depth in enumerate(c["depths"]):
            t, h, w = grids[s]
            C = C0 * 2 ** s
            heads = c["num_heads"][s]
            qs = 32 ** -0.5 * LOG2E
            for i in range(depth):
                p = f"features.{2 * s}.{i}."
                shift_full = [0 if i % 2 == 0 else wk // 2 for wk in full]
                window, shift = window_and_shift((t, h, w), full, shift_full)
                pk_ = sd * k / (nblocks - 1) if nblocks > 1 else 0.0
                k += 1
                y = A.layer_norm(x, self.P(p + "norm1.weight"), self.P(p + "norm1.bias"), eps)
                qkv = A.linear(y, self.P(p + "attn.qkv.weight"), self.P(p + "attn.qkv.bias"), qrows=C, qscale=qs)
                o = A.window_attention(qkv, self.P(p + "attn.relative_position_bias_table"), B, (t, h, w), heads,
                                       window, shift, full)
                x = x + drop_path(A.linear(o, self.P(p + "attn.proj.weight"), self.P(p + "attn.proj.bias"), out_f32=True),
                                  pk_)
                y = A.layer_norm(x, self.P(p + "norm2.weight"), self.P(p + "norm2.bias"), eps)
                hd = A.gelu_erf(A.linear(y, self.P(p + "mlp.0.weight"), self.P(p + "mlp.0.bias")))
                x = x + drop_path(A.linear(hd, self.P(p + "mlp.3.weight"), self.P(p + "mlp.3.bias"), out_f32=True), pk_)
            if s < len(c["depths"]) - 1:
                p = f"features.{2 * s + 1}."
                xv = x.reshape(B, t, h, w, C)
                xv = torch.nn.functional.pad(xv, (0, 0, 0, w % 2, 0, h % 2))  # torchvision _patch_merging_pad
                xm = torch.cat([xv[:, :, 0::2, 0::2], xv[:, :, 1::2, 0::2], xv[:, :, 0::2, 1::2], xv[:, :, 1::2, 1::2]], -1)
                y = A.layer_norm(xm.reshape(-1, 4 * C), self.P(p + "norm.weight"), self.P(p + "norm.bias"), eps)
                x = A.linear(y, self.P(p + "reduction.weight"), None, out_f32=True)
        t, h, w = grids[-1]
        return A.pool_head(x, self.P("norm.weight"), self.P("norm.bias"), self.P("head.weight"), self.P("head.bias"), B,
                           t * h * w, eps)

    def forward_logits(self, video: torch.Tensor) -> torch.Tensor:
        """logits f32 [B, classes] (a workspace buffer, overwritten by the next call); with
        `concurrent_streams = n > 1` the batch is split over n HIP streams (vclip_amd.streams):
        one part's small late-stage launches run beside another part's early stages."""
        B, Cin = video.shape[0], video.shape[1]
        if Cin != 3:
            raise ValueError("video must be [B, 3, T, H, W]")
        if (self.graph_replay and self.kernel_events is None and not streams.serial()
                and not torch.cuda.is_current_stream_capturing()):
            from .streams import GraphReplay
            if self._graphs is None:
                self._graphs = GraphReplay()
            key = (video.data_ptr(), tuple(video.shape), tuple(video.stride()), video.dtype, self.concurrent_streams, None if self.split_sizes is None else tuple(self.split_sizes),
                   str(video.device), self._weights_version())
            return self._graphs.run(key, video, self._forward_eager,
                                    keep=lambda: (self._packed, tuple(self._ws_used), self._bias_cache))
        return self._forward_eager(video)

    def _forward_eager(self, video: torch.Tensor) -> torch.Tensor:
        self._ws_used = []  # the workspaces this forward addresses (a captured graph keeps exactly these)
        B = video.shape[0]
        ns = max(1, min(int(self.concurrent_streams or 1), B))
        if ns == 1:
            return self._forward_part(video, 0)
        from .streams import run_split
        return run_split(self, video, ns, self._forward_part, self.num_classes, prepare=lambda: self._prepare(video))

    def _prepare(self, video: torch.Tensor):
        """Packed weights and every block's bias operand for this clip geometry, built on the current
        stream (streams.run_split builds them before the batch is forked over the side streams)."""
        _, _, T, H, W = video.shape
        self._pack(video.device)
        c = self.cfg
        for s, (t, h, w) in enumerate(self.geometry(video.shape[0], T, H, W)):
            for i in range(c["depths"][s]):
                shift_full = [0 if i % 2 == 0 else k // 2 for k in c["window_size"]]
                window, _ = window_and_shift((t, h, w), c["window_size"], shift_full)
                self._biasT(s, i, window, video.device)

    def _forward_part(self, video: torch.Tensor, part: int, out=None) -> torch.Tensor:
        c = self.cfg
        B, Cin, T, H, W = video.shape
        pk = self._pack(video.device)
        grids = self.geometry(B, T, H, W)
        ws = self._workspace(B, grids, video.device, part)
        eps = c["layer_norm_eps"]
        pt, ph, pw = c["patch_size"]
        t0, h0, w0 = grids[0]
        M0 = ws["stages"][0]["M"]
        tm = ops.timed
        C0 = c["embed_dim"]
        n0 = B * t0 * h0 * w0
        K0 = 3 * pt * ph * pw
        # algorithmic work per launch for an installed ops.OpRecorder: real tokens and channels (the
        # GEMMs run on channels padded to 128)
        tm("im2col_kernel", "im2col", B * 3 * T * H * W * 4 + n0 * K0 * 2, "byte", ops.tubelet_im2col, video,
           (pt, ph, pw), ws["A_emb"], layout="bcthw")
        ops.gemm(ws["A_emb"], pk["w_emb"], pk["b_emb"], "bias_f32", ws["E"], m=M0, flop=2.0 * n0 * C0 * K0, op="embed")
        X = ws["stages"][0]["X"]
        tm("layernorm_f32", "layernorm", n0 * C0 * 8, "byte", ops.layernorm_f32, ws["E"], pk["ln_emb"][0],
           pk["ln_emb"][1], eps, X, m=n0)
        for s, (st, sw) in enumerate(zip(pk["stages"], ws["stages"])):
            t, h, w = grids[s]
            ntok = B * t * h * w
            C, hid = st["C"], st["hid"]
            X, Y, QKV, O, Hd = sw["X"], sw["Y"], sw["QKV"], sw["O"], sw["Hd"]
            for i, blk in enumerate(st["blocks"]):
                shift_full = [0 if i % 2 == 0 else k // 2 for k in c["window_size"]]
                window, shift = window_and_shift((t, h, w), c["window_size"], shift_full)
                biasT = self._biasT(s, i, window, video.device)
                tm("layernorm_grp_kernel", f"layernorm.s{s}", ntok * C * 6, "byte", ops.layernorm, X, blk["ln1"][0],
                   blk["ln1"][1], eps, Y, m=ntok)
                ops.gemm(Y, blk["w_qkv"], blk["b_qkv"], "bias", QKV, flop=2.0 * ntok * 3 * C * C, op=f"qkv.s{s}",
                         nbytes=ops.gemm_bytes(ntok, 3 * C, C, "bias"))
                ev = self.kernel_events
                if ev is not None:  # recorded on the current stream, the one the kernel runs on
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                n = window[0] * window[1] * window[2]
                tm("window_attn_mb_d32_kernel", f"window_attention.s{s}", 4.0 * ntok * n * 32 * st["heads"], "flop",
                   ops.window_attention3d, QKV, B, (t, h, w), st["heads"], window, shift, biasT, O)
                if ev is not None:
                    e1.record()
                    # QK^T + PV over each token's window (window clipped to the grid), head_dim 32;
                    # algorithmic bytes: q, k, v read and the output written once (4 x 32 x 2 B per
                    # token-head)
                    ev.append((e0, e1, 4.0 * ntok * n * 32 * st["heads"], 256.0 * ntok * st["heads"]))
                ops.gemm(O, blk["w_proj"], blk["b_proj"], "bias_resid_f32", X, flop=2.0 * ntok * C * C, op=f"proj.s{s}",
                         nbytes=ops.gemm_bytes(ntok, C, C, "bias_resid_f32"))
                tm("layernorm_grp_kernel", f"layernorm.s{s}", ntok * C * 6, "byte", ops.layernorm, X, blk["ln2"][0],
                   blk["ln2"][1], eps, Y, m=ntok)
                ops.gemm(Y, blk["w_1"], blk["b_1"], "bias_gelu_erf", Hd, flop=2.0 * ntok * hid * C, op=f"fc1.s{s}",
                         nbytes=ops.gemm_bytes(ntok, hid, C, "bias_gelu_erf"))
                ops.gemm(Hd, blk["w_2"], blk["b_2"], "bias_resid_f32", X, flop=2.0 * ntok * C * hid, op=f"fc2.s{s}",
                         nbytes=ops.gemm_bytes(ntok, C, hid, "bias_resid_f32"))
            if s < len(grids) - 1:
                nxt = ws["stages"][s + 1]
                t2, h2, w2 = grids[s + 1]
                n2 = B * t2 * h2 * w2
                tm("patch_merge_ln_grp_kernel", "patch_merge_layernorm", ntok * C * 4 + n2 * 4 * C * 2, "byte",
                   ops.patch_merge_layernorm, X, B, (t, h, w), st["C"], st["merge_ln"][0], st["merge_ln"][1], eps,
                   sw["Mg"])
                ops.gemm(sw["Mg"], st["w_red"], st["b_red"], "bias_f32", nxt["X"], m=nxt["M"],
                         flop=2.0 * n2 * 2 * C * 4 * C, op="reduction")
        t, h, w = grids[-1]
        return ops.pool_head(ws["stages"][-1]["X"], B, t * h * w, pk["norm"][0], pk["norm"][1], eps, pk["w_head"],
                             pk["b_head"], out=ws["logits"] if out is None else out, work=ws["pool_work"])


def create_model(logger=None, model_size="tiny", pretrained=True, num_classes=2, device="cuda", weights_seed: int = 0):
    """Drop-in for videoswintransformer/swin_video_classifier/models/swin3d.py:7-53.

    The reference loads torchvision's Kinetics-400 weights (`Swin3D_*_Weights.DEFAULT`) and
    replaces the head; this image has no network, so the architecture of `model_size` is
    built with seeded synthetic weights (vclip_amd.weights) unless a checkpoint is loaded
    afterwards with `load_state_dict` (torchvision key names, `module.` prefixes stripped).
    """
    if model_size not in SWIN3D_CONFIGS:
        raise ValueError(f"Unknown model size: {model_size}")
    if logger:
        logger.info(f"Creating Video Swin Transformer ({model_size}) model...")
    cfg = SWIN3D_CONFIGS[model_size]
    model = Swin3d(cfg, num_classes=num_classes)
    from .weights import make_swin3d_weights
    model.load_state_dict(make_swin3d_weights(dict(cfg, num_classes=num_classes), seed=weights_seed))
    if logger:
        logger.info(f"Modified classification head to output {num_classes} classes")
    return model.to(device) if device else model
