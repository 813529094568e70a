"""torch.autograd Functions over the libvclip kernels, for the train steps composed in Python
(TimeSformer: vclip_amd/timesformer.py `_forward_train`; Swin3D: vclip_amd/swin3d.py `_forward_train`).

Every arithmetic op here is a HIP kernel of libvclip.so, forward and backward:
  linear      bf16 MFMA GEMM + bias (vc_gemm_bf16) / dgrad GEMM on the packed W^T / split-K wgrad
              (vc_wgrad_bf16) / bias column sums (vc_colsum); an optional row block of the weight is
              pre-scaled (the q rows: scale * log2 e folded as in the inference path, with the chain
              rule applied to the fp32 master weight and bias);
  layer_norm  vc_layernorm_f32_bf16 / vc_layernorm_f32, backward vc_layernorm_bwd;
  attention   flash forward with the base-2 log-sum-exp (vc_attention_fwd_lse) / flash backward
              (vc_attention_bwd) — joint or spatial (TimeSformer B*T sequences of 1 + P tokens);
  temporal_attention  vc_temporal_attention / vc_temporal_attention_bwd (clip layout, T <= 32);
  gelu_erf    vc_gelu_erf / vc_gelu_erf_bwd;
  cls_head    vc_cls_head / vc_cls_head_bwd (final LayerNorm on the CLS rows + classifier);
  window_attention  vc_window_attention3d_lse / vc_window_attention3d_bwd (Swin3D, head_dim 32, the
              relative-position bias table differentiable) + vc_colsum of its per-window partials;
  pool_head   vc_pool_head_pooled / vc_pool_head_bwd + vc_layernorm_bwd (Swin3D's final LayerNorm,
              token mean and classifier);
  im2col_cl / batchnorm / maxpool / resnet_head   the ResNet3D train step (conv3d_bwd.hip):
              vc_conv3d_im2col / vc_col2im_cl, BatchNorm3d with batch statistics (+ residual, ReLU)
              vc_batchnorm_train_fwd / _bwd, vc_maxpool3d / vc_maxpool3d_bwd, the head with its
              dropout vc_resnet_head_train / vc_pool_head_bwd / vc_resnet_head_train_bwd.
The tensors between them (residual adds, the clip <-> frame permutes, the CLS frame mean) are
ordinary torch tensor ops: layout glue, autograd's bookkeeping.  Rows are padded internally to the
kernels' tile multiples; the returned tensors have exactly the caller's rows.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib, ops
from .ops import _p, _stream


def _round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


def _padded(x: torch.Tensor, rows: int, dtype=None) -> torch.Tensor:
    """Contiguous copy of x (converted to dtype) with zero rows up to `rows`."""
    dtype = dtype or x.dtype
    out = torch.zeros((rows,) + tuple(x.shape[1:]), dtype=dtype, device=x.device)
    out[: x.shape[0]].copy_(x)
    return out


_ZEROS = {}


def _zeros_f32(n, device):
    """A shared all-zero f32 [n] (the dgrad GEMM's bias); never written."""
    key = (n, str(device))
    z = _ZEROS.get(key)
    if z is None:
        z = _ZEROS[key] = torch.zeros(n, dtype=torch.float32, device=device)
    return z


def _as_operand(x, rows, cols):
    """x as a bf16 [rows, cols] GEMM operand: x itself when it already is one (contiguous rows,
    no padding needed), else a zero-padded copy."""
    if (x.dtype == torch.bfloat16 and x.shape[0] == rows and x.shape[1] == cols and x.stride(1) == 1
            and x.stride(0) == cols):
        return x
    xp = torch.zeros(rows, cols, dtype=torch.bfloat16, device=x.device)
    xp[: x.shape[0], : x.shape[1]].copy_(x)
    return xp


class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, out_f32: bool, qrows: int, qscale: float):
        M, K = x.shape
        N = w.shape[0]
        # the GEMM tiles need M % 256 (rows), N and K % 128 (both also serve as the dgrad / wgrad
        # GEMMs' output widths): zero rows / columns, exactly 0 through every product
        Mp, Np, Kp = _round_up(M, 256), _round_up(N, 128), _round_up(K, 128)
        xp = _as_operand(x.detach(), Mp, Kp)
        wc = w.detach().float()
        if (Np, Kp) != (N, K):
            wc = torch.zeros(Np, Kp, dtype=torch.float32, device=x.device)
            wc[:N, :K].copy_(w.detach())
        wc = wc.contiguous()
        wb = torch.empty(Np, Kp, dtype=torch.bfloat16, device=x.device)
        wt = torch.empty(Kp, Np, dtype=torch.bfloat16, device=x.device)
        ops.pack_weight(wc, wb, wt, nscaled=qrows, scale=qscale)
        if b is None:
            bb = _zeros_f32(Np, x.device)
        elif Np == N and not qrows and b.dtype == torch.float32 and b.is_contiguous():
            bb = b.detach()
        else:
            bb = torch.zeros(Np, dtype=torch.float32, device=x.device)
            bb[:N].copy_(b.detach())
            if qrows:
                bb[:qrows] *= qscale
        out = torch.empty(Mp, Np, dtype=torch.float32 if out_f32 else torch.bfloat16, device=x.device)
        ops.gemm(xp, wb, bb, "bias_f32" if out_f32 else "bias", out)
        ctx.save_for_backward(xp, wt)
        ctx.M, ctx.N, ctx.K, ctx.qrows, ctx.qscale, ctx.xdtype = M, N, K, qrows, qscale, x.dtype
        ctx.has_bias = b is not None
        return out[:M, :N] if Np != N else out[:M]

    @staticmethod
    def backward(ctx, dy):
        xp, wt = ctx.saved_tensors
        Mp, Kp = xp.shape
        Np = wt.shape[1]
        M, N, K = ctx.M, ctx.N, ctx.K
        dyp = _as_operand(dy, Mp, Np)
        dx = torch.empty(Mp, Kp, dtype=torch.bfloat16, device=dy.device)
        ops.gemm(dyp, wt, _zeros_f32(Kp, dy.device), "bias", dx)
        dw = torch.empty(Np, Kp, dtype=torch.float32, device=dy.device)
        ops.wgrad(dyp, xp, dw, ops.wgrad_work(Mp, Np, Kp, dy.device), nscaled=ctx.qrows, scale=ctx.qscale)
        db = None
        if ctx.has_bias:
            db = torch.empty(Np, dtype=torch.float32, device=dy.device)
            ops.colsum(dyp, db, ops.colsum_work(M, Np, dy.device), m=M, nscaled=ctx.qrows, scale=ctx.qscale)
            db = db[:N]
        dx = dx[:M, :K] if Kp != K else dx[:M]
        dw = dw[:N, :K] if (Np, Kp) != (N, K) else dw
        return dx.to(ctx.xdtype), dw, db, None, None, None


def linear(x, w, b, out_f32=False, qrows=0, qscale=1.0):
    """y = x @ w.T + b with bf16 operands (x bf16 [M, K], w / b fp32 masters, b may be None), fp32
    accumulation; rows < qrows of w and b act multiplied by qscale.  Any M, N, K (padded inside)."""
    return _Linear.apply(x, w, b, out_f32, qrows, qscale)


class _LayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, g, b, eps: float, out_bf16: bool):
        x = x.contiguous().float()
        M, D = x.shape
        y = torch.empty(M, D, dtype=torch.bfloat16 if out_bf16 else torch.float32, device=x.device)
        gc, bc = g.detach().float().contiguous(), b.detach().float().contiguous()
        if out_bf16:
            ops.layernorm(x, gc, bc, eps, y)
        else:
            ops.layernorm_f32(x, gc, bc, eps, y)
        ctx.save_for_backward(x, gc)
        ctx.eps = eps
        return y

    @staticmethod
    def backward(ctx, dy):
        x, g = ctx.saved_tensors
        M, D = x.shape
        dyf = dy.float().contiguous()
        dx = torch.zeros(M, D, dtype=torch.float32, device=x.device)
        dxb = torch.empty(M, D, dtype=torch.bfloat16, device=x.device)
        dg = torch.empty(D, dtype=torch.float32, device=x.device)
        dbeta = torch.empty(D, dtype=torch.float32, device=x.device)
        nb = min(512, (M + 3) // 4)
        work = torch.empty((nb + (nb + 31) // 32) * 4 * D, dtype=torch.float32, device=x.device)
        ops.layernorm_bwd(dyf, x, g, ctx.eps, dx, dxb, dg, dbeta, work)
        return dx, dg, dbeta, None, None


def layer_norm(x, g, b, eps, out_bf16=True):
    """Row LayerNorm of f32 x [M, D] -> bf16 (out_bf16) or f32."""
    return _LayerNorm.apply(x, g, b, eps, out_bf16)


class _Attention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, B: int, S: int, H: int):
        rows = (B - 1) * S + _round_up(S, 64) + 64
        qp = _padded(qkv, max(rows, qkv.shape[0]))
        out = torch.zeros(qp.shape[0], H * 64, dtype=torch.bfloat16, device=qkv.device)
        lse = torch.empty(B * H * S, dtype=torch.float32, device=qkv.device)
        ops.attention_fwd_lse(qp, B, S, H, out, lse)
        ctx.save_for_backward(qp, out, lse)
        ctx.dims = (B, S, H, qkv.shape[0])
        return out[: qkv.shape[0]]

    @staticmethod
    def backward(ctx, dout):
        qp, out, lse = ctx.saved_tensors
        B, S, H, M = ctx.dims
        dp = _padded(dout, qp.shape[0], torch.bfloat16)
        delta = torch.empty(B * H * S, dtype=torch.float32, device=dout.device)
        dqkv = torch.zeros_like(qp)
        ops.attention_bwd(qp, out, dp, lse, delta, B, S, H, dqkv)
        return dqkv[:M], None, None, None


def attention(qkv, B, S, H):
    """softmax(q' k^T) v per (sequence, head) for B sequences of S rows of q'|k|v (q' prescaled by
    scale * log2 e), bf16 [B*S, 3*H*64] -> bf16 [B*S, H*64]."""
    return _Attention.apply(qkv, B, S, H)


class _TemporalAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, B: int, P: int, T: int, H: int):
        qkv = qkv.contiguous()
        out = torch.zeros(qkv.shape[0], H * 64, dtype=torch.bfloat16, device=qkv.device)
        ops.temporal_attention(qkv, B, P, T, H, 1.0, out, q_prescaled=True)
        ctx.save_for_backward(qkv)
        ctx.dims = (B, P, T, H)
        return out

    @staticmethod
    def backward(ctx, dout):
        (qkv,) = ctx.saved_tensors
        B, P, T, H = ctx.dims
        d = dout.to(torch.bfloat16).contiguous()
        dqkv = torch.zeros_like(qkv)
        _lib.call("vc_temporal_attention_bwd", _p(qkv), qkv.stride(0), _p(d), d.stride(0), B, P, T, H, 64, _p(dqkv),
                  dqkv.stride(0), _stream(qkv))
        return dqkv, None, None, None, None


def temporal_attention(qkv, B, P, T, H):
    """TimeSformer temporal attention on the clip layout (rows b*(1+P*T) + 1 + p*T + t; CLS rows of
    the output are zero and get no gradient), q' prescaled."""
    return _TemporalAttention.apply(qkv, B, P, T, H)


class _GeluErf(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = x.contiguous()
        M, N = x.shape
        y = torch.empty_like(x)
        _lib.call("vc_gelu_erf", _p(x), x.stride(0), M, N, _p(y), y.stride(0), _stream(x))
        ctx.save_for_backward(x)
        return y

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        M, N = x.shape
        dy = dy.contiguous()
        if dy.dtype not in (torch.bfloat16, torch.float32):
            dy = dy.float()
        dx = torch.empty_like(x)
        _lib.call("vc_gelu_erf_bwd", _p(dy), int(dy.dtype == torch.bfloat16), dy.stride(0), _p(x), x.stride(0), M, N,
                  _p(dx), dx.stride(0), _stream(x))
        return dx


def gelu_erf(x):
    """Exact GELU of bf16 [M, N]."""
    return _GeluErf.apply(x)


class _ClsHead(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, g, b, wc, bc, B: int, S: int, eps: float):
        x = x.contiguous().float()
        gc, bcn, wcc, bcc = (t.detach().float().contiguous() for t in (g, b, wc, bc))
        logits = ops.cls_head(x, B, S, gc, bcn, eps, wcc, bcc)
        ctx.save_for_backward(x, gc, bcn, wcc)
        ctx.dims = (B, S, eps)
        return logits.clone()

    @staticmethod
    def backward(ctx, dlogits):
        x, g, b, wc = ctx.saved_tensors
        B, S, eps = ctx.dims
        D = g.numel()
        dx = torch.zeros_like(x)
        dxb = torch.zeros(x.shape, dtype=torch.bfloat16, device=x.device)
        dwc = torch.empty_like(wc)
        dbc = torch.empty(wc.shape[0], dtype=torch.float32, device=x.device)
        dg = torch.empty(D, dtype=torch.float32, device=x.device)
        db = torch.empty(D, dtype=torch.float32, device=x.device)
        ops.cls_head_bwd(x, B, S, g, b, eps, wc, dlogits.float().contiguous(), dx, dxb, dwc, dbc, dg, db)
        return dx, dg, db, dwc, dbc, None, None, None


def cls_head(x, g, b, wc, bc, B, S, eps):
    """logits = classifier(LayerNorm(x[b*S])) over the CLS rows of f32 x [B*S, D]."""
    return _ClsHead.apply(x, g, b, wc, bc, B, S, eps)


class _WindowAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, table, B: int, grid, heads: int, window, shift, full_window):
        from .swin3d import expand_bias
        T, H, W = grid
        rows = B * T * H * W
        biasT = expand_bias(table.detach(), full_window, window, qkv.device)
        out = torch.empty(rows, heads * 32, dtype=torch.bfloat16, device=qkv.device)
        lse = torch.empty(rows * heads, dtype=torch.float32, device=qkv.device)
        ops.window_attention3d(qkv, B, grid, heads, window, shift, biasT, out, lse=lse)
        ctx.save_for_backward(qkv, out, lse, table)
        ctx.dims = (B, tuple(grid), heads, tuple(window), tuple(shift), tuple(full_window))
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, out, lse, table = ctx.saved_tensors
        B, grid, heads, window, shift, full_window = ctx.dims
        T, H, W = grid
        ft, fh, fw = full_window
        ntab = (2 * ft - 1) * (2 * fh - 1) * (2 * fw - 1)
        nwin = B * (T // window[0]) * (H // window[1]) * (W // window[2])
        d = dout.to(torch.bfloat16).contiguous()
        dqkv = torch.empty(qkv.shape[0], 3 * heads * 32, dtype=torch.bfloat16, device=qkv.device)
        part = torch.empty(nwin, heads * ntab, dtype=torch.float32, device=qkv.device)
        tab = table.detach().float().contiguous()
        ops.window_attention3d_bwd(qkv, out, d, lse, B, grid, heads, window, shift, full_window, tab, dqkv, part)
        dtab = torch.empty(heads * ntab, dtype=torch.float32, device=qkv.device)
        ops.colsum(part, dtab, ops.colsum_work(part.shape[0], dtab.numel(), part.device))  # fixed order
        return dqkv, dtab.view(heads, ntab).t(), None, None, None, None, None, None


def window_attention(qkv, table, B, grid, heads, window, shift, full_window):
    """Swin 3D shifted-window attention (head_dim 32) with the relative-position bias table
    [ntab, heads] as a differentiable input; qkv bf16 [B*T*H*W rows, 3*heads*32] (q' prescaled)."""
    return _WindowAttention.apply(qkv, table, B, tuple(grid), heads, tuple(window), tuple(shift), tuple(full_window))


class _PoolHead(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, g, b, wc, bc, B: int, ntok: int, eps: float):
        x = x.contiguous().float()
        D = g.numel()
        gc, bcn, wcc, bcc = (t.detach().float().contiguous() for t in (g, b, wc, bc))
        nl = wcc.shape[0]
        logits = torch.empty(B, nl, dtype=torch.float32, device=x.device)
        pooled = torch.empty(B, D, dtype=torch.float32, device=x.device)
        work = torch.empty(B * 64 * D, dtype=torch.float32, device=x.device)
        _lib.call("vc_pool_head_pooled", _p(x), x.stride(0), B, ntok, D, _p(gc), _p(bcn), eps, _p(wcc), _p(bcc), nl,
                  _p(logits), _p(work), _p(pooled), _stream(x))
        ctx.save_for_backward(x, gc, wcc, pooled)
        ctx.dims = (B, ntok, eps)
        return logits

    @staticmethod
    def backward(ctx, dlogits):
        x, g, wc, pooled = ctx.saved_tensors
        B, ntok, eps = ctx.dims
        D, nl = g.numel(), wc.shape[0]
        dl = dlogits.float().contiguous()
        dpooled = torch.empty(B, D, dtype=torch.float32, device=x.device)
        dwc = torch.empty(nl, D, dtype=torch.float32, device=x.device)
        dbc = torch.empty(nl, dtype=torch.float32, device=x.device)
        _lib.call("vc_pool_head_bwd", _p(pooled), _p(dl), _p(wc), B, D, nl, 1.0 / ntok, _p(dpooled), _p(dwc), _p(dbc),
                  _stream(x))
        dy = dpooled.repeat_interleave(ntok, 0)  # the mean's backward: every token of clip b gets dpooled[b]
        M = x.shape[0]
        dx = torch.zeros(M, D, dtype=torch.float32, device=x.device)
        dxb = torch.empty(M, D, dtype=torch.bfloat16, device=x.device)
        dg = torch.empty(D, dtype=torch.float32, device=x.device)
        db = torch.empty(D, dtype=torch.float32, device=x.device)
        nb = min(512, (M + 3) // 4)
        work = torch.empty((nb + (nb + 31) // 32) * 4 * D, dtype=torch.float32, device=x.device)
        ops.layernorm_bwd(dy, x, g, eps, dx, dxb, dg, db, work)
        return dx, dg, db, dwc, dbc, None, None, None


def pool_head(x, g, b, wc, bc, B, ntok, eps):
    """torchvision SwinTransformer3d head: logits = Linear(mean over each clip's ntok tokens of
    LayerNorm(x)) for f32 x [B*ntok, D]."""
    return _PoolHead.apply(x, g, b, wc, bc, B, ntok, eps)


def _i3(v):
    return (ctypes.c_int * 3)(*[int(x) for x in v])


class _Im2colCL(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, B: int, grid, C: int, kernel, stride, pad):
        To, Ho, Wo = ops.conv_out_size(grid, kernel, stride, pad)
        M = B * To * Ho * Wo
        a = torch.empty(M, kernel[0] * kernel[1] * kernel[2] * C, dtype=torch.bfloat16, device=x.device)
        ops.conv3d_im2col(x, "cl_bf16", B, grid, C, kernel, stride, pad, a)
        ctx.dims = (B, tuple(grid), C, tuple(kernel), tuple(stride), tuple(pad), x.shape[0])
        return a

    @staticmethod
    def backward(ctx, da):
        B, grid, C, kernel, stride, pad, rows = ctx.dims
        da = da.to(torch.bfloat16)
        if da.stride(1) != 1:
            da = da.contiguous()
        dx = torch.empty(rows, C, dtype=torch.float32, device=da.device)
        T, H, W = grid
        _lib.call("vc_col2im_cl", _p(da), da.stride(0), B, T, H, W, C, ctypes.addressof(k := _i3(kernel)),
                  ctypes.addressof(s_ := _i3(stride)), ctypes.addressof(p_ := _i3(pad)), _p(dx), C, _stream(da))
        return dx, None, None, None, None, None, None


def im2col_cl(x, B, grid, C, kernel, stride, pad):
    """Conv3d patches of channels-last bf16 rows [B*T*H*W, C] -> bf16 [B*To*Ho*Wo, kt*kh*kw*C]
    (columns (kt, kh, kw, c)), differentiable w.r.t. x (col2im)."""
    return _Im2colCL.apply(x, B, tuple(grid), C, tuple(kernel), tuple(stride), tuple(pad))


def _bn_work(M, C, device):
    splits = min(4096, max(1, (M + 127) // 128))  # conv3d_bwd.hip bn_splits
    return torch.empty(splits * 2 * C, dtype=torch.float32, device=device)


class _BatchNormTrain(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y, gamma, beta, res, running_mean, running_var, relu: bool, eps: float, momentum: float):
        y = y.contiguous().float()
        M, C = y.shape
        g, b = gamma.detach().float().contiguous(), beta.detach().float().contiguous()
        z = torch.empty(M, C, dtype=torch.bfloat16, device=y.device)
        stat = torch.empty(2, C, dtype=torch.float32, device=y.device)
        work = _bn_work(M, C, y.device)
        if res is not None:
            res = res.to(torch.bfloat16)
            if res.stride(1) != 1:
                res = res.contiguous()
        rm = running_mean.detach() if running_mean is not None else None
        rv = running_var.detach() if running_var is not None else None
        _lib.call("vc_batchnorm_train_fwd", _p(y), y.stride(0), M, C, _p(g), _p(b), eps, momentum,
                  _p(rm) if rm is not None else None, _p(rv) if rv is not None else None,
                  _p(res) if res is not None else None, 1, res.stride(0) if res is not None else 0, int(relu), _p(z),
                  C, _p(stat), _p(work), work.numel(), _stream(y))
        ctx.save_for_backward(y, stat, g, z)
        ctx.relu, ctx.has_res = relu, res is not None
        return z

    @staticmethod
    def backward(ctx, dz):
        y, stat, g, z = ctx.saved_tensors
        M, C = y.shape
        dz = dz.float().contiguous()
        dy = torch.empty(M, C, dtype=torch.float32, device=y.device)
        dres = torch.empty(M, C, dtype=torch.float32, device=y.device) if ctx.has_res else None
        dg = torch.empty(C, dtype=torch.float32, device=y.device)
        db = torch.empty(C, dtype=torch.float32, device=y.device)
        work = _bn_work(M, C, y.device)
        _lib.call("vc_batchnorm_train_bwd", _p(y), C, M, C, _p(stat), _p(g), _p(dz), C, _p(z), C, int(ctx.relu), _p(dy), C,
                  _p(dres) if dres is not None else None, C, _p(dg), _p(db), _p(work), work.numel(), _stream(y))
        return dy, dg, db, dres, None, None, None, None, None


def batchnorm(y, gamma, beta, running_mean=None, running_var=None, res=None, relu=False, eps=1e-5, momentum=0.1):
    """nn.BatchNorm3d in training mode on channels-last f32 rows [M, C] (batch statistics; the
    running statistics updated in place) -> bf16 relu?(BN(y) + res)."""
    return _BatchNormTrain.apply(y, gamma, beta, res, running_mean, running_var, relu, eps, momentum)


class _MaxPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, B: int, grid, C: int, kernel, stride, pad):
        x = x.contiguous()
        To, Ho, Wo = ops.conv_out_size(grid, kernel, stride, pad)
        y = torch.empty(B * To * Ho * Wo, C, dtype=torch.bfloat16, device=x.device)
        ops.maxpool3d(x, B, grid, C, kernel, stride, pad, y)
        ctx.save_for_backward(x)
        ctx.dims = (B, tuple(grid), C, tuple(kernel), tuple(stride), tuple(pad))
        return y

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        B, grid, C, kernel, stride, pad = ctx.dims
        dyf = dy.float().contiguous()
        dx = torch.empty(x.shape[0], C, dtype=torch.float32, device=x.device)
        T, H, W = grid
        _lib.call("vc_maxpool3d_bwd", _p(x), x.stride(0), _p(dyf), 0, C, B, T, H, W, C,
                  ctypes.addressof(k := _i3(kernel)), ctypes.addressof(s_ := _i3(stride)),
                  ctypes.addressof(p_ := _i3(pad)), _p(dx), C, _stream(x))
        return dx, None, None, None, None, None, None


def maxpool(x, B, grid, C, kernel, stride, pad):
    """MaxPool3d on channels-last bf16 rows, differentiable (gradient to each window's first max)."""
    return _MaxPool.apply(x, B, tuple(grid), C, tuple(kernel), tuple(stride), tuple(pad))


class _ResnetHead(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, wc, bc, keep, B: int, T: int, HW: int, pool_t: int):
        x = x.contiguous()
        C = x.shape[1]
        wcc, bcc = wc.detach().float().contiguous(), bc.detach().float().contiguous()
        nl = wcc.shape[0]
        u = torch.empty(B, C, dtype=torch.float32, device=x.device)
        logits = torch.empty(B, nl, dtype=torch.float32, device=x.device)
        keep = keep.float().contiguous()
        _lib.call("vc_resnet_head_train", _p(x), x.stride(0), B, T, HW, C, pool_t, _p(keep), _p(wcc), _p(bcc), nl, _p(u),
                  _p(logits), _stream(x))
        ctx.save_for_backward(u, wcc, keep)
        ctx.dims = (B, T, HW, C, pool_t, x.shape[0])
        return logits

    @staticmethod
    def backward(ctx, dlogits):
        u, wc, keep = ctx.saved_tensors
        B, T, HW, C, pool_t, rows = ctx.dims
        nl = wc.shape[0]
        dl = dlogits.float().contiguous()
        du = torch.empty(B, C, dtype=torch.float32, device=u.device)
        dwc = torch.empty(nl, C, dtype=torch.float32, device=u.device)
        dbc = torch.empty(nl, dtype=torch.float32, device=u.device)
        _lib.call("vc_pool_head_bwd", _p(u), _p(dl), _p(wc), B, C, nl, 1.0, _p(du), _p(dwc), _p(dbc), _stream(u))
        dx = torch.empty(rows, C, dtype=torch.float32, device=u.device)
        _lib.call("vc_resnet_head_train_bwd", _p(du), B, T, HW, C, pool_t, _p(keep), _p(dx), C, _stream(u))
        return dx, dwc, dbc, None, None, None, None, None


def resnet_head(x, wc, bc, keep, B, T, HW, pool_t):
    """pytorchvideo ResNetBasicHead (AvgPool3d((pool_t, H, W), stride 1) -> Dropout -> Linear ->
    AdaptiveAvgPool3d(1)) on the final channels-last map [B*T*HW, C]; keep = the dropout scale
    per (clip, pooled position, channel)."""
    return _ResnetHead.apply(x, wc, bc, keep, B, T, HW, pool_t)

