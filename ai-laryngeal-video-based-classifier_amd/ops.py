"""torch-tensor front end of the libvclip.so kernels.

Each function validates shapes/dtypes/devices on the host (a kernel is never launched
on operands whose shape it does not support), then calls the C-ABI with raw device
pointers and torch's current HIP stream, so the work orders correctly with torch ops
and is captured by torch.cuda graphs.  No CPU fallback exists: CPU tensors raise.
"""
from __future__ import annotations

import torch

from . import _lib

EPI = {"bias": 0, "bias_gelu_tanh": 1, "bias_gelu_erf": 2, "bias_resid_f32": 3, "embed_f32": 4, "bias_f32": 5,
       "bias_relu": 6, "bias_resid_relu": 7, "bias_add_f32": 8, "bias_gelu_tanh_save": 9, "dgelu_tanh": 10}
GATHER_KIND = {"u8": 0, "f32": 1, "bf16": 2}


def _dev(*ts):
    for t in ts:
        if not isinstance(t, torch.Tensor) or t.device.type != "cuda":
            raise _lib.VclipError("vclip ops need CUDA(HIP) tensors; there is no CPU path")


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def _p(t):
    return t.data_ptr()


def _need(cond, msg):
    if not cond:
        raise _lib.VclipError(msg)


def frame_gather(frames: torch.Tensor, idx: torch.Tensor, kind: str = "f32", scale: float = 1.0 / 63.75,
                 shift: float = -3.0, out: torch.Tensor | None = None) -> torch.Tensor:
    """frames u8 [N,F,H,W,C], idx int64 [N,T] -> u8 [N,T,H,W,C] or f32/bf16 [N,T,C,H,W]."""
    _dev(frames, idx)
    _need(frames.dtype == torch.uint8 and frames.dim() == 5 and frames.is_contiguous(), "frames: u8 [N,F,H,W,C]")
    _need(idx.dtype == torch.int64 and idx.dim() == 2 and idx.is_contiguous() and idx.shape[0] == frames.shape[0],
          "idx: int64 [N,T]")
    N, F, H, W, C = frames.shape
    T = idx.shape[1]
    if kind == "u8":
        shape, dt = (N, T, H, W, C), torch.uint8
    else:
        shape, dt = (N, T, C, H, W), (torch.float32 if kind == "f32" else torch.bfloat16)
    if out is None:
        out = torch.empty(shape, dtype=dt, device=frames.device)
    _need(tuple(out.shape) == shape and out.dtype == dt and out.is_contiguous(), "frame_gather: bad out")
    _lib.call("vc_frame_gather", _p(frames), N, F, H, W, C, _p(idx), T, GATHER_KIND[kind], scale, shift, _p(out),
              _stream(frames))
    return out


TOKEN_ORDER = {"time_major": 0, "patch_major": 1}
VIDEO_LAYOUT = {"btchw": 0, "bcthw": 1}
# 16-bit operand types (include/vclip.h VC_ELEM_*): bf16 everywhere; fp16 for the inference forward
H16 = (torch.bfloat16, torch.float16)
ELEM_F16 = 1
ELEM_BF16 = 0


def tubelet_im2col(pix: torch.Tensor, tubelet, out: torch.Tensor, order: str = "time_major",
                   layout: str = "btchw") -> torch.Tensor:
    """pix f32 [B,T,C,H,W] (layout "btchw") or [B,C,T,H,W] ("bcthw") -> out bf16
    [>= B*nt*nh*nw, >= C*kt*kh*kw] (rows / columns beyond are untouched).
    order "time_major": token (t', hp, wp) (ViViT, Swin); "patch_major": token (hp, wp, t') (TimeSformer)."""
    _dev(pix, out)
    _need(pix.dtype == torch.float32 and pix.dim() == 5 and pix.is_contiguous(), "pixel_values: f32 5-D contiguous")
    if layout == "btchw":
        B, T, C, H, W = pix.shape
    else:
        B, C, T, H, W = pix.shape
    kt, kh, kw = tubelet
    ntok = B * (T // kt) * (H // kh) * (W // kw)
    _need(out.dtype in H16 and out.dim() == 2 and out.shape[0] >= ntok and out.shape[1] >= C * kt * kh * kw
          and out.stride(1) == 1, "im2col out: bf16 / fp16 [rows, >= C*kt*kh*kw]")
    _need(H % kh == 0 and W % kw == 0 and T % kt == 0 and kw % 4 == 0, "im2col: shape not divisible by the patch")
    if out.dtype == torch.float16:
        _lib.call("vc_patch_im2col_h16", _p(pix), B, T, C, H, W, kt, kh, kw, TOKEN_ORDER[order], VIDEO_LAYOUT[layout],
                  ELEM_F16, _p(out), out.stride(0), _stream(pix))
    else:
        _lib.call("vc_patch_im2col", _p(pix), B, T, C, H, W, kt, kh, kw, TOKEN_ORDER[order], VIDEO_LAYOUT[layout],
                  _p(out), out.stride(0), _stream(pix))
    return out


class OpRecorder:
    """HIP events around every launch an instrumented forward makes while this recorder is installed
    (`with ops.recording(rec):`), on the stream each launch runs on.  Entries (kernel, op, e0, e1,
    work, unit): `kernel` names the kernel instantiation the launch ran (GEMMs: the tile config vc_gemm
    picked and the epilogue, i.e. one rocprofv3 kernel name), `work` its algorithmic work (FLOP or
    bytes, unit "flop" / "byte") as the caller states it (real rows and channels, not the padding)."""

    def __init__(self):
        self.entries = []

    def begin(self):
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record()
        return e0

    def end(self, e0, kernel, op, work, unit):
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        self.entries.append((kernel, op, e0, e1, float(work), unit))

    def summary(self, n_steps: int, step_ms: float):
        """per kernel: launches per step, mean launch ms, share of the step, achieved rate (TFLOP/s or
        GB/s of algorithmic work), the ops that ran it; sorted by share"""
        agg = {}
        for kernel, op, e0, e1, work, unit in self.entries:
            if kernel in agg and agg[kernel]["unit"] != unit:  # one kernel, launches on both sides of the ridge
                kernel = f"{kernel} [{'HBM' if unit == 'byte' else 'MFMA'}-bound launches]"
            a = agg.setdefault(kernel, {"ms": [], "work": 0.0, "unit": unit, "ops": set()})
            a["ms"].append(e0.elapsed_time(e1))
            a["work"] += work
            a["ops"].add(op)
        out = {}
        for k, a in agg.items():
            tot = sum(a["ms"])
            rate = a["work"] / (tot * 1e-3) / (1e12 if a["unit"] == "flop" else 1e9)
            out[k] = {"launches_per_step": round(len(a["ms"]) / n_steps, 2), "avg_launch_ms": round(tot / len(a["ms"]), 4),
                      "share_of_step": round(tot / n_steps / step_ms, 4), "achieved": round(rate, 1),
                      "unit": "TFLOP/s" if a["unit"] == "flop" else "GB/s", "ops": sorted(a["ops"])}
        return dict(sorted(out.items(), key=lambda kv: -kv[1]["share_of_step"]))

    def summary_ops(self, n_steps: int, step_ms: float):
        """per op label (e.g. ResNet3D's "conv_b.s3": conv_b of res stage 3): launches per step, ms per
        step, share of the step, achieved rate, the kernels that ran it; sorted by share"""
        agg = {}
        for kernel, op, e0, e1, work, unit in self.entries:
            if op in agg and agg[op]["unit"] != unit:
                op = f"{op} [{'HBM' if unit == 'byte' else 'MFMA'}-bound launches]"
            a = agg.setdefault(op, {"ms": 0.0, "n": 0, "work": 0.0, "unit": unit, "kernels": set()})
            a["ms"] += e0.elapsed_time(e1)
            a["n"] += 1
            a["work"] += work
            a["kernels"].add(kernel)
        out = {}
        for k, a in agg.items():
            rate = a["work"] / (a["ms"] * 1e-3) / (1e12 if a["unit"] == "flop" else 1e9)
            out[k] = {"launches_per_step": round(a["n"] / n_steps, 2), "ms_per_step": round(a["ms"] / n_steps, 4),
                      "share_of_step": round(a["ms"] / n_steps / step_ms, 4), "achieved": round(rate, 1),
                      "unit": "TFLOP/s" if a["unit"] == "flop" else "GB/s", "kernels": sorted(a["kernels"])}
        return dict(sorted(out.items(), key=lambda kv: -kv[1]["share_of_step"]))


_REC = [None]


class recording:
    """`with ops.recording(rec): model.forward_logits(x)`: instrumented launches append to rec."""

    def __init__(self, rec: OpRecorder):
        self.rec = rec

    def __enter__(self):
        self.prev = _REC[0]
        _REC[0] = self.rec
        return self.rec

    def __exit__(self, *exc):
        _REC[0] = self.prev


def timed(kernel: str, op: str, work: float, unit: str, fn, *args, **kw):
    """fn(*args, **kw), between HIP events when a recorder is installed (one attribute test otherwise)"""
    rec = _REC[0]
    if rec is None:
        return fn(*args, **kw)
    e0 = rec.begin()
    r = fn(*args, **kw)
    rec.end(e0, kernel, op, work, unit)
    return r


# rocprofv3 names of the GEMM kernels per tile config (csrc/gemm.hip kCfgs; E = the epilogue, ET = 0 bf16)
GEMM_KERNEL = {3: "gemm_bf16_big_kernel<{E}, {ET}>", 4: "gemm_bf16_persist_kernel<{E}, {ET}>",
               5: "gemm_bf16_kernel<128, 128, 2, 4, {E}, 2, {ET}>", 7: "gemm_bf16_kernel<64, 128, 2, 4, {E}, 2, {ET}>",
               8: "gemm_pp_kernel<{E}, {ET}>", 15: "gemm_ppd_kernel<{E}, {ET}>", 20: "conv_c_stream_kernel<{K}, {BN}>",
               21: "gemm_bf16_kernel<64, 128, 2, 4, {E}, 4, {ET}>"}


# roofline ridge of the bf16 matrix pipe against HBM (MI355X_MICROARCH.md: 2.5 PFLOP/s dense, 8 TB/s):
# a launch whose algorithmic FLOP per byte falls below it is bounded by HBM, and its table row is
# filed under its bytes (GB/s vs 8 TB/s) instead of its FLOP
RIDGE_FLOP_PER_BYTE = 2500e12 / 8e12
# bytes per output element an epilogue moves (output written, plus the residual / aux it reads)
_EPI_OUT_BYTES = {"bias": 2, "bias_gelu_tanh": 2, "bias_gelu_erf": 2, "bias_resid_f32": 8, "embed_f32": 8,
                  "bias_f32": 4, "bias_relu": 2, "bias_resid_relu": 4, "bias_add_f32": 8, "bias_gelu_tanh_save": 4,
                  "dgelu_tanh": 4}


def gemm_bytes(M: int, N: int, K: int, epilogue: str, esize: int = 2) -> float:
    """algorithmic HBM bytes of one GEMM launch: A and W read once, the epilogue's output (and residual /
    aux operand) once"""
    return float(M * K * esize + N * K * esize + M * N * _EPI_OUT_BYTES[epilogue])


def gemm_kernel_name(M, N, K, epilogue: str, out, aux=None, cfg: int = -1, f16: bool = False) -> str:
    e = EPI[epilogue]
    if cfg < 0:
        cfg = _lib.load().vc_gemm_pick(M, N, K, e, out.stride(0), aux.stride(0) if aux is not None else 0,
                                       _p(aux) if aux is not None else None)
    return GEMM_KERNEL.get(cfg, f"gemm cfg {cfg}").format(E=e, ET=1 if f16 else 0, K=K, BN=256 if K <= 128 else 128)


def gemm(a: torch.Tensor, w: torch.Tensor, bias: torch.Tensor, epilogue: str, out: torch.Tensor,
         aux: torch.Tensor | None = None, group: int = 0, group_stride: int = 0, group_offset: int = 0,
         m: int | None = None, cfg: int = -1, flop: float | None = None, op: str = "gemm",
         nbytes: float | None = None) -> torch.Tensor:
    """out (+)= epilogue(a[:m] @ w.T + bias).  a bf16 [M,K], w bf16 [N,K], bias f32 [N]; or a, w (and the
    16-bit out) fp16 for the inference epilogues (bias / gelu / resid_f32 / embed_f32).  `flop` / `op`:
    the algorithmic work and op name an installed OpRecorder files this launch under (default
    2 M N K of the operand shapes); `nbytes` (default: gemm_bytes of the operand shapes, scaled by
    flop / 2 M N K) its algorithmic bytes: the launch is filed under whichever bounds it -- bytes when
    flop / bytes is below RIDGE_FLOP_PER_BYTE (or when only `nbytes` is given), FLOP otherwise."""
    rec = _REC[0]
    if rec is not None:
        M_ = a.shape[0] if m is None else m
        label = gemm_kernel_name(M_, w.shape[0], a.shape[1], epilogue, out, aux, cfg, a.dtype == torch.float16)
        e0 = rec.begin()
        _gemm(a, w, bias, epilogue, out, aux, group, group_stride, group_offset, m, cfg)
        if nbytes is not None and flop is None:
            rec.end(e0, label, op, nbytes, "byte")
        else:
            fl0 = 2.0 * M_ * w.shape[0] * a.shape[1]
            fl = fl0 if flop is None else flop
            # default bytes: the operand shapes' (scaled like the FLOP when the caller states real rows /
            # channels instead of the padded ones)
            nb = nbytes if nbytes is not None else (
                gemm_bytes(M_, w.shape[0], a.shape[1], epilogue, a.element_size()) * (fl / fl0))
            if nb is not None and fl / nb < RIDGE_FLOP_PER_BYTE:
                rec.end(e0, label, op, nb, "byte")
            else:
                rec.end(e0, label, op, fl, "flop")
        return out
    return _gemm(a, w, bias, epilogue, out, aux, group, group_stride, group_offset, m, cfg)


def _gemm(a, w, bias, epilogue, out, aux, group, group_stride, group_offset, m, cfg):
    _dev(a, w, bias, out)
    M = a.shape[0] if m is None else m
    K = a.shape[1]
    N = w.shape[0]
    _need(a.dtype in H16 and w.dtype == a.dtype and bias.dtype == torch.float32, "gemm dtypes (a, w: bf16 or fp16)")
    f16 = a.dtype == torch.float16
    _need(a.stride(1) == 1 and w.stride(1) == 1 and out.stride(-1) == 1 and w.shape[1] == K, "gemm layout")
    _need(bias.numel() == N and bias.is_contiguous(), "gemm bias")
    e = EPI[epilogue]
    _need(not f16 or e <= 4, "gemm: fp16 operands support the inference epilogues only")
    if e in (0, 1, 2, 6, 7, 9, 10):
        _need(out.dtype == a.dtype, "gemm out must have the operand type for this epilogue")
    else:
        _need(out.dtype == torch.float32, "gemm out must be f32 for this epilogue")
    if e in (7, 9, 10):
        _need(aux is not None and aux.dtype == torch.bfloat16 and aux.stride(1) == 1 and aux.shape[0] >= M and
              aux.shape[1] >= N, f"{epilogue}: aux must be bf16 [>= M, >= N]")
    if e == 8:
        _need(aux is not None and aux.dtype == torch.float32 and aux.stride(1) == 1 and aux.shape[0] >= M and
              aux.shape[1] >= N, "bias_add_f32: aux must be the f32 residual [>= M, >= N]")
    if e == 4:
        _need(aux is not None and aux.dtype == torch.float32 and aux.stride(1) == 1 and group > 0, "embed aux")
        _need((M - 1) // group * group_stride + group_offset + (M - 1) % group < out.shape[0], "embed out rows")
    else:
        _need(out.shape[0] >= M, "gemm out rows")
    _need(a.shape[0] >= M, "gemm a rows")
    aux_p = _p(aux) if aux is not None else None
    ldaux = aux.stride(0) if aux is not None else 0
    if f16:
        _lib.call("vc_gemm_h16", _p(a), a.stride(0), _p(w), w.stride(0), M, N, K, _p(bias), e, _p(out),
                  out.stride(0), aux_p, ldaux, group, group_stride, group_offset, ELEM_F16, cfg, _stream(a))
    else:
        _lib.call("vc_gemm_bf16_cfg", _p(a), a.stride(0), _p(w), w.stride(0), M, N, K, _p(bias), e, _p(out),
                  out.stride(0), aux_p, ldaux, group, group_stride, group_offset, cfg, _stream(a))
    return out


def gemm_wrap(a: torch.Tensor, ka: int, w: torch.Tensor, bias: torch.Tensor, epilogue: str, out: torch.Tensor,
              aux: torch.Tensor | None = None, group: int = 0, group_stride: int = 0, group_offset: int = 0,
              m: int | None = None, flop: float | None = None, op: str = "gemm") -> torch.Tensor:
    """vc_gemm_h16_wrap: out (+)= epilogue(A . W^T + bias) with A = a[:m, :ka] wrapping along K: W [N, K]
    with ka <= K <= 2 ka is [W1 | W2] and the product A.W1 + A.W2 (the split-operand fp16 build)."""
    _dev(a, w, bias, out)
    M = a.shape[0] if m is None else m
    N, K = w.shape
    _need(a.dtype in H16 and w.dtype == a.dtype and bias.dtype == torch.float32 and a.stride(1) == 1 and
          w.stride(1) == 1 and a.shape[1] >= ka, "gemm_wrap operands")
    e = EPI[epilogue]
    _need(e <= 4, "gemm_wrap: inference epilogues only")
    if e == 4:
        _need(aux is not None and aux.dtype == torch.float32 and group > 0, "gemm_wrap embed aux")
        _need((M - 1) // group * group_stride + group_offset + (M - 1) % group < out.shape[0], "gemm_wrap embed out rows")
    else:
        _need(out.shape[0] >= M, "gemm_wrap out rows")
    rec = _REC[0]
    e0 = rec.begin() if rec is not None else None
    _lib.call("vc_gemm_h16_wrap", _p(a), a.stride(0), ka, _p(w), w.stride(0), M, N, K, _p(bias), e, _p(out),
              out.stride(0), _p(aux) if aux is not None else None, aux.stride(0) if aux is not None else 0, group,
              group_stride, group_offset, ELEM_F16 if a.dtype == torch.float16 else 0, _stream(a))
    if rec is not None:
        rec.end(e0, f"gemm_pp_kernel<{e}, {1 if a.dtype == torch.float16 else 0}>", op,
                2.0 * M * N * K if flop is None else flop, "flop")
    return out


def patch_im2col_split(pix: torch.Tensor, tubelet, out: torch.Tensor, order: str = "time_major",
                       layout: str = "btchw") -> torch.Tensor:
    """[A_hi | A_lo] im2col (vc_patch_im2col_split_h16): out 16-bit [>= tokens, >= 2 K]."""
    _dev(pix, out)
    if layout == "btchw":
        B, T, C, H, W = pix.shape
    else:
        B, C, T, H, W = pix.shape
    kt, kh, kw = tubelet
    _need(pix.dtype == torch.float32 and pix.is_contiguous() and out.dtype in H16 and out.stride(1) == 1 and
          out.shape[1] >= 2 * C * kt * kh * kw, "patch_im2col_split")
    _lib.call("vc_patch_im2col_split_h16", _p(pix), B, T, C, H, W, kt, kh, kw, TOKEN_ORDER[order], VIDEO_LAYOUT[layout],
              ELEM_F16 if out.dtype == torch.float16 else 0, _p(out), out.stride(0), _stream(pix))
    return out


_NUM_CUS = {}


def _num_cus(dev: torch.device) -> int:
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    if key not in _NUM_CUS:
        _NUM_CUS[key] = torch.cuda.get_device_properties(key).multi_processor_count
    return _NUM_CUS[key]


def layernorm(x: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, eps: float, out: torch.Tensor,
              m: int | None = None) -> torch.Tensor:
    """LayerNorm of the first gamma.numel() columns of each row (x f32 -> out bf16 or fp16)."""
    _dev(x, gamma, beta, out)
    M = x.shape[0] if m is None else m
    D = gamma.numel()
    _need(x.dtype == torch.float32 and out.dtype in H16 and x.stride(1) == 1 and out.stride(1) == 1,
          "layernorm: x f32, out bf16 / fp16, unit column stride")
    _need(beta.numel() == D and x.shape[1] >= D and out.shape[1] >= D and out.shape[0] >= M and x.shape[0] >= M,
          "layernorm shapes")
    if out.dtype == torch.float16:
        _lib.call("vc_layernorm_f32_h16", _p(x), x.stride(0), M, D, _p(gamma), _p(beta), eps, ELEM_F16, _p(out),
                  out.stride(0), _stream(x))
    else:
        _lib.call("vc_layernorm_f32_bf16", _p(x), x.stride(0), M, D, _p(gamma), _p(beta), eps, _p(out), out.stride(0),
                  _stream(x))
    return out


def layernorm_f32(x: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, eps: float, out: torch.Tensor,
                  m: int | None = None) -> torch.Tensor:
    """f32 -> f32 LayerNorm over the first gamma.numel() columns of each row."""
    _dev(x, gamma, beta, out)
    M = x.shape[0] if m is None else m
    D = gamma.numel()
    _need(x.dtype == torch.float32 and out.dtype == torch.float32 and x.stride(1) == 1 and out.stride(1) == 1,
          "layernorm_f32 dtypes")
    _need(beta.numel() == D and x.shape[1] >= D and out.shape[1] >= D and x.shape[0] >= M and out.shape[0] >= M,
          "layernorm_f32 shapes")
    _lib.call("vc_layernorm_f32", _p(x), x.stride(0), M, D, _p(gamma), _p(beta), eps, _p(out), out.stride(0), _stream(x))
    return out


LOG2E = 1.4426950408889634


def attention(qkv: torch.Tensor, B: int, S: int, H: int, scale: float, out: torch.Tensor,
              q_prescaled: bool = False) -> torch.Tensor:
    """qkv bf16 [rows, 3*H*64] (q|k|v per token row b*S+s) -> out bf16 [rows, H*64] (or fp16 -> fp16).
    q_prescaled: q already holds q * scale * log2(e) (folded into the projection)."""
    _dev(qkv, out)
    _need(qkv.dtype in H16 and out.dtype == qkv.dtype and qkv.stride(1) == 1 and out.stride(1) == 1,
          "attention dtypes/layout")
    _need(qkv.shape[1] >= 3 * H * 64 and out.shape[1] >= H * 64, "attention columns")
    # the kernel reads K/V rows up to (B-1)*S + roundup(S,64) - 1
    _need(qkv.shape[0] >= (B - 1) * S + (S + 63) // 64 * 64, "attention: qkv needs row padding to a 64-key tile")
    _need(out.shape[0] >= B * S, "attention out rows")
    if qkv.dtype == torch.float16:
        _lib.call("vc_attention_fwd_h16", _p(qkv), qkv.stride(0), B, S, H, 64, scale, int(bool(q_prescaled)), ELEM_F16,
                  _p(out), out.stride(0), _stream(qkv))
    else:
        _lib.call("vc_attention_fwd", _p(qkv), qkv.stride(0), B, S, H, 64, scale, int(bool(q_prescaled)), _p(out),
                  out.stride(0), _stream(qkv))
    return out


def spin(iters: int, device, blocks: int = 1) -> None:
    """`blocks` one-wave workgroups sleeping `iters` x s_sleep 127 each, on the current stream of `device`
    (streams.pick_streams)."""
    _lib.call("vc_spin", int(iters), int(blocks), torch.cuda.current_stream(device).cuda_stream)


def cls_init(cls: torch.Tensor, pos: torch.Tensor, x: torch.Tensor, B: int, S: int) -> torch.Tensor:
    _dev(cls, pos, x)
    D = cls.numel()
    _need(x.dtype == torch.float32 and x.shape[0] >= B * S and x.shape[1] >= D, "cls_init x")
    _lib.call("vc_cls_init", _p(cls), _p(pos), _p(x), x.stride(0), B, S, D, _stream(x))
    return x


def cls_head(x: torch.Tensor, B: int, S: int, gamma, beta, eps: float, wc: torch.Tensor, bc: torch.Tensor,
             out: torch.Tensor | None = None) -> torch.Tensor:
    _dev(x, gamma, beta, wc, bc)
    D = gamma.numel()
    nl = wc.shape[0]
    _need(wc.dtype == torch.float32 and wc.is_contiguous() and wc.shape[1] == D, "cls_head weight f32 [nl, D]")
    if out is None:
        out = torch.empty((B, nl), dtype=torch.float32, device=x.device)
    _lib.call("vc_cls_head", _p(x), x.stride(0), B, S, D, _p(gamma), _p(beta), eps, _p(wc), _p(bc), nl, _p(out),
              _stream(x))
    return out


def temporal_attention(qkv: torch.Tensor, B: int, P: int, T: int, H: int, scale: float, out: torch.Tensor,
                       q_prescaled: bool = False) -> torch.Tensor:
    """TimeSformer temporal attention on the clip layout (rows b*(1+P*T) + 1 + p*T + t):
    qkv bf16 [rows, 3*H*64] -> out bf16 [rows, H*64] (CLS rows untouched)."""
    _dev(qkv, out)
    _need(qkv.dtype == torch.bfloat16 and out.dtype == torch.bfloat16 and qkv.stride(1) == 1 and out.stride(1) == 1,
          "temporal_attention dtypes/layout")
    _need(qkv.shape[1] >= 3 * H * 64 and out.shape[1] >= H * 64, "temporal_attention columns")
    _need(qkv.shape[0] >= B * (1 + P * T) and out.shape[0] >= B * (1 + P * T), "temporal_attention rows")
    _need(T <= 32, "temporal_attention: T <= 32")
    _lib.call("vc_temporal_attention", _p(qkv), qkv.stride(0), B, P, T, H, 64, scale, int(bool(q_prescaled)), _p(out),
              out.stride(0), _stream(qkv))
    return out


DIVIDED_MODE = {"temporal_to_spatial": 0, "spatial_to_mlp": 1}


def divided_add_layernorm(x: torch.Tensor, y: torch.Tensor, B: int, P: int, T: int, gamma, beta, eps: float,
                          mode: str, h: torch.Tensor) -> torch.Tensor:
    """Residual add + LayerNorm across the TimeSformer clip / frame layouts (see include/vclip.h)."""
    _dev(x, y, gamma, beta, h)
    D = gamma.numel()
    _need(x.dtype == torch.float32 and y.dtype == torch.bfloat16 and h.dtype == torch.bfloat16, "divided_add_ln dtypes")
    _need(x.stride(1) == 1 and y.stride(1) == 1 and h.stride(1) == 1 and D % 4 == 0 and D <= 1024, "divided_add_ln")
    rows_c, rows_f = B * (1 + P * T), B * T * (1 + P)
    _need(x.shape[0] >= rows_c and x.shape[1] >= D and y.shape[1] >= D and h.shape[1] >= D, "divided_add_ln shapes")
    if mode == "temporal_to_spatial":
        _need(y.shape[0] >= rows_c and h.shape[0] >= rows_f, "divided_add_ln rows")
    else:
        _need(y.shape[0] >= rows_f and h.shape[0] >= rows_c, "divided_add_ln rows")
    _lib.call("vc_divided_add_layernorm", _p(x), x.stride(0), _p(y), y.stride(0), B, P, T, D, _p(gamma), _p(beta), eps,
              DIVIDED_MODE[mode], _p(h), h.stride(0), _stream(x))
    return h


def window_attention3d(qkv: torch.Tensor, B: int, grid, heads: int, window, shift, biasT: torch.Tensor,
                       out: torch.Tensor, lse: torch.Tensor | None = None) -> torch.Tensor:
    """Swin 3D shifted-window attention (head_dim 32) on the token layout [B][T][H][W]:
    qkv bf16 [>= B*T*H*W, >= 3*heads*32] (q pre-scaled by d^-1/2 * log2 e) -> out bf16 [rows,
    >= heads*32].  biasT: the f32 accumulator-fragment bias of swin3d.expand_bias (the bias as
    the QK^T C operand; also the train-step form with `lse`), or the fp16 operand-fragment bias
    of swin3d.expand_bias_mb (inference: bias and shift mask on the matrix pipe,
    vc_window_attention3d_mb).  See include/vclip.h."""
    _dev(qkv, biasT, out)
    T, H, W = grid
    wt, wh, ww = window
    st, sh, sw = shift
    vol = wt * wh * ww
    np_ = (vol + 63) // 64 * 64
    _need(qkv.dtype == torch.bfloat16 and out.dtype == torch.bfloat16 and qkv.stride(1) == 1 and out.stride(1) == 1,
          "window_attention3d dtypes")
    _need(biasT.dtype in (torch.float32, torch.float16) and biasT.is_contiguous() and biasT.numel() == heads * np_ * np_,
          "window_attention3d bias: f32 (swin3d.expand_bias) or fp16 (swin3d.expand_bias_mb) table of heads*np*np")
    _need(qkv.shape[0] >= B * T * H * W and out.shape[0] >= B * T * H * W, "window_attention3d rows")
    _need(qkv.shape[1] >= 3 * heads * 32 and out.shape[1] >= heads * 32, "window_attention3d columns")
    _need(T % wt == 0 and H % wh == 0 and W % ww == 0, "window_attention3d: grid must be whole windows")
    if biasT.dtype == torch.float16:
        _need(lse is None, "window_attention3d: the train-step form (lse) takes the f32 bias")
        _lib.call("vc_window_attention3d_mb", _p(qkv), qkv.stride(0), B, T, H, W, heads, 32, wt, wh, ww, st, sh, sw,
                  _p(biasT), np_, _p(out), out.stride(0), _stream(qkv))
        return out
    if lse is not None:  # train step: + base-2 log-sum-exp per (token row, head)
        _dev(lse)
        _need(lse.dtype == torch.float32 and lse.is_contiguous() and lse.numel() >= B * T * H * W * heads,
              "window_attention3d lse: f32 [rows * heads]")
        _lib.call("vc_window_attention3d_lse", _p(qkv), qkv.stride(0), B, T, H, W, heads, 32, wt, wh, ww, st, sh, sw,
                  _p(biasT), np_, _p(out), out.stride(0), _p(lse), _stream(qkv))
        return out
    _lib.call("vc_window_attention3d", _p(qkv), qkv.stride(0), B, T, H, W, heads, 32, wt, wh, ww, st, sh, sw, _p(biasT),
              np_, _p(out), out.stride(0), _stream(qkv))
    return out


def window_attention3d_bwd(qkv: torch.Tensor, out: torch.Tensor, dout: torch.Tensor, lse: torch.Tensor, B: int, grid,
                           heads: int, window, shift, full_window, table: torch.Tensor, dqkv: torch.Tensor,
                           dtable_part: torch.Tensor) -> torch.Tensor:
    """Backward of window_attention3d: dqkv (bf16 rows, d q' | dk | dv) and the per-(window, head)
    bias-table gradient partials dtable_part f32 [B * nwindows, heads, ntab] (sum over dim 0)."""
    _dev(qkv, out, dout, lse, table, dqkv, dtable_part)
    T, H, W = grid
    wt, wh, ww = window
    st, sh, sw = shift
    ft, fh, fw = full_window
    ntab = (2 * ft - 1) * (2 * fh - 1) * (2 * fw - 1)
    nwin = B * (T // wt) * (H // wh) * (W // ww)
    for nm, t in (("qkv", qkv), ("out", out), ("dout", dout), ("dqkv", dqkv)):
        _need(t.dtype == torch.bfloat16 and t.stride(1) == 1 and t.shape[0] >= B * T * H * W, f"window bwd {nm}")
    _need(table.dtype == torch.float32 and table.is_contiguous() and tuple(table.shape) == (ntab, heads),
          "window bwd table: f32 [ntab, heads]")
    _need(dtable_part.dtype == torch.float32 and dtable_part.is_contiguous() and dtable_part.numel() >= nwin * heads * ntab,
          "window bwd dtable_part: f32 [B * nwindows * heads * ntab]")
    _lib.call("vc_window_attention3d_bwd", _p(qkv), qkv.stride(0), _p(out), out.stride(0), _p(dout), dout.stride(0),
              _p(lse), B, T, H, W, heads, 32, wt, wh, ww, st, sh, sw, ft, fh, fw, _p(table), _p(dqkv), dqkv.stride(0),
              _p(dtable_part), _stream(qkv))
    return dqkv


def patch_merge_layernorm(x: torch.Tensor, B: int, grid, C: int, gamma, beta, eps: float,
                          out: torch.Tensor) -> torch.Tensor:
    """x f32 [>= B*T*H*W, >= C] -> out bf16 [>= B*T*ceil(H/2)*ceil(W/2), >= 4C]."""
    _dev(x, gamma, beta, out)
    T, H, W = grid
    _need(x.dtype == torch.float32 and out.dtype == torch.bfloat16 and x.stride(1) == 1 and out.stride(1) == 1,
          "patch_merge dtypes")
    _need(gamma.numel() == 4 * C and out.shape[1] >= 4 * C and x.shape[1] >= C, "patch_merge columns")
    _need(x.shape[0] >= B * T * H * W and out.shape[0] >= B * T * ((H + 1) // 2) * ((W + 1) // 2), "patch_merge rows")
    _lib.call("vc_patch_merge_layernorm", _p(x), x.stride(0), B, T, H, W, C, _p(gamma), _p(beta), eps, _p(out),
              out.stride(0), _stream(x))
    return out


def pool_head(x: torch.Tensor, B: int, ntok: int, gamma, beta, eps: float, wc: torch.Tensor, bc: torch.Tensor,
              out: torch.Tensor | None = None, work: torch.Tensor | None = None) -> torch.Tensor:
    """logits = head(mean over each clip's ntok rows of LN(x)) (Swin3D final norm + avgpool + head)."""
    _dev(x, gamma, beta, wc, bc)
    D = gamma.numel()
    nl = wc.shape[0]
    _need(wc.dtype == torch.float32 and wc.is_contiguous() and wc.shape[1] == D and x.shape[0] >= B * ntok,
          "pool_head shapes")
    if out is None:
        out = torch.empty((B, nl), dtype=torch.float32, device=x.device)
    if work is None or work.numel() < B * 64 * D:
        work = torch.empty(B * 64 * D, dtype=torch.float32, device=x.device)
    _lib.call("vc_pool_head", _p(x), x.stride(0), B, ntok, D, _p(gamma), _p(beta), eps, _p(wc), _p(bc), nl, _p(out),
              _p(work), _stream(x))
    return out


CONV_IN = {"ncthw_f32": 0, "cl_bf16": 1}


def conv_out_size(size, k, s, p):
    return tuple((n + 2 * pp - kk) // ss + 1 for n, kk, ss, pp in zip(size, k, s, p))


def conv3d_im2col(x: torch.Tensor, kind: str, B: int, grid, C: int, kernel, stride, pad, out: torch.Tensor) -> torch.Tensor:
    """im2col of a 3D convolution: x f32 [B,C,T,H,W] (kind "ncthw_f32") or channels-last bf16 rows
    [>= B*T*H*W, >= C] ("cl_bf16") -> out bf16 [>= B*To*Ho*Wo, >= kvol*C]."""
    import ctypes
    _dev(x, out)
    T, H, W = grid
    To, Ho, Wo = conv_out_size(grid, kernel, stride, pad)
    kvol = kernel[0] * kernel[1] * kernel[2]
    _need(out.dtype == torch.bfloat16 and out.stride(1) == 1 and out.shape[0] >= B * To * Ho * Wo and
          out.shape[1] >= kvol * C, "conv3d_im2col out")
    if kind == "ncthw_f32":
        _need(x.dtype == torch.float32 and x.is_contiguous() and tuple(x.shape) == (B, C, T, H, W), "conv3d_im2col x")
        ldx = 0
    else:
        _need(x.dtype == torch.bfloat16 and x.stride(1) == 1 and x.shape[0] >= B * T * H * W and x.shape[1] >= C,
              "conv3d_im2col x")
        ldx = x.stride(0)
    k, s, p = ((ctypes.c_int * 3)(*v) for v in (kernel, stride, pad))
    _lib.call("vc_conv3d_im2col", _p(x), ldx, CONV_IN[kind], B, T, H, W, C, ctypes.addressof(k), ctypes.addressof(s),
              ctypes.addressof(p), _p(out), out.stride(0), _stream(x))
    return out


_ZERO_ROW = {}


def zero_row(device) -> torch.Tensor:
    """The shared 64-element zero bf16 row the implicit convolutions read for padding taps (one per
    device).  Created once, on the caller's stream, which is then waited for: a split forward's parts
    read it from side streams that are ordered only after the caller's stream, so a zero-fill queued on
    one part's stream could still be pending when another part's first conv reads it."""
    z = _ZERO_ROW.get(device)
    if z is None:
        z = torch.zeros(64, dtype=torch.bfloat16, device=device)
        if not torch.cuda.is_current_stream_capturing():
            torch.cuda.current_stream(device).synchronize()
        _ZERO_ROW[device] = z
    return z


def conv3d_gemm(x: torch.Tensor, B: int, grid, C: int, kernel, stride, pad, w: torch.Tensor, bias: torch.Tensor,
                epilogue: str, out: torch.Tensor, aux: torch.Tensor | None = None, flop: float | None = None,
                op: str = "conv", n: int | None = None, ring: int = 0, tile: int = 0) -> torch.Tensor:
    """Implicit-GEMM Conv3d (vc_conv3d_gemm_bf16): x channels-last bf16 rows [>= B*T*H*W, >= C],
    w bf16 [>= N, >= kvol*C] (columns (kt, kh, kw, c)), out bf16 [>= roundup(B*To*Ho*Wo, 128), >= N]
    (256-row multiples when N % 128 != 0: 256 x 64 tiles); N = n (a multiple of 64) or w's rows."""
    import ctypes
    _dev(x, w, bias, out)
    T, H, W = grid
    To, Ho, Wo = conv_out_size(grid, kernel, stride, pad)
    kvol = kernel[0] * kernel[1] * kernel[2]
    M = B * To * Ho * Wo
    N = w.shape[0] if n is None else n
    rt = 128 if N % 128 == 0 else 256
    _need(x.dtype == torch.bfloat16 and x.stride(1) == 1 and x.shape[0] >= B * T * H * W and x.shape[1] >= C,
          "conv3d_gemm x")
    _need(w.dtype == torch.bfloat16 and w.stride(1) == 1 and w.shape[1] >= kvol * C and w.shape[0] >= N and
          bias.numel() >= N and bias.dtype == torch.float32, "conv3d_gemm weights")
    _need(out.dtype == torch.bfloat16 and out.stride(1) == 1 and out.shape[0] >= (M + rt - 1) // rt * rt and
          out.shape[1] >= N, "conv3d_gemm out rows (a multiple of the tile height)")
    e = EPI[epilogue]
    if e == 7:
        # the tile epilogue reads the residual for every row of the padded tile
        _need(aux is not None and aux.dtype == torch.bfloat16 and aux.stride(1) == 1 and
              aux.shape[0] >= (M + rt - 1) // rt * rt and aux.shape[1] >= N,
              "conv3d_gemm residual (rows up to the tile-height multiple of the output rows)")
    zrow = zero_row(x.device)
    k, s, p = ((ctypes.c_int * 3)(*v) for v in (kernel, stride, pad))
    rec = _REC[0]
    if rec is not None:
        # the label first: nothing but the launch may sit between the two events (a first
        # get_device_properties inside them once timed as an 8-ms launch)
        tl = "256, 64, 8, 1"
        if rt == 128:  # 64 x 128 tiles when the 128 x 128 grid has fewer tiles than CUs (csrc/gemm.hip)
            small = tile == 1 or (tile == 0 and ((M + 127) // 128) * (N // 128) < _num_cus(x.device) and e in (0, 6))
            tl = "64, 128, 2, 4" if small else "128, 128, 2, 4"
        nt = (((M + 127) // 128) * (N // 128) if tl == "128, 128, 2, 4" else ((M + 63) // 64) * (N // 128)
              if tl == "64, 128, 2, 4" else ((M + 255) // 256) * (N // 64))
        cus = _num_cus(x.device)  # csrc/gemm.hip pick_ring (128 x 128: 3-deep only within one round of CUs)
        st = ring if ring else (3 if (nt <= cus if tl == "128, 128, 2, 4" else nt < 2 * cus) else 2)
        if st == 4 and rt != 128:
            st = 3
        label = f"conv_gemm_kernel<{tl}, {e}, {st}, 0>"
    e0 = rec.begin() if rec is not None else None
    _lib.call("vc_conv3d_gemm_bf16_cfg", _p(x), x.stride(0), B, T, H, W, C, ctypes.addressof(k), ctypes.addressof(s),
              ctypes.addressof(p), _p(zrow), _p(w), w.stride(0), N, _p(bias), e, _p(out), out.stride(0),
              _p(aux) if aux is not None else None, aux.stride(0) if aux is not None else 0, ring, tile, _stream(x))
    if rec is not None:
        rec.end(e0, label, op, 2.0 * M * N * kvol * C if flop is None else flop, "flop")
    return out


def conv3d_stem_pack(x: torch.Tensor, pad, out: torch.Tensor) -> torch.Tensor:
    """f32 clip [B, C<=4, T, H, W] -> zero-padded channels-last bf16 [B, T+2pt, H+2ph, W+2pw, 4] (out, any
    shape with that many contiguous elements)."""
    import ctypes
    _dev(x, out)
    B, C, T, H, W = x.shape
    _need(x.dtype == torch.float32 and x.is_contiguous() and C <= 4, "conv3d_stem_pack x")
    _need(out.dtype == torch.bfloat16 and out.is_contiguous() and
          out.numel() >= B * (T + 2 * pad[0]) * (H + 2 * pad[1]) * (W + 2 * pad[2]) * 4, "conv3d_stem_pack out")
    p = (ctypes.c_int * 3)(*pad)
    _lib.call("vc_conv3d_stem_pack", _p(x), B, C, T, H, W, ctypes.addressof(p), _p(out), _stream(x))
    return out


def conv3d_stem_gemm(xp: torch.Tensor, B: int, grid, kernel, stride, pad, w: torch.Tensor, bias: torch.Tensor,
                     epilogue: str, out: torch.Tensor, flop: float | None = None, op: str = "stem",
                     n: int | None = None) -> torch.Tensor:
    """The stem Conv3d as an implicit GEMM over conv3d_stem_pack's padded clip (vc_conv3d_stem_gemm_bf16);
    w bf16 [N, >= 64 * ceil(kt*kh/2)] in the segment column order, out bf16 [>= roundup(M, 128), >= N]."""
    import ctypes
    _dev(xp, w, bias, out)
    T, H, W = grid
    To, Ho, Wo = conv_out_size(grid, kernel, stride, pad)
    M = B * To * Ho * Wo
    N = w.shape[0] if n is None else n
    rt = 128 if N % 128 == 0 else 256
    K = 64 * ((kernel[0] * kernel[1] + 1) // 2)
    _need(xp.dtype == torch.bfloat16 and xp.is_contiguous(), "conv3d_stem_gemm xp")
    _need(w.dtype == torch.bfloat16 and w.stride(1) == 1 and w.shape[1] >= K and w.shape[0] >= N and
          bias.numel() >= N and bias.dtype == torch.float32, "conv3d_stem_gemm weights")
    _need(out.dtype == torch.bfloat16 and out.stride(1) == 1 and out.shape[0] >= (M + rt - 1) // rt * rt and
          out.shape[1] >= N, "conv3d_stem_gemm out")
    # each (kt, kh) tap row is read as 8 pixels x 4 channels from a 16-B aligned start: an even padded width,
    # and the last output's window (8 pixels from 2 wo) inside the packed clip
    Tp, Hp, Wp = T + 2 * pad[0], H + 2 * pad[1], W + 2 * pad[2]
    _need(Wp % 2 == 0 and stride[2] % 2 == 0, "conv3d_stem_gemm: the padded width must be even (16-B aligned "
          "8-pixel reads; the forward takes the im2col stem otherwise)")
    last = ((((B - 1) * Tp + (To - 1) * stride[0] + kernel[0] - 1) * Hp + (Ho - 1) * stride[1] + kernel[1] - 1) * Wp
            + (Wo - 1) * stride[2] + 8) * 4
    _need(xp.numel() >= last, "conv3d_stem_gemm: the packed clip ends before the last window's 8-pixel read")
    zrow = zero_row(xp.device)
    k, s, p = ((ctypes.c_int * 3)(*v) for v in (kernel, stride, pad))
    rec = _REC[0]
    e0 = rec.begin() if rec is not None else None
    e = EPI[epilogue]
    _lib.call("vc_conv3d_stem_gemm_bf16", _p(xp), B, T, H, W, ctypes.addressof(k), ctypes.addressof(s),
              ctypes.addressof(p), _p(zrow), _p(w), w.stride(0), N, _p(bias), e, _p(out), out.stride(0),
              _stream(xp))
    if rec is not None:
        tile = "128, 128, 2, 4" if rt == 128 else "256, 64, 8, 1"
        rec.end(e0, f"conv_gemm_kernel<{tile}, {e}, 2, 1>", op, 2.0 * M * N * K if flop is None else flop, "flop")
    return out


def maxpool3d(x: torch.Tensor, B: int, grid, C: int, kernel, stride, pad, out: torch.Tensor) -> torch.Tensor:
    import ctypes
    _dev(x, out)
    To, Ho, Wo = conv_out_size(grid, kernel, stride, pad)
    T, H, W = grid
    _need(x.dtype == torch.bfloat16 and out.dtype == torch.bfloat16 and x.shape[0] >= B * T * H * W and
          out.shape[0] >= B * To * Ho * Wo and x.shape[1] >= C and out.shape[1] >= C, "maxpool3d shapes")
    k, s, p = ((ctypes.c_int * 3)(*v) for v in (kernel, stride, pad))
    _lib.call("vc_maxpool3d", _p(x), x.stride(0), B, T, H, W, C, ctypes.addressof(k), ctypes.addressof(s),
              ctypes.addressof(p), _p(out), out.stride(0), _stream(x))
    return out


def avgpool_head(x: torch.Tensor, B: int, grid, C: int, pool_kernel, wc: torch.Tensor, bc: torch.Tensor,
                 work: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
    import ctypes
    _dev(x, wc, bc, work, out)
    T, H, W = grid
    nl = wc.shape[0]
    _need(x.dtype == torch.bfloat16 and x.shape[0] >= B * T * H * W and x.shape[1] >= C, "avgpool_head x")
    _need(wc.dtype == torch.float32 and wc.is_contiguous() and wc.shape[1] == C and work.numel() >= B * C * 33 and
          out.shape == (B, nl), "avgpool_head shapes")
    pk = (ctypes.c_int * 3)(*pool_kernel)
    _lib.call("vc_avgpool_head", _p(x), x.stride(0), B, T, H, W, C, ctypes.addressof(pk), _p(wc), _p(bc), nl,
              _p(work), _p(out), _stream(x))
    return out


# ---- train step -----------------------------------------------------------

def attention_fwd_lse(qkv: torch.Tensor, B: int, S: int, H: int, out: torch.Tensor, lse: torch.Tensor,
                      scale: float = 0.125, q_prescaled: bool = True) -> torch.Tensor:
    """vc_attention_fwd that also stores the base-2 log-sum-exp lse f32 [B*H*S]."""
    _dev(qkv, out, lse)
    _need(lse.dtype == torch.float32 and lse.is_contiguous() and lse.numel() >= B * H * S, "lse: f32 [B*H*S]")
    _need(qkv.dtype == torch.bfloat16 and out.dtype == torch.bfloat16 and qkv.stride(1) == 1 and out.stride(1) == 1,
          "attention dtypes/layout")
    _need(qkv.shape[1] >= 3 * H * 64 and out.shape[1] >= H * 64, "attention columns")
    _need(qkv.shape[0] >= (B - 1) * S + (S + 63) // 64 * 64, "attention: qkv needs row padding to a 64-key tile")
    _need(out.shape[0] >= B * S, "attention out rows")
    _lib.call("vc_attention_fwd_lse", _p(qkv), qkv.stride(0), B, S, H, 64, scale, int(bool(q_prescaled)), _p(out),
              out.stride(0), _p(lse), _stream(qkv))
    return out


def attention_bwd(qkv: torch.Tensor, out: torch.Tensor, dout: torch.Tensor, lse: torch.Tensor, delta: torch.Tensor,
                  B: int, S: int, H: int, dqkv: torch.Tensor, stream2: torch.cuda.Stream | None = None) -> torch.Tensor:
    """dqkv (q part = dL/dq' of the stored pre-scaled q', then dk, dv) of the joint attention.
    `stream2`: the dQ kernel runs there beside dK/dV (vc_attention_bwd_2s); the current stream waits
    for it before anything enqueued after this call."""
    _dev(qkv, out, dout, lse, delta, dqkv)
    for t, nm in ((qkv, "qkv"), (out, "out"), (dout, "dout"), (dqkv, "dqkv")):
        _need(t.dtype == torch.bfloat16 and t.stride(1) == 1, f"attention_bwd: {nm} bf16 with unit column stride")
    _need(lse.dtype == torch.float32 and delta.dtype == torch.float32 and lse.numel() >= B * H * S and
          delta.numel() >= B * H * S, "attention_bwd: lse / delta f32 [B*H*S]")
    pad = (B - 1) * S + (S + 63) // 64 * 64
    _need(qkv.shape[0] >= pad and dout.shape[0] >= pad, "attention_bwd: qkv / dout need row padding to a 64-row tile")
    _need(out.shape[0] >= B * S and dqkv.shape[0] >= B * S, "attention_bwd rows")
    _need(qkv.shape[1] >= 3 * H * 64 and dqkv.shape[1] >= 3 * H * 64 and out.shape[1] >= H * 64 and
          dout.shape[1] >= H * 64, "attention_bwd columns")
    if stream2 is not None:
        _lib.call("vc_attention_bwd_2s", _p(qkv), qkv.stride(0), _p(out), out.stride(0), _p(dout), dout.stride(0),
                  _p(lse), _p(delta), B, S, H, 64, _p(dqkv), dqkv.stride(0), _stream(qkv), stream2.cuda_stream)
        return dqkv
    _lib.call("vc_attention_bwd", _p(qkv), qkv.stride(0), _p(out), out.stride(0), _p(dout), dout.stride(0), _p(lse),
              _p(delta), B, S, H, 64, _p(dqkv), dqkv.stride(0), _stream(qkv))
    return dqkv


def layernorm_bwd(dy: torch.Tensor, x: torch.Tensor, gamma: torch.Tensor, eps: float, dx: torch.Tensor,
                  dxb: torch.Tensor, dgamma: torch.Tensor, dbeta: torch.Tensor, work: torch.Tensor,
                  m: int | None = None, dsum_in: torch.Tensor | None = None,
                  dsum_out: torch.Tensor | None = None) -> torch.Tensor:
    """dx += LayerNorm backward of dy (f32, in place), dxb = bf16(dx); dgamma / dbeta overwritten;
    optional dsum_in / dsum_out = column sums of dx before / after (bias gradients)."""
    _dev(dy, x, gamma, dx, dxb, dgamma, dbeta, work)
    M = x.shape[0] if m is None else m
    D = gamma.numel()
    _need(dy.dtype == torch.float32 and x.dtype == torch.float32 and dx.dtype == torch.float32 and
          dxb.dtype == torch.bfloat16 and work.dtype == torch.float32, "layernorm_bwd dtypes")
    _need(all(t.shape[0] >= M and t.shape[1] >= D and t.stride(1) == 1 for t in (dy, x, dx, dxb)), "layernorm_bwd shapes")
    _need(dgamma.numel() == D and dbeta.numel() == D and dgamma.is_contiguous() and dbeta.is_contiguous(),
          "layernorm_bwd dgamma/dbeta")
    _need((dsum_in is None) == (dsum_out is None), "layernorm_bwd: dsum_in and dsum_out go together")
    if dsum_in is not None:
        _dev(dsum_in, dsum_out)
        _need(all(t.dtype == torch.float32 and t.is_contiguous() and t.numel() == D for t in (dsum_in, dsum_out)),
              "layernorm_bwd dsum_in / dsum_out f32 [D]")
    _lib.call("vc_layernorm_bwd", _p(dy), dy.stride(0), _p(x), x.stride(0), M, D, _p(gamma), eps, _p(dx), dx.stride(0),
              _p(dxb), dxb.stride(0), _p(dgamma), _p(dbeta), _p(dsum_in) if dsum_in is not None else None,
              _p(dsum_out) if dsum_out is not None else None, _p(work), work.numel(), _stream(x))
    return dx


def colsum(x: torch.Tensor, out: torch.Tensor, work: torch.Tensor | None = None, m: int | None = None,
           nscaled: int = 0, scale: float = 1.0) -> torch.Tensor:
    """out[n] = s(n) * sum over the first m rows of x[:, n] (x f32 or bf16 2-D, unit column stride)."""
    _dev(x, out)
    R = x.shape[0] if m is None else m
    N = out.numel()
    _need(x.dtype in (torch.float32, torch.bfloat16) and x.dim() == 2 and x.stride(1) == 1 and x.shape[1] >= N and
          x.shape[0] >= R, "colsum input")
    _need(out.dtype == torch.float32 and out.is_contiguous(), "colsum out f32")
    wp, wn = (_p(work), work.numel()) if work is not None else (None, 0)
    _lib.call("vc_colsum", _p(x), 0 if x.dtype == torch.float32 else 1, x.stride(0), R, N, nscaled, scale, _p(out), wp,
              wn, _stream(x))
    return out


def colsum_work(R: int, N: int, device) -> torch.Tensor:
    """Scratch for vc_colsum's full row split (S1 + S2 partial rows of N floats)."""
    s1 = min(2048, max(1, (R + 63) // 64))
    return torch.empty((s1 + (s1 + 63) // 64) * N, dtype=torch.float32, device=device)


def wgrad_work(M: int, N1: int, N2: int, device) -> torch.Tensor:
    """Scratch for vc_wgrad_bf16's split-K partials at the split count the kernel aims for
    (train.hip vc_wgrad_bf16: ~512 workgroups of 128 x 128, ~256 of 256 x 256)."""
    if N1 % 256 == 0 and N2 % 256 == 0:
        sp = min(-(-256 // ((N1 // 256) * (N2 // 256))), (M // 32) // 4)
    else:
        sp = min(-(-512 // ((N1 // 128) * (N2 // 128))), (M // 64) // 2)
    return torch.empty(max(2, sp) * N1 * N2, dtype=torch.float32, device=device)


def wgrad_kernel_name(M: int, N1: int, N2: int, work_elems: int) -> str:
    """The rocprofv3 name of the kernel vc_wgrad_bf16 runs for this call: csrc/train.hip's own plan
    (vc_wgrad_pick: split count from the device's CU count and the scratch size, then the ping-pong kernel
    when every split has >= 3 32-row half-tiles, unless VCLIP_WGRAD_PP=0)"""
    k = _lib.load().vc_wgrad_pick(M, N1, N2, work_elems) & 15
    return {0: "trn::wgrad_kernel", 1: "trn::wgrad_big_kernel", 2: "trn::wgrad_pp_kernel"}[k]


def wgrad(g: torch.Tensor, x: torch.Tensor, out: torch.Tensor, work: torch.Tensor | None = None,
          nscaled: int = 0, scale: float = 1.0, m: int | None = None) -> torch.Tensor:
    """out[n1][n2] = s(n1) * sum_m g[m][n1] x[m][n2]  (g bf16 [M, N1], x bf16 [M, N2], out f32 [N1, N2])."""
    _dev(g, x, out)
    M = g.shape[0] if m is None else m
    N1, N2 = out.shape
    _need(g.dtype == torch.bfloat16 and x.dtype == torch.bfloat16 and out.dtype == torch.float32, "wgrad dtypes")
    _need(g.stride(1) == 1 and x.stride(1) == 1 and out.stride(1) == 1 and g.shape[1] >= N1 and x.shape[1] >= N2 and
          g.shape[0] >= M and x.shape[0] >= M, "wgrad shapes")
    wp, wn = (_p(work), work.numel()) if work is not None else (None, 0)
    rec = _REC[0]
    if rec is not None:  # one entry per vc_wgrad_bf16 call: the split-K kernel plus its partial reduction
        label = wgrad_kernel_name(M, N1, N2, wn) + " (+ wgrad_reduce_kernel)"
        e0 = rec.begin()
    _lib.call("vc_wgrad_bf16", _p(g), g.stride(0), _p(x), x.stride(0), M, N1, N2, nscaled, scale, _p(out),
              out.stride(0), wp, wn, _stream(g))
    if rec is not None:
        rec.end(e0, label, "wgrad", 2.0 * M * N1 * N2, "flop")
    return out


def cls_head_bwd(x, B, S, gamma, beta, eps, wc, dlogits, dx, dxb, dwc, dbc, dgamma, dbeta):
    _dev(x, gamma, beta, wc, dlogits, dx, dxb, dwc, dbc, dgamma, dbeta)
    D = gamma.numel()
    nl = wc.shape[0]
    _need(dlogits.dtype == torch.float32 and dlogits.is_contiguous() and tuple(dlogits.shape) == (B, nl),
          "cls_head_bwd dlogits f32 [B, nl]")
    _need(x.shape[0] >= B * S and dx.shape[0] >= B * S and dxb.shape[0] >= B * S, "cls_head_bwd rows")
    _lib.call("vc_cls_head_bwd", _p(x), x.stride(0), B, S, D, _p(gamma), _p(beta), eps, _p(wc), nl, _p(dlogits),
              _p(dx), dx.stride(0), _p(dxb), dxb.stride(0), _p(dwc), _p(dbc), _p(dgamma), _p(dbeta), _stream(x))


def embed_bwd(dx: torch.Tensor, B: int, S: int, dpos: torch.Tensor, dcls: torch.Tensor, demb: torch.Tensor):
    _dev(dx, dpos, dcls, demb)
    D = dcls.numel()
    _need(dx.dtype == torch.float32 and dx.shape[0] >= B * S and dx.stride(1) == 1, "embed_bwd dx")
    _need(dpos.dtype == torch.float32 and dpos.is_contiguous() and dpos.numel() == S * D, "embed_bwd dpos")
    _need(demb.dtype == torch.bfloat16 and demb.shape[0] >= B * (S - 1) and demb.shape[1] >= D and demb.stride(1) == 1,
          "embed_bwd demb")
    _lib.call("vc_embed_bwd", _p(dx), dx.stride(0), B, S, D, _p(dpos), _p(dcls), _p(demb), demb.stride(0), _stream(dx))


def adamw(param, grad, exp_avg, exp_avg_sq, lr, beta1, beta2, eps, weight_decay, step, grad_scale=1.0):
    _dev(param, grad, exp_avg, exp_avg_sq)
    n = param.numel()
    _need(all(t.dtype == torch.float32 and t.is_contiguous() and t.numel() == n for t in
              (param, grad, exp_avg, exp_avg_sq)), "adamw: contiguous f32 buffers of one size")
    _lib.call("vc_adamw", _p(param), _p(grad), _p(exp_avg), _p(exp_avg_sq), n, lr, beta1, beta2, eps, weight_decay,
              int(step), grad_scale, _stream(param))


def adamw_step_table(beta1: float, beta2: float, lr: float, steps: int, device) -> torch.Tensor:
    """Device f32 [steps, 2]: row t-1 = (lr / (1 - beta1^t), sqrt(1 - beta2^t)) exactly as vc_adamw derives them
    for step t (vc_adamw_step_table computes them in the library with the same double arithmetic)."""
    import numpy as np
    host = np.zeros((steps, 2), dtype=np.float32)
    _lib.call("vc_adamw_step_table", beta1, beta2, lr, steps, host.ctypes.data)
    return torch.from_numpy(host).to(device)


def adamw_tab(param, grad, exp_avg, exp_avg_sq, lr, beta1, beta2, eps, weight_decay, tab, counter, grad_scale=1.0):
    """adamw() with the step on the device: step = counter + 1 (int64 [1] device tensor), constants from tab
    (adamw_step_table); the counter is not advanced here (adamw_step_tick)."""
    _dev(param, grad, exp_avg, exp_avg_sq, tab, counter)
    n = param.numel()
    _need(all(t.dtype == torch.float32 and t.is_contiguous() and t.numel() == n for t in
              (param, grad, exp_avg, exp_avg_sq)), "adamw_tab: contiguous f32 buffers of one size")
    _need(tab.dtype == torch.float32 and tab.is_contiguous() and tab.dim() == 2 and tab.shape[1] == 2 and
          counter.dtype == torch.int64 and counter.numel() >= 1, "adamw_tab: tab f32 [steps, 2], counter int64")
    _lib.call("vc_adamw_tab", _p(param), _p(grad), _p(exp_avg), _p(exp_avg_sq), n, lr, beta1, beta2, eps,
              weight_decay, _p(tab), _p(counter), tab.shape[0], grad_scale, _stream(param))


def adamw_step_tick(counter: torch.Tensor):
    _dev(counter)
    _need(counter.dtype == torch.int64, "adamw_step_tick: int64 counter")
    _lib.call("vc_adamw_step_tick", _p(counter), _stream(counter))


def adamw_multi(params, grads, exp_avgs, exp_avg_sqs, lr, beta1, beta2, eps, weight_decay, step, grad_scale=1.0):
    """vc_adamw on every (param, grad, exp_avg, exp_avg_sq) quadruple in one launch."""
    rows, c0 = [], 0
    for p, g, m, v in zip(params, grads, exp_avgs, exp_avg_sqs):
        _dev(p, g, m, v)
        n = p.numel()
        _need(all(t.dtype == torch.float32 and t.is_contiguous() and t.numel() == n for t in (p, g, m, v)),
              "adamw_multi: contiguous f32 buffers of one size per entry")
        rows.append([p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), n, c0])
        c0 += (n + 1023) // 1024
    if not rows:
        return
    # the device table is cached by content: in a steady training loop the caching allocator hands
    # the gradients the same addresses every step, so the table is uploaded once (a host -> device
    # copy per step would synchronise the host with the stream)
    key = tuple(x for r in rows for x in r[:5])
    tab = _ADAMW_TABLES.get(key)
    if tab is None or tab.device != params[0].device:
        if len(_ADAMW_TABLES) >= 8:
            _ADAMW_TABLES.clear()
        tab = _ADAMW_TABLES[key] = torch.tensor(rows, dtype=torch.int64).to(params[0].device)
    _lib.call("vc_adamw_multi", _p(tab), len(rows), c0, lr, beta1, beta2, eps, weight_decay, int(step), grad_scale,
              _stream(params[0]))
    return tab


_ADAMW_TABLES = {}


def pack_weight(src: torch.Tensor, dst: torch.Tensor | None = None, dst_t: torch.Tensor | None = None,
                nscaled: int = 0, scale: float = 1.0):
    _dev(src)
    N, K = src.shape
    _need(src.dtype == torch.float32 and src.is_contiguous(), "pack_weight src f32 contiguous [N, K]")
    if dst is not None:
        _need(dst.dtype == torch.bfloat16 and dst.is_contiguous() and tuple(dst.shape) == (N, K), "pack_weight dst")
    if dst_t is not None:
        _need(dst_t.dtype == torch.bfloat16 and dst_t.is_contiguous() and tuple(dst_t.shape) == (K, N), "pack_weight dst_t")
    _lib.call("vc_pack_weight", _p(src), N, K, nscaled, scale, _p(dst) if dst is not None else None,
              _p(dst_t) if dst_t is not None else None, _stream(src))
