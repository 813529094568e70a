"""ORACLE — test infrastructure only.  numpy restatements of the byte/layout work:

* frame gather: `frames[clip][clamp(idx)]` exactly as the reference dataset picks the
  sampled frames out of a decoded clip (vivit_transformer/vivit_classifier/data_config/
  dataset.py:248-255, positions clamped to the decoded range), optionally followed by the
  ViViT processor affine x*(1/63.75) - 3 and the [T,H,W,C] -> [T,C,H,W] stack
  (trainer.py:62-95; VivitImageProcessor rescale(1/127.5, offset) + normalize(0.5, 0.5));
* tubelet im2col: the Conv3d k=s=(2,16,16) patch extraction of
  TF5/models/vivit/modeling_vivit.py:64-67 (token order t,h,w; column order c,kt,kh,kw).
"""
import numpy as np


def gather_u8(frames, idx):
    """frames u8 [N,F,H,W,C], idx int [N,T] -> u8 [N,T,H,W,C]."""
    N, F = frames.shape[:2]
    idx = np.clip(np.asarray(idx, dtype=np.int64), 0, F - 1)
    return np.stack([frames[n][idx[n]] for n in range(N)])


def gather_norm(frames, idx, scale=np.float32(1.0 / 63.75), shift=np.float32(-3.0)):
    """-> f32 [N,T,C,H,W] = x*scale + shift computed in fp32 (single rounding per op)."""
    g = gather_u8(frames, idx).astype(np.float32)
    y = g * np.float32(scale) + np.float32(shift)
    return np.ascontiguousarray(y.transpose(0, 1, 4, 2, 3))


def tubelet_im2col(pix, tubelet=(2, 16, 16), order="time_major"):
    """pix f32 [B,T,C,H,W] -> [B*nt*nh*nw, C*kt*kh*kw] (same dtype).  Token rows in (t',hp,wp)
    order (ViViT Conv3d flatten, modeling_vivit.py:64-67) or, order="patch_major", (hp,wp,t')
    (TimeSformer per-frame Conv2d + patch-major re-order, modeling_timesformer.py:121-143)."""
    B, T, C, H, W = pix.shape
    kt, kh, kw = tubelet
    x = pix.reshape(B, T // kt, kt, C, H // kh, kh, W // kw, kw)
    # -> B, nt, nh, nw, C, kt, kh, kw   (or B, nh, nw, nt, ... for patch-major)
    x = x.transpose(0, 1, 4, 6, 3, 2, 5, 7) if order == "time_major" else x.transpose(0, 4, 6, 1, 3, 2, 5, 7)
    return np.ascontiguousarray(x.reshape(B * (T // kt) * (H // kh) * (W // kw), C * kt * kh * kw))


def pil_resize_emulated(img, out_hw, coeffs):
    """Pillow BILINEAR resize of one uint8 image [H, W, C] restated in numpy integer arithmetic
    (Resample.c: horizontal pass, then vertical, each accumulating from 1 << 21 with 22-bit
    fixed-point coefficients and clip8).  `coeffs(in, out)` -> (bounds, coef, ksize)."""
    H, W, C = img.shape
    H2, W2 = out_hw

    def pas(x, axis, n_in, n_out):
        b, c, _ = coeffs(n_in, n_out)
        shape = list(x.shape)
        shape[axis] = n_out
        out = np.zeros(shape, np.int64)
        for o in range(n_out):
            s = np.full([d for i, d in enumerate(x.shape) if i != axis], 1 << 21, np.int64)
            for t in range(b[o, 1]):
                s = s + np.take(x, b[o, 0] + t, axis=axis) * int(c[o, t])
            if axis == 0:
                out[o] = s
            else:
                out[:, o] = s
        return np.where(out >= (1 << 30), 255, np.where(out <= 0, 0, out >> 22))

    x = img.astype(np.int64)
    if W2 != W:
        x = pas(x, 1, W, W2)
    if H2 != H:
        x = pas(x, 0, H, H2)
    return x.astype(np.uint8)
