"""OpenCV `cv2.resize(frame, (W, H))` (INTER_LINEAR, uint8) restated, host side.

The reference resizes decoded frames that are not 224x224 with cv2's default INTER_LINEAR
(vivit_transformer/vivit_classifier/data_config/dataset.py:271-277, :348;
vivit_transformer/inference.py:155).  cv2 is not in this image, so this is a
restatement of OpenCV's published resize (modules/imgproc/src/resize.cpp, 4.x), parity unpinned:

* coefficient tables (`resize` -> `resizeGeneric_`): for destination column dx,
  fx = float((dx + 0.5) * scale_x - 0.5), sx = floor(fx), fx -= sx; sx < 0 -> (sx, fx) = (0, 0);
  sx >= W_src - 1 -> (sx, fx) = (W_src - 1, 0); alpha = (round(2048 (1 - fx)), 2048 - that) —
  11-bit fixed point (INTER_RESIZE_COEF_BITS); rows likewise;
* horizontal pass (HResizeLinear): int row = S[sx] a0 + S[sx + cn] a1, or S[sx] * 2048 past the
  last column pair;
* vertical pass as the SIMD kernel VResizeLinearVec_32s8u runs it on every x86 / ARM build:
  out = (((row0 >> 4) * b0 >> 16) + ((row1 >> 4) * b1 >> 16) + 2) >> 2, saturated to uint8;
* an exact 2x downscale in both axes takes INTER_AREA's fast path instead (cv2.resize switches
  INTER_LINEAR to it): out = (a + b + c + d + 2) >> 2 over each 2x2 block.

The GPU kernel `vc_resize_linear_u8` (csrc/preprocess.hip) computes the same integers; both are
checked against the pure-Python loop restatement in oracle/cv2_resize_ref.py.
"""
from __future__ import annotations

import numpy as np

COEF_BITS = 11
COEF_SCALE = 1 << COEF_BITS


def linear_tables(src: int, dst: int, clamp: bool = True):
    """One axis of the coefficient tables: (offsets int32 [dst], a0 int32 [dst], a1 int32 [dst],
    limit).  Columns (clamp=True) get OpenCV's border handling: sx < 0 -> (0, fx=0), sx >= src-1
    -> (src-1, fx=0), and every column from `limit` on is the copy S[sx] * 2048.  Rows
    (clamp=False) keep sx and fy as computed; the row fetch clamps sy and sy+1 to [0, src-1]."""
    scale = 1.0 / (dst / src)  # cv2: inv_scale = dst / src (double), scale = 1 / inv_scale
    ofs = np.zeros(dst, np.int32)
    a0 = np.zeros(dst, np.int32)
    a1 = np.zeros(dst, np.int32)
    limit = dst
    one = np.float32(1.0)
    k = np.float32(COEF_SCALE)
    for d in range(dst):
        f = np.float32((d + 0.5) * scale - 0.5)
        s = int(np.floor(f))
        f = np.float32(f - np.float32(s))
        if clamp:
            if s < 0:
                f, s = np.float32(0.0), 0
            if s + 1 >= src:
                limit = min(limit, d)
                if s >= src - 1:
                    f, s = np.float32(0.0), src - 1
        ofs[d] = s
        # saturate_cast<short>(cbuf[k] * 2048): cvRound, ties to even
        a0[d] = int(np.rint(np.float32(one - f) * k))
        a1[d] = int(np.rint(np.float32(f * k)))
    return ofs, a0, a1, limit


def is_area_fast_2x(src_hw, dst_hw) -> bool:
    (sh, sw), (dh, dw) = src_hw, dst_hw
    return sh == 2 * dh and sw == 2 * dw


def resize_linear_u8(frames: np.ndarray, size) -> np.ndarray:
    """frames uint8 [..., H, W, C] -> [..., h, w, C] with size = (w, h) as cv2.resize takes it."""
    w, h = int(size[0]), int(size[1])
    f = np.asarray(frames)
    if f.dtype != np.uint8:
        raise ValueError("resize_linear_u8: uint8 frames expected")
    H, W = f.shape[-3], f.shape[-2]
    if (H, W) == (h, w):
        return f.copy()
    if is_area_fast_2x((H, W), (h, w)):
        x = f.astype(np.int32)
        s = x[..., 0::2, 0::2, :] + x[..., 0::2, 1::2, :] + x[..., 1::2, 0::2, :] + x[..., 1::2, 1::2, :]
        return ((s + 2) >> 2).astype(np.uint8)
    xo, xa0, xa1, xlim = linear_tables(W, w, clamp=True)
    yo, yb0, yb1, _ = linear_tables(H, h, clamp=False)
    x = f.astype(np.int32)
    xo1 = np.minimum(xo + 1, W - 1)
    # horizontal pass on every source row (HResizeLinear)
    rows = x[..., xo, :] * xa0[:, None] + x[..., xo1, :] * xa1[:, None]
    if xlim < w:
        rows[..., xlim:, :] = x[..., xo[xlim:], :] * COEF_SCALE
    # vertical pass (VResizeLinearVec_32s8u rounding), rows clip(sy) / clip(sy + 1)
    r0 = rows[..., np.clip(yo, 0, H - 1), :, :] >> 4
    r1 = rows[..., np.clip(yo + 1, 0, H - 1), :, :] >> 4
    b0 = yb0[:, None, None]
    b1 = yb1[:, None, None]
    out = (((r0 * b0) >> 16) + ((r1 * b1) >> 16) + 2) >> 2
    return np.clip(out, 0, 255).astype(np.uint8)
