"""ORACLE — test infrastructure only, never the product path.

Pure-Python loop restatement of OpenCV's cv2.resize(src, (w, h)) for uint8 with the default
INTER_LINEAR (modules/imgproc/src/resize.cpp, OpenCV 4.x: resizeGeneric_ coefficient tables,
HResizeLinear, VResizeLinearVec_32s8u's SIMD rounding; the exact-2x case takes INTER_AREA's fast
path as cv2.resize does).  The reference calls it at
vivit_transformer/vivit_classifier/data_config/dataset.py:271-277 and :348 and
vivit_transformer/inference.py:155.  cv2 (unpinned in requirements.txt) is not installed in this
image: PARITY UNPINNED — this checks the product's host (vclip_amd/resize.py) and GPU
(vc_resize_linear_u8) implementations against the published algorithm, per element, for small
frames.

Allowed importers: tests/ only.
"""
import math
import struct


def _f32(x):
    return struct.unpack("f", struct.pack("f", x))[0]


def _rint(x):
    # round half to even (cvRound under the default rounding mode)
    r = math.floor(x + 0.5)
    if x + 0.5 == r and r % 2 == 1:
        r -= 1
    return int(r)


def _axis(src, dst, clamp):
    scale = 1.0 / (dst / src)
    tab = []
    limit = dst
    for d in range(dst):
        f = _f32((d + 0.5) * scale - 0.5)
        s = math.floor(f)
        f = _f32(f - s)
        if clamp:
            if s < 0:
                f, s = 0.0, 0
            if s + 1 >= src:
                limit = min(limit, d)
                if s >= src - 1:
                    f, s = 0.0, src - 1
        tab.append((s, _rint(_f32(_f32(1.0 - f) * 2048.0)), _rint(_f32(f * 2048.0))))
    return tab, limit


def resize_linear_u8(img, w, h):
    """img: nested lists [H][W][C] of ints 0..255 -> [h][w][C]."""
    H, W, C = len(img), len(img[0]), len(img[0][0])
    if H == 2 * h and W == 2 * w:
        return [[[(img[2 * y][2 * x][c] + img[2 * y][2 * x + 1][c] + img[2 * y + 1][2 * x][c] +
                   img[2 * y + 1][2 * x + 1][c] + 2) >> 2 for c in range(C)] for x in range(w)] for y in range(h)]
    xt, xlim = _axis(W, w, True)
    yt, _ = _axis(H, h, False)

    def hrow(sy):
        row = img[min(max(sy, 0), H - 1)]
        out = []
        for dx, (sx, a0, a1) in enumerate(xt):
            if dx >= xlim:
                out.append([row[sx][c] * 2048 for c in range(C)])
            else:
                out.append([row[sx][c] * a0 + row[sx + 1][c] * a1 for c in range(C)])
        return out

    res = []
    for sy, b0, b1 in yt:
        r0, r1 = hrow(sy), hrow(sy + 1)
        res.append([[min(255, max(0, (((r0[x][c] >> 4) * b0 >> 16) + ((r1[x][c] >> 4) * b1 >> 16) + 2) >> 2))
                     for c in range(C)] for x in range(w)])
    return res
