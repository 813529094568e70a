// Shared by the Swin window-attention forward (window.hip) and backward (window_bwd.hip).
#pragma once
#include "common.hpp"

namespace vc {

__device__ __forceinline__ int kchunk_swz(int r, int c) { return c ^ ((r >> 2) & 3); }

struct WinGeom {
    int T, H, W;      // token grid (multiples of the window)
    int wt, wh, ww;   // window
    int st, sh, sw;   // shift (0 where none)
    int nwt, nwh, nww;
};

// Shift-region label of one dimension for a rolled coordinate c (torchvision's t/h/w
// slices: 0 below P-w, 1 in [P-w, P-s), 2 from P-s; with s == 0 the slices are (0,-w),
// (-w,0) = empty and (0,None) = all, so every position gets 2).  Inside ONE window a
// dimension takes at most two of these values ({0} or {1,2} or {2}), so "label == 2" is
// one bit and the 3-bit code (t,h,w) compares equal exactly when the labels do.
__device__ __forceinline__ int region_bit(int c, int P, int w, int s) {
    if (s == 0) return 1;
    return c >= P - s ? 1 : 0;
}

// Window-local token n of window (wi_t, wi_h, wi_w) of clip b -> global token row (torchvision's
// roll by -shift and window partition, read by index); *label (optional) = its shift-region code.
__device__ __forceinline__ int64_t win_token_row(const WinGeom& g, int b, int wi_t, int wi_h, int wi_w, int n,
                                                 int* label) {
    const int hw = g.wh * g.ww;
    const int i = n / hw, j = (n / g.ww) % g.wh, k = n % g.ww;
    const int tr = wi_t * g.wt + i, hr = wi_h * g.wh + j, wr = wi_w * g.ww + k;
    if (label)
        *label = 4 * region_bit(tr, g.T, g.wt, g.st) + 2 * region_bit(hr, g.H, g.wh, g.sh) + region_bit(wr, g.W, g.ww, g.sw);
    int t = tr + g.st, hh = hr + g.sh, w = wr + g.sw;
    t -= t >= g.T ? g.T : 0;
    hh -= hh >= g.H ? g.H : 0;
    w -= w >= g.W ? g.W : 0;
    return (((int64_t)b * g.T + t) * g.H + hh) * g.W + w;
}

struct FullWin {
    int T, H, W;  // the model's window_size: the relative-position index is defined on it
};

// torchvision define_relative_position_index for window-local indices q, k (coordinates in the
// FULL window's flattening, as its [:vol, :vol] slice takes them when the window shrinks) is
// linear in the two tokens' coordinates:
//   idx(q, k) = ((qt - kt + T - 1) (2H - 1) + (qh - kh + H - 1)) (2W - 1) + (qw - kw + W - 1)
//             = code(q) - code(k) + code_max,   code(n) = nt S1 + nh S2 + nw,
// S1 = (2H - 1)(2W - 1), S2 = 2W - 1, code_max = (T - 1) S1 + (H - 1) S2 + W - 1.
__device__ __forceinline__ int rel_code(int n, const FullWin& f) {
    const int hw = f.H * f.W;
    return (n / hw) * (2 * f.H - 1) * (2 * f.W - 1) + ((n / f.W) % f.H) * (2 * f.W - 1) + n % f.W;
}
__device__ __forceinline__ int rel_code_max(const FullWin& f) {
    return (f.T - 1) * (2 * f.H - 1) * (2 * f.W - 1) + (f.H - 1) * (2 * f.W - 1) + f.W - 1;
}

}  // namespace vc
