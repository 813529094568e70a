// Clip preprocessing on the GPU:
//  * resample_u8_kernel — one axis of Pillow's BILINEAR resize of uint8 images, bit-exact:
//    fixed-point coefficients (22 fraction bits) precomputed on the host exactly as Pillow's
//    precompute_coeffs + normalize_coeffs_8bpc do, accumulation from 1 << 21, clip8 per pass
//    (Pillow Resample.c ImagingResampleHorizontal_8bpc / Vertical_8bpc).  The ViViT processor
//    (VivitImageProcessor: PIL bilinear shortest edge 224 -> 256, centre crop 224, x/63.75 - 3;
//    vivit_transformer/vivit_classifier/trainers/trainer.py:22-26, 62-95) is two passes plus
//    video_transform_kernel.
//  * video_transform_kernel — frame-index gather (pytorchvideo UniformTemporalSubsample /
//    the sampled indices), optional torch-semantics bilinear resize (F.interpolate,
//    align_corners=False: pytorchvideo ShortSideScale), crop (torchvision CenterCrop), per-channel
//    affine x*scale[c] + shift[c] (Normalize / the /255 of the inference scripts), and the output
//    layout [B][T][C][h][w] (HF pixel_values) or [B][C][T][h][w] (torchvision video models).
//  * resize_linear_u8_kernel — OpenCV cv2.resize(frame, (w, h)) INTER_LINEAR on uint8 frames (the
//    reference's resize of decoded frames to 224x224, vivit dataset.py:271-277, :348,
//    inference.py:155): 11-bit fixed-point coefficient tables from the host (vclip_amd/resize.py,
//    OpenCV resizeGeneric_'s float math), the exact horizontal pass, VResizeLinearVec_32s8u's
//    vertical rounding, and INTER_AREA's 2x2 fast path for an exact 2x downscale.
#include "common.hpp"

namespace vc {

constexpr int PIL_PRECISION_BITS = 32 - 8 - 2;

__device__ __forceinline__ unsigned char clip8(int in) {
    if (in >= (1 << PIL_PRECISION_BITS << 8)) return 255;
    if (in <= 0) return 0;
    return (unsigned char)(in >> PIL_PRECISION_BITS);
}

// axis 0: horizontal (W -> Wo), axis 1: vertical (H -> Ho).  One thread per output pixel.
__global__ void __launch_bounds__(256) resample_u8_kernel(const uint8_t* __restrict__ src, int64_t N, int H, int W, int C,
                                                          int axis, int outsz, const int* __restrict__ bounds,
                                                          const int* __restrict__ coef, int ksize,
                                                          uint8_t* __restrict__ dst) {
    const int Ho = axis ? outsz : H, Wo = axis ? W : outsz;
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= N * Ho * Wo) return;
    const int xo = i % Wo;
    const int yo = (i / Wo) % Ho;
    const int64_t n = i / ((int64_t)Wo * Ho);
    const int o = axis ? yo : xo;
    const int mn = bounds[2 * o], cnt = bounds[2 * o + 1];
    const int* k = coef + (int64_t)o * ksize;
    const uint8_t* base = src + n * H * W * C;
    for (int c = 0; c < C; ++c) {
        int ss = 1 << (PIL_PRECISION_BITS - 1);
        for (int x = 0; x < cnt; ++x) {
            const int sy = axis ? mn + x : yo, sx = axis ? xo : mn + x;
            ss += (int)base[((int64_t)sy * W + sx) * C + c] * k[x];
        }
        dst[((n * Ho + yo) * (int64_t)Wo + xo) * C + c] = clip8(ss);
    }
}

struct VideoXform {
    int F, H, W;        // source frames per clip, frame size (uint8 HxWx3)
    int T;              // frames per output clip
    int Hr, Wr;         // resize target (== H, W: no resize)
    int top, left;      // crop origin in the (resized) frame
    int ch, cw;         // crop size = output frame size
    float sc[3], sh[3]; // per-channel affine
    int layout;         // 0: [B][T][C][ch][cw], 1: [B][C][T][ch][cw]
    int bf16;
};

// clip_p (optional, train-time transforms): per clip int32 {resize h, resize w, crop top, crop
// left, horizontal flip} (pytorchvideo RandomShortSideScale, torchvision RandomCrop /
// RandomHorizontalFlip with their parameters drawn on the host); overrides p's resize / crop.
__global__ void __launch_bounds__(256) video_transform_kernel(const uint8_t* __restrict__ frames,
                                                              const int64_t* __restrict__ idx, int64_t nclip, VideoXform p,
                                                              const int* __restrict__ clip_p, void* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t per_frame = (int64_t)p.ch * p.cw;
    if (i >= nclip * p.T * per_frame) return;
    const int j = i % p.cw;
    const int r = (i / p.cw) % p.ch;
    const int t = (i / per_frame) % p.T;
    const int64_t b = i / (per_frame * p.T);
    int64_t f = idx[b * p.T + t];
    f = f < 0 ? 0 : (f >= p.F ? p.F - 1 : f);
    const uint8_t* fr = frames + (b * p.F + f) * (int64_t)p.H * p.W * 3;
    int jj = j;
    if (clip_p) {
        const int* cp = clip_p + b * 5;
        p.Hr = cp[0]; p.Wr = cp[1]; p.top = cp[2]; p.left = cp[3];
        if (cp[4]) jj = p.cw - 1 - j;  // F.hflip of the cropped clip
    }
    const int y = r + p.top, x = jj + p.left;
    float v[3];
    if (p.Hr == p.H && p.Wr == p.W) {
#pragma unroll
        for (int c = 0; c < 3; ++c) v[c] = (float)fr[((int64_t)y * p.W + x) * 3 + c];
    } else {
        // torch upsample_bilinear2d, align_corners=False: src = max((dst + 0.5) * in/out - 0.5, 0)
        const float rh = (float)p.H / (float)p.Hr, rw = (float)p.W / (float)p.Wr;
        float hr = (y + 0.5f) * rh - 0.5f, wr = (x + 0.5f) * rw - 0.5f;
        hr = hr < 0.f ? 0.f : hr;
        wr = wr < 0.f ? 0.f : wr;
        const int h1 = (int)hr, w1 = (int)wr;
        const int h1p = h1 < p.H - 1 ? 1 : 0, w1p = w1 < p.W - 1 ? 1 : 0;
        const float l1h = hr - (float)h1, l0h = 1.f - l1h, l1w = wr - (float)w1, l0w = 1.f - l1w;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const float p00 = fr[((int64_t)h1 * p.W + w1) * 3 + c], p01 = fr[((int64_t)h1 * p.W + w1 + w1p) * 3 + c];
            const float p10 = fr[((int64_t)(h1 + h1p) * p.W + w1) * 3 + c];
            const float p11 = fr[((int64_t)(h1 + h1p) * p.W + w1 + w1p) * 3 + c];
            v[c] = l0h * (l0w * p00 + l1w * p01) + l1h * (l0w * p10 + l1w * p11);
        }
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const float o = v[c] * p.sc[c] + p.sh[c];
        const int64_t oi = p.layout == 0 ? (((b * p.T + t) * 3 + c) * per_frame + (int64_t)r * p.cw + j)
                                         : (((b * 3 + c) * p.T + t) * per_frame + (int64_t)r * p.cw + j);
        if (p.bf16)
            reinterpret_cast<uint16_t*>(out)[oi] = f2bf(o);
        else
            reinterpret_cast<float*>(out)[oi] = o;
    }
}

// One thread per output pixel (all C <= 4 channels).  tab: int32 xofs[w] | xa0[w] | xa1[w] |
// yofs[h] | yb0[h] | yb1[h]; columns >= xlim copy S[xofs] * 2048 (HResizeLinear's xmax).
__global__ void __launch_bounds__(256) resize_linear_u8_kernel(const uint8_t* __restrict__ src, int64_t N, int H, int W,
                                                               int C, int h, int w, const int* __restrict__ tab,
                                                               int xlim, int area2x, uint8_t* __restrict__ dst) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= N * h * w) return;
    const int dx = i % w;
    const int dy = (i / w) % h;
    const int64_t n = i / ((int64_t)w * h);
    const uint8_t* img = src + n * (int64_t)H * W * C;
    uint8_t* o = dst + ((n * h + dy) * (int64_t)w + dx) * C;
    if (area2x) {
        const uint8_t* p0 = img + ((int64_t)(2 * dy) * W + 2 * dx) * C;
        const uint8_t* p1 = p0 + (int64_t)W * C;
        for (int c = 0; c < C; ++c) o[c] = (uint8_t)(((int)p0[c] + p0[C + c] + p1[c] + p1[C + c] + 2) >> 2);
        return;
    }
    const int sx = tab[dx], a0 = tab[w + dx], a1 = tab[2 * w + dx];
    const int sy = tab[3 * w + dy], b0 = tab[3 * w + h + dy], b1 = tab[3 * w + 2 * h + dy];
    const int y0 = sy < 0 ? 0 : (sy > H - 1 ? H - 1 : sy);
    const int y1 = sy + 1 < 0 ? 0 : (sy + 1 > H - 1 ? H - 1 : sy + 1);
    const uint8_t* r0 = img + (int64_t)y0 * W * C;
    const uint8_t* r1 = img + (int64_t)y1 * W * C;
    for (int c = 0; c < C; ++c) {
        int h0, h1;
        if (dx < xlim) {
            h0 = (int)r0[sx * C + c] * a0 + (int)r0[(sx + 1) * C + c] * a1;
            h1 = (int)r1[sx * C + c] * a0 + (int)r1[(sx + 1) * C + c] * a1;
        } else {
            h0 = (int)r0[sx * C + c] * 2048;
            h1 = (int)r1[sx * C + c] * 2048;
        }
        // VResizeLinearVec_32s8u: int16 lanes of row >> 4, mul_hi by the 11-bit betas, (+2) >> 2
        int v = ((((h0 >> 4) * b0) >> 16) + (((h1 >> 4) * b1) >> 16) + 2) >> 2;
        o[c] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
    }
}

}  // namespace vc

using namespace vc;

extern "C" {

int vc_resample_u8(const uint8_t* src, int64_t N, int64_t H, int64_t W, int64_t C, int axis, int64_t out_size,
                   const int* bounds, const int* coeffs, int64_t ksize, uint8_t* dst, hipStream_t stream) {
    if (!src || !bounds || !coeffs || !dst) return fail(VC_ERR_INVALID_ARG, "vc_resample_u8: null pointer");
    if (N <= 0 || H <= 0 || W <= 0 || C <= 0 || C > 4 || out_size <= 0 || ksize <= 0 || (axis != 0 && axis != 1))
        return fail(VC_ERR_INVALID_ARG, "vc_resample_u8: bad shape");
    const int64_t total = N * (axis ? out_size * W : H * out_size);
    resample_u8_kernel<<<(unsigned)((total + 255) / 256), 256, 0, stream>>>(src, N, (int)H, (int)W, (int)C, axis,
                                                                           (int)out_size, bounds, coeffs, (int)ksize, dst);
    return check_launch("vc_resample_u8");
}

int vc_resize_linear_u8(const uint8_t* src, int64_t N, int64_t H, int64_t W, int64_t C, int64_t h, int64_t w,
                        const int* tables, int64_t xlim, int area2x, uint8_t* dst, hipStream_t stream) {
    if (!src || !dst || (!tables && !area2x)) return fail(VC_ERR_INVALID_ARG, "vc_resize_linear_u8: null pointer");
    if (N <= 0 || H <= 0 || W <= 0 || C <= 0 || C > 4 || h <= 0 || w <= 0 || xlim < 0 || xlim > w ||
        (area2x && (H != 2 * h || W != 2 * w)))
        return fail(VC_ERR_INVALID_ARG, "vc_resize_linear_u8: bad shape");
    const int64_t total = N * h * w;
    resize_linear_u8_kernel<<<(unsigned)((total + 255) / 256), 256, 0, stream>>>(src, N, (int)H, (int)W, (int)C, (int)h,
                                                                                (int)w, tables, (int)xlim, area2x, dst);
    return check_launch("vc_resize_linear_u8");
}

int vc_video_transform(const uint8_t* frames, int64_t nclips, int64_t F, int64_t H, int64_t W, const int64_t* idx,
                       int64_t T, int64_t resize_h, int64_t resize_w, int64_t top, int64_t left, int64_t crop_h,
                       int64_t crop_w, const float* scale3, const float* shift3, int layout, int out_bf16, void* out,
                       hipStream_t stream) {
    if (!frames || !idx || !scale3 || !shift3 || !out) return fail(VC_ERR_INVALID_ARG, "vc_video_transform: null pointer");
    if (nclips <= 0 || F <= 0 || H <= 0 || W <= 0 || T <= 0 || resize_h <= 0 || resize_w <= 0 || top < 0 || left < 0 ||
        crop_h <= 0 || crop_w <= 0 || top + crop_h > resize_h || left + crop_w > resize_w || (layout != 0 && layout != 1))
        return fail(VC_ERR_INVALID_ARG, "vc_video_transform: bad geometry");
    VideoXform p;
    p.F = (int)F; p.H = (int)H; p.W = (int)W; p.T = (int)T;
    p.Hr = (int)resize_h; p.Wr = (int)resize_w;
    p.top = (int)top; p.left = (int)left; p.ch = (int)crop_h; p.cw = (int)crop_w;
    for (int c = 0; c < 3; ++c) { p.sc[c] = scale3[c]; p.sh[c] = shift3[c]; }
    p.layout = layout;
    p.bf16 = out_bf16 ? 1 : 0;
    const int64_t total = nclips * T * crop_h * crop_w;
    video_transform_kernel<<<(unsigned)((total + 255) / 256), 256, 0, stream>>>(frames, idx, nclips, p, nullptr, out);
    return check_launch("vc_video_transform");
}

int vc_video_transform_clips(const uint8_t* frames, int64_t nclips, int64_t F, int64_t H, int64_t W, const int64_t* idx,
                             int64_t T, const int* clip_params, int64_t crop_h, int64_t crop_w, const float* scale3,
                             const float* shift3, int layout, int out_bf16, void* out, hipStream_t stream) {
    if (!frames || !idx || !clip_params || !scale3 || !shift3 || !out)
        return fail(VC_ERR_INVALID_ARG, "vc_video_transform_clips: null pointer");
    if (nclips <= 0 || F <= 0 || H <= 0 || W <= 0 || T <= 0 || crop_h <= 0 || crop_w <= 0 || (layout != 0 && layout != 1))
        return fail(VC_ERR_INVALID_ARG, "vc_video_transform_clips: bad geometry");
    // the per-clip crop windows are validated by the caller on the host (they live in device memory here)
    VideoXform p;
    p.F = (int)F; p.H = (int)H; p.W = (int)W; p.T = (int)T;
    p.Hr = (int)H; p.Wr = (int)W;
    p.top = 0; p.left = 0; p.ch = (int)crop_h; p.cw = (int)crop_w;
    for (int c = 0; c < 3; ++c) { p.sc[c] = scale3[c]; p.sh[c] = shift3[c]; }
    p.layout = layout;
    p.bf16 = out_bf16 ? 1 : 0;
    const int64_t total = nclips * T * crop_h * crop_w;
    video_transform_kernel<<<(unsigned)((total + 255) / 256), 256, 0, stream>>>(frames, idx, nclips, p, clip_params, out);
    return check_launch("vc_video_transform_clips");
}

}  // extern "C"
