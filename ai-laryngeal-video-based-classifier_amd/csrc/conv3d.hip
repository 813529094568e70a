// 3D convolution pieces of the ResNet3D-50 path (pytorchvideo create_resnet):
// convolutions run as im2col + the MFMA GEMM (BatchNorm folded into the weights / bias on
// the host, ReLU and the residual add fused into the GEMM epilogue); activations are
// channels-last bf16 rows ((b*T + t)*H + h)*W + w.
#include "common.hpp"

namespace vc {

// ---------------------------------------------------------------------------------
// im2col from the f32 [B][C][T][H][W] clip (the model input; C is small, e.g. the stem's 3):
// A[m][(c, kt, kh, kw)] (PyTorch Conv3d weight order), zero padding, columns zero-filled up
// to the next multiple of 8 (the GEMM's K padding).
// ---------------------------------------------------------------------------------
struct Conv3dGeom {
    int T, H, W, C;         // input
    int To, Ho, Wo;         // output
    int kt, kh, kw;
    int st, sh, sw;
    int pt, ph, pw;
};

// A workgroup owns 64 consecutive output positions (one per lane, so a load instruction reads
// 64 neighbouring output pixels of one input row: coalesced) and all column chunks of their
// rows (the 4 waves stride over the chunks, so every line of those rows is completed by one
// workgroup).  The column -> (c, kt, kh, kw) decomposition comes from an LDS table.
__global__ void __launch_bounds__(256) im2col_ncthw_kernel(const float* __restrict__ x, int64_t M, int nchunk, Conv3dGeom g,
                                                           int K, uint16_t* __restrict__ A, int64_t lda) {
    __shared__ unsigned tab[2048];  // c | it << 8 | ih << 16 | iw << 24
    for (int k = threadIdx.x; k < nchunk * 8; k += 256) {
        unsigned v = 0xffffffffu;
        if (k < K) {
            const int iw = k % g.kw, ih = (k / g.kw) % g.kh, it = (k / (g.kw * g.kh)) % g.kt, c = k / (g.kw * g.kh * g.kt);
            v = (unsigned)c | ((unsigned)it << 8) | ((unsigned)ih << 16) | ((unsigned)iw << 24);
        }
        tab[k] = v;
    }
    __syncthreads();
    const int64_t m = (int64_t)blockIdx.x * 64 + (threadIdx.x & 63);
    if (m >= M) return;
    const int wave = threadIdx.x >> 6;
    const int wo = m % g.Wo;
    const int ho = (m / g.Wo) % g.Ho;
    const int to = (m / ((int64_t)g.Wo * g.Ho)) % g.To;
    const int64_t b = m / ((int64_t)g.Wo * g.Ho * g.To);
    const int t0 = to * g.st - g.pt, y0 = ho * g.sh - g.ph, x0 = wo * g.sw - g.pw;
    const float* xb = x + b * g.C * (int64_t)g.T * g.H * g.W;
    uint16_t* arow = A + m * lda;
    for (int kc = wave; kc < nchunk; kc += 4) {
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const unsigned tv = tab[kc * 8 + e];
            float val = 0.f;
            if (tv != 0xffffffffu) {
                const int c = tv & 255, t = t0 + ((tv >> 8) & 255), y = y0 + ((tv >> 16) & 255), xx = x0 + (tv >> 24);
                if (t >= 0 && t < g.T && y >= 0 && y < g.H && xx >= 0 && xx < g.W)
                    val = xb[(((int64_t)c * g.T + t) * g.H + y) * g.W + xx];
            }
            v[e] = val;
        }
        uint4 o;
        o.x = pack2bf(v[0], v[1]);
        o.y = pack2bf(v[2], v[3]);
        o.z = pack2bf(v[4], v[5]);
        o.w = pack2bf(v[6], v[7]);
        *reinterpret_cast<uint4*>(arow + kc * 8) = o;
    }
}

// ---------------------------------------------------------------------------------
// im2col from channels-last bf16 activations: A[m][(kt, kh, kw, c)], 16-B chunks (C % 8 == 0),
// zero padding.  One thread per (output position, kernel tap, 8-channel chunk).
// ---------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) im2col_cl_kernel(const uint16_t* __restrict__ x, int64_t ldx, int64_t total,
                                                        Conv3dGeom g, uint16_t* __restrict__ A, int64_t lda) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= total) return;
    const int C8 = g.C >> 3;
    int64_t r = i;
    const int c8 = r % C8;
    r /= C8;
    const int tap = r % (g.kt * g.kh * g.kw);
    const int64_t m = r / (g.kt * g.kh * g.kw);
    const int iw = tap % g.kw, ih = (tap / g.kw) % g.kh, it = tap / (g.kw * g.kh);
    const int wo = m % g.Wo;
    const int ho = (m / g.Wo) % g.Ho;
    const int to = (m / ((int64_t)g.Wo * g.Ho)) % g.To;
    const int64_t b = m / ((int64_t)g.Wo * g.Ho * g.To);
    const int t = to * g.st - g.pt + it, y = ho * g.sh - g.ph + ih, xx = wo * g.sw - g.pw + iw;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (t >= 0 && t < g.T && y >= 0 && y < g.H && xx >= 0 && xx < g.W)
        v = *reinterpret_cast<const uint4*>(x + (((b * g.T + t) * g.H + y) * (int64_t)g.W + xx) * ldx + c8 * 8);
    *reinterpret_cast<uint4*>(A + m * lda + (int64_t)tap * g.C + c8 * 8) = v;
}

// ---------------------------------------------------------------------------------
// MaxPool3d on channels-last bf16 (padding = -inf, as torch).  One thread per (output
// position, 8-channel chunk).
// ---------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) maxpool_cl_kernel(const uint16_t* __restrict__ x, int64_t ldx, int64_t total,
                                                         Conv3dGeom g, uint16_t* __restrict__ y, int64_t ldy) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= total) return;
    const int C8 = g.C >> 3;
    const int c8 = i % C8;
    const int64_t m = i / C8;
    const int wo = m % g.Wo;
    const int ho = (m / g.Wo) % g.Ho;
    const int to = (m / ((int64_t)g.Wo * g.Ho)) % g.To;
    const int64_t b = m / ((int64_t)g.Wo * g.Ho * g.To);
    float mx[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) mx[e] = -INFINITY;
    for (int it = 0; it < g.kt; ++it)
        for (int ih = 0; ih < g.kh; ++ih)
            for (int iw = 0; iw < g.kw; ++iw) {
                const int t = to * g.st - g.pt + it, yy = ho * g.sh - g.ph + ih, xx = wo * g.sw - g.pw + iw;
                if (t < 0 || t >= g.T || yy < 0 || yy >= g.H || xx < 0 || xx >= g.W) continue;
                const uint4 u = *reinterpret_cast<const uint4*>(x + (((b * g.T + t) * g.H + yy) * (int64_t)g.W + xx) * ldx + c8 * 8);
                const unsigned w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    mx[2 * e] = fmaxf(mx[2 * e], bf2f((unsigned short)(w[e] & 0xffff)));
                    mx[2 * e + 1] = fmaxf(mx[2 * e + 1], bf2f((unsigned short)(w[e] >> 16)));
                }
            }
    uint4 o;
    o.x = pack2bf(mx[0], mx[1]);
    o.y = pack2bf(mx[2], mx[3]);
    o.z = pack2bf(mx[4], mx[5]);
    o.w = pack2bf(mx[6], mx[7]);
    *reinterpret_cast<uint4*>(y + m * ldy + c8 * 8) = o;
}

// ---------------------------------------------------------------------------------
// pytorchvideo ResNetBasicHead with output_with_global_average: AvgPool3d(k, stride 1) ->
// Linear per pooled position -> AdaptiveAvgPool3d(1).  Linear commutes with the averages, so
// logits = W . pooled + b with pooled[c] = sum_{t,h,w} wt[t] wh[h] ww[w] x[t,h,w,c], where
// w_d(i) = #{pool windows along d containing i} / (#windows_d * k_d).  Stage 1: grid
// (B, C/256) per-channel weighted sums (fixed order: deterministic); stage 2: GEMV.
// ---------------------------------------------------------------------------------
__device__ __forceinline__ float pool_w(int i, int D, int k) {
    const int nwin = D - k + 1;
    const int lo = i - k + 1 > 0 ? i - k + 1 : 0;
    const int hi = i < nwin - 1 ? i : nwin - 1;
    return (float)(hi - lo + 1) / (float)(nwin * k);
}

constexpr int HEAD_CHUNKS = 32;

// stage 1: grid (B, C/256, HEAD_CHUNKS): each thread a channel, a strided share of positions
__global__ void __launch_bounds__(256) head_pool_kernel(const uint16_t* __restrict__ x, int64_t ldx, int T, int H, int W,
                                                        int C, int kt, int kh, int kw, float* __restrict__ part) {
    const int b = blockIdx.x;
    const int c = blockIdx.y * 256 + threadIdx.x;
    const int ch = blockIdx.z;
    if (c >= C) return;
    const int npos = T * H * W;
    float s = 0.f;
    for (int pos = ch; pos < npos; pos += HEAD_CHUNKS) {
        const int xx = pos % W, y = (pos / W) % H, t = pos / (W * H);
        s += pool_w(t, T, kt) * pool_w(y, H, kh) * pool_w(xx, W, kw) * bf2f(x[((int64_t)b * npos + pos) * ldx + c]);
    }
    part[((int64_t)b * HEAD_CHUNKS + ch) * C + c] = s;
}

// stage 2: sum the chunks in order (deterministic) -> pooled
__global__ void __launch_bounds__(256) head_reduce_kernel(const float* __restrict__ part, int C, float* __restrict__ pooled) {
    const int b = blockIdx.x;
    const int c = blockIdx.y * 256 + threadIdx.x;
    if (c >= C) return;
    float s = 0.f;
    for (int ch = 0; ch < HEAD_CHUNKS; ++ch) s += part[((int64_t)b * HEAD_CHUNKS + ch) * C + c];
    pooled[(int64_t)b * C + c] = s;
}

__global__ void __launch_bounds__(256) head_gemv_kernel(const float* __restrict__ pooled, int C,
                                                        const float* __restrict__ Wc, const float* __restrict__ bc,
                                                        int nl, float* __restrict__ logits) {
    const int b = blockIdx.x;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int c = w; c < nl; c += 4) {
        float a = 0.f;
        for (int n = lane; n < C; n += 64) a += pooled[(int64_t)b * C + n] * Wc[(int64_t)c * C + n];
        a = wave_sum(a);
        if (lane == 0) logits[(int64_t)b * nl + c] = a + bc[c];
    }
}

static Conv3dGeom make_geom(int64_t T, int64_t H, int64_t W, int64_t C, const int* k, const int* s, const int* p) {
    Conv3dGeom g;
    g.T = (int)T; g.H = (int)H; g.W = (int)W; g.C = (int)C;
    g.kt = k[0]; g.kh = k[1]; g.kw = k[2];
    g.st = s[0]; g.sh = s[1]; g.sw = s[2];
    g.pt = p[0]; g.ph = p[1]; g.pw = p[2];
    g.To = (int)((T + 2 * p[0] - k[0]) / s[0] + 1);
    g.Ho = (int)((H + 2 * p[1] - k[1]) / s[1] + 1);
    g.Wo = (int)((W + 2 * p[2] - k[2]) / s[2] + 1);
    return g;
}

static bool geom_ok(const int* k, const int* s, const int* p) {
    for (int d = 0; d < 3; ++d)
        if (k[d] <= 0 || s[d] <= 0 || p[d] < 0 || p[d] >= k[d]) return false;
    return true;
}

}  // namespace vc

using namespace vc;

extern "C" {

int vc_conv3d_im2col(const void* x, int64_t ldx, int input_kind, int64_t B, int64_t T, int64_t H, int64_t W,
                     int64_t C, const int* kernel, const int* stride, const int* pad, uint16_t* A, int64_t lda,
                     hipStream_t stream) {
    if (!x || !A || !kernel || !stride || !pad) return fail(VC_ERR_INVALID_ARG, "vc_conv3d_im2col: null pointer");
    if (!geom_ok(kernel, stride, pad) || B <= 0 || T <= 0 || H <= 0 || W <= 0 || C <= 0)
        return fail(VC_ERR_INVALID_ARG, "vc_conv3d_im2col: bad geometry");
    const Conv3dGeom g = make_geom(T, H, W, C, kernel, stride, pad);
    const int64_t kvol = (int64_t)g.kt * g.kh * g.kw;
    if (lda < kvol * C) return fail(VC_ERR_INVALID_ARG, "vc_conv3d_im2col: lda < kernel volume * C");
    const int64_t M = B * g.To * g.Ho * g.Wo;
    if (input_kind == VC_CONV_IN_NCTHW_F32) {
        const int K = (int)(kvol * C);
        const int nchunk = (K + 7) / 8;
        if (lda < nchunk * 8 || lda % 8 || ((uintptr_t)A & 15) || nchunk * 8 > 2048 || C > 255 || g.kt > 255 ||
            g.kh > 255 || g.kw > 255)
            return fail(VC_ERR_INVALID_ARG, "vc_conv3d_im2col: NCTHW input needs lda >= roundup(K, 8) <= 2048, 16-B rows");
        im2col_ncthw_kernel<<<(unsigned)((M + 63) / 64), 256, 0, stream>>>((const float*)x, M, nchunk, g, K, A, lda);
    } else if (input_kind == VC_CONV_IN_CL_BF16) {
        if (C % 8 || ldx % 8 || lda % 8 || ((uintptr_t)x | (uintptr_t)A) & 15)
            return fail(VC_ERR_INVALID_ARG, "vc_conv3d_im2col: channels-last input needs C % 8 == 0 and 16-B rows");
        const int64_t total = M * kvol * (C / 8);
        im2col_cl_kernel<<<(unsigned)((total + 255) / 256), 256, 0, stream>>>((const uint16_t*)x, ldx, total, g, A, lda);
    } else {
        return fail(VC_ERR_INVALID_ARG, "vc_conv3d_im2col: bad input_kind");
    }
    return check_launch("vc_conv3d_im2col");
}

int vc_maxpool3d(const uint16_t* x, int64_t ldx, int64_t B, int64_t T, int64_t H, int64_t W, int64_t C,
                 const int* kernel, const int* stride, const int* pad, uint16_t* y, int64_t ldy, hipStream_t stream) {
    if (!x || !y || !kernel || !stride || !pad) return fail(VC_ERR_INVALID_ARG, "vc_maxpool3d: null pointer");
    if (!geom_ok(kernel, stride, pad) || C % 8 || ldx % 8 || ldy % 8 || ((uintptr_t)x | (uintptr_t)y) & 15)
        return fail(VC_ERR_INVALID_ARG, "vc_maxpool3d: bad geometry / C % 8 / alignment");
    const Conv3dGeom g = make_geom(T, H, W, C, kernel, stride, pad);
    const int64_t total = B * g.To * g.Ho * g.Wo * (C / 8);
    maxpool_cl_kernel<<<(unsigned)((total + 255) / 256), 256, 0, stream>>>(x, ldx, total, g, y, ldy);
    return check_launch("vc_maxpool3d");
}

int vc_avgpool_head(const uint16_t* x, int64_t ldx, int64_t B, int64_t T, int64_t H, int64_t W, int64_t C,
                    const int* pool_kernel, const float* Wc, const float* bc, int64_t num_labels, float* work,
                    float* logits, hipStream_t stream) {
    if (!x || !pool_kernel || !Wc || !bc || !work || !logits) return fail(VC_ERR_INVALID_ARG, "vc_avgpool_head: null pointer");
    if (pool_kernel[0] > T || pool_kernel[1] > H || pool_kernel[2] > W || pool_kernel[0] <= 0 || pool_kernel[1] <= 0 ||
        pool_kernel[2] <= 0)
        return fail(VC_ERR_INVALID_ARG, "vc_avgpool_head: pool kernel larger than the feature map");
    float* part = work + B * C;  // work: [B*C] pooled, then [B*HEAD_CHUNKS*C] partials
    head_pool_kernel<<<dim3((unsigned)B, (unsigned)((C + 255) / 256), HEAD_CHUNKS), 256, 0, stream>>>(
        x, ldx, (int)T, (int)H, (int)W, (int)C, pool_kernel[0], pool_kernel[1], pool_kernel[2], part);
    head_reduce_kernel<<<dim3((unsigned)B, (unsigned)((C + 255) / 256)), 256, 0, stream>>>(part, (int)C, work);
    head_gemv_kernel<<<(unsigned)B, 256, 0, stream>>>(work, (int)C, Wc, bc, (int)num_labels, logits);
    return check_launch("vc_avgpool_head");
}

}  // extern "C"
