// ResNet3D-50 train step (resnet50-3d-video/video_classifier/trainers/trainer.py:106-123:
// model.train(), outputs = model(inputs), CrossEntropyLoss, loss.backward(), Adam.step()): the
// pieces the convolution GEMMs (vc_gemm_bf16 / vc_wgrad_bf16 through vclip_amd/autograd_ops.py)
// do not cover, on channels-last rows ((b*T + t)*H + h)*W + w:
//  * col2im_cl_kernel     — backward of vc_conv3d_im2col (channels-last): dX[pos][c] = sum over
//    the (output position, tap) pairs that read pos of dA[m][tap*C + c], as a gather (each input
//    element sums its <= kt*kh*kw contributions in a fixed order: deterministic, no atomics);
//  * maxpool_bwd_cl_kernel — MaxPool3d backward: the gradient of an output goes to the FIRST
//    maximum of its window in scan order (torch's max_pool3d index), gathered per input element;
//  * BatchNorm3d in training mode (batch statistics; nn.BatchNorm3d): bn_partial_kernel (per-
//    channel partial sums over row chunks, three modes) + bn_finalize_kernel (fixed-order chunk
//    sums -> mean / rstd / running-stat update, or dbeta / dgamma), bn_apply_kernel
//    (z = relu?(gamma * (y - mean) * rstd + beta (+ residual)), bf16 out) and bn_bwd_kernel
//    (dy = gamma * rstd * (g - dbeta / M - xhat * dgamma / M), g = dz masked by z > 0);
//  * the ResNetBasicHead in training mode: AvgPool3d((kt,kh,kw), stride 1) -> Dropout (mask from
//    the host) -> Linear per position -> AdaptiveAvgPool3d(1): the Linear commutes with the
//    means, so logits = W . u + b with u[b][c] = sum_rows x[row][c] * w(b, t(row), c) and w the
//    per-(t, c) weight of the kept pool windows covering t (head_train_fwd_kernel); its backward
//    dx = du * w (head_train_bwd_kernel; du from vc_pool_head_bwd).
#include "common.hpp"

namespace vc {
namespace rbwd {

struct Geom {
    int T, H, W, C;     // input
    int To, Ho, Wo;     // output
    int kt, kh, kw;
    int st, sh, sw;
    int pt, ph, pw;
};

__device__ __forceinline__ float ldf(const float* p) { return *p; }
__device__ __forceinline__ float ldf(const uint16_t* p) { return bf2f(*p); }

// one thread per (input position, channel): sum over taps in (it, ih, iw) order
__global__ void __launch_bounds__(256) col2im_cl_kernel(const uint16_t* __restrict__ dA, int64_t lda, int64_t total,
                                                        Geom g, float* __restrict__ dx, int64_t lddx) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= total) return;
    const int c = (int)(i % g.C);
    const int64_t p = i / g.C;
    const int x = (int)(p % g.W);
    const int y = (int)((p / g.W) % g.H);
    const int t = (int)((p / ((int64_t)g.W * g.H)) % g.T);
    const int64_t b = p / ((int64_t)g.W * g.H * g.T);
    float s = 0.f;
    for (int it = 0; it < g.kt; ++it) {
        const int tn = t + g.pt - it;
        if (tn < 0 || tn % g.st) continue;
        const int to = tn / g.st;
        if (to >= g.To) continue;
        for (int ih = 0; ih < g.kh; ++ih) {
            const int yn = y + g.ph - ih;
            if (yn < 0 || yn % g.sh) continue;
            const int ho = yn / g.sh;
            if (ho >= g.Ho) continue;
            for (int iw = 0; iw < g.kw; ++iw) {
                const int xn = x + g.pw - iw;
                if (xn < 0 || xn % g.sw) continue;
                const int wo = xn / g.sw;
                if (wo >= g.Wo) continue;
                const int64_t m = ((b * g.To + to) * g.Ho + ho) * (int64_t)g.Wo + wo;
                const int tap = (it * g.kh + ih) * g.kw + iw;
                s += bf2f(dA[m * lda + (int64_t)tap * g.C + c]);
            }
        }
    }
    dx[p * lddx + c] = s;
}

// one thread per (input position, channel): every output window containing the position whose
// first maximum (scan order it, ih, iw; padding never wins) is this position passes its gradient
template <typename TD>
__global__ void __launch_bounds__(256) maxpool_bwd_cl_kernel(const uint16_t* __restrict__ x, int64_t ldx,
                                                             const TD* __restrict__ dy, int64_t lddy, int64_t total,
                                                             Geom g, float* __restrict__ dx, int64_t lddx) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= total) return;
    const int c = (int)(i % g.C);
    const int64_t p = i / g.C;
    const int xw = (int)(p % g.W);
    const int y = (int)((p / g.W) % g.H);
    const int t = (int)((p / ((int64_t)g.W * g.H)) % g.T);
    const int64_t b = p / ((int64_t)g.W * g.H * g.T);
    float s = 0.f;
    // output windows containing the position: o * stride - pad <= i < o * stride - pad + k
    auto lo_hi = [](int i, int k, int st, int pd, int n, int& lo, int& hi) {
        const int a = i + pd - k + 1;
        lo = a <= 0 ? 0 : (a + st - 1) / st;
        hi = (i + pd) / st;
        if (hi > n - 1) hi = n - 1;
    };
    int tlo, thi, hlo, hhi, wlo, whi;
    lo_hi(t, g.kt, g.st, g.pt, g.To, tlo, thi);
    lo_hi(y, g.kh, g.sh, g.ph, g.Ho, hlo, hhi);
    lo_hi(xw, g.kw, g.sw, g.pw, g.Wo, wlo, whi);
    for (int to = tlo; to <= thi; ++to) {
        const int t0 = to * g.st - g.pt;
        for (int ho = hlo; ho <= hhi; ++ho) {
            const int y0 = ho * g.sh - g.ph;
            for (int wo = wlo; wo <= whi; ++wo) {
                const int x0 = wo * g.sw - g.pw;
                // the window's first maximum
                float best = -INFINITY;
                int64_t arg = -1;
                for (int it = 0; it < g.kt; ++it)
                    for (int ih = 0; ih < g.kh; ++ih)
                        for (int iw = 0; iw < g.kw; ++iw) {
                            const int tt = t0 + it, yy = y0 + ih, xx = x0 + iw;
                            if (tt < 0 || tt >= g.T || yy < 0 || yy >= g.H || xx < 0 || xx >= g.W) continue;
                            const int64_t q = ((b * g.T + tt) * g.H + yy) * (int64_t)g.W + xx;
                            const float v = bf2f(x[q * ldx + c]);
                            if (v > best || arg < 0) { best = v; arg = q; }
                        }
                if (arg == p) {
                    const int64_t m = ((b * g.To + to) * g.Ho + ho) * (int64_t)g.Wo + wo;
                    s += ldf(dy + m * lddy + c);
                }
            }
        }
    }
    dx[p * lddx + c] = s;
}

// ---- BatchNorm (training mode) ----------------------------------------------------------
// Partial per-channel sums over row chunk blockIdx.y of rps rows (threads: Cb channels x
// 256 / Cb row phases, combined in LDS in a fixed order).
//  MODE 0: s1 = sum y
//  MODE 1: s1 = sum (y - mean)^2                       (mean = stat[0][c])
//  MODE 2: s1 = sum g, s2 = sum g * xhat, g = dz (z > 0 if relu), xhat = (y - mean) * rstd
template <int MODE>
__global__ void __launch_bounds__(256) bn_partial_kernel(const float* __restrict__ y, int64_t ldy, int64_t M, int C,
                                                         int64_t rps, const float* __restrict__ stat,
                                                         const float* __restrict__ dz, int64_t lddz,
                                                         const uint16_t* __restrict__ z, int64_t ldz, int relu,
                                                         float* __restrict__ part) {
    __shared__ float red[2][256];
    const int Cb = C < 256 ? C : 256;
    const int nph = 256 / Cb;
    const int c = blockIdx.x * 256 + (threadIdx.x % Cb);
    const int ph = threadIdx.x / Cb;
    float s1 = 0.f, s2 = 0.f;
    if (ph < nph && c < C) {
        const int64_t r0 = (int64_t)blockIdx.y * rps, r1 = r0 + rps < M ? r0 + rps : M;
        const float mean = MODE >= 1 ? stat[c] : 0.f;
        const float rstd = MODE == 2 ? stat[C + c] : 0.f;
        for (int64_t r = r0 + ph; r < r1; r += nph) {
            const float v = y[r * ldy + c];
            if (MODE == 0) {
                s1 += v;
            } else if (MODE == 1) {
                const float d = v - mean;
                s1 += d * d;
            } else {
                float gz = dz[r * lddz + c];
                if (relu && !(bf2f(z[r * ldz + c]) > 0.f)) gz = 0.f;
                s1 += gz;
                s2 += gz * (v - mean) * rstd;
            }
        }
    }
    red[0][threadIdx.x] = s1;
    red[1][threadIdx.x] = s2;
    __syncthreads();
    if (ph == 0 && c < C) {
        for (int k = 1; k < nph; ++k) {
            s1 += red[0][threadIdx.x + k * Cb];
            s2 += red[1][threadIdx.x + k * Cb];
        }
        part[(int64_t)blockIdx.y * 2 * C + c] = s1;
        part[(int64_t)blockIdx.y * 2 * C + C + c] = s2;
    }
}

//  MODE 0: stat[0][c] = mean;  MODE 1: stat[1][c] = rstd, running stats updated (momentum, the
//  unbiased variance, as nn.BatchNorm3d);  MODE 2: out0 = dbeta, out1 = dgamma.
//  One workgroup per channel: thread t sums splits t, t + 256, ..., then a fixed-order LDS tree.
template <int MODE>
__global__ void __launch_bounds__(256) bn_finalize_kernel(const float* __restrict__ part, int nsplit, int64_t M, int C,
                                                          float eps, float momentum, float* __restrict__ stat,
                                                          float* __restrict__ run_mean, float* __restrict__ run_var,
                                                          float* __restrict__ out0, float* __restrict__ out1) {
    __shared__ float red[2][256];
    const int c = blockIdx.x, t = threadIdx.x;
    float s1 = 0.f, s2 = 0.f;
    for (int k = t; k < nsplit; k += 256) {
        s1 += part[(int64_t)k * 2 * C + c];
        if (MODE == 2) s2 += part[(int64_t)k * 2 * C + C + c];
    }
    red[0][t] = s1;
    red[1][t] = s2;
    __syncthreads();
#pragma unroll
    for (int w = 128; w >= 1; w >>= 1) {
        if (t < w) {
            red[0][t] += red[0][t + w];
            if (MODE == 2) red[1][t] += red[1][t + w];
        }
        __syncthreads();
    }
    if (t != 0) return;
    s1 = red[0][0];
    s2 = red[1][0];
    if (MODE == 0) {
        stat[c] = s1 / (float)M;
    } else if (MODE == 1) {
        const float var = s1 / (float)M;
        stat[C + c] = rsqrtf(var + eps);
        if (run_mean) {
            run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * stat[c];
            run_var[c] = (1.f - momentum) * run_var[c] + momentum * (M > 1 ? s1 / (float)(M - 1) : var);
        }
    } else {
        out0[c] = s1;
        out1[c] = s2;
    }
}

// z = gamma (y - mean) rstd + beta (+ res), ReLU optional, bf16 rows (C % 4 == 0)
template <typename TR>
__global__ void __launch_bounds__(256) bn_apply_kernel(const float* __restrict__ y, int64_t ldy, int64_t M, int C,
                                                       const float* __restrict__ stat, const float* __restrict__ gamma,
                                                       const float* __restrict__ beta, const TR* __restrict__ res,
                                                       int64_t ldr, int relu, uint16_t* __restrict__ z, int64_t ldz) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int C4 = C >> 2;
    if (i >= M * C4) return;
    const int64_t r = i / C4;
    const int c = (int)(i - r * C4) * 4;
    const float4 v = *reinterpret_cast<const float4*>(y + r * ldy + c);
    float o[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        o[e] = gamma[c + e] * (o[e] - stat[c + e]) * stat[C + c + e] + beta[c + e];
        if (res) o[e] += ldf(res + r * ldr + c + e);
        if (relu) o[e] = fmaxf(o[e], 0.f);
    }
    uint2 p;
    p.x = pack2bf(o[0], o[1]);
    p.y = pack2bf(o[2], o[3]);
    *reinterpret_cast<uint2*>(z + r * ldz + c) = p;
}

// dy = gamma rstd (g - dbeta / M - xhat dgamma / M), g = dz (z > 0); dres = g (optional)
__global__ void __launch_bounds__(256) bn_bwd_kernel(const float* __restrict__ y, int64_t ldy, int64_t M, int C,
                                                     const float* __restrict__ stat, const float* __restrict__ gamma,
                                                     const float* __restrict__ dbeta, const float* __restrict__ dgamma,
                                                     const float* __restrict__ dz, int64_t lddz,
                                                     const uint16_t* __restrict__ z, int64_t ldz, int relu,
                                                     float* __restrict__ dy, int64_t lddy, float* __restrict__ dres,
                                                     int64_t lddr) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= M * C) return;
    const int64_t r = i / C;
    const int c = (int)(i - r * C);
    float g = dz[r * lddz + c];
    if (relu && !(bf2f(z[r * ldz + c]) > 0.f)) g = 0.f;
    const float mean = stat[c], rstd = stat[C + c];
    const float xh = (y[r * ldy + c] - mean) * rstd;
    const float invM = 1.0f / (float)M;
    dy[r * lddy + c] = gamma[c] * rstd * (g - dbeta[c] * invM - xh * dgamma[c] * invM);
    if (dres) dres[r * lddr + c] = g;
}

// ---- head (training mode) ----------------------------------------------------------------
// keep: f32 [B][P][C] dropout scale per pooled position (0 or 1 / (1 - p)), P = T - kt + 1 (the
// final map is kh x kw = H x W: one spatial window).  w(b, t, c) = sum over the windows p that
// cover t of keep[b][p][c] / (P * kt * H * W).
__device__ __forceinline__ float head_w(const float* keep, int b, int t, int c, int T, int kt, int C) {
    const int P = T - kt + 1;
    const int lo = t - kt + 1 > 0 ? t - kt + 1 : 0, hi = t < P - 1 ? t : P - 1;
    float s = 0.f;
    for (int p = lo; p <= hi; ++p) s += keep[((int64_t)b * P + p) * C + c];
    return s;
}

// u[b][c] = sum_{t, hw} x[b, t, hw, c] * w(b, t, c) / (P kt HW): grid (B, C / 256), one thread a
// channel, positions in a fixed order (deterministic)
__global__ void __launch_bounds__(256) head_train_fwd_kernel(const uint16_t* __restrict__ x, int64_t ldx, int T, int HW,
                                                             int C, int kt, const float* __restrict__ keep,
                                                             float* __restrict__ u) {
    const int b = blockIdx.x;
    const int c = blockIdx.y * 256 + threadIdx.x;
    if (c >= C) return;
    const int P = T - kt + 1;
    const float norm = 1.0f / ((float)P * kt * HW);
    float s = 0.f;
    for (int t = 0; t < T; ++t) {
        float st = 0.f;
        for (int q = 0; q < HW; ++q) st += bf2f(x[((int64_t)(b * T + t) * HW + q) * ldx + c]);
        s += st * head_w(keep, b, t, c, T, kt, C);
    }
    u[(int64_t)b * C + c] = s * norm;
}

__global__ void __launch_bounds__(256) head_train_bwd_kernel(const float* __restrict__ du, int T, int HW, int C, int kt,
                                                             const float* __restrict__ keep, int64_t total,
                                                             float* __restrict__ dx, int64_t lddx) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= total) return;
    const int c = (int)(i % C);
    const int64_t row = i / C;
    const int t = (int)((row / HW) % T);
    const int b = (int)(row / ((int64_t)HW * T));
    const int P = T - kt + 1;
    dx[row * lddx + c] = du[(int64_t)b * C + c] * head_w(keep, b, t, c, T, kt, C) / ((float)P * kt * HW);
}

// logits[b][c] = Wc[c] . u[b] + bc[c] (fp32), one workgroup per clip
__global__ void __launch_bounds__(256) head_logits_kernel(const float* __restrict__ u, int C, const float* __restrict__ Wc,
                                                          const float* __restrict__ bc, int nl, float* __restrict__ logits) {
    const int b = blockIdx.x;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int c = w; c < nl; c += 4) {
        float a = 0.f;
        for (int n = lane; n < C; n += 64) a += u[(int64_t)b * C + n] * Wc[(int64_t)c * C + n];
        a = wave_sum(a);
        if (lane == 0) logits[(int64_t)b * nl + c] = a + bc[c];
    }
}

static Geom make_geom(int64_t T, int64_t H, int64_t W, int64_t C, const int* k, const int* s, const int* p) {
    Geom g;
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

}  // namespace rbwd
}  // namespace vc

using namespace vc;
using namespace vc::rbwd;

extern "C" {

int vc_col2im_cl(const uint16_t* dA, int64_t lda, int64_t B, int64_t T, int64_t H, int64_t W, int64_t C,
                 const int* kernel, const int* stride, const int* pad, float* dx, int64_t lddx, hipStream_t stream) {
    if (!dA || !dx || !kernel || !stride || !pad) return fail(VC_ERR_INVALID_ARG, "vc_col2im_cl: null pointer");
    if (!geom_ok(kernel, stride, pad) || B <= 0 || T <= 0 || H <= 0 || W <= 0 || C <= 0 || lddx < C)
        return fail(VC_ERR_INVALID_ARG, "vc_col2im_cl: bad geometry");
    const Geom g = make_geom(T, H, W, C, kernel, stride, pad);
    if (lda < (int64_t)g.kt * g.kh * g.kw * C) return fail(VC_ERR_INVALID_ARG, "vc_col2im_cl: lda < kernel volume * C");
    const int64_t total = B * T * H * W * C;
    col2im_cl_kernel<<<(unsigned)((total + 255) / 256), 256, 0, stream>>>(dA, lda, total, g, dx, lddx);
    return check_launch("vc_col2im_cl");
}

int vc_maxpool3d_bwd(const uint16_t* x, int64_t ldx, const void* dy, int dy_bf16, int64_t lddy, int64_t B, int64_t T,
                     int64_t H, int64_t W, int64_t C, const int* kernel, const int* stride, const int* pad, float* dx,
                     int64_t lddx, hipStream_t stream) {
    if (!x || !dy || !dx || !kernel || !stride || !pad) return fail(VC_ERR_INVALID_ARG, "vc_maxpool3d_bwd: null pointer");
    if (!geom_ok(kernel, stride, pad) || B <= 0 || C <= 0) return fail(VC_ERR_INVALID_ARG, "vc_maxpool3d_bwd: bad geometry");
    const Geom g = make_geom(T, H, W, C, kernel, stride, pad);
    const int64_t total = B * T * H * W * C;
    if (dy_bf16)
        maxpool_bwd_cl_kernel<uint16_t><<<(unsigned)((total + 255) / 256), 256, 0, stream>>>(
            x, ldx, (const uint16_t*)dy, lddy, total, g, dx, lddx);
    else
        maxpool_bwd_cl_kernel<float><<<(unsigned)((total + 255) / 256), 256, 0, stream>>>(x, ldx, (const float*)dy, lddy,
                                                                                         total, g, dx, lddx);
    return check_launch("vc_maxpool3d_bwd");
}

// row chunks of the partial-sum pass: ~128 rows each (thousands of workgroups at the
// 400k-row stage-1 maps), at most 4096
static int64_t bn_splits(int64_t M) {
    int64_t s = (M + 127) / 128;
    return s < 1 ? 1 : (s > 4096 ? 4096 : s);
}

int vc_batchnorm_train_fwd(const float* y, int64_t ldy, int64_t M, int64_t C, const float* gamma, const float* beta,
                           float eps, float momentum, float* running_mean, float* running_var, const void* res,
                           int res_bf16, int64_t ldr, int relu, uint16_t* z, int64_t ldz, float* stat, float* work,
                           int64_t work_elems, hipStream_t stream) {
    if (!y || !gamma || !beta || !z || !stat || !work) return fail(VC_ERR_INVALID_ARG, "vc_batchnorm_train_fwd: null pointer");
    if (M <= 0 || C <= 0 || C % 4 || ldy % 4 || ldy < C || ldz < C || ((uintptr_t)y & 15))
        return fail(VC_ERR_INVALID_ARG, "vc_batchnorm_train_fwd: bad shape (C % 4, 16-B rows)");
    if ((running_mean == nullptr) != (running_var == nullptr))
        return fail(VC_ERR_INVALID_ARG, "vc_batchnorm_train_fwd: running_mean and running_var go together");
    const int64_t ns = bn_splits(M), rps = (M + ns - 1) / ns;
    if (work_elems < ns * 2 * C) return fail(VC_ERR_INVALID_ARG, "vc_batchnorm_train_fwd: work too small");
    const dim3 gp((unsigned)((C + 255) / 256), (unsigned)ns);
    const unsigned gf = (unsigned)C;
    bn_partial_kernel<0><<<gp, 256, 0, stream>>>(y, ldy, M, (int)C, rps, stat, nullptr, 0, nullptr, 0, 0, work);
    bn_finalize_kernel<0><<<gf, 256, 0, stream>>>(work, (int)ns, M, (int)C, eps, momentum, stat, nullptr, nullptr,
                                                  nullptr, nullptr);
    bn_partial_kernel<1><<<gp, 256, 0, stream>>>(y, ldy, M, (int)C, rps, stat, nullptr, 0, nullptr, 0, 0, work);
    bn_finalize_kernel<1><<<gf, 256, 0, stream>>>(work, (int)ns, M, (int)C, eps, momentum, stat, running_mean,
                                                  running_var, nullptr, nullptr);
    const unsigned ga = (unsigned)((M * (C / 4) + 255) / 256);
    if (res && res_bf16)
        bn_apply_kernel<uint16_t><<<ga, 256, 0, stream>>>(y, ldy, M, (int)C, stat, gamma, beta, (const uint16_t*)res, ldr,
                                                         relu, z, ldz);
    else
        bn_apply_kernel<float><<<ga, 256, 0, stream>>>(y, ldy, M, (int)C, stat, gamma, beta, (const float*)res, ldr, relu,
                                                      z, ldz);
    return check_launch("vc_batchnorm_train_fwd");
}

int vc_batchnorm_train_bwd(const float* y, int64_t ldy, int64_t M, int64_t C, const float* stat, const float* gamma,
                           const float* dz, int64_t lddz, const uint16_t* z, int64_t ldz, int relu, float* dy,
                           int64_t lddy, float* dres, int64_t lddr, float* dgamma, float* dbeta, float* work,
                           int64_t work_elems, hipStream_t stream) {
    if (!y || !stat || !gamma || !dz || !dy || !dgamma || !dbeta || !work || (relu && !z))
        return fail(VC_ERR_INVALID_ARG, "vc_batchnorm_train_bwd: null pointer");
    if (M <= 0 || C <= 0 || ldy < C || lddz < C || lddy < C) return fail(VC_ERR_INVALID_ARG, "vc_batchnorm_train_bwd: bad shape");
    const int64_t ns = bn_splits(M), rps = (M + ns - 1) / ns;
    if (work_elems < ns * 2 * C) return fail(VC_ERR_INVALID_ARG, "vc_batchnorm_train_bwd: work too small");
    bn_partial_kernel<2><<<dim3((unsigned)((C + 255) / 256), (unsigned)ns), 256, 0, stream>>>(
        y, ldy, M, (int)C, rps, stat, dz, lddz, z, ldz, relu, work);
    bn_finalize_kernel<2><<<(unsigned)C, 256, 0, stream>>>(work, (int)ns, M, (int)C, 0.f, 0.f, nullptr,
                                                                          nullptr, nullptr, dbeta, dgamma);
    bn_bwd_kernel<<<(unsigned)((M * C + 255) / 256), 256, 0, stream>>>(y, ldy, M, (int)C, stat, gamma, dbeta, dgamma, dz,
                                                                       lddz, z, ldz, relu, dy, lddy, dres, lddr);
    return check_launch("vc_batchnorm_train_bwd");
}

int vc_resnet_head_train(const uint16_t* x, int64_t ldx, int64_t B, int64_t T, int64_t HW, int64_t C, int pool_t,
                         const float* keep, const float* Wc, const float* bc, int64_t num_labels, float* u,
                         float* logits, hipStream_t stream) {
    if (!x || !keep || !u || !Wc || !bc || !logits) return fail(VC_ERR_INVALID_ARG, "vc_resnet_head_train: null pointer");
    if (B <= 0 || T <= 0 || HW <= 0 || C <= 0 || pool_t <= 0 || pool_t > T || num_labels <= 0)
        return fail(VC_ERR_INVALID_ARG, "vc_resnet_head_train: bad shape");
    head_train_fwd_kernel<<<dim3((unsigned)B, (unsigned)((C + 255) / 256)), 256, 0, stream>>>(x, ldx, (int)T, (int)HW,
                                                                                            (int)C, pool_t, keep, u);
    head_logits_kernel<<<(unsigned)B, 256, 0, stream>>>(u, (int)C, Wc, bc, (int)num_labels, logits);
    return check_launch("vc_resnet_head_train");
}

int vc_resnet_head_train_bwd(const float* du, int64_t B, int64_t T, int64_t HW, int64_t C, int pool_t, const float* keep,
                             float* dx, int64_t lddx, hipStream_t stream) {
    if (!du || !keep || !dx) return fail(VC_ERR_INVALID_ARG, "vc_resnet_head_train_bwd: null pointer");
    if (B <= 0 || T <= 0 || HW <= 0 || C <= 0 || pool_t <= 0 || pool_t > T || lddx < C)
        return fail(VC_ERR_INVALID_ARG, "vc_resnet_head_train_bwd: bad shape");
    const int64_t total = B * T * HW * C;
    head_train_bwd_kernel<<<(unsigned)((total + 255) / 256), 256, 0, stream>>>(du, (int)T, (int)HW, (int)C, pool_t, keep,
                                                                              total, dx, lddx);
    return check_launch("vc_resnet_head_train_bwd");
}

}  // extern "C"
