// HBM-bound kernels of the path: frame gather/normalise, tubelet im2col, LayerNorm,
// CLS init and the classifier head.  Plus the C-ABI error plumbing.
#include "common.hpp"

#include <cstdio>

namespace vc {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        g_last_error = std::string(what) + ": " + hipGetErrorString(e);
        return (int)e;
    }
    return 0;
}

// ---------------------------------------------------------------------------------
// Frame gather.  One thread moves 16 B of a source frame row (u8 mode) or 4 pixels
// (float modes: 12 source bytes -> 3 planes x 4 values).
// frames [nclips][F][H][W][C] u8; idx [nclips][T]; clamp like dataset.py:252-253.
// ---------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) gather_u8_kernel(const uint8_t* __restrict__ frames, int64_t F,
                                                        int64_t frame_bytes, const int64_t* __restrict__ idx,
                                                        int64_t T, uint8_t* __restrict__ out) {
    const int64_t clip_t = blockIdx.y;  // clip * T + t
    const int64_t clip = clip_t / T;
    int64_t f = idx[clip_t];
    f = f < 0 ? 0 : (f > F - 1 ? F - 1 : f);
    const uint8_t* src = frames + (clip * F + f) * frame_bytes;
    uint8_t* dst = out + clip_t * frame_bytes;
    const int64_t n16 = frame_bytes >> 4;
    for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n16; i += (int64_t)gridDim.x * 256)
        reinterpret_cast<uint4*>(dst)[i] = reinterpret_cast<const uint4*>(src)[i];
    // tail bytes (frame_bytes not a multiple of 16)
    const int64_t tail0 = n16 << 4;
    if (blockIdx.x == 0)
        for (int64_t i = tail0 + threadIdx.x; i < frame_bytes; i += 256) dst[i] = src[i];
}

template <bool BF16>
__global__ void __launch_bounds__(256) gather_norm_kernel(const uint8_t* __restrict__ frames, int64_t F,
                                                          int64_t HW, const int64_t* __restrict__ idx, int64_t T,
                                                          float scale, float shift, void* __restrict__ out) {
    // C == 3 (RGB) specialisation: thread handles 4 consecutive pixels = 12 bytes.
    const int64_t clip_t = blockIdx.y;
    const int64_t clip = clip_t / T;
    int64_t f = idx[clip_t];
    f = f < 0 ? 0 : (f > F - 1 ? F - 1 : f);
    const uint8_t* src = frames + (clip * F + f) * HW * 3;
    const int64_t nq = HW >> 2;
    for (int64_t q = blockIdx.x * 256 + threadIdx.x; q < nq; q += (int64_t)gridDim.x * 256) {
        const uint32_t* s32 = reinterpret_cast<const uint32_t*>(src + q * 12);
        uint32_t w0 = s32[0], w1 = s32[1], w2 = s32[2];
        uint8_t b[12];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            b[i] = (w0 >> (8 * i)) & 0xff;
            b[4 + i] = (w1 >> (8 * i)) & 0xff;
            b[8 + i] = (w2 >> (8 * i)) & 0xff;
        }
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            float v0 = (float)b[0 * 3 + c] * scale + shift;
            float v1 = (float)b[1 * 3 + c] * scale + shift;
            float v2 = (float)b[2 * 3 + c] * scale + shift;
            float v3 = (float)b[3 * 3 + c] * scale + shift;
            const int64_t o = (clip_t * 3 + c) * HW + q * 4;
            if (BF16) {
                uint2 p;
                p.x = pack2bf(v0, v1);
                p.y = pack2bf(v2, v3);
                *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(out) + o) = p;
            } else {
                *reinterpret_cast<float4*>(reinterpret_cast<float*>(out) + o) = make_float4(v0, v1, v2, v3);
            }
        }
    }
    // tail pixels (HW % 4)
    if (blockIdx.x == 0) {
        for (int64_t p = (nq << 2) + threadIdx.x; p < HW; p += 256)
            for (int c = 0; c < 3; ++c) {
                float v = (float)src[p * 3 + c] * scale + shift;
                const int64_t o = (clip_t * 3 + c) * HW + p;
                if (BF16)
                    reinterpret_cast<uint16_t*>(out)[o] = f2bf(v);
                else
                    reinterpret_cast<float*>(out)[o] = v;
            }
    }
}

// ---------------------------------------------------------------------------------
// Tubelet im2col.  pixel f32 [B][T][C][H][W] (layout 0, HF video models) or [B][C][T][H][W]
// (layout 1, torchvision video models) -> A[token][(c,kt,kh,kw)] bf16, token in (b,t',hp,wp)
// order (order 0, ViViT / Swin) or (b,hp,wp,t') order (order 1: patch-major, time-minor,
// the TimeSformer token order).  One thread converts VEC consecutive pixels of one image
// row (VEC = 8, or 4 for 4-wide patches such as Swin's 2x4x4).
// ---------------------------------------------------------------------------------
// klo > 0 (the split-operand build): the 16-bit rounding residual x - (float)to16(x) also goes to
// column klo + k, so A = [A_hi | A_lo] (vc_patch_im2col_split_h16).
template <int VEC, int ET = VC_ELEM_BF16>
__global__ void __launch_bounds__(256) im2col_kernel(const float* __restrict__ pix, int64_t totalv, int T, int C,
                                                     int H, int W, int kt, int kh, int kw, int order, int layout,
                                                     uint16_t* __restrict__ A, int64_t lda, int64_t klo = 0) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= totalv) return;
    const int WV = W / VEC;
    int64_t r = i;
    const int xv = r % WV;
    r /= WV;
    const int y = r % H;
    r /= H;
    const int c = r % C;
    r /= C;
    const int t = r % T;
    const int64_t b = r / T;
    const int64_t plane = layout ? ((b * C + c) * T + t) : ((b * T + t) * C + c);
    const float4* s = reinterpret_cast<const float4*>(pix + (plane * H + y) * (int64_t)W + xv * VEC);
    const int nt = T / kt, nh = H / kh, nw = W / kw;
    const int tp = t / kt, it = t % kt, hp = y / kh, ih = y % kh;
    const int x = xv * VEC, wp = x / kw, iw = x % kw;
    const int64_t m = order ? ((b * nh + hp) * nw + wp) * (int64_t)nt + tp : ((b * nt + tp) * nh + hp) * (int64_t)nw + wp;
    const int64_t k = (((int64_t)c * kt + it) * kh + ih) * kw + iw;
    const float4 u = s[0];
    if constexpr (VEC == 8) {
        const float4 v = s[1];
        uint4 o;
        o.x = pack2<ET>(u.x, u.y);
        o.y = pack2<ET>(u.z, u.w);
        o.z = pack2<ET>(v.x, v.y);
        o.w = pack2<ET>(v.z, v.w);
        *reinterpret_cast<uint4*>(A + m * lda + k) = o;
        if (klo > 0) {
            auto lo = [](unsigned p, float a, float b) {
                return pack2<ET>(a - from16<ET>((unsigned short)(p & 0xffff)), b - from16<ET>((unsigned short)(p >> 16)));
            };
            uint4 l;
            l.x = lo(o.x, u.x, u.y);
            l.y = lo(o.y, u.z, u.w);
            l.z = lo(o.z, v.x, v.y);
            l.w = lo(o.w, v.z, v.w);
            *reinterpret_cast<uint4*>(A + m * lda + klo + k) = l;
        }
    } else {
        uint2 o;
        o.x = pack2<ET>(u.x, u.y);
        o.y = pack2<ET>(u.z, u.w);
        *reinterpret_cast<uint2*>(A + m * lda + k) = o;
    }
}

// ---------------------------------------------------------------------------------
// LayerNorm f32 -> bf16, one wave per row, D = 64*V*4 (V float4 per lane).  R rows per wave (rows
// w, w + 4, ... of the workgroup's 4R): every row's loads, and gamma / beta, are issued before the
// first reduction, so a wave keeps R x 3 KB in flight instead of one row's (the kernel is HBM-latency
// bound at one row per wave: 13.1 us for 12800 rows, 0.55 of HBM peak, round 5).  Same arithmetic per
// row for any R.
// ---------------------------------------------------------------------------------
template <int V, int ET = VC_ELEM_BF16, int R = 1>
__global__ void __launch_bounds__(256) layernorm_kernel(const float* __restrict__ x, int64_t ldx, int64_t M,
                                                        const float* __restrict__ g, const float* __restrict__ be,
                                                        float eps, uint16_t* __restrict__ y, int64_t ldy) {
    // no FMA contraction: the R row slots of a wave must round identically (a row's result may not
    // depend on its slot, i.e. on its position in the batch -- batch invariance)
#pragma clang fp contract(off)
    const int lane = threadIdx.x & 63;
    const int64_t row0 = (int64_t)blockIdx.x * 4 * R + (threadIdx.x >> 6);
    if (row0 >= M) return;
    constexpr int D = V * 256;
    const float4* g4 = reinterpret_cast<const float4*>(g);
    const float4* b4 = reinterpret_cast<const float4*>(be);
    float4 gg[V], bb[V], v[R][V];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int64_t row = row0 + 4 * r;
        const float4* xr = reinterpret_cast<const float4*>(x + (row < M ? row : row0) * ldx);
#pragma unroll
        for (int i = 0; i < V; ++i) v[r][i] = xr[i * 64 + lane];
    }
#pragma unroll
    for (int i = 0; i < V; ++i) {
        gg[i] = g4[i * 64 + lane];
        bb[i] = b4[i * 64 + lane];
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int64_t row = row0 + 4 * r;
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < V; ++i) s += (v[r][i].x + v[r][i].y) + (v[r][i].z + v[r][i].w);
        const float mean = wave_sum(s) * (1.0f / D);
        float q = 0.f;
#pragma unroll
        for (int i = 0; i < V; ++i) {
            float a = v[r][i].x - mean, b = v[r][i].y - mean, c = v[r][i].z - mean, d = v[r][i].w - mean;
            q += (a * a + b * b) + (c * c + d * d);
        }
        const float rstd = rsqrtf(wave_sum(q) * (1.0f / D) + eps);
        if (row < M) {
#pragma unroll
            for (int i = 0; i < V; ++i) {
                uint2 o;
                o.x = pack2<ET>((v[r][i].x - mean) * rstd * gg[i].x + bb[i].x, (v[r][i].y - mean) * rstd * gg[i].y + bb[i].y);
                o.y = pack2<ET>((v[r][i].z - mean) * rstd * gg[i].z + bb[i].z, (v[r][i].w - mean) * rstd * gg[i].w + bb[i].w);
                *reinterpret_cast<uint2*>(y + row * ldy + (i * 64 + lane) * 4) = o;
            }
        }
    }
}

// LayerNorm for any D % 4 == 0, D <= 1024 (Swin's 96/192/384, TimeSformer-tiny 128 ...):
// one wave per row held in registers (up to 4 float4 per lane, masked), single HBM pass.
template <bool OUTF32, int ET = VC_ELEM_BF16>
__global__ void __launch_bounds__(256) layernorm_reg_kernel(const float* __restrict__ x, int64_t ldx, int64_t M, int D,
                                                            const float* __restrict__ g, const float* __restrict__ be,
                                                            float eps, void* __restrict__ y, int64_t ldy) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= M) return;
    const float* xr = x + row * ldx;
    float4 v[4];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int n = (i * 64 + lane) * 4;
        v[i] = n < D ? *reinterpret_cast<const float4*>(xr + n) : make_float4(0.f, 0.f, 0.f, 0.f);
        s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
    }
    const float mean = wave_sum(s) / (float)D;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        if ((i * 64 + lane) * 4 < D) {
            const float a = v[i].x - mean, b = v[i].y - mean, c = v[i].z - mean, d = v[i].w - mean;
            q += (a * a + b * b) + (c * c + d * d);
        }
    }
    const float rstd = rsqrtf(wave_sum(q) / (float)D + eps);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int n = (i * 64 + lane) * 4;
        if (n < D) {
            const float4 gg = *reinterpret_cast<const float4*>(g + n), bb = *reinterpret_cast<const float4*>(be + n);
            const float o0 = (v[i].x - mean) * rstd * gg.x + bb.x, o1 = (v[i].y - mean) * rstd * gg.y + bb.y;
            const float o2 = (v[i].z - mean) * rstd * gg.z + bb.z, o3 = (v[i].w - mean) * rstd * gg.w + bb.w;
            if constexpr (OUTF32) {
                *reinterpret_cast<float4*>(reinterpret_cast<float*>(y) + row * ldy + n) = make_float4(o0, o1, o2, o3);
            } else {
                uint2 o;
                o.x = pack2<ET>(o0, o1);
                o.y = pack2<ET>(o2, o3);
                *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(y) + row * ldy + n) = o;
            }
        }
    }
}

// Narrow-row LayerNorm (Swin's D = 96 / 192 / 384 at 200k / 50k / 12k rows): L lanes per row,
// 64 / L rows per wave, each lane V float4 (masked past D), single HBM pass, reductions over
// the L-lane group.  A whole wave per 96-wide row (layernorm_reg_kernel) leaves 40 of 64
// lanes idle and launches one wave per 384 bytes: 47 us for Swin-T stage 1 at B = 4 (2.5 TB/s).
template <int L, int V, bool OUTF32, int ET = VC_ELEM_BF16>
__global__ void __launch_bounds__(256) layernorm_grp_kernel(const float* __restrict__ x, int64_t ldx, int64_t M, int D,
                                                            const float* __restrict__ g, const float* __restrict__ be,
                                                            float eps, void* __restrict__ y, int64_t ldy) {
    const int sub = threadIdx.x & (L - 1);
    const int64_t row = ((int64_t)blockIdx.x * 256 + threadIdx.x) / L;
    if (row >= M) return;  // whole L-lane groups exit together
    const float* xr = x + row * ldx;
    float4 v[V];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < V; ++i) {
        const int n = (i * L + sub) * 4;
        v[i] = n < D ? *reinterpret_cast<const float4*>(xr + n) : make_float4(0.f, 0.f, 0.f, 0.f);
        s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
    }
    const float mean = group_sum<L>(s) / (float)D;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < V; ++i) {
        if ((i * L + sub) * 4 < D) {
            const float a = v[i].x - mean, b = v[i].y - mean, c = v[i].z - mean, d = v[i].w - mean;
            q += (a * a + b * b) + (c * c + d * d);
        }
    }
    const float rstd = rsqrtf(group_sum<L>(q) / (float)D + eps);
#pragma unroll
    for (int i = 0; i < V; ++i) {
        const int n = (i * L + sub) * 4;
        if (n < D) {
            const float4 gg = *reinterpret_cast<const float4*>(g + n), bb = *reinterpret_cast<const float4*>(be + n);
            const float o0 = (v[i].x - mean) * rstd * gg.x + bb.x, o1 = (v[i].y - mean) * rstd * gg.y + bb.y;
            const float o2 = (v[i].z - mean) * rstd * gg.z + bb.z, o3 = (v[i].w - mean) * rstd * gg.w + bb.w;
            if constexpr (OUTF32) {
                *reinterpret_cast<float4*>(reinterpret_cast<float*>(y) + row * ldy + n) = make_float4(o0, o1, o2, o3);
            } else {
                uint2 o;
                o.x = pack2<ET>(o0, o1);
                o.y = pack2<ET>(o2, o3);
                *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(y) + row * ldy + n) = o;
            }
        }
    }
}

// lanes per row for a narrow LayerNorm: the smallest L in {8, 16, 32} with D <= L * 3 float4
// (else L * 4), 0 when D needs the whole-wave kernel
static inline int grp_lanes(int64_t D, int* V) {
    for (int L = 8; L <= 32; L *= 2) {
        if (D <= L * 12) { *V = 3; return L; }
        if (D <= L * 16) { *V = 4; return L; }
    }
    return 0;
}

template <bool OUTF32, int ET = VC_ELEM_BF16>
static bool launch_ln_grp(const float* x, int64_t ldx, int64_t M, int64_t D, const float* g, const float* be, float eps,
                          void* y, int64_t ldy, hipStream_t stream) {
    int V = 0;
    const int L = grp_lanes(D, &V);
    if (!L) return false;
    const unsigned nb = (unsigned)((M * L + 255) / 256);
#define VC_LN_GRP(LL, VV) layernorm_grp_kernel<LL, VV, OUTF32, ET><<<nb, 256, 0, stream>>>(x, ldx, M, (int)D, g, be, eps, y, ldy)
    if (L == 8) { if (V == 3) VC_LN_GRP(8, 3); else VC_LN_GRP(8, 4); }
    else if (L == 16) { if (V == 3) VC_LN_GRP(16, 3); else VC_LN_GRP(16, 4); }
    else { if (V == 3) VC_LN_GRP(32, 3); else VC_LN_GRP(32, 4); }
#undef VC_LN_GRP
    return true;
}

// Generic-width LayerNorm (any D): one wave per row, three passes over the row (L1/L2-resident).
// OUTF32: the output is f32 (y is a float*), e.g. Swin's patch_embed.norm feeding the residual stream.
template <bool OUTF32 = false, int ET = VC_ELEM_BF16>
__global__ void __launch_bounds__(256) layernorm_any_kernel(const float* __restrict__ x, int64_t ldx, int64_t M,
                                                            int D, const float* __restrict__ g,
                                                            const float* __restrict__ be, float eps,
                                                            void* __restrict__ y, int64_t ldy) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= M) return;
    const float* xr = x + row * ldx;
    float s = 0.f;
    for (int n = lane; n < D; n += 64) s += xr[n];
    const float mean = wave_sum(s) / (float)D;
    float q = 0.f;
    for (int n = lane; n < D; n += 64) {
        const float d = xr[n] - mean;
        q += d * d;
    }
    const float rstd = rsqrtf(wave_sum(q) / (float)D + eps);
    for (int n = lane; n < D; n += 64) {
        const float v = (xr[n] - mean) * rstd * g[n] + be[n];
        if constexpr (OUTF32)
            reinterpret_cast<float*>(y)[row * ldy + n] = v;
        else
            reinterpret_cast<uint16_t*>(y)[row * ldy + n] = to16<ET>(v);
    }
}

__global__ void cls_init_kernel(const float* __restrict__ cls, const float* __restrict__ pos, float* __restrict__ x,
                                int64_t ldx, int64_t S, int64_t D) {
    const int64_t b = blockIdx.x;
    for (int64_t n = threadIdx.x; n < D; n += blockDim.x) x[b * S * ldx + n] = cls[n] + pos[n];
}

// LN of each clip's CLS row then the tiny classifier GEMV, fp32 throughout.
__global__ void __launch_bounds__(256) cls_head_kernel(const float* __restrict__ x, int64_t ldx, int64_t S, int64_t D,
                                                       const float* __restrict__ g, const float* __restrict__ be,
                                                       float eps, const float* __restrict__ Wc,
                                                       const float* __restrict__ bc, int64_t nl,
                                                       float* __restrict__ logits) {
    __shared__ float red[8];
    __shared__ float ybuf[4096];
    const int64_t b = blockIdx.x;
    const float* xr = x + b * S * ldx;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    float s = 0.f;
    for (int64_t n = tid; n < D; n += 256) s += xr[n];
    s = wave_sum(s);
    if (lane == 0) red[w] = s;
    __syncthreads();
    const float mean = (red[0] + red[1] + red[2] + red[3]) / (float)D;
    __syncthreads();
    float q = 0.f;
    for (int64_t n = tid; n < D; n += 256) {
        float d = xr[n] - mean;
        q += d * d;
    }
    q = wave_sum(q);
    if (lane == 0) red[w] = q;
    __syncthreads();
    const float rstd = rsqrtf((red[0] + red[1] + red[2] + red[3]) / (float)D + eps);
    for (int64_t n = tid; n < D; n += 256) ybuf[n] = (xr[n] - mean) * rstd * g[n] + be[n];
    __syncthreads();
    for (int64_t c = w; c < nl; c += 4) {
        float a = 0.f;
        for (int64_t n = lane; n < D; n += 64) a += ybuf[n] * Wc[c * D + n];
        a = wave_sum(a);
        if (lane == 0) logits[b * nl + c] = a + bc[c];
    }
}

// `blocks` one-wave workgroups, each sleeping `iters` x s_sleep 127 (about 8k clocks each): the
// hardware-queue probe of vclip_amd.streams.pick_streams -- spins on two streams overlap iff the streams
// sit on different hardware queues (kernels of streams that share one run one after the other)
__global__ void __launch_bounds__(64) spin_kernel(int64_t iters) {
    for (int64_t i = 0; i < iters; ++i) __builtin_amdgcn_s_sleep(127);
}

}  // namespace vc

using namespace vc;

extern "C" {

int vc_spin(int64_t iters, int64_t blocks, hipStream_t stream) {
    if (iters < 0 || iters > (int64_t{1} << 20)) return fail(VC_ERR_INVALID_ARG, "vc_spin: iters outside [0, 2^20]");
    if (blocks < 1 || blocks > (int64_t{1} << 20)) return fail(VC_ERR_INVALID_ARG, "vc_spin: blocks outside [1, 2^20]");
    spin_kernel<<<(unsigned)blocks, 64, 0, stream>>>(iters);
    return check_launch("vc_spin");
}

const char* vc_version(void) { return "vclip 0.1.0 gfx950"; }

const char* vc_last_error(void) { return g_last_error.c_str(); }

int vc_frame_gather(const uint8_t* frames, int64_t nclips, int64_t F, int64_t H, int64_t W, int64_t C,
                    const int64_t* idx, int64_t T, int out_kind, float scale, float shift, void* out,
                    hipStream_t stream) {
    if (!frames || !idx || !out) return fail(VC_ERR_INVALID_ARG, "vc_frame_gather: null pointer");
    if (nclips <= 0 || F <= 0 || H <= 0 || W <= 0 || C <= 0 || T <= 0)
        return fail(VC_ERR_INVALID_ARG, "vc_frame_gather: non-positive size");
    if (nclips * T > 65535) return fail(VC_ERR_INVALID_ARG, "vc_frame_gather: nclips*T > 65535");
    const int64_t HW = H * W;
    if (out_kind == VC_GATHER_U8_NHWC) {
        const int64_t fb = HW * C;
        if (((uintptr_t)frames | (uintptr_t)out) & 15 || fb & 15)
            return fail(VC_ERR_INVALID_ARG, "vc_frame_gather(u8): frames/out need 16-B alignment and frame size % 16 == 0");
        int64_t nb = (fb / 16 + 255) / 256;
        dim3 grid((unsigned)(nb > 256 ? 256 : nb), (unsigned)(nclips * T));
        gather_u8_kernel<<<grid, 256, 0, stream>>>(frames, F, fb, idx, T, (uint8_t*)out);
        return check_launch("vc_frame_gather");
    }
    if (C != 3) return fail(VC_ERR_UNSUPPORTED, "vc_frame_gather: float modes need C == 3");
    if (((uintptr_t)frames & 3) || ((uintptr_t)out & 15) || (HW & 3))
        return fail(VC_ERR_INVALID_ARG, "vc_frame_gather: alignment (frames 4 B, out 16 B, H*W % 4 == 0)");
    int64_t nb = (HW / 4 + 255) / 256;
    dim3 grid((unsigned)(nb > 256 ? 256 : nb), (unsigned)(nclips * T));
    if (out_kind == VC_GATHER_F32_NCHW)
        gather_norm_kernel<false><<<grid, 256, 0, stream>>>(frames, F, HW, idx, T, scale, shift, out);
    else if (out_kind == VC_GATHER_BF16_NCHW)
        gather_norm_kernel<true><<<grid, 256, 0, stream>>>(frames, F, HW, idx, T, scale, shift, out);
    else
        return fail(VC_ERR_INVALID_ARG, "vc_frame_gather: bad out_kind");
    return check_launch("vc_frame_gather");
}

int vc_patch_im2col_h16(const float* pixel_values, int64_t B, int64_t T, int64_t C, int64_t H, int64_t W, int kt,
                        int kh, int kw, int token_order, int layout, int elem, uint16_t* A, int64_t lda,
                        hipStream_t stream) {
    if (elem != VC_ELEM_BF16 && elem != VC_ELEM_F16) return fail(VC_ERR_INVALID_ARG, "vc_patch_im2col: bad elem");
    if (!pixel_values || !A) return fail(VC_ERR_INVALID_ARG, "vc_patch_im2col: null pointer");
    if (kt <= 0 || kh <= 0 || kw <= 0 || T % kt || H % kh || W % kw || kw % 4 || W % 4 || lda % 4 ||
        lda < C * kt * kh * kw || ((uintptr_t)pixel_values & 15) || ((uintptr_t)A & 7))
        return fail(VC_ERR_INVALID_ARG, "vc_patch_im2col: shape not divisible by the patch / 4-wide rows / alignment");
    if (token_order != VC_TOKENS_TIME_MAJOR && token_order != VC_TOKENS_PATCH_MAJOR)
        return fail(VC_ERR_INVALID_ARG, "vc_patch_im2col: bad token_order");
    if (layout != VC_VIDEO_BTCHW && layout != VC_VIDEO_BCTHW) return fail(VC_ERR_INVALID_ARG, "vc_patch_im2col: bad layout");
    if (kw % 8 == 0 && lda % 8 == 0 && !((uintptr_t)A & 15)) {
        const int64_t totalv = B * T * C * H * (W / 8);
        const unsigned nb = (unsigned)((totalv + 255) / 256);
        if (elem == VC_ELEM_F16)
            im2col_kernel<8, VC_ELEM_F16><<<nb, 256, 0, stream>>>(pixel_values, totalv, (int)T, (int)C, (int)H, (int)W,
                                                                 kt, kh, kw, token_order, layout, A, lda);
        else
            im2col_kernel<8><<<nb, 256, 0, stream>>>(pixel_values, totalv, (int)T, (int)C, (int)H, (int)W, kt, kh, kw,
                                                    token_order, layout, A, lda);
    } else {
        const int64_t totalv = B * T * C * H * (W / 4);
        const unsigned nb = (unsigned)((totalv + 255) / 256);
        if (elem == VC_ELEM_F16)
            im2col_kernel<4, VC_ELEM_F16><<<nb, 256, 0, stream>>>(pixel_values, totalv, (int)T, (int)C, (int)H, (int)W,
                                                                 kt, kh, kw, token_order, layout, A, lda);
        else
            im2col_kernel<4><<<nb, 256, 0, stream>>>(pixel_values, totalv, (int)T, (int)C, (int)H, (int)W, kt, kh, kw,
                                                    token_order, layout, A, lda);
    }
    return check_launch("vc_patch_im2col");
}

// A = [A_hi | A_lo] (2 K columns, K = C kt kh kw): the 16-bit operand and its rounding residual, for
// vc_gemm_h16_wrap with W = [W_hi | W_hi | W_lo] (A_hi W_hi + A_lo W_hi + A_hi W_lo).  8-wide patches.
int vc_patch_im2col_split_h16(const float* pixel_values, int64_t B, int64_t T, int64_t C, int64_t H, int64_t W,
                              int kt, int kh, int kw, int token_order, int layout, int elem, uint16_t* A, int64_t lda,
                              hipStream_t stream) {
    if (elem != VC_ELEM_BF16 && elem != VC_ELEM_F16) return fail(VC_ERR_INVALID_ARG, "vc_patch_im2col_split: bad elem");
    if (!pixel_values || !A) return fail(VC_ERR_INVALID_ARG, "vc_patch_im2col_split: null pointer");
    const int64_t K = C * kt * kh * kw;
    if (kt <= 0 || kh <= 0 || kw <= 0 || T % kt || H % kh || W % kw || kw % 8 || W % 8 || lda % 8 || lda < 2 * K ||
        K % 8 || ((uintptr_t)pixel_values & 15) || ((uintptr_t)A & 15))
        return fail(VC_ERR_INVALID_ARG, "vc_patch_im2col_split: needs 8-wide patches, lda >= 2K, 16-B alignment");
    if (token_order != VC_TOKENS_TIME_MAJOR && token_order != VC_TOKENS_PATCH_MAJOR)
        return fail(VC_ERR_INVALID_ARG, "vc_patch_im2col_split: bad token_order");
    if (layout != VC_VIDEO_BTCHW && layout != VC_VIDEO_BCTHW)
        return fail(VC_ERR_INVALID_ARG, "vc_patch_im2col_split: bad layout");
    const int64_t totalv = B * T * C * H * (W / 8);
    const unsigned nb = (unsigned)((totalv + 255) / 256);
    if (elem == VC_ELEM_F16)
        im2col_kernel<8, VC_ELEM_F16><<<nb, 256, 0, stream>>>(pixel_values, totalv, (int)T, (int)C, (int)H, (int)W, kt,
                                                             kh, kw, token_order, layout, A, lda, K);
    else
        im2col_kernel<8><<<nb, 256, 0, stream>>>(pixel_values, totalv, (int)T, (int)C, (int)H, (int)W, kt, kh, kw,
                                                token_order, layout, A, lda, K);
    return check_launch("vc_patch_im2col_split");
}

int vc_patch_im2col(const float* pixel_values, int64_t B, int64_t T, int64_t C, int64_t H, int64_t W, int kt, int kh,
                    int kw, int token_order, int layout, uint16_t* A, int64_t lda, hipStream_t stream) {
    return vc_patch_im2col_h16(pixel_values, B, T, C, H, W, kt, kh, kw, token_order, layout, VC_ELEM_BF16, A, lda,
                               stream);
}

int vc_tubelet_im2col(const float* pixel_values, int64_t B, int64_t T, int64_t C, int64_t H, int64_t W, int kt,
                      int kh, int kw, uint16_t* A, int64_t lda, hipStream_t stream) {
    return vc_patch_im2col(pixel_values, B, T, C, H, W, kt, kh, kw, VC_TOKENS_TIME_MAJOR, VC_VIDEO_BTCHW, A, lda, stream);
}

// Row LayerNorm f32 -> 16-bit (ET) for any D: register kernels for the ViViT widths, the
// grouped / register / three-pass kernels for the rest.
extern "C++" template <int ET>
static int layernorm16(const float* x, int64_t ldx, int64_t M, int64_t D, const float* gamma, const float* beta,
                       float eps, uint16_t* y, int64_t ldy, hipStream_t stream) {
    if (!x || !gamma || !beta || !y) return fail(VC_ERR_INVALID_ARG, "vc_layernorm: null pointer");
    if (ldx % 4 || ldy % 4) return fail(VC_ERR_INVALID_ARG, "vc_layernorm: ld must be a multiple of 4");
    const unsigned nb = (unsigned)((M + 3) / 4);
    switch (D) {
        case 256: layernorm_kernel<1, ET><<<nb, 256, 0, stream>>>(x, ldx, M, gamma, beta, eps, y, ldy); break;
        case 512: layernorm_kernel<2, ET><<<nb, 256, 0, stream>>>(x, ldx, M, gamma, beta, eps, y, ldy); break;
        case 768:  // two rows per wave
            layernorm_kernel<3, ET, 2><<<(unsigned)((M + 7) / 8), 256, 0, stream>>>(x, ldx, M, gamma, beta, eps, y, ldy);
            break;
        case 1024: layernorm_kernel<4, ET><<<nb, 256, 0, stream>>>(x, ldx, M, gamma, beta, eps, y, ldy); break;
        default:
            if (D <= 0 || D > 65536) return fail(VC_ERR_INVALID_ARG, "vc_layernorm: bad D");
            if (D <= 1024 && D % 4 == 0 && !(((uintptr_t)x | (uintptr_t)gamma | (uintptr_t)beta) & 15) && !((uintptr_t)y & 7)) {
                if (launch_ln_grp<false, ET>(x, ldx, M, D, gamma, beta, eps, y, ldy, stream)) break;
                layernorm_reg_kernel<false, ET><<<nb, 256, 0, stream>>>(x, ldx, M, (int)D, gamma, beta, eps, y, ldy);
            } else
                layernorm_any_kernel<false, ET><<<nb, 256, 0, stream>>>(x, ldx, M, (int)D, gamma, beta, eps, y, ldy);
    }
    return check_launch("vc_layernorm_f32_h16");
}

int vc_layernorm_f32_h16(const float* x, int64_t ldx, int64_t M, int64_t D, const float* gamma, const float* beta,
                         float eps, int elem, uint16_t* y, int64_t ldy, hipStream_t stream) {
    if (elem == VC_ELEM_F16) return layernorm16<VC_ELEM_F16>(x, ldx, M, D, gamma, beta, eps, y, ldy, stream);
    if (elem == VC_ELEM_BF16) return layernorm16<VC_ELEM_BF16>(x, ldx, M, D, gamma, beta, eps, y, ldy, stream);
    return fail(VC_ERR_INVALID_ARG, "vc_layernorm: bad elem");
}

int vc_layernorm_f32_bf16(const float* x, int64_t ldx, int64_t M, int64_t D, const float* gamma, const float* beta,
                          float eps, uint16_t* y, int64_t ldy, hipStream_t stream) {
    return layernorm16<VC_ELEM_BF16>(x, ldx, M, D, gamma, beta, eps, y, ldy, stream);
}

int vc_layernorm_f32(const float* x, int64_t ldx, int64_t M, int64_t D, const float* gamma, const float* beta,
                     float eps, float* y, int64_t ldy, hipStream_t stream) {
    if (!x || !gamma || !beta || !y) return fail(VC_ERR_INVALID_ARG, "vc_layernorm_f32: null pointer");
    if (D <= 0 || D > 65536 || ldx < D || ldy < D) return fail(VC_ERR_INVALID_ARG, "vc_layernorm_f32: bad D / ld");
    const unsigned nb = (unsigned)((M + 3) / 4);
    if (D <= 1024 && D % 4 == 0 && ldx % 4 == 0 && ldy % 4 == 0 &&
        !(((uintptr_t)x | (uintptr_t)gamma | (uintptr_t)beta | (uintptr_t)y) & 15)) {
        if (!launch_ln_grp<true>(x, ldx, M, D, gamma, beta, eps, y, ldy, stream))
            layernorm_reg_kernel<true><<<nb, 256, 0, stream>>>(x, ldx, M, (int)D, gamma, beta, eps, y, ldy);
    } else
        layernorm_any_kernel<true><<<nb, 256, 0, stream>>>(x, ldx, M, (int)D, gamma, beta, eps, y, ldy);
    return check_launch("vc_layernorm_f32");
}

int vc_cls_init(const float* cls, const float* pos, float* x, int64_t ldx, int64_t B, int64_t S, int64_t D,
                hipStream_t stream) {
    if (!cls || !pos || !x) return fail(VC_ERR_INVALID_ARG, "vc_cls_init: null pointer");
    cls_init_kernel<<<(unsigned)B, 256, 0, stream>>>(cls, pos, x, ldx, S, D);
    return check_launch("vc_cls_init");
}

int vc_cls_head(const float* x, int64_t ldx, int64_t B, int64_t S, int64_t D, const float* gamma, const float* beta,
                float eps, const float* Wc, const float* bc, int64_t num_labels, float* logits, hipStream_t stream) {
    if (!x || !gamma || !beta || !Wc || !bc || !logits) return fail(VC_ERR_INVALID_ARG, "vc_cls_head: null pointer");
    if (D > 4096) return fail(VC_ERR_UNSUPPORTED, "vc_cls_head: D > 4096");
    cls_head_kernel<<<(unsigned)B, 256, 0, stream>>>(x, ldx, S, D, gamma, beta, eps, Wc, bc, num_labels, logits);
    return check_launch("vc_cls_head");
}

}  // extern "C"
