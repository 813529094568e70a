// Backward kernels of the TimeSformer train step (the TimeSformer folder's
// main.py trains by default, timesformer/timesformer_classifier/trainers/trainer.py:139-174).
//
//  * temporal_attn_bwd_kernel — autograd of the temporal branch's self-attention
//    (TimesformerSelfAttention over the T frames of one patch, TF5/models/timesformer/
//    modeling_timesformer.py:148-180 as called from :332-349): per (sequence, head) the T x T
//    scores are recomputed from q' (= q * scale * log2 e, the stored q|k|v layout of the forward),
//    P = softmax, dV = P^T dO, dP = dO V^T, dS = ln2 * P o (dP - rowsum(P o dP)),
//    dQ' = dS K, dK = dS^T Q'.  T <= 32 keys: VALU work, one wave per (sequence, head), the T x T
//    tiles in LDS.  Deterministic (no atomics).
//  * gelu_erf_fwd_kernel / gelu_erf_bwd_kernel — exact GELU (TimeSformer / Swin hidden_act
//    "gelu") as a separate op for the train step: the forward uses the same branch-free
//    erfc restatement as the fused GEMM epilogue (common.hpp gelu_erf), the backward
//    dx = dy * (Phi(x) + x phi(x)).
#include "common.hpp"

namespace vc {

constexpr float LN2 = 0.6931471805599453f;

__device__ __forceinline__ void load_row64(const uint16_t* src, float (&v)[64]) {
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        const v8s raw = *reinterpret_cast<const v8s*>(src + 8 * c);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[8 * c + j] = bf2f((unsigned short)raw[j]);
    }
}

__device__ __forceinline__ float dot_row64(const float (&a)[64], const uint16_t* row) {
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        const v8s raw = *reinterpret_cast<const v8s*>(row + 8 * c);
#pragma unroll
        for (int j = 0; j < 8; ++j) s = __builtin_fmaf(a[8 * c + j], bf2f((unsigned short)raw[j]), s);
    }
    return s;
}

__device__ __forceinline__ void axpy_row64(float (&acc)[64], float a, const uint16_t* row) {
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        const v8s raw = *reinterpret_cast<const v8s*>(row + 8 * c);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[8 * c + j] = __builtin_fmaf(a, bf2f((unsigned short)raw[j]), acc[8 * c + j]);
    }
}

__device__ __forceinline__ void store_row64(uint16_t* dst, const float (&v)[64]) {
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        uint4 w;
        w.x = pack2bf(v[8 * c + 0], v[8 * c + 1]);
        w.y = pack2bf(v[8 * c + 2], v[8 * c + 3]);
        w.z = pack2bf(v[8 * c + 4], v[8 * c + 5]);
        w.w = pack2bf(v[8 * c + 6], v[8 * c + 7]);
        *reinterpret_cast<uint4*>(dst + 8 * c) = w;
    }
}

// grid (B*P sequences, H heads), 64 threads; lane i < T: query i (pass 1), key i (pass 2).
// Rows of sequence n = b*P + p in qkv / dout / dqkv: the clip layout of the forward,
// b*(1 + P*T) + 1 + p*T + t (CLS row first, patch-major, time-minor; CLS rows untouched).
__global__ void __launch_bounds__(64) temporal_attn_bwd_kernel(const uint16_t* __restrict__ qkv, int64_t ld,
                                                               const uint16_t* __restrict__ dout, int64_t lddo, int P,
                                                               int T, int H, uint16_t* __restrict__ dqkv, int64_t lddq) {
    __shared__ float Ps[32][33];
    __shared__ float dSs[32][33];
    const int n = blockIdx.x, h = blockIdx.y, i = threadIdx.x;
    const int D = H * 64;
    const int64_t r0 = (int64_t)(n / P) * (1 + (int64_t)P * T) + 1 + (int64_t)(n % P) * T;
    const uint16_t* qb = qkv + r0 * ld + h * 64;
    const uint16_t* kb = qb + D;
    const uint16_t* vb = qb + 2 * D;
    const uint16_t* db = dout + r0 * lddo + h * 64;
    if (i < T) {
        float q[64], g[64];
        load_row64(qb + (int64_t)i * ld, q);
        load_row64(db + (int64_t)i * lddo, g);
        float m = -INFINITY;
        for (int u = 0; u < T; ++u) {
            const float s = dot_row64(q, kb + (int64_t)u * ld);
            Ps[i][u] = s;
            m = fmaxf(m, s);
        }
        float l = 0.f;
        for (int u = 0; u < T; ++u) {
            const float e = exp2f(Ps[i][u] - m);
            Ps[i][u] = e;
            l += e;
        }
        const float inv = 1.0f / l;
        float delta = 0.f;
        for (int u = 0; u < T; ++u) {
            const float p = Ps[i][u] * inv;
            Ps[i][u] = p;
            const float dp = dot_row64(g, vb + (int64_t)u * ld);
            dSs[i][u] = dp;
            delta = __builtin_fmaf(p, dp, delta);
        }
        float dq[64];
#pragma unroll
        for (int d = 0; d < 64; ++d) dq[d] = 0.f;
        for (int u = 0; u < T; ++u) {
            const float ds = LN2 * Ps[i][u] * (dSs[i][u] - delta);
            dSs[i][u] = ds;
            axpy_row64(dq, ds, kb + (int64_t)u * ld);
        }
        store_row64(dqkv + (r0 + i) * lddq + h * 64, dq);
    }
    __syncthreads();
    if (i < T) {
        float dk[64], dv[64];
#pragma unroll
        for (int d = 0; d < 64; ++d) { dk[d] = 0.f; dv[d] = 0.f; }
        for (int t = 0; t < T; ++t) {
            axpy_row64(dk, dSs[t][i], qb + (int64_t)t * ld);
            axpy_row64(dv, Ps[t][i], db + (int64_t)t * lddo);
        }
        store_row64(dqkv + (r0 + i) * lddq + D + h * 64, dk);
        store_row64(dqkv + (r0 + i) * lddq + 2 * D + h * 64, dv);
    }
}

// exact GELU on bf16 rows [M][N] (ld), 8 elements per thread
__global__ void __launch_bounds__(256) gelu_erf_fwd_kernel(const uint16_t* __restrict__ x, int64_t ldx, int64_t M,
                                                           int N, uint16_t* __restrict__ y, int64_t ldy) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int per_row = N / 8;
    if (i >= M * per_row) return;
    const int64_t m = i / per_row;
    const int c = (int)(i % per_row) * 8;
    const v8s raw = *reinterpret_cast<const v8s*>(x + m * ldx + c);
    uint4 w;
    unsigned* wp = reinterpret_cast<unsigned*>(&w);
#pragma unroll
    for (int j = 0; j < 4; ++j)
        wp[j] = pack2bf(gelu_erf(bf2f((unsigned short)raw[2 * j])), gelu_erf(bf2f((unsigned short)raw[2 * j + 1])));
    *reinterpret_cast<uint4*>(y + m * ldy + c) = w;
}

__device__ __forceinline__ float dgelu_erf(float x) {
    // d/dx x Phi(x) = Phi(x) + x phi(x); Phi from the same erfc restatement as gelu_erf
    const float t = __builtin_amdgcn_rcpf(__builtin_fmaf(0.23164189f, __builtin_fabsf(x), 1.0f));
    float p = __builtin_fmaf(t, 0.5307027145f, -0.7265760135f);
    p = __builtin_fmaf(t, p, 0.7107068705f);
    p = __builtin_fmaf(t, p, -0.142248368f);
    p = __builtin_fmaf(t, p, 0.127414796f);
    const float e = __builtin_amdgcn_exp2f(x * x * -0.72134752044448170f);  // exp(-x^2/2)
    const float hh = t * p * e;
    const float Phi = x >= 0.0f ? 1.0f - hh : hh;
    return Phi + x * e * 0.3989422804014327f;  // phi(x) = exp(-x^2/2) / sqrt(2 pi)
}

// dx = dy * gelu'(x); dy f32 or bf16 (dy_bf16), x bf16 (the pre-activation), dx bf16
__global__ void __launch_bounds__(256) gelu_erf_bwd_kernel(const void* __restrict__ dy, int dy_bf16, int64_t lddy,
                                                           const uint16_t* __restrict__ x, int64_t ldx, int64_t M,
                                                           int N, uint16_t* __restrict__ dx, int64_t lddx) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int per_row = N / 8;
    if (i >= M * per_row) return;
    const int64_t m = i / per_row;
    const int c = (int)(i % per_row) * 8;
    const v8s raw = *reinterpret_cast<const v8s*>(x + m * ldx + c);
    float g[8];
    if (dy_bf16) {
        const v8s gr = *reinterpret_cast<const v8s*>(reinterpret_cast<const uint16_t*>(dy) + m * lddy + c);
#pragma unroll
        for (int j = 0; j < 8; ++j) g[j] = bf2f((unsigned short)gr[j]);
    } else {
        const float* gp = reinterpret_cast<const float*>(dy) + m * lddy + c;
        const float4 a = *reinterpret_cast<const float4*>(gp), b = *reinterpret_cast<const float4*>(gp + 4);
        g[0] = a.x; g[1] = a.y; g[2] = a.z; g[3] = a.w; g[4] = b.x; g[5] = b.y; g[6] = b.z; g[7] = b.w;
    }
    uint4 w;
    unsigned* wp = reinterpret_cast<unsigned*>(&w);
#pragma unroll
    for (int j = 0; j < 4; ++j)
        wp[j] = pack2bf(g[2 * j] * dgelu_erf(bf2f((unsigned short)raw[2 * j])),
                        g[2 * j + 1] * dgelu_erf(bf2f((unsigned short)raw[2 * j + 1])));
    *reinterpret_cast<uint4*>(dx + m * lddx + c) = w;
}

}  // namespace vc

using namespace vc;

extern "C" {

int vc_temporal_attention_bwd(const uint16_t* qkv, int64_t ld, const uint16_t* dout, int64_t lddo, int64_t B, int64_t P,
                              int64_t T, int64_t H, int64_t head_dim, uint16_t* dqkv, int64_t lddq, hipStream_t stream) {
    const int64_t N = B * P;
    if (!qkv || !dout || !dqkv) return fail(VC_ERR_INVALID_ARG, "vc_temporal_attention_bwd: null pointer");
    if (head_dim != 64) return fail(VC_ERR_UNSUPPORTED, "vc_temporal_attention_bwd: head_dim must be 64");
    if (B <= 0 || P <= 0 || N <= 0 || T <= 0 || T > 32 || H <= 0 || H > 65535 || ld < 3 * H * 64 || lddq < 3 * H * 64 || lddo < H * 64 ||
        ld % 8 || lddo % 8 || lddq % 8 || N > 0x7fffffff)
        return fail(VC_ERR_INVALID_ARG, "vc_temporal_attention_bwd: bad shape (T <= 32) / leading dimension");
    if ((((uintptr_t)qkv) | ((uintptr_t)dout) | ((uintptr_t)dqkv)) & 15)
        return fail(VC_ERR_INVALID_ARG, "vc_temporal_attention_bwd: pointers must be 16-byte aligned");
    temporal_attn_bwd_kernel<<<dim3((unsigned)N, (unsigned)H), 64, 0, stream>>>(qkv, ld, dout, lddo, (int)P, (int)T, (int)H,
                                                                                dqkv, lddq);
    return check_launch("vc_temporal_attention_bwd");
}

int vc_gelu_erf(const uint16_t* x, int64_t ldx, int64_t M, int64_t N, uint16_t* y, int64_t ldy, hipStream_t stream) {
    if (!x || !y) return fail(VC_ERR_INVALID_ARG, "vc_gelu_erf: null pointer");
    if (M <= 0 || N <= 0 || N % 8 || ldx % 8 || ldy % 8 || ldx < N || ldy < N)
        return fail(VC_ERR_INVALID_ARG, "vc_gelu_erf: need N % 8 == 0 and 16-byte rows");
    const int64_t total = M * (N / 8);
    gelu_erf_fwd_kernel<<<(unsigned)((total + 255) / 256), 256, 0, stream>>>(x, ldx, M, (int)N, y, ldy);
    return check_launch("vc_gelu_erf");
}

int vc_gelu_erf_bwd(const void* dy, int dy_bf16, int64_t lddy, const uint16_t* x, int64_t ldx, int64_t M, int64_t N,
                    uint16_t* dx, int64_t lddx, hipStream_t stream) {
    if (!dy || !x || !dx) return fail(VC_ERR_INVALID_ARG, "vc_gelu_erf_bwd: null pointer");
    if (M <= 0 || N <= 0 || N % 8 || lddy % 8 || ldx % 8 || lddx % 8 || lddy < N || ldx < N || lddx < N)
        return fail(VC_ERR_INVALID_ARG, "vc_gelu_erf_bwd: need N % 8 == 0 and 16-byte rows");
    const int64_t total = M * (N / 8);
    gelu_erf_bwd_kernel<<<(unsigned)((total + 255) / 256), 256, 0, stream>>>(dy, dy_bf16, lddy, x, ldx, M, (int)N, dx,
                                                                           lddx);
    return check_launch("vc_gelu_erf_bwd");
}

}  // extern "C"
