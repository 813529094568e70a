// Backward kernels of the TimeSformer train step (the TimeSformer folder's
// main.py trains by default, timesformer/timesformer_classifier/trainers/trainer.py:139-174).
//
//  * temporal_attn_bwd_kernel — autograd of the temporal branch's self-attention
//    (TimesformerSelfAttention over the T frames of one patch, TF5/models/timesformer/
//    modeling_timesformer.py:148-180 as called from :332-349): per (sequence, head) the T x T
//    scores are recomputed from q' (= q * scale * log2 e, the stored q|k|v layout of the forward),
//    P = softmax, dV = P^T dO, dP = dO V^T, dS = ln2 * P o (dP - rowsum(P o dP)),
//    dQ' = dS K, dK = dS^T Q'.  T <= 32 keys: VALU work, one wave per (sequence, head), the rows and
//    the T x T tiles in LDS, every lane busy in every phase.  Deterministic (no atomics).
//  * gelu_erf_fwd_kernel / gelu_erf_bwd_kernel — exact GELU (TimeSformer / Swin hidden_act
//    "gelu") as a separate op for the train step: the forward uses the same branch-free
//    erfc restatement as the fused GEMM epilogue (common.hpp gelu_erf), the backward
//    dx = dy * (Phi(x) + x phi(x)).
#include "common.hpp"

namespace vc {

constexpr float LN2 = 0.6931471805599453f;

// grid (B*P sequences, H heads), one wave; TT = the T bucket (8 / 16 / 32), T <= TT at run time.
// Rows of sequence n = b*P + p in qkv / dout / dqkv: the clip layout of the forward,
// b*(1 + P*T) + 1 + p*T + t (CLS row first, patch-major, time-minor; CLS rows untouched).
// All 64 lanes work in every phase: (1) the q', k, v, dO rows of the (sequence, head) are read
// with 16-byte loads, 8 lanes per 128-byte row, into fp32 LDS rows; (2) one lane per (query,
// key) pair forms the score s and dP = dO . v; (3) lane i < T turns its row into P and
// dS = ln2 P o (dP - delta); (4) lane d (the head dimension) forms column d of dQ', dK, dV;
// (5) those are staged back through LDS and stored as 16-byte bf16 rows.
constexpr int TB_LD = 68;  // fp32 LDS row stride: 16-byte aligned rows, banks skewed by 4

template <int TT>
__global__ void __launch_bounds__(64) temporal_attn_bwd_kernel(const uint16_t* __restrict__ qkv, int64_t ld,
                                                               const uint16_t* __restrict__ dout, int64_t lddo, int P,
                                                               int T, int H, uint16_t* __restrict__ dqkv, int64_t lddq) {
    __shared__ __attribute__((aligned(16))) float sq[TT][TB_LD], sk[TT][TB_LD], sv[TT][TB_LD], sg[TT][TB_LD];
    __shared__ __attribute__((aligned(16))) float sP[TT][TT + 4], sD[TT][TT + 4];
    const int n = blockIdx.x, h = blockIdx.y, l = threadIdx.x;
    const int D = H * 64;
    const int64_t r0 = (int64_t)(n / P) * (1 + (int64_t)P * T) + 1 + (int64_t)(n % P) * T;
    const uint16_t* qb = qkv + r0 * ld + h * 64;
    const uint16_t* db = dout + r0 * lddo + h * 64;

    for (int idx = l; idx < T * 8; idx += 64) {
        const int t = idx >> 3, c = 8 * (idx & 7);
        const uint16_t* row = qb + (int64_t)t * ld + c;
        const v8s rq = *reinterpret_cast<const v8s*>(row);
        const v8s rk = *reinterpret_cast<const v8s*>(row + D);
        const v8s rv = *reinterpret_cast<const v8s*>(row + 2 * D);
        const v8s rg = *reinterpret_cast<const v8s*>(db + (int64_t)t * lddo + c);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            sq[t][c + j] = bf2f((unsigned short)rq[j]);
            sk[t][c + j] = bf2f((unsigned short)rk[j]);
            sv[t][c + j] = bf2f((unsigned short)rv[j]);
            sg[t][c + j] = bf2f((unsigned short)rg[j]);
        }
    }
    __syncthreads();

    for (int pr = l; pr < T * T; pr += 64) {
        const int i = pr / T, u = pr - i * T;
        float s = 0.f, dp = 0.f;
#pragma unroll
        for (int d = 0; d < 64; d += 4) {
            const float4 a = *reinterpret_cast<const float4*>(&sq[i][d]);
            const float4 b = *reinterpret_cast<const float4*>(&sk[u][d]);
            const float4 g = *reinterpret_cast<const float4*>(&sg[i][d]);
            const float4 v = *reinterpret_cast<const float4*>(&sv[u][d]);
            s = __builtin_fmaf(a.x, b.x, s);
            s = __builtin_fmaf(a.y, b.y, s);
            s = __builtin_fmaf(a.z, b.z, s);
            s = __builtin_fmaf(a.w, b.w, s);
            dp = __builtin_fmaf(g.x, v.x, dp);
            dp = __builtin_fmaf(g.y, v.y, dp);
            dp = __builtin_fmaf(g.z, v.z, dp);
            dp = __builtin_fmaf(g.w, v.w, dp);
        }
        sP[i][u] = s;
        sD[i][u] = dp;
    }
    __syncthreads();

    if (l < T) {
        float m = -INFINITY;
        for (int u = 0; u < T; ++u) m = fmaxf(m, sP[l][u]);
        float sum = 0.f;
        for (int u = 0; u < T; ++u) {
            const float e = exp2f(sP[l][u] - m);
            sP[l][u] = e;
            sum += e;
        }
        const float inv = 1.0f / sum;
        float delta = 0.f;
        for (int u = 0; u < T; ++u) {
            const float p = sP[l][u] * inv;
            sP[l][u] = p;
            delta = __builtin_fmaf(p, sD[l][u], delta);
        }
        for (int u = 0; u < T; ++u) sD[l][u] = LN2 * sP[l][u] * (sD[l][u] - delta);
    }
    __syncthreads();

    // lane l = head dimension d: dQ'[i] = sum_u dS[i][u] k[u], dK[u] = sum_i dS[i][u] q'[i],
    // dV[u] = sum_i P[i][u] dO[i]
    float col[TT], dq[TT], dk[TT], dv[TT];
#pragma unroll
    for (int t = 0; t < TT; ++t) col[t] = t < T ? sk[t][l] : 0.f;
#pragma unroll
    for (int i = 0; i < TT; ++i) {
        float acc = 0.f;
#pragma unroll
        for (int u = 0; u < TT; ++u)
            if (u < T) acc = __builtin_fmaf(sD[i < T ? i : 0][u], col[u], acc);
        dq[i] = acc;
    }
#pragma unroll
    for (int t = 0; t < TT; ++t) col[t] = t < T ? sq[t][l] : 0.f;
#pragma unroll
    for (int u = 0; u < TT; ++u) {
        float acc = 0.f;
#pragma unroll
        for (int i = 0; i < TT; ++i)
            if (i < T) acc = __builtin_fmaf(sD[i][u < T ? u : 0], col[i], acc);
        dk[u] = acc;
    }
#pragma unroll
    for (int t = 0; t < TT; ++t) col[t] = t < T ? sg[t][l] : 0.f;
#pragma unroll
    for (int u = 0; u < TT; ++u) {
        float acc = 0.f;
#pragma unroll
        for (int i = 0; i < TT; ++i)
            if (i < T) acc = __builtin_fmaf(sP[i][u < T ? u : 0], col[i], acc);
        dv[u] = acc;
    }
    __syncthreads();
#pragma unroll
    for (int t = 0; t < TT; ++t)
        if (t < T) {
            sq[t][l] = dq[t];
            sk[t][l] = dk[t];
            sv[t][l] = dv[t];
        }
    __syncthreads();

    for (int idx = l; idx < T * 8; idx += 64) {
        const int t = idx >> 3, c = 8 * (idx & 7);
        uint16_t* row = dqkv + (r0 + t) * lddq + h * 64 + c;
        float (*src[3])[TB_LD] = {sq, sk, sv};
#pragma unroll
        for (int part = 0; part < 3; ++part) {
            const float4 a = *reinterpret_cast<const float4*>(&src[part][t][c]);
            const float4 b = *reinterpret_cast<const float4*>(&src[part][t][c + 4]);
            uint4 w;
            w.x = pack2bf(a.x, a.y);
            w.y = pack2bf(a.z, a.w);
            w.z = pack2bf(b.x, b.y);
            w.w = pack2bf(b.z, b.w);
            *reinterpret_cast<uint4*>(row + part * D) = w;
        }
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
    const dim3 grid((unsigned)N, (unsigned)H);
    if (T <= 8)
        temporal_attn_bwd_kernel<8><<<grid, 64, 0, stream>>>(qkv, ld, dout, lddo, (int)P, (int)T, (int)H, dqkv, lddq);
    else if (T <= 16)
        temporal_attn_bwd_kernel<16><<<grid, 64, 0, stream>>>(qkv, ld, dout, lddo, (int)P, (int)T, (int)H, dqkv, lddq);
    else
        temporal_attn_bwd_kernel<32><<<grid, 64, 0, stream>>>(qkv, ld, dout, lddo, (int)P, (int)T, (int)H, dqkv, lddq);
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
