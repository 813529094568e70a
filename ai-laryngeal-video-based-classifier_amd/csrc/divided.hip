// TimeSformer divided space-time attention: the pieces around the shared GEMM / flash
// attention kernels (TF5/models/timesformer/modeling_timesformer.py:332-398).
//
// Token layouts (D = hidden size, P = patches per frame, T = frames):
//   clip layout   x[b][r], r = 0 (CLS) or 1 + p*T + t   (patch-major, time-minor: the model's
//                 residual stream, modeling_timesformer.py:115-143)
//   frame layout  h[(b*T + t)][j], j = 0 (CLS copy) or 1 + p  (one 1+P sequence per frame:
//                 the spatial-attention input of :355-364)
// Temporal attention runs on the clip layout (a patch's T tokens are contiguous rows);
// the spatial branch runs the joint flash kernel on the frame layout with B' = B*T,
// S' = 1 + P.  The row permutes are folded into the residual + LayerNorm kernels below,
// so no separate transpose pass touches HBM.
#include "common.hpp"

namespace vc {

// ---------------------------------------------------------------------------------
// Temporal attention: for every (clip, patch, head) a softmax over the T frames of that
// patch.  T is tiny (8), so this is VALU work: one thread per (query row, head); the T key
// / value rows of its patch are re-read from L1/L2.  Scores and softmax in fp32.
// ---------------------------------------------------------------------------------
template <int TMAX>
__global__ void __launch_bounds__(256) temporal_attn_kernel(const uint16_t* __restrict__ qkv, int64_t ld, int64_t nq,
                                                            int P, int T, int H, float c, int exp2_mode,
                                                            uint16_t* __restrict__ out, int64_t ldo) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= nq) return;
    const int hh = (int)(i % H);
    const int64_t qi = i / H;              // (b, p, t)
    const int t = (int)(qi % T);
    const int64_t bp = qi / T;             // b*P + p
    const int64_t b = bp / P, p = bp % P;
    const int64_t row0 = b * (1 + (int64_t)P * T) + 1 + p * T;  // first frame of this patch
    const int Dm = H * 64;

    float q[64];
    {
        const uint4* qp = reinterpret_cast<const uint4*>(qkv + (row0 + t) * ld + hh * 64);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint4 u = qp[j];
            const unsigned w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                q[8 * j + 2 * e] = bf2f((unsigned short)(w[e] & 0xffff)) * c;
                q[8 * j + 2 * e + 1] = bf2f((unsigned short)(w[e] >> 16)) * c;
            }
        }
    }
    float s[TMAX];
    float m = -INFINITY;
#pragma unroll
    for (int k = 0; k < TMAX; ++k) {
        if (k < T) {
            const uint4* kp = reinterpret_cast<const uint4*>(qkv + (row0 + k) * ld + Dm + hh * 64);
            float a = 0.f;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const uint4 u = kp[j];
                const unsigned w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    a += q[8 * j + 2 * e] * bf2f((unsigned short)(w[e] & 0xffff));
                    a += q[8 * j + 2 * e + 1] * bf2f((unsigned short)(w[e] >> 16));
                }
            }
            s[k] = a;
            m = fmaxf(m, a);
        }
    }
    float l = 0.f;
#pragma unroll
    for (int k = 0; k < TMAX; ++k) {
        if (k < T) {
            s[k] = exp2_mode ? exp2f(s[k] - m) : __expf(s[k] - m);
            l += s[k];
        }
    }
    const float inv = 1.0f / l;
    float o[64];
#pragma unroll
    for (int d = 0; d < 64; ++d) o[d] = 0.f;
#pragma unroll
    for (int k = 0; k < TMAX; ++k) {
        if (k < T) {
            const uint4* vp = reinterpret_cast<const uint4*>(qkv + (row0 + k) * ld + 2 * Dm + hh * 64);
            const float pk = s[k] * inv;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const uint4 u = vp[j];
                const unsigned w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    o[8 * j + 2 * e] += pk * bf2f((unsigned short)(w[e] & 0xffff));
                    o[8 * j + 2 * e + 1] += pk * bf2f((unsigned short)(w[e] >> 16));
                }
            }
        }
    }
    uint4* op = reinterpret_cast<uint4*>(out + (row0 + t) * ldo + hh * 64);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        uint4 u;
        u.x = pack2bf(o[8 * j + 0], o[8 * j + 1]);
        u.y = pack2bf(o[8 * j + 2], o[8 * j + 3]);
        u.z = pack2bf(o[8 * j + 4], o[8 * j + 5]);
        u.w = pack2bf(o[8 * j + 6], o[8 * j + 7]);
        op[j] = u;
    }
}

// ---------------------------------------------------------------------------------
// Temporal attention, one workgroup per (clip, patch): the patch's T contiguous q|k|v rows
// (T x 3*H*64 bf16, 36.9 KB at TimeSformer-B T = 8) are copied into LDS with coalesced
// 16-byte loads (whole rows, so every HBM byte is read once), then two threads per
// (frame, head) pair each own 32 of the 64 dims: partial QK^T dots joined by one lane
// exchange, fp32 softmax over the T keys, P.V for the thread's 32 dims, 64-byte stores.
// The thread-per-query kernel above reads each 128-byte head slice with eight strided
// 16-byte loads per lane and re-reads K/V rows T times through L1/L2 (1.7 TB/s at B = 16).
// ---------------------------------------------------------------------------------
template <int TMAX>
__global__ void __launch_bounds__(256) temporal_attn_lds_kernel(const uint16_t* __restrict__ qkv, int64_t ld, int P,
                                                                int T, int H, float c, int exp2_mode,
                                                                uint16_t* __restrict__ out, int64_t ldo) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int64_t bp = blockIdx.x;  // b*P + p
    const int64_t b = bp / P, p = bp % P;
    const int64_t row0 = b * (1 + (int64_t)P * T) + 1 + p * T;
    const int rw = 3 * H * 8;  // 16-byte pieces per staged row
    uint4* lds = reinterpret_cast<uint4*>(smem);
    for (int i = threadIdx.x; i < T * rw; i += blockDim.x) {
        const int t = i / rw, j = i - t * rw;
        lds[i] = reinterpret_cast<const uint4*>(qkv + (row0 + t) * ld)[j];
    }
    __syncthreads();
    const int hf = threadIdx.x & 1;
    // the block is sized to one lane pair per (frame, head) where it can be (vc_temporal_attention):
    // TimeSformer-B T x H = 96 pairs on 192 threads instead of 96 of 256 lanes busy
    for (int pair = threadIdx.x >> 1; pair < T * H; pair += blockDim.x >> 1) {  // uniform trip count per lane pair
        const int t = pair / H, hh = pair - t * H;
        const uint4* qp = lds + t * rw + hh * 8 + hf * 4;
        // QK^T on the packed bf16 pairs (v_dot2c_f32_bf16: two exact bf16 products into the f32 sum per
        // instruction, no bf16 -> f32 unpacking of q and k: round 5, 2 instead of ~5 VALU per product
        // pair); the scale c applies to the finished dot
        unsigned qw[16];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint4 u = qp[j];
            qw[4 * j] = u.x; qw[4 * j + 1] = u.y; qw[4 * j + 2] = u.z; qw[4 * j + 3] = u.w;
        }
        float s[TMAX];
        float m = -INFINITY;
#pragma unroll
        for (int k = 0; k < TMAX; ++k) {
            if (k < T) {
                const uint4* kp = lds + k * rw + (H + hh) * 8 + hf * 4;
                float a = 0.f;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const uint4 u = kp[j];
                    a = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(v2bf, qw[4 * j]), __builtin_bit_cast(v2bf, u.x), a, false);
                    a = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(v2bf, qw[4 * j + 1]), __builtin_bit_cast(v2bf, u.y), a, false);
                    a = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(v2bf, qw[4 * j + 2]), __builtin_bit_cast(v2bf, u.z), a, false);
                    a = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(v2bf, qw[4 * j + 3]), __builtin_bit_cast(v2bf, u.w), a, false);
                }
                a += __shfl_xor(a, 1, 64);
                a *= c;
                s[k] = a;
                m = fmaxf(m, a);
            }
        }
        float l = 0.f;
#pragma unroll
        for (int k = 0; k < TMAX; ++k) {
            if (k < T) {
                s[k] = exp2_mode ? exp2f(s[k] - m) : __expf(s[k] - m);
                l += s[k];
            }
        }
        const float inv = 1.0f / l;
        float o[32];
#pragma unroll
        for (int d = 0; d < 32; ++d) o[d] = 0.f;
#pragma unroll
        for (int k = 0; k < TMAX; ++k) {
            if (k < T) {
                const uint4* vp = lds + k * rw + (2 * H + hh) * 8 + hf * 4;
                const float pk = s[k] * inv;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const uint4 u = vp[j];
                    const unsigned w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        o[8 * j + 2 * e] += pk * bf2f((unsigned short)(w[e] & 0xffff));
                        o[8 * j + 2 * e + 1] += pk * bf2f((unsigned short)(w[e] >> 16));
                    }
                }
            }
        }
        uint4* op = reinterpret_cast<uint4*>(out + (row0 + t) * ldo + hh * 64 + hf * 32);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            uint4 u;
            u.x = pack2bf(o[8 * j + 0], o[8 * j + 1]);
            u.y = pack2bf(o[8 * j + 2], o[8 * j + 3]);
            u.z = pack2bf(o[8 * j + 4], o[8 * j + 5]);
            u.w = pack2bf(o[8 * j + 6], o[8 * j + 7]);
            op[j] = u;
        }
    }
}

// ---------------------------------------------------------------------------------
// Residual add + LayerNorm with the clip <-> frame permutes folded in.  One wave per
// clip-layout row; D % 4 == 0 and D <= 1024 (each lane holds up to 4 float4).
//   mode 0 (temporal -> spatial):  x[r] += y[r] (patch rows; y bf16 clip layout);
//          LN(x[r]) -> h frame layout; the CLS row is LN-ed unchanged and copied to all T frames.
//   mode 1 (spatial -> MLP):  x[r] += y[frame row of r] (y bf16 frame layout); the CLS row
//          gets the mean over frames of the T per-frame CLS rows (:383-386); LN(x[r]) -> h
//          clip layout.
// ---------------------------------------------------------------------------------
__device__ __forceinline__ float4 ld_bf16x4(const uint16_t* p) {
    const uint2 u = *reinterpret_cast<const uint2*>(p);
    return make_float4(bf2f((unsigned short)(u.x & 0xffff)), bf2f((unsigned short)(u.x >> 16)),
                       bf2f((unsigned short)(u.y & 0xffff)), bf2f((unsigned short)(u.y >> 16)));
}

// Grid: x = 4 clip-layout rows per workgroup, y = clip.  Row indices are wave-uniform (scalar
// index arithmetic: the per-lane 64-bit divisions of the first version sat in front of every
// address); NV = float4 per lane (D <= 256 NV), so D = 768 runs 3 straight-line loads per lane
// for x and y each, all issued before the first add.
template <int NV>
__global__ void __launch_bounds__(256) tsf_add_ln_kernel(float* __restrict__ x, int64_t ldx,
                                                         const uint16_t* __restrict__ y, int64_t ldy, int P,
                                                         int T, int D, const float* __restrict__ g,
                                                         const float* __restrict__ be, float eps, int mode,
                                                         uint16_t* __restrict__ h, int64_t ldh) {
    const int lane = threadIdx.x & 63;
    const int S = 1 + P * T;
    const int r = (int)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    if (r >= S) return;
    const int64_t b = blockIdx.y;
    const int64_t row = b * S + r;
    const int p = r > 0 ? (r - 1) / T : 0, t = r > 0 ? (r - 1) - p * T : 0;
    const int64_t frow = (b * T + t) * (1 + P) + 1 + p;  // frame-layout row of a patch token
    const float* xr = x + row * ldx;
    const uint16_t* yr = y + (mode == 0 ? row : frow) * ldy;
    float4 v[NV];
    uint2 yv[NV];
    float s = 0.f;
    // every load of the row (x and, for patch rows, y) is issued before the first add / store
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        const int n = (i * 64 + lane) * 4;
        v[i] = make_float4(0.f, 0.f, 0.f, 0.f);
        yv[i] = make_uint2(0u, 0u);
        if (n < D) {
            v[i] = *reinterpret_cast<const float4*>(xr + n);
            if (r > 0) yv[i] = *reinterpret_cast<const uint2*>(yr + n);
        }
    }
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        const int n = (i * 64 + lane) * 4;
        if (n < D) {
            float4 a = v[i];
            if (r > 0) {
                const uint2 u = yv[i];
                a.x += bf2f((unsigned short)(u.x & 0xffff)); a.y += bf2f((unsigned short)(u.x >> 16));
                a.z += bf2f((unsigned short)(u.y & 0xffff)); a.w += bf2f((unsigned short)(u.y >> 16));
            } else if (mode == 1) {
                float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
                for (int tt = 0; tt < T; ++tt) {
                    const float4 d = ld_bf16x4(y + ((b * T + tt) * (1 + P)) * ldy + n);
                    acc.x += d.x; acc.y += d.y; acc.z += d.z; acc.w += d.w;
                }
                const float it = 1.0f / (float)T;
                a.x += acc.x * it; a.y += acc.y * it; a.z += acc.z * it; a.w += acc.w * it;
            }
            if (r > 0 || mode == 1) *reinterpret_cast<float4*>(x + row * ldx + n) = a;
            v[i] = a;
            s += (a.x + a.y) + (a.z + a.w);
        }
    }
    const float mean = wave_sum(s) / (float)D;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        if ((i * 64 + lane) * 4 < D) {
            const float a = v[i].x - mean, bb = v[i].y - mean, c = v[i].z - mean, d = v[i].w - mean;
            q += (a * a + bb * bb) + (c * c + d * d);
        }
    }
    const float rstd = rsqrtf(wave_sum(q) / (float)D + eps);
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        const int n = (i * 64 + lane) * 4;
        if (n < D) {
            const float4 gg = *reinterpret_cast<const float4*>(g + n), bb = *reinterpret_cast<const float4*>(be + n);
            uint2 o;
            o.x = pack2bf((v[i].x - mean) * rstd * gg.x + bb.x, (v[i].y - mean) * rstd * gg.y + bb.y);
            o.y = pack2bf((v[i].z - mean) * rstd * gg.z + bb.z, (v[i].w - mean) * rstd * gg.w + bb.w);
            if (mode == 1) {
                *reinterpret_cast<uint2*>(h + row * ldh + n) = o;
            } else if (r > 0) {
                *reinterpret_cast<uint2*>(h + frow * ldh + n) = o;
            } else {
                for (int tt = 0; tt < T; ++tt) *reinterpret_cast<uint2*>(h + ((b * T + tt) * (1 + P)) * ldh + n) = o;
            }
        }
    }
}

}  // namespace vc

using namespace vc;

extern "C" {

int vc_temporal_attention(const uint16_t* qkv, int64_t ld, int64_t B, int64_t P, int64_t T, int64_t H,
                          int64_t head_dim, float scale, int q_prescaled, uint16_t* out, int64_t ldo,
                          hipStream_t stream) {
    if (!qkv || !out) return fail(VC_ERR_INVALID_ARG, "vc_temporal_attention: null pointer");
    if (head_dim != 64) return fail(VC_ERR_UNSUPPORTED, "vc_temporal_attention: head_dim must be 64");
    if (B <= 0 || P <= 0 || T <= 0 || H <= 0 || ld < 3 * H * 64 || ldo < H * 64 || ld % 8 || ldo % 8)
        return fail(VC_ERR_INVALID_ARG, "vc_temporal_attention: bad shape / leading dimension");
    if ((((uintptr_t)qkv) | ((uintptr_t)out)) & 15)
        return fail(VC_ERR_INVALID_ARG, "vc_temporal_attention: pointers must be 16-byte aligned");
    const int64_t nq = B * P * T * H;
    const unsigned nb = (unsigned)((nq + 255) / 256);
    // q_prescaled: q already carries scale*log2(e) (folded into the projection) -> exp2
    const float c = q_prescaled ? 1.0f : scale;
    const int64_t lds = T * 3 * H * 64 * 2;  // one patch's q|k|v rows
    if (T <= 16 && lds <= 64 * 1024 && B * P < (1LL << 31)) {
        const unsigned nwg = (unsigned)(B * P);
        // one lane pair per (frame, head), whole waves, at most 256 threads (TimeSformer-B: 192)
        const int64_t want = (2 * T * H + 63) / 64 * 64;
        const unsigned nt = (unsigned)(want < 256 ? want : 256);
        if (T <= 8)
            temporal_attn_lds_kernel<8><<<nwg, nt, lds, stream>>>(qkv, ld, (int)P, (int)T, (int)H, c, q_prescaled, out, ldo);
        else
            temporal_attn_lds_kernel<16><<<nwg, nt, lds, stream>>>(qkv, ld, (int)P, (int)T, (int)H, c, q_prescaled, out, ldo);
    } else if (T <= 8)
        temporal_attn_kernel<8><<<nb, 256, 0, stream>>>(qkv, ld, nq, (int)P, (int)T, (int)H, c, q_prescaled, out, ldo);
    else if (T <= 16)
        temporal_attn_kernel<16><<<nb, 256, 0, stream>>>(qkv, ld, nq, (int)P, (int)T, (int)H, c, q_prescaled, out, ldo);
    else if (T <= 32)
        temporal_attn_kernel<32><<<nb, 256, 0, stream>>>(qkv, ld, nq, (int)P, (int)T, (int)H, c, q_prescaled, out, ldo);
    else
        return fail(VC_ERR_UNSUPPORTED, "vc_temporal_attention: T > 32");
    return check_launch("vc_temporal_attention");
}

int vc_divided_add_layernorm(float* x, int64_t ldx, const uint16_t* y, int64_t ldy, int64_t B, int64_t P, int64_t T,
                             int64_t D, const float* gamma, const float* beta, float eps, int mode, uint16_t* h,
                             int64_t ldh, hipStream_t stream) {
    if (!x || !y || !gamma || !beta || !h) return fail(VC_ERR_INVALID_ARG, "vc_divided_add_layernorm: null pointer");
    if (D % 4 || D > 1024 || ldx % 4 || ldy % 4 || ldh % 4 || (mode != 0 && mode != 1) || B <= 0 || P <= 0 || T <= 0)
        return fail(VC_ERR_INVALID_ARG, "vc_divided_add_layernorm: bad shape / mode");
    const int64_t S = 1 + P * T;
    if (S >= (1LL << 30) || B > 65535) return fail(VC_ERR_INVALID_ARG, "vc_divided_add_layernorm: too many rows");
    const dim3 grid((unsigned)((S + 3) / 4), (unsigned)B);
    const int nv = (int)((D + 255) / 256);
#define VC_TSF_LN(NV_)                                                                                           \
    tsf_add_ln_kernel<NV_><<<grid, 256, 0, stream>>>(x, ldx, y, ldy, (int)P, (int)T, (int)D, gamma, beta, eps, mode, h, \
                                                     ldh)
    if (nv == 1) VC_TSF_LN(1);
    else if (nv == 2) VC_TSF_LN(2);
    else if (nv == 3) VC_TSF_LN(3);
    else VC_TSF_LN(4);
#undef VC_TSF_LN
    return check_launch("vc_divided_add_layernorm");
}

}  // extern "C"
