// bf16 MFMA GEMM with fused epilogues: C[M][N] = A[M][K] . W[N][K]^T (+ epilogue).
//
// gfx950 design (cdna_hip_programming.md §5):
//   * 128x128x64 block tile, 4 waves (2x2), 64x64 per wave = 2x2 v_mfma_f32_32x32x16_bf16;
//   * A and W tiles staged HBM->LDS by global_load_lds_dwordx4 (16 B/lane, 1 KiB per
//     wave-instruction), double-buffered; XOR swizzle of the 16-B chunk applied on the
//     SOURCE address (LDS image stays lane-linear, §5.4 rule 21) and on the ds_read_b128;
//   * operands swapped (MFMA A = W rows, B = activation rows) so each lane's accumulator
//     holds 4 consecutive output columns -> 8/16-byte epilogue stores;
//   * bijective XCD remap of the block id so one XCD walks a contiguous band of row tiles
//     (A rows stay in that XCD's L2 across the N tiles).
#include "common.hpp"

namespace vc {

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int TILE_BYTES = BM * BK * 2;  // 16 KiB per operand tile

// physical 16-B chunk of logical chunk c in tile row r (128-B rows): spreads the 16 rows a
// ds_read_b128 lane group touches over all 16 slots of the 256-B bank row.
__device__ __forceinline__ int swz(int r, int c) { return c ^ ((r >> 1) & 7); }

__device__ __forceinline__ void glds16(const void* gsrc, void* lds_base) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)gsrc,
                                     (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}

// Stage a 128-row x 64-col bf16 tile (rows r0.., cols k0..) of a row-major matrix into LDS.
// Wave w fills rows [32w, 32w+32): 4 wave-instructions of 8 rows each.
__device__ __forceinline__ void stage_tile(const uint16_t* __restrict__ g, int64_t ld, int64_t r0, int64_t k0,
                                           char* lds_tile, int wave, int lane) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int row = wave * 32 + i * 8 + (lane >> 3);
        const int c = swz(row, lane & 7);
        const uint16_t* src = g + (r0 + row) * ld + k0 + c * 8;
        glds16(src, lds_tile + (wave * 32 + i * 8) * 128);
    }
}

__device__ __forceinline__ v8bf lds_frag(const char* tile, int row, int chunk) {
    const v8s v = *reinterpret_cast<const v8s*>(tile + row * 128 + swz(row, chunk) * 16);
    return __builtin_bit_cast(v8bf, v);
}

template <int EPI>
__global__ void __launch_bounds__(256, 2)
gemm_bf16_kernel(const uint16_t* __restrict__ A, int64_t lda, const uint16_t* __restrict__ W, int64_t ldw,
                 int nbm, int nbn, int K, const float* __restrict__ bias, void* __restrict__ out, int64_t ldo,
                 const float* __restrict__ aux, int64_t ldaux, int64_t G, int64_t gstride, int64_t goff) {
    __shared__ __attribute__((aligned(16))) char smem[4 * TILE_BYTES];

    // XCD-aware bijective remap (blocks b and b+8 share an XCD under round-robin dispatch)
    const int nwg = nbm * nbn;
    const int bid = blockIdx.x;
    const int xcd = bid & 7, q = nwg >> 3, rr = nwg & 7;
    const int wgid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (bid >> 3);
    const int tm = wgid / nbn, tn = wgid % nbn;
    const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 1, wn = wave & 1;
    const int r = lane & 31, h = lane >> 5;

    v16f acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

    const int nk = K / BK;
    stage_tile(A, lda, m0, 0, smem, wave, lane);
    stage_tile(W, ldw, n0, 0, smem + TILE_BYTES, wave, lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    for (int kt = 0; kt < nk; ++kt) {
        const int cur = kt & 1;
        char* At = smem + cur * 2 * TILE_BYTES;
        char* Wt = At + TILE_BYTES;
        if (kt + 1 < nk) {
            char* An = smem + (cur ^ 1) * 2 * TILE_BYTES;
            stage_tile(A, lda, m0, (int64_t)(kt + 1) * BK, An, wave, lane);
            stage_tile(W, ldw, n0, (int64_t)(kt + 1) * BK, An + TILE_BYTES, wave, lane);
        }
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
            const int ch = kk * 2 + h;
            v8bf wf0 = lds_frag(Wt, wn * 64 + r, ch);
            v8bf wf1 = lds_frag(Wt, wn * 64 + 32 + r, ch);
            v8bf af0 = lds_frag(At, wm * 64 + r, ch);
            v8bf af1 = lds_frag(At, wm * 64 + 32 + r, ch);
            acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf0, af0, acc[0][0], 0, 0, 0);
            acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf1, af0, acc[0][1], 0, 0, 0);
            acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf0, af1, acc[1][0], 0, 0, 0);
            acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf1, af1, acc[1][1], 0, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }

    // Epilogue.  acc[i][j] holds D[n][m]: lane -> m = ..+ i*32 + r; reg 4g+e -> n = ..+ j*32 + 8g + 4h + e.
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int64_t m = m0 + wm * 64 + i * 32 + r;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int64_t n = n0 + wn * 64 + j * 32 + g * 8 + h * 4;
                const float4 bb = *reinterpret_cast<const float4*>(bias + n);
                float v0 = acc[i][j][4 * g + 0] + bb.x;
                float v1 = acc[i][j][4 * g + 1] + bb.y;
                float v2 = acc[i][j][4 * g + 2] + bb.z;
                float v3 = acc[i][j][4 * g + 3] + bb.w;
                if (EPI == VC_EPI_BIAS_BF16 || EPI == VC_EPI_BIAS_GELU_TANH || EPI == VC_EPI_BIAS_GELU_ERF) {
                    if (EPI == VC_EPI_BIAS_GELU_TANH) {
                        v0 = gelu_tanh(v0); v1 = gelu_tanh(v1); v2 = gelu_tanh(v2); v3 = gelu_tanh(v3);
                    } else if (EPI == VC_EPI_BIAS_GELU_ERF) {
                        v0 = gelu_erf(v0); v1 = gelu_erf(v1); v2 = gelu_erf(v2); v3 = gelu_erf(v3);
                    }
                    uint2 p;
                    p.x = pack2bf(v0, v1);
                    p.y = pack2bf(v2, v3);
                    *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(out) + m * ldo + n) = p;
                } else if (EPI == VC_EPI_BIAS_RESID_F32) {
                    float4* o = reinterpret_cast<float4*>(reinterpret_cast<float*>(out) + m * ldo + n);
                    float4 x = *o;
                    x.x += v0; x.y += v1; x.z += v2; x.w += v3;
                    *o = x;
                } else {  // VC_EPI_EMBED_F32
                    const int64_t gi = m / G, gr = m - gi * G;
                    const float4 a = *reinterpret_cast<const float4*>(aux + gr * ldaux + n);
                    float4* o = reinterpret_cast<float4*>(reinterpret_cast<float*>(out) +
                                                          (gi * gstride + goff + gr) * ldo + n);
                    *o = make_float4(v0 + a.x, v1 + a.y, v2 + a.z, v3 + a.w);
                }
            }
        }
    }
}

}  // namespace vc

using namespace vc;

extern "C" int vc_gemm_bf16(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw, int64_t M, int64_t N,
                            int64_t K, const float* bias, int epilogue, void* out, int64_t ldo, const float* aux,
                            int64_t ldaux, int64_t G, int64_t group_stride, int64_t group_offset,
                            hipStream_t stream) {
    if (!A || !W || !bias || !out) return fail(VC_ERR_INVALID_ARG, "vc_gemm_bf16: null pointer");
    if (M <= 0 || N <= 0 || K <= 0 || M % BM || N % BN || K % BK)
        return fail(VC_ERR_INVALID_ARG, "vc_gemm_bf16: need M%128==0, N%128==0, K%64==0 (got M=" +
                                            std::to_string(M) + " N=" + std::to_string(N) + " K=" + std::to_string(K) + ")");
    if (lda % 8 || ldw % 8 || ldo % 4 || lda < K || ldw < K || ldo < N)
        return fail(VC_ERR_INVALID_ARG, "vc_gemm_bf16: bad leading dimension");
    if ((((uintptr_t)A) | ((uintptr_t)W) | ((uintptr_t)out) | ((uintptr_t)bias)) & 15)
        return fail(VC_ERR_INVALID_ARG, "vc_gemm_bf16: pointers must be 16-byte aligned");
    if (epilogue == VC_EPI_EMBED_F32 && (!aux || G <= 0 || ldaux % 4))
        return fail(VC_ERR_INVALID_ARG, "vc_gemm_bf16: EMBED epilogue needs aux, G > 0");
    const int nbm = (int)(M / BM), nbn = (int)(N / BN);
    const int64_t nwg = (int64_t)nbm * nbn;
    if (nwg > (1 << 30)) return fail(VC_ERR_INVALID_ARG, "vc_gemm_bf16: grid too large");
#define VC_LAUNCH(E)                                                                                              \
    gemm_bf16_kernel<E><<<(unsigned)nwg, 256, 0, stream>>>(A, lda, W, ldw, nbm, nbn, (int)K, bias, out, ldo, aux, \
                                                          ldaux, G, group_stride, group_offset)
    switch (epilogue) {
        case VC_EPI_BIAS_BF16: VC_LAUNCH(VC_EPI_BIAS_BF16); break;
        case VC_EPI_BIAS_GELU_TANH: VC_LAUNCH(VC_EPI_BIAS_GELU_TANH); break;
        case VC_EPI_BIAS_GELU_ERF: VC_LAUNCH(VC_EPI_BIAS_GELU_ERF); break;
        case VC_EPI_BIAS_RESID_F32: VC_LAUNCH(VC_EPI_BIAS_RESID_F32); break;
        case VC_EPI_EMBED_F32: VC_LAUNCH(VC_EPI_EMBED_F32); break;
        default: return fail(VC_ERR_INVALID_ARG, "vc_gemm_bf16: bad epilogue");
    }
#undef VC_LAUNCH
    return check_launch("vc_gemm_bf16");
}
