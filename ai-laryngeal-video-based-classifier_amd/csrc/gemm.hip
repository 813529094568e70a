// bf16 MFMA GEMM with fused epilogues: C[M][N] = A[M][K] . W[N][K]^T (+ epilogue).
//
// gfx950 design (cdna_hip_programming.md §5):
//   * 512-thread workgroups (8 waves), block tile BM x BN x 64, wave tile (BM/WM) x (BN/WN)
//     built from v_mfma_f32_32x32x16_bf16;
//   * A and W tiles staged HBM->LDS by global_load_lds_dwordx4 (16 B/lane, 1 KiB per
//     wave-instruction) into a 3-slot LDS ring: tile t+2 is issued while tile t is
//     computed, and the end-of-tile wait is a COUNTED `s_waitcnt vmcnt(N)` that retires
//     only tile t+1, followed by a raw s_barrier (no __syncthreads: it would drain the
//     ring with vmcnt(0)) — §5 "Pipelining across barriers";
//   * the 16-B chunk XOR swizzle is applied on the SOURCE address (lane-linear LDS image,
//     §5.4 rule 21) and on every ds_read_b128, so each 16-lane read group hits 16
//     distinct bank slots;
//   * fragment registers double-buffered across the four 16-deep k-steps of a tile so
//     LDS latency overlaps the MFMAs of the previous k-step;
//   * operands swapped (MFMA A = W rows, B = activation rows) so each lane's accumulator
//     holds 4 consecutive output columns -> 8/16-byte epilogue stores;
//   * bijective XCD remap of the block id: one XCD walks a contiguous band of row tiles,
//     keeping its A panel in that XCD's L2 across the N tiles (§5.5 T1).
#include "common.hpp"

#include <cmath>
#include <type_traits>

namespace vc {

constexpr int GBK = 64;

// physical 16-B chunk of logical chunk c in LDS row r (128-B rows): the 16 rows one
// ds_read_b128 lane group touches land on all 16 slots of the 256-B bank row.
__device__ __forceinline__ int swz(int r, int c) { return c ^ ((r >> 1) & 7); }

// LDS-DMA of 16 B per lane (1 KiB per wave-instruction) to LDS byte address `lds_addr`
// (wave-uniform, M0).  Issued from inline asm so hipcc's wait-count scoreboard does not
// see it: with a compiler-visible global_load_lds in the loop hipcc falls back to
// lgkmcnt(0) before every MFMA; here its ds_read waits stay counted, and the DMA is
// retired by our own vmcnt(N) (cdna_hip_programming.md §5.7 item 1, glds16_asm recipe).
// m0 is declared clobbered rather than saved and restored around each piece (2 SALU fewer;
// hipcc re-materialises m0 itself wherever it needs it).
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_addr) {
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
                 :
                 : "v"(gsrc), "s"(lds_addr)
                 : "memory", "m0");
}

// the saddr form: wave-uniform 64-bit base in SGPRs + a 32-bit per-lane byte offset (one VGPR per
// source stream instead of a 64-bit address pair)
__device__ __forceinline__ void glds16s(const void* sbase, uint32_t voff, uint32_t lds_addr) {
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1"
                 :
                 : "v"(voff), "s"(sbase), "s"(lds_addr)
                 : "memory", "m0");
}

__device__ __forceinline__ uint32_t lds_addr_of(const void* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}

__device__ __forceinline__ v8s lds_frag(const char* tile, int row, int chunk) {
    return *reinterpret_cast<const v8s*>(tile + row * 128 + swz(row, chunk) * 16);
}

// s_waitcnt through the builtin (not inline asm) so the compiler's own wait-count
// scoreboard sees it: simm16 = vmcnt[3:0] | expcnt[6:4] | lgkmcnt[11:8] | vmcnt_hi[15:14].
template <int NW>
__device__ __forceinline__ void wait_vm() {
    static_assert(NW >= 0 && NW < 64, "vmcnt immediate");
    __builtin_amdgcn_s_waitcnt((NW & 15) | ((NW >> 4) << 14) | 0x0F70);  // vmcnt(NW) only
}

// wait until at most min(n, MAXT) tiles of LPT loads each are outstanding (n uniform; n < 0 -> 0)
template <int LPT, int MAXT>
__device__ __forceinline__ void wait_tiles(int n) {
    if constexpr (MAXT > 0) {
        if (n >= MAXT) {
            wait_vm<LPT * MAXT>();
            return;
        }
        wait_tiles<LPT, MAXT - 1>(n);
    } else {
        wait_vm<0>();
    }
}

__device__ __forceinline__ void block_sync_lds() {
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");  // compiler fence: LDS was written by DMA behind its back
    __builtin_amdgcn_sched_barrier(0);
}

// One lane's 4 consecutive output columns n..n+3 of row m (bias already added): the epilogue
// body shared by the 32x32 and 16x16 block layouts.
template <int EPI, int ET>
__device__ __forceinline__ void store4(int64_t m, int64_t n, float v0, float v1, float v2, float v3,
                                       void* __restrict__ out, int64_t ldo, const float* __restrict__ aux,
                                       int64_t ldaux, int64_t G, int64_t gstride, int64_t goff) {
    if (EPI == VC_EPI_BIAS_GELU_TANH_SAVE || EPI == VC_EPI_DGELU_TANH) {
        uint2* ap = reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(const_cast<float*>(aux)) + m * ldaux + n);
        if (EPI == VC_EPI_BIAS_GELU_TANH_SAVE) {
            // keep the bf16 pre-activation for the backward's gelu'
            uint2 pre;
            pre.x = pack2bf(v0, v1);
            pre.y = pack2bf(v2, v3);
            *ap = pre;
            v0 = gelu_tanh(v0); v1 = gelu_tanh(v1); v2 = gelu_tanh(v2); v3 = gelu_tanh(v3);
        } else {
            const uint2 pre = *ap;
            v0 *= dgelu_tanh(bf2f((unsigned short)(pre.x & 0xffff)));
            v1 *= dgelu_tanh(bf2f((unsigned short)(pre.x >> 16)));
            v2 *= dgelu_tanh(bf2f((unsigned short)(pre.y & 0xffff)));
            v3 *= dgelu_tanh(bf2f((unsigned short)(pre.y >> 16)));
        }
        uint2 p;
        p.x = pack2bf(v0, v1);
        p.y = pack2bf(v2, v3);
        *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(out) + m * ldo + n) = p;
    } else if (EPI == VC_EPI_BIAS_ADD_F32) {
        const float4 a = *reinterpret_cast<const float4*>(aux + m * ldaux + n);
        *reinterpret_cast<float4*>(reinterpret_cast<float*>(out) + m * ldo + n) =
            make_float4(a.x + v0, a.y + v1, a.z + v2, a.w + v3);
    } else if (EPI == VC_EPI_BIAS_BF16 || EPI == VC_EPI_BIAS_GELU_TANH || EPI == VC_EPI_BIAS_GELU_ERF ||
        EPI == VC_EPI_BIAS_RELU_BF16 || EPI == VC_EPI_BIAS_RESID_RELU_BF16) {
        if (EPI == VC_EPI_BIAS_GELU_TANH) {
            v0 = gelu_tanh(v0); v1 = gelu_tanh(v1); v2 = gelu_tanh(v2); v3 = gelu_tanh(v3);
        } else if (EPI == VC_EPI_BIAS_GELU_ERF) {
            v0 = gelu_erf(v0); v1 = gelu_erf(v1); v2 = gelu_erf(v2); v3 = gelu_erf(v3);
        } else if (EPI == VC_EPI_BIAS_RELU_BF16 || EPI == VC_EPI_BIAS_RESID_RELU_BF16) {
            if (EPI == VC_EPI_BIAS_RESID_RELU_BF16) {
                const uint2 rr = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(aux) + m * ldaux + n);
                v0 += bf2f((unsigned short)(rr.x & 0xffff)); v1 += bf2f((unsigned short)(rr.x >> 16));
                v2 += bf2f((unsigned short)(rr.y & 0xffff)); v3 += bf2f((unsigned short)(rr.y >> 16));
            }
            v0 = fmaxf(v0, 0.f); v1 = fmaxf(v1, 0.f); v2 = fmaxf(v2, 0.f); v3 = fmaxf(v3, 0.f);
        }
        uint2 p;
        p.x = pack2<ET>(v0, v1);
        p.y = pack2<ET>(v2, v3);
        *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(out) + m * ldo + n) = p;
    } else if (EPI == VC_EPI_BIAS_RESID_F32) {
        float4* o = reinterpret_cast<float4*>(reinterpret_cast<float*>(out) + m * ldo + n);
        float4 x = *o;
        x.x += v0; x.y += v1; x.z += v2; x.w += v3;
        *o = x;
    } else if (EPI == VC_EPI_BIAS_F32) {
        *reinterpret_cast<float4*>(reinterpret_cast<float*>(out) + m * ldo + n) = make_float4(v0, v1, v2, v3);
    } else {  // VC_EPI_EMBED_F32
        const int64_t gi = m / G, gr = m - gi * G;
        const float4 a = *reinterpret_cast<const float4*>(aux + gr * ldaux + n);
        float4* o = reinterpret_cast<float4*>(reinterpret_cast<float*>(out) +
                                              (gi * gstride + goff + gr) * ldo + n);
        *o = make_float4(v0 + a.x, v1 + a.y, v2 + a.z, v3 + a.w);
    }
}

// Epilogue shared by the GEMM kernels.  acc[i][j] holds D[n][m] of a 32x32 block:
// lane -> m = mb + 32i + r; reg 4g+e -> n = nb + 32j + 8g + 4h + e (4 consecutive columns).
// ET: 16-bit type of the plain 16-bit outputs (epilogues 0-2; the others are bf16-only)
template <int EPI, int MI, int NI, int ET = VC_ELEM_BF16>
__device__ __forceinline__ void store_tile(const v16f (&acc)[MI][NI], int64_t mb, int64_t nb, int r, int h,
                                           const float* __restrict__ bias, void* __restrict__ out, int64_t ldo,
                                           const float* __restrict__ aux, int64_t ldaux, int64_t G, int64_t gstride,
                                           int64_t goff) {
    // plain bf16 outputs on 16-B aligned rows: lane-pair swap -> one 16-B store per two column
    // groups (cdna_hip_programming.md T21, as in the persistent kernel's epilogue) instead of
    // four 8-B stores per 32 columns
    constexpr bool PLAIN_BF16 = EPI == VC_EPI_BIAS_BF16 || EPI == VC_EPI_BIAS_GELU_TANH ||
                                EPI == VC_EPI_BIAS_GELU_ERF || EPI == VC_EPI_BIAS_RELU_BF16;
    if constexpr (PLAIN_BF16) {
        if ((ldo & 7) == 0 && ((uintptr_t)out & 15) == 0) {
#pragma unroll
            for (int i = 0; i < MI; ++i) {
                uint16_t* orow = reinterpret_cast<uint16_t*>(out) + (mb + i * 32 + r) * ldo;
#pragma unroll
                for (int j = 0; j < NI; ++j) {
                    unsigned pk[4][2];
#pragma unroll
                    for (int g = 0; g < 4; ++g) {
                        const float4 bb = *reinterpret_cast<const float4*>(bias + nb + j * 32 + g * 8 + h * 4);
                        float v0 = acc[i][j][4 * g + 0] + bb.x, v1 = acc[i][j][4 * g + 1] + bb.y;
                        float v2 = acc[i][j][4 * g + 2] + bb.z, v3 = acc[i][j][4 * g + 3] + bb.w;
                        if (EPI == VC_EPI_BIAS_GELU_TANH) {
                            v0 = gelu_tanh(v0); v1 = gelu_tanh(v1); v2 = gelu_tanh(v2); v3 = gelu_tanh(v3);
                        } else if (EPI == VC_EPI_BIAS_GELU_ERF) {
                            v0 = gelu_erf(v0); v1 = gelu_erf(v1); v2 = gelu_erf(v2); v3 = gelu_erf(v3);
                        } else if (EPI == VC_EPI_BIAS_RELU_BF16) {
                            v0 = fmaxf(v0, 0.f); v1 = fmaxf(v1, 0.f); v2 = fmaxf(v2, 0.f); v3 = fmaxf(v3, 0.f);
                        }
                        pk[g][0] = pack2<ET>(v0, v1);
                        pk[g][1] = pack2<ET>(v2, v3);
                    }
#pragma unroll
                    for (int g = 0; g < 4; g += 2) {
                        // lower half: cols 8g..8g+7 (own g | upper's g); upper half: 8g+8..8g+15
                        auto s0 = __builtin_amdgcn_permlane32_swap(pk[g][0], pk[g + 1][0], false, false);
                        auto s1 = __builtin_amdgcn_permlane32_swap(pk[g][1], pk[g + 1][1], false, false);
                        uint4 v;
                        v.x = s0[0]; v.y = s1[0]; v.z = s0[1]; v.w = s1[1];
                        *reinterpret_cast<uint4*>(orow + nb + j * 32 + g * 8 + h * 8) = v;
                    }
                }
            }
            return;
        }
    }
#pragma unroll
    for (int i = 0; i < MI; ++i) {
        const int64_t m = mb + i * 32 + r;
#pragma unroll
        for (int j = 0; j < NI; ++j) {
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int64_t n = nb + j * 32 + g * 8 + h * 4;
                const float4 bb = *reinterpret_cast<const float4*>(bias + n);
                store4<EPI, ET>(m, n, acc[i][j][4 * g + 0] + bb.x, acc[i][j][4 * g + 1] + bb.y, acc[i][j][4 * g + 2] + bb.z,
                                acc[i][j][4 * g + 3] + bb.w, out, ldo, aux, ldaux, G, gstride, goff);
            }
        }
    }
}

// Epilogue of the 16x16x32 kernels: acc[i][j] holds D[n][m] of a 16x16 block, lane (c16, q) ->
// m = mb + 16i + c16, reg e -> n = nb + 16j + 4q + e.  Plain 16-bit outputs pair blocks j, j+1
// with v_permlane16_swap so each lane stores 8 consecutive columns (16 B).
// bias[nb + 16j + 4q .. + 3] for the NI column blocks of a lane: loaded at kernel entry, so the epilogue
// does not open with NI dependent global loads (a ping-pong tile's epilogue took 3.3 us to issue with
// them, 1/6 of its K = 768 main loop: tools/gemm_stamps.py, round 5)
template <int NI>
__device__ __forceinline__ void load_bias16(const float* __restrict__ bias, int64_t nb, int q, float4 (&bb)[NI]) {
#pragma unroll
    for (int j = 0; j < NI; ++j) bb[j] = *reinterpret_cast<const float4*>(bias + nb + j * 16 + 4 * q);
}

template <int EPI, int MI, int NI, int ET = VC_ELEM_BF16>
__device__ __forceinline__ void store_tile16(const v4f (&acc)[MI][NI], int64_t mb, int64_t nb, int c16, int q,
                                             const float4 (&bq)[NI], void* __restrict__ out, int64_t ldo,
                                             const float* __restrict__ aux, int64_t ldaux, int64_t G, int64_t gstride,
                                             int64_t goff) {
    constexpr bool PLAIN16 = EPI == VC_EPI_BIAS_BF16 || EPI == VC_EPI_BIAS_GELU_TANH || EPI == VC_EPI_BIAS_GELU_ERF ||
                             EPI == VC_EPI_BIAS_RELU_BF16;
    if constexpr (PLAIN16 && NI % 2 == 0) {
        if ((ldo & 7) == 0 && ((uintptr_t)out & 15) == 0) {
#pragma unroll
            for (int i = 0; i < MI; ++i) {
                uint16_t* orow = reinterpret_cast<uint16_t*>(out) + (mb + i * 16 + c16) * ldo;
#pragma unroll
                for (int jp = 0; jp < NI / 2; ++jp) {
                    unsigned pk[2][2];
#pragma unroll
                    for (int s = 0; s < 2; ++s) {
                        const float4 bb = bq[2 * jp + s];
                        float v0 = acc[i][2 * jp + s][0] + bb.x, v1 = acc[i][2 * jp + s][1] + bb.y;
                        float v2 = acc[i][2 * jp + s][2] + bb.z, v3 = acc[i][2 * jp + s][3] + bb.w;
                        if (EPI == VC_EPI_BIAS_GELU_TANH) {
                            v0 = gelu_tanh(v0); v1 = gelu_tanh(v1); v2 = gelu_tanh(v2); v3 = gelu_tanh(v3);
                        } else if (EPI == VC_EPI_BIAS_GELU_ERF) {
                            v0 = gelu_erf(v0); v1 = gelu_erf(v1); v2 = gelu_erf(v2); v3 = gelu_erf(v3);
                        } else if (EPI == VC_EPI_BIAS_RELU_BF16) {
                            v0 = fmaxf(v0, 0.f); v1 = fmaxf(v1, 0.f); v2 = fmaxf(v2, 0.f); v3 = fmaxf(v3, 0.f);
                        }
                        pk[s][0] = pack2<ET>(v0, v1);
                        pk[s][1] = pack2<ET>(v2, v3);
                    }
                    // even q: block 2jp, columns 4q .. 4q+7; odd q: block 2jp+1, columns 4(q-1) .. 4(q-1)+7
                    auto s0 = __builtin_amdgcn_permlane16_swap(pk[0][0], pk[1][0], false, false);
                    auto s1 = __builtin_amdgcn_permlane16_swap(pk[0][1], pk[1][1], false, false);
                    uint4 v;
                    v.x = s0[0]; v.y = s1[0]; v.z = s0[1]; v.w = s1[1];
                    *reinterpret_cast<uint4*>(orow + nb + (2 * jp + (q & 1)) * 16 + 4 * (q & 2)) = v;
                }
            }
            return;
        }
    }
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j) {
            const int64_t m = mb + i * 16 + c16, n = nb + j * 16 + 4 * q;
            const float4 bb = bq[j];
            store4<EPI, ET>(m, n, acc[i][j][0] + bb.x, acc[i][j][1] + bb.y, acc[i][j][2] + bb.z, acc[i][j][3] + bb.w,
                            out, ldo, aux, ldaux, G, gstride, goff);
        }
}

// ST: LDS ring depth in tiles (prefetch distance ST - 1).  ST = 2 at 128x128 needs 64 KiB of
// LDS, so two workgroups share a CU and one's epilogue overlaps the other's main loop.
// f32 residual epilogue: this wave's residual elements are loaded into registers before the K
// loop, so their latency overlaps the main loop instead of opening the epilogue (+20 VGPRs at
// 128x128; +0.4 % on the ViViT-B forward in an interleaved A/B, round 1).
// (A static s_setprio for one of two co-resident workgroups measured slower here, unlike in
// the attention kernel: o_proj 67.0 vs 64.4 us, fc2 152.6 vs 151.0; round 1.)
// The wave tile is built from 16x16 blocks of v_mfma_f32_16x16x32, two 32-deep k-steps per
// 64-deep tile (the shape sustains more FLOP/s than 32x32x16 under the power-limited clock; see
// the persistent kernel below): ViViT-B B=8 o_proj 552 vs 516 TF/s, fc2 864 vs 784 at 128x128.
template <int BM, int BN, int WM, int WN, int EPI, int ST = 3, int ET = VC_ELEM_BF16>
__global__ void __launch_bounds__(512, ST == 2 ? 2 : 1)
gemm_bf16_kernel(const uint16_t* __restrict__ A, int64_t lda, const uint16_t* __restrict__ W, int64_t ldw,
                 int nbm, int nbn, int K, const float* __restrict__ bias, void* __restrict__ out, int64_t ldo,
                 const float* __restrict__ aux, int64_t ldaux, int64_t G, int64_t gstride, int64_t goff) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    static_assert(ST >= 2 && ST <= 8, "ring depth");
    constexpr int SLOT = (BM + BN) * 128;       // bytes per ring slot (A then W, 128-B rows)
    constexpr int TM = BM / WM, TN = BN / WN;   // wave tile
    constexpr int MI = TM / 16, NI = TN / 16;
    constexpr int AL = BM / 64, BL = BN / 64;   // glds per thread per tile (8 rows per wave-instr, 8 waves)
    constexpr int LPT = AL + BL;
    static_assert(WM * WN == 8 && TM % 32 == 0 && TN % 32 == 0, "8 waves, 32-multiple wave tiles");

    const int nwg = nbm * nbn;
    const int bid = blockIdx.x;
    const int xcd = bid & 7, xq = nwg >> 3, rr = nwg & 7;
    const int wgid = (xcd < rr ? xcd * (xq + 1) : rr * (xq + 1) + (xcd - rr) * xq) + (bid >> 3);
    const int tm = wgid / nbn, tn = wgid % nbn;
    const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / WN, wn = wave % WN;
    const int c16 = lane & 15, q = lane >> 4;
    float4 bq[NI];  // this lane's bias columns, loaded now (their latency hides under the main loop)
    load_bias16<NI>(bias, n0 + wn * TN, q, bq);

    // per-lane staging sources (k offset added per tile)
    const uint16_t* asrc[AL];
    const uint16_t* bsrc[BL];
#pragma unroll
    for (int i = 0; i < AL; ++i) {
        const int row = wave * (BM / 8) + i * 8 + (lane >> 3);
        asrc[i] = A + (m0 + row) * lda + swz(row, lane & 7) * 8;
    }
#pragma unroll
    for (int i = 0; i < BL; ++i) {
        const int row = wave * (BN / 8) + i * 8 + (lane >> 3);
        bsrc[i] = W + (n0 + row) * ldw + swz(row, lane & 7) * 8;
    }
    const uint32_t lds0 = __builtin_amdgcn_readfirstlane(lds_addr_of(smem));
    auto stage = [&](int t, int slot) {
        const uint32_t s = lds0 + slot * SLOT;
        const int64_t k0 = (int64_t)t * GBK;
#pragma unroll
        for (int i = 0; i < AL; ++i)
            glds16(asrc[i] + k0, __builtin_amdgcn_readfirstlane(s + (wave * (BM / 8) + i * 8) * 128));
#pragma unroll
        for (int i = 0; i < BL; ++i)
            glds16(bsrc[i] + k0, __builtin_amdgcn_readfirstlane(s + BM * 128 + (wave * (BN / 8) + i * 8) * 128));
    };

    v4f acc[MI][NI];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

    const int nk = K / GBK;
    stage(0, 0);
    // lane (c16, q) holds output row m0 + wm*TM + 16i + c16, columns n0 + wn*TN + 16j + 4q .. +3
    constexpr bool RPRE = EPI == VC_EPI_BIAS_RESID_F32;
    float4 xres[RPRE ? MI : 1][RPRE ? NI : 1];
    if constexpr (RPRE) {
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int j = 0; j < NI; ++j)
                xres[i][j] = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(out) +
                                                              (m0 + wm * TM + i * 16 + c16) * ldo + n0 + wn * TN +
                                                              j * 16 + 4 * q);
    }
    // the bf16 residual of the ResNet3D conv_c epilogue likewise, when K is one k-tile (res2's
    // K = 64: otherwise its fetch in the epilogue is a second serialized round trip per tile;
    // 138.4 vs 143.1 us at 401408 x 256).  At K >= 128 the early loads delay the operand DMAs
    // behind them and cost more than they hide (res3 K = 128 67.6 vs 58.4 us, res4 K = 256 43.4 vs
    // 38.9; cfg 14 = this kernel with the prefetch off, round 4).  G < 0: the cfg-14 ablation.
    constexpr bool APRE = EPI == VC_EPI_BIAS_RESID_RELU_BF16;
    const bool apre = APRE && G >= 0 && K <= GBK;
    uint2 xaux[APRE ? MI : 1][APRE ? NI : 1];
    if constexpr (APRE) {
        if (apre) {
#pragma unroll
            for (int i = 0; i < MI; ++i)
#pragma unroll
                for (int j = 0; j < NI; ++j)
                    xaux[i][j] = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(aux) +
                                                                 (m0 + wm * TM + i * 16 + c16) * ldaux + n0 + wn * TN +
                                                                 j * 16 + 4 * q);
        }
    }
    // tiles 1 .. ST-2 in flight too; then retire tile 0 (the tiles issued after it may stay in flight)
#pragma unroll
    for (int u = 1; u < ST - 1; ++u)
        if (u < nk) stage(u, u);
    wait_tiles<LPT, ST - 2>(nk - 1);
    block_sync_lds();

    // one k-tile; FAST (compile time) when t <= nk - ST: tile t+ST-1 is staged and the retire count
    // is the steady-state one, so the steady loop carries no runtime tests (round 6: their scalar
    // compares and branches cost the ping-pong kernel 4 %)
    auto ktile = [&](auto FAST, int t) __attribute__((always_inline)) {
        const int slot = t % ST;
        if constexpr (decltype(FAST)::value) stage(t + ST - 1, (t + ST - 1) % ST);
        else if (t + ST - 1 < nk) stage(t + ST - 1, (t + ST - 1) % ST);
        const char* At = smem + slot * SLOT;
        const char* Wt = At + BM * 128;

        v8s af[2][MI], wf[2][NI];
        {
            // two 32-deep k-steps: lane (c16, q) reads row 16i + c16, 16-B chunk 4kk + q (the 16
            // rows of a ds_read_b128 lane group land on 16 distinct bank slots under swz)
#pragma unroll
            for (int i = 0; i < MI; ++i) af[0][i] = lds_frag(At, wm * TM + i * 16 + c16, q);
#pragma unroll
            for (int j = 0; j < NI; ++j) wf[0][j] = lds_frag(Wt, wn * TN + j * 16 + c16, q);
#pragma unroll
            for (int i = 0; i < MI; ++i) af[1][i] = lds_frag(At, wm * TM + i * 16 + c16, 4 + q);
#pragma unroll
            for (int j = 0; j < NI; ++j) wf[1][j] = lds_frag(Wt, wn * TN + j * 16 + c16, 4 + q);
#pragma unroll
            for (int kk = 0; kk < 2; ++kk)
#pragma unroll
                for (int i = 0; i < MI; ++i)
#pragma unroll
                    for (int j = 0; j < NI; ++j)
                        acc[i][j] = mfma16x32<ET>(wf[kk][j], af[kk][i], acc[i][j]);
        }
        // retire tile t+1 (tiles t+2 .. t+ST-1 may stay in flight), then all waves pass the barrier
        if constexpr (decltype(FAST)::value) wait_vm<LPT * (ST - 2)>();
        else wait_tiles<LPT, ST - 2>(nk - 2 - t);
        block_sync_lds();
    };
    // the 64-row tiles (cfgs 7 / 21: K = 96 .. 384, two to six k-tiles) keep the one tested loop: split
    // they ran 1.8-3 % slower (round 6, tools/r06_i.sh)
    if constexpr (BM >= 128) {
        int t = 0;
        for (; t <= nk - ST; ++t) ktile(std::true_type{}, t);
        for (; t < nk; ++t) ktile(std::false_type{}, t);
    } else {
        for (int t = 0; t < nk; ++t) {
            const int slot = t % ST;
            if (t + ST - 1 < nk) stage(t + ST - 1, (t + ST - 1) % ST);
            const char* At = smem + slot * SLOT;
            const char* Wt = At + BM * 128;

            v8s af[2][MI], wf[2][NI];
            {
                // two 32-deep k-steps: lane (c16, q) reads row 16i + c16, 16-B chunk 4kk + q (the 16
                // rows of a ds_read_b128 lane group land on 16 distinct bank slots under swz)
#pragma unroll
                for (int i = 0; i < MI; ++i) af[0][i] = lds_frag(At, wm * TM + i * 16 + c16, q);
#pragma unroll
                for (int j = 0; j < NI; ++j) wf[0][j] = lds_frag(Wt, wn * TN + j * 16 + c16, q);
#pragma unroll
                for (int i = 0; i < MI; ++i) af[1][i] = lds_frag(At, wm * TM + i * 16 + c16, 4 + q);
#pragma unroll
                for (int j = 0; j < NI; ++j) wf[1][j] = lds_frag(Wt, wn * TN + j * 16 + c16, 4 + q);
#pragma unroll
                for (int kk = 0; kk < 2; ++kk)
#pragma unroll
                    for (int i = 0; i < MI; ++i)
#pragma unroll
                        for (int j = 0; j < NI; ++j)
                            acc[i][j] = mfma16x32<ET>(wf[kk][j], af[kk][i], acc[i][j]);
            }
            // retire tile t+1 (tiles t+2 .. t+ST-1 may stay in flight), then all waves pass the barrier
            wait_tiles<LPT, ST - 2>(nk - 2 - t);
            block_sync_lds();
        }
    }

    if constexpr (RPRE) {
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int j = 0; j < NI; ++j)
            {
                const int64_t m = m0 + wm * TM + i * 16 + c16, n = n0 + wn * TN + j * 16 + 4 * q;
                const float4 bb = bq[j];
                float4 x = xres[i][j];
                x.x += acc[i][j][0] + bb.x;
                x.y += acc[i][j][1] + bb.y;
                x.z += acc[i][j][2] + bb.z;
                x.w += acc[i][j][3] + bb.w;
                *reinterpret_cast<float4*>(reinterpret_cast<float*>(out) + m * ldo + n) = x;
            }
    } else {
        bool done = false;
        if constexpr (APRE) {
            if (apre) {
#pragma unroll
                for (int i = 0; i < MI; ++i)
#pragma unroll
                    for (int j = 0; j < NI; ++j) {
                        const int64_t m = m0 + wm * TM + i * 16 + c16, n = n0 + wn * TN + j * 16 + 4 * q;
                        const float4 bb = bq[j];
                        const uint2 rr = xaux[i][j];
                        const float v0 = fmaxf(acc[i][j][0] + bb.x + bf2f((unsigned short)(rr.x & 0xffff)), 0.f);
                        const float v1 = fmaxf(acc[i][j][1] + bb.y + bf2f((unsigned short)(rr.x >> 16)), 0.f);
                        const float v2 = fmaxf(acc[i][j][2] + bb.z + bf2f((unsigned short)(rr.y & 0xffff)), 0.f);
                        const float v3 = fmaxf(acc[i][j][3] + bb.w + bf2f((unsigned short)(rr.y >> 16)), 0.f);
                        uint2 p;
                        p.x = pack2<ET>(v0, v1);
                        p.y = pack2<ET>(v2, v3);
                        *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(out) + m * ldo + n) = p;
                    }
                done = true;
            }
        }
        if (!done)
            store_tile16<EPI, MI, NI, ET>(acc, m0 + wm * TM, n0 + wn * TN, c16, q, bq, out, ldo, aux, ldaux, G,
                                          gstride, goff);
    }
}

// ---------------------------------------------------------------------------------
// 256x256 block tile, BK = 32 half-tiles in a 4-slot LDS ring (4 x 32 KiB).  Eight waves
// as 2 (rows) x 4 (cols), wave tile 128 x 64 = 4 x 2 blocks of 32x32x16 MFMAs.  Half-tile
// t+3 is issued while t is computed; the end-of-step wait retires only t+1
// (vmcnt(8): t+2 and t+3 stay in flight across the barrier).  64-B LDS rows; the chunk
// swizzle c ^ ((row >> 2) & 2) makes every ds_read_b128 lane group conflict-free.
// ---------------------------------------------------------------------------------
// Lane (c16, q) of a ds_read_b128 reads row R0 + c16, chunk q; a lane group is {q0: rows 0-3,
// 12-15; q1: rows 4-11} (or the same with q2 / q3), and its 16 lanes must hit the 16 distinct 16-B
// slots 4 (row & 3) + chunk of the 256-B bank row.  c ^ ((row >> 2) & 2) does (rows 0-3 / 12-15 of
// q0 take chunks 0 / 2, rows 4-7 / 8-11 of q1 chunks 1 / 3); the earlier c ^ ((row >> 2) & 3)
// put rows 0-3 (q0) and 4-7 (q1) on the same chunk: 2-way conflicts on every fragment read
// (SQ_LDS_BANK_CONFLICT = half of SQ_LDS_IDX_ACTIVE on the 256x256 kernels, round 4).
__device__ __forceinline__ int swz64(int r, int c) { return c ^ ((r >> 2) & 2); }

__device__ __forceinline__ v8s lds_frag64(const char* tile, int row, int chunk) {
    return *reinterpret_cast<const v8s*>(tile + row * 64 + swz64(row, chunk) * 16);
}

template <int EPI, int ET = VC_ELEM_BF16>
__global__ void __launch_bounds__(512, 1)
gemm_bf16_big_kernel(const uint16_t* __restrict__ A, int64_t lda, const uint16_t* __restrict__ W, int64_t ldw,
                     int nbm, int nbn, int K, const float* __restrict__ bias, void* __restrict__ out, int64_t ldo,
                     const float* __restrict__ aux, int64_t ldaux, int64_t G, int64_t gstride, int64_t goff) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int BM = 256, BN = 256, BKH = 32, NS = 4;
    constexpr int SLOT = (BM + BN) * 64;   // 32 KiB
    constexpr int TM = 128, TN = 64, MI = 8, NI = 4;  // wave tile of 16 x 16 blocks

    const int nwg = nbm * nbn;
    const int bid = blockIdx.x;
    const int xcd = bid & 7, xq = nwg >> 3, rr = nwg & 7;
    const int wgid = (xcd < rr ? xcd * (xq + 1) : rr * (xq + 1) + (xcd - rr) * xq) + (bid >> 3);
    const int tm = wgid / nbn, tn = wgid % nbn;
    const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 2, wn = wave & 3;
    const int c16 = lane & 15, q = lane >> 4;
    float4 bq[NI];  // this lane's bias columns, loaded now (their latency hides under the main loop)
    load_bias16<NI>(bias, n0 + wn * TN, q, bq);

    // staging: wave w fills A rows [32w, 32w+32) and W rows [32w, 32w+32), 16 rows per glds
    const uint16_t* asrc[2];
    const uint16_t* bsrc[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int row = wave * 32 + i * 16 + (lane >> 2);
        const int c = swz64(row, lane & 3);
        asrc[i] = A + (m0 + row) * lda + c * 8;
        bsrc[i] = W + (n0 + row) * ldw + c * 8;
    }
    const uint32_t lds0 = __builtin_amdgcn_readfirstlane(lds_addr_of(smem));
    auto stage = [&](int t) {
        const uint32_t s = lds0 + (t % NS) * SLOT;
        const int64_t k0 = (int64_t)t * BKH;
#pragma unroll
        for (int i = 0; i < 2; ++i) glds16(asrc[i] + k0, __builtin_amdgcn_readfirstlane(s + (wave * 32 + i * 16) * 64));
#pragma unroll
        for (int i = 0; i < 2; ++i)
            glds16(bsrc[i] + k0, __builtin_amdgcn_readfirstlane(s + BM * 64 + (wave * 32 + i * 16) * 64));
    };

    v4f acc[MI][NI];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

    const int nk = K / BKH;
    // fragments of half-tile t, one 32-deep k-step of v_mfma_f32_16x16x32: lane (c16, q) reads
    // row 16i + c16, 16-B chunk q (the persistent kernel's operand map)
    auto read_frags = [&](int t, v8s (&fa)[MI], v8s (&fw)[NI]) __attribute__((always_inline)) {
        const char* At = smem + (t % NS) * SLOT;
        const char* Wt = At + BM * 64;
#pragma unroll
        for (int i = 0; i < MI; ++i) fa[i] = lds_frag64(At, wm * TM + i * 16 + c16, q);
#pragma unroll
        for (int j = 0; j < NI; ++j) fw[j] = lds_frag64(Wt, wn * TN + j * 16 + c16, q);
    };
    auto mfmas = [&](const v8s (&fa)[MI], const v8s (&fw)[NI]) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int j = 0; j < NI; ++j) acc[i][j] = mfma16x32<ET>(fw[j], fa[i], acc[i][j]);
    };
    auto retire = [&](int u) __attribute__((always_inline)) {  // half-tile u + 1 resident
        if (u + 3 < nk) wait_vm<8>();
        else if (u + 2 < nk) wait_vm<4>();
        else wait_vm<0>();
        block_sync_lds();
    };

    // prologue: half-tiles 0..2 in flight; wait for 0 and read its fragments
    v8s fa0[MI], fw0[NI], fa1[MI], fw1[NI];
    stage(0);
    if (nk > 1) stage(1);
    if (nk > 2) stage(2);
    if (nk > 2) wait_vm<8>();
    else if (nk > 1) wait_vm<4>();
    else wait_vm<0>();
    block_sync_lds();
    read_frags(0, fa0, fw0);

    // half-tile t's 32 MFMAs run while t + 1's fragments are read behind the barrier that
    // publishes it (vmcnt retires only t + 1); fragment sets alternate (nk = K / 32 is even)
    for (int t = 0; t < nk - 2; t += 2) {
        if (t + 3 < nk) stage(t + 3);
        mfmas(fa0, fw0);
        retire(t);
        read_frags(t + 1, fa1, fw1);
        if (t + 4 < nk) stage(t + 4);
        mfmas(fa1, fw1);
        retire(t + 1);
        read_frags(t + 2, fa0, fw0);
    }
    mfmas(fa0, fw0);
    wait_vm<0>();
    block_sync_lds();
    read_frags(nk - 1, fa1, fw1);
    mfmas(fa1, fw1);
    store_tile16<EPI, MI, NI, ET>(acc, m0 + wm * TM, n0 + wn * TN, c16, q, bq, out, ldo, aux, ldaux, G, gstride, goff);
}

// ---------------------------------------------------------------------------------
// Streaming 1x1x1-conv kernel for the ResNet3D conv_c (cfg 20; round 5): out = relu(A.W^T + b + res),
// bf16 residual, K in {64, 128}.  At K = 64 / 128 the launch is HBM-bound (res2: 461 MB per launch for
// 26 GFLOP): the 128 x 128 two-workgroups-per-CU kernel loaded, computed and stored each tile in turn
// and moved 3.4 TB/s (0.43 of peak).  Here one 512-thread workgroup per CU keeps its 128 x 256 tile
// column (n) fixed -- W [256][K] staged into LDS once -- and walks the m tiles r, r + R, ...; while tile
// i is computed and stored, tile i+1's A rows (registers -> the other LDS buffer) and its residual
// (registers) are in flight.  Those loads are inline asm with explicit vmcnt waits: compiler-visible
// loads were re-ordered behind the stores and waited for with vmcnt(0-3) before the epilogue, which
// serialised the pipeline again.  vmcnt counts loads and stores in issue order; per step: ACH A
// loads, 8 residual loads, 8 stores.  Residual and output move as 16-B lanes (v_permlane16_swap pairs
// blocks 2jp, 2jp+1: 64-B row segments instead of 32-B ones).  Workgroups of one m tile (same r,
// different n tiles) sit R apart in block id, R % 8 == 0: same XCD.  Same k order, MFMA chain and
// epilogue arithmetic per output as cfg 5: bit-identical.
// ---------------------------------------------------------------------------------
__device__ __forceinline__ void gld16_asm(v4u& r, const void* p) {
    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(r) : "v"(p));
}
template <int N>
__device__ __forceinline__ void vm_wait_asm() {
    static_assert(N >= 0 && N < 64, "vmcnt immediate");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
template <class T>
__device__ __forceinline__ void vtie(T& r) {
    asm volatile("" : "+v"(r));
}

template <int KD, int BN>
__global__ void __launch_bounds__(512, 1)
conv_c_stream_kernel(const uint16_t* __restrict__ A, int64_t lda, const uint16_t* __restrict__ W, int64_t ldw,
                     int nbm, int R, const float* __restrict__ bias, uint16_t* __restrict__ out, int64_t ldo,
                     const uint16_t* __restrict__ res, int64_t ldres) {
    static_assert((KD == 64 || KD == 128) ? BN == 256 : (KD == 256 && BN == 128), "K 64 / 128 (N tile 256) or 256 (128)");
    constexpr int BM = 128, NKT = KD / 64, TM = 64, TN = BN / 4, MI = 4, NI = TN / 16, NP = NI / 2;
    // K <= 128: two A buffers in LDS; K = 256: one (W 64 KiB + A 64 KiB), the next tile's rows waiting
    // in registers until every wave is done with the current one (a second barrier per tile)
    constexpr bool DBUF = KD <= 128;
    constexpr int ACH = BM * 8 * NKT / 512;  // 16-B chunks of the A tile per thread
    constexpr int NRES = MI * NP;            // 16-B residual loads (and output stores) per thread per tile
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* Ws = smem;                      // NKT x [BN rows][128 B]
    char* As = smem + NKT * BN * 128;     // (2 buffers x) NKT x [128 rows][128 B]
    constexpr int ABUF = NKT * BM * 128;

    const int tn = blockIdx.x / R, r0 = blockIdx.x - tn * R;
    if (r0 >= nbm) return;
    const int64_t n0 = (int64_t)tn * BN;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 2, wn = wave & 3;
    const int c16 = lane & 15, q = lane >> 4;
    float4 bq[NI];
    load_bias16<NI>(bias, n0 + wn * TN, q, bq);

    // W [BN][KD] -> LDS (row-swizzled 16-B chunks), once
#pragma unroll
    for (int s = 0; s < BN * 8 * NKT / 512; ++s) {
        const int c = tid + 512 * s, kt = c / (BN * 8), rw = (c >> 3) & (BN - 1), ch = c & 7;
        const uint4 v = *reinterpret_cast<const uint4*>(W + (n0 + rw) * ldw + kt * 64 + ch * 8);
        *reinterpret_cast<uint4*>(Ws + kt * BN * 128 + rw * 128 + swz(rw, ch) * 16) = v;
    }
    // a lane's 16-B row segment of column-block pair jp (as store_tile16's PLAIN16 layout)
    const int64_t ncol = n0 + wn * TN + (q & 1) * 16 + 4 * (q & 2);
    v4u areg[ACH];
    auto load_a = [&](int mt) __attribute__((always_inline)) {
        const int64_t m0 = (int64_t)mt * BM;
#pragma unroll
        for (int s = 0; s < ACH; ++s) {
            const int c = tid + 512 * s, kt = c / (BM * 8), rw = (c >> 3) & (BM - 1), ch = c & 7;
            gld16_asm(areg[s], A + (m0 + rw) * lda + kt * 64 + ch * 8);
        }
    };
    auto store_a = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
        for (int s = 0; s < ACH; ++s) {
            const int c = tid + 512 * s, kt = c / (BM * 8), rw = (c >> 3) & (BM - 1), ch = c & 7;
            *reinterpret_cast<v4u*>(As + buf * ABUF + kt * BM * 128 + rw * 128 + swz(rw, ch) * 16) = areg[s];
        }
    };
    auto load_res = [&](int mt, v4u (&rr)[NRES]) __attribute__((always_inline)) {
        const int64_t m0 = (int64_t)mt * BM;
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int jp = 0; jp < NP; ++jp)
                gld16_asm(rr[i * NP + jp], res + (m0 + wm * TM + i * 16 + c16) * ldres + ncol + jp * 32);
    };
    // one m tile: issue tile `nm`'s loads, compute `mt` from LDS buffer `buf`, epilogue with rc
    // (loaded one step earlier), then stage nm's A rows into buffer buf ^ 1
    auto step = [&](int mt, int buf, v4u (&rc)[NRES], v4u (&rn)[NRES]) __attribute__((always_inline)) -> bool {
        const int nxt = mt + R;
        const bool more = nxt < nbm;
        const int nm = more ? nxt : mt;  // the last step re-reads its own tile (uniform vmcnt accounting)
        load_a(nm);
        load_res(nm, rn);
        v4f acc[MI][NI];
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int j = 0; j < NI; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kt = 0; kt < NKT; ++kt) {
            const char* At = As + buf * ABUF + kt * BM * 128;
            const char* Wt = Ws + kt * BN * 128;
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) {
                v8s af[MI];
#pragma unroll
                for (int i = 0; i < MI; ++i) af[i] = lds_frag(At, wm * TM + i * 16 + c16, 4 * kk + q);
#pragma unroll
                for (int j = 0; j < NI; ++j) {  // one W fragment live at a time (register budget)
                    const v8s wf = lds_frag(Wt, wn * TN + j * 16 + c16, 4 * kk + q);
#pragma unroll
                    for (int i = 0; i < MI; ++i) acc[i][j] = mfma16x32<VC_ELEM_BF16>(wf, af[i], acc[i][j]);
                }
            }
        }
        // rc landed: younger than its loads are the previous step's NRES stores and this step's loads
        vm_wait_asm<NRES + ACH + NRES>();
#pragma unroll
        for (int u = 0; u < NRES; ++u) vtie(rc[u]);
        const int64_t m0 = (int64_t)mt * BM;
#pragma unroll
        for (int i = 0; i < MI; ++i) {
            uint16_t* orow = out + (m0 + wm * TM + i * 16 + c16) * ldo + ncol;
#pragma unroll
            for (int jp = 0; jp < NP; ++jp) {
                // residual back into the accumulator layout: the inverse of the output's lane swap
                const v4u r = rc[i * NP + jp];
                const auto t0 = __builtin_amdgcn_permlane16_swap(r.x, r.z, false, false);
                const auto t1 = __builtin_amdgcn_permlane16_swap(r.y, r.w, false, false);
                const unsigned rw[2][2] = {{t0[0], t1[0]}, {t0[1], t1[1]}};
                unsigned pk[2][2];
#pragma unroll
                for (int sb = 0; sb < 2; ++sb) {
                    const int j = 2 * jp + sb;
                    const float4 bb = bq[j];
                    float v0 = acc[i][j][0] + bb.x, v1 = acc[i][j][1] + bb.y, v2 = acc[i][j][2] + bb.z,
                          v3 = acc[i][j][3] + bb.w;
                    v0 += bf2f((unsigned short)(rw[sb][0] & 0xffff)); v1 += bf2f((unsigned short)(rw[sb][0] >> 16));
                    v2 += bf2f((unsigned short)(rw[sb][1] & 0xffff)); v3 += bf2f((unsigned short)(rw[sb][1] >> 16));
                    pk[sb][0] = pack2<VC_ELEM_BF16>(fmaxf(v0, 0.f), fmaxf(v1, 0.f));
                    pk[sb][1] = pack2<VC_ELEM_BF16>(fmaxf(v2, 0.f), fmaxf(v3, 0.f));
                }
                const auto s0 = __builtin_amdgcn_permlane16_swap(pk[0][0], pk[1][0], false, false);
                const auto s1 = __builtin_amdgcn_permlane16_swap(pk[0][1], pk[1][1], false, false);
                v4u v;
                v.x = s0[0]; v.y = s1[0]; v.z = s0[1]; v.w = s1[1];
                *reinterpret_cast<v4u*>(orow + jp * 32) = v;
            }
        }
        if (!more) {
            vm_wait_asm<0>();
            return false;
        }
        // nm's A rows landed: younger are its NRES residual loads and this step's NRES stores
        vm_wait_asm<NRES + NRES>();
#pragma unroll
        for (int s = 0; s < ACH; ++s) vtie(areg[s]);
        if constexpr (!DBUF) block_sync_lds();  // every wave done reading the one A buffer
        store_a(DBUF ? buf ^ 1 : 0);
        block_sync_lds();
        return true;
    };

    v4u r0b[NRES], r1b[NRES];
    int mt = r0;
    load_a(mt);
    load_res(mt, r0b);
    vm_wait_asm<0>();
#pragma unroll
    for (int s = 0; s < ACH; ++s) vtie(areg[s]);
#pragma unroll
    for (int u = 0; u < NRES; ++u) vtie(r0b[u]);
    store_a(0);
    block_sync_lds();
    for (;;) {  // two steps per trip: the residual registers alternate without copies
        if (!step(mt, 0, r0b, r1b)) break;
        mt += R;
        if (!step(mt, DBUF ? 1 : 0, r1b, r0b)) break;
        mt += R;
    }
}

// ---------------------------------------------------------------------------------
// Persistent 256x256 kernel for the 16-bit-output epilogues (q|k|v, fc1; cfg 4): one workgroup
// per CU walks its tiles; the next tile's first three half-tiles (BK = 32, 4-slot LDS ring,
// counted vmcnt, one barrier per half-tile) go in flight BEFORE the current tile's epilogue,
// so the epilogue stores and the prologue latency hide behind the next tile's loads.  The bias
// lives in LDS (no VMEM in the epilogue, so the counted vmcnt stays exact).  Wave tile 128 x 64
// = 8 x 4 blocks of v_mfma_f32_16x16x32, one MFMA per block per half-tile.  Under the power-limited clocks of a dense
// MFMA loop the 16x16x32 shape sustains more FLOP/s than 32x32x16 at equal cycles per FLOP
// (MI355X_MICROARCH.md DVFS item 7: 1.12-1.14x with LDS-fed operands; measured here, same
// schedule on 32x32x16: 4096^3 1279 vs 1139 TF/s, ViViT-B q|k|v 1007 vs 911, fc1 964 vs 928).  Per half-tile a wave
// runs two 16-MFMA groups over output rows 0-63 / 64-127 of its tile: the row-64..127 A
// fragments are read under the first group, the next half-tile's row-0..63 A and all W
// fragments (second register set) under the second, after the barrier that publishes it.
// Epilogue: lane (c = l & 15, q = l >> 4) holds 4 consecutive columns of row c per block;
// v_permlane16_swap pairs blocks j, j+1 so each lane stores 8 consecutive columns (16 B).
// ---------------------------------------------------------------------------------
template <int EPI, int ET = VC_ELEM_BF16>
__global__ void __launch_bounds__(512, 1)
gemm_bf16_persist_kernel(const uint16_t* __restrict__ A, int64_t lda, const uint16_t* __restrict__ W, int64_t ldw,
                      int nbm, int nbn, int K, int N, const float* __restrict__ bias, uint16_t* __restrict__ out,
                      int64_t ldo, uint16_t* __restrict__ pre_out, int64_t ldpre) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int BM = 256, BN = 256, BKH = 32, NS = 4;
    constexpr int SLOT = (BM + BN) * 64;  // 32 KiB
    constexpr int TM = 128, TN = 64, MI = 8, NI = 4, MH = MI / 2;
    constexpr bool SAVE = EPI == VC_EPI_BIAS_GELU_TANH_SAVE;
    constexpr int NST = MI * (NI / 2) * (SAVE ? 2 : 1);  // 16-B stores per wave per tile epilogue
    float* bias_lds = reinterpret_cast<float*>(smem + NS * SLOT);

    const int ntiles = nbm * nbn;
    const int G = gridDim.x;
    const int b = blockIdx.x;
    const int lane_slot = (b & 7) * (G >> 3) + (b >> 3);

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 2, wn = wave & 3;
    const int c16 = lane & 15, q = lane >> 4;

    for (int n = tid * 4; n < N; n += 512 * 4)
        *reinterpret_cast<float4*>(bias_lds + n) = *reinterpret_cast<const float4*>(bias + n);
    __syncthreads();

    const uint32_t lds0 = __builtin_amdgcn_readfirstlane(lds_addr_of(smem));
    const int nk = K / BKH;
    const int arow = wave * 32 + (lane >> 2);
    const int acol0 = swz64(arow, lane & 3) * 8;
    const int acol1 = swz64(arow + 16, lane & 3) * 8;
    auto stage = [&](int64_t m0, int64_t n0, int t, int slotidx) __attribute__((always_inline)) {
        const uint32_t s = lds0 + (slotidx % NS) * SLOT;
        const int64_t k0 = (int64_t)t * BKH;
        glds16(A + (m0 + arow) * lda + k0 + acol0, __builtin_amdgcn_readfirstlane(s + (wave * 32) * 64));
        glds16(A + (m0 + arow + 16) * lda + k0 + acol1, __builtin_amdgcn_readfirstlane(s + (wave * 32 + 16) * 64));
        glds16(W + (n0 + arow) * ldw + k0 + acol0, __builtin_amdgcn_readfirstlane(s + BM * 64 + (wave * 32) * 64));
        glds16(W + (n0 + arow + 16) * ldw + k0 + acol1,
               __builtin_amdgcn_readfirstlane(s + BM * 64 + (wave * 32 + 16) * 64));
    };
    // fragments of a half-tile (ring slot): A rows wm*TM + 16i + c16 for i in [i0, i0 + 4) and W rows
    // wn*TN + 16j + c16 for j in [j0, j0 + 2), k-chunk q
    auto read_a = [&](int slotidx, int i0, v8s (&fa)[4]) __attribute__((always_inline)) {
        const char* At = smem + (slotidx % NS) * SLOT;
#pragma unroll
        for (int i = 0; i < 4; ++i) fa[i] = lds_frag64(At, wm * TM + (i0 + i) * 16 + c16, q);
    };
    auto read_w = [&](int slotidx, int j0, v8s (&fw)[2]) __attribute__((always_inline)) {
        const char* Wt = smem + (slotidx % NS) * SLOT + BM * 64;
#pragma unroll
        for (int j = 0; j < 2; ++j) fw[j] = lds_frag64(Wt, wn * TN + (j0 + j) * 16 + c16, q);
    };
    v4f acc[MI][NI];
    // one output quadrant (4 x 2 blocks) of the wave tile: 8 MFMAs
    auto quad = [&](auto I0, auto J0, const v8s (&fa)[4], const v8s (&fw)[2]) __attribute__((always_inline)) {
        constexpr int i0 = decltype(I0)::value, j0 = decltype(J0)::value;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[i0 + i][j0 + j] = mfma16x32<ET>(fw[j], fa[i], acc[i0 + i][j0 + j]);
    };
    // NR fragment reads ride between a quadrant's 8 MFMAs
    auto interleave = [&](auto NR) __attribute__((always_inline)) {
        constexpr int nr = decltype(NR)::value;
#pragma unroll
        for (int i = 0; i < nr; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 8 - nr, 0);
    };
    using C0 = std::integral_constant<int, 0>;
    using C2 = std::integral_constant<int, 2>;
    using C4 = std::integral_constant<int, 4>;
    using C6 = std::integral_constant<int, 6>;
    auto tile_origin = [&](int it, int64_t& m0, int64_t& n0) __attribute__((always_inline)) {
        const int tile = it * G + lane_slot;
        const int tm = tile / nbn, tn = tile - (tile / nbn) * nbn;
        m0 = (int64_t)tm * BM;
        n0 = (int64_t)tn * BN;
    };

    int it = 0;
    if (it * G + lane_slot >= ntiles) return;
    int64_t m0, n0;
    tile_origin(0, m0, n0);
    int sbase = 0;
    stage(m0, n0, 0, sbase + 0);
    stage(m0, n0, 1, sbase + 1);
    stage(m0, n0, 2, sbase + 2);
    wait_vm<8>();
    block_sync_lds();
    // two register sets for the fragments that cross a half-tile boundary (A rows 0-63, W
    // columns 0-31 and 32-63); A rows 64-127 are read and consumed inside one half-tile
    v8s aloA[4], w01A[2], w23A[2], aloB[4], w01B[2], w23B[2], ahi[4];
    auto read_head = [&](int slotidx) __attribute__((always_inline)) {
        read_a(slotidx, 0, aloA);
        read_w(slotidx, 0, w01A);
        read_w(slotidx, 2, w23A);
    };
    read_head(sbase);
    bool first = true;

    // half-tile t (t < nk - 1), quadrants (lo, 01) (lo, 23) | barrier | (hi, 23) (hi, 01):
    // rows 64-127 of t are read under the first quadrant, t + 1's lo / 01 / 23 fragments under the
    // last two, after the barrier that publishes t + 1.  PH (compile time, so the steady-state
    // body is one branch-free block): 0 head (t = 0, 1: stage t + 3; the previous epilogue's NST
    // stores are younger than half-tile t + 1), 1 main (stage t + 3, retire t + 1 with t + 2,
    // t + 3 in flight), 2 (t = nk - 3: retire t + 1 with t + 2 in flight), 3 (t = nk - 2: drain).
    auto step = [&](auto PH, int t, v8s (&alo)[4], v8s (&w01)[2], v8s (&w23)[2], v8s (&alo2)[4],
                    v8s (&w012)[2], v8s (&w232)[2]) __attribute__((always_inline)) {
        constexpr int ph = decltype(PH)::value;
        if constexpr (ph <= 1) stage(m0, n0, t + 3, sbase + t + 3);
        read_a(sbase + t, 4, ahi);
        quad(C0{}, C0{}, alo, w01);
        interleave(C4{});
        quad(C0{}, C2{}, alo, w23);
        if constexpr (ph == 0) {
            if (first) wait_vm<8>();
            else wait_vm<8 + NST>();
        } else if constexpr (ph == 1) {
            wait_vm<8>();
        } else if constexpr (ph == 2) {
            wait_vm<4>();
        } else {
            wait_vm<0>();
        }
        block_sync_lds();
        read_a(sbase + t + 1, 0, alo2);
        read_w(sbase + t + 1, 0, w012);
        quad(C4{}, C2{}, ahi, w23);
        interleave(C6{});
        read_w(sbase + t + 1, 2, w232);
        quad(C4{}, C0{}, ahi, w01);
        interleave(C2{});
    };
    auto last = [&](int t, v8s (&alo)[4], v8s (&w01)[2], v8s (&w23)[2]) __attribute__((always_inline)) {
        __builtin_amdgcn_sched_barrier(0);  // keeps the scheduler from overlapping two half-tiles' fragments
        read_a(sbase + t, 4, ahi);
        quad(C0{}, C0{}, alo, w01);
        quad(C0{}, C2{}, alo, w23);
        quad(C4{}, C2{}, ahi, w23);
        quad(C4{}, C0{}, ahi, w01);
    };
    using Head = std::integral_constant<int, 0>;
    using Main = std::integral_constant<int, 1>;
    using Tail4 = std::integral_constant<int, 2>;
    using Tail0 = std::integral_constant<int, 3>;

    while (true) {
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int j = 0; j < NI; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
        step(Head{}, 0, aloA, w01A, w23A, aloB, w01B, w23B);
        step(Head{}, 1, aloB, w01B, w23B, aloA, w01A, w23A);
        // nk = K / 32 is even (K % 64 == 0): main pairs t = 2 .. nk - 5, one more main step, the
        // tail nk - 3, nk - 2 and the last half-tile nk - 1 -- one straight-line path, so each
        // accumulator stays in its registers (a parity-dependent two-way tail made hipcc rename
        // the accumulators across the join and spill ~300 VGPRs)
        int t = 2;
        for (; t < nk - 4; t += 2) {
            step(Main{}, t, aloA, w01A, w23A, aloB, w01B, w23B);
            step(Main{}, t + 1, aloB, w01B, w23B, aloA, w01A, w23A);
        }
        step(Main{}, t, aloA, w01A, w23A, aloB, w01B, w23B);
        step(Tail4{}, t + 1, aloB, w01B, w23B, aloA, w01A, w23A);
        step(Tail0{}, t + 2, aloA, w01A, w23A, aloB, w01B, w23B);
        last(t + 3, aloB, w01B, w23B);

        ++it;
        const bool more = it * G + lane_slot < ntiles;
        int64_t nm0 = 0, nn0 = 0;
        const int nbase = sbase + nk;
        if (more) {
            tile_origin(it, nm0, nn0);
            stage(nm0, nn0, 0, nbase + 0);
            stage(nm0, nn0, 1, nbase + 1);
            stage(nm0, nn0, 2, nbase + 2);
        }

        // epilogue: + bias (LDS), activation, 16-bit, permlane16 pairs -> 16-B row stores
#pragma unroll
        for (int i = 0; i < MI; ++i) {
            const int64_t m = m0 + wm * TM + i * 16 + c16;
            uint16_t* orow = out + m * ldo;
            uint16_t* prow = SAVE ? pre_out + m * ldpre : nullptr;
#pragma unroll
            for (int jp = 0; jp < NI / 2; ++jp) {
                unsigned pk[2][2], pp[2][2];
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    const int nl = (int)n0 + wn * TN + (2 * jp + s) * 16 + 4 * q;
                    const float4 bb = *reinterpret_cast<const float4*>(bias_lds + nl);
                    float v0 = acc[i][2 * jp + s][0] + bb.x, v1 = acc[i][2 * jp + s][1] + bb.y;
                    float v2 = acc[i][2 * jp + s][2] + bb.z, v3 = acc[i][2 * jp + s][3] + bb.w;
                    if constexpr (SAVE) {
                        pp[s][0] = pack2bf(v0, v1);
                        pp[s][1] = pack2bf(v2, v3);
                    }
                    if (EPI == VC_EPI_BIAS_GELU_TANH || SAVE) {
                        v0 = gelu_tanh(v0); v1 = gelu_tanh(v1); v2 = gelu_tanh(v2); v3 = gelu_tanh(v3);
                    } else if (EPI == VC_EPI_BIAS_GELU_ERF) {
                        v0 = gelu_erf(v0); v1 = gelu_erf(v1); v2 = gelu_erf(v2); v3 = gelu_erf(v3);
                    } else if (EPI == VC_EPI_BIAS_RELU_BF16) {
                        v0 = fmaxf(v0, 0.f); v1 = fmaxf(v1, 0.f); v2 = fmaxf(v2, 0.f); v3 = fmaxf(v3, 0.f);
                    }
                    pk[s][0] = pack2<ET>(v0, v1);
                    pk[s][1] = pack2<ET>(v2, v3);
                }
                // even q: block 2jp, columns 4q .. 4q+7; odd q: block 2jp+1, columns 4(q-1) .. 4(q-1)+7
                const int64_t col = n0 + wn * TN + (2 * jp + (q & 1)) * 16 + 4 * (q & 2);
                auto s0 = __builtin_amdgcn_permlane16_swap(pk[0][0], pk[1][0], false, false);
                auto s1 = __builtin_amdgcn_permlane16_swap(pk[0][1], pk[1][1], false, false);
                uint4 v;
                v.x = s0[0]; v.y = s1[0]; v.z = s0[1]; v.w = s1[1];
                *reinterpret_cast<uint4*>(orow + col) = v;
                if constexpr (SAVE) {
                    auto u0 = __builtin_amdgcn_permlane16_swap(pp[0][0], pp[1][0], false, false);
                    auto u1 = __builtin_amdgcn_permlane16_swap(pp[0][1], pp[1][1], false, false);
                    uint4 u;
                    u.x = u0[0]; u.y = u1[0]; u.z = u0[1]; u.w = u1[1];
                    *reinterpret_cast<uint4*>(prow + col) = u;
                }
            }
        }
        if (!more) break;
        first = false;
        m0 = nm0;
        n0 = nn0;
        sbase = nbase;
        wait_vm<8 + NST>();
        block_sync_lds();
        read_head(sbase);
    }
}

// ---------------------------------------------------------------------------------
// 256x256 ping-pong kernel (cfg 8).  The two waves that share a SIMD belong to different wave
// groups (waves 0-3 = output rows 0-127 of the tile, waves 4-7 = rows 128-255; a workgroup's
// waves 0-3 and 4-7 each cover the 4 SIMDs), and group 1 runs one barrier behind group 0: while
// one group's 16 MFMAs run, the other group issues its LDS reads and LDS-DMAs and waits for them,
// so each SIMD's matrix pipe alternates between its two waves instead of both waves stalling on
// their reads at the same time (cdna_hip_programming.md §5, the 256^2 8-phase template).
//   * K in 32-deep halves, one LDS ring slot each (A 256 x 32 then W 256 x 32, 64-B rows with
//     the swz64 chunk swizzle): 4 slots = 128 KiB, one workgroup per CU;
//   * two phases per K-half u, 16 MFMAs (v_mfma_f32_16x16x32) each:
//       a(u): read A rows 0-63 of the wave tile + all 4 W fragments, stage W(u+2), MFMA rows 0-63;
//       b(u): read A rows 64-127, stage A(u+3), vmcnt(6) (retires K-half u+1), MFMA rows 64-127;
//     phase body: reads | LDS-DMA | [vmcnt] | s_barrier | lgkmcnt(0) | MFMAs | s_barrier;
//   * RAW: a K-half is retired by every wave's counted vmcnt before the first barrier of phase
//     b(u) and read from phase a(u+1) on, one barrier later for the lagging group; WAR: a slot is
//     restaged >= 2 phases after its last read (W(u+2) into W(u-2)'s slot 4 phases after, A(u+3)
//     into A(u-1)'s slot 2 phases after);
//   * per phase each wave issues 2 LDS-DMAs (16 KiB per workgroup), 3 phases' DMAs in flight.
// Epilogue: the shared store_tile16 (all epilogues); a workgroup per output tile with the
// bijective XCD remap, consecutive tiles of one XCD walking the N tiles of one A row panel.
// ---------------------------------------------------------------------------------
template <int EPI, int ET = VC_ELEM_BF16>
__global__ void __launch_bounds__(512, 1)
gemm_pp_kernel(const uint16_t* __restrict__ A, int64_t lda, const uint16_t* __restrict__ W, int64_t ldw, int nbm,
               int nbn, int K, const float* __restrict__ bias, void* __restrict__ out, int64_t ldo,
               const float* __restrict__ aux, int64_t ldaux, int64_t G, int64_t gstride, int64_t goff, int nka) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int BM = 256, BN = 256, BKH = 32, NS = 4;
    constexpr int SLOT = (BM + BN) * 64;  // 32 KiB
    constexpr int TM = 128, TN = BN / 4, MI = 8, NI = TN / 16;

    const int nwg = nbm * nbn;
    const int bid = blockIdx.x;
    const int xcd = bid & 7, xq = nwg >> 3, rr = nwg & 7;
    const int wgid = (xcd < rr ? xcd * (xq + 1) : rr * (xq + 1) + (xcd - rr) * xq) + (bid >> 3);
    const int tm = wgid / nbn, tn = wgid % nbn;
    const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 2, wn = wave & 3;
    const int c16 = lane & 15, q = lane >> 4;
    float4 bq[NI];  // this lane's bias columns, loaded now (their latency hides under the main loop)
    load_bias16<NI>(bias, n0 + wn * TN, q, bq);

    // staging: wave w fills A rows [32w, 32w + 32) and W rows [32w, 32w + 32), 16 rows per LDS-DMA
    const int arow = wave * 32 + (lane >> 2);
    const uint16_t* ag0 = A + (m0 + arow) * lda + swz64(arow, lane & 3) * 8;
    const uint16_t* ag1 = A + (m0 + arow + 16) * lda + swz64(arow + 16, lane & 3) * 8;
    const uint16_t* wg0 = W + (n0 + arow) * ldw + swz64(arow, lane & 3) * 8;
    const uint16_t* wg1 = W + (n0 + arow + 16) * ldw + swz64(arow + 16, lane & 3) * 8;
    const uint32_t lds0 = __builtin_amdgcn_readfirstlane(lds_addr_of(smem));
    // nka: K-halves of A; W may be longer (K <= 2 nka): A's columns wrap, so W = [W_hi | W_lo] against
    // A gives A.W_hi + A.W_lo in one accumulation chain (vc_gemm_h16_wrap, the split-weight fp16 build)
    auto stage_a = [&](int u) __attribute__((always_inline)) {
        const uint32_t s = lds0 + (u & (NS - 1)) * SLOT + wave * 32 * 64;
        const int ku = u < nka ? u : u - nka;
        glds16(ag0 + ku * BKH, __builtin_amdgcn_readfirstlane(s));
        glds16(ag1 + ku * BKH, __builtin_amdgcn_readfirstlane(s + 16 * 64));
    };
    auto stage_w = [&](int u) __attribute__((always_inline)) {
        const uint32_t s = lds0 + (u & (NS - 1)) * SLOT + BM * 64 + wave * 32 * 64;
        glds16(wg0 + u * BKH, __builtin_amdgcn_readfirstlane(s));
        glds16(wg1 + u * BKH, __builtin_amdgcn_readfirstlane(s + 16 * 64));
    };
    auto read_a = [&](int u, int i0, v8s (&fa)[4]) __attribute__((always_inline)) {
        const char* At = smem + (u & (NS - 1)) * SLOT;
#pragma unroll
        for (int i = 0; i < 4; ++i) fa[i] = lds_frag64(At, wm * TM + i0 + i * 16 + c16, q);
    };
    auto read_w = [&](int u, v8s (&fw)[NI]) __attribute__((always_inline)) {
        const char* Wt = smem + (u & (NS - 1)) * SLOT + BM * 64;
#pragma unroll
        for (int j = 0; j < NI; ++j) fw[j] = lds_frag64(Wt, wn * TN + j * 16 + c16, q);
    };

    v4f acc[MI][NI];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

    auto mma = [&](auto I0, const v8s (&fa)[4], const v8s (&fw)[NI]) __attribute__((always_inline)) {
        constexpr int i0 = decltype(I0)::value;
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's fragment reads
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < NI; ++j) acc[i0 + i][j] = mfma16x32<ET>(fw[j], fa[i], acc[i0 + i][j]);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
    };
    using C0 = std::integral_constant<int, 0>;
    using C4 = std::integral_constant<int, 4>;

    const int nk = K / BKH;  // even, >= 4
    v8s alo[4], ahi[4], wA[NI], wB[NI];
    // FAST (compile time): a K-half of the steady state, u + 3 < nk -- every staging, retire count and
    // barrier of the phase is known to be needed, so the phase carries no runtime tests (their scalar
    // compares and branches sat between the fragment reads and the barrier the other group waits on)
    auto phase_a = [&](auto FAST, int u, v8s (&fw)[NI]) __attribute__((always_inline)) {
        read_a(u, 0, alo);
        read_w(u, fw);
        if constexpr (decltype(FAST)::value) stage_w(u + 2);
        else if (u + 2 < nk) stage_w(u + 2);
        __builtin_amdgcn_sched_barrier(0);
        mma(C0{}, alo, fw);
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
    };
    auto phase_b = [&](auto FAST, int u, const v8s (&fw)[NI]) __attribute__((always_inline)) {
        read_a(u, 64, ahi);
        if constexpr (decltype(FAST)::value) {
            stage_a(u + 3);
            wait_vm<6>();
        } else if (u + 3 < nk) {
            stage_a(u + 3);
            wait_vm<6>();
        } else if (u + 2 < nk) {
            wait_vm<4>();
        } else {
            wait_vm<0>();
        }
        __builtin_amdgcn_sched_barrier(0);
        mma(C4{}, ahi, fw);
        // the lagging group skips its last barrier: both groups then pass the same number
        if constexpr (decltype(FAST)::value) __builtin_amdgcn_s_barrier();
        else if (u + 1 < nk || wm == 0) __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
    };
    using T_ = std::true_type;
    using F_ = std::false_type;

    // prologue: A0 W0 A1 W1 A2 in flight, retire A0 W0, publish; group 1 falls one barrier behind
    stage_a(0);
    stage_w(0);
    stage_a(1);
    stage_w(1);
    stage_a(2);
    wait_vm<6>();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (wm == 1) __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);

    int u = 0;
    for (; u + 4 < nk; u += 2) {  // K-halves u, u + 1 with u + 1 + 3 < nk
        phase_a(T_{}, u, wA);
        phase_b(T_{}, u, wA);
        phase_a(T_{}, u + 1, wB);
        phase_b(T_{}, u + 1, wB);
    }
    for (; u < nk; u += 2) {
        phase_a(F_{}, u, wA);
        phase_b(F_{}, u, wA);
        phase_a(F_{}, u + 1, wB);
        phase_b(F_{}, u + 1, wB);
    }
    store_tile16<EPI, MI, NI, ET>(acc, m0 + wm * TM, n0 + wn * TN, c16, q, bq, out, ldo, aux, ldaux, G, gstride,
                                  goff);
}

// ---------------------------------------------------------------------------------
// Persistent 256x256 ping-pong kernel with DEFERRED epilogue stores (cfg 15; q|k|v, fc1 at K >= 640).
// What bounded the K = 768 launches was not the main loop but the output write:
// every CU stores its 128-KiB tile at the same moment -- a 32-MB burst at ~4 TB/s with the matrix
// pipes idle -- and the in-order vmcnt makes the DMAs issued after a store wait for it.  Here a
// tile's epilogue only computes (bias from LDS, activation, 16-bit pack, permlane16 pairing) into 16
// packed 16-B row pieces per wave held in registers, and the stores go out during the NEXT tile, one
// per K-half in phase b for its first 16 K-halves: the chip's write stream is spread over the main
// loop (~3 TB/s) instead of bursting between tiles.  Each store is younger than the DMAs of the
// K-half it retires next, so the counted wait of phase b(u) allows the stores of phases b(u - 1) and
// b(u) on top of the 6 DMAs (vmcnt(6 + NY)); a store issued two phases earlier must have completed.
// The last tile of a workgroup stores its pieces at once.  Same K order and MFMA chain per output as
// cfgs 4 / 8 / 10: bit-identical.  One fragment register set per role (A rows, W columns) -- the
// ping-pong's reads of a phase come after the previous phase's MFMAs issued -- which leaves room for
// the 64 pending registers next to the 128 accumulators.
// ---------------------------------------------------------------------------------
template <int EPI, int ET = VC_ELEM_BF16>
__global__ void __launch_bounds__(512, 1)
gemm_ppd_kernel(const uint16_t* __restrict__ A, int64_t lda, const uint16_t* __restrict__ W, int64_t ldw, int nbm,
                int nbn, int K, int N, const float* __restrict__ bias, uint16_t* __restrict__ out, int64_t ldo) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int BM = 256, BN = 256, BKH = 32, NS = 4;
    constexpr int SLOT = (BM + BN) * 64;  // 32 KiB
    constexpr int TM = 128, TN = 64, MI = 8, NI = 4;
    constexpr int NST = MI * (NI / 2);  // 16-B row pieces per wave per tile, all deferred
    constexpr int NDEF = NST, P0 = 0;
    static_assert(EPI == VC_EPI_BIAS_BF16 || EPI == VC_EPI_BIAS_GELU_TANH || EPI == VC_EPI_BIAS_GELU_ERF ||
                      EPI == VC_EPI_BIAS_RELU_BF16,
                  "16-bit-output epilogues without a second output");
    float* bias_lds = reinterpret_cast<float*>(smem + NS * SLOT);

    const int ntiles = nbm * nbn;
    const int G = gridDim.x;
    const int b = blockIdx.x;
    const int lane_slot = (b & 7) * (G >> 3) + (b >> 3);
    const int mine = lane_slot < ntiles ? (ntiles - 1 - lane_slot) / G + 1 : 0;  // tiles of this workgroup
    if (mine == 0) return;

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 2, wn = wave & 3;
    const int c16 = lane & 15, q = lane >> 4;

    for (int n = tid * 4; n < N; n += 512 * 4)
        *reinterpret_cast<float4*>(bias_lds + n) = *reinterpret_cast<const float4*>(bias + n);
    __syncthreads();

    const int nk = K / BKH;  // even, >= 20
    const int total = mine * nk;
    const uint32_t lds0 = __builtin_amdgcn_readfirstlane(lds_addr_of(smem));
    const int arow = wave * 32 + (lane >> 2);
    // per-lane BYTE offsets from the wave-uniform panel base (32-bit: a 256-row panel is < 4 GiB)
    const uint32_t aoff0 = (uint32_t)(arow * lda + swz64(arow, lane & 3) * 8) * 2;
    const uint32_t aoff1 = (uint32_t)((arow + 16) * lda + swz64(arow + 16, lane & 3) * 8) * 2;
    const uint32_t woff0 = (uint32_t)(arow * ldw + swz64(arow, lane & 3) * 8) * 2;
    const uint32_t woff1 = (uint32_t)((arow + 16) * ldw + swz64(arow + 16, lane & 3) * 8) * 2;
    auto tile_origin = [&](int it, int64_t& m0, int64_t& n0) __attribute__((always_inline)) {
        const int tile = it * G + lane_slot;
        const int tm = tile / nbn;
        m0 = (int64_t)tm * BM;
        n0 = (int64_t)(tile - tm * nbn) * BN;
    };
    struct Cursor {
        int it, u;
        const uint16_t* p;
    };
    auto cursor_at = [&](bool is_a) __attribute__((always_inline)) {
        Cursor c;
        c.it = 0;
        c.u = 0;
        int64_t m0, n0;
        tile_origin(0, m0, n0);
        c.p = is_a ? A + m0 * lda : W + n0 * ldw;
        return c;
    };
    Cursor ca = cursor_at(true), cw = cursor_at(false);
    auto advance = [&](Cursor& c, bool is_a) __attribute__((always_inline)) {
        if (++c.u == nk) {
            c.u = 0;
            ++c.it;
            if (c.it < mine) {
                int64_t m0, n0;
                tile_origin(c.it, m0, n0);
                c.p = is_a ? A + m0 * lda : W + n0 * ldw;
            }
        }
    };
    auto stage_a = [&](int U) __attribute__((always_inline)) {
        const uint32_t s = lds0 + (U & (NS - 1)) * SLOT + wave * 32 * 64;
        glds16s(ca.p + ca.u * BKH, aoff0, __builtin_amdgcn_readfirstlane(s));
        glds16s(ca.p + ca.u * BKH, aoff1, __builtin_amdgcn_readfirstlane(s + 16 * 64));
        advance(ca, true);
    };
    auto stage_w = [&](int U) __attribute__((always_inline)) {
        const uint32_t s = lds0 + (U & (NS - 1)) * SLOT + BM * 64 + wave * 32 * 64;
        glds16s(cw.p + cw.u * BKH, woff0, __builtin_amdgcn_readfirstlane(s));
        glds16s(cw.p + cw.u * BKH, woff1, __builtin_amdgcn_readfirstlane(s + 16 * 64));
        advance(cw, false);
    };
    auto read_a = [&](int U, int i0, v8s (&fa)[4]) __attribute__((always_inline)) {
        const char* At = smem + (U & (NS - 1)) * SLOT;
#pragma unroll
        for (int i = 0; i < 4; ++i) fa[i] = lds_frag64(At, wm * TM + i0 + i * 16 + c16, q);
    };
    auto read_w = [&](int U, v8s (&fw)[4]) __attribute__((always_inline)) {
        const char* Wt = smem + (U & (NS - 1)) * SLOT + BM * 64;
#pragma unroll
        for (int j = 0; j < 4; ++j) fw[j] = lds_frag64(Wt, wn * TN + j * 16 + c16, q);
    };

    v4f acc[MI][NI];
    uint4 pend[NST];      // the previous tile's packed output pieces (P0 .. NST - 1 stored during this tile)
    int64_t pm0 = 0, pn0 = 0;  // ... and that tile's origin
    auto mma = [&](auto I0, auto FIRST, const v8s (&fa)[4], const v8s (&fw)[4]) __attribute__((always_inline)) {
        constexpr int i0 = decltype(I0)::value;
        constexpr bool first = decltype(FIRST)::value;
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                acc[i0 + i][j] = mfma16x32<ET>(fw[j], fa[i], first ? v4f{0.f, 0.f, 0.f, 0.f} : acc[i0 + i][j]);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
    };
    // piece s of the pending tile: rows i = s / 2 (16-row block of the wave tile), column pair jp = s % 2
    // (wave-uniform base of the piece's 16-row block + one loop-invariant per-lane byte offset)
    const uint32_t soff = (uint32_t)(c16 * ldo + (q & 1) * 16 + 4 * (q & 2)) * 2;
    auto store_piece = [&](auto S) __attribute__((always_inline)) {
        constexpr int sI = decltype(S)::value;
        constexpr int i = sI >> 1, jp = sI & 1;
        const uint16_t* base = out + (pm0 + wm * TM + i * 16) * ldo + pn0 + wn * TN + jp * 32;
        *reinterpret_cast<uint4*>(reinterpret_cast<char*>(const_cast<uint16_t*>(base)) + soff) = pend[sI];
    };
    // pieces s .. P0 - 1, at once (recursion over compile-time indices)
    auto store_first = [&](auto S) __attribute__((always_inline)) {
        auto rec = [&](auto self, auto T) __attribute__((always_inline)) {
            constexpr int t = decltype(T)::value;
            if constexpr (t < P0) {
                store_piece(std::integral_constant<int, t>{});
                self(self, std::integral_constant<int, t + 1>{});
            }
        };
        rec(rec, S);
    };
    using C0 = std::integral_constant<int, 0>;
    using C4 = std::integral_constant<int, 4>;
    using T_ = std::true_type;
    using F_ = std::false_type;

    v8s fa[4], fw[4];
    auto phase_a = [&](auto FIRST, int U) __attribute__((always_inline)) {
        read_a(U, 0, fa);
        read_w(U, fw);
        if (U + 2 < total) stage_w(U + 2);
        __builtin_amdgcn_sched_barrier(0);
        mma(C0{}, FIRST, fa, fw);
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
    };
    // ST: the pending piece stored in this phase (-1: none); NY: stores younger than K-half U + 1's DMAs
    auto phase_b = [&](auto FIRST, auto ST, auto NY, int U) __attribute__((always_inline)) {
        constexpr int st = decltype(ST)::value, ny = decltype(NY)::value;
        read_a(U, 64, fa);
        if (U + 3 < total) {
            stage_a(U + 3);
            if constexpr (st >= 0) store_piece(std::integral_constant<int, st >= 0 ? st : 0>{});
            wait_vm<6 + ny>();
        } else if (U + 2 < total) {
            if constexpr (st >= 0) store_piece(std::integral_constant<int, st >= 0 ? st : 0>{});
            wait_vm<4 + ny>();
        } else {
            if constexpr (st >= 0) store_piece(std::integral_constant<int, st >= 0 ? st : 0>{});
            wait_vm<0>();
        }
        __builtin_amdgcn_sched_barrier(0);
        mma(C4{}, FIRST, fa, fw);
        if (U + 1 < total || wm == 0) __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
    };
    // one tile's K-halves; STORES: the previous tile's pieces go out in phase b of K-halves 0 .. 15
    // (nk >= 20, so the ring's drain at the end of the last tile never meets a store phase)
    auto run_tile = [&](auto STORES, int U) __attribute__((always_inline)) {
        constexpr bool stores = decltype(STORES)::value;
        using N0 = std::integral_constant<int, 0>;
        using NO = std::integral_constant<int, -1>;
        if constexpr (stores) {
            // K-half 0 .. NDEF - 1 store piece P0 + u in phase b; NY counts the stores of b(u - 1), b(u)
            phase_a(T_{}, U);
            phase_b(T_{}, std::integral_constant<int, P0>{}, std::integral_constant<int, 1>{}, U);
            auto body = [&](auto S) __attribute__((always_inline)) {
                constexpr int sI = decltype(S)::value;
                if constexpr (sI < NDEF) {
                    phase_a(F_{}, U + sI);
                    phase_b(F_{}, std::integral_constant<int, P0 + sI>{}, std::integral_constant<int, 2>{}, U + sI);
                }
            };
            body(std::integral_constant<int, 1>{});
            body(std::integral_constant<int, 2>{});
            body(std::integral_constant<int, 3>{});
            body(std::integral_constant<int, 4>{});
            body(std::integral_constant<int, 5>{});
            body(std::integral_constant<int, 6>{});
            body(std::integral_constant<int, 7>{});
            body(std::integral_constant<int, 8>{});
            body(std::integral_constant<int, 9>{});
            body(std::integral_constant<int, 10>{});
            body(std::integral_constant<int, 11>{});
            body(std::integral_constant<int, 12>{});
            body(std::integral_constant<int, 13>{});
            body(std::integral_constant<int, 14>{});
            body(std::integral_constant<int, 15>{});
            phase_a(F_{}, U + NDEF);
            phase_b(F_{}, NO{}, std::integral_constant<int, 1>{}, U + NDEF);
            int u = NDEF + 1;
            if constexpr (NDEF % 2 == 0) {
                phase_a(F_{}, U + u);
                phase_b(F_{}, NO{}, N0{}, U + u);
                ++u;
            }
            for (; u < nk; u += 2) {
                phase_a(F_{}, U + u);
                phase_b(F_{}, NO{}, N0{}, U + u);
                phase_a(F_{}, U + u + 1);
                phase_b(F_{}, NO{}, N0{}, U + u + 1);
            }
        } else {
            phase_a(T_{}, U);
            phase_b(T_{}, NO{}, N0{}, U);
            phase_a(F_{}, U + 1);
            phase_b(F_{}, NO{}, N0{}, U + 1);
            for (int u = 2; u < nk; u += 2) {
                phase_a(F_{}, U + u);
                phase_b(F_{}, NO{}, N0{}, U + u);
                phase_a(F_{}, U + u + 1);
                phase_b(F_{}, NO{}, N0{}, U + u + 1);
            }
        }
    };
    // epilogue arithmetic of the tile just finished into pend: + bias (LDS), activation, 16-bit,
    // permlane16 pairs (even q: block 2jp, columns 4q .. 4q+7; odd q: block 2jp+1)
    auto finish = [&](int64_t m0, int64_t n0) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < MI; ++i) {
#pragma unroll
            for (int jp = 0; jp < NI / 2; ++jp) {
                unsigned pk[2][2];
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) {
                    const int nl = (int)n0 + wn * TN + (2 * jp + s2) * 16 + 4 * q;
                    const float4 bb = *reinterpret_cast<const float4*>(bias_lds + nl);
                    float v0 = acc[i][2 * jp + s2][0] + bb.x, v1 = acc[i][2 * jp + s2][1] + bb.y;
                    float v2 = acc[i][2 * jp + s2][2] + bb.z, v3 = acc[i][2 * jp + s2][3] + bb.w;
                    if (EPI == VC_EPI_BIAS_GELU_TANH) {
                        v0 = gelu_tanh(v0); v1 = gelu_tanh(v1); v2 = gelu_tanh(v2); v3 = gelu_tanh(v3);
                    } else if (EPI == VC_EPI_BIAS_GELU_ERF) {
                        v0 = gelu_erf(v0); v1 = gelu_erf(v1); v2 = gelu_erf(v2); v3 = gelu_erf(v3);
                    } else if (EPI == VC_EPI_BIAS_RELU_BF16) {
                        v0 = fmaxf(v0, 0.f); v1 = fmaxf(v1, 0.f); v2 = fmaxf(v2, 0.f); v3 = fmaxf(v3, 0.f);
                    }
                    pk[s2][0] = pack2<ET>(v0, v1);
                    pk[s2][1] = pack2<ET>(v2, v3);
                }
                auto s0 = __builtin_amdgcn_permlane16_swap(pk[0][0], pk[1][0], false, false);
                auto s1 = __builtin_amdgcn_permlane16_swap(pk[0][1], pk[1][1], false, false);
                pend[2 * i + jp] = make_uint4(s0[0], s1[0], s0[1], s1[1]);
            }
        }
        pm0 = m0;
        pn0 = n0;
        __builtin_amdgcn_sched_barrier(0);
        store_first(std::integral_constant<int, 0>{});
    };

    // prologue: A0 W0 A1 W1 A2 of the first tile in flight, retire A0 W0, publish; group 1 one barrier behind
    stage_a(0);
    stage_w(0);
    stage_a(1);
    stage_w(1);
    stage_a(2);
    wait_vm<6>();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (wm == 1) __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);

    int64_t m0, n0;
    tile_origin(0, m0, n0);
    run_tile(F_{}, 0);
    finish(m0, n0);
    for (int it = 1; it < mine; ++it) {
        tile_origin(it, m0, n0);
        run_tile(T_{}, it * nk);
        finish(m0, n0);
    }
    auto store_rest = [&](auto self, auto T) __attribute__((always_inline)) {
        constexpr int t = decltype(T)::value;
        if constexpr (t < NST) {
            store_piece(std::integral_constant<int, t>{});
            self(self, std::integral_constant<int, t + 1>{});
        }
    };
    store_rest(store_rest, std::integral_constant<int, P0>{});
}

// ---------------------------------------------------------------------------------
// Implicit-GEMM 3D convolution on channels-last bf16 activations (ResNet3D conv_a / conv_b /
// strided branch1; round 4): the cfg 5 machinery (BM x BN x 64 block tile, 8 waves, LDS-DMA
// ring, two workgroups per CU), with the A operand's rows gathered straight from the input
// activations: 64-deep k-tile t covers channels c0 .. c0 + 63 of kernel tap `tap` (C % 64 == 0,
// columns (kt, kh, kw, c) as vc_conv3d_im2col writes them), so the A row of output position m is
// the 128-B segment of input row in(m, tap) -- or of a 128-B zero row where the tap falls in the
// padding.  The im2col matrix (up to 9x the activations: 462 MB at ResNet3D stage 1, B = 4) is
// never written or read back.  Per k-tile the tap decomposition is wave-uniform scalar work; each
// lane's AL output rows keep their (b, t, h, w) origin in registers.
// ---------------------------------------------------------------------------------
struct ConvGeomG {
    int Tin, Hin, Win, C;
    int To, Ho, Wo;
    int kt, kh, kw;
    int st, sh, sw;
    int pt, ph, pw;
    int64_t M;  // B * To * Ho * Wo
};

// MODE 1 (the stem, vc_conv3d_stem_gemm_bf16): X is the zero-padded channels-last clip
// [B][Tp][Hp][Wp][4] bf16 (vc_conv3d_stem_pack: 3 channels + a zero 4th); the K columns are
// segments of 32 = one (kt, kh) tap row of 8 pixels x 4 channels (kw <= 8), two segments per 64-deep
// k-tile, so an A row's 16-B chunk is 2 pixels of the padded clip (16-B aligned: the window's first
// pixel index is even for stride-2 w); segments past kt * kh read the zero row.
template <int BM, int BN, int WM, int WN, int EPI, int ST = 2, int MODE = 0>
__global__ void __launch_bounds__(512, (ST == 2 || BM * BN <= 64 * 128) ? 2 : 1)
conv_gemm_kernel(const uint16_t* __restrict__ X, int64_t ldx, ConvGeomG g, const uint16_t* __restrict__ zrow,
                 const uint16_t* __restrict__ W, int64_t ldw, int nbm, int nbn, int K, const float* __restrict__ bias,
                 void* __restrict__ out, int64_t ldo, const float* __restrict__ aux, int64_t ldaux) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int SLOT = (BM + BN) * 128;
    constexpr int TM = BM / WM, TN = BN / WN;
    constexpr int MI = TM / 16, NI = TN / 16;
    constexpr int AL = BM / 64, BL = BN / 64;
    constexpr int LPT = AL + BL;
    static_assert(WM * WN == 8 && TM % 16 == 0 && TN % 32 == 0, "8 waves");

    const int nwg = nbm * nbn;
    const int bid = blockIdx.x;
    const int xcd = bid & 7, xq = nwg >> 3, rr = nwg & 7;
    const int wgid = (xcd < rr ? xcd * (xq + 1) : rr * (xq + 1) + (xcd - rr) * xq) + (bid >> 3);
    const int tm = wgid / nbn, tn = wgid % nbn;
    const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / WN, wn = wave % WN;
    const int c16 = lane & 15, q = lane >> 4;
    float4 bq[NI];  // this lane's bias columns, loaded now (their latency hides under the main loop)
    load_bias16<NI>(bias, n0 + wn * TN, q, bq);

    // this lane's A rows: output position -> batch offset (input rows) and the input origin of the window
    int64_t rbase[AL];
    int rt[AL], rh[AL], rw[AL], rch[AL];
    bool rok[AL];
#pragma unroll
    for (int i = 0; i < AL; ++i) {
        const int row = wave * (BM / 8) + i * 8 + (lane >> 3);
        const int64_t m = m0 + row;
        rok[i] = m < g.M;
        const int64_t mm = rok[i] ? m : 0;
        const int wo = (int)(mm % g.Wo);
        const int ho = (int)((mm / g.Wo) % g.Ho);
        const int to = (int)((mm / ((int64_t)g.Wo * g.Ho)) % g.To);
        const int64_t b = mm / ((int64_t)g.Wo * g.Ho * g.To);
        if constexpr (MODE == 1) {  // pixel index of the window's first tap in the padded clip
            rbase[i] = ((b * g.Tin + (int64_t)to * g.st) * g.Hin + (int64_t)ho * g.sh) * g.Win + (int64_t)wo * g.sw;
        } else {
            rbase[i] = b * g.Tin * g.Hin * (int64_t)g.Win;
        }
        rt[i] = to * g.st - g.pt;
        rh[i] = ho * g.sh - g.ph;
        rw[i] = wo * g.sw - g.pw;
        rch[i] = swz(row, lane & 7) * 8;
    }
    // MODE 0: element offset of each row's tap-(0, 0, 0) input position (outside the clip for rows whose
    // window starts in the padding: only combined with a tap offset that lands inside, checked per tap)
    int64_t roff[AL];
#pragma unroll
    for (int i = 0; i < AL; ++i)
        roff[i] = (rbase[i] + ((int64_t)rt[i] * g.Hin + rh[i]) * g.Win + rw[i]) * ldx + rch[i];

    const uint16_t* bsrc[BL];
#pragma unroll
    for (int i = 0; i < BL; ++i) {
        const int row = wave * (BN / 8) + i * 8 + (lane >> 3);
        bsrc[i] = W + (n0 + row) * ldw + swz(row, lane & 7) * 8;
    }
    const uint32_t lds0 = __builtin_amdgcn_readfirstlane(lds_addr_of(smem));
    // the tap of the next k-tile to stage, walked incrementally (stage() runs for t = 0, 1, 2, ... in
    // order): wave-uniform scalar counters instead of five integer divisions per k-tile (round 5: the
    // divisions and per-row 64-bit address products made the res4 / res5 convolutions 1.3-1.7x slower
    // than a plain GEMM of the same shape, tools/conv_vs_gemm.py).  MODE 0: channel block c0 of tap
    // (it, ih, iw); MODE 1: (kt, kh) segment 2t as (sa_t, sa_h), 2t + 1 derived from it
    int s_c0 = 0, s_iw = 0, s_ih = 0, s_it = 0;
    int64_t s_toff = 0;  // MODE 0: element offset of (s_it, s_ih, s_iw, s_c0) from a row's tap-(0, 0, 0) position
    auto stage = [&](int t, int slot) {
        const uint32_t s = lds0 + slot * SLOT;
        const int k0 = t * 64;
        if constexpr (MODE == 1) {
            // segment 2t = (s_it, s_ih), 2t + 1 = the next (it, ih) in row-major order
            int it1 = s_it, ih1 = s_ih + 1;
            if (ih1 == g.kh) { ih1 = 0; ++it1; }
            const int nseg = g.kt * g.kh;
#pragma unroll
            for (int i = 0; i < AL; ++i) {
                const int lc = rch[i] >> 3;  // this row's logical 16-B chunk (the source side of the swizzle)
                const int hi = lc >> 2, sub = lc & 3;
                const int seg = 2 * t + hi;
                const bool sok = seg < nseg;
                const int it = hi ? it1 : s_it, ih = hi ? ih1 : s_ih;
                const int64_t soff = ((int64_t)it * g.Hin + ih) * g.Win * 4 + sub * 8;
                const uint16_t* src = (rok[i] && sok) ? X + rbase[i] * 4 + soff : zrow + rch[i];
                glds16(src, __builtin_amdgcn_readfirstlane(s + (wave * (BM / 8) + i * 8) * 128));
            }
            s_it = it1;
            s_ih = ih1 + 1;
            if (s_ih == g.kh) { s_ih = 0; ++s_it; }
        } else {
#pragma unroll
            for (int i = 0; i < AL; ++i) {
                const int ti = rt[i] + s_it, hi = rh[i] + s_ih, wi = rw[i] + s_iw;
                const bool ok = rok[i] && (unsigned)ti < (unsigned)g.Tin && (unsigned)hi < (unsigned)g.Hin &&
                                (unsigned)wi < (unsigned)g.Win;
                const uint16_t* src = ok ? X + (roff[i] + s_toff) : zrow + rch[i];
                glds16(src, __builtin_amdgcn_readfirstlane(s + (wave * (BM / 8) + i * 8) * 128));
            }
            s_c0 += 64;
            s_toff += 64;
            if (s_c0 == g.C) {  // next tap: its offset recomputed once per C / 64 k-tiles
                s_c0 = 0;
                if (++s_iw == g.kw) {
                    s_iw = 0;
                    if (++s_ih == g.kh) {
                        s_ih = 0;
                        ++s_it;
                    }
                }
                s_toff = (((int64_t)s_it * g.Hin + s_ih) * g.Win + s_iw) * ldx;
            }
        }
#pragma unroll
        for (int i = 0; i < BL; ++i)
            glds16(bsrc[i] + k0, __builtin_amdgcn_readfirstlane(s + BM * 128 + (wave * (BN / 8) + i * 8) * 128));
    };

    v4f acc[MI][NI];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

    const int nk = K / 64;
    stage(0, 0);
    // tiles 1 .. ST-2 in flight too; then retire tile 0 (the tiles issued after it may stay in flight)
#pragma unroll
    for (int u = 1; u < ST - 1; ++u)
        if (u < nk) stage(u, u);
    wait_tiles<LPT, ST - 2>(nk - 1);
    block_sync_lds();

    auto ktile = [&](auto FAST, int t) {  // FAST: t <= nk - ST, no runtime tests (see gemm_bf16_kernel)
        const int slot = t % ST;
        if constexpr (decltype(FAST)::value) stage(t + ST - 1, (t + ST - 1) % ST);
        else if (t + ST - 1 < nk) stage(t + ST - 1, (t + ST - 1) % ST);
        const char* At = smem + slot * SLOT;
        const char* Wt = At + BM * 128;
        v8s af[2][MI], wf[2][NI];
#pragma unroll
        for (int i = 0; i < MI; ++i) af[0][i] = lds_frag(At, wm * TM + i * 16 + c16, q);
#pragma unroll
        for (int j = 0; j < NI; ++j) wf[0][j] = lds_frag(Wt, wn * TN + j * 16 + c16, q);
#pragma unroll
        for (int i = 0; i < MI; ++i) af[1][i] = lds_frag(At, wm * TM + i * 16 + c16, 4 + q);
#pragma unroll
        for (int j = 0; j < NI; ++j) wf[1][j] = lds_frag(Wt, wn * TN + j * 16 + c16, 4 + q);
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
            for (int i = 0; i < MI; ++i)
#pragma unroll
                for (int j = 0; j < NI; ++j) acc[i][j] = mfma16x32<VC_ELEM_BF16>(wf[kk][j], af[kk][i], acc[i][j]);
        // retire tile t + 1; the tiles staged after it (up to ST - 2) may stay in flight
        if constexpr (decltype(FAST)::value) wait_vm<LPT * (ST - 2)>();
        else wait_tiles<LPT, ST - 2>(nk - 2 - t);
        block_sync_lds();
    };
    int t = 0;
    for (; t <= nk - ST; ++t) ktile(std::true_type{}, t);
    for (; t < nk; ++t) ktile(std::false_type{}, t);
    store_tile16<EPI, MI, NI, VC_ELEM_BF16>(acc, m0 + wm * TM, n0 + wn * TN, c16, q, bq, out, ldo, aux, ldaux, 1, 0,
                                            0);
}

template <int BM, int BN, int WM, int WN, int E, int MODE, int ST>
static int launch_conv_st(const uint16_t* X, int64_t ldx, const ConvGeomG& g, const uint16_t* zrow, const uint16_t* W,
                          int64_t ldw, int nbm, int nbn, int K, const float* bias, void* out, int64_t ldo,
                          const float* aux, int64_t ldaux, hipStream_t stream) {
    constexpr int lds = ST * (BM + BN) * 128;
    static bool attr_set = false;
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute((const void*)conv_gemm_kernel<BM, BN, WM, WN, E, ST, MODE>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        if (e != hipSuccess) return fail((int)e, std::string("vc_conv3d_gemm_bf16: hipFuncSetAttribute: ") + hipGetErrorString(e));
        attr_set = true;
    }
    conv_gemm_kernel<BM, BN, WM, WN, E, ST, MODE><<<(unsigned)(nbm * nbn), 512, lds, stream>>>(
        X, ldx, g, zrow, W, ldw, nbm, nbn, K, bias, out, ldo, aux, ldaux);
    return check_launch("vc_conv3d_gemm_bf16");
}

// ring: LDS ring depth in k-tiles (2: two workgroups per CU at every tile; 3: one more k-tile in
// flight, one workgroup per CU except at 64 x 128)
template <int BM, int BN, int WM, int WN, int E, int MODE = 0>
static int launch_conv(const uint16_t* X, int64_t ldx, const ConvGeomG& g, const uint16_t* zrow, const uint16_t* W,
                       int64_t ldw, int nbm, int nbn, int K, const float* bias, void* out, int64_t ldo, const float* aux,
                       int64_t ldaux, hipStream_t stream, int ring = 2) {
    if constexpr (MODE == 0 && BN == 128)
        if (ring == 4)
            return launch_conv_st<BM, BN, WM, WN, E, MODE, 4>(X, ldx, g, zrow, W, ldw, nbm, nbn, K, bias, out, ldo, aux,
                                                              ldaux, stream);
    if (ring >= 3)  // ring 4 on 256 x 64 tiles and the stem: 3
        return launch_conv_st<BM, BN, WM, WN, E, MODE, 3>(X, ldx, g, zrow, W, ldw, nbm, nbn, K, bias, out, ldo, aux,
                                                          ldaux, stream);
    return launch_conv_st<BM, BN, WM, WN, E, MODE, 2>(X, ldx, g, zrow, W, ldw, nbm, nbn, K, bias, out, ldo, aux, ldaux,
                                                      stream);
}

// Tile configurations (BM, BN), indexed by the cfg number of vc_gemm_bf16_cfg / model.gemm_cfg; the
// numbers are stable, a retired configuration keeps its slot as {0, 0} (rejected).  Round 6 pruned the
// product library to the configurations pick_cfg chooses (3, 4, 5, 7, 8, 15, 20, 21); the round-4/5
// timing ablations and diagnostics (11-14, 16, 18, 19), the 3-slot 128-wide / 256x128 / 128x256 tiles
// (0-2), the 160x256 / 256x128 / persistent ping-pong kernels (17, 9, 10), the deeper Swin rings (22, 23)
// and the 256x192 ping-pong tile (24) were measured and not picked (their source:
// tools/experiments/gemm_retired_r06.hip.txt and the git history).
struct GemmCfg {
    int bm, bn;
};
static const GemmCfg kCfgs[] = {{0, 0},     {0, 0},     {0, 0},    {256, 256}, {256, 256}, {128, 128}, {0, 0},
                                 {64, 128},  {256, 256}, {0, 0},    {0, 0},     {0, 0},     {0, 0},     {0, 0},
                                 {0, 0},     {256, 256}, {0, 0},    {0, 0},     {0, 0},     {0, 0},     {128, 128},
                                 {64, 128}};
constexpr int kNumCfgs = 22;

template <int BM, int BN, int WM, int WN, int E, int ST = 3, int ET = VC_ELEM_BF16>
static int launch_cfg(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw, int nbm, int nbn, int K,
                      const float* bias, void* out, int64_t ldo, const float* aux, int64_t ldaux, int64_t G,
                      int64_t gs, int64_t go, hipStream_t stream) {
    constexpr int lds = ST * (BM + BN) * 128;
    static bool attr_set = false;  // per instantiation; benign race (idempotent)
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute((const void*)gemm_bf16_kernel<BM, BN, WM, WN, E, ST, ET>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        if (e != hipSuccess) return fail((int)e, std::string("vc_gemm_bf16: hipFuncSetAttribute: ") + hipGetErrorString(e));
        attr_set = true;
    }
    gemm_bf16_kernel<BM, BN, WM, WN, E, ST, ET><<<(unsigned)(nbm * nbn), 512, lds, stream>>>(
        A, lda, W, ldw, nbm, nbn, K, bias, out, ldo, aux, ldaux, G, gs, go);
    return check_launch("vc_gemm_bf16");
}

template <int E, int ET>
static int launch_big(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw, int nbm, int nbn, int K,
                      const float* bias, void* out, int64_t ldo, const float* aux, int64_t ldaux, int64_t G,
                      int64_t gs, int64_t go, hipStream_t stream) {
    constexpr int lds = 4 * 512 * 64;
    static bool attr_set = false;
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute((const void*)gemm_bf16_big_kernel<E, ET>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        if (e != hipSuccess) return fail((int)e, std::string("vc_gemm_bf16: hipFuncSetAttribute: ") + hipGetErrorString(e));
        attr_set = true;
    }
    gemm_bf16_big_kernel<E, ET><<<(unsigned)(nbm * nbn), 512, lds, stream>>>(A, lda, W, ldw, nbm, nbn, K, bias, out, ldo,
                                                                     aux, ldaux, G, gs, go);
    return check_launch("vc_gemm_bf16");
}

template <int E, int ET>
static int launch_pp(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw, int nbm, int nbn, int K,
                     const float* bias, void* out, int64_t ldo, const float* aux, int64_t ldaux, int64_t G,
                     int64_t gs, int64_t go, hipStream_t stream, int ka = 0) {
    constexpr int lds = 4 * 512 * 64;
    static bool attr_set = false;
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute((const void*)gemm_pp_kernel<E, ET>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        if (e != hipSuccess) return fail((int)e, std::string("vc_gemm_bf16: hipFuncSetAttribute: ") + hipGetErrorString(e));
        attr_set = true;
    }
    gemm_pp_kernel<E, ET><<<(unsigned)(nbm * nbn), 512, lds, stream>>>(A, lda, W, ldw, nbm, nbn, K, bias, out,
                                                                           ldo, aux, ldaux, G, gs, go,
                                                                           (ka > 0 ? ka : K) / 32);
    return check_launch("vc_gemm_bf16");
}

static int num_cus() {
    static int n = 0;
    if (!n) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        hipDeviceProp_t p;
        if (hipGetDeviceProperties(&p, dev) == hipSuccess) n = p.multiProcessorCount;
        if (n <= 0) n = 256;
    }
    return n;
}

template <int E, int ET>
static int launch_persist(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw, int nbm, int nbn, int K,
                            int N, const float* bias, void* out, int64_t ldo, hipStream_t stream,
                            const float* aux = nullptr, int64_t ldaux = 0) {
    const int lds = 4 * 512 * 64 + N * 4;
    static bool attr_set = false;
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute((const void*)gemm_bf16_persist_kernel<E, ET>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if (e != hipSuccess) return fail((int)e, std::string("vc_gemm_bf16: hipFuncSetAttribute: ") + hipGetErrorString(e));
        attr_set = true;
    }
    const int ntiles = nbm * nbn;
    int grid = num_cus() / 8 * 8;
    if (grid > (ntiles + 7) / 8 * 8) grid = (ntiles + 7) / 8 * 8;
    gemm_bf16_persist_kernel<E, ET><<<(unsigned)grid, 512, lds, stream>>>(A, lda, W, ldw, nbm, nbn, K, N, bias,
                                                                         (uint16_t*)out, ldo,
                                                                         (uint16_t*)const_cast<float*>(aux), ldaux);
    return check_launch("vc_gemm_bf16");
}

template <int E, int ET>
static int launch_ppd(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw, int nbm, int nbn, int K, int N,
                      const float* bias, void* out, int64_t ldo, hipStream_t stream) {
    const int lds = 4 * 512 * 64 + N * 4;
    static bool attr_set = false;
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute((const void*)gemm_ppd_kernel<E, ET>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if (e != hipSuccess) return fail((int)e, std::string("vc_gemm_bf16: hipFuncSetAttribute: ") + hipGetErrorString(e));
        attr_set = true;
    }
    const int ntiles = nbm * nbn;
    int grid = num_cus() / 8 * 8;
    if (grid > (ntiles + 7) / 8 * 8) grid = (ntiles + 7) / 8 * 8;
    gemm_ppd_kernel<E, ET><<<(unsigned)grid, 512, lds, stream>>>(A, lda, W, ldw, nbm, nbn, K, N, bias,
                                                                       (uint16_t*)out, ldo);
    return check_launch("vc_gemm_bf16");
}

template <int KD, int BN>
static int launch_conv_c_stream(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw, int64_t M, int64_t N,
                                const float* bias, void* out, int64_t ldo, const float* aux, int64_t ldaux,
                                hipStream_t stream) {
    constexpr int lds = (KD / 64) * BN * 128 + (KD <= 128 ? 2 : 1) * (KD / 64) * 128 * 128;
    static bool attr_set = false;
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute((const void*)conv_c_stream_kernel<KD, BN>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        if (e != hipSuccess) return fail((int)e, std::string("vc_gemm_bf16: hipFuncSetAttribute: ") + hipGetErrorString(e));
        attr_set = true;
    }
    const int nbm = (int)(M / 128), nbn = (int)(N / BN);
    // about one workgroup per CU over all n tiles; R a multiple of 8 (the n tiles of one m tile share an XCD)
    int R = (num_cus() + nbn - 1) / nbn;
    R = (R + 7) / 8 * 8;
    if (R > (nbm + 7) / 8 * 8) R = (nbm + 7) / 8 * 8;
    conv_c_stream_kernel<KD, BN><<<(unsigned)(R * nbn), 512, lds, stream>>>(
        A, lda, W, ldw, nbm, R, bias, (uint16_t*)out, ldo, reinterpret_cast<const uint16_t*>(aux), ldaux);
    return check_launch("vc_gemm_bf16");
}

template <int E, int ET>
static int launch_epi(int cfg, const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw, int64_t M, int64_t N,
                      int K, const float* bias, void* out, int64_t ldo, const float* aux, int64_t ldaux, int64_t G,
                      int64_t gs, int64_t go, hipStream_t s) {
    const int nbm = (int)(M / kCfgs[cfg].bm), nbn = (int)(N / kCfgs[cfg].bn);
    switch (cfg) {
        case 3: return launch_big<E, ET>(A, lda, W, ldw, nbm, nbn, K, bias, out, ldo, aux, ldaux, G, gs, go, s);
        case 5: return launch_cfg<128, 128, 2, 4, E, 2, ET>(A, lda, W, ldw, nbm, nbn, K, bias, out, ldo, aux, ldaux, G, gs, go, s);
        case 7: return launch_cfg<64, 128, 2, 4, E, 2, ET>(A, lda, W, ldw, nbm, nbn, K, bias, out, ldo, aux, ldaux, G, gs, go, s);
        // round 5: a deeper ring for the latency-bound small launches (Swin-T's per-stream parts)
        case 21: return launch_cfg<64, 128, 2, 4, E, 4, ET>(A, lda, W, ldw, nbm, nbn, K, bias, out, ldo, aux, ldaux, G, gs, go, s);
        case 8: return launch_pp<E, ET>(A, lda, W, ldw, nbm, nbn, K, bias, out, ldo, aux, ldaux, G, gs, go, s);
        case 20:  // streaming 1x1x1 conv with the bf16 residual (ResNet3D conv_c), K 64 / 128 (N % 256), 256
            if constexpr (E == VC_EPI_BIAS_RESID_RELU_BF16 && ET == VC_ELEM_BF16) {
                if (K == 64 && N % 256 == 0)
                    return launch_conv_c_stream<64, 256>(A, lda, W, ldw, M, N, bias, out, ldo, aux, ldaux, s);
                if (K == 128 && N % 256 == 0)
                    return launch_conv_c_stream<128, 256>(A, lda, W, ldw, M, N, bias, out, ldo, aux, ldaux, s);
                if (K == 256) return launch_conv_c_stream<256, 128>(A, lda, W, ldw, M, N, bias, out, ldo, aux, ldaux, s);
            }
            return fail(VC_ERR_INVALID_ARG, "vc_gemm_bf16: cfg 20 is bias_resid_relu with K 64 / 128 (N % 256) or 256");
        case 4:
            if constexpr (E == VC_EPI_BIAS_BF16 || E == VC_EPI_BIAS_GELU_TANH || E == VC_EPI_BIAS_GELU_ERF ||
                          E == VC_EPI_BIAS_RELU_BF16 || E == VC_EPI_BIAS_GELU_TANH_SAVE)
                return launch_persist<E, ET>(A, lda, W, ldw, nbm, nbn, K, (int)N, bias, out, ldo, s, aux, ldaux);
            return fail(VC_ERR_INVALID_ARG, "vc_gemm_bf16: cfg 4 supports bf16-output epilogues only");
        case 15:
            if constexpr (E == VC_EPI_BIAS_BF16 || E == VC_EPI_BIAS_GELU_TANH || E == VC_EPI_BIAS_GELU_ERF ||
                          E == VC_EPI_BIAS_RELU_BF16)
                return launch_ppd<E, ET>(A, lda, W, ldw, nbm, nbn, K, (int)N, bias, out, ldo, s);
            return fail(VC_ERR_INVALID_ARG, "vc_gemm_bf16: cfg 15 supports the plain 16-bit-output epilogues only");
    }
    return fail(VC_ERR_INVALID_ARG, "vc_gemm_bf16: bad config");
}

// Default tile choice (measured on MI355X, tools/tune_gemm.py at the ViViT-B B=8 inference
// shapes and tools/tune_train_gemm.py at the B=4 train-step shapes):
//   * bf16-output epilogues the persistent 256x256 kernel supports: cfg 4 whenever M, N % 256
//     (q|k|v 785 vs 675 TF/s at B=8, 769 vs 619 at B=4; o_proj dgrad 578 vs 527);
//   * the 256x256 kernel when its tiles fit one round of CUs and the GEMM is not tiny (B=4:
//     fc2 683 vs 647, fc1 dgrad 771 vs 694, q|k|v dgrad 727 vs 668 TF/s);
//   * otherwise the 128x128 two-workgroups-per-CU kernel (cfg 5), which beat cfgs 0-2 on every
//     shape measured: B=8 fc2 768 vs 677, o_proj 491 vs 430, fc1 (erf/other epilogues) 664 vs 602.
static int pick_cfg(int64_t M, int64_t N, int64_t K, int epi) {
    const bool bf16_out = epi == VC_EPI_BIAS_BF16 || epi == VC_EPI_BIAS_GELU_TANH || epi == VC_EPI_BIAS_GELU_ERF ||
                          epi == VC_EPI_BIAS_RELU_BF16 || epi == VC_EPI_BIAS_GELU_TANH_SAVE;
    const int64_t t256 = (M / 256) * (N / 256);
    // round 5: plain-bias outputs with at least a round of 256 x 256 tiles on the persistent kernel with
    // deferred stores (cfg 15): q|k|v 12800 x 2304 x 768 49.9 vs 52.6 us (cfg 8), 25344 rows 92.8 vs 97.7
    // (cfg 4); per tile after the first 21.2 vs 23.3 us (tools/gemm_stamps.py).  Not with a GELU: its
    // epilogue arithmetic at the tile boundary is serial there (fc1 81.0 vs 75.9 us)
    if (epi == VC_EPI_BIAS_BF16 && M % 256 == 0 && N % 256 == 0 && K % 64 == 0 && K >= 640 && N <= 8192 &&
        t256 >= 256)
        return 15;
    // round 5: the ResNet3D conv_c at K = 64 / 128 (HBM-bound) on the streaming kernel
    // (K = 256 on 128-column tiles, one A buffer: res4 25088x1024x256 27.4 vs 43.7 us, 4.24 TB/s)
    if (epi == VC_EPI_BIAS_RESID_RELU_BF16 && M % 128 == 0 &&
        (((K == 64 || K == 128) && N % 256 == 0) || (K == 256 && N % 128 == 0)))
        return 20;
    // round 5, Swin-T's per-stream parts (B = 1 of the 4-stream headline; tools/pp_check.py --swinpart
    // --graph, hipGraph-timed): the 64x128 tile where 128x128 tiles are under ~2.5 rounds of CUs and N is
    // wide (stage 2 fc1 3328x1536x384 10.7 vs 11.7 us, stage 3 q|k|v 1024x2304x768 9.6 vs 10.8, stage 1
    // fc1 12544x768x256 13.4 vs 14.9); the f32-residual GEMMs below a round of 128x128 tiles likewise
    // (stage 3 proj 1024x768x768 8.4 vs 12.0), and with a 4-deep ring when K is long (stage 3 fc2
    // 1024x768x3072: 48 k-tiles per workgroup, latency-bound: 21.0 vs 38.1)
    const int64_t t128 = (M / 128) * (N / 128);
    if ((epi == VC_EPI_BIAS_BF16 || epi == VC_EPI_BIAS_GELU_ERF) && M % 64 == 0 && N % 128 == 0 && N >= 768 &&
        t128 < 640 && !(M % 256 == 0 && N % 256 == 0 && t256 >= 64 && epi == VC_EPI_BIAS_BF16 && K >= 192))
        return 7;
    if (epi == VC_EPI_BIAS_RESID_F32 && M % 64 == 0 && N % 128 == 0 && t128 < 256) {
        if (K >= 2048 && (M / 64) * (N / 128) < 128) return 21;
        return 7;
    }
    // exact-GELU outputs below ~4 rounds of 256x256 tiles: cfg 5 (Swin-T stages 2-4 fc1,
    // tools/tune_swin_gemm.py: 28 vs 36 us at 12544x1536x384, 46 vs 55 at 6400x3072x768)
    // (round 4: the ping-pong kernel, cfg 8, where the tiles fill <= 2.5 rounds of CUs: fc1 at 12800 rows
    // 75.7 vs 78.7 us, q|k|v 50.7 vs 50.5; in the ViViT-B B = 8 two-stream forward +0.3 %)
    if (bf16_out && M % 256 == 0 && N % 256 == 0 && K % 64 == 0 && K >= 192 && N <= 8192 && t256 >= 64 &&
        t256 <= 640 && !(epi == VC_EPI_BIAS_GELU_ERF && t256 < 1024))
        return 8;
    if (bf16_out && M % 256 == 0 && N % 256 == 0 && K % 32 == 0 && K >= 192 && N <= 8192 && t256 >= 64 &&
        !(epi == VC_EPI_BIAS_GELU_ERF && t256 < 1024))
        return 4;
    // (t256 >= 128: Swin-T stage 4 fc2, 6400x768x3072 with 75 tiles, runs 51 us on cfg 5 vs 79 on cfg 3)
    // round 4: the ping-pong kernel (cfg 8) instead of cfg 3: fc2 at 12800 rows 79.2 vs 87.4 us; in the
    // ViViT-B B = 8 two-stream forward 957.9 -> 967.8 clips/s (tools/ab_model_cfg.py, interleaved)
    if (M % 256 == 0 && N % 256 == 0 && K % 64 == 0 && K >= 128 && t256 >= 128 && t256 <= 256 &&
        !(N <= 768 && K <= 768))
        return 8;
    if (M % 256 == 0 && N % 256 == 0 && K % 32 == 0 && t256 >= 128 && t256 <= 256 && !(N <= 768 && K <= 768))
        return 3;
    // narrow f32-residual outputs (N <= 384): 64x128 tiles, twice the workgroups to hide the
    // residual round trip (Swin-T proj / fc2: 44 vs 46 us at 200704x128x128, 14 vs 16 at 12544x384x384)
    if (epi == VC_EPI_BIAS_RESID_F32 && N <= 384 && M % 64 == 0) return 7;
    return 5;
}

}  // namespace vc

using namespace vc;

// elem = VC_ELEM_F16: the fp16 operand build of the inference epilogues 0-4 (bf16 for the rest)
extern "C" int vc_gemm_h16(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw, int64_t M, int64_t N,
                           int64_t K, const float* bias, int epilogue, void* out, int64_t ldo, const float* aux,
                           int64_t ldaux, int64_t G, int64_t group_stride, int64_t group_offset, int elem, int cfg,
                           hipStream_t stream) {
    if (elem != VC_ELEM_BF16 && elem != VC_ELEM_F16) return fail(VC_ERR_INVALID_ARG, "vc_gemm: bad elem");
    if (elem == VC_ELEM_F16 && epilogue > VC_EPI_EMBED_F32)
        return fail(VC_ERR_UNSUPPORTED, "vc_gemm: fp16 operands support epilogues 0-4 (the inference forward) only");
    if (!A || !W || !bias || !out) return fail(VC_ERR_INVALID_ARG, "vc_gemm_bf16: null pointer");
    if (M <= 0 || N <= 0 || K <= 0 || M % 128 || N % 128 || K % GBK)
        return fail(VC_ERR_INVALID_ARG, "vc_gemm_bf16: need M % 128 == 0, N % 128 == 0, K % 64 == 0 (got M=" +
                                            std::to_string(M) + " N=" + std::to_string(N) + " K=" + std::to_string(K) + ")");
    if (lda % 8 || ldw % 8 || ldo % 4 || lda < K || ldw < K || ldo < N)
        return fail(VC_ERR_INVALID_ARG, "vc_gemm_bf16: bad leading dimension");
    if ((((uintptr_t)A) | ((uintptr_t)W) | ((uintptr_t)out) | ((uintptr_t)bias)) & 15)
        return fail(VC_ERR_INVALID_ARG, "vc_gemm_bf16: pointers must be 16-byte aligned");
    if (epilogue == VC_EPI_EMBED_F32 && (!aux || G <= 0 || ldaux % 4))
        return fail(VC_ERR_INVALID_ARG, "vc_gemm_bf16: EMBED epilogue needs aux, G > 0");
    if (epilogue == VC_EPI_BIAS_RESID_RELU_BF16 && (!aux || ldaux % 4 || ldaux < N || ((uintptr_t)aux & 7)))
        return fail(VC_ERR_INVALID_ARG, "vc_gemm_bf16: RESID_RELU epilogue needs a bf16 residual (aux) with ldaux >= N");
    if ((epilogue == VC_EPI_BIAS_GELU_TANH_SAVE || epilogue == VC_EPI_DGELU_TANH) &&
        (!aux || ldaux % 4 || ldaux < N || ((uintptr_t)aux & 7)))
        return fail(VC_ERR_INVALID_ARG, "vc_gemm_bf16: GELU_SAVE / DGELU epilogues need a bf16 aux with ldaux >= N");
    if (epilogue == VC_EPI_BIAS_ADD_F32 && (!aux || ldaux % 4 || ldaux < N || ((uintptr_t)aux & 15)))
        return fail(VC_ERR_INVALID_ARG, "vc_gemm_bf16: BIAS_ADD_F32 epilogue needs an f32 aux with ldaux >= N");
    // the persistent kernel writes 16-byte row chunks of out (and of the saved pre-activation)
    const bool st16_ok = ldo % 8 == 0 && (epilogue != VC_EPI_BIAS_GELU_TANH_SAVE || (ldaux % 8 == 0 && !((uintptr_t)aux & 15)));
    // the streaming conv_c kernel (cfg 20) moves 16-B pieces of out and of the bf16 residual and has no
    // grouped-row addressing
    const bool c20_ok = ldo % 8 == 0 && ldaux % 8 == 0 && !(((uintptr_t)out | (uintptr_t)aux) & 15) && G <= 1;
    if (cfg < 0) {
        cfg = pick_cfg(M, N, K, epilogue);
        if ((cfg == 4 || cfg == 15) && (!st16_ok || ((uintptr_t)out & 15))) cfg = 5;
        if (cfg == 20 && !c20_ok) cfg = 5;
    }
    if (cfg == 20 && !c20_ok)
        return fail(VC_ERR_INVALID_ARG, "vc_gemm_bf16: cfg 20 needs ldo, ldaux % 8 == 0, 16-B aligned out / aux, G <= 1");
    if (cfg < 0 || cfg >= kNumCfgs || kCfgs[cfg].bm == 0 || M % kCfgs[cfg].bm || N % kCfgs[cfg].bn)
        return fail(VC_ERR_INVALID_ARG, "vc_gemm_bf16: no tile config divides M x N");
    if ((M / kCfgs[cfg].bm) * (N / kCfgs[cfg].bn) > (1 << 30)) return fail(VC_ERR_INVALID_ARG, "vc_gemm_bf16: grid too large");
    const int k = (int)K;
    if (cfg == 8 && K < 128) return fail(VC_ERR_INVALID_ARG, "vc_gemm_bf16: cfg 8 needs K >= 128");
    if (cfg == 15 && (K < 640 || K % 64 || N > 8192 || ldo % 8 || ((uintptr_t)out & 15)))
        return fail(VC_ERR_INVALID_ARG, "vc_gemm_bf16: cfg 15 needs K >= 640, K % 64 == 0, N <= 8192, 16-B output rows");
    if (cfg == 4 && (K / 32 < 6 || N > 8192 || !st16_ok ||
                     (epilogue > VC_EPI_BIAS_GELU_ERF && epilogue != VC_EPI_BIAS_RELU_BF16 &&
                      epilogue != VC_EPI_BIAS_GELU_TANH_SAVE)))
        return fail(VC_ERR_INVALID_ARG, "vc_gemm_bf16: cfg 4 needs K>=192, N<=8192, ldo%8==0, a 16-bit-output epilogue");
#define VC_GEMM_CASE(E)                                                                                         \
    case E:                                                                                                     \
        return elem == VC_ELEM_F16 ? launch_epi<(E) <= VC_EPI_EMBED_F32 ? (E) : 0, VC_ELEM_F16>(                  \
                                         cfg, A, lda, W, ldw, M, N, k, bias, out, ldo, aux, ldaux, G, group_stride, \
                                         group_offset, stream)                                                  \
                                   : launch_epi<E, VC_ELEM_BF16>(cfg, A, lda, W, ldw, M, N, k, bias, out, ldo, aux, \
                                                                 ldaux, G, group_stride, group_offset, stream);
    switch (epilogue) {
        VC_GEMM_CASE(VC_EPI_BIAS_BF16)
        VC_GEMM_CASE(VC_EPI_BIAS_GELU_TANH)
        VC_GEMM_CASE(VC_EPI_BIAS_GELU_ERF)
        VC_GEMM_CASE(VC_EPI_BIAS_RESID_F32)
        VC_GEMM_CASE(VC_EPI_EMBED_F32)
        VC_GEMM_CASE(VC_EPI_BIAS_F32)
        VC_GEMM_CASE(VC_EPI_BIAS_RELU_BF16)
        VC_GEMM_CASE(VC_EPI_BIAS_RESID_RELU_BF16)
        VC_GEMM_CASE(VC_EPI_BIAS_ADD_F32)
        VC_GEMM_CASE(VC_EPI_BIAS_GELU_TANH_SAVE)
        VC_GEMM_CASE(VC_EPI_DGELU_TANH)
    }
#undef VC_GEMM_CASE
    return fail(VC_ERR_INVALID_ARG, "vc_gemm_bf16: bad epilogue");
}

// Implicit-GEMM Conv3d (conv_gemm_kernel): out[m][n] = epilogue(sum_(tap, c) x[in(m, tap)][c] *
// Wt[n][tap * C + c] + bias[n]); output rows m < B*To*Ho*Wo (rows up to the next multiple of 128
// are written too: the caller's buffer has them), zero_row: >= 64 zero bf16 (16-B aligned).
extern "C" int vc_conv3d_gemm_bf16_cfg(const uint16_t* x, int64_t ldx, int64_t B, int64_t T, int64_t H, int64_t W,
                                       int64_t C, const int* kernel, const int* stride, const int* pad,
                                       const uint16_t* zero_row, const uint16_t* Wt, int64_t ldw, int64_t N,
                                       const float* bias, int epilogue, void* out, int64_t ldo, const void* aux,
                                       int64_t ldaux, int ring, int tile, hipStream_t stream) {
    if (ring != 0 && ring != 2 && ring != 3 && ring != 4)
        return fail(VC_ERR_INVALID_ARG, "vc_conv3d_gemm_bf16_cfg: ring must be 0, 2, 3 or 4");
    if (tile < 0 || tile > 2) return fail(VC_ERR_INVALID_ARG, "vc_conv3d_gemm_bf16_cfg: tile must be 0, 1 or 2");
    // ring 0 (automatic): a 3-deep ring when the grid has fewer tiles than two per CU (the workgroups
    // are few, so each one's DMA latency is exposed; ResNet3D res4 / res5 at B = 4: +1.1 / +1.5 % of
    // the forward each), else 2 (res2 / res3: -3.7 / -2.5 %), tools/ab_resnet3d_ring.py, round 4
    // (round 5: a 3-deep ring puts 128 x 128 tiles at ONE workgroup per CU (96 KiB of LDS), so there it pays
    // only when the tiles fit one round of CUs: res3 conv_b, 392 tiles, ring 2 +1.6 % of the forward,
    // tools/ab_resnet3d_conv.py; 64 x 128 and 256 x 64 tiles keep two workgroups per CU at ring 3)
    auto pick_ring = [&](int64_t tiles, bool big = false) {
        if (ring) return ring;
        const int64_t cus = num_cus();
        return (big ? tiles <= cus : tiles < 2 * cus) ? 3 : 2;
    };
    if (!x || !kernel || !stride || !pad || !zero_row || !Wt || !bias || !out)
        return fail(VC_ERR_INVALID_ARG, "vc_conv3d_gemm_bf16: null pointer");
    for (int d = 0; d < 3; ++d)
        if (kernel[d] <= 0 || stride[d] <= 0 || pad[d] < 0 || kernel[d] > 255)
            return fail(VC_ERR_INVALID_ARG, "vc_conv3d_gemm_bf16: bad kernel / stride / pad");
    if (B <= 0 || T <= 0 || H <= 0 || W <= 0 || C <= 0 || C % 64 || N <= 0 || N % 64)
        return fail(VC_ERR_INVALID_ARG, "vc_conv3d_gemm_bf16: need C % 64 == 0 and N % 64 == 0");
    ConvGeomG g;
    g.Tin = (int)T; g.Hin = (int)H; g.Win = (int)W; g.C = (int)C;
    g.kt = kernel[0]; g.kh = kernel[1]; g.kw = kernel[2];
    g.st = stride[0]; g.sh = stride[1]; g.sw = stride[2];
    g.pt = pad[0]; g.ph = pad[1]; g.pw = pad[2];
    g.To = (int)((T + 2 * g.pt - g.kt) / g.st + 1);
    g.Ho = (int)((H + 2 * g.ph - g.kh) / g.sh + 1);
    g.Wo = (int)((W + 2 * g.pw - g.kw) / g.sw + 1);
    if (g.To <= 0 || g.Ho <= 0 || g.Wo <= 0) return fail(VC_ERR_INVALID_ARG, "vc_conv3d_gemm_bf16: empty output");
    g.M = B * g.To * g.Ho * (int64_t)g.Wo;
    const int64_t K = (int64_t)g.kt * g.kh * g.kw * C;
    if (ldx % 8 || ldx < C || ldw % 8 || ldw < K || ldo < N || K > (1LL << 30))
        return fail(VC_ERR_INVALID_ARG, "vc_conv3d_gemm_bf16: bad leading dimension");
    if ((((uintptr_t)x) | ((uintptr_t)Wt) | ((uintptr_t)out) | ((uintptr_t)bias) | ((uintptr_t)zero_row)) & 15)
        return fail(VC_ERR_INVALID_ARG, "vc_conv3d_gemm_bf16: pointers must be 16-byte aligned");
    const float* auxf = reinterpret_cast<const float*>(aux);
    if (N % 128) {
        // 64 output channels (ResNet3D stage 1): 256 x 64 tiles (8 waves as 8 x 1), no padded-channel MFMAs
        const int nbm = (int)((g.M + 255) / 256), nbn = (int)(N / 64);
        if ((int64_t)nbm * nbn > (1 << 30)) return fail(VC_ERR_INVALID_ARG, "vc_conv3d_gemm_bf16: grid too large");
        if (ldo % 8) return fail(VC_ERR_INVALID_ARG, "vc_conv3d_gemm_bf16: ldo % 8");
        ring = pick_ring((int64_t)nbm * nbn);
        if (epilogue == VC_EPI_BIAS_RELU_BF16)
            return launch_conv<256, 64, 8, 1, VC_EPI_BIAS_RELU_BF16>(x, ldx, g, zero_row, Wt, ldw, nbm, nbn, (int)K, bias,
                                                                      out, ldo, auxf, ldaux, stream, ring);
        if (epilogue == VC_EPI_BIAS_BF16)
            return launch_conv<256, 64, 8, 1, VC_EPI_BIAS_BF16>(x, ldx, g, zero_row, Wt, ldw, nbm, nbn, (int)K, bias, out,
                                                                 ldo, auxf, ldaux, stream, ring);
        return fail(VC_ERR_INVALID_ARG, "vc_conv3d_gemm_bf16: N % 128 != 0 supports bias / bias_relu only");
    }
    const int nbm = (int)((g.M + 127) / 128), nbn = (int)(N / 128);
    if ((int64_t)nbm * nbn > (1 << 30)) return fail(VC_ERR_INVALID_ARG, "vc_conv3d_gemm_bf16: grid too large");
    if (tile == 1 && !(ldo % 8 == 0 && (epilogue == VC_EPI_BIAS_RELU_BF16 || epilogue == VC_EPI_BIAS_BF16)))
        return fail(VC_ERR_INVALID_ARG, "vc_conv3d_gemm_bf16_cfg: 64 x 128 tiles need bias / bias_relu, ldo % 8 == 0");
    // fewer 128 x 128 tiles than CUs (ResNet3D stage 4: 49 x 4 at B = 4): 64 x 128 tiles, twice the workgroups
    if (tile == 1 || (tile == 0 && nbm * nbn < num_cus() && ldo % 8 == 0 &&
                      (epilogue == VC_EPI_BIAS_RELU_BF16 || epilogue == VC_EPI_BIAS_BF16))) {
        const int nbm64 = (int)((g.M + 63) / 64);
        ring = pick_ring((int64_t)nbm64 * nbn);
        if (epilogue == VC_EPI_BIAS_RELU_BF16)
            return launch_conv<64, 128, 2, 4, VC_EPI_BIAS_RELU_BF16>(x, ldx, g, zero_row, Wt, ldw, nbm64, nbn, (int)K,
                                                                      bias, out, ldo, auxf, ldaux, stream, ring);
        return launch_conv<64, 128, 2, 4, VC_EPI_BIAS_BF16>(x, ldx, g, zero_row, Wt, ldw, nbm64, nbn, (int)K, bias, out,
                                                             ldo, auxf, ldaux, stream, ring);
    }
    ring = pick_ring((int64_t)nbm * nbn, true);
    switch (epilogue) {
        case VC_EPI_BIAS_BF16:
            if (ldo % 8) break;
            return launch_conv<128, 128, 2, 4, VC_EPI_BIAS_BF16>(x, ldx, g, zero_row, Wt, ldw, nbm, nbn, (int)K, bias,
                                                                  out, ldo, auxf, ldaux, stream, ring);
        case VC_EPI_BIAS_RELU_BF16:
            if (ldo % 8) break;
            return launch_conv<128, 128, 2, 4, VC_EPI_BIAS_RELU_BF16>(x, ldx, g, zero_row, Wt, ldw, nbm, nbn, (int)K,
                                                                       bias, out, ldo, auxf, ldaux, stream, ring);
        case VC_EPI_BIAS_RESID_RELU_BF16:
            if (!aux || ldaux % 4 || ldaux < N || ((uintptr_t)aux & 7)) break;
            return launch_conv<128, 128, 2, 4, VC_EPI_BIAS_RESID_RELU_BF16>(x, ldx, g, zero_row, Wt, ldw, nbm, nbn,
                                                                             (int)K, bias, out, ldo, auxf, ldaux, stream, ring);
        default:
            break;
    }
    return fail(VC_ERR_INVALID_ARG, "vc_conv3d_gemm_bf16: epilogue must be bias / bias_relu / bias_resid_relu "
                                    "(16-B output rows; resid_relu: a bf16 aux with ldaux >= N)");
}

extern "C" int vc_conv3d_gemm_bf16_ring(const uint16_t* x, int64_t ldx, int64_t B, int64_t T, int64_t H, int64_t W,
                                        int64_t C, const int* kernel, const int* stride, const int* pad,
                                        const uint16_t* zero_row, const uint16_t* Wt, int64_t ldw, int64_t N,
                                        const float* bias, int epilogue, void* out, int64_t ldo, const void* aux,
                                        int64_t ldaux, int ring, hipStream_t stream) {
    if (ring != 0 && ring != 2 && ring != 3)
        return fail(VC_ERR_INVALID_ARG, "vc_conv3d_gemm_bf16_ring: ring must be 0, 2 or 3");
    return vc_conv3d_gemm_bf16_cfg(x, ldx, B, T, H, W, C, kernel, stride, pad, zero_row, Wt, ldw, N, bias, epilogue, out,
                                   ldo, aux, ldaux, ring, 0, stream);
}

extern "C" int vc_conv3d_gemm_bf16(const uint16_t* x, int64_t ldx, int64_t B, int64_t T, int64_t H, int64_t W,
                                   int64_t C, const int* kernel, const int* stride, const int* pad,
                                   const uint16_t* zero_row, const uint16_t* Wt, int64_t ldw, int64_t N,
                                   const float* bias, int epilogue, void* out, int64_t ldo, const void* aux,
                                   int64_t ldaux, hipStream_t stream) {
    return vc_conv3d_gemm_bf16_cfg(x, ldx, B, T, H, W, C, kernel, stride, pad, zero_row, Wt, ldw, N, bias, epilogue, out,
                                   ldo, aux, ldaux, 0, 0, stream);
}

// Stem input packing for vc_conv3d_stem_gemm_bf16: f32 [B][C][T][H][W] (C <= 4) -> bf16
// [B][T + 2pt][H + 2ph][W + 2pw][4], zero in the padding and the unused channels.  One thread per
// padded pixel: C strided f32 reads (coalesced along w), one 8-B store.
__global__ void __launch_bounds__(256) stem_pack_kernel(const float* __restrict__ x, int C, int T, int H, int W, int pt,
                                                        int ph, int pw, int Tp, int Hp, int Wp, int64_t total,
                                                        uint16_t* __restrict__ xp) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= total) return;
    int64_t r = i;
    const int wq = (int)(r % Wp);
    r /= Wp;
    const int hq = (int)(r % Hp);
    r /= Hp;
    const int tq = (int)(r % Tp);
    const int64_t b = r / Tp;
    const int t = tq - pt, h = hq - ph, w = wq - pw;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    if ((unsigned)t < (unsigned)T && (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W) {
        const int64_t plane = (int64_t)T * H * W;
        const float* src = x + b * C * plane + ((int64_t)t * H + h) * W + w;
        for (int c = 0; c < C; ++c) v[c] = src[c * plane];
    }
    uint2 o;
    o.x = pack2bf(v[0], v[1]);
    o.y = pack2bf(v[2], v[3]);
    *reinterpret_cast<uint2*>(xp + i * 4) = o;
}

extern "C" int vc_conv3d_stem_pack(const float* x, int64_t B, int64_t C, int64_t T, int64_t H, int64_t W,
                                   const int* pad, uint16_t* xp, hipStream_t stream) {
    if (!x || !pad || !xp) return fail(VC_ERR_INVALID_ARG, "vc_conv3d_stem_pack: null pointer");
    if (B <= 0 || C <= 0 || C > 4 || T <= 0 || H <= 0 || W <= 0 || pad[0] < 0 || pad[1] < 0 || pad[2] < 0 ||
        ((uintptr_t)xp & 7))
        return fail(VC_ERR_INVALID_ARG, "vc_conv3d_stem_pack: bad shape (C <= 4) / alignment");
    const int Tp = (int)T + 2 * pad[0], Hp = (int)H + 2 * pad[1], Wp = (int)W + 2 * pad[2];
    const int64_t total = B * Tp * (int64_t)Hp * Wp;
    stem_pack_kernel<<<(unsigned)((total + 255) / 256), 256, 0, stream>>>(x, (int)C, (int)T, (int)H, (int)W, pad[0],
                                                                          pad[1], pad[2], Tp, Hp, Wp, total, xp);
    return check_launch("vc_conv3d_stem_pack");
}

// Stem Conv3d as an implicit GEMM over the packed clip (conv_gemm_kernel MODE 1): Wt [N][>= K]
// with K = 64 * ceil(kt * kh / 2) columns (seg = kt_i * kh + kh_i; column seg * 32 + kw_i * 4 + c),
// zero where kw_i >= kw or c >= C; the output rows up to the next multiple of 128 are written.
extern "C" int vc_conv3d_stem_gemm_bf16(const uint16_t* xp, int64_t B, int64_t T, int64_t H, int64_t W,
                                        const int* kernel, const int* stride, const int* pad, const uint16_t* zero_row,
                                        const uint16_t* Wt, int64_t ldw, int64_t N, const float* bias, int epilogue,
                                        void* out, int64_t ldo, hipStream_t stream) {
    if (!xp || !kernel || !stride || !pad || !zero_row || !Wt || !bias || !out)
        return fail(VC_ERR_INVALID_ARG, "vc_conv3d_stem_gemm_bf16: null pointer");
    for (int d = 0; d < 3; ++d)
        if (kernel[d] <= 0 || stride[d] <= 0 || pad[d] < 0)
            return fail(VC_ERR_INVALID_ARG, "vc_conv3d_stem_gemm_bf16: bad kernel / stride / pad");
    if (kernel[2] > 8 || stride[2] % 2 || B <= 0 || N <= 0 || N % 64)
        return fail(VC_ERR_INVALID_ARG, "vc_conv3d_stem_gemm_bf16: need kw <= 8, an even w stride, N % 64 == 0");
    ConvGeomG g;
    g.Tin = (int)T + 2 * pad[0]; g.Hin = (int)H + 2 * pad[1]; g.Win = (int)W + 2 * pad[2]; g.C = 4;
    g.kt = kernel[0]; g.kh = kernel[1]; g.kw = kernel[2];
    g.st = stride[0]; g.sh = stride[1]; g.sw = stride[2];
    g.pt = 0; g.ph = 0; g.pw = 0;
    g.To = (int)((g.Tin - g.kt) / g.st + 1);
    g.Ho = (int)((g.Hin - g.kh) / g.sh + 1);
    g.Wo = (int)((g.Win - g.kw) / g.sw + 1);
    if (g.To <= 0 || g.Ho <= 0 || g.Wo <= 0 || g.Win % 2) return fail(VC_ERR_INVALID_ARG, "vc_conv3d_stem_gemm_bf16: geometry");
    g.M = B * g.To * g.Ho * (int64_t)g.Wo;
    const int64_t K = 64 * ((g.kt * g.kh + 1) / 2);
    if (ldw % 8 || ldw < K || ldo < N || ldo % 8)
        return fail(VC_ERR_INVALID_ARG, "vc_conv3d_stem_gemm_bf16: bad leading dimension");
    if ((((uintptr_t)xp) | ((uintptr_t)Wt) | ((uintptr_t)out) | ((uintptr_t)bias) | ((uintptr_t)zero_row)) & 15)
        return fail(VC_ERR_INVALID_ARG, "vc_conv3d_stem_gemm_bf16: pointers must be 16-byte aligned");
    if (N % 128) {
        const int nbm = (int)((g.M + 255) / 256), nbn = (int)(N / 64);
        if ((int64_t)nbm * nbn > (1 << 30)) return fail(VC_ERR_INVALID_ARG, "vc_conv3d_stem_gemm_bf16: grid too large");
        if (epilogue == VC_EPI_BIAS_RELU_BF16)
            return launch_conv<256, 64, 8, 1, VC_EPI_BIAS_RELU_BF16, 1>(xp, 0, g, zero_row, Wt, ldw, nbm, nbn, (int)K,
                                                                         bias, out, ldo, nullptr, 0, stream);
        return fail(VC_ERR_INVALID_ARG, "vc_conv3d_stem_gemm_bf16: N % 128 != 0 supports bias_relu only");
    }
    const int nbm = (int)((g.M + 127) / 128), nbn = (int)(N / 128);
    if ((int64_t)nbm * nbn > (1 << 30)) return fail(VC_ERR_INVALID_ARG, "vc_conv3d_stem_gemm_bf16: grid too large");
    if (epilogue == VC_EPI_BIAS_RELU_BF16)
        return launch_conv<128, 128, 2, 4, VC_EPI_BIAS_RELU_BF16, 1>(xp, 0, g, zero_row, Wt, ldw, nbm, nbn, (int)K, bias,
                                                                      out, ldo, nullptr, 0, stream);
    if (epilogue == VC_EPI_BIAS_BF16)
        return launch_conv<128, 128, 2, 4, VC_EPI_BIAS_BF16, 1>(xp, 0, g, zero_row, Wt, ldw, nbm, nbn, (int)K, bias,
                                                                 out, ldo, nullptr, 0, stream);
    return fail(VC_ERR_INVALID_ARG, "vc_conv3d_stem_gemm_bf16: epilogue must be bias / bias_relu");
}

// vc_gemm_h16 on the ping-pong kernel with A's columns wrapping at ka (ka <= K <= 2 ka): W = [W1 | W2]
// ([N][K]) against A [M][ka] sums A.W1 + A.W2[:, :K - ka] in one fp32 MFMA chain.  With W1 / W2 the
// fp16 high / low parts of fp32 weights this is the split-weight product (fp16 operands, ~fp32 weights).
extern "C" int vc_gemm_h16_wrap(const uint16_t* A, int64_t lda, int64_t ka, const uint16_t* W, int64_t ldw, int64_t M,
                                int64_t N, int64_t K, const float* bias, int epilogue, void* out, int64_t ldo,
                                const float* aux, int64_t ldaux, int64_t G, int64_t group_stride, int64_t group_offset,
                                int elem, hipStream_t stream) {
    if (elem != VC_ELEM_BF16 && elem != VC_ELEM_F16) return fail(VC_ERR_INVALID_ARG, "vc_gemm_h16_wrap: bad elem");
    if (!A || !W || !bias || !out) return fail(VC_ERR_INVALID_ARG, "vc_gemm_h16_wrap: null pointer");
    if (M <= 0 || N <= 0 || M % 256 || N % 256 || ka <= 0 || ka % 64 || K % 64 || K < ka || K > 2 * ka || K < 128)
        return fail(VC_ERR_INVALID_ARG, "vc_gemm_h16_wrap: need M, N % 256 == 0, ka, K % 64 == 0, ka <= K <= 2 ka");
    if (lda % 8 || ldw % 8 || ldo % 8 || lda < ka || ldw < K || ldo < N)
        return fail(VC_ERR_INVALID_ARG, "vc_gemm_h16_wrap: bad leading dimension");
    if ((((uintptr_t)A) | ((uintptr_t)W) | ((uintptr_t)out) | ((uintptr_t)bias)) & 15)
        return fail(VC_ERR_INVALID_ARG, "vc_gemm_h16_wrap: pointers must be 16-byte aligned");
    if (epilogue == VC_EPI_EMBED_F32 && (!aux || G <= 0 || ldaux % 4))
        return fail(VC_ERR_INVALID_ARG, "vc_gemm_h16_wrap: EMBED epilogue needs aux, G > 0");
    const int nbm = (int)(M / 256), nbn = (int)(N / 256), k = (int)K, kai = (int)ka;
#define VC_WRAP_CASE(E)                                                                                                \
    case E:                                                                                                            \
        return elem == VC_ELEM_F16 ? launch_pp<E, VC_ELEM_F16>(A, lda, W, ldw, nbm, nbn, k, bias, out, ldo, aux, ldaux, G, \
                                                               group_stride, group_offset, stream, kai)               \
                                   : launch_pp<E, VC_ELEM_BF16>(A, lda, W, ldw, nbm, nbn, k, bias, out, ldo, aux, ldaux, \
                                                                G, group_stride, group_offset, stream, kai);
    switch (epilogue) {
        VC_WRAP_CASE(VC_EPI_BIAS_BF16)
        VC_WRAP_CASE(VC_EPI_BIAS_GELU_TANH)
        VC_WRAP_CASE(VC_EPI_BIAS_GELU_ERF)
        VC_WRAP_CASE(VC_EPI_BIAS_RESID_F32)
        VC_WRAP_CASE(VC_EPI_EMBED_F32)
    }
#undef VC_WRAP_CASE
    return fail(VC_ERR_INVALID_ARG, "vc_gemm_h16_wrap: epilogue must be one of the inference epilogues 0-4");
}

// the tile config vc_gemm_bf16 / vc_gemm_h16 run with cfg = -1 (host only: no launch, no GPU)
extern "C" int vc_gemm_pick(int64_t M, int64_t N, int64_t K, int epilogue, int64_t ldo, int64_t ldaux,
                            const void* aux) {
    const bool st16_ok =
        ldo % 8 == 0 && (epilogue != VC_EPI_BIAS_GELU_TANH_SAVE || (ldaux % 8 == 0 && !((uintptr_t)aux & 15)));
    int cfg = pick_cfg(M, N, K, epilogue);
    if ((cfg == 4 || cfg == 15) && !st16_ok) cfg = 5;
    if (cfg == 20 && (ldo % 8 || ldaux % 8 || ((uintptr_t)aux & 15))) cfg = 5;
    return cfg;
}

extern "C" int vc_gemm_bf16_cfg(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw, int64_t M, int64_t N,
                                int64_t K, const float* bias, int epilogue, void* out, int64_t ldo, const float* aux,
                                int64_t ldaux, int64_t G, int64_t group_stride, int64_t group_offset, int cfg,
                                hipStream_t stream) {
    return vc_gemm_h16(A, lda, W, ldw, M, N, K, bias, epilogue, out, ldo, aux, ldaux, G, group_stride, group_offset,
                       VC_ELEM_BF16, cfg, stream);
}

extern "C" int vc_gemm_bf16(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw, int64_t M, int64_t N,
                            int64_t K, const float* bias, int epilogue, void* out, int64_t ldo, const float* aux,
                            int64_t ldaux, int64_t G, int64_t group_stride, int64_t group_offset,
                            hipStream_t stream) {
    return vc_gemm_bf16_cfg(A, lda, W, ldw, M, N, K, bias, epilogue, out, ldo, aux, ldaux, G, group_stride,
                            group_offset, -1, stream);
}
