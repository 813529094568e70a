// Fused joint space-time attention forward (flash-style), head_dim 64, bf16 MFMA.
//
// Replaces eager_attention_forward of ViViT (TF5/models/vivit/modeling_vivit.py:149-174):
// softmax(scale * Q K^T) V per (clip, head) over all S = 1 + 16*14*14 = 3137 tokens,
// without materialising the S x S scores (472 MB fp32 per clip per layer in the eager path).
//
// gfx950 structure (cdna_hip_programming.md Appendix B "Fused attention prefill"):
//   * workgroup = 4 waves; each wave owns 32 query rows of one (clip, head); two
//     workgroups per CU (two waves per SIMD);
//   * K/V tiles of 64 keys staged by LDS-DMA (global_load_lds, issued from inline asm so
//     hipcc's LDS wait counts stay exact) into a 4-slot ring; a counted vmcnt retires only
//     the tile needed next, one raw s_barrier per tile; K image XOR-swizzled for ds_read_b128,
//     V image swizzled for the ds_read_b64_tr_b16 transpose read;
//   * swapped QK^T (S^T = K . Q^T): a query's scores live in ONE lane column, so the row
//     max needs one cross-half exchange and only on the rare re-base path;
//   * the running row max enters the QK^T MFMA chain as its initial accumulator
//     (S' = Q'.K^T - m, with scale*log2 e folded into Q'), so the inference path per score
//     is exp2 + cvt: no per-tile max and no VALU row sum.  The row sum l rides on the matrix
//     pipe: one v_mfma_f32_16x16x32 per 16-key step multiplies the P^T fragment (already the
//     B operand of P.V) by a constant 0/1 selector, so l sums exactly the 16-bit P that P.V
//     consumes.  m is tile 0's exact row max and is never re-based in the common case: P is
//     exact at any magnitude until exp2 overflows (a score 128 above m), and a row sum above
//     2^64 (or inf / NaN) makes the workgroup repeat the pass re-basing on every tile's exact
//     max.  The training forward (WLSE) keeps f32 VALU row sums, which double as the
//     detector of a grown max (defer-max, cdna_hip_programming.md T13: re-base when a
//     partial sum exceeds 2^8), so its log-sum-exp is the f32 one the backward assumes;
//   * S'^T accumulator registers feed P.V directly as the B operand of O^T = V^T . P^T
//     (§3 "An accumulator tile as the next MFMA's operand"); P never touches LDS;
//   * software pipeline inside each wave: the QK^T MFMAs of tile t+1 are issued before
//     tile t's softmax, so the MFMA pipe runs them while the VALU does exp2/cvt (inference:
//     pinned by sched_barrier fences, see iter());
//   * output rows widened to 16-byte stores with v_permlane32_swap (T21).
#include "common.hpp"

#include <type_traits>

namespace vc {

constexpr int AK = 64;                      // keys per tile
constexpr int KV_TILE_BYTES = AK * 64 * 2;  // 8 KiB (one of K or V)
constexpr int KV_SLOT = 2 * KV_TILE_BYTES;  // K then V
constexpr int NSLOT = 4;
constexpr float LIM = 256.0f;  // WLSE: partial row-sum bound (P <= 2^8) before the running max is re-based

// Experiment hook (round 5, tools/ab_attn.sh -DVC_ATTN_SWEXP=k): the first k of every 32 exp2 of a
// wave-tile on the VALU instead of v_exp_f32 -- round to nearest by the 1.5 * 2^23 trick, a cubic on
// [-1/2, 1/2] (rel. error 1e-4, below bf16's 2^-9), the integer part added into the exponent bits:
// 9 plain VALU ops (4 issue cycles each) for one 8-cycle transcendental.
#ifndef VC_ATTN_SWEXP
#define VC_ATTN_SWEXP 0
#endif
__device__ __forceinline__ float sw_exp2(float x) {
    x = fmaxf(x, -126.0f);
    const float t = x + 12582912.0f;
    const float f = x - (t - 12582912.0f);
    float p = __builtin_fmaf(f, 0.0550292665f, 0.2422569819f);
    p = __builtin_fmaf(f, p, 0.6932530550f);
    p = __builtin_fmaf(f, p, 0.9999513387f);
    return __builtin_bit_cast(float, __builtin_bit_cast(unsigned, p) + (__builtin_bit_cast(unsigned, t) << 23));
}

__device__ __forceinline__ int kswz(int r, int c) { return c ^ ((r >> 1) & 7); }
__device__ __forceinline__ int vswz(int r, int c) { return c ^ (((r >> 1) & 1) << 2); }

// LDS-DMA of one 16-byte piece per lane, saddr form: 64-bit wave-uniform base in SGPRs +
// 32-bit per-lane offset, so the per-tile address advance is scalar arithmetic.  hipcc never
// uses m0 in this kernel (checked in the ISA: every m0 access is one of these asm blocks), so
// m0 is declared clobbered instead of saved / restored (2 SALU fewer per piece, +0.8 %).
__device__ __forceinline__ void adma16s(const void* sbase, uint32_t voff, uint32_t lds_addr) {
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1"
                 :
                 : "v"(voff), "s"(sbase), "s"(lds_addr)
                 : "memory", "m0");
}

template <int N>
__device__ __forceinline__ void attn_wait_vm() {
    static_assert(N >= 0 && N < 16, "vmcnt");
    __builtin_amdgcn_s_waitcnt(0x0F70 | N);
}

__device__ __forceinline__ void attn_sync() {
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
}

// One 4-wave workgroup = 128 queries of one (clip, head); each wave owns 32 query rows, two
// workgroups per CU (two waves per SIMD, 256 VGPRs each).  Measured alternatives (DESIGN.md
// §5): 64 queries per wave (every K/V fragment feeding two MFMAs) needs ~330 registers and ran
// 1.3x slower at two waves per SIMD; at ONE wave per SIMD (256 queries per workgroup, 32-key
// pipeline halves, a three-stage QK^T / exp2 / P.V in-wave pipeline, no spills:
// tools/experiments/attention_w64.hip.txt, round 3) 295.5 vs 253.7 us at ViViT-B B = 8 -- the
// scores land in AGPRs (VGPRs full) and every exp2 needs a v_accvgpr_read first, which makes the
// single wave issue-bound; an 8-wave ping-pong workgroup (MFMA and softmax phases of the two waves of a
// SIMD offset by a barrier, tools/experiments/attention_pingpong.hip.txt) ran 295-330 us vs
// 264 us; split-half softmax, K-fragment prefetch, a 5-slot ring and a P.V lag were neutral
// to 8.5 % slower (round 1).
// REBASE_ALWAYS: the LIM = 0 build of the threshold test (re-base the running max on every
// tile, cdna_hip_programming.md rule 26: must agree with the shipped build to rounding).
// WLSE: also store the base-2 log-sum-exp of each query's scores, lse[(b*H + h)*S + q] =
// m + log2(l) (running max and row sum), from which the backward kernels recompute P.
// ET: 16-bit operand type of q|k|v, P and out (VC_ELEM_BF16 / VC_ELEM_F16).
template <bool REBASE_ALWAYS, bool WLSE, int ET = VC_ELEM_BF16>
__global__ void __launch_bounds__(256, 2)
attn_fwd_d64_kernel(const uint16_t* __restrict__ qkv, int64_t ld, int S, int H, float c_log2,
                    uint16_t* __restrict__ out, int64_t ldo, float* __restrict__ lse) {
    constexpr int QB = 1;
    constexpr int AQ = 128;  // query rows per workgroup (4 waves x 32)
    constexpr int NS = NSLOT;
    extern __shared__ __attribute__((aligned(16))) char smem[];

    // XCD-aware order: the workgroups of one (clip, head) share its K/V; give every XCD a
    // contiguous range of linear ids so they meet in that XCD's L2 (blocks L and L+8 share
    // an XCD under round-robin dispatch; bijective remap, §5 "XCD swizzle must be bijective")
    const int nq = gridDim.x, nwg = gridDim.x * gridDim.y;
    const int L = blockIdx.y * nq + blockIdx.x;
    const int xq = nwg >> 3, xr = nwg & 7, xcd = L & 7;
    const int wg = (xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + (L >> 3);
    const int qblk = wg % nq;
    const int bh = wg / nq;
    const int b = bh / H, hh = bh % H;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 31, h = lane >> 5;

    const int64_t tok0 = (int64_t)b * S;
    const uint16_t* qbase = qkv + hh * 64;
    const uint16_t* kbase = qkv + (int64_t)H * 64 + hh * 64 + tok0 * ld;
    const uint16_t* vbase = qkv + (int64_t)2 * H * 64 + hh * 64 + tok0 * ld;
    const uint32_t lds0 = __builtin_amdgcn_readfirstlane(
        (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)smem);

    // ---- Q'^T fragments (B operand of S^T = K.Q'^T): lane holds Q'[q][d = 16kk + 8h + 0..7]
    v8s qf[QB][4];
#pragma unroll
    for (int qb = 0; qb < QB; ++qb) {
        const int q = qblk * AQ + (wave * QB + qb) * 32 + r;
        const int qc = q < S ? q : S - 1;
        const uint16_t* qrow = qbase + (tok0 + qc) * ld + 8 * h;
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
            const v8s raw = *reinterpret_cast<const v8s*>(qrow + 16 * kk);
            if (c_log2 == 1.0f) {
                qf[qb][kk] = raw;  // producer folded the scale into q
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) qf[qb][kk][j] = (short)to16<ET>(from16<ET>((unsigned short)raw[j]) * c_log2);
            }
        }
    }

    // staging: 64 key rows of K and V (8 rows x 128 B per wave-instruction), wave w: rows 16w..16w+15;
    // per-lane byte offsets are loop-invariant, the tile advance goes into the scalar base
    const int srow = wave * 16 + (lane >> 3), spc = lane & 7;
    const uint32_t ko0 = (uint32_t)(srow * ld + kswz(srow, spc) * 8) * 2;
    const uint32_t ko1 = (uint32_t)((srow + 8) * ld + kswz(srow + 8, spc) * 8) * 2;
    const uint32_t vo0 = (uint32_t)(srow * ld + vswz(srow, spc) * 8) * 2;
    const uint32_t vo1 = (uint32_t)((srow + 8) * ld + vswz(srow + 8, spc) * 8) * 2;
    auto stage = [&](int t) {
        const uint32_t s = lds0 + (t % NS) * KV_SLOT + wave * 16 * 128;
        const uint16_t* kt = kbase + (int64_t)t * AK * ld;
        const uint16_t* vt = vbase + (int64_t)t * AK * ld;
        adma16s(kt, ko0, __builtin_amdgcn_readfirstlane(s));
        adma16s(kt, ko1, __builtin_amdgcn_readfirstlane(s + 8 * 128));
        adma16s(vt, vo0, __builtin_amdgcn_readfirstlane(s + KV_TILE_BYTES));
        adma16s(vt, vo1, __builtin_amdgcn_readfirstlane(s + KV_TILE_BYTES + 8 * 128));
    };

    // per-lane constant LDS byte offsets (relative to a ring slot):
    //  K row read (ds_read_b128) of k-step kk for key block 0 (block 1 = +32 rows = +4096 B)
    int koff[4];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) koff[kk] = r * 128 + kswz(r, kk * 2 + h) * 16;
    //  V^T transpose read (ds_read_b64_tr_b16) for d-block db; the key-row part
    //  kb*32 + 16s (+8) is a multiple of 4 rows and goes into the immediate offset
    const int gi = lane & 15;
    const int tq = gi >> 2, tp = gi & 3;
    const int gcol = ((lane >> 4) & 1) * 16 + tp * 4;
    int voff[2];
#pragma unroll
    for (int db = 0; db < 2; ++db) {
        const int col = db * 32 + gcol;
        const int ra = 4 * h + tq;
        voff[db] = KV_TILE_BYTES + ra * 128 + vswz(ra, col >> 3) * 16 + (col & 7) * 2;
    }

    v16f o[QB][2];   // O^T[d][q] per query block, d-blocks 0/1
    v16f minit[QB];  // -running max of this lane's query, broadcast: initial accumulator of S'
    // Row sums.  WLSE (training forward): f32 partial sums on the VALU (packed pairs), which
    // double as the grown-max detector.  Inference: on the matrix pipe, D = Sel . P^T over a
    // 16x16x32 block, where the P^T fragment of a 16-key step (lane (r, h) holds P[query r][8
    // keys]) is read as the 32 x 16 B operand (lane l: k-group l >> 4 = (r >> 4) + 2h, column
    // l & 15 = r & 15).  Sel[i][k] = 1 when the k-group parity (query r >= 16) equals i >> 3,
    // so D rows 0-7 sum query j's 16 keys and rows 8-15 query j + 16's; lane l then holds the
    // sum of query (l & 15) + 16 (l >> 5).  It sums exactly the 16-bit P that P.V consumes.
    v2f l_run[QB];
    v4f lsum[QB];
    v8s sel;
    {
        const short one = ET == VC_ELEM_F16 ? (short)0x3C00 : (short)0x3F80;
        const short v = (((lane >> 4) & 1) == ((lane & 15) >> 3)) ? one : (short)0;
#pragma unroll
        for (int j = 0; j < 8; ++j) sel[j] = v;
    }

    // ---- S'^T = K . Q'^T - m for QB query blocks x two 32-key blocks of tile t; each K
    //      fragment feeds QB MFMAs (-m enters as the C operand of the first k-step);
    //      KB1 = false skips key block 1 (a last tile holding <= 32 keys)
    auto qk_mfma = [&](const char* slot, v16f (&sc)[QB][2], bool kb1 = true) {
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
            const v8s k0 = *reinterpret_cast<const v8s*>(slot + koff[kk]);
#pragma unroll
            for (int qb = 0; qb < QB; ++qb) sc[qb][0] = mfma32x16<ET>(k0, qf[qb][kk], kk == 0 ? minit[qb] : sc[qb][0]);
            if (kb1) {
                const v8s k1 = *reinterpret_cast<const v8s*>(slot + koff[kk] + 4096);
#pragma unroll
                for (int qb = 0; qb < QB; ++qb) sc[qb][1] = mfma32x16<ET>(k1, qf[qb][kk], kk == 0 ? minit[qb] : sc[qb][1]);
            }
        }
    };
    //      keys beyond S masked to -inf (last tile only; key block 1 not computed at all when
    //      the tile holds <= 32 keys: TimeSformer's 197-token rows end 5 keys into their 4th tile)
    auto qk = [&](const char* slot, int t, v16f (&sc)[QB][2]) {
        const int kv0 = t * AK;
        if (kv0 + AK > S) {
            const bool kb1 = kv0 + 32 < S;
            qk_mfma(slot, sc, kb1);
#pragma unroll
            for (int qb = 0; qb < QB; ++qb)
#pragma unroll
                for (int e = 0; e < 16; ++e) {
                    const int key = (e & 3) + 8 * (e >> 2) + 4 * h;
                    if (kv0 + key >= S) sc[qb][0][e] = -INFINITY;
                    if (!kb1 || kv0 + 32 + key >= S) sc[qb][1][e] = -INFINITY;
                }
        } else {
            qk_mfma(slot, sc);
        }
    };
    auto exp_all = [&](v16f (&sc)[QB][2]) {
#pragma unroll
        for (int qb = 0; qb < QB; ++qb)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                sc[qb][0][e] = __builtin_amdgcn_exp2f(sc[qb][0][e]);
                sc[qb][1][e] = __builtin_amdgcn_exp2f(sc[qb][1][e]);
            }
    };
    // this lane's partial row sums of P (32 keys) as packed pairs (WLSE path)
    auto psum = [&](const v16f (&sc)[QB][2], v2f (&ps)[QB]) {
#pragma unroll
        for (int qb = 0; qb < QB; ++qb) {
            v2f u[8];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                u[j] = v2f{sc[qb][0][4 * j], sc[qb][0][4 * j + 1]} + v2f{sc[qb][0][4 * j + 2], sc[qb][0][4 * j + 3]};
                u[4 + j] = v2f{sc[qb][1][4 * j], sc[qb][1][4 * j + 1]} + v2f{sc[qb][1][4 * j + 2], sc[qb][1][4 * j + 3]};
            }
            ps[qb] = ((u[0] + u[1]) + (u[2] + u[3])) + ((u[4] + u[5]) + (u[6] + u[7]));
        }
    };
    // exact row max of S (both lane halves); plain fmaxf, not inline-asm v_max3: the
    // hazard recognizer must see these reads of fresh MFMA results to pad them
    auto rowmax_of = [&](const v16f (&sc)[2]) {
        float m0 = fmaxf(sc[0][0], sc[1][0]), m1 = fmaxf(sc[0][1], sc[1][1]);
#pragma unroll
        for (int e = 2; e < 16; e += 2) {
            m0 = fmaxf(m0, fmaxf(sc[0][e], sc[1][e]));
            m1 = fmaxf(m1, fmaxf(sc[0][e + 1], sc[1][e + 1]));
        }
        const float m = fmaxf(m0, m1);
        return fmaxf(m, __shfl_xor(m, 32, 64));
    };
    // re-base the running max of every query on the exact max of tile t's S' (which is
    // relative to the old max): O, the row sums, the C operand and tile t+1's S' follow
    auto rebase = [&](auto next_c, v16f (&sc)[QB][2], v16f (&sn)[QB][2]) {
        constexpr int NEXT = decltype(next_c)::value;
#pragma unroll
        for (int qb = 0; qb < QB; ++qb) {
            const float delta = fmaxf(rowmax_of(sc[qb]), 0.f);
            const float alpha = __builtin_amdgcn_exp2f(-delta);
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                sc[qb][0][e] -= delta;
                sc[qb][1][e] -= delta;
                o[qb][0][e] *= alpha;
                o[qb][1][e] *= alpha;
                minit[qb][e] -= delta;
            }
            if constexpr (NEXT != 2) {
#pragma unroll
                for (int e = 0; e < 16; ++e) { sn[qb][0][e] -= delta; sn[qb][1][e] -= delta; }
            }
            if constexpr (WLSE) {
                l_run[qb] *= alpha;
            } else {
                // lane l's row sum belongs to query (l & 15) + 16 (l >> 5), not to this lane's
                lsum[qb] *= __shfl(alpha, (lane & 15) + ((lane >> 5) << 4), 64);
            }
        }
    };

    const int ntiles = (S + AK - 1) / AK;
    // Static wave priority for one of the two workgroups that share a CU (MI355X_MICROARCH.md
    // "Two waves per SIMD" item 4: priority outranks age, so one fixed winner instead of the
    // age-based arbitration flipping between them): initially co-resident blocks are L and
    // L + 256, so prio 1 by bit 8 of L.  +1.2 % (three interleaved A/Bs at B = 8: 259/263,
    // 256/259, 258/261 us; priority by block-id bit 3 instead: neutral).
    if ((L >> 8) & 1) __builtin_amdgcn_s_setprio(1);

    // One pass over the keys.  RB = 1 re-bases the running max on every tile (exact max, P <= 1).
    // RB = 0: WLSE re-bases only when a partial row sum exceeds LIM (P > 2^8 or inf / NaN);
    // inference never re-bases inside the pass — P is relative to tile 0's max, which is exact
    // for any magnitude until exp2 overflows — and the caller repeats the pass with RB = 1 when
    // a row sum came out non-finite or above 2^64.
    // a wave whose 32 queries all lie past S (the last query block of a clip) computes
    // nothing: it only stages its share of every tile and joins the barriers
    const bool live = qblk * AQ + wave * 32 < S;
    auto dead_pass = [&]() {
        stage(0);
        if (ntiles > 1) stage(1);
        if (ntiles > 2) stage(2);
        if (ntiles > 2) attn_wait_vm<4>();
        else attn_wait_vm<0>();
        attn_sync();
        for (int t = 0; t < ntiles; ++t) {
            if (t + NS - 1 < ntiles) stage(t + NS - 1);
            if (t + 2 < ntiles) {
                if (t + 3 < ntiles) attn_wait_vm<4>();
                else attn_wait_vm<0>();
                attn_sync();
            }
        }
    };
    auto pass = [&](auto rb_c) {
        constexpr bool RB = decltype(rb_c)::value;
#pragma unroll
        for (int qb = 0; qb < QB; ++qb) {
#pragma unroll
            for (int e = 0; e < 16; ++e) { o[qb][0][e] = 0.f; o[qb][1][e] = 0.f; minit[qb][e] = 0.f; }
            l_run[qb] = v2f{0.f, 0.f};
            lsum[qb] = v4f{0.f, 0.f, 0.f, 0.f};
        }
        if (!live) {
            dead_pass();
            return;
        }
        stage(0);
        if (ntiles > 1) stage(1);
        if (ntiles > 2) stage(2);
        if (ntiles > 2) attn_wait_vm<4>();  // tiles 0 and 1 resident, 2 in flight
        else attn_wait_vm<0>();
        attn_sync();
        // tile 0 establishes the running max m
        v16f scur[QB][2];
        qk(smem, 0, scur);
#pragma unroll
        for (int qb = 0; qb < QB; ++qb) {
            const float m = rowmax_of(scur[qb]);
#pragma unroll
            for (int e = 0; e < 16; ++e) { scur[qb][0][e] -= m; scur[qb][1][e] -= m; minit[qb][e] = -m; }
        }

        // one iteration: S' of tile t+1 is computed (MFMA) while tile t's softmax runs on the
        // VALU, then O += P_t V_t.  Ring of NSLOT = 4: slot t (V_t), slot t+1 (K_{t+1}) are
        // read, t+2 lands, t+3 is staged into the slot read one iteration ago.
        // NEXT: 0 = tile t+1 is a full tile, 1 = tile t+1 may be partial (masked), 2 = t is last.
        // In the unrolled main loop the slots are compile-time constants, so every LDS address is
        // a loop-invariant per-lane VGPR plus an immediate offset.
        // V^T fragments of 16-key step g (key rows 16g .. 16g + 15 of the slot) for d-blocks 0 / 1
        auto vread = [&](const char* slot, int g, v8s (&vv)[2]) {
#pragma unroll
            for (int db = 0; db < 2; ++db) {
                const char* pa = slot + voff[db] + g * 16 * 128;
                const v4s va = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)pa);
                const v4s vb = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(pa + 8 * 128));
                vv[db][0] = va[0]; vv[db][1] = va[1]; vv[db][2] = va[2]; vv[db][3] = va[3];
                vv[db][4] = vb[0]; vv[db][5] = vb[1]; vv[db][6] = vb[2]; vv[db][7] = vb[3];
            }
        };
        auto iter = [&](auto next_c, const char* slot, const char* nslot, int t) {
            constexpr int NEXT = decltype(next_c)::value;
            // PIPE (inference, full next tile): the in-wave software pipeline pinned by sched_barrier
            // fences.  Left to itself hipcc sank tile t+1's QK^T MFMAs below tile t's P.V (ISA of
            // round 2's build): the 8 QK^T MFMAs ran back to back with this wave's VALU idle, and the
            // 32 exp2 stalled the P.V MFMAs that consume them.  Phase A: per k-step the next k-step's
            // K fragments (after the last one: the first 16-key step's V^T), then tile t+1's two QK^T
            // MFMAs with 3 exp2 of tile t in each one's shadow (8 + 3 x 8 issue cycles ~ one 32-cycle
            // MFMA); phase B: per 16-key step the next step's V^T reads, P.V (2) + row sum (1), then
            // the next step's 4 P packs.  Bit-identical; ViViT-B B = 8 247.8 -> 244.2 us, B = 4
            // 133.9 -> 129.7 us per launch (tools/ab_attn.py, interleaved in one process, round 3;
            // fences around every MFMA as well: 245.1 / 129.0, not kept).
            // NEXT = 3: a main-loop iteration whose staging (tile t+3), retire count and barrier are known to
            // be needed: no runtime tests (their scalar compares and branches, ~5 per tile, leave the loop)
            constexpr bool FULLNEXT = NEXT == 0 || NEXT == 3;
            constexpr bool PIPE = !RB && FULLNEXT && QB == 1;
            if constexpr (NEXT == 3) stage(t + NS - 1);
            else if (t + NS - 1 < ntiles) stage(t + NS - 1);
            v16f snext[QB][2];
            v8s vcur[2], vnxt[2];  // PIPE: V^T fragments (d-blocks 0 / 1) of the current / next 16-key step
            if constexpr (PIPE) {
                // exp2 of tile t's scores in 16-key-step order (step g = regs 8 (g & 1) .. of key block
                // g >> 1), so step g's P can be packed as soon as its 8 exp2 are done
                auto ex = [&](int i) {
                    if (i < VC_ATTN_SWEXP) scur[0][i >> 4][i & 15] = sw_exp2(scur[0][i >> 4][i & 15]);
                    else scur[0][i >> 4][i & 15] = __builtin_amdgcn_exp2f(scur[0][i >> 4][i & 15]);
                };
                v8s ka = *reinterpret_cast<const v8s*>(nslot + koff[0]);
                v8s kb = *reinterpret_cast<const v8s*>(nslot + koff[0] + 4096);
                ex(0); ex(1); ex(2); ex(3);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) {
                    v8s na, nb;
                    if (kk < 3) {
                        na = *reinterpret_cast<const v8s*>(nslot + koff[kk + 1]);
                        nb = *reinterpret_cast<const v8s*>(nslot + koff[kk + 1] + 4096);
                    } else {
                        vread(slot, 0, vcur);
                    }
                    snext[0][0] = mfma32x16<ET>(ka, qf[0][kk], kk == 0 ? minit[0] : snext[0][0]);
                    ex(4 + 6 * kk); ex(5 + 6 * kk); ex(6 + 6 * kk);
                    snext[0][1] = mfma32x16<ET>(kb, qf[0][kk], kk == 0 ? minit[0] : snext[0][1]);
                    ex(7 + 6 * kk); ex(8 + 6 * kk); ex(9 + 6 * kk);
                    ka = na;
                    kb = nb;
                    __builtin_amdgcn_sched_barrier(0);
                }
                ex(28); ex(29); ex(30); ex(31);
            } else if constexpr (FULLNEXT) {
                qk_mfma(nslot, snext);
            } else if constexpr (NEXT == 1) {
                qk(nslot, t + 1, snext);
            }

            // ---- online softmax: scores are relative to the running max already
            if constexpr (PIPE) {
                // exp2 done in phase A; the training forward's f32 row sums and grown-max check follow
                if constexpr (WLSE) {
                    v2f ps[QB];
                    psum(scur, ps);
                    if (__any(!(ps[0][0] + ps[0][1] <= LIM))) {
                        qk(slot, t, scur);
                        rebase(next_c, scur, snext);
                        exp_all(scur);
                        psum(scur, ps);
                    }
                    l_run[0] += ps[0];
                }
            } else if constexpr (WLSE) {
                // deferred max: every P is >= 0, so a partial row sum <= LIM bounds every P of
                // the tile by LIM (an overflow shows up as inf); only when it fails is tile t
                // recomputed against an exact re-based max
                v2f ps[QB];
                exp_all(scur);
                psum(scur, ps);
                bool grow = RB;
#pragma unroll
                for (int qb = 0; qb < QB; ++qb) grow = grow || !(ps[qb][0] + ps[qb][1] <= LIM);
                if (__any(grow)) {
                    qk(slot, t, scur);
                    rebase(next_c, scur, snext);
                    exp_all(scur);
                    psum(scur, ps);
                }
#pragma unroll
                for (int qb = 0; qb < QB; ++qb) l_run[qb] += ps[qb];
            } else {
                if constexpr (RB) rebase(next_c, scur, snext);
                exp_all(scur);
            }

            // ---- O^T += V^T . P^T: P fragment of (key block kb, k-step s2) = regs 8s2..8s2+7;
            //      every V^T fragment read from LDS feeds QB MFMAs; inference also feeds the
            //      fragment to the row-sum MFMA
            const bool pv_kb1 = NEXT != 2 || t * AK + 32 < S;
            if constexpr (PIPE) {
                // 16-key step g: step g + 1's V^T reads, then step g's P.V (2) and row-sum MFMAs, then
                // step g + 1's P packs (in the MFMAs' shadow); one scheduling group per step
                auto pack = [&](int g) {
                    v4u pu;
#pragma unroll
                    for (int jj = 0; jj < 4; ++jj)
                        pu[jj] = pack2<ET>(scur[0][g >> 1][8 * (g & 1) + 2 * jj], scur[0][g >> 1][8 * (g & 1) + 2 * jj + 1]);
                    return __builtin_bit_cast(v8s, pu);
                };
                v8s pf = pack(0);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    if (g < 3) vread(slot, g + 1, vnxt);
                    o[0][0] = mfma32x16<ET>(vcur[0], pf, o[0][0]);
                    o[0][1] = mfma32x16<ET>(vcur[1], pf, o[0][1]);
                    if constexpr (!WLSE) lsum[0] = mfma16x32<ET>(sel, pf, lsum[0]);
                    if (g < 3) {
                        pf = pack(g + 1);
                        vcur[0] = vnxt[0];
                        vcur[1] = vnxt[1];
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
            } else
#pragma unroll
            for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) {
                    if (kb == 1 && !pv_kb1) continue;
                    v8s pf[QB];
#pragma unroll
                    for (int qb = 0; qb < QB; ++qb) {
                        v4u pu;
#pragma unroll
                        for (int jj = 0; jj < 4; ++jj)
                            pu[jj] = pack2<ET>(scur[qb][kb][8 * s2 + 2 * jj], scur[qb][kb][8 * s2 + 2 * jj + 1]);
                        pf[qb] = __builtin_bit_cast(v8s, pu);
                    }
#pragma unroll
                    for (int db = 0; db < 2; ++db) {
                        const char* pa = slot + voff[db] + (kb * 32 + 16 * s2) * 128;
                        v4s va = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)pa);
                        v4s vb = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(pa + 8 * 128));
                        v8s vv;
                        vv[0] = va[0]; vv[1] = va[1]; vv[2] = va[2]; vv[3] = va[3];
                        vv[4] = vb[0]; vv[5] = vb[1]; vv[6] = vb[2]; vv[7] = vb[3];
#pragma unroll
                        for (int qb = 0; qb < QB; ++qb) o[qb][db] = mfma32x16<ET>(vv, pf[qb], o[qb][db]);
                    }
                    if constexpr (!WLSE) {
#pragma unroll
                        for (int qb = 0; qb < QB; ++qb) lsum[qb] = mfma16x32<ET>(sel, pf[qb], lsum[qb]);
                    }
                }

            // ---- tile t+2 must be resident for the next iteration's K read (t+3 may stay in
            //      flight); the barrier also retires every wave's reads of slot t before the
            //      next iteration stages t+4 into it
            if constexpr (NEXT == 3) {
                attn_wait_vm<4>();
                attn_sync();
            } else if (t + 2 < ntiles) {
                if (t + 3 < ntiles) attn_wait_vm<4>();
                else attn_wait_vm<0>();
                attn_sync();
            }
            if constexpr (NEXT != 2) {
#pragma unroll
                for (int qb = 0; qb < QB; ++qb) { scur[qb][0] = snext[qb][0]; scur[qb][1] = snext[qb][1]; }
            }
        };

        using full_c = std::integral_constant<int, 0>;
        using fast_c = std::integral_constant<int, 3>;
        const int nfull = S / AK;  // full tiles
        int t = 0;
        // iterations t..t+3 all have a full next tile and stage tile (t+3)+3 < ntiles with tile (t+3)+3 in
        // flight: no runtime tests inside
        for (; t + 5 <= nfull && t + 6 < ntiles; t += NS) {
            iter(fast_c{}, smem + 0 * KV_SLOT, smem + 1 * KV_SLOT, t);
            iter(fast_c{}, smem + 1 * KV_SLOT, smem + 2 * KV_SLOT, t + 1);
            iter(fast_c{}, smem + 2 * KV_SLOT, smem + 3 * KV_SLOT, t + 2);
            iter(fast_c{}, smem + 3 * KV_SLOT, smem + 0 * KV_SLOT, t + 3);
        }
        for (; t + 5 <= nfull; t += NS) {  // iterations t..t+3 all have a full next tile
            iter(full_c{}, smem + 0 * KV_SLOT, smem + 1 * KV_SLOT, t);
            iter(full_c{}, smem + 1 * KV_SLOT, smem + 2 * KV_SLOT, t + 1);
            iter(full_c{}, smem + 2 * KV_SLOT, smem + 3 * KV_SLOT, t + 2);
            iter(full_c{}, smem + 3 * KV_SLOT, smem + 0 * KV_SLOT, t + 3);
        }
        for (; t < ntiles; ++t) {  // at most NS + 1 iterations: runtime slot, mask-checked next tile
            const char* slot = smem + (t % NS) * KV_SLOT;
            const char* nslot = smem + ((t + 1) % NS) * KV_SLOT;
            if (t + 1 < ntiles) iter(std::integral_constant<int, 1>{}, slot, nslot, t);
            else iter(std::integral_constant<int, 2>{}, slot, nslot, t);
        }
    };

    // total row sum of this lane's query
    auto row_total = [&](int qb) {
        if constexpr (WLSE) {
            const float l_own = l_run[qb][0] + l_run[qb][1];
            return l_own + __shfl_xor(l_own, 32, 64);
        } else {
            // query r's row sum sits in lane (r & 15) + 32 (r >> 4)
            return __shfl(lsum[qb][0], (r & 15) + ((r >> 4) << 5), 64);
        }
    };

    if constexpr (WLSE || REBASE_ALWAYS) {
        pass(std::integral_constant<bool, REBASE_ALWAYS>{});
    } else {
        pass(std::false_type{});
        // a row sum above 2^64 (some score ~50 or more above tile 0's max, before any P can
        // overflow at 128) or non-finite (inf / NaN input): the whole workgroup repeats the
        // pass re-basing on every tile.  Every
        // tile staged by the first pass was retired inside it, so the ring is free.
        bool bad = false;
#pragma unroll
        for (int qb = 0; qb < QB; ++qb) bad = bad || !(row_total(qb) <= 0x1p64f);
        if (__syncthreads_or(bad)) pass(std::true_type{});
    }

    // ---- normalise and store O[q][d]: reg 4g+e of block db -> d = 32db + 8g + 4h + e;
    //      lane pairs (h=0/1) swap halves so each lane stores 16 contiguous bytes
#pragma unroll
    for (int qb = 0; qb < QB; ++qb) {
        const int q = qblk * AQ + (wave * QB + qb) * 32 + r;
        const int qc = q < S ? q : S - 1;
        const float l_tot = row_total(qb);
        const float inv = 1.0f / l_tot;
        if constexpr (WLSE) {
            if (h == 0 && q < S) lse[(int64_t)bh * S + q] = -minit[qb][0] + __log2f(l_tot);
        }
        unsigned pk[2][4][2];
#pragma unroll
        for (int db = 0; db < 2; ++db)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                pk[db][g][0] = pack2<ET>(o[qb][db][4 * g + 0] * inv, o[qb][db][4 * g + 1] * inv);
                pk[db][g][1] = pack2<ET>(o[qb][db][4 * g + 2] * inv, o[qb][db][4 * g + 3] * inv);
            }
        uint16_t* orow = out + (tok0 + qc) * ldo + hh * 64;
#pragma unroll
        for (int db = 0; db < 2; ++db)
#pragma unroll
            for (int g = 0; g < 4; g += 2) {
                auto x0 = __builtin_amdgcn_permlane32_swap(pk[db][g][0], pk[db][g + 1][0], false, false);
                auto x1 = __builtin_amdgcn_permlane32_swap(pk[db][g][1], pk[db][g + 1][1], false, false);
                uint4 v;
                v.x = x0[0]; v.y = x1[0]; v.z = x0[1]; v.w = x1[1];
                if (q < S) *reinterpret_cast<uint4*>(orow + db * 32 + g * 8 + h * 8) = v;
            }
    }
}

template <bool REBASE_ALWAYS, bool WLSE, int ET = VC_ELEM_BF16>
static void launch_attn(const uint16_t* qkv, int64_t ld, int64_t B, int64_t S, int64_t H, float c_log2, uint16_t* out,
                        int64_t ldo, hipStream_t stream, float* lse = nullptr) {
    dim3 grid((unsigned)((S + 127) / 128), (unsigned)(B * H));
    attn_fwd_d64_kernel<REBASE_ALWAYS, WLSE, ET><<<grid, 256, NSLOT * KV_SLOT, stream>>>(qkv, ld, (int)S, (int)H, c_log2,
                                                                                   out, ldo, lse);
}

// attention_short.hip: one workgroup per (sequence, head) with all keys in LDS, for S <= 256
int launch_attn_short(const uint16_t* qkv, int64_t ld, int64_t B, int64_t S, int64_t H, float c_log2, uint16_t* out,
                      int64_t ldo, int elem, hipStream_t stream);
constexpr int64_t SHORT_MAX_S = 256;

}  // namespace vc

using namespace vc;

static int attn_checks(const uint16_t* qkv, int64_t ld, int64_t B, int64_t S, int64_t H, int64_t head_dim,
                       const uint16_t* out, int64_t ldo) {
    if (!qkv || !out) return fail(VC_ERR_INVALID_ARG, "vc_attention_fwd: null pointer");
    if (head_dim != 64) return fail(VC_ERR_UNSUPPORTED, "vc_attention_fwd: head_dim must be 64");
    if (B <= 0 || S <= 0 || H <= 0 || ld < 3 * H * 64 || ldo < H * 64 || ld % 8 || ldo % 8)
        return fail(VC_ERR_INVALID_ARG, "vc_attention_fwd: bad shape / leading dimension");
    if ((((uintptr_t)qkv) | ((uintptr_t)out)) & 15)
        return fail(VC_ERR_INVALID_ARG, "vc_attention_fwd: pointers must be 16-byte aligned");
    if (B * H > 65535 || S > (1 << 24)) return fail(VC_ERR_INVALID_ARG, "vc_attention_fwd: grid too large");
    return 0;
}

extern "C" int vc_attention_fwd(const uint16_t* qkv, int64_t ld, int64_t B, int64_t S, int64_t H, int64_t head_dim,
                                float scale, int q_prescaled, uint16_t* out, int64_t ldo, hipStream_t stream) {
    if (int rc = attn_checks(qkv, ld, B, S, H, head_dim, out, ldo)) return rc;
    const float c_log2 = q_prescaled ? 1.0f : scale * 1.4426950408889634f;
    if (S <= SHORT_MAX_S) return launch_attn_short(qkv, ld, B, S, H, c_log2, out, ldo, VC_ELEM_BF16, stream);
    launch_attn<false, false>(qkv, ld, B, S, H, c_log2, out, ldo, stream);
    return check_launch("vc_attention_fwd");
}

// vc_attention_fwd with the 16-bit operand type as an argument (fp16: the inference forward's
// higher-precision build, same kernel and MFMA rate).
extern "C" int vc_attention_fwd_h16(const uint16_t* qkv, int64_t ld, int64_t B, int64_t S, int64_t H,
                                    int64_t head_dim, float scale, int q_prescaled, int elem, uint16_t* out,
                                    int64_t ldo, hipStream_t stream) {
    if (int rc = attn_checks(qkv, ld, B, S, H, head_dim, out, ldo)) return rc;
    const float c_log2 = q_prescaled ? 1.0f : scale * 1.4426950408889634f;
    if (S <= SHORT_MAX_S && (elem == VC_ELEM_F16 || elem == VC_ELEM_BF16))
        return launch_attn_short(qkv, ld, B, S, H, c_log2, out, ldo, elem, stream);
    if (elem == VC_ELEM_F16) launch_attn<false, false, VC_ELEM_F16>(qkv, ld, B, S, H, c_log2, out, ldo, stream);
    else if (elem == VC_ELEM_BF16) launch_attn<false, false>(qkv, ld, B, S, H, c_log2, out, ldo, stream);
    else return fail(VC_ERR_INVALID_ARG, "vc_attention_fwd_h16: bad elem");
    return check_launch("vc_attention_fwd_h16");
}

// Training forward: vc_attention_fwd plus the base-2 log-sum-exp per (clip, head, query).
extern "C" int vc_attention_fwd_lse(const uint16_t* qkv, int64_t ld, int64_t B, int64_t S, int64_t H, int64_t head_dim,
                                    float scale, int q_prescaled, uint16_t* out, int64_t ldo, float* lse,
                                    hipStream_t stream) {
    if (int rc = attn_checks(qkv, ld, B, S, H, head_dim, out, ldo)) return rc;
    if (!lse) return fail(VC_ERR_INVALID_ARG, "vc_attention_fwd_lse: null lse");
    const float c_log2 = q_prescaled ? 1.0f : scale * 1.4426950408889634f;
    launch_attn<false, true>(qkv, ld, B, S, H, c_log2, out, ldo, stream, lse);
    return check_launch("vc_attention_fwd_lse");
}

// Test build of the defer-max threshold (cdna_hip_programming.md rule 26): re-base the running
// max on EVERY tile (LIM = 0).  Must agree with vc_attention_fwd to rounding.
extern "C" int vc_attention_fwd_rebase_always(const uint16_t* qkv, int64_t ld, int64_t B, int64_t S, int64_t H,
                                              float scale, uint16_t* out, int64_t ldo, hipStream_t stream) {
    if (int rc = attn_checks(qkv, ld, B, S, H, 64, out, ldo)) return rc;
    launch_attn<true, false>(qkv, ld, B, S, H, scale * 1.4426950408889634f, out, ldo, stream);
    return check_launch("vc_attention_fwd_rebase_always");
}
