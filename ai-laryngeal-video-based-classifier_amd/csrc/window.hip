// Video Swin 3D shifted-window attention, head_dim 32, bf16 MFMA.
//
// Replaces torchvision's ShiftedWindowAttention3d core (shifted_window_attention_3d: roll,
// window partition, q.k^T * d^-1/2 + relative-position bias (+ -100 between shift regions),
// softmax, .v, window reverse, roll back — as called by the reference's swin3d_t,
// videoswintransformer/swin_video_classifier/models/swin3d.py:24-26).
//
// No data moves for the roll / partition / reverse: the window token n of window
// (wt_i, wh_i, ww_i) at rolled grid position (wt_i*Wt + i, ...) is the token at original
// position ((wt_i*Wt + i + st) mod T, ...), so the kernel gathers its q|k|v rows by index
// from the projection output (token layout [B][T][H][W]) and scatters the output rows back
// to the same positions, where the proj GEMM + residual run per token.
//
// One workgroup = 4 waves = one (window, head).  The window's K and V (vol <= 448 tokens x
// 32 dims, bf16) are staged once into LDS (57 KB, 2 workgroups per CU); each wave walks
// 32-query blocks: S^T = K.Q'^T with the bias tile as the MFMA C operand (pre-scaled by
// log2 e like Q', -inf on padded keys; stored in fragment order so each lane's 16 values
// are one contiguous 64-B read, prefetched a tile ahead), the shift-region mask as -inf
// (torchvision adds -100: exp(-100) ~ 4e-44 is below fp32 resolution of the row sum, so the
// results agree), online softmax in exp2, O^T += V^T.P^T with V^T from ds_read_b64_tr_b16.
#include "window_common.hpp"

#include <cstdlib>
#include <type_traits>

namespace vc {

constexpr int WNP_MAX = 448;  // max padded window volume (8*7*7 = 392 -> 448)

// Softmax, inference: scores are exponentiated as they come (the bias occupies the QK^T C
// operand, so a running max would cost a subtraction per score) and the row sums run on the
// matrix pipe (attention.hip's selector MFMA over the P.V operand); a row sum outside
// [2^-64, 2^64] (overflow, underflow, inf / NaN) makes the wave repeat the query block with the
// ViViT kernel's deferred running max: scores relative to a max m fixed by the first key tile,
// f32 VALU row sums, m re-based when a lane's partial row sum exceeds LIM (O and l scaled by
// 2^-delta).  The training forward (WLSE) uses the max-free pass with f32 VALU sums.  Measured
// on Swin-T B=4 (round 2, process-level A/B): 2.915 -> 2.880 ms per forward (+1.2 %).  Round 1:
// the deferred max was 1-5 % faster per launch than a per-tile max.  Where the rest goes: the fragment-order f32 bias
// stream (784 KB per (window, head) workgroup, one tile of prefetch) costs 15-20 %; the
// shift-region mask +15-25 % on the shifted blocks; stages 3-4 fill only 384 / 192 of the 512
// workgroup slots (splitting a pair's query blocks over more workgroups measured slower: each
// re-stages the window's K/V); 13 query blocks over 4 waves leave one wave a block longer.
// WLSE (train step): also store each query's base-2 log-sum-exp lse[row * heads + head] = m +
// log2(l) (row = global token row), from which window_bwd.hip recomputes P.
constexpr float WLIM = 256.0f;

template <bool WLSE>
__global__ void __launch_bounds__(256, 2)
window_attn_d32_kernel(const uint16_t* __restrict__ qkv, int64_t ld, WinGeom g, int heads, int vol, int NP,
                       const float* __restrict__ biasF, int masked, uint16_t* __restrict__ out, int64_t ldo,
                       float* __restrict__ lse) {
    __shared__ __attribute__((aligned(16))) char kv[2 * WNP_MAX * 64];
    __shared__ unsigned lab4[WNP_MAX / 8];  // 4-bit region code per window token (15: padding)

    const int head = blockIdx.y;
    const int nwin = g.nwt * g.nwh * g.nww;
    const int b = blockIdx.x / nwin;
    int r = blockIdx.x - b * nwin;
    const int wi_t = r / (g.nwh * g.nww);
    r -= wi_t * g.nwh * g.nww;
    const int wi_h = r / g.nww, wi_w = r - (r / g.nww) * g.nww;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int C = heads * 32;

    auto token_row = [&](int n, int* label) -> int64_t { return win_token_row(g, b, wi_t, wi_h, wi_w, n, label); };

    // ---- stage K (swizzled 16-B chunks) and V (plain 64-B rows) of this window/head in LDS
    char* Ks = kv;
    char* Vs = kv + WNP_MAX * 64;
    for (int c = tid; c < NP * 4; c += 256) {
        const int n = c >> 2, ch = c & 3;
        uint4 kval = make_uint4(0, 0, 0, 0), vval = make_uint4(0, 0, 0, 0);
        if (n < vol) {
            const int64_t row = token_row(n, nullptr);
            const uint16_t* src = qkv + row * ld + head * 32 + ch * 8;
            kval = *reinterpret_cast<const uint4*>(src + C);
            vval = *reinterpret_cast<const uint4*>(src + 2 * C);
        }
        *reinterpret_cast<uint4*>(Ks + n * 64 + kchunk_swz(n, ch) * 16) = kval;
        *reinterpret_cast<uint4*>(Vs + n * 64 + ch * 16) = vval;
    }
    // the shift mask only matters in windows whose tokens span several shift regions (the last
    // window along a shifted dimension); elsewhere every label is equal and the mask is skipped
    // (padded keys are -inf through the bias either way)
    int diff = 0;
    if (masked) {
        int lb0 = 0;
        token_row(0, &lb0);
        for (int w8 = tid; w8 < NP / 8; w8 += 256) {
            unsigned v = 0;
            for (int e = 0; e < 8; ++e) {
                int lb = 15;
                if (w8 * 8 + e < vol) {
                    token_row(w8 * 8 + e, &lb);
                    diff |= lb != lb0;
                }
                v |= (unsigned)lb << (4 * e);
            }
            lab4[w8] = v;
        }
    }
    const bool mixed = __syncthreads_or(diff) != 0;

    const int rr = lane & 31, h = lane >> 5;
    // per-lane LDS offsets: K fragment (key rr of a 32-key block, 16-B chunk 2kk+h)
    int koff[2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) koff[kk] = rr * 64 + kchunk_swz(rr, 2 * kk + h) * 16;
    // V^T transpose read: rows 4h + tq (+8), columns gcol..gcol+3
    const int gi = lane & 15;
    const int tq = gi >> 2, tp = gi & 3;
    const int gcol = ((lane >> 4) & 1) * 16 + tp * 4;
    const int voff = (4 * h + tq) * 64 + gcol * 2;
    const int nqb = (vol + 31) / 32;
    const int ntile = NP / 64;
    // bias fragments: biasF[head][qb][t][kb][lane][16] f32 = this lane's 16 C-operand values
    const float* bh = biasF + (int64_t)head * (NP / 32) * ntile * 2 * 64 * 16 + lane * 16;
    auto load_bias = [&](int qb, int t, v16f (&c)[2]) {
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
            const float4* bp = reinterpret_cast<const float4*>(bh + (((int64_t)qb * ntile + t) * 2 + kb) * 64 * 16);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float4 u = bp[j];
                c[kb][4 * j] = u.x; c[kb][4 * j + 1] = u.y; c[kb][4 * j + 2] = u.z; c[kb][4 * j + 3] = u.w;
            }
        }
    };

    // 0/1 selector A operand of the row-sum MFMA: Sel[i][k] = 1 when k-group parity == i >> 3
    v8bf sel;
    {
        const __bf16 v = (((lane >> 4) & 1) == ((lane & 15) >> 3)) ? (__bf16)1.0f : (__bf16)0.0f;
#pragma unroll
        for (int j = 0; j < 8; ++j) sel[j] = v;
    }
    // query blocks of this (window, head) are dealt over the 4 waves
    for (int qb = wave; qb < nqb; qb += 4) {
        const int qn = qb * 32 + rr;  // this lane's query (window-local)
        const int qc = qn < vol ? qn : vol - 1;
        int qlab = 0;
        const int64_t qrow = token_row(qc, masked ? &qlab : nullptr);
        v8bf qf[2];
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
            qf[kk] = __builtin_bit_cast(v8bf, *reinterpret_cast<const v8s*>(qkv + qrow * ld + head * 32 + 16 * kk + 8 * h));
        v16f o;
        float m_run, l_run;
        // SAFE = false: scores are used as they come (no running max, no per-score subtraction):
        // exp2 of a bf16-range score is exact in relative terms until it overflows (a score above
        // ~127 in log2 units) or every key of the row underflows; a row sum outside
        // [2^-64, 2^64] (or inf / NaN) makes this wave repeat the query block with SAFE = true,
        // the deferred running max fixed by tile 0 and re-based when a partial row sum exceeds
        // WLIM.  Both passes are wave-local (K / V stay in LDS for the whole window).
        auto attend = [&](auto safe_c) {
            constexpr bool SAFE = decltype(safe_c)::value;
            // fast inference pass: row sums on the matrix pipe (attention.hip's selector MFMA over
            // the P.V operand; lane l ends with the sum of query (l & 15) + 16 (l >> 5)); the
            // exact pass and the training forward keep f32 VALU sums
            constexpr bool MSUM = !SAFE && !WLSE;
            o = v16f{};
            m_run = SAFE ? -1e30f : 0.f;
            v4f lsum = {0.f, 0.f, 0.f, 0.f};
            v16f bnext[2];
            load_bias(qb, 0, bnext);
            // (bias fragments two tiles ahead instead of one: 238 VGPRs, 2 % slower per forward)
            v2f l2 = {0.f, 0.f};
            for (int t = 0; t < ntile; ++t) {
                v16f sc[2] = {bnext[0], bnext[1]};
                if (t + 1 < ntile) load_bias(qb, t + 1, bnext);
#pragma unroll
                for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
                    for (int kb = 0; kb < 2; ++kb) {
                        const v8bf kf = __builtin_bit_cast(v8bf, *reinterpret_cast<const v8s*>(Ks + (t * 64 + kb * 32) * 64 + koff[kk]));
                        sc[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[kk], sc[kb], 0, 0, 0);
                    }
                }
                if (mixed) {
#pragma unroll
                    for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
                        for (int g4 = 0; g4 < 4; ++g4) {
                            const int k0 = t * 64 + kb * 32 + 8 * g4 + 4 * h;
                            const unsigned wv = lab4[k0 >> 3] >> (4 * (k0 & 7));
#pragma unroll
                            for (int e = 0; e < 4; ++e)
                                if ((int)((wv >> (4 * e)) & 15) != qlab) sc[kb][4 * g4 + e] = -INFINITY;
                        }
                    }
                }
                auto rowmax = [&]() {
                    float a = fmaxf(sc[0][0], sc[1][0]), c = fmaxf(sc[0][1], sc[1][1]);
#pragma unroll
                    for (int e = 2; e < 16; e += 2) {
                        a = fmaxf(a, fmaxf(sc[0][e], sc[1][e]));
                        c = fmaxf(c, fmaxf(sc[0][e + 1], sc[1][e + 1]));
                    }
                    const float x = fmaxf(a, c);
                    return fmaxf(x, __shfl_xor(x, 32, 64));
                };
                if constexpr (SAFE) {
                    if (t == 0) m_run = fmaxf(rowmax(), -1e30f);  // first tile fixes m (fully masked rows: -1e30)
                }
                v16f p[2];
                auto expsum = [&]() {
#pragma unroll
                    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                        for (int e = 0; e < 16; ++e) p[kb][e] = __builtin_amdgcn_exp2f(SAFE ? sc[kb][e] - m_run : sc[kb][e]);
                    v2f u[8];
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        u[j] = v2f{p[0][4 * j], p[0][4 * j + 1]} + v2f{p[0][4 * j + 2], p[0][4 * j + 3]};
                        u[4 + j] = v2f{p[1][4 * j], p[1][4 * j + 1]} + v2f{p[1][4 * j + 2], p[1][4 * j + 3]};
                    }
                    return ((u[0] + u[1]) + (u[2] + u[3])) + ((u[4] + u[5]) + (u[6] + u[7]));
                };
                v2f ps = {0.f, 0.f};
                if constexpr (MSUM) {
#pragma unroll
                    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                        for (int e = 0; e < 16; ++e) p[kb][e] = __builtin_amdgcn_exp2f(sc[kb][e]);
                } else {
                    ps = expsum();
                }
                if (SAFE && __any(!(ps[0] + ps[1] <= WLIM))) {  // rare: re-base m on this tile's exact max
                    const float delta = fmaxf(rowmax() - m_run, 0.f);
                    const float alpha = __builtin_amdgcn_exp2f(-delta);
                    m_run += delta;
#pragma unroll
                    for (int e = 0; e < 16; ++e) o[e] *= alpha;
                    l2 *= alpha;
                    ps = expsum();
                }
                l2 += ps;
#pragma unroll
                for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                    for (int s2 = 0; s2 < 2; ++s2) {
                        v4u pu;
#pragma unroll
                        for (int jj = 0; jj < 4; ++jj) pu[jj] = pack2bf(p[kb][8 * s2 + 2 * jj], p[kb][8 * s2 + 2 * jj + 1]);
                        const v8bf pf = __builtin_bit_cast(v8bf, pu);
                        const char* pa = Vs + (t * 64 + kb * 32 + 16 * s2) * 64 + voff;
                        const v4s va = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)pa);
                        const v4s vb = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(pa + 8 * 64));
                        v8s vv;
                        vv[0] = va[0]; vv[1] = va[1]; vv[2] = va[2]; vv[3] = va[3];
                        vv[4] = vb[0]; vv[5] = vb[1]; vv[6] = vb[2]; vv[7] = vb[3];
                        o = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(v8bf, vv), pf, o, 0, 0, 0);
                        if constexpr (MSUM) lsum = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sel, pf, lsum, 0, 0, 0);
                    }
            }
            if constexpr (MSUM) {
                // this lane's half of query rr's sum (the caller adds the h = 1 half): the whole
                // sum sits in lane (rr & 15) + 32 (rr >> 4); halve it for the two lane halves
                l_run = 0.5f * __shfl(lsum[0], (rr & 15) + ((rr >> 4) << 5), 64);
            } else {
                l_run = l2[0] + l2[1];
            }
        };
        attend(std::false_type{});
        {
            const float lt = l_run + __shfl_xor(l_run, 32, 64);
            if (__any(!(lt >= 0x1p-64f && lt <= 0x1p64f))) attend(std::true_type{});
        }

        // ---- O^T[d][q]: reg 4g+e -> d = 8g + 4h + e; lane pairs swap halves -> 16-B stores
        const float l_tot = l_run + __shfl_xor(l_run, 32, 64);
        const float inv = 1.0f / l_tot;
        if constexpr (WLSE) {
            if (h == 0 && qn < vol) lse[qrow * heads + head] = m_run + __log2f(l_tot);
        }
        unsigned pk[4][2];
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
            pk[g4][0] = pack2bf(o[4 * g4 + 0] * inv, o[4 * g4 + 1] * inv);
            pk[g4][1] = pack2bf(o[4 * g4 + 2] * inv, o[4 * g4 + 3] * inv);
        }
        uint16_t* orow = out + qrow * ldo + head * 32;
#pragma unroll
        for (int g4 = 0; g4 < 4; g4 += 2) {
            auto x0 = __builtin_amdgcn_permlane32_swap(pk[g4][0], pk[g4 + 1][0], false, false);
            auto x1 = __builtin_amdgcn_permlane32_swap(pk[g4][1], pk[g4 + 1][1], false, false);
            uint4 v;
            v.x = x0[0]; v.y = x1[0]; v.z = x0[1]; v.w = x1[1];
            if (qn < vol) *reinterpret_cast<uint4*>(orow + g4 * 8 + h * 8) = v;
        }
    }
}

// ---------------------------------------------------------------------------------
// Inference kernel with the relative-position bias and the shift mask on the matrix pipe.
//
// The kernel above adds the bias as the QK^T MFMA's C operand: 16 f32 values per lane per 32-key
// block streamed from L2 (784 KB per (window, head) workgroup) and copied into the accumulators,
// and applies the shift mask as three VALU ops per score.  Timing ablations of that kernel on
// Swin-T B=4 (all 12 launches of a forward): 745 us; without the bias stream 525; without bias
// and mask 438.  Here both become MFMAs on operands the matrix pipe reads directly:
//   * bias: S^T += I . Bias^T, I the 32x32 identity as two 16-deep A fragments (constant per
//     lane), Bias^T the B operand: 8 fp16 per lane per 16 keys, a 16-B load (half the f32 bytes,
//     no register copies);
//   * shift mask (windows spanning several shift regions only): S^T += A_m . B_m with A_m[k] =
//     (one-hot of key k's 3-bit region code, 1) and B_m[q] = (2^14 x one-hot of query q's code,
//     -2^14): 0 where the codes agree and -2^14 elsewhere (exp2 -> 0, as torchvision's -100 and
//     the kernel above's -inf); the key rows (32 B each) are staged in LDS with K and V.
// The mask MFMA runs first and the bias second, both exact (products 0 / +-2^14 / one bias
// value), so an unmasked score is bias + q'.k accumulated as before; a padded key's bias is
// -2^14.  The bias operand is fp16 (v_mfma_f32_32x32x16_f16 beside the bf16 score MFMAs, one f32
// accumulator): 2^-12 relative rounding, 8x finer than bf16, at the same MFMA count -- at trained
// table magnitudes (|bias| ~ 5) ~2e-3 log2 units instead of ~1.4e-2.
// ---------------------------------------------------------------------------------
constexpr float WMB_BIG = 16384.0f;

__global__ void __launch_bounds__(256, 2)
window_attn_mb_d32_kernel(const uint16_t* __restrict__ qkv, int64_t ld, WinGeom g, int heads, int vol, int NP,
                          const uint16_t* __restrict__ biasB, int masked, uint16_t* __restrict__ out, int64_t ldo) {
    __shared__ __attribute__((aligned(16))) char kv[2 * WNP_MAX * 64];
    __shared__ __attribute__((aligned(16))) char kon[WNP_MAX * 32];  // per key: one-hot region code | (1, 0 x 7)

    // (window, head) of this workgroup: head pairs (2p, 2p + 1) outermost, so the workgroups in
    // flight share two heads' bias (the L2 working set stays ~2 x 364 KB at any head count); within
    // a pair, ids i and i + 8 are the two heads of one window, on the same XCD (id mod 8) and
    // dispatched together, so the 128-B line holding both heads' 64-B q / k / v slices of a token
    // is fetched into that XCD's L2 once
    const int nwin_all = (int)(gridDim.x / heads);
    int head, wlin;
    {
        const int id = blockIdx.x;
        const int pair_ids = 2 * nwin_all;
        const int full = (heads / 2) * pair_ids;
        if (id < full) {
            const int pr = id / pair_ids;
            const int rem = id - pr * pair_ids;
            const int full8 = (nwin_all / 8) * 16;
            int hh;
            if (rem < full8) {
                hh = (rem >> 3) & 1;
                wlin = (rem >> 4) * 8 + (rem & 7);
            } else {
                const int tail = nwin_all & 7, rem2 = rem - full8;
                hh = rem2 / tail;
                wlin = (nwin_all & ~7) + rem2 - hh * tail;
            }
            head = 2 * pr + hh;
        } else {  // odd head count: the last head alone
            head = heads - 1;
            wlin = id - full;
        }
    }
    const int nwin = g.nwt * g.nwh * g.nww;
    const int b = wlin / nwin;
    int r = wlin - b * nwin;
    const int wi_t = r / (g.nwh * g.nww);
    r -= wi_t * g.nwh * g.nww;
    const int wi_h = r / g.nww, wi_w = r - (r / g.nww) * g.nww;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int C = heads * 32;

    auto token_row = [&](int n, int* label) -> int64_t { return win_token_row(g, b, wi_t, wi_h, wi_w, n, label); };

    // ---- stage K (swizzled 16-B chunks) and V (plain 64-B rows) of this window/head in LDS
    char* Ks = kv;
    char* Vs = kv + WNP_MAX * 64;
    {
        // every load issued before the first LDS write (a rolled loop waited out one gather
        // latency per 256 chunks): <= 7 chunks of 16 B per thread at NP = 448
        constexpr int NCH = WNP_MAX * 4 / 256;
        uint4 kval[NCH], vval[NCH];
#pragma unroll
        for (int j = 0; j < NCH; ++j) {
            const int c = tid + 256 * j, n = c >> 2, ch = c & 3;
            kval[j] = make_uint4(0, 0, 0, 0);
            vval[j] = make_uint4(0, 0, 0, 0);
            if (n < vol) {
                const int64_t row = token_row(n, nullptr);
                const uint16_t* src = qkv + row * ld + head * 32 + ch * 8;
                kval[j] = *reinterpret_cast<const uint4*>(src + C);
                vval[j] = *reinterpret_cast<const uint4*>(src + 2 * C);
            }
        }
#pragma unroll
        for (int j = 0; j < NCH; ++j) {
            const int c = tid + 256 * j, n = c >> 2, ch = c & 3;
            if (n < NP) {
                *reinterpret_cast<uint4*>(Ks + n * 64 + kchunk_swz(n, ch) * 16) = kval[j];
                *reinterpret_cast<uint4*>(Vs + n * 64 + ch * 16) = vval[j];
            }
        }
    }
    // region codes: the mask matters only in windows whose tokens span several shift regions
    int diff = 0;
    if (masked) {
        int lb0 = 0;
        token_row(0, &lb0);
        for (int n = tid; n < NP; n += 256) {
            int lb = 15;  // padding key: no region (its bias is -2^14 anyway)
            if (n < vol) {
                token_row(n, &lb);
                diff |= lb != lb0;
            }
            unsigned w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
            for (int j = 0; j < 4; ++j) w[j] = (lb >> 1) == j ? 0x3F80u << (16 * (lb & 1)) : 0u;
            *reinterpret_cast<uint4*>(kon + n * 32) = make_uint4(w[0], w[1], w[2], w[3]);
            *reinterpret_cast<uint4*>(kon + n * 32 + 16) = make_uint4(0x3F80u, 0u, 0u, 0u);
        }
    }
    const bool mixed = __syncthreads_or(diff) != 0;

    const int rr = lane & 31, h = lane >> 5;
    int koff[2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) koff[kk] = rr * 64 + kchunk_swz(rr, 2 * kk + h) * 16;
    const int gi = lane & 15;
    const int tq = gi >> 2, tp = gi & 3;
    const int gcol = ((lane >> 4) & 1) * 16 + tp * 4;
    const int voff = (4 * h + tq) * 64 + gcol * 2;
    const int nqb = (vol + 31) / 32;
    const int ntile = NP / 64;

    // identity A fragments: lane (rr, h) of slice s holds I[rr][16s + 8h + m], m = 0..7
    v8s ident[2];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int m = 0; m < 8; ++m) ident[s2][m] = rr == 16 * s2 + 8 * h + m ? (short)0x3C00 : (short)0;  // fp16 1.0
    v8bf sel;
    {
        const __bf16 v = (((lane >> 4) & 1) == ((lane & 15) >> 3)) ? (__bf16)1.0f : (__bf16)0.0f;
#pragma unroll
        for (int j = 0; j < 8; ++j) sel[j] = v;
    }

    // this wave's query blocks qb = wave, wave + 4, ..: the next block's Q fragments and the next
    // tile's bias fragments (the next block's tile 0 across a block boundary) are loaded while the
    // current tile computes
    struct QBlock {
        v8bf qf[2];
        v8s qm;  // B operand of the mask MFMA: h = 0 lanes 2^14 x one-hot(code), h = 1 lanes (-2^14, 0 x 7)
        int64_t qrow;
    };
    auto load_qblock = [&](int qb, QBlock& Q) __attribute__((always_inline)) {
        const int qn = qb * 32 + rr;
        const int qc = qn < vol ? qn : vol - 1;
        int qlab = 0;
        Q.qrow = token_row(qc, masked ? &qlab : nullptr);
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
            Q.qf[kk] = __builtin_bit_cast(v8bf, *reinterpret_cast<const v8s*>(qkv + Q.qrow * ld + head * 32 + 16 * kk + 8 * h));
#pragma unroll
        for (int m = 0; m < 8; ++m)
            Q.qm[m] = h == 0 ? (m == qlab ? (short)0x4680 : (short)0) : (m == 0 ? (short)0xC680 : (short)0);
    };
    // bias fragments of (query block, tile): [t][kb][s] 1 KiB each (64 lanes x 16 B)
    // (a wave-uniform base in SGPRs + the lane's constant 16-B offset: no address VGPR that a later
    // instruction overwrites while the load is in flight)
    // bias fragments of (query block, tile): [t][kb][s] 1 KiB each (64 lanes x 16 B), from a
    // wave-uniform base
    auto load_bias = [&](int qb, int t, v8s (&bf)[4]) __attribute__((always_inline)) {
        typedef const __attribute__((address_space(1))) v8s gv8s;
        const uint64_t a = (uint64_t)(uintptr_t)(biasB + (((int64_t)head * (NP / 32) + qb) * ntile + t) * 4 * 512);
        // readfirstlane returns int: each half goes through uint32_t, or a low word with bit 31 set
        // would sign-extend over the high word
        const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32));
        gv8s* bq = reinterpret_cast<gv8s*>(((uint64_t)hi << 32) | (uint64_t)lo) + lane;
#pragma unroll
        for (int j = 0; j < 4; ++j) bf[j] = bq[j * 64];
    };
    // S'^T of 32 keys (key block kb of tile t): (mask) + bias + K . Q'^T
    auto scores_kb = [&](auto mixed_c, const QBlock& Q, int t, const v8s (&bf)[4], int kb) __attribute__((always_inline)) {
        constexpr bool MIXED = decltype(mixed_c)::value;
        v16f acc = v16f{};
        if constexpr (MIXED) {
            const v8s km = *reinterpret_cast<const v8s*>(kon + (t * 64 + kb * 32 + rr) * 32 + h * 16);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(v8bf, km), __builtin_bit_cast(v8bf, Q.qm),
                                                          acc, 0, 0, 0);
        }
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(v8h, ident[s2]),
                                                         __builtin_bit_cast(v8h, bf[kb * 2 + s2]), acc, 0, 0, 0);
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            const v8bf kf = __builtin_bit_cast(v8bf, *reinterpret_cast<const v8s*>(Ks + (t * 64 + kb * 32) * 64 + koff[kk]));
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, Q.qf[kk], acc, 0, 0, 0);
        }
        return acc;
    };
    // S'^T of 64 keys: (mask) + bias + K . Q'^T
    auto scores = [&](auto mixed_c, const QBlock& Q, int t, const v8s (&bf)[4], v16f (&sc)[2]) __attribute__((always_inline)) {
        constexpr bool MIXED = decltype(mixed_c)::value;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
            v16f acc = v16f{};
            if constexpr (MIXED) {
                const v8s km = *reinterpret_cast<const v8s*>(kon + (t * 64 + kb * 32 + rr) * 32 + h * 16);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(v8bf, km), __builtin_bit_cast(v8bf, Q.qm),
                                                              acc, 0, 0, 0);
            }
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2)
                acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(v8h, ident[s2]),
                                                             __builtin_bit_cast(v8h, bf[kb * 2 + s2]), acc, 0, 0, 0);
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) {
                const v8bf kf = __builtin_bit_cast(v8bf, *reinterpret_cast<const v8s*>(Ks + (t * 64 + kb * 32) * 64 + koff[kk]));
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, Q.qf[kk], acc, 0, 0, 0);
            }
            sc[kb] = acc;
        }
    };
    // O^T += V^T . P^T for one tile (P packed from p); row sums on the matrix pipe (lsum) or none
    // (the exact pass keeps f32 VALU sums)
    v16f o;
    auto pv = [&](int t, const v16f (&p)[2], v4f* lsum) __attribute__((always_inline)) {
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
                v4u pu;
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) pu[jj] = pack2bf(p[kb][8 * s2 + 2 * jj], p[kb][8 * s2 + 2 * jj + 1]);
                const v8bf pf = __builtin_bit_cast(v8bf, pu);
                const char* pa = Vs + (t * 64 + kb * 32 + 16 * s2) * 64 + voff;
                const v4s va = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)pa);
                const v4s vb = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(pa + 8 * 64));
                v8s vv;
                vv[0] = va[0]; vv[1] = va[1]; vv[2] = va[2]; vv[3] = va[3];
                vv[4] = vb[0]; vv[5] = vb[1]; vv[6] = vb[2]; vv[7] = vb[3];
                o = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(v8bf, vv), pf, o, 0, 0, 0);
                if (lsum) *lsum = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sel, pf, *lsum, 0, 0, 0);
            }
    };
    // the same for key block kb only (the fast pass's pipelined order; accumulation order unchanged)
    auto pv_kb = [&](int t, const v16f& p, int kb, v4f& lsum) __attribute__((always_inline)) {
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
            v4u pu;
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) pu[jj] = pack2bf(p[8 * s2 + 2 * jj], p[8 * s2 + 2 * jj + 1]);
            const v8bf pf = __builtin_bit_cast(v8bf, pu);
            const char* pa = Vs + (t * 64 + kb * 32 + 16 * s2) * 64 + voff;
            const v4s va = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)pa);
            const v4s vb = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(pa + 8 * 64));
            v8s vv;
            vv[0] = va[0]; vv[1] = va[1]; vv[2] = va[2]; vv[3] = va[3];
            vv[4] = vb[0]; vv[5] = vb[1]; vv[6] = vb[2]; vv[7] = vb[3];
            o = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(v8bf, vv), pf, o, 0, 0, 0);
            lsum = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sel, pf, lsum, 0, 0, 0);
        }
    };
    // exact pass of one block (rare: a row sum outside [2^-64, 2^64], inf / NaN): the deferred
    // running max fixed by tile 0, re-based on a tile's exact max when a lane's partial row sum
    // exceeds WLIM
    auto exact = [&](auto mixed_c, const QBlock& Q, int qb) __attribute__((always_inline)) {
        o = v16f{};
        float m_run = -1e30f;
        v2f l2 = {0.f, 0.f};
        for (int t = 0; t < ntile; ++t) {
            v8s bf[4];
            load_bias(qb, t, bf);
            v16f sc[2];
            scores(mixed_c, Q, t, bf, sc);
            auto rowmax = [&]() {
                float a = fmaxf(sc[0][0], sc[1][0]), c = fmaxf(sc[0][1], sc[1][1]);
#pragma unroll
                for (int e = 2; e < 16; e += 2) {
                    a = fmaxf(a, fmaxf(sc[0][e], sc[1][e]));
                    c = fmaxf(c, fmaxf(sc[0][e + 1], sc[1][e + 1]));
                }
                const float x = fmaxf(a, c);
                return fmaxf(x, __shfl_xor(x, 32, 64));
            };
            if (t == 0) m_run = fmaxf(rowmax(), -1e30f);
            v16f p[2];
            auto expsum = [&]() {
#pragma unroll
                for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                    for (int e = 0; e < 16; ++e) p[kb][e] = __builtin_amdgcn_exp2f(sc[kb][e] - m_run);
                v2f u[8];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    u[j] = v2f{p[0][4 * j], p[0][4 * j + 1]} + v2f{p[0][4 * j + 2], p[0][4 * j + 3]};
                    u[4 + j] = v2f{p[1][4 * j], p[1][4 * j + 1]} + v2f{p[1][4 * j + 2], p[1][4 * j + 3]};
                }
                return ((u[0] + u[1]) + (u[2] + u[3])) + ((u[4] + u[5]) + (u[6] + u[7]));
            };
            v2f ps = expsum();
            if (__any(!(ps[0] + ps[1] <= WLIM))) {
                const float delta = fmaxf(rowmax() - m_run, 0.f);
                const float alpha = __builtin_amdgcn_exp2f(-delta);
                m_run += delta;
#pragma unroll
                for (int e = 0; e < 16; ++e) o[e] *= alpha;
                l2 *= alpha;
                ps = expsum();
            }
            l2 += ps;
            pv(t, p, nullptr);
        }
        const float l_run = l2[0] + l2[1];
        return l_run + __shfl_xor(l_run, 32, 64);
    };
    // the wave's blocks: fast pass (scores exponentiated as they come, no running max, row sums on
    // the matrix pipe), the exact pass when a row sum leaves [2^-64, 2^64], 16-B output stores
    // Loads in flight are never carried across a loop back edge: the next tile's bias fragments
    // are issued at the top of a tile and moved into place at its bottom, the next block's Q at
    // the top of the block's last tile (a prefetch held across the tile loop, or left to the
    // scheduler, was waited for at the first MFMA of the next tile).
    // nt_c: the tile count as a compile-time constant (7: 392-token windows, every standard Swin
    // config; the loop unrolls fully and the bias hand-over is a rename, no copies) or 0 (any
    // window: rolled loop)
    auto run = [&](auto mixed_c, auto nt_c) __attribute__((always_inline)) {
        constexpr int NT = decltype(nt_c)::value;
        const int nt = NT ? NT : ntile;
        QBlock cur, nxt;
        v8s bcur[4], bnxt[4];
        if (wave >= nqb) return;
        load_qblock(wave, cur);
        load_bias(wave, 0, bcur);
        for (int qb = wave; qb < nqb; qb += 4) {
            const bool more = qb + 4 < nqb;
            o = v16f{};
            v4f lsum = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int t = 0; t < nt; ++t) {
                const bool last = t + 1 == nt;
                if (!last) load_bias(qb, t + 1, bnxt);
                else if (more) {
                    load_bias(qb + 4, 0, bnxt);
                    load_qblock(qb + 4, nxt);
                }
                __builtin_amdgcn_sched_barrier(0);
                // key block 1's score MFMAs run under key block 0's exp2, key block 0's P.V under
                // key block 1's exp2 (sched_barrier fences pin the groups; hipcc had issued every
                // score MFMA of the tile before the first exp2)
                v16f s0 = scores_kb(mixed_c, cur, t, bcur, 0);
                __builtin_amdgcn_sched_barrier(0);
                v16f s1 = scores_kb(mixed_c, cur, t, bcur, 1);
#pragma unroll
                for (int e = 0; e < 16; ++e) s0[e] = __builtin_amdgcn_exp2f(s0[e]);
                __builtin_amdgcn_sched_barrier(0);
                pv_kb(t, s0, 0, lsum);
#pragma unroll
                for (int e = 0; e < 16; ++e) s1[e] = __builtin_amdgcn_exp2f(s1[e]);
                __builtin_amdgcn_sched_barrier(0);
                pv_kb(t, s1, 1, lsum);
                if (!last || more) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) bcur[j] = bnxt[j];
                }
            }
            // query rr's sum sits in lane (rr & 15) + 32 (rr >> 4)
            float l_tot = __shfl(lsum[0], (rr & 15) + ((rr >> 4) << 5), 64);
            const int qn = qb * 32 + rr;
            if (__any(qn < vol && !(l_tot >= 0x1p-64f && l_tot <= 0x1p64f))) l_tot = exact(mixed_c, cur, qb);
            // ---- O^T[d][q]: reg 4g+e -> d = 8g + 4h + e; lane pairs swap halves -> 16-B stores
            const float inv = 1.0f / l_tot;
            unsigned pk[4][2];
#pragma unroll
            for (int g4 = 0; g4 < 4; ++g4) {
                pk[g4][0] = pack2bf(o[4 * g4 + 0] * inv, o[4 * g4 + 1] * inv);
                pk[g4][1] = pack2bf(o[4 * g4 + 2] * inv, o[4 * g4 + 3] * inv);
            }
            uint16_t* orow = out + cur.qrow * ldo + head * 32;
#pragma unroll
            for (int g4 = 0; g4 < 4; g4 += 2) {
                auto x0 = __builtin_amdgcn_permlane32_swap(pk[g4][0], pk[g4 + 1][0], false, false);
                auto x1 = __builtin_amdgcn_permlane32_swap(pk[g4][1], pk[g4 + 1][1], false, false);
                uint4 v;
                v.x = x0[0]; v.y = x1[0]; v.z = x0[1]; v.w = x1[1];
                if (qn < vol) *reinterpret_cast<uint4*>(orow + g4 * 8 + h * 8) = v;
            }
            if (more) cur = nxt;
        }
    };
    using NT7 = std::integral_constant<int, 7>;
    using NTX = std::integral_constant<int, 0>;
    if (ntile == 7) {
        if (mixed) run(std::true_type{}, NT7{});
        else run(std::false_type{}, NT7{});
    } else {
        if (mixed) run(std::true_type{}, NTX{});
        else run(std::false_type{}, NTX{});
    }
}

// ---------------------------------------------------------------------------------
// PatchMerging gather + LayerNorm(4C): out[(b,t,i,j)] = LN(cat(x[2i,2j], x[2i+1,2j],
// x[2i,2j+1], x[2i+1,2j+1])) (zero rows past an odd H/W edge, torchvision _patch_merging_pad).
// One wave per output token, 4C <= 4096.
// ---------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) patch_merge_ln_kernel(const float* __restrict__ x, int64_t ldx, int64_t B,
                                                             int T, int H, int W, int C,
                                                             const float* __restrict__ g,
                                                             const float* __restrict__ be, float eps,
                                                             uint16_t* __restrict__ y, int64_t ldy) {
    const int lane = threadIdx.x & 63;
    const int H2 = (H + 1) / 2, W2 = (W + 1) / 2;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= B * T * H2 * W2) return;
    const int j = (int)(row % W2);
    const int i = (int)((row / W2) % H2);
    const int64_t bt = row / ((int64_t)W2 * H2);
    const int C4 = 4 * C;
    float s = 0.f;
    // pass 1: sum (values re-read from L1/L2 in passes 2-3)
    auto val = [&](int n) -> float {
        const int q = n / C, c = n - q * C;  // q: 0 (2i,2j) 1 (2i+1,2j) 2 (2i,2j+1) 3 (2i+1,2j+1)
        const int hh = 2 * i + (q & 1), ww = 2 * j + (q >> 1);
        if (hh >= H || ww >= W) return 0.f;
        return x[((bt * H + hh) * W + ww) * ldx + c];
    };
    for (int n = lane; n < C4; n += 64) s += val(n);
    const float mean = wave_sum(s) / (float)C4;
    float q = 0.f;
    for (int n = lane; n < C4; n += 64) {
        const float d = val(n) - mean;
        q += d * d;
    }
    const float rstd = rsqrtf(wave_sum(q) / (float)C4 + eps);
    for (int n = lane; n < C4; n += 64) y[row * ldy + n] = f2bf((val(n) - mean) * rstd * g[n] + be[n]);
}

// Same merge + LayerNorm with float4 loads held in registers: L lanes per merged row (64 / L
// rows per wave), each lane V float4 of the 4C concatenation, one HBM pass (C % 4 == 0).
// The scalar kernel above re-reads each value three times and recomputes the quadrant index
// per element: 78 us for Swin-T stage 1 -> 2 at B = 4 (1.5 TB/s).
template <int L, int V>
__global__ void __launch_bounds__(256) patch_merge_ln_grp_kernel(const float* __restrict__ x, int64_t ldx, int64_t B,
                                                                 int T, int H, int W, int C,
                                                                 const float* __restrict__ g,
                                                                 const float* __restrict__ be, float eps,
                                                                 uint16_t* __restrict__ y, int64_t ldy) {
    const int sub = threadIdx.x & (L - 1);
    const int H2 = (H + 1) / 2, W2 = (W + 1) / 2;
    const int64_t row = ((int64_t)blockIdx.x * 256 + threadIdx.x) / L;
    if (row >= B * T * H2 * W2) return;  // whole L-lane groups exit together
    const int j = (int)(row % W2);
    const int i = (int)((row / W2) % H2);
    const int64_t bt = row / ((int64_t)W2 * H2);
    const int C4 = 4 * C;
    float4 v[V];
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < V; ++k) {
        const int n = (k * L + sub) * 4;
        v[k] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (n < C4) {
            const int q = n / C, c = n - q * C;  // q: 0 (2i,2j) 1 (2i+1,2j) 2 (2i,2j+1) 3 (2i+1,2j+1)
            const int hh = 2 * i + (q & 1), ww = 2 * j + (q >> 1);
            if (hh < H && ww < W) v[k] = *reinterpret_cast<const float4*>(x + ((bt * H + hh) * W + ww) * ldx + c);
        }
        s += (v[k].x + v[k].y) + (v[k].z + v[k].w);
    }
    const float mean = group_sum<L>(s) / (float)C4;
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < V; ++k) {
        if ((k * L + sub) * 4 < C4) {
            const float a = v[k].x - mean, b = v[k].y - mean, c = v[k].z - mean, d = v[k].w - mean;
            q += (a * a + b * b) + (c * c + d * d);
        }
    }
    const float rstd = rsqrtf(group_sum<L>(q) / (float)C4 + eps);
#pragma unroll
    for (int k = 0; k < V; ++k) {
        const int n = (k * L + sub) * 4;
        if (n < C4) {
            const float4 gg = *reinterpret_cast<const float4*>(g + n), bb = *reinterpret_cast<const float4*>(be + n);
            uint2 o;
            o.x = pack2bf((v[k].x - mean) * rstd * gg.x + bb.x, (v[k].y - mean) * rstd * gg.y + bb.y);
            o.y = pack2bf((v[k].z - mean) * rstd * gg.z + bb.z, (v[k].w - mean) * rstd * gg.w + bb.w);
            *reinterpret_cast<uint2*>(y + row * ldy + n) = o;
        }
    }
}

// ---------------------------------------------------------------------------------
// Final LayerNorm over every token, mean over the clip's tokens, classifier GEMV (fp32):
// logits[b] = W . mean_n LN(x[b, n]) + bias  (torchvision SwinTransformer3d.forward:
// norm -> avgpool -> flatten -> head).  Two deterministic stages (no atomics, fixed sum
// order): pool_partial_kernel — grid (B, POOL_CHUNKS), each wave normalises whole rows held
// in registers (D <= 1024) and accumulates them, the 4 waves reduce through LDS into
// work[b][chunk][:]; pool_final_kernel — grid B, sums the chunks in order, / ntok, GEMV.
// ---------------------------------------------------------------------------------
constexpr int POOL_CHUNKS = 64;

__global__ void __launch_bounds__(256) pool_partial_kernel(const float* __restrict__ x, int64_t ldx, int64_t ntok,
                                                           int D, const float* __restrict__ g,
                                                           const float* __restrict__ be, float eps,
                                                           float* __restrict__ work) {
    __shared__ float red[4][1024];
    const int b = blockIdx.x, ch = blockIdx.y;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    float4 acc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int64_t tk = (int64_t)ch * 4 + w; tk < ntok; tk += POOL_CHUNKS * 4) {
        const float* xr = x + ((int64_t)b * ntok + tk) * ldx;
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
                const float a0 = v[i].x - mean, a1 = v[i].y - mean, a2 = v[i].z - mean, a3 = v[i].w - mean;
                q += (a0 * a0 + a1 * a1) + (a2 * a2 + a3 * a3);
            }
        }
        const float rstd = rsqrtf(wave_sum(q) / (float)D + eps);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int n = (i * 64 + lane) * 4;
            if (n < D) {
                const float4 gg = *reinterpret_cast<const float4*>(g + n), bb = *reinterpret_cast<const float4*>(be + n);
                acc[i].x += (v[i].x - mean) * rstd * gg.x + bb.x;
                acc[i].y += (v[i].y - mean) * rstd * gg.y + bb.y;
                acc[i].z += (v[i].z - mean) * rstd * gg.z + bb.z;
                acc[i].w += (v[i].w - mean) * rstd * gg.w + bb.w;
            }
        }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int n = (i * 64 + lane) * 4;
        if (n < D) *reinterpret_cast<float4*>(&red[w][n]) = acc[i];
    }
    __syncthreads();
    for (int n = threadIdx.x; n < D; n += 256)
        work[((int64_t)b * POOL_CHUNKS + ch) * D + n] = (red[0][n] + red[1][n]) + (red[2][n] + red[3][n]);
}

// pooled (optional, train step): the pooled features [B][D] the head saw, for its backward
__global__ void __launch_bounds__(256) pool_final_kernel(const float* __restrict__ work, int64_t ntok, int D,
                                                         const float* __restrict__ Wc, const float* __restrict__ bc,
                                                         int nl, float* __restrict__ logits, float* __restrict__ pooled_out) {
    __shared__ float pooled[1024];
    const int b = blockIdx.x;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int n = threadIdx.x; n < D; n += 256) {
        float s = 0.f;
        for (int c = 0; c < POOL_CHUNKS; ++c) s += work[((int64_t)b * POOL_CHUNKS + c) * D + n];
        pooled[n] = s / (float)ntok;
        if (pooled_out) pooled_out[(int64_t)b * D + n] = pooled[n];
    }
    __syncthreads();
    for (int c = w; c < nl; c += 4) {
        float a = 0.f;
        for (int n = lane; n < D; n += 64) a += pooled[n] * Wc[(int64_t)c * D + n];
        a = wave_sum(a);
        if (lane == 0) logits[(int64_t)b * nl + c] = a + bc[c];
    }
}

}  // namespace vc

using namespace vc;

extern "C" {

static int window_fwd(const uint16_t* qkv, int64_t ld, int64_t B, int64_t T, int64_t H, int64_t W, int64_t heads,
                      int64_t head_dim, int wt, int wh, int ww, int st, int sh, int sw, const float* biasF, int64_t np,
                      uint16_t* out, int64_t ldo, float* lse, hipStream_t stream) {
    if (!qkv || !biasF || !out) return fail(VC_ERR_INVALID_ARG, "vc_window_attention3d: null pointer");
    if (head_dim != 32) return fail(VC_ERR_UNSUPPORTED, "vc_window_attention3d: head_dim must be 32");
    if (wt <= 0 || wh <= 0 || ww <= 0 || T % wt || H % wh || W % ww)
        return fail(VC_ERR_UNSUPPORTED, "vc_window_attention3d: the token grid must be whole windows (no padding)");
    if (st < 0 || sh < 0 || sw < 0 || st >= wt || sh >= wh || sw >= ww)
        return fail(VC_ERR_INVALID_ARG, "vc_window_attention3d: shift must be in [0, window)");
    const int vol = wt * wh * ww;
    if (np != (vol + 63) / 64 * 64 || np > WNP_MAX)
        return fail(VC_ERR_INVALID_ARG, "vc_window_attention3d: np must be roundup(window volume, 64) <= 448");
    if (ld < 3 * heads * 32 || ldo < heads * 32 || ld % 8 || ldo % 8 || ((uintptr_t)qkv | (uintptr_t)out) & 15)
        return fail(VC_ERR_INVALID_ARG, "vc_window_attention3d: bad leading dimension / alignment");
    WinGeom g{(int)T, (int)H, (int)W, wt, wh, ww, st, sh, sw, (int)(T / wt), (int)(H / wh), (int)(W / ww)};
    const int64_t nwin = B * g.nwt * g.nwh * g.nww;
    if (nwin > 0x7fffffff || heads > 65535) return fail(VC_ERR_INVALID_ARG, "vc_window_attention3d: grid too large");
    dim3 grid((unsigned)nwin, (unsigned)heads);
    if ((uintptr_t)biasF & 15) return fail(VC_ERR_INVALID_ARG, "vc_window_attention3d: biasF must be 16-B aligned");
    const int mk = (st | sh | sw) ? 1 : 0;
    if (lse)
        window_attn_d32_kernel<true><<<grid, 256, 0, stream>>>(qkv, ld, g, (int)heads, vol, (int)np, biasF, mk, out, ldo, lse);
    else
        window_attn_d32_kernel<false><<<grid, 256, 0, stream>>>(qkv, ld, g, (int)heads, vol, (int)np, biasF, mk, out, ldo,
                                                                nullptr);
    return check_launch("vc_window_attention3d");
}

int vc_window_attention3d(const uint16_t* qkv, int64_t ld, int64_t B, int64_t T, int64_t H, int64_t W, int64_t heads,
                          int64_t head_dim, int wt, int wh, int ww, int st, int sh, int sw, const float* biasF,
                          int64_t np, uint16_t* out, int64_t ldo, hipStream_t stream) {
    return window_fwd(qkv, ld, B, T, H, W, heads, head_dim, wt, wh, ww, st, sh, sw, biasF, np, out, ldo, nullptr, stream);
}

int vc_window_attention3d_mb(const uint16_t* qkv, int64_t ld, int64_t B, int64_t T, int64_t H, int64_t W, int64_t heads,
                             int64_t head_dim, int wt, int wh, int ww, int st, int sh, int sw, const uint16_t* biasB,
                             int64_t np, uint16_t* out, int64_t ldo, hipStream_t stream) {
    if (!qkv || !biasB || !out) return fail(VC_ERR_INVALID_ARG, "vc_window_attention3d_mb: null pointer");
    if (head_dim != 32) return fail(VC_ERR_UNSUPPORTED, "vc_window_attention3d_mb: head_dim must be 32");
    if (wt <= 0 || wh <= 0 || ww <= 0 || T % wt || H % wh || W % ww)
        return fail(VC_ERR_UNSUPPORTED, "vc_window_attention3d_mb: the token grid must be whole windows (no padding)");
    if (st < 0 || sh < 0 || sw < 0 || st >= wt || sh >= wh || sw >= ww)
        return fail(VC_ERR_INVALID_ARG, "vc_window_attention3d_mb: shift must be in [0, window)");
    const int vol = wt * wh * ww;
    if (np != (vol + 63) / 64 * 64 || np > WNP_MAX)
        return fail(VC_ERR_INVALID_ARG, "vc_window_attention3d_mb: np must be roundup(window volume, 64) <= 448");
    if (ld < 3 * heads * 32 || ldo < heads * 32 || ld % 8 || ldo % 8 || ((uintptr_t)qkv | (uintptr_t)out) & 15)
        return fail(VC_ERR_INVALID_ARG, "vc_window_attention3d_mb: bad leading dimension / alignment");
    if ((uintptr_t)biasB & 15) return fail(VC_ERR_INVALID_ARG, "vc_window_attention3d_mb: biasB must be 16-B aligned");
    WinGeom g{(int)T, (int)H, (int)W, wt, wh, ww, st, sh, sw, (int)(T / wt), (int)(H / wh), (int)(W / ww)};
    const int64_t nwin = B * g.nwt * g.nwh * g.nww;
    if (nwin > 0x7fffffff || heads > 65535) return fail(VC_ERR_INVALID_ARG, "vc_window_attention3d_mb: grid too large");
    if (nwin * heads > 0x7fffffff) return fail(VC_ERR_INVALID_ARG, "vc_window_attention3d_mb: grid too large");
    const int mk = (st | sh | sw) ? 1 : 0;
    window_attn_mb_d32_kernel<<<(unsigned)(nwin * heads), 256, 0, stream>>>(qkv, ld, g, (int)heads, vol, (int)np, biasB, mk, out, ldo);
    return check_launch("vc_window_attention3d_mb");
}

int vc_window_attention3d_lse(const uint16_t* qkv, int64_t ld, int64_t B, int64_t T, int64_t H, int64_t W,
                              int64_t heads, int64_t head_dim, int wt, int wh, int ww, int st, int sh, int sw,
                              const float* biasF, int64_t np, uint16_t* out, int64_t ldo, float* lse,
                              hipStream_t stream) {
    if (!lse) return fail(VC_ERR_INVALID_ARG, "vc_window_attention3d_lse: null lse");
    return window_fwd(qkv, ld, B, T, H, W, heads, head_dim, wt, wh, ww, st, sh, sw, biasF, np, out, ldo, lse, stream);
}

int vc_patch_merge_layernorm(const float* x, int64_t ldx, int64_t B, int64_t T, int64_t H, int64_t W, int64_t C,
                             const float* gamma, const float* beta, float eps, uint16_t* y, int64_t ldy,
                             hipStream_t stream) {
    if (!x || !gamma || !beta || !y) return fail(VC_ERR_INVALID_ARG, "vc_patch_merge_layernorm: null pointer");
    if (C <= 0 || 4 * C > 4096 || ldx < C || ldy < 4 * C)
        return fail(VC_ERR_INVALID_ARG, "vc_patch_merge_layernorm: bad C / leading dimension");
    const int64_t rows = B * T * ((H + 1) / 2) * ((W + 1) / 2);
    const int64_t n4 = C;  // float4 pieces per merged row (4C / 4)
    if (C % 4 == 0 && ldx % 4 == 0 && ldy % 4 == 0 && n4 <= 512 &&
        !(((uintptr_t)x | (uintptr_t)gamma | (uintptr_t)beta) & 15) && !((uintptr_t)y & 7)) {
        int L = 64, V = n4 <= 192 ? 3 : n4 <= 256 ? 4 : n4 <= 384 ? 6 : 8;
        for (int l = 8; l <= 32; l *= 2)
            if (n4 <= 4 * l) { L = l; V = n4 <= 3 * l ? 3 : 4; break; }
        const unsigned nb = (unsigned)((rows * L + 255) / 256);
#define VC_PM_GRP(LL, VV)                                                                                       \
    patch_merge_ln_grp_kernel<LL, VV><<<nb, 256, 0, stream>>>(x, ldx, B, (int)T, (int)H, (int)W, (int)C, gamma, \
                                                               beta, eps, y, ldy)
        if (L == 8) { if (V == 3) VC_PM_GRP(8, 3); else VC_PM_GRP(8, 4); }
        else if (L == 16) { if (V == 3) VC_PM_GRP(16, 3); else VC_PM_GRP(16, 4); }
        else if (L == 32) { if (V == 3) VC_PM_GRP(32, 3); else VC_PM_GRP(32, 4); }
        else if (V == 3) VC_PM_GRP(64, 3);
        else if (V == 4) VC_PM_GRP(64, 4);
        else if (V == 6) VC_PM_GRP(64, 6);
        else VC_PM_GRP(64, 8);
#undef VC_PM_GRP
        return check_launch("vc_patch_merge_layernorm");
    }
    patch_merge_ln_kernel<<<(unsigned)((rows + 3) / 4), 256, 0, stream>>>(x, ldx, B, (int)T, (int)H, (int)W, (int)C,
                                                                        gamma, beta, eps, y, ldy);
    return check_launch("vc_patch_merge_layernorm");
}

int vc_pool_head_pooled(const float* x, int64_t ldx, int64_t B, int64_t ntok, int64_t D, const float* gamma,
                        const float* beta, float eps, const float* Wc, const float* bc, int64_t num_labels, float* logits,
                        float* work, float* pooled, hipStream_t stream) {
    if (!x || !gamma || !beta || !Wc || !bc || !logits || !work)
        return fail(VC_ERR_INVALID_ARG, "vc_pool_head: null pointer");
    if (D <= 0 || D > 1024 || D % 4 || ldx % 4 || ntok <= 0 || ((uintptr_t)x & 15))
        return fail(VC_ERR_UNSUPPORTED, "vc_pool_head: D % 4 == 0, D <= 1024, 16-B aligned rows, ntok > 0");
    pool_partial_kernel<<<dim3((unsigned)B, POOL_CHUNKS), 256, 0, stream>>>(x, ldx, ntok, (int)D, gamma, beta, eps, work);
    pool_final_kernel<<<(unsigned)B, 256, 0, stream>>>(work, ntok, (int)D, Wc, bc, (int)num_labels, logits, pooled);
    return check_launch("vc_pool_head");
}

int vc_pool_head(const float* x, int64_t ldx, int64_t B, int64_t ntok, int64_t D, const float* gamma,
                 const float* beta, float eps, const float* Wc, const float* bc, int64_t num_labels, float* logits,
                 float* work, hipStream_t stream) {
    return vc_pool_head_pooled(x, ldx, B, ntok, D, gamma, beta, eps, Wc, bc, num_labels, logits, work, nullptr, stream);
}

// Backward of the classifier GEMV of vc_pool_head_pooled (fp32): dpooled[b] = scale * dlogits[b] . Wc,
// dWc[c] = sum_b dlogits[b][c] pooled[b], dbc[c] = sum_b dlogits[b][c] (fixed summation order)
__global__ void __launch_bounds__(256) head_bwd_kernel(const float* __restrict__ pooled, const float* __restrict__ dlog,
                                                       const float* __restrict__ Wc, int B, int D, int nl, float scale,
                                                       float* __restrict__ dpooled, float* __restrict__ dWc,
                                                       float* __restrict__ dbc) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < (int64_t)B * D + (int64_t)nl * D + nl;
         i += (int64_t)gridDim.x * 256) {
        if (i < (int64_t)B * D) {
            const int b = (int)(i / D), n = (int)(i % D);
            float s = 0.f;
            for (int c = 0; c < nl; ++c) s += dlog[b * nl + c] * Wc[(int64_t)c * D + n];
            dpooled[i] = s * scale;
        } else if (i < (int64_t)B * D + (int64_t)nl * D) {
            const int64_t j = i - (int64_t)B * D;
            const int c = (int)(j / D), n = (int)(j % D);
            float s = 0.f;
            for (int b = 0; b < B; ++b) s += dlog[b * nl + c] * pooled[(int64_t)b * D + n];
            dWc[j] = s;
        } else {
            const int c = (int)(i - (int64_t)B * D - (int64_t)nl * D);
            float s = 0.f;
            for (int b = 0; b < B; ++b) s += dlog[b * nl + c];
            dbc[c] = s;
        }
    }
}

int vc_pool_head_bwd(const float* pooled, const float* dlogits, const float* Wc, int64_t B, int64_t D, int64_t num_labels,
                     float scale, float* dpooled, float* dWc, float* dbc, hipStream_t stream) {
    if (!pooled || !dlogits || !Wc || !dpooled || !dWc || !dbc) return fail(VC_ERR_INVALID_ARG, "vc_pool_head_bwd: null pointer");
    if (B <= 0 || D <= 0 || num_labels <= 0) return fail(VC_ERR_INVALID_ARG, "vc_pool_head_bwd: bad shape");
    const int64_t n = B * D + num_labels * D + num_labels;
    head_bwd_kernel<<<(unsigned)((n + 255) / 256), 256, 0, stream>>>(pooled, dlogits, Wc, (int)B, (int)D, (int)num_labels,
                                                                    scale, dpooled, dWc, dbc);
    return check_launch("vc_pool_head_bwd");
}

}  // extern "C"
