// Short-sequence attention forward (S <= 256 tokens, head_dim 64): TimeSformer's spatial branch,
// B*T sequences of 1 + 196 tokens per head (TF5/models/timesformer/modeling_timesformer.py:148-180,
// the spatial half of the divided layer :332-398).
//
// The long-sequence kernel (attention.hip) streams 64-key tiles with an online softmax; at S = 197 it
// runs two 128-query workgroups per (sequence, head), each re-reading the sequence's K/V, four key
// tiles of which the last is 5/64 full, the running-max machinery for four tiles, and a second
// workgroup with one dead wave.  Here ONE 8-wave workgroup owns a (sequence, head):
//   * the whole K and V of the sequence (S rounded up to 32 keys: 224 at S = 197, 56 KiB) are staged
//     into LDS once by LDS-DMA (K image XOR-swizzled for ds_read_b128, V for ds_read_b64_tr_b16, the
//     long kernel's images);
//   * the sequence's ceil(S / 32) query blocks of 32 are dealt round-robin over 8 waves (7 blocks at
//     S = 197: one each), whose Q fragments load while K / V stage;
//   * per query block, 32 keys at a time: S'^T = K . Q'^T (swapped QK^T: a query's scores in one lane
//     column), P = exp2(S') packed to 16 bits straight from the accumulators as the B operand of
//     O^T = V^T . P^T, the row sum on the matrix pipe (P^T times a 0/1 selector, as attention.hip);
//     no running max at all (exp2 is exact in relative terms until it overflows): a row sum outside
//     [2^-64, 2^64] makes the wave repeat the block against the exact row max; the QK^T of the next
//     32 keys overlaps the current block's exponentials; 16-byte output stores;
//   * two workgroups per CU (56 KiB of LDS and <= 128 registers each): four waves per SIMD from two
//     workgroups overlap one's exponentials with another's MFMAs.
#include "common.hpp"

namespace vc {
namespace ashort {

constexpr int MAXS = 256;                   // longest sequence
constexpr int ROWB = 128;                   // bytes per K / V row (64 x 16 bit)

__device__ __forceinline__ int kswz(int r, int c) { return c ^ ((r >> 1) & 7); }
__device__ __forceinline__ int vswz(int r, int c) { return c ^ (((r >> 1) & 1) << 2); }

__device__ __forceinline__ void adma16s(const void* sbase, uint32_t voff, uint32_t lds_addr) {
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1"
                 :
                 : "v"(voff), "s"(sbase), "s"(lds_addr)
                 : "memory", "m0");
}

// One 32-query block of one (sequence, head) against all NKB key blocks staged in LDS (ktile / vtile
// images): qf = the block's Q'^T fragments (query row clamped to S - 1 past the sequence); writes the
// block's output rows (q < S) to orow.
template <int ET, int NKB>
__device__ __forceinline__ void query_block(const char* ktile, const char* vtile, v8s (&qf)[4], const int (&koff)[4],
                                            const int (&voff)[2], const v8s& sel, int S, int q, int h,
                                            float c_log2, uint16_t* orow) {
    if (c_log2 != 1.0f) {  // q not pre-scaled by the producer: fold scale * log2 e here
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
#pragma unroll
            for (int j = 0; j < 8; ++j) qf[kk][j] = (short)to16<ET>(from16<ET>((unsigned short)qf[kk][j]) * c_log2);
    }
    const int r = q & 31;
    v16f o[2];
    v4f lsum;
    // one 32-key block: S'^T = K_kb . Q'^T
    auto qk = [&](int kb) __attribute__((always_inline)) {
        v16f acc = v16f{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
            const v8s kf = *reinterpret_cast<const v8s*>(ktile + kb * 32 * ROWB + koff[kk]);
            acc = mfma32x16<ET>(kf, qf[kk], acc);
        }
        if (kb == NKB - 1 && NKB * 32 > S) {  // keys past S -> -inf
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int key = kb * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
                if (key >= S) acc[e] = -INFINITY;
            }
        }
        return acc;
    };
    // P = exp2(S' - m) of one key block (packed, the B operand of P.V) and O^T += V^T . P^T,
    // the row sum on the matrix pipe
    auto pv = [&](int kb, const v16f& sc, float m) __attribute__((always_inline)) {
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
            v4u pu;
#pragma unroll
            for (int jj = 0; jj < 4; ++jj)
                pu[jj] = pack2<ET>(__builtin_amdgcn_exp2f(sc[8 * s2 + 2 * jj] - m),
                                   __builtin_amdgcn_exp2f(sc[8 * s2 + 2 * jj + 1] - m));
            const v8s pf = __builtin_bit_cast(v8s, pu);
#pragma unroll
            for (int db = 0; db < 2; ++db) {
                const char* pa = vtile + voff[db] + (kb * 32 + 16 * s2) * ROWB;
                v4s va = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)pa);
                v4s vb = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(pa + 8 * ROWB));
                v8s vv;
                vv[0] = va[0]; vv[1] = va[1]; vv[2] = va[2]; vv[3] = va[3];
                vv[4] = vb[0]; vv[5] = vb[1]; vv[6] = vb[2]; vv[7] = vb[3];
                o[db] = mfma32x16<ET>(vv, pf, o[db]);
            }
            lsum = mfma16x32<ET>(sel, pf, lsum);
        }
    };
    auto reset = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int db = 0; db < 2; ++db)
            o[db] = v16f{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        lsum = v4f{0.f, 0.f, 0.f, 0.f};
    };
    // fast pass, no max at all: exp2 of a score is exact in relative terms until it overflows
    // (a score above ~127 in log2 units) or the whole row underflows; the QK^T of block kb+1 is
    // independent of block kb's exp2 / P.V, so the scheduler overlaps them.
    reset();
    {
        v16f cur = qk(0);
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb) {
            v16f nxt;
            if (kb + 1 < NKB) nxt = qk(kb + 1);
            pv(kb, cur, 0.f);
            if (kb + 1 < NKB) cur = nxt;
            // one key block of look-ahead (hoisting every block's QK^T keeps 16 registers of
            // scores per block live and spilled)
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    // a row sum outside [2^-64, 2^64] (overflow, underflow, inf / NaN input): repeat the block
    // against the exact row max (two passes over the keys; rare)
    const float l_fast = __shfl(lsum[0], (r & 15) + ((r >> 4) << 5), 64);
    if (__any(q < S && !(l_fast >= 0x1p-64f && l_fast <= 0x1p64f))) {  // padding queries never count
        float m = -INFINITY;
#pragma unroll 1
        for (int kb = 0; kb < NKB; ++kb) {
            const v16f sc = qk(kb);
#pragma unroll
            for (int e = 0; e < 16; ++e) m = fmaxf(m, sc[e]);
        }
        m = fmaxf(m, __shfl_xor(m, 32, 64));
        reset();
#pragma unroll 1
        for (int kb = 0; kb < NKB; ++kb) pv(kb, qk(kb), m);
    }
    // query r's row sum sits in lane (r & 15) + 32 (r >> 4)
    const float inv = 1.0f / __shfl(lsum[0], (r & 15) + ((r >> 4) << 5), 64);
    unsigned pk[2][4][2];
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            pk[db][g][0] = pack2<ET>(o[db][4 * g + 0] * inv, o[db][4 * g + 1] * inv);
            pk[db][g][1] = pack2<ET>(o[db][4 * g + 2] * inv, o[db][4 * g + 3] * inv);
        }
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

// per-lane constant LDS offsets: K row reads (key block 0; block kb at + 32 kb rows), the V^T
// transpose reads of d-block db, and the 0/1 selector of the row-sum MFMA
__device__ __forceinline__ void lane_offsets(int lane, int (&koff)[4], int (&voff)[2]) {
    const int r = lane & 31, h = lane >> 5;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) koff[kk] = r * ROWB + kswz(r, kk * 2 + h) * 16;
    const int gi = lane & 15;
    const int tq = gi >> 2, tp = gi & 3;
    const int gcol = ((lane >> 4) & 1) * 16 + tp * 4;
#pragma unroll
    for (int db = 0; db < 2; ++db) {
        const int col = db * 32 + gcol;
        const int ra = 4 * h + tq;
        voff[db] = ra * ROWB + vswz(ra, col >> 3) * 16 + (col & 7) * 2;
    }
}

template <int ET>
__device__ __forceinline__ v8s row_sum_selector(int lane) {
    const short one = ET == VC_ELEM_F16 ? (short)0x3C00 : (short)0x3F80;
    const short v = (((lane >> 4) & 1) == ((lane & 15) >> 3)) ? one : (short)0;
    v8s sel;
#pragma unroll
    for (int j = 0; j < 8; ++j) sel[j] = v;
    return sel;
}

__device__ __forceinline__ void load_q(const uint16_t* qbase, int64_t tok0, int64_t ld, int qc, int h, v8s (&qf)[4]) {
    const uint16_t* qrow = qbase + (tok0 + qc) * ld + 8 * h;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) qf[kk] = *reinterpret_cast<const v8s*>(qrow + 16 * kk);
}

// NKB: 32-key blocks staged and computed (ceil(S / 32), compile time so the score array stays in
// registers); S: real keys (masked beyond).
constexpr int NW = 8;  // waves per workgroup

template <int ET, int NKB>
__global__ void __launch_bounds__(NW * 64, 2 * NW / 4)
attn_short_d64_kernel(const uint16_t* __restrict__ qkv, int64_t ld, int S, int H, float c_log2,
                      uint16_t* __restrict__ out, int64_t ldo) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int NROW = NKB * 32;
    char* ktile = smem;
    char* vtile = smem + NROW * ROWB;

    const int bh = blockIdx.x;
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

    // ---- Q'^T fragments of the wave's query block (nqb <= NW: at most one per wave): issued before
    //      the K / V staging so their latency overlaps it (query rows past S clamp to S - 1; not stored)
    const int nqb = (S + 31) / 32;
    const int q = wave * 32 + r;
    const int qc = q < S ? q : S - 1;
    v8s qf[4];
    if (wave < nqb) load_q(qbase, tok0, ld, qc, h, qf);

    // ---- stage all NROW rows of K and V: piece p = rows 8p .. 8p+7 (1 KiB), wave w takes p = w, w+NW, ..
    {
        const int spc = lane & 7;
#pragma unroll
        for (int p = wave; p < NROW / 8; p += NW) {
            const int row = 8 * p + (lane >> 3);
            const uint32_t ko = (uint32_t)(row * ld + kswz(row, spc) * 8) * 2;
            const uint32_t vo = (uint32_t)(row * ld + vswz(row, spc) * 8) * 2;
            adma16s(kbase, ko, __builtin_amdgcn_readfirstlane(lds0 + p * 8 * ROWB));
            adma16s(vbase, vo, __builtin_amdgcn_readfirstlane(lds0 + NROW * ROWB + p * 8 * ROWB));
        }
    }
    int koff[4], voff[2];
    lane_offsets(lane, koff, voff);
    const v8s sel = row_sum_selector<ET>(lane);

    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this wave's pieces landed
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();        // ... and every other wave's
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);

    if (wave < nqb)
        query_block<ET, NKB>(ktile, vtile, qf, koff, voff, sel, S, q, h, c_log2, out + (tok0 + qc) * ldo + hh * 64);
}


template <int ET, int NKB>
static int launch_nkb(const uint16_t* qkv, int64_t ld, int64_t B, int64_t S, int64_t H, float c_log2, uint16_t* out,
                      int64_t ldo, hipStream_t stream) {
    const int items = (int)(B * H);
    const int lds = 2 * NKB * 32 * ROWB;
    attn_short_d64_kernel<ET, NKB><<<(unsigned)items, NW * 64, lds, stream>>>(qkv, ld, (int)S, (int)H, c_log2, out, ldo);
    return 0;
}

template <int ET>
static int launch_et(const uint16_t* qkv, int64_t ld, int64_t B, int64_t S, int64_t H, float c_log2, uint16_t* out,
                     int64_t ldo, hipStream_t stream) {
    switch ((S + 31) / 32) {
        case 1: return launch_nkb<ET, 1>(qkv, ld, B, S, H, c_log2, out, ldo, stream);
        case 2: return launch_nkb<ET, 2>(qkv, ld, B, S, H, c_log2, out, ldo, stream);
        case 3: return launch_nkb<ET, 3>(qkv, ld, B, S, H, c_log2, out, ldo, stream);
        case 4: return launch_nkb<ET, 4>(qkv, ld, B, S, H, c_log2, out, ldo, stream);
        case 5: return launch_nkb<ET, 5>(qkv, ld, B, S, H, c_log2, out, ldo, stream);
        case 6: return launch_nkb<ET, 6>(qkv, ld, B, S, H, c_log2, out, ldo, stream);
        case 7: return launch_nkb<ET, 7>(qkv, ld, B, S, H, c_log2, out, ldo, stream);
        default: return launch_nkb<ET, 8>(qkv, ld, B, S, H, c_log2, out, ldo, stream);
    }
}

}  // namespace ashort

// attention.hip routes S <= 256 here (inference forward)
int launch_attn_short(const uint16_t* qkv, int64_t ld, int64_t B, int64_t S, int64_t H, float c_log2, uint16_t* out,
                      int64_t ldo, int elem, hipStream_t stream) {
    if (S < 1 || S > ashort::MAXS) return fail(VC_ERR_INVALID_ARG, "attention (short): S must be in [1, 256]");
    const int rc = elem == VC_ELEM_F16 ? ashort::launch_et<VC_ELEM_F16>(qkv, ld, B, S, H, c_log2, out, ldo, stream)
                                       : ashort::launch_et<VC_ELEM_BF16>(qkv, ld, B, S, H, c_log2, out, ldo, stream);
    if (rc) return rc;
    return check_launch("vc_attention_fwd (short)");
}

}  // namespace vc
