// Joint attention backward (flash-style, P recomputed from the forward's log-sum-exp),
// head_dim 64, bf16 MFMA with fp32 accumulation.
//
// The gradient of eager_attention_forward (TF5/models/vivit/modeling_vivit.py:149-174), i.e.
// what autograd runs for loss.backward() in the reference's train step
// (vivit_transformer/vivit_classifier/trainers/trainer.py:145).  The forward works in the
// log2 domain: S' = q'.k with q' = q * scale * log2(e) (what the qkv buffer holds), P =
// exp2(S' - lse2).  Then, with dO the gradient of the attention output and
// Delta = rowsum(dO o O):
//     dV = P^T dO,   dP = dO V^T,   dS' = ln2 * P o (dP - Delta),
//     dK = dS'^T q', dq' = dS' K           (dq' is the gradient w.r.t. the stored q').
// Three launches, all deterministic (no atomics):
//   prep  : Delta per (clip, head, query);
//   dK/dV : one wave per 32 keys, looping over 64-query tiles of Q' / dO staged in LDS;
//   dQ    : one wave per 32 queries (the forward's structure), looping over 64-key tiles.
// MFMA operand plumbing (cdna_hip_programming.md §3 "An accumulator tile as the next MFMA's
// operand", T10): every product that sums over the accumulator's register (row) index takes
// it straight from registers; the other operand comes from LDS either as plain rows
// (ds_read_b128) or transposed (ds_read_b64_tr_b16) in the matching permuted k order.
#include "common.hpp"

namespace vc {
namespace abwd {

constexpr int TILE_BYTES = 64 * 64 * 2;  // one [64 rows][64 bf16] image, 128-B rows
constexpr float LN2 = 0.69314718055994531f;

// 16-B chunk swizzle of a 128-B-row image that is conflict-free both for ds_read_b128 row
// reads (lane r reads row r) and for ds_read_b64_tr_b16 reads of 4-row blocks:
// chunk c of row r lives at c ^ brev3((r >> 1) & 7).  Invariant under row offsets that are
// multiples of 16.
__device__ __forceinline__ int bswz(int r, int c) {
    const int m = (r >> 1) & 7;
    return c ^ (((m & 1) << 2) | (m & 2) | ((m >> 2) & 1));
}

// A/B fragment of k-step kk from a row image: lane (r, h) gets row `row`, columns 16kk+8h..+7
__device__ __forceinline__ v8bf row_frag(const char* tile, int off) {
    return __builtin_bit_cast(v8bf, *reinterpret_cast<const v8s*>(tile + off));
}

// transposed fragment (T10): columns 32db + (lane>>4 & 1)*16 + 4tp .. +3 of rows kr + 4h + tq
// and kr + 4h + tq + 8 -> 8 k-values in the permuted order of an accumulator's registers
__device__ __forceinline__ v8bf tr_frag(const char* tile, int offa, int offb) {
    v4s va = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(tile + offa));
    v4s vb = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(tile + offb));
    v8s vv;
    vv[0] = va[0]; vv[1] = va[1]; vv[2] = va[2]; vv[3] = va[3];
    vv[4] = vb[0]; vv[5] = vb[1]; vv[6] = vb[2]; vv[7] = vb[3];
    return __builtin_bit_cast(v8bf, vv);
}

// regs 8 s2 .. 8 s2 + 7 of an accumulator as an MFMA operand: four v_cvt_pk_bf16_f32 (RNE, as the
// element-wise cast, which hipcc lowered to conversions plus v_perm / v_alignbit repacking)
__device__ __forceinline__ v8bf to_bf8(const v16f& x, int s2) {
    v4u u;
#pragma unroll
    for (int j = 0; j < 4; ++j) u[j] = pack2bf(x[8 * s2 + 2 * j], x[8 * s2 + 2 * j + 1]);
    return __builtin_bit_cast(v8bf, u);
}

// per-lane LDS byte offsets of the transposed reads (rows 4h + tq and +8), per 32-column block
struct TrOffsets {
    int a[2], b[2];
};
__device__ __forceinline__ TrOffsets tr_offsets(int lane) {
    const int h = lane >> 5, gi = lane & 15, tq = gi >> 2, tp = gi & 3;
    const int gcol = ((lane >> 4) & 1) * 16 + tp * 4;
    TrOffsets o;
#pragma unroll
    for (int db = 0; db < 2; ++db) {
        const int col = db * 32 + gcol;
        const int ra = 4 * h + tq, rb = ra + 8;
        o.a[db] = ra * 128 + bswz(ra, col >> 3) * 16 + (col & 7) * 2;
        o.b[db] = rb * 128 + bswz(rb, col >> 3) * 16 + (col & 7) * 2;
    }
    return o;
}

// Store a [32 rows (lane)][64 cols (2 x 16 regs)] accumulator pair as bf16 rows: reg 4g+e of
// block db -> column 32db + 8g + 4h + e; lane pairs swap halves for 16-B stores (T21).
__device__ __forceinline__ void store_rows(uint16_t* row, const v16f (&acc)[2], float scale, int h, bool valid) {
    unsigned pk[2][4][2];
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            pk[db][g][0] = pack2bf(acc[db][4 * g + 0] * scale, acc[db][4 * g + 1] * scale);
            pk[db][g][1] = pack2bf(acc[db][4 * g + 2] * scale, acc[db][4 * g + 3] * scale);
        }
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
        for (int g = 0; g < 4; g += 2) {
            auto x0 = __builtin_amdgcn_permlane32_swap(pk[db][g][0], pk[db][g + 1][0], false, false);
            auto x1 = __builtin_amdgcn_permlane32_swap(pk[db][g][1], pk[db][g + 1][1], false, false);
            uint4 v;
            v.x = x0[0]; v.y = x1[0]; v.z = x0[1]; v.w = x1[1];
            if (valid) *reinterpret_cast<uint4*>(row + db * 32 + g * 8 + h * 8) = v;
        }
}

// s_waitcnt vmcnt(0) through the builtin, so the compiler's wait-count scoreboard sees it.
// Round 5: registers loaded ahead of a main loop and first used inside it make hipcc put that wait
// INSIDE the loop (at the first use), where it also drains the next tile's prefetch loads every
// iteration -- the prefetch then hides nothing (the dQ kernel waited vmcnt(0) before its first MFMAs
// each tile; dK/dV negated its prefetched -lse right after the load, same effect)
__device__ __forceinline__ void vm_drain() { __builtin_amdgcn_s_waitcnt(0x0F70); }

// bijective XCD-aware remap of the linear workgroup id (as the forward kernel)
__device__ __forceinline__ int xcd_remap(int L, int nwg) {
    const int xq = nwg >> 3, xr = nwg & 7, xcd = L & 7;
    return (xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + (L >> 3);
}

// ---------------------------------------------------------------------------------
// Delta[(b*H + h)*S + s] = sum_d dO[b*S+s][h*64+d] * O[b*S+s][h*64+d]  (fp32)
// ---------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) attn_bwd_prep_kernel(const uint16_t* __restrict__ dout, int64_t lddo,
                                                           const uint16_t* __restrict__ out, int64_t ldo, int64_t n,
                                                           int S, int H, float* __restrict__ delta) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int hh = (int)(i % H);
    const int64_t row = i / H;
    const uint4* a = reinterpret_cast<const uint4*>(dout + row * lddo + hh * 64);
    const uint4* o = reinterpret_cast<const uint4*>(out + row * ldo + hh * 64);
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const uint4 x = a[j], y = o[j];
        const unsigned xs[4] = {x.x, x.y, x.z, x.w}, ys[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            s += bf2f((unsigned short)(xs[k] & 0xffff)) * bf2f((unsigned short)(ys[k] & 0xffff));
            s += bf2f((unsigned short)(xs[k] >> 16)) * bf2f((unsigned short)(ys[k] >> 16));
        }
    }
    const int64_t b = row / S, sq = row - b * S;
    delta[(b * H + hh) * S + sq] = s;
}

// ---------------------------------------------------------------------------------
// dK, dV: workgroup = 128 keys of one (clip, head), wave w owns keys 32w..32w+31.
// Per 64-query tile (double-buffered LDS: Q' image, dO image, lse[64], Delta[64]):
//   S  [q][key] = Q'.K^T        A = Q' rows (LDS b128), B = K (registers)
//   P           = exp2(S - lse) (lse per accumulator register = per query)
//   dV^T[d][key] += dO^T . P    A = dO^T (LDS tr), B = P (registers)
//   dP [q][key] = dO.V^T        A = dO rows (LDS b128), B = V (registers)
//   dS          = P o (dP - Delta)
//   dK^T[d][key] += Q'^T . dS   A = Q'^T (LDS tr), B = dS (registers)
// ---------------------------------------------------------------------------------
constexpr int SLOT_A = 2 * TILE_BYTES + 2 * 64 * 4;

__global__ void __launch_bounds__(256, 2)
attn_bwd_dkdv_kernel(const uint16_t* __restrict__ qkv, int64_t ld, const uint16_t* __restrict__ dout, int64_t lddo,
                     const float* __restrict__ lse, const float* __restrict__ delta, int S, int H,
                     uint16_t* __restrict__ dqkv, int64_t lddq) {
    __shared__ __attribute__((aligned(16))) char smem[2 * SLOT_A];
    const int nk = gridDim.x;
    const int wg = xcd_remap(blockIdx.y * nk + blockIdx.x, nk * gridDim.y);
    const int kblk = wg % nk, bh = wg / nk;
    const int b = bh / H, hh = bh % H;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 31, h = lane >> 5;

    const int64_t tok0 = (int64_t)b * S;
    const uint16_t* qbase = qkv + tok0 * ld + hh * 64;
    const uint16_t* kbase = qkv + tok0 * ld + (int64_t)H * 64 + hh * 64;
    const uint16_t* vbase = qkv + tok0 * ld + (int64_t)2 * H * 64 + hh * 64;
    const uint16_t* dobase = dout + tok0 * lddo + hh * 64;
    const float* lseb = lse + (int64_t)bh * S;
    const float* delb = delta + (int64_t)bh * S;

    const int key = kblk * 128 + wave * 32 + r;
    const int kc = key < S ? key : S - 1;
    v8bf kf[4], vf[4];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
        kf[kk] = __builtin_bit_cast(v8bf, *reinterpret_cast<const v8s*>(kbase + (int64_t)kc * ld + 16 * kk + 8 * h));
        vf[kk] = __builtin_bit_cast(v8bf, *reinterpret_cast<const v8s*>(vbase + (int64_t)kc * ld + 16 * kk + 8 * h));
    }
    int roff[4];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) roff[kk] = r * 128 + bswz(r, 2 * kk + h) * 16;
    const TrOffsets tro = tr_offsets(lane);

    v16f dv[2], dk[2];
#pragma unroll
    for (int e = 0; e < 16; ++e) { dv[0][e] = 0.f; dv[1][e] = 0.f; dk[0][e] = 0.f; dk[1][e] = 0.f; }

    const int nt = (S + 63) / 64;
    // tile prefetch lives in plain registers (a struct captured by lambdas ended up in scratch)
    uint4 pq0, pq1, pd0, pd1;
    float tf = 0.f;  // the raw lse (threads 0-63) / Delta (64-127) of the prefetched tile
    const int sr0 = tid >> 3, sc = tid & 7;
    const int so0 = sr0 * 128 + bswz(sr0, sc) * 16, so1 = (sr0 + 32) * 128 + bswz(sr0 + 32, sc) * 16;
    // LDS holds -lse and -Delta: they initialise the S and dP accumulators (so the MFMAs emit
    // S - lse and dP - Delta directly); a query past S gets -lse = -inf, i.e. P = 0
#define ABWD_LOAD_A(t)                                                                                  \
    {                                                                                                   \
        const uint16_t* qs = qbase + ((int64_t)(t) * 64 + sr0) * ld + sc * 8;                           \
        const uint16_t* ds = dobase + ((int64_t)(t) * 64 + sr0) * lddo + sc * 8;                        \
        pq0 = *reinterpret_cast<const uint4*>(qs);                                                      \
        pq1 = *reinterpret_cast<const uint4*>(qs + 32 * ld);                                            \
        pd0 = *reinterpret_cast<const uint4*>(ds);                                                      \
        pd1 = *reinterpret_cast<const uint4*>(ds + 32 * lddo);                                          \
        {   /* every thread loads (no branch); used only at ABWD_STORE_A, after the tile's compute */   \
            const int q = (t) * 64 + (tid & 63);                                                        \
            const int qc = q < S ? q : S - 1;                                                           \
            tf = ((tid >> 6) & 1) ? delb[qc] : lseb[qc];                                                \
        }                                                                                               \
    }
#define ABWD_STORE_A(slot, t)                                                                           \
    {                                                                                                   \
        *reinterpret_cast<uint4*>((slot) + so0) = pq0;                                                  \
        *reinterpret_cast<uint4*>((slot) + so1) = pq1;                                                  \
        *reinterpret_cast<uint4*>((slot) + TILE_BYTES + so0) = pd0;                                     \
        *reinterpret_cast<uint4*>((slot) + TILE_BYTES + so1) = pd1;                                     \
        if (tid < 128)                                                                                  \
            reinterpret_cast<float*>((slot) + 2 * TILE_BYTES)[tid] =                                    \
                (tid < 64 && (t) * 64 + tid >= S) ? -INFINITY : -tf;                                    \
    }
    ABWD_LOAD_A(0);
    ABWD_STORE_A(smem, 0);
    vm_drain();
    __syncthreads();

    for (int t = 0; t < nt; ++t) {
        const char* cur = smem + (t & 1) * SLOT_A;
        const char* qi = cur;
        const char* di = cur + TILE_BYTES;
        const float* fl = reinterpret_cast<const float*>(cur + 2 * TILE_BYTES);  // [0,64) lse, [64,128) Delta
        if (t + 1 < nt) ABWD_LOAD_A(t + 1);
        // the two 32-query blocks' chains interleaved (sched_barrier fences pin the group order):
        // QK0 + dP0 | QK1 || exp0 | dV0 || dS0 | dP1 || exp1 | dK0 || dS1 | dV1 | dK1
        v16f s0, dp0, s1, dp1;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const float4 L0 = *reinterpret_cast<const float4*>(fl + 8 * g + 4 * h);
            const float4 D0 = *reinterpret_cast<const float4*>(fl + 64 + 8 * g + 4 * h);
            const float4 L1 = *reinterpret_cast<const float4*>(fl + 32 + 8 * g + 4 * h);
            const float4 D1 = *reinterpret_cast<const float4*>(fl + 64 + 32 + 8 * g + 4 * h);
            s0[4 * g + 0] = L0.x; s0[4 * g + 1] = L0.y; s0[4 * g + 2] = L0.z; s0[4 * g + 3] = L0.w;
            dp0[4 * g + 0] = D0.x; dp0[4 * g + 1] = D0.y; dp0[4 * g + 2] = D0.z; dp0[4 * g + 3] = D0.w;
            s1[4 * g + 0] = L1.x; s1[4 * g + 1] = L1.y; s1[4 * g + 2] = L1.z; s1[4 * g + 3] = L1.w;
            dp1[4 * g + 0] = D1.x; dp1[4 * g + 1] = D1.y; dp1[4 * g + 2] = D1.z; dp1[4 * g + 3] = D1.w;
        }
        auto dv_mfma = [&](int qb, const v16f& p) {
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
                const v8bf pf = to_bf8(p, s2);
                const int kr = (qb * 32 + 16 * s2) * 128;
#pragma unroll
                for (int db = 0; db < 2; ++db)
                    dv[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_frag(di, tro.a[db] + kr, tro.b[db] + kr), pf,
                                                                     dv[db], 0, 0, 0);
            }
        };
        auto dk_mfma = [&](int qb, const v16f& ds) {
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
                const v8bf sf = to_bf8(ds, s2);
                const int kr = (qb * 32 + 16 * s2) * 128;
#pragma unroll
                for (int db = 0; db < 2; ++db)
                    dk[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_frag(qi, tro.a[db] + kr, tro.b[db] + kr), sf,
                                                                     dk[db], 0, 0, 0);
            }
        };
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
            s0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(row_frag(qi, roff[kk]), kf[kk], s0, 0, 0, 0);
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
            dp0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(row_frag(di, roff[kk]), vf[kk], dp0, 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
            s1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(row_frag(qi, 4096 + roff[kk]), kf[kk], s1, 0, 0, 0);
#pragma unroll
        for (int e = 0; e < 16; ++e) s0[e] = __builtin_amdgcn_exp2f(s0[e]);
        __builtin_amdgcn_sched_barrier(0);
        dv_mfma(0, s0);
#pragma unroll
        for (int e = 0; e < 16; ++e) dp0[e] = s0[e] * dp0[e];
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
            dp1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(row_frag(di, 4096 + roff[kk]), vf[kk], dp1, 0, 0, 0);
#pragma unroll
        for (int e = 0; e < 16; ++e) s1[e] = __builtin_amdgcn_exp2f(s1[e]);
        __builtin_amdgcn_sched_barrier(0);
        dk_mfma(0, dp0);
#pragma unroll
        for (int e = 0; e < 16; ++e) dp1[e] = s1[e] * dp1[e];
        __builtin_amdgcn_sched_barrier(0);
        dv_mfma(1, s1);
        dk_mfma(1, dp1);
        if (t + 1 < nt) ABWD_STORE_A(smem + ((t + 1) & 1) * SLOT_A, t + 1);
        __syncthreads();
    }
#undef ABWD_LOAD_A
#undef ABWD_STORE_A
    uint16_t* drow = dqkv + (tok0 + kc) * lddq + hh * 64;
    store_rows(drow + (int64_t)H * 64, dk, LN2, h, key < S);
    store_rows(drow + (int64_t)2 * H * 64, dv, 1.0f, h, key < S);
}

// ---------------------------------------------------------------------------------
// dQ: workgroup = 128 queries of one (clip, head), wave w owns queries 32w..32w+31.
// Per 64-key tile (double-buffered LDS: K image, V image):
//   S^T [key][q] = K.Q'^T       A = K rows (LDS b128), B = Q' (registers)
//   P^T          = exp2(S^T - lse[q])   (per lane)
//   dP^T[key][q] = V.dO^T       A = V rows (LDS b128), B = dO (registers)
//   dS^T         = P^T o (dP^T - Delta[q])
//   dQ^T[d][q]  += K^T . dS^T   A = K^T (LDS tr), B = dS^T (registers)
// ---------------------------------------------------------------------------------
constexpr int SLOT_B = 2 * TILE_BYTES;

__global__ void __launch_bounds__(256, 2)
attn_bwd_dq_kernel(const uint16_t* __restrict__ qkv, int64_t ld, const uint16_t* __restrict__ dout, int64_t lddo,
                   const float* __restrict__ lse, const float* __restrict__ delta, int S, int H,
                   uint16_t* __restrict__ dqkv, int64_t lddq) {
    __shared__ __attribute__((aligned(16))) char smem[2 * SLOT_B];
    const int nq = gridDim.x;
    const int wg = xcd_remap(blockIdx.y * nq + blockIdx.x, nq * gridDim.y);
    const int qblk = wg % nq, bh = wg / nq;
    const int b = bh / H, hh = bh % H;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 31, h = lane >> 5;

    const int64_t tok0 = (int64_t)b * S;
    const uint16_t* qbase = qkv + tok0 * ld + hh * 64;
    const uint16_t* kbase = qkv + tok0 * ld + (int64_t)H * 64 + hh * 64;
    const uint16_t* vbase = qkv + tok0 * ld + (int64_t)2 * H * 64 + hh * 64;
    const uint16_t* dobase = dout + tok0 * lddo + hh * 64;

    const int q = qblk * 128 + wave * 32 + r;
    const int qc = q < S ? q : S - 1;
    v8bf qf[4], df[4];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
        qf[kk] = __builtin_bit_cast(v8bf, *reinterpret_cast<const v8s*>(qbase + (int64_t)qc * ld + 16 * kk + 8 * h));
        df[kk] = __builtin_bit_cast(v8bf, *reinterpret_cast<const v8s*>(dobase + (int64_t)qc * lddo + 16 * kk + 8 * h));
    }
    const float lq = lse[(int64_t)bh * S + qc];
    const float dq_delta = delta[(int64_t)bh * S + qc];
    int roff[4];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) roff[kk] = r * 128 + bswz(r, 2 * kk + h) * 16;
    const TrOffsets tro = tr_offsets(lane);

    v16f dq[2];
#pragma unroll
    for (int e = 0; e < 16; ++e) { dq[0][e] = 0.f; dq[1][e] = 0.f; }

    const int nt = (S + 63) / 64;
    uint4 pk0, pk1, pv0, pv1;
    const int sr0 = tid >> 3, sc = tid & 7;
    const int so0 = sr0 * 128 + bswz(sr0, sc) * 16, so1 = (sr0 + 32) * 128 + bswz(sr0 + 32, sc) * 16;
#define ABWD_LOAD_B(t)                                                                                  \
    {                                                                                                   \
        const uint16_t* ks = kbase + ((int64_t)(t) * 64 + sr0) * ld + sc * 8;                           \
        const uint16_t* vs = vbase + ((int64_t)(t) * 64 + sr0) * ld + sc * 8;                           \
        pk0 = *reinterpret_cast<const uint4*>(ks);                                                      \
        pk1 = *reinterpret_cast<const uint4*>(ks + 32 * ld);                                            \
        pv0 = *reinterpret_cast<const uint4*>(vs);                                                      \
        pv1 = *reinterpret_cast<const uint4*>(vs + 32 * ld);                                            \
    }
#define ABWD_STORE_B(slot)                                                                              \
    {                                                                                                   \
        *reinterpret_cast<uint4*>((slot) + so0) = pk0;                                                  \
        *reinterpret_cast<uint4*>((slot) + so1) = pk1;                                                  \
        *reinterpret_cast<uint4*>((slot) + TILE_BYTES + so0) = pv0;                                     \
        *reinterpret_cast<uint4*>((slot) + TILE_BYTES + so1) = pv1;                                     \
    }
    ABWD_LOAD_B(0);
    ABWD_STORE_B(smem);
    __syncthreads();

    // accumulator inits: S^T - lse and dP^T - Delta; register 4g+e of key block kb holds key
    // t*64 + 32kb + 8g + 4h + e (keys past S of the last tile are set to -inf after the MFMAs, P = 0)
    v16f negL, negD;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
        negL[e] = -lq;
        negD[e] = -dq_delta;
    }
    // qf / df landed before the loop (see vm_drain): the empty asm "uses" them here, so hipcc waits for
    // their loads at this point and not inside the loop
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) asm volatile("" : "+v"(qf[kk]), "+v"(df[kk]));
    auto dq_mfma = [&](const char* ki, int kb, const v16f& ds) {
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
            const v8bf sf = to_bf8(ds, s2);
            const int kr = (kb * 32 + 16 * s2) * 128;
#pragma unroll
            for (int db = 0; db < 2; ++db)
                dq[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_frag(ki, tro.a[db] + kr, tro.b[db] + kr), sf, dq[db],
                                                                 0, 0, 0);
        }
    };
    for (int t = 0; t < nt; ++t) {
        const char* ki = smem + (t & 1) * SLOT_B;
        const char* vi = ki + TILE_BYTES;
        if (t + 1 < nt) ABWD_LOAD_B(t + 1);
        // the two 32-key blocks' chains interleaved (sched_barrier fences pin the group order):
        // S0, dP0 | S1, dP1 || dS0 = exp2(S0) dP0 | dQ0 || dS1 | dQ1
        v16f st0 = negL, dpt0 = negD, st1 = negL, dpt1 = negD;
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
            st0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(row_frag(ki, roff[kk]), qf[kk], st0, 0, 0, 0);
            dpt0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(row_frag(vi, roff[kk]), df[kk], dpt0, 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
            st1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(row_frag(ki, 4096 + roff[kk]), qf[kk], st1, 0, 0, 0);
            dpt1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(row_frag(vi, 4096 + roff[kk]), df[kk], dpt1, 0, 0, 0);
        }
        if (t == nt - 1) {
            const int k0 = t * 64;
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                if (k0 + 8 * (e >> 2) + 4 * h + (e & 3) >= S) st0[e] = -INFINITY;
                if (k0 + 32 + 8 * (e >> 2) + 4 * h + (e & 3) >= S) st1[e] = -INFINITY;
            }
        }
        // dS^T = P^T o (dP^T - Delta)
#pragma unroll
        for (int e = 0; e < 16; ++e) st0[e] = __builtin_amdgcn_exp2f(st0[e]) * dpt0[e];
        __builtin_amdgcn_sched_barrier(0);
        dq_mfma(ki, 0, st0);
#pragma unroll
        for (int e = 0; e < 16; ++e) st1[e] = __builtin_amdgcn_exp2f(st1[e]) * dpt1[e];
        __builtin_amdgcn_sched_barrier(0);
        dq_mfma(ki, 1, st1);
        if (t + 1 < nt) ABWD_STORE_B(smem + ((t + 1) & 1) * SLOT_B);
        __syncthreads();
    }
#undef ABWD_LOAD_B
#undef ABWD_STORE_B
    store_rows(dqkv + (tok0 + qc) * lddq + hh * 64, dq, LN2, h, q < S);
}

}  // namespace abwd
}  // namespace vc

using namespace vc;
using namespace vc::abwd;

extern "C" int vc_attention_bwd_2s(const uint16_t* qkv, int64_t ld, const uint16_t* out, int64_t ldo,
                                   const uint16_t* dout, int64_t lddo, const float* lse, float* delta, int64_t B,
                                   int64_t S, int64_t H, int64_t head_dim, uint16_t* dqkv, int64_t lddq,
                                   hipStream_t stream, hipStream_t stream2);

extern "C" int vc_attention_bwd(const uint16_t* qkv, int64_t ld, const uint16_t* out, int64_t ldo, const uint16_t* dout,
                                int64_t lddo, const float* lse, float* delta, int64_t B, int64_t S, int64_t H,
                                int64_t head_dim, uint16_t* dqkv, int64_t lddq, hipStream_t stream) {
    if (!qkv || !out || !dout || !lse || !delta || !dqkv) return fail(VC_ERR_INVALID_ARG, "vc_attention_bwd: null pointer");
    if (head_dim != 64) return fail(VC_ERR_UNSUPPORTED, "vc_attention_bwd: head_dim must be 64");
    if (B <= 0 || S <= 0 || H <= 0 || ld < 3 * H * 64 || lddq < 3 * H * 64 || ldo < H * 64 || lddo < H * 64 ||
        ld % 8 || ldo % 8 || lddo % 8 || lddq % 8)
        return fail(VC_ERR_INVALID_ARG, "vc_attention_bwd: bad shape / leading dimension");
    if ((((uintptr_t)qkv) | ((uintptr_t)out) | ((uintptr_t)dout) | ((uintptr_t)dqkv) | ((uintptr_t)lse) |
         ((uintptr_t)delta)) & 15)
        return fail(VC_ERR_INVALID_ARG, "vc_attention_bwd: pointers must be 16-byte aligned");
    if (B * H > 65535 || S > (1 << 24)) return fail(VC_ERR_INVALID_ARG, "vc_attention_bwd: grid too large");
    return vc_attention_bwd_2s(qkv, ld, out, ldo, dout, lddo, lse, delta, B, S, H, head_dim, dqkv, lddq, stream, nullptr);
}

// dK/dV and dQ write disjoint column ranges of dqkv from the same inputs: with a second stream the
// dQ kernel runs beside dK/dV (its workgroups fill the other's last partial round), and `stream`
// waits for it before returning
extern "C" int vc_attention_bwd_2s(const uint16_t* qkv, int64_t ld, const uint16_t* out, int64_t ldo,
                                   const uint16_t* dout, int64_t lddo, const float* lse, float* delta, int64_t B,
                                   int64_t S, int64_t H, int64_t head_dim, uint16_t* dqkv, int64_t lddq,
                                   hipStream_t stream, hipStream_t stream2) {
    if (!qkv || !out || !dout || !lse || !delta || !dqkv) return fail(VC_ERR_INVALID_ARG, "vc_attention_bwd: null pointer");
    if (head_dim != 64) return fail(VC_ERR_UNSUPPORTED, "vc_attention_bwd: head_dim must be 64");
    if (B <= 0 || S <= 0 || H <= 0 || ld < 3 * H * 64 || lddq < 3 * H * 64 || ldo < H * 64 || lddo < H * 64 ||
        ld % 8 || ldo % 8 || lddo % 8 || lddq % 8)
        return fail(VC_ERR_INVALID_ARG, "vc_attention_bwd: bad shape / leading dimension");
    if ((((uintptr_t)qkv) | ((uintptr_t)out) | ((uintptr_t)dout) | ((uintptr_t)dqkv) | ((uintptr_t)lse) |
         ((uintptr_t)delta)) & 15)
        return fail(VC_ERR_INVALID_ARG, "vc_attention_bwd: pointers must be 16-byte aligned");
    if (B * H > 65535 || S > (1 << 24)) return fail(VC_ERR_INVALID_ARG, "vc_attention_bwd: grid too large");
    const int64_t n = B * S * H;
    attn_bwd_prep_kernel<<<(unsigned)((n + 255) / 256), 256, 0, stream>>>(dout, lddo, out, ldo, n, (int)S, (int)H, delta);
    const dim3 grid((unsigned)((S + 127) / 128), (unsigned)(B * H));
    const bool two = stream2 != nullptr && stream2 != stream;
    hipEvent_t e_prep = nullptr, e_dq = nullptr;
    if (two) {
        hipError_t e = hipEventCreateWithFlags(&e_prep, hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&e_dq, hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventRecord(e_prep, stream);
        if (e == hipSuccess) e = hipStreamWaitEvent(stream2, e_prep, 0);
        if (e != hipSuccess) {
            if (e_prep) (void)hipEventDestroy(e_prep);
            if (e_dq) (void)hipEventDestroy(e_dq);
            return fail((int)e, std::string("vc_attention_bwd_2s: event: ") + hipGetErrorString(e));
        }
    }
    attn_bwd_dkdv_kernel<<<grid, 256, 0, stream>>>(qkv, ld, dout, lddo, lse, delta, (int)S, (int)H, dqkv, lddq);
    attn_bwd_dq_kernel<<<grid, 256, 0, two ? stream2 : stream>>>(qkv, ld, dout, lddo, lse, delta, (int)S, (int)H, dqkv,
                                                                 lddq);
    if (two) {
        hipError_t e = hipEventRecord(e_dq, stream2);
        if (e == hipSuccess) e = hipStreamWaitEvent(stream, e_dq, 0);
        (void)hipEventDestroy(e_prep);  // released once complete
        (void)hipEventDestroy(e_dq);
        if (e != hipSuccess) return fail((int)e, std::string("vc_attention_bwd_2s: event: ") + hipGetErrorString(e));
    }
    return check_launch("vc_attention_bwd");
}
