// Fused joint space-time attention forward (flash-style), head_dim 64, bf16 MFMA.
//
// Replaces eager_attention_forward of ViViT (TF5/models/vivit/modeling_vivit.py:149-174):
// softmax(scale * Q K^T) V per (clip, head) over all S = 1 + 16*14*14 = 3137 tokens,
// without materialising the S x S scores (472 MB fp32 per clip per layer in the eager path).
//
// gfx950 structure (cdna_hip_programming.md Appendix B "Fused attention prefill"):
//   * workgroup = 4 waves = 128 query rows of one (clip, head); wave = 32 rows;
//   * K/V tiles of 64 keys staged by LDS-DMA (global_load_lds, issued from inline asm so
//     hipcc's LDS wait counts stay exact) into a 3-slot ring; a counted vmcnt retires only
//     the next tile, one raw s_barrier per tile; K image XOR-swizzled for ds_read_b128,
//     V image swizzled for the ds_read_b64_tr_b16 transpose read;
//   * swapped QK^T (S^T = K . Q^T): a query's scores live in ONE lane column, so the row
//     max needs one cross-half exchange and only on the rare rescale path;
//   * the running row max enters the QK^T MFMA chain as its initial accumulator
//     (S' = Q.K^T*c - m, with c = scale*log2 e folded into Q), so the common path per
//     score is max3 + exp2 + add + cvt; the max is re-based only when a score exceeds
//     it by more than THR (defer-max, cdna_hip_programming.md T13: P <= 2^THR);
//   * S'^T accumulator registers feed P.V directly as the B operand of O^T = V^T . P^T
//     (§3 "An accumulator tile as the next MFMA's operand"); P never touches LDS;
//   * output rows widened to 16-byte stores with v_permlane32_swap (T21).
#include "common.hpp"

namespace vc {

constexpr int AQ = 128;  // query rows per workgroup
constexpr int AK = 64;   // keys per tile
constexpr int KV_TILE_BYTES = AK * 64 * 2;  // 8 KiB (one of K or V)
constexpr int KV_SLOT = 2 * KV_TILE_BYTES;  // K then V
constexpr int NSLOT = 3;
constexpr float THR = 8.0f;  // log2-domain headroom before the running max is re-based (2^THR = 256)

__device__ __forceinline__ int kswz(int r, int c) { return c ^ ((r >> 1) & 7); }
__device__ __forceinline__ int vswz(int r, int c) { return c ^ (((r >> 1) & 1) << 2); }

__device__ __forceinline__ void adma16(const void* gsrc, uint32_t lds_addr) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(gsrc), "s"(lds_addr)
                 : "memory");
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

template <int ABL>  // timing ablations: 1 no loop loads, 2 no exp, 4 no PV MFMA, 8 no QK MFMA
__global__ void __launch_bounds__(256, 2)
attn_fwd_d64_kernel(const uint16_t* __restrict__ qkv, int64_t ld, int S, int H, float c_log2,
                    uint16_t* __restrict__ out, int64_t ldo) {
    __shared__ __attribute__((aligned(16))) char smem[NSLOT * KV_SLOT];

    const int qblk = blockIdx.x;
    const int bh = blockIdx.y;
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

    // ---- Q^T fragments (B operand of S^T = K.Q^T): lane holds Q[q=r][d = 16kk + 8h + 0..7],
    //      pre-scaled by c = scale*log2(e) so exp2 needs no multiply
    const int q = qblk * AQ + wave * 32 + r;
    const int qc = q < S ? q : S - 1;
    v8bf qf[4];
    {
        const uint16_t* qrow = qbase + (tok0 + qc) * ld + 8 * h;
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
            const v8s raw = *reinterpret_cast<const v8s*>(qrow + 16 * kk);
            if (c_log2 == 1.0f) {
                qf[kk] = __builtin_bit_cast(v8bf, raw);  // producer folded the scale into q
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) qf[kk][j] = (__bf16)(bf2f((unsigned short)raw[j]) * c_log2);
            }
        }
    }

    // staging: 64 key rows of K and V (8 rows x 128 B per wave-instruction), wave w: rows 16w..16w+15
    const int srow = wave * 16 + (lane >> 3), spc = lane & 7;
    const uint16_t* ksrc0 = kbase + (int64_t)srow * ld + kswz(srow, spc) * 8;
    const uint16_t* ksrc1 = kbase + (int64_t)(srow + 8) * ld + kswz(srow + 8, spc) * 8;
    const uint16_t* vsrc0 = vbase + (int64_t)srow * ld + vswz(srow, spc) * 8;
    const uint16_t* vsrc1 = vbase + (int64_t)(srow + 8) * ld + vswz(srow + 8, spc) * 8;
    auto stage = [&](int t) {
        const uint32_t s = lds0 + (t % NSLOT) * KV_SLOT + wave * 16 * 128;
        const int64_t off = (int64_t)t * AK * ld;
        adma16(ksrc0 + off, __builtin_amdgcn_readfirstlane(s));
        adma16(ksrc1 + off, __builtin_amdgcn_readfirstlane(s + 8 * 128));
        adma16(vsrc0 + off, __builtin_amdgcn_readfirstlane(s + KV_TILE_BYTES));
        adma16(vsrc1 + off, __builtin_amdgcn_readfirstlane(s + KV_TILE_BYTES + 8 * 128));
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

    v16f o0, o1;  // O^T[d][q]: d-block 0 and 1
#pragma unroll
    for (int e = 0; e < 16; ++e) { o0[e] = 0.f; o1[e] = 0.f; }
    v16f minit;  // -running max of this lane's query, broadcast: initial accumulator of S'
#pragma unroll
    for (int e = 0; e < 16; ++e) minit[e] = 0.f;
    float m_run = 0.f, l_run = 0.f;

    const int ntiles = (S + AK - 1) / AK;
    stage(0);
    if (ntiles > 1) {
        stage(1);
        attn_wait_vm<4>();
    } else {
        attn_wait_vm<0>();
    }
    attn_sync();

    for (int t = 0; t < ntiles; ++t) {
        if (!(ABL & 1) && t + 2 < ntiles) stage(t + 2);
        const char* slot = smem + (t % NSLOT) * KV_SLOT;

        // ---- S'^T = K . Q'^T - m_run for the two 32-key blocks (-m_run enters as the C operand)
        v16f s0, s1;
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
            const v8bf k0 = __builtin_bit_cast(v8bf, *reinterpret_cast<const v8s*>(slot + koff[kk]));
            const v8bf k1 = __builtin_bit_cast(v8bf, *reinterpret_cast<const v8s*>(slot + koff[kk] + 4096));
            if constexpr (ABL & 8) {
                asm volatile("" ::"v"(k0), "v"(k1));
                if (kk == 0) { s0 = minit; s1 = minit; }
            } else {
                s0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(k0, qf[kk], kk == 0 ? minit : s0, 0, 0, 0);
                s1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(k1, qf[kk], kk == 0 ? minit : s1, 0, 0, 0);
            }
        }
        // ---- mask keys beyond S (last tile only)
        const int kv0 = t * AK;
        if (kv0 + AK > S) {
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int key = (e & 3) + 8 * (e >> 2) + 4 * h;
                if (kv0 + key >= S) s0[e] = -INFINITY;
                if (kv0 + 32 + key >= S) s1[e] = -INFINITY;
            }
        }

        // ---- online softmax: scores are already relative to m_run; re-base only when a row
        //      grew by more than THR (tile 0 always establishes m_run)
        float mx = fmaxf(fmaxf(s0[0], s0[1]), fmaxf(s1[0], s1[1]));
#pragma unroll
        for (int e = 2; e < 16; e += 2) mx = fmaxf(mx, fmaxf(fmaxf(s0[e], s0[e + 1]), fmaxf(s1[e], s1[e + 1])));
        if (t == 0 || __any(mx > THR)) {
            const float rowmax = fmaxf(mx, __shfl_xor(mx, 32, 64));
            const float delta = (t == 0) ? rowmax : fmaxf(rowmax, 0.f);
            const float alpha = (t == 0) ? 0.f : __builtin_amdgcn_exp2f(-delta);
            m_run = (t == 0) ? rowmax : m_run + delta;
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                s0[e] -= delta;
                s1[e] -= delta;
                o0[e] *= alpha;
                o1[e] *= alpha;
                minit[e] = -m_run;
            }
            l_run *= alpha;
        }
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            if constexpr (!(ABL & 2)) {
                s0[e] = __builtin_amdgcn_exp2f(s0[e]);
                s1[e] = __builtin_amdgcn_exp2f(s1[e]);
            }
        }
        float a0 = (s0[0] + s0[1]) + (s0[2] + s0[3]), a1 = (s0[4] + s0[5]) + (s0[6] + s0[7]);
        float a2 = (s0[8] + s0[9]) + (s0[10] + s0[11]), a3 = (s0[12] + s0[13]) + (s0[14] + s0[15]);
        float b0 = (s1[0] + s1[1]) + (s1[2] + s1[3]), b1 = (s1[4] + s1[5]) + (s1[6] + s1[7]);
        float b2 = (s1[8] + s1[9]) + (s1[10] + s1[11]), b3 = (s1[12] + s1[13]) + (s1[14] + s1[15]);
        l_run += ((a0 + a1) + (a2 + a3)) + ((b0 + b1) + (b2 + b3));

        // ---- O^T += V^T . P^T: P fragment of (block kb, k-step s2) = regs 8s2..8s2+7 as bf16
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
                v8bf pf;
#pragma unroll
                for (int jj = 0; jj < 8; ++jj) pf[jj] = (__bf16)(kb == 0 ? s0[8 * s2 + jj] : s1[8 * s2 + jj]);
#pragma unroll
                for (int db = 0; db < 2; ++db) {
                    const char* pa = slot + voff[db] + (kb * 32 + 16 * s2) * 128;
                    v4s va = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)pa);
                    v4s vb = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(pa + 8 * 128));
                    v8s vv;
                    vv[0] = va[0]; vv[1] = va[1]; vv[2] = va[2]; vv[3] = va[3];
                    vv[4] = vb[0]; vv[5] = vb[1]; vv[6] = vb[2]; vv[7] = vb[3];
                    const v8bf vf = __builtin_bit_cast(v8bf, vv);
                    if constexpr (ABL & 4) {
                        asm volatile("" ::"v"(vf), "v"(pf));
                    } else if (db == 0) {
                        o0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf, o0, 0, 0, 0);
                    } else {
                        o1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf, o1, 0, 0, 0);
                    }
                }
            }

        // ---- retire tile t+1 (t+2 may stay in flight), then every wave passes the barrier
        if (t + 1 < ntiles) {
            if (t + 2 < ntiles) attn_wait_vm<4>();
            else attn_wait_vm<0>();
            attn_sync();
        }
    }

    // ---- normalise and store O[q][d]: reg 4g+e of block db -> d = 32db + 8g + 4h + e;
    //      lane pairs (h=0/1) swap halves so each lane stores 16 contiguous bytes
    const float l_tot = l_run + __shfl_xor(l_run, 32, 64);
    const float inv = 1.0f / l_tot;
    unsigned pk[2][4][2];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        pk[0][g][0] = pack2bf(o0[4 * g + 0] * inv, o0[4 * g + 1] * inv);
        pk[0][g][1] = pack2bf(o0[4 * g + 2] * inv, o0[4 * g + 3] * inv);
        pk[1][g][0] = pack2bf(o1[4 * g + 0] * inv, o1[4 * g + 1] * inv);
        pk[1][g][1] = pack2bf(o1[4 * g + 2] * inv, o1[4 * g + 3] * inv);
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

}  // namespace vc

using namespace vc;

extern "C" int vc_attention_fwd(const uint16_t* qkv, int64_t ld, int64_t B, int64_t S, int64_t H, int64_t head_dim,
                                float scale, int q_prescaled, uint16_t* out, int64_t ldo, hipStream_t stream) {
    if (!qkv || !out) return fail(VC_ERR_INVALID_ARG, "vc_attention_fwd: null pointer");
    if (head_dim != 64) return fail(VC_ERR_UNSUPPORTED, "vc_attention_fwd: head_dim must be 64");
    if (B <= 0 || S <= 0 || H <= 0 || ld < 3 * H * 64 || ldo < H * 64 || ld % 8 || ldo % 8)
        return fail(VC_ERR_INVALID_ARG, "vc_attention_fwd: bad shape / leading dimension");
    if ((((uintptr_t)qkv) | ((uintptr_t)out)) & 15)
        return fail(VC_ERR_INVALID_ARG, "vc_attention_fwd: pointers must be 16-byte aligned");
    if (B * H > 65535 || S > (1 << 24)) return fail(VC_ERR_INVALID_ARG, "vc_attention_fwd: grid too large");
    const float c_log2 = q_prescaled ? 1.0f : scale * 1.4426950408889634f;
    dim3 grid((unsigned)((S + AQ - 1) / AQ), (unsigned)(B * H));
    attn_fwd_d64_kernel<0><<<grid, 256, 0, stream>>>(qkv, ld, (int)S, (int)H, c_log2, out, ldo);
    return check_launch("vc_attention_fwd");
}

// Timing-only ablations of the attention kernel (results are wrong by design).
extern "C" int vc_attention_fwd_ablation(const uint16_t* qkv, int64_t ld, int64_t B, int64_t S, int64_t H,
                                         float scale, uint16_t* out, int64_t ldo, int abl, hipStream_t stream) {
    const float c_log2 = scale * 1.4426950408889634f;
    dim3 grid((unsigned)((S + AQ - 1) / AQ), (unsigned)(B * H));
#define VC_ABL(N) case N: attn_fwd_d64_kernel<N><<<grid, 256, 0, stream>>>(qkv, ld, (int)S, (int)H, c_log2, out, ldo); break;
    switch (abl) {
        VC_ABL(0) VC_ABL(1) VC_ABL(2) VC_ABL(4) VC_ABL(6) VC_ABL(8) VC_ABL(12) VC_ABL(14) VC_ABL(15)
        default: return fail(VC_ERR_INVALID_ARG, "bad ablation");
    }
#undef VC_ABL
    return check_launch("vc_attention_fwd_ablation");
}
