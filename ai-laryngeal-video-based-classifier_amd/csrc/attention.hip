// Fused joint space-time attention forward (flash-style), head_dim 64, bf16 MFMA.
//
// Replaces eager_attention_forward of ViViT (TF5/models/vivit/modeling_vivit.py:149-174):
// softmax(scale * Q K^T) V per (clip, head) over all S = 1 + 16*14*14 = 3137 tokens,
// without materialising the S x S scores (472 MB fp32 per clip per layer in the eager path).
//
// gfx950 structure (cdna_hip_programming.md Appendix B "Fused attention prefill"):
//   * workgroup = 4 waves = 128 query rows of one (clip, head); wave = 32 rows;
//   * K/V tiles of 64 keys staged by global_load_lds into a 2-deep LDS ring;
//     K image XOR-swizzled for ds_read_b128, V image swizzled for ds_read_b64_tr_b16;
//   * swapped QK^T (S^T = K . Q^T): the score column of a query lives in ONE lane,
//     so the online-softmax row max / sum need a single cross-half exchange;
//   * S^T accumulator registers feed P.V directly as the B operand of O^T = V^T . P^T
//     (§3 "An accumulator tile as the next MFMA's operand"), V^T fragments come from the
//     hardware transpose read — P never touches LDS;
//   * exp2 with the softmax scale folded into one FMA per score; running max/sum in fp32.
#include "common.hpp"

namespace vc {

constexpr int AQ = 128;  // query rows per workgroup
constexpr int AK = 64;   // keys per tile
constexpr int KV_TILE_BYTES = AK * 64 * 2;  // 8 KiB (one of K or V)

__device__ __forceinline__ int kswz(int r, int c) { return c ^ ((r >> 1) & 7); }
__device__ __forceinline__ int vswz(int r, int c) { return c ^ (((r >> 1) & 1) << 2); }

__device__ __forceinline__ void glds16a(const void* gsrc, void* lds_base) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)gsrc,
                                     (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}

// Stage 64 key rows (K and V of head hh) starting at token row `row0` into one ring slot.
// 8 wave-instructions per operand (8 rows x 128 B each); wave w issues rows [16w, 16w+16).
__device__ __forceinline__ void stage_kv(const uint16_t* __restrict__ kbase, const uint16_t* __restrict__ vbase,
                                         int64_t ld, int64_t row0, char* slot, int wave, int lane) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int row = wave * 16 + i * 8 + (lane >> 3);
        const int pc = lane & 7;
        const uint16_t* ks = kbase + (row0 + row) * ld + kswz(row, pc) * 8;
        const uint16_t* vs = vbase + (row0 + row) * ld + vswz(row, pc) * 8;
        glds16a(ks, slot + (wave * 16 + i * 8) * 128);
        glds16a(vs, slot + KV_TILE_BYTES + (wave * 16 + i * 8) * 128);
    }
}

__global__ void __launch_bounds__(256, 2)
attn_fwd_d64_kernel(const uint16_t* __restrict__ qkv, int64_t ld, int S, int H, float c_log2,
                    uint16_t* __restrict__ out, int64_t ldo) {
    __shared__ __attribute__((aligned(16))) char smem[4 * KV_TILE_BYTES];

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

    // ---- Q^T fragments (B operand of S^T = K.Q^T): lane holds Q[q=r][d = 16kk + 8h + 0..7]
    const int q = qblk * AQ + wave * 32 + r;
    const int qc = q < S ? q : S - 1;
    v8bf qf[4];
    {
        const uint16_t* qrow = qbase + (tok0 + qc) * ld + 8 * h;
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) qf[kk] = __builtin_bit_cast(v8bf, *reinterpret_cast<const v8s*>(qrow + 16 * kk));
    }

    v16f o0, o1;  // O^T[d][q]: d-block 0 and 1
#pragma unroll
    for (int e = 0; e < 16; ++e) { o0[e] = 0.f; o1[e] = 0.f; }
    float m_run = -INFINITY, l_run = 0.f;

    const int ntiles = (S + AK - 1) / AK;
    stage_kv(kbase, vbase, ld, 0, smem, wave, lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    // per-lane constant parts of the V^T transpose-read address (16-lane group geometry)
    const int gi = lane & 15;               // lane within its 16-lane group
    const int tq = gi >> 2, tp = gi & 3;    // row q and column quad p it addresses
    const int gcol = ((lane >> 4) & 1) * 16 + tp * 4;  // column inside a 32-wide d block

    for (int t = 0; t < ntiles; ++t) {
        char* Kt = smem + (t & 1) * 2 * KV_TILE_BYTES;
        char* Vt = Kt + KV_TILE_BYTES;
        if (t + 1 < ntiles) stage_kv(kbase, vbase, ld, (int64_t)(t + 1) * AK, smem + ((t + 1) & 1) * 2 * KV_TILE_BYTES, wave, lane);

        // ---- S^T = K . Q^T for two 32-key blocks
        v16f s0, s1;
#pragma unroll
        for (int e = 0; e < 16; ++e) { s0[e] = 0.f; s1[e] = 0.f; }
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
            const int ch = kk * 2 + h;
            const int r0 = r, r1 = 32 + r;
            v8bf k0 = __builtin_bit_cast(v8bf, *reinterpret_cast<const v8s*>(Kt + r0 * 128 + kswz(r0, ch) * 16));
            v8bf k1 = __builtin_bit_cast(v8bf, *reinterpret_cast<const v8s*>(Kt + r1 * 128 + kswz(r1, ch) * 16));
            s0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(k0, qf[kk], s0, 0, 0, 0);
            s1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(k1, qf[kk], s1, 0, 0, 0);
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

        // ---- online softmax (one query per lane column; halves h=0/1 hold 16+16 keys each)
        float mx = s0[0];
#pragma unroll
        for (int e = 1; e < 16; ++e) mx = fmaxf(mx, s0[e]);
#pragma unroll
        for (int e = 0; e < 16; ++e) mx = fmaxf(mx, s1[e]);
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        const float m_new = fmaxf(m_run, mx);
        const float alpha = __builtin_amdgcn_exp2f((m_run - m_new) * c_log2);
        const float nb = -m_new * c_log2;
        float psum = 0.f;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            s0[e] = __builtin_amdgcn_exp2f(fmaf(s0[e], c_log2, nb));
            s1[e] = __builtin_amdgcn_exp2f(fmaf(s1[e], c_log2, nb));
            psum += s0[e] + s1[e];
        }
        l_run = l_run * alpha + psum;
        m_run = m_new;
#pragma unroll
        for (int e = 0; e < 16; ++e) { o0[e] *= alpha; o1[e] *= alpha; }

        // ---- P fragments: regs 8s..8s+7 of S^T block kb -> bf16 x8 (k-step s)
        v8bf pf[2][2];
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                pf[0][s][j] = (__bf16)s0[8 * s + j];
                pf[1][s][j] = (__bf16)s1[8 * s + j];
            }

        // ---- O^T += V^T . P^T  (V^T fragments via ds_read_b64_tr_b16)
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const int R0 = kb * 32 + 16 * s + 4 * h;
#pragma unroll
                for (int db = 0; db < 2; ++db) {
                    const int col = db * 32 + gcol;
                    const int ra = R0 + tq, rb = R0 + 8 + tq;
                    const char* pa = Vt + ra * 128 + vswz(ra, col >> 3) * 16 + (col & 7) * 2;
                    const char* pb = Vt + rb * 128 + vswz(rb, col >> 3) * 16 + (col & 7) * 2;
                    v4s va = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)pa);
                    v4s vb = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)pb);
                    v8s vv;
                    vv[0] = va[0]; vv[1] = va[1]; vv[2] = va[2]; vv[3] = va[3];
                    vv[4] = vb[0]; vv[5] = vb[1]; vv[6] = vb[2]; vv[7] = vb[3];
                    const v8bf vf = __builtin_bit_cast(v8bf, vv);
                    if (db == 0)
                        o0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf[kb][s], o0, 0, 0, 0);
                    else
                        o1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf[kb][s], o1, 0, 0, 0);
                }
            }

        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }

    // ---- normalise and store O[q][d]: reg 4g+e of block db -> d = 32db + 8g + 4h + e
    const float l_tot = l_run + __shfl_xor(l_run, 32, 64);
    const float inv = 1.0f / l_tot;
    if (q < S) {
        uint16_t* orow = out + (tok0 + q) * ldo + hh * 64;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            uint2 p0, p1;
            p0.x = pack2bf(o0[4 * g + 0] * inv, o0[4 * g + 1] * inv);
            p0.y = pack2bf(o0[4 * g + 2] * inv, o0[4 * g + 3] * inv);
            p1.x = pack2bf(o1[4 * g + 0] * inv, o1[4 * g + 1] * inv);
            p1.y = pack2bf(o1[4 * g + 2] * inv, o1[4 * g + 3] * inv);
            *reinterpret_cast<uint2*>(orow + 8 * g + 4 * h) = p0;
            *reinterpret_cast<uint2*>(orow + 32 + 8 * g + 4 * h) = p1;
        }
    }
}

}  // namespace vc

using namespace vc;

extern "C" int vc_attention_fwd(const uint16_t* qkv, int64_t ld, int64_t B, int64_t S, int64_t H, int64_t head_dim,
                                float scale, uint16_t* out, int64_t ldo, hipStream_t stream) {
    if (!qkv || !out) return fail(VC_ERR_INVALID_ARG, "vc_attention_fwd: null pointer");
    if (head_dim != 64) return fail(VC_ERR_UNSUPPORTED, "vc_attention_fwd: head_dim must be 64");
    if (B <= 0 || S <= 0 || H <= 0 || ld < 3 * H * 64 || ldo < H * 64 || ld % 8 || ldo % 4)
        return fail(VC_ERR_INVALID_ARG, "vc_attention_fwd: bad shape / leading dimension");
    if ((((uintptr_t)qkv) | ((uintptr_t)out)) & 15)
        return fail(VC_ERR_INVALID_ARG, "vc_attention_fwd: pointers must be 16-byte aligned");
    if (B * H > 65535 || S > (1 << 24)) return fail(VC_ERR_INVALID_ARG, "vc_attention_fwd: grid too large");
    const float c_log2 = scale * 1.4426950408889634f;
    dim3 grid((unsigned)((S + AQ - 1) / AQ), (unsigned)(B * H));
    attn_fwd_d64_kernel<<<grid, 256, 0, stream>>>(qkv, ld, (int)S, (int)H, c_log2, out, ldo);
    return check_launch("vc_attention_fwd");
}
