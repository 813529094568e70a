// Backward of the Video Swin 3D shifted-window attention, head_dim 32 (the Swin3D train step:
// videoswintransformer/swin_video_classifier/trainers/trainer.py:105-122 runs loss.backward()
// through torchvision's shifted_window_attention_3d).
//
// Forward (window.hip, log2 domain): S' = q'.k + b2[idx(q,k)] (-inf between shift regions and on
// padded keys), P = exp2(S' - lse2), with q' = q * d^-1/2 * log2 e as the q|k|v buffer stores it
// and b2 = the relative-position bias table * log2 e.  In natural units s = ln2 * q'.k + b, so with
// dO the output gradient and Delta = rowsum(dO o O):
//     dV = P^T dO,   dP = dO V^T,   G = ds = P o (dP - Delta),
//     dq' = ln2 * G K,   dK = ln2 * G^T q',   dtable[idx(q,k)] += G[q][k]   (over windows, clips).
//
// One workgroup (8 waves) per (window, head): the window's q', K, V and dO rows are gathered by
// index (the forward's roll / partition read; window_common.hpp) into LDS once (4 x 28 KB at 448
// padded tokens), with each query's lse and Delta, each token's relative-position code and
// region label, the head's bias-table column and a private dtable accumulator.  Phase 1: each wave owns 32-key blocks and loops over the query blocks
// (S and dP with the key block in registers, dV^T and dK^T accumulated by MFMAs whose other
// operand is a transposed LDS read); phase 2: each wave owns 32-query blocks for dq'^T.  The bias
// gradient is summed per (window, head) into the LDS table by ds_add_f32 (its order within a
// workgroup is not fixed: the table gradient is reproducible to fp32 rounding, not bit for bit)
// and written out per workgroup; the host reduces the partials over windows (vc_colsum, fixed
// order).  dq'|dk|dv rows are written exactly once (the windows partition the tokens).
#include "window_common.hpp"

#include <cmath>

namespace vc {
namespace wbwd {

constexpr float LN2 = 0.6931471805599453f;
constexpr float LOG2E = 1.4426950408889634f;
constexpr int NPMAX = 448;

// transposed fragment of a 64-B-row LDS image (ds_read_b64_tr_b16, rows +0 / +8)
__device__ __forceinline__ v8s tr_frag(const char* img, int offa, int offb) {
    const v4s va = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(img + offa));
    const v4s vb = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(img + offb));
    v8s vv;
    vv[0] = va[0]; vv[1] = va[1]; vv[2] = va[2]; vv[3] = va[3];
    vv[4] = vb[0]; vv[5] = vb[1]; vv[6] = vb[2]; vv[7] = vb[3];
    return vv;
}

// accumulator registers 8s2 .. 8s2+7 as a bf16 MFMA operand
__device__ __forceinline__ v8s bf8_of(const v16f& x, int s2) {
    v4u u;
#pragma unroll
    for (int j = 0; j < 4; ++j) u[j] = pack2bf(x[8 * s2 + 2 * j], x[8 * s2 + 2 * j + 1]);
    return __builtin_bit_cast(v8s, u);
}

// store a [32 d (registers)][lane] accumulator as one 64-B bf16 row per lane (x scale): register
// 4g+e holds d = 8g + 4h + e; lane pairs swap halves so each lane writes two 16-B pieces
__device__ __forceinline__ void store_row32(uint16_t* row, const v16f& acc, float scale, int h) {
    unsigned pk[4][2];
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
        pk[g4][0] = pack2bf(acc[4 * g4 + 0] * scale, acc[4 * g4 + 1] * scale);
        pk[g4][1] = pack2bf(acc[4 * g4 + 2] * scale, acc[4 * g4 + 3] * scale);
    }
#pragma unroll
    for (int g4 = 0; g4 < 4; g4 += 2) {
        auto x0 = __builtin_amdgcn_permlane32_swap(pk[g4][0], pk[g4 + 1][0], false, false);
        auto x1 = __builtin_amdgcn_permlane32_swap(pk[g4][1], pk[g4 + 1][1], false, false);
        uint4 v;
        v.x = x0[0]; v.y = x1[0]; v.z = x0[1]; v.w = x1[1];
        *reinterpret_cast<uint4*>(row + g4 * 8 + h * 8) = v;
    }
}

__global__ void __launch_bounds__(512, 1)
window_attn_bwd_d32_kernel(const uint16_t* __restrict__ qkv, int64_t ld, const uint16_t* __restrict__ out,
                           int64_t ldo, const uint16_t* __restrict__ dout, int64_t lddo, const float* __restrict__ lse,
                           WinGeom g, FullWin fw, int heads, int vol, int NP, const float* __restrict__ table, int ntab,
                           int masked, uint16_t* __restrict__ dqkv, int64_t lddq, float* __restrict__ dtab_part) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* Qs = smem;
    char* Ks = Qs + NP * 64;
    char* Vs = Ks + NP * 64;
    char* Ds = Vs + NP * 64;
    float* lse_s = reinterpret_cast<float*>(Ds + NP * 64);
    float* del_s = lse_s + NP;
    float* btab = del_s + NP;
    float* dtab = btab + ntab;
    int* cl_s = reinterpret_cast<int*>(dtab + ntab);  // per token: rel_code << 4 | region label (15: padding)

    const int head = blockIdx.y;
    const int nwin = g.nwt * g.nwh * g.nww;
    const int b = blockIdx.x / nwin;
    int rr = blockIdx.x - b * nwin;
    const int wi_t = rr / (g.nwh * g.nww);
    rr -= wi_t * g.nwh * g.nww;
    const int wi_h = rr / g.nww, wi_w = rr - (rr / g.nww) * g.nww;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int C = heads * 32;
    auto token_row = [&](int n, int* label) -> int64_t { return win_token_row(g, b, wi_t, wi_h, wi_w, n, label); };

    // ---- stage q', k, v, dO rows (swizzled 16-B chunks), lse, Delta, labels, the bias column
    for (int c = tid; c < NP * 4; c += 512) {
        const int n = c >> 2, ch = c & 3;
        uint4 qv = make_uint4(0, 0, 0, 0), kv = qv, vv = qv, dv = qv;
        if (n < vol) {
            const int64_t row = token_row(n, nullptr);
            const uint16_t* src = qkv + row * ld + head * 32 + ch * 8;
            qv = *reinterpret_cast<const uint4*>(src);
            kv = *reinterpret_cast<const uint4*>(src + C);
            vv = *reinterpret_cast<const uint4*>(src + 2 * C);
            dv = *reinterpret_cast<const uint4*>(dout + row * lddo + head * 32 + ch * 8);
        }
        const int off = n * 64 + kchunk_swz(n, ch) * 16;
        *reinterpret_cast<uint4*>(Qs + off) = qv;
        *reinterpret_cast<uint4*>(Ks + off) = kv;
        *reinterpret_cast<uint4*>(Vs + off) = vv;
        *reinterpret_cast<uint4*>(Ds + off) = dv;
    }
    for (int n = tid; n < NP; n += 512) {
        float l = INFINITY, d = 0.f;  // padded queries: P = exp2(-inf) = 0
        if (n < vol) {
            const int64_t row = token_row(n, nullptr);
            l = lse[row * heads + head];
            const uint4* a = reinterpret_cast<const uint4*>(dout + row * lddo + head * 32);
            const uint4* o = reinterpret_cast<const uint4*>(out + row * ldo + head * 32);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint4 x = a[j], y = o[j];
                const unsigned xs[4] = {x.x, x.y, x.z, x.w}, ys[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    d += bf2f((unsigned short)(xs[k] & 0xffff)) * bf2f((unsigned short)(ys[k] & 0xffff));
                    d += bf2f((unsigned short)(xs[k] >> 16)) * bf2f((unsigned short)(ys[k] >> 16));
                }
            }
        }
        lse_s[n] = l;
        del_s[n] = d;
    }
    for (int i = tid; i < ntab; i += 512) {
        btab[i] = table[(int64_t)i * heads + head] * LOG2E;
        dtab[i] = 0.f;
    }
    for (int n = tid; n < NP; n += 512) {
        int lb = 15, code = 0;
        if (n < vol) {
            lb = 0;
            if (masked) token_row(n, &lb);
            code = rel_code(n, fw);
        }
        cl_s[n] = code * 16 + lb;
    }
    __syncthreads();

    const int r = lane & 31, h = lane >> 5;
    const int code_max = rel_code_max(fw);  // window_common.hpp: idx(q, k) = code(q) - code(k) + code_max
    // row-fragment offsets (lane (r, h): row r of a 32-row block, chunk 2kk + h) and transposed
    // offsets (rows 4h + tq and +8 of a 16-row k-step, columns gcol .. gcol+3); the swizzle term of
    // both depends only on the row mod 16, so block / k-step offsets are plain multiples of 64 B
    int roff[2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) roff[kk] = r * 64 + kchunk_swz(r, 2 * kk + h) * 16;
    const int gi = lane & 15, tq = gi >> 2, tp = gi & 3;
    const int gcol = ((lane >> 4) & 1) * 16 + tp * 4;
    const int ra = 4 * h + tq, rb = ra + 8;
    const int toa = ra * 64 + kchunk_swz(ra, gcol >> 3) * 16 + (gcol & 7) * 2;
    const int tob = rb * 64 + kchunk_swz(rb, gcol >> 3) * 16 + (gcol & 7) * 2;
    const int nblk = (vol + 31) / 32;

    // ---- phase 1: dK, dV (and the bias gradient) per 32-key block
    for (int kb = wave; kb < nblk; kb += 8) {
        const int key = kb * 32 + r;
        v8s kf[2], vf[2];
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            kf[kk] = *reinterpret_cast<const v8s*>(Ks + kb * 32 * 64 + roff[kk]);
            vf[kk] = *reinterpret_cast<const v8s*>(Vs + kb * 32 * 64 + roff[kk]);
        }
        const int ckl = cl_s[key];  // padded key: label 15 (matches no query: every query is masked)
        const int klab = ckl & 15, kbase = code_max - (ckl >> 4);
        v16f dvacc = {}, dkacc = {};
        for (int qb = 0; qb < nblk; ++qb) {
            // S[q][key] - lse[q] + bias: register i holds query 32qb + (i & 3) + 8(i >> 2) + 4h
            v16f s, dp;
            int idx[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int q = qb * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
                const int cq = cl_s[q];
                const bool ok = key < vol && (cq & 15) == klab;  // padded q: label 15, never a real key's
                idx[i] = ok ? (cq >> 4) + kbase : -1;
                s[i] = ok ? btab[idx[i]] - lse_s[q] : -INFINITY;
                dp[i] = -del_s[q];
            }
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) {
                const v8s qa = *reinterpret_cast<const v8s*>(Qs + qb * 32 * 64 + roff[kk]);
                const v8s da = *reinterpret_cast<const v8s*>(Ds + qb * 32 * 64 + roff[kk]);
                s = mfma32x16<VC_ELEM_BF16>(qa, kf[kk], s);
                dp = mfma32x16<VC_ELEM_BF16>(da, vf[kk], dp);
            }
            v16f p;
#pragma unroll
            for (int i = 0; i < 16; ++i) p[i] = __builtin_amdgcn_exp2f(s[i]);
            v16f gr;
#pragma unroll
            for (int i = 0; i < 16; ++i) gr[i] = p[i] * dp[i];
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
                const int kr = (qb * 32 + 16 * s2) * 64;
                // dV^T[d][key] += dO^T P,  dK^T[d][key] += q'^T G
                dvacc = mfma32x16<VC_ELEM_BF16>(tr_frag(Ds, toa + kr, tob + kr), bf8_of(p, s2), dvacc);
                dkacc = mfma32x16<VC_ELEM_BF16>(tr_frag(Qs, toa + kr, tob + kr), bf8_of(gr, s2), dkacc);
            }
#pragma unroll
            for (int i = 0; i < 16; ++i)
                if (idx[i] >= 0) atomicAdd(&dtab[idx[i]], gr[i]);
        }
        if (key < vol) {
            uint16_t* drow = dqkv + token_row(key, nullptr) * lddq + head * 32;
            store_row32(drow + C, dkacc, LN2, h);
            store_row32(drow + 2 * C, dvacc, 1.0f, h);
        }
    }

    // ---- phase 2: dq' per 32-query block
    for (int qb = wave; qb < nblk; qb += 8) {
        const int q = qb * 32 + r;
        v8s qf[2], df[2];
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            qf[kk] = *reinterpret_cast<const v8s*>(Qs + qb * 32 * 64 + roff[kk]);
            df[kk] = *reinterpret_cast<const v8s*>(Ds + qb * 32 * 64 + roff[kk]);
        }
        const int cql = cl_s[q];
        const int qlab = q < vol ? (cql & 15) : 14, qbase = (cql >> 4) + code_max;
        const float lq = lse_s[q], dq_delta = del_s[q];
        v16f dqacc = {};
        for (int kb = 0; kb < nblk; ++kb) {
            // S^T[key][q]: register i holds key 32kb + (i & 3) + 8(i >> 2) + 4h
            v16f st, dpt;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int key = kb * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
                const int ck = cl_s[key];
                const bool ok = (ck & 15) == qlab;  // padded key (15) or padded query (14): masked
                st[i] = ok ? btab[qbase - (ck >> 4)] - lq : -INFINITY;
                dpt[i] = -dq_delta;
            }
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) {
                const v8s ka = *reinterpret_cast<const v8s*>(Ks + kb * 32 * 64 + roff[kk]);
                const v8s va = *reinterpret_cast<const v8s*>(Vs + kb * 32 * 64 + roff[kk]);
                st = mfma32x16<VC_ELEM_BF16>(ka, qf[kk], st);
                dpt = mfma32x16<VC_ELEM_BF16>(va, df[kk], dpt);
            }
            v16f gt;
#pragma unroll
            for (int i = 0; i < 16; ++i) gt[i] = __builtin_amdgcn_exp2f(st[i]) * dpt[i];
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
                const int kr = (kb * 32 + 16 * s2) * 64;
                dqacc = mfma32x16<VC_ELEM_BF16>(tr_frag(Ks, toa + kr, tob + kr), bf8_of(gt, s2), dqacc);  // dq'^T += K^T G^T
            }
        }
        if (q < vol) store_row32(dqkv + token_row(q, nullptr) * lddq + head * 32, dqacc, LN2, h);
    }
    __syncthreads();
    float* part = dtab_part + ((int64_t)blockIdx.x * heads + head) * ntab;
    for (int i = tid; i < ntab; i += 512) part[i] = dtab[i];
}

}  // namespace wbwd
}  // namespace vc

using namespace vc;
using namespace vc::wbwd;

extern "C" int vc_window_attention3d_bwd(const uint16_t* qkv, int64_t ld, const uint16_t* out, int64_t ldo,
                                         const uint16_t* dout, int64_t lddo, const float* lse, int64_t B, int64_t T,
                                         int64_t H, int64_t W, int64_t heads, int64_t head_dim, int wt, int wh, int ww,
                                         int st, int sh, int sw, int full_t, int full_h, int full_w, const float* table,
                                         uint16_t* dqkv, int64_t lddq, float* dtable_part, hipStream_t stream) {
    if (!qkv || !out || !dout || !lse || !table || !dqkv || !dtable_part)
        return fail(VC_ERR_INVALID_ARG, "vc_window_attention3d_bwd: null pointer");
    if (head_dim != 32) return fail(VC_ERR_UNSUPPORTED, "vc_window_attention3d_bwd: head_dim must be 32");
    if (wt <= 0 || wh <= 0 || ww <= 0 || T % wt || H % wh || W % ww)
        return fail(VC_ERR_UNSUPPORTED, "vc_window_attention3d_bwd: the token grid must be whole windows");
    if (st < 0 || sh < 0 || sw < 0 || st >= wt || sh >= wh || sw >= ww)
        return fail(VC_ERR_INVALID_ARG, "vc_window_attention3d_bwd: shift must be in [0, window)");
    if (wt > full_t || wh > full_h || ww > full_w)
        return fail(VC_ERR_INVALID_ARG, "vc_window_attention3d_bwd: window larger than the full window");
    const int vol = wt * wh * ww;
    const int NP = (vol + 63) / 64 * 64;
    if (NP > NPMAX) return fail(VC_ERR_UNSUPPORTED, "vc_window_attention3d_bwd: window volume > 448");
    if (ld < 3 * heads * 32 || lddq < 3 * heads * 32 || ldo < heads * 32 || lddo < heads * 32 || ld % 8 || ldo % 8 ||
        lddo % 8 || lddq % 8 || ((uintptr_t)qkv | (uintptr_t)out | (uintptr_t)dout | (uintptr_t)dqkv) & 15)
        return fail(VC_ERR_INVALID_ARG, "vc_window_attention3d_bwd: bad leading dimension / alignment");
    const int ntab = (2 * full_t - 1) * (2 * full_h - 1) * (2 * full_w - 1);
    const size_t lds = (size_t)4 * NP * 64 + 3 * NP * 4 + 2 * (size_t)ntab * 4;
    if (lds > 160 * 1024) return fail(VC_ERR_UNSUPPORTED, "vc_window_attention3d_bwd: window / table too large for LDS");
    WinGeom g{(int)T, (int)H, (int)W, wt, wh, ww, st, sh, sw, (int)(T / wt), (int)(H / wh), (int)(W / ww)};
    const int64_t nwin = B * g.nwt * g.nwh * g.nww;
    if (nwin > 0x7fffffff || heads > 65535) return fail(VC_ERR_INVALID_ARG, "vc_window_attention3d_bwd: grid too large");
    static bool attr = false;
    if (!attr) {
        hipError_t e = hipFuncSetAttribute((const void*)window_attn_bwd_d32_kernel,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if (e != hipSuccess) return fail((int)e, std::string("vc_window_attention3d_bwd: ") + hipGetErrorString(e));
        attr = true;
    }
    const FullWin fw{full_t, full_h, full_w};
    const int mk = (st | sh | sw) ? 1 : 0;
    window_attn_bwd_d32_kernel<<<dim3((unsigned)nwin, (unsigned)heads), 512, lds, stream>>>(
        qkv, ld, out, ldo, dout, lddo, lse, g, fw, (int)heads, vol, NP, table, ntab, mk, dqkv, lddq, dtable_part);
    return check_launch("vc_window_attention3d_bwd");
}
