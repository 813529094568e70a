// Training-step kernels of the ViViT train step: the backward of every
// non-attention op of VivitLayer / VivitEmbeddings / the classifier, the weight-gradient GEMM,
// and the optimizer.  Reference: vivit_transformer/vivit_classifier/trainers/trainer.py:140-146
// (criterion(outputs.logits, labels); loss.backward(); optimizer.step()) with
// AdamW(lr 1e-3, weight_decay 0.01) from vivit_transformer/main.py:150-155.
//
// Every reduction is deterministic (fixed-order partial sums, no atomics), so a gradient is
// bit-identical run to run and across data-parallel replicas fed the same shard.
#include "common.hpp"

#include <type_traits>

#include <cstdlib>

#include <algorithm>
#include <cmath>

namespace vc {
namespace trn {

// ---------------------------------------------------------------------------------
// LayerNorm backward, fused with the residual-gradient add and its bf16 copy.
// One wave per row (D = 256*V), rows grid-strided; per-lane column partials of dgamma /
// dbeta in registers, combined across the 4 waves in LDS -> part[block][2][D].
//   xhat = (x - mean) * rstd,  g = dy * gamma,
//   dx  += rstd * (g - mean(g) - xhat * mean(g * xhat))     (nn.LayerNorm backward)
// ---------------------------------------------------------------------------------
// SUMS: also the column sums of dx before and after the update (the bias gradients of the
// Linear layers whose outputs these residual gradients are) -> part[block][4][D].
// MASK: a width D <= 256 V that is any multiple of 4 (Swin's 96 / 192 / 384 / 1536): lanes past D
// load zeros and store nothing; otherwise D = 256 V exactly.
template <int V, bool SUMS, bool MASK = false>
__global__ void __launch_bounds__(256) ln_bwd_kernel(const float* __restrict__ dy, int64_t lddy,
                                                     const float* __restrict__ x, int64_t ldx,
                                                     const float* __restrict__ gamma, float eps, int64_t M,
                                                     float* __restrict__ dx, int64_t lddx, uint16_t* __restrict__ dxb,
                                                     int64_t lddxb, float* __restrict__ part, int Drt = V * 256) {
    constexpr int DV = V * 256;
    const int D = MASK ? Drt : DV;
    constexpr int NP = SUMS ? 4 : 2;
    __shared__ float red[4][NP * DV];
    float4 so[SUMS ? V : 1], sn[SUMS ? V : 1];
    if constexpr (SUMS) {
#pragma unroll
        for (int i = 0; i < V; ++i) { so[i] = make_float4(0.f, 0.f, 0.f, 0.f); sn[i] = so[i]; }
    }
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    float4 pg[V], pb[V], g4[V];
#pragma unroll
    for (int i = 0; i < V; ++i) {
        pg[i] = make_float4(0.f, 0.f, 0.f, 0.f);
        pb[i] = pg[i];
        g4[i] = (!MASK || (i * 64 + lane) * 4 < D) ? reinterpret_cast<const float4*>(gamma)[i * 64 + lane]
                                                    : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    auto in_row = [&](int i) { return !MASK || (i * 64 + lane) * 4 < D; };
    for (int64_t row = (int64_t)blockIdx.x * 4 + w; row < M; row += (int64_t)gridDim.x * 4) {
        const float4* xr = reinterpret_cast<const float4*>(x + row * ldx);
        const float4* dr = reinterpret_cast<const float4*>(dy + row * lddy);
        float4 xv[V], dv[V];
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < V; ++i) {
            xv[i] = in_row(i) ? xr[i * 64 + lane] : make_float4(0.f, 0.f, 0.f, 0.f);
            dv[i] = in_row(i) ? dr[i * 64 + lane] : make_float4(0.f, 0.f, 0.f, 0.f);
            s += (xv[i].x + xv[i].y) + (xv[i].z + xv[i].w);
        }
        const float invD = MASK ? 1.0f / (float)D : 1.0f / DV;
        const float mean = wave_sum(s) * invD;
        float q = 0.f;
#pragma unroll
        for (int i = 0; i < V; ++i) {
            if (!in_row(i)) continue;
            const float a = xv[i].x - mean, b = xv[i].y - mean, c = xv[i].z - mean, d = xv[i].w - mean;
            q += (a * a + b * b) + (c * c + d * d);
        }
        const float rstd = rsqrtf(wave_sum(q) * invD + eps);
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int i = 0; i < V; ++i) {
            xv[i].x = (xv[i].x - mean) * rstd; xv[i].y = (xv[i].y - mean) * rstd;
            xv[i].z = (xv[i].z - mean) * rstd; xv[i].w = (xv[i].w - mean) * rstd;
            const float a = dv[i].x * g4[i].x, b = dv[i].y * g4[i].y, c = dv[i].z * g4[i].z, d = dv[i].w * g4[i].w;
            s1 += (a + b) + (c + d);
            s2 += (a * xv[i].x + b * xv[i].y) + (c * xv[i].z + d * xv[i].w);
            pg[i].x += dv[i].x * xv[i].x; pg[i].y += dv[i].y * xv[i].y;
            pg[i].z += dv[i].z * xv[i].z; pg[i].w += dv[i].w * xv[i].w;
            pb[i].x += dv[i].x; pb[i].y += dv[i].y; pb[i].z += dv[i].z; pb[i].w += dv[i].w;
        }
        const float c1 = wave_sum(s1) * invD, c2 = wave_sum(s2) * invD;
        float4* dxr = reinterpret_cast<float4*>(dx + row * lddx);
#pragma unroll
        for (int i = 0; i < V; ++i) {
            if (!in_row(i)) continue;
            float4 o = dxr[i * 64 + lane];
            if constexpr (SUMS) { so[i].x += o.x; so[i].y += o.y; so[i].z += o.z; so[i].w += o.w; }
            o.x += rstd * (dv[i].x * g4[i].x - c1 - xv[i].x * c2);
            o.y += rstd * (dv[i].y * g4[i].y - c1 - xv[i].y * c2);
            o.z += rstd * (dv[i].z * g4[i].z - c1 - xv[i].z * c2);
            o.w += rstd * (dv[i].w * g4[i].w - c1 - xv[i].w * c2);
            dxr[i * 64 + lane] = o;
            if constexpr (SUMS) { sn[i].x += o.x; sn[i].y += o.y; sn[i].z += o.z; sn[i].w += o.w; }
            uint2 ob;
            ob.x = pack2bf(o.x, o.y);
            ob.y = pack2bf(o.z, o.w);
            *reinterpret_cast<uint2*>(dxb + row * lddxb + (i * 64 + lane) * 4) = ob;
        }
    }
#pragma unroll
    for (int i = 0; i < V; ++i) {
        if (!in_row(i)) continue;
        reinterpret_cast<float4*>(red[w])[i * 64 + lane] = pg[i];
        reinterpret_cast<float4*>(red[w] + D)[i * 64 + lane] = pb[i];
        if constexpr (SUMS) {
            reinterpret_cast<float4*>(red[w] + 2 * D)[i * 64 + lane] = so[i];
            reinterpret_cast<float4*>(red[w] + 3 * D)[i * 64 + lane] = sn[i];
        }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < NP * D; c += 256)
        part[(int64_t)blockIdx.x * NP * D + c] = (red[0][c] + red[1][c]) + (red[2][c] + red[3][c]);
}

// ---------------------------------------------------------------------------------
// Column sums (bias gradients, partial-sum reductions).  Pass 1: block (x, y) sums rows
// [y*rps, (y+1)*rps) of its 256 columns -> out[y][col].  The final pass (one row split)
// applies the per-column scale and writes either one output or two (cols < n0 -> out0,
// else out1: dgamma | dbeta of a LayerNorm).
// ---------------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ float ld_as_f32(const T* p);
template <>
__device__ __forceinline__ float ld_as_f32<float>(const float* p) { return *p; }
template <>
__device__ __forceinline__ float ld_as_f32<uint16_t>(const uint16_t* p) { return bf2f(*p); }

// Column sums of the per-block LayerNorm partials: segment s of D columns -> outs[s].
struct Outs4 {
    float* p[4];
};
__global__ void __launch_bounds__(256) seg_colsum_kernel(const float* __restrict__ in, int64_t R, int64_t D, int nseg,
                                                         Outs4 outs) {
    __shared__ float red[4][64];
    const int c = threadIdx.x & 63, g = threadIdx.x >> 6;
    const int64_t W = D * nseg, col = (int64_t)blockIdx.x * 64 + c;
    float s = 0.f;
    if (col < W)
        for (int64_t r = g; r < R; r += 4) s += in[r * W + col];
    red[g][c] = s;
    __syncthreads();
    if (g == 0 && col < W) {
        const int seg = (int)(col / D);
        outs.p[seg][col - seg * D] = (red[0][c] + red[1][c]) + (red[2][c] + red[3][c]);
    }
}

template <typename T>
__global__ void __launch_bounds__(256) colsum_kernel(const T* __restrict__ in, int64_t ld, int64_t R, int64_t N,
                                                     int64_t rps, float* __restrict__ out0, int64_t n0,
                                                     float* __restrict__ out1, int64_t nscaled, float scale) {
    const int64_t col = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (col >= N) return;
    const int64_t r0 = (int64_t)blockIdx.y * rps;
    const int64_t r1 = r0 + rps < R ? r0 + rps : R;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    int64_t r = r0;
    for (; r + 4 <= r1; r += 4) {
        s0 += ld_as_f32<T>(in + r * ld + col);
        s1 += ld_as_f32<T>(in + (r + 1) * ld + col);
        s2 += ld_as_f32<T>(in + (r + 2) * ld + col);
        s3 += ld_as_f32<T>(in + (r + 3) * ld + col);
    }
    for (; r < r1; ++r) s0 += ld_as_f32<T>(in + r * ld + col);
    float s = (s0 + s1) + (s2 + s3);
    if (col < nscaled) s *= scale;
    if (gridDim.y > 1)
        out0[(int64_t)blockIdx.y * N + col] = s;
    else if (col < n0)
        out0[col] = s;
    else
        out1[col - n0] = s;
}

// The first level of colsum_kernel<uint16_t> with 8 consecutive columns per lane (one 16-B load per row
// instead of eight 2-B ones: the 2-B version moved 1.6 TB/s on the ViViT-B train step's q|k|v / fc1 bias
// gradients, round 5).  Each column keeps colsum_kernel's order exactly (rows r0 + 4i + j into
// accumulator j, the tail into accumulator 0, (s0 + s1) + (s2 + s3)), so the partials are bit-identical.
// Needs N % 8 == 0, ld % 8 == 0 and a 16-B aligned input; 64 lanes = 512 columns per block.
__global__ void __launch_bounds__(64) colsum_bf16x8_kernel(const uint16_t* __restrict__ in, int64_t ld, int64_t R,
                                                           int64_t N, int64_t rps, float* __restrict__ out) {
    const int64_t col = ((int64_t)blockIdx.x * 64 + threadIdx.x) * 8;
    if (col >= N) return;
    const int64_t r0 = (int64_t)blockIdx.y * rps;
    const int64_t r1 = r0 + rps < R ? r0 + rps : R;
    float acc[4][8];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[j][e] = 0.f;
    auto add = [&](int j, const uint4 u) __attribute__((always_inline)) {
        const unsigned w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            acc[j][2 * e] += bf2f((unsigned short)(w[e] & 0xffff));
            acc[j][2 * e + 1] += bf2f((unsigned short)(w[e] >> 16));
        }
    };
    const uint16_t* p = in + col;
    int64_t r = r0;
    for (; r + 4 <= r1; r += 4) {
        const uint4 u0 = *reinterpret_cast<const uint4*>(p + r * ld);
        const uint4 u1 = *reinterpret_cast<const uint4*>(p + (r + 1) * ld);
        const uint4 u2 = *reinterpret_cast<const uint4*>(p + (r + 2) * ld);
        const uint4 u3 = *reinterpret_cast<const uint4*>(p + (r + 3) * ld);
        add(0, u0);
        add(1, u1);
        add(2, u2);
        add(3, u3);
    }
    for (; r < r1; ++r) add(0, *reinterpret_cast<const uint4*>(p + r * ld));
    float4 o0, o1;
    o0.x = (acc[0][0] + acc[1][0]) + (acc[2][0] + acc[3][0]);
    o0.y = (acc[0][1] + acc[1][1]) + (acc[2][1] + acc[3][1]);
    o0.z = (acc[0][2] + acc[1][2]) + (acc[2][2] + acc[3][2]);
    o0.w = (acc[0][3] + acc[1][3]) + (acc[2][3] + acc[3][3]);
    o1.x = (acc[0][4] + acc[1][4]) + (acc[2][4] + acc[3][4]);
    o1.y = (acc[0][5] + acc[1][5]) + (acc[2][5] + acc[3][5]);
    o1.z = (acc[0][6] + acc[1][6]) + (acc[2][6] + acc[3][6]);
    o1.w = (acc[0][7] + acc[1][7]) + (acc[2][7] + acc[3][7]);
    float* q = out + (int64_t)blockIdx.y * N + col;
    *reinterpret_cast<float4*>(q) = o0;
    *reinterpret_cast<float4*>(q + 4) = o1;
}

// Column sums in up to three fixed-order levels (deterministic for a given R, N): R rows -> S1 =
// min(2048, ceil(R / 64)) partial rows (64 rows per block, so a narrow N still spreads over
// thousands of workgroups) -> S2 = ceil(S1 / 64) -> the output; work >= (S1 + S2) * N floats
// (fewer splits when it is smaller; no work: one pass with one block per 256 columns).
template <typename T>
static int colsum_launch(const T* in, int64_t ld, int64_t R, int64_t N, float* out0, int64_t n0, float* out1,
                         int64_t nscaled, float scale, float* work, int64_t work_elems, hipStream_t stream) {
    const unsigned nbx = (unsigned)((N + 255) / 256);
    int64_t s1 = (R + 63) / 64;
    if (s1 > 2048) s1 = 2048;
    while (s1 > 1 && (s1 + (s1 + 63) / 64) * N > work_elems) s1 /= 2;
    if (s1 <= 1) {
        colsum_kernel<T><<<dim3(nbx, 1), 256, 0, stream>>>(in, ld, R, N, R, out0, n0, out1, nscaled, scale);
        return 0;
    }
    const int64_t rps = (R + s1 - 1) / s1;
    s1 = (R + rps - 1) / rps;
    if (std::is_same<T, uint16_t>::value && N % 8 == 0 && ld % 8 == 0 && !((uintptr_t)in & 15) && !((uintptr_t)work & 15))
        colsum_bf16x8_kernel<<<dim3((unsigned)((N + 511) / 512), (unsigned)s1), 64, 0, stream>>>(
            reinterpret_cast<const uint16_t*>(in), ld, R, N, rps, work);
    else
        colsum_kernel<T><<<dim3(nbx, (unsigned)s1), 256, 0, stream>>>(in, ld, R, N, rps, work, N, nullptr, 0, 1.0f);
    if (s1 <= 64) {
        colsum_kernel<float><<<dim3(nbx, 1), 256, 0, stream>>>(work, N, s1, N, s1, out0, n0, out1, nscaled, scale);
        return 0;
    }
    const int64_t s2 = (s1 + 63) / 64;
    float* w2 = work + s1 * N;
    colsum_kernel<float><<<dim3(nbx, (unsigned)s2), 256, 0, stream>>>(work, N, s1, N, 64, w2, N, nullptr, 0, 1.0f);
    colsum_kernel<float><<<dim3(nbx, 1), 256, 0, stream>>>(w2, N, s2, N, s2, out0, n0, out1, nscaled, scale);
    return 0;
}

// ---------------------------------------------------------------------------------
// Weight-gradient GEMM: dW[n1][n2] = rowscale(n1) * sum_m G[m][n1] * X[m][n2]
// (G = output gradient, X = layer input, both bf16 row-major [M][*], fp32 accumulate).
// The reduction index m is the ROW index of both operands, so both MFMA operands are read
// from row-major LDS images with ds_read_b64_tr_b16 (T10).  Block tile 128 (n1) x 128 (n2),
// 4 waves as 2 x 2 of 64 x 64; split-K over m (grid.y) into fp32 partials + a reduce pass,
// because the weight shapes give only 36-144 output tiles for 256 CUs.
// Operands swapped (A = X, B = G) so each lane holds 4 consecutive n2 -> float4 stores.
// ---------------------------------------------------------------------------------
constexpr int WTILE = 64 * 128 * 2;  // one [64 m][128 cols] bf16 tile = two [64][64] panels
constexpr int WSLOT = 2 * WTILE;

// 16-B chunk swizzle of the 128-B rows read by ds_read_b64_tr_b16 (two 32-lane groups, 8 B per
// lane): a group reads rows {0-3, 8-11} (+4 for the second read, +16 for lanes 32-63) at chunks
// 2cb, 2cb + 1 of each row, so for m = (row >> 1) & 7 the XOR term must differ above bit 0 across
// m in {0, 1, 4, 5} and across {2, 3, 6, 7}: ((m & 1) << 1) | (m & 4) is conflict-free (the
// round-3 term ((m & 1) << 2) | (m & 2) | ((m >> 2) & 1) gave rows 0 and 8 the chunk pairs {2cb,
// 2cb + 1} and {2cb + 1, 2cb}: 2-way conflicts, SQ_LDS_BANK_CONFLICT = 2 cycles per read).
__device__ __forceinline__ int bswz(int r, int c) {
    const int m = (r >> 1) & 7;
    return c ^ (((m & 1) << 1) | (m & 4));
}

__device__ __forceinline__ v8bf tr_frag(const char* tile, int offa, int offb) {
    v4s va = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(tile + offa));
    v4s vb = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(tile + offb));
    v8s vv;
    vv[0] = va[0]; vv[1] = va[1]; vv[2] = va[2]; vv[3] = va[3];
    vv[4] = vb[0]; vv[5] = vb[1]; vv[6] = vb[2]; vv[7] = vb[3];
    return __builtin_bit_cast(v8bf, vv);
}

__global__ void __launch_bounds__(256, 2)
wgrad_kernel(const uint16_t* __restrict__ G, int64_t ldg, const uint16_t* __restrict__ X, int64_t ldx, int64_t M,
             int nJ, int64_t mchunk, float* __restrict__ out, int64_t ldo, int64_t split_stride, int64_t nscaled,
             float scale) {
    __shared__ __attribute__((aligned(16))) char smem[2 * WSLOT];
    const int ntiles = gridDim.x;
    const int L = blockIdx.x;
    const int xq = ntiles >> 3, xr = ntiles & 7, xcd = L & 7;
    const int tile = (xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + (L >> 3);
    const int ti = tile / nJ, tj = tile % nJ;
    const int64_t n1_0 = (int64_t)ti * 128, n2_0 = (int64_t)tj * 128;
    const int64_t mb = (int64_t)blockIdx.y * mchunk;
    const int64_t me = mb + mchunk < M ? mb + mchunk : M;
    const int nt = (int)((me - mb) / 64);

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = tid >> 6;
    const int w1 = wave >> 1, w2 = wave & 1;  // n1 panel, n2 panel of this wave
    // transposed reads for v_mfma_f32_16x16x32 operands (as wgrad_big_kernel): in each 16-lane
    // group gg, lane 4gq + gp addresses row 8gg + gq (+4) and columns 16cb + 4gp of a panel
    const int gq = (lane & 15) >> 2, gp = lane & 3, gg = lane >> 4;
    int off1[4], off2[4];
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
        const int col = cb * 16 + gp * 4;
        const int r1 = 8 * gg + gq, r2 = r1 + 4;
        off1[cb] = r1 * 128 + bswz(r1, col >> 3) * 16 + (col & 7) * 2;
        off2[cb] = r2 * 128 + bswz(r2, col >> 3) * 16 + (col & 7) * 2;
    }

    // staging: 64 rows x 16 chunks of each operand, 4 chunks per thread per operand
    uint4 rg[4], rx[4];
    auto load = [&](int t) {
        const int64_t m0 = mb + (int64_t)t * 64;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int idx = tid + 256 * i, row = idx >> 4, cc = idx & 15;
            rg[i] = *reinterpret_cast<const uint4*>(G + (m0 + row) * ldg + n1_0 + cc * 8);
            rx[i] = *reinterpret_cast<const uint4*>(X + (m0 + row) * ldx + n2_0 + cc * 8);
        }
    };
    auto store = [&](char* slot) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int idx = tid + 256 * i, row = idx >> 4, cc = idx & 15;
            const int off = (cc >> 3) * 8192 + row * 128 + bswz(row, cc & 7) * 16;
            *reinterpret_cast<uint4*>(slot + off) = rg[i];
            *reinterpret_cast<uint4*>(slot + WTILE + off) = rx[i];
        }
    };

    v4f acc[4][4];  // [n2 block i][n1 block j] of 16 x 16: lane -> n1, regs -> 4 consecutive n2
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

    if (nt > 0) {
        load(0);
        store(smem);
    }
    __syncthreads();
    for (int t = 0; t < nt; ++t) {
        const char* gt = smem + (t & 1) * WSLOT + w1 * 8192;
        const char* xt = smem + (t & 1) * WSLOT + WTILE + w2 * 8192;
        if (t + 1 < nt) load(t + 1);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {  // two 32-deep k-steps per 64-row tile
            const int kr = ks * 32 * 128;
            v8bf a[4], b[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) a[i] = tr_frag(xt, off1[i] + kr, off2[i] + kr);
#pragma unroll
            for (int j = 0; j < 4; ++j) b[j] = tr_frag(gt, off1[j] + kr, off2[j] + kr);
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
        }
        if (t + 1 < nt) store(smem + ((t + 1) & 1) * WSLOT);
        __syncthreads();
    }

    float* o = out + (int64_t)blockIdx.y * split_stride;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int64_t n1 = n1_0 + w1 * 64 + j * 16 + (lane & 15);
        const float sc = n1 < nscaled ? scale : 1.0f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int64_t n2 = n2_0 + w2 * 64 + i * 16 + 4 * gg;
            *reinterpret_cast<float4*>(o + n1 * ldo + n2) =
                make_float4(acc[i][j][0] * sc, acc[i][j][1] * sc, acc[i][j][2] * sc, acc[i][j][3] * sc);
        }
    }
}

// ---------------------------------------------------------------------------------
// The same weight gradient on the forward GEMM's 256x256 machinery (gemm.hip
// gemm_bf16_big_kernel): 8 waves as 2 (n2) x 4 (n1), wave tile 128 (n2) x 64 (n1); 32-row
// half-tiles of both operands staged HBM->LDS by LDS-DMA into a 4-slot ring (2 x 16 KiB per
// slot: four [32 rows][64 cols] panels per operand, chunk-swizzled on the SOURCE address so
// the lane-linear DMA image is the bswz image), tile t+3 issued while t is computed, a counted
// vmcnt retiring only t+1 before the one barrier per half-tile; both MFMA operands read with
// ds_read_b64_tr_b16 (the reduction index m is the row index of the images).  N1, N2 % 256 == 0.
// ---------------------------------------------------------------------------------
__device__ __forceinline__ void wg_glds16(const void* gsrc, uint32_t lds_addr) {  // m0 clobbered, not restored
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
                 :
                 : "v"(gsrc), "s"(lds_addr)
                 : "memory", "m0");
}
template <int NW>
__device__ __forceinline__ void wg_wait_vm() {
    static_assert(NW >= 0 && NW < 16, "vmcnt immediate");
    __builtin_amdgcn_s_waitcnt(NW | 0x0F70);
}
__device__ __forceinline__ void wg_sync() {
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");  // LDS was written by DMA behind the compiler's back
    __builtin_amdgcn_sched_barrier(0);
}

constexpr int WPANEL = 32 * 128;    // [32 rows][64 bf16]
constexpr int WOPND = 4 * WPANEL;   // 256 columns of one operand
constexpr int WBSLOT = 2 * WOPND;   // G then X: 32 KiB
constexpr int WBNS = 4;

__global__ void __launch_bounds__(512, 1)
wgrad_big_kernel(const uint16_t* __restrict__ G, int64_t ldg, const uint16_t* __restrict__ X, int64_t ldx, int64_t M,
                 int nJ, int64_t mchunk, float* __restrict__ out, int64_t ldo, int64_t split_stride, int64_t nscaled,
                 float scale) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int ntiles = gridDim.x;
    const int L = blockIdx.x;
    const int xq = ntiles >> 3, xr = ntiles & 7, xcd = L & 7;
    const int tile = (xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + (L >> 3);
    const int ti = tile / nJ, tj = tile % nJ;
    const int64_t n1_0 = (int64_t)ti * 256, n2_0 = (int64_t)tj * 256;
    const int64_t mb = (int64_t)blockIdx.y * mchunk;
    const int64_t me = mb + mchunk < M ? mb + mchunk : M;
    const int nk = (int)((me - mb) / 32);

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int w2 = wave >> 2, w1 = wave & 3;

    // staging: wave w DMAs pieces q = 2w, 2w+1 of each operand (piece = 8 rows of one panel)
    int64_t gsrc[2], xsrc[2];
    uint32_t ldst[2];
#pragma unroll
    for (int pp = 0; pp < 2; ++pp) {
        const int q = 2 * wave + pp, panel = q >> 2, row = (q & 3) * 8 + (lane >> 3);
        const int lch = bswz(row, lane & 7);  // xor swizzle: its own inverse
        gsrc[pp] = (int64_t)row * ldg + n1_0 + panel * 64 + lch * 8;
        xsrc[pp] = (int64_t)row * ldx + n2_0 + panel * 64 + lch * 8;
        ldst[pp] = panel * WPANEL + (q & 3) * 8 * 128;
    }
    const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)smem);
    auto stage = [&](int t) {
        const uint32_t s = lds0 + (t % WBNS) * WBSLOT;
        const int64_t m0 = mb + (int64_t)t * 32;
#pragma unroll
        for (int pp = 0; pp < 2; ++pp) {
            wg_glds16(G + m0 * ldg + gsrc[pp], __builtin_amdgcn_readfirstlane(s + ldst[pp]));
            wg_glds16(X + m0 * ldx + xsrc[pp], __builtin_amdgcn_readfirstlane(s + WOPND + ldst[pp]));
        }
    };

    // transposed reads for v_mfma_f32_16x16x32 operands (T10): in each 16-lane group g = lane >> 4,
    // lane 4q + p addresses row 8g + q (+4 for the second read) and columns 16cb + 4p .. +3 of a
    // panel, so lane i of the group receives column i with k rows 8g .. 8g + 7 -- the same k order
    // for both operands, which is all a sum over k needs
    const int gq = (lane & 15) >> 2, gp = lane & 3, gg = lane >> 4;
    int off1[4], off2[4];
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
        const int col = cb * 16 + gp * 4;
        const int r1 = 8 * gg + gq, r2 = r1 + 4;
        off1[cb] = r1 * 128 + bswz(r1, col >> 3) * 16 + (col & 7) * 2;
        off2[cb] = r2 * 128 + bswz(r2, col >> 3) * 16 + (col & 7) * 2;
    }
    constexpr int MI = 8, NI = 4;  // n2 blocks of 16 (wave: 128), n1 blocks of 16 (wave: 64)
    auto read_frags = [&](int t, v8bf (&fa)[MI], v8bf (&fb)[NI]) __attribute__((always_inline)) {
        const char* gt = smem + (t % WBNS) * WBSLOT;
        const char* xt = gt + WOPND;
#pragma unroll
        for (int i = 0; i < MI; ++i) {  // n2 block i: panel 2*w2 + i/4, column block i % 4
            const char* pn = xt + (2 * w2 + (i >> 2)) * WPANEL;
            fa[i] = tr_frag(pn, off1[i & 3], off2[i & 3]);
        }
#pragma unroll
        for (int j = 0; j < NI; ++j) fb[j] = tr_frag(gt + w1 * WPANEL, off1[j], off2[j]);  // n1 block j: panel w1
    };
    v4f acc[MI][NI];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
    auto mfmas = [&](const v8bf (&fa)[MI], const v8bf (&fb)[NI]) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int j = 0; j < NI; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    };
    // retire half-tile u + 1 once u + 3 may have been staged (4 pieces per wave per half-tile)
    auto retire = [&](auto FAST, int u) __attribute__((always_inline)) {
        if constexpr (decltype(FAST)::value) wg_wait_vm<8>();
        else if (u + 3 < nk) wg_wait_vm<8>();
        else if (u + 2 < nk) wg_wait_vm<4>();
        else wg_wait_vm<0>();
        wg_sync();
    };

    if (nk > 0) {
        v8bf fa0[MI], fb0[NI], fa1[MI], fb1[NI];
        stage(0);
        if (nk > 1) stage(1);
        if (nk > 2) stage(2);
        if (nk > 2) wg_wait_vm<8>();
        else if (nk > 1) wg_wait_vm<4>();
        else wg_wait_vm<0>();
        wg_sync();
        read_frags(0, fa0, fb0);
        // one 32-deep k-step per half-tile: its MFMAs run while the next half-tile's fragments
        // are read behind the barrier that publishes it; fragment sets alternate
        // FAST (compile time) while t + 4 < nk: every stage and retire is the steady-state one, so
        // that loop carries no runtime tests
        auto step2 = [&](auto FAST, int t) __attribute__((always_inline)) {
            constexpr bool fast = decltype(FAST)::value;
            if (fast || t + 3 < nk) stage(t + 3);
            mfmas(fa0, fb0);
            retire(FAST, t);
            read_frags(t + 1, fa1, fb1);
            if (fast || t + 4 < nk) stage(t + 4);
            mfmas(fa1, fb1);
            retire(FAST, t + 1);
            read_frags(t + 2, fa0, fb0);
        };
        int t = 0;
        for (; t + 4 < nk; t += 2) step2(std::true_type{}, t);
        for (; t + 2 < nk; t += 2) step2(std::false_type{}, t);
        mfmas(fa0, fb0);
        if (t + 1 < nk) {
            wg_wait_vm<0>();
            wg_sync();
            read_frags(t + 1, fa1, fb1);
            mfmas(fa1, fb1);
        }
    }

    // lane holds n1 = 16j + (lane & 15) and n2 = 16i + 4(lane >> 4) .. +3 of the wave tile
    float* o = out + (int64_t)blockIdx.y * split_stride;
#pragma unroll
    for (int j = 0; j < NI; ++j) {
        const int64_t n1 = n1_0 + w1 * 64 + j * 16 + (lane & 15);
        const float sc = n1 < nscaled ? scale : 1.0f;
#pragma unroll
        for (int i = 0; i < MI; ++i) {
            const int64_t n2 = n2_0 + w2 * 128 + i * 16 + 4 * gg;
            *reinterpret_cast<float4*>(o + n1 * ldo + n2) =
                make_float4(acc[i][j][0] * sc, acc[i][j][1] * sc, acc[i][j][2] * sc, acc[i][j][3] * sc);
        }
    }
}

// ---------------------------------------------------------------------------------
// The weight gradient on the forward GEMM's ping-pong schedule (gemm.hip gemm_pp_kernel; round 5):
// wgrad_big_kernel's tile (256 n1 x 256 n2, 8 waves as 2 (n2) x 4 (n1), wave tile 128 x 64), its
// slot layout and transposed fragment reads, but the two waves of each SIMD belong to groups one
// barrier apart (waves 0-3: n2 0-127, waves 4-7: n2 128-255), so one group's 16 MFMAs run while the
// other issues its fragment reads and LDS-DMAs.  Per 32-row half-tile u: phase a reads X blocks 0-3
// of the wave and all 4 G blocks, stages G(u+2), MFMAs; phase b reads X blocks 4-7, stages X(u+3),
// retires half-tile u+1 (vmcnt(6)), MFMAs with the same G fragments.  WAR: G(u+2) overwrites G(u-2),
// last read in a(u-2); X(u+3) overwrites X(u-1), last read in b(u-1): both after the lagging group's
// reads completed (the gemm_pp_kernel argument).  Same MFMA chain per output as wgrad_big_kernel:
// bit-identical.  Needs >= 3 half-tiles per split.
// ---------------------------------------------------------------------------------
__global__ void __launch_bounds__(512, 1)
wgrad_pp_kernel(const uint16_t* __restrict__ G, int64_t ldg, const uint16_t* __restrict__ X, int64_t ldx, int64_t M,
                int nJ, int64_t mchunk, float* __restrict__ out, int64_t ldo, int64_t split_stride, int64_t nscaled,
                float scale) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int ntiles = gridDim.x;
    const int L = blockIdx.x;
    const int xq = ntiles >> 3, xr = ntiles & 7, xcd = L & 7;
    const int tile = (xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + (L >> 3);
    const int ti = tile / nJ, tj = tile % nJ;
    const int64_t n1_0 = (int64_t)ti * 256, n2_0 = (int64_t)tj * 256;
    const int64_t mb = (int64_t)blockIdx.y * mchunk;
    const int64_t me = mb + mchunk < M ? mb + mchunk : M;
    const int nk = (int)((me - mb) / 32);

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int w2 = wave >> 2, w1 = wave & 3;

    // staging: wave w DMAs pieces q = 2w, 2w+1 of each operand (piece = 8 rows of one [32][64] panel);
    // per-lane byte offsets from the wave-uniform half-tile bases
    uint32_t goff[2], xoff[2], ldst[2];
#pragma unroll
    for (int pp = 0; pp < 2; ++pp) {
        const int q = 2 * wave + pp, panel = q >> 2, row = (q & 3) * 8 + (lane >> 3);
        const int lch = bswz(row, lane & 7);
        goff[pp] = (uint32_t)(row * ldg + panel * 64 + lch * 8) * 2;
        xoff[pp] = (uint32_t)(row * ldx + panel * 64 + lch * 8) * 2;
        ldst[pp] = panel * WPANEL + (q & 3) * 8 * 128;
    }
    const uint16_t* Gp = G + mb * ldg + n1_0;
    const uint16_t* Xp = X + mb * ldx + n2_0;
    const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)smem);
    auto dma = [&](const void* base, uint32_t voff, uint32_t l) __attribute__((always_inline)) {
        asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1"
                     :
                     : "v"(voff), "s"(base), "s"(l)
                     : "memory", "m0");
    };
    auto stage_g = [&](int u) __attribute__((always_inline)) {
        const uint32_t sl = lds0 + (u % WBNS) * WBSLOT;
        const uint16_t* b = Gp + (int64_t)u * 32 * ldg;
#pragma unroll
        for (int pp = 0; pp < 2; ++pp) dma(b, goff[pp], __builtin_amdgcn_readfirstlane(sl + ldst[pp]));
    };
    auto stage_x = [&](int u) __attribute__((always_inline)) {
        const uint32_t sl = lds0 + (u % WBNS) * WBSLOT + WOPND;
        const uint16_t* b = Xp + (int64_t)u * 32 * ldx;
#pragma unroll
        for (int pp = 0; pp < 2; ++pp) dma(b, xoff[pp], __builtin_amdgcn_readfirstlane(sl + ldst[pp]));
    };

    const int gq = (lane & 15) >> 2, gp = lane & 3, gg = lane >> 4;
    int off1[4], off2[4];
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
        const int col = cb * 16 + gp * 4;
        const int r1 = 8 * gg + gq, r2 = r1 + 4;
        off1[cb] = r1 * 128 + bswz(r1, col >> 3) * 16 + (col & 7) * 2;
        off2[cb] = r2 * 128 + bswz(r2, col >> 3) * 16 + (col & 7) * 2;
    }
    constexpr int MI = 8, NI = 4;
    v4f acc[MI][NI];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
    v8bf fa[4], fb[NI];
    // X blocks i0 .. i0 + 3 of the wave (panel 2 w2 + i0 / 4)
    auto read_x = [&](int u, int i0) __attribute__((always_inline)) {
        const char* pn = smem + (u % WBNS) * WBSLOT + WOPND + (2 * w2 + (i0 >> 2)) * WPANEL;
#pragma unroll
        for (int i = 0; i < 4; ++i) fa[i] = tr_frag(pn, off1[i], off2[i]);
    };
    auto read_g = [&](int u) __attribute__((always_inline)) {
        const char* pn = smem + (u % WBNS) * WBSLOT + w1 * WPANEL;
#pragma unroll
        for (int j = 0; j < NI; ++j) fb[j] = tr_frag(pn, off1[j], off2[j]);
    };
    auto mma = [&](int i0) __attribute__((always_inline)) {
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's fragment reads
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < NI; ++j)
                acc[i0 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i0 + i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
    };
    // FAST (compile time) while u + 3 < nk: steady-state staging and retire counts, no runtime tests
    auto phase_a = [&](auto FAST, int u) __attribute__((always_inline)) {
        read_x(u, 0);
        read_g(u);
        if constexpr (decltype(FAST)::value) stage_g(u + 2);
        else if (u + 2 < nk) stage_g(u + 2);
        __builtin_amdgcn_sched_barrier(0);
        mma(0);
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
    };
    auto phase_b = [&](auto FAST, int u) __attribute__((always_inline)) {
        read_x(u, 4);
        if constexpr (decltype(FAST)::value) {
            stage_x(u + 3);
            wg_wait_vm<6>();
        } else if (u + 3 < nk) {
            stage_x(u + 3);
            wg_wait_vm<6>();
        } else if (u + 2 < nk) {
            wg_wait_vm<4>();
        } else {
            wg_wait_vm<0>();
        }
        __builtin_amdgcn_sched_barrier(0);
        mma(4);
        // the lagging group skips its last barrier: both groups then pass the same number
        if constexpr (decltype(FAST)::value) __builtin_amdgcn_s_barrier();
        else if (u + 1 < nk || w2 == 0) __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
    };

    // prologue: X0 G0 X1 G1 X2 in flight, retire X0 G0, publish; group 1 one barrier behind
    stage_x(0);
    stage_g(0);
    stage_x(1);
    stage_g(1);
    stage_x(2);
    wg_wait_vm<6>();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (w2 == 1) __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    int u = 0;
    for (; u + 3 < nk; ++u) {
        phase_a(std::true_type{}, u);
        phase_b(std::true_type{}, u);
    }
    for (; u < nk; ++u) {
        phase_a(std::false_type{}, u);
        phase_b(std::false_type{}, u);
    }

    float* o = out + (int64_t)blockIdx.y * split_stride;
#pragma unroll
    for (int j = 0; j < NI; ++j) {
        const int64_t n1 = n1_0 + w1 * 64 + j * 16 + (lane & 15);
        const float sc = n1 < nscaled ? scale : 1.0f;
#pragma unroll
        for (int i = 0; i < MI; ++i) {
            const int64_t n2 = n2_0 + w2 * 128 + i * 16 + 4 * gg;
            *reinterpret_cast<float4*>(o + n1 * ldo + n2) =
                make_float4(acc[i][j][0] * sc, acc[i][j][1] * sc, acc[i][j][2] * sc, acc[i][j][3] * sc);
        }
    }
}

// out[n1][n2] = sum_z ws[z][n1][n2] (the scale was applied per split)
__global__ void __launch_bounds__(256) wgrad_reduce_kernel(const float* __restrict__ ws, int64_t n4, int splits,
                                                           int64_t N2, float* __restrict__ out, int64_t ldo) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n4) return;
    const float4* w = reinterpret_cast<const float4*>(ws);
    float4 s = w[i];
    for (int z = 1; z < splits; ++z) {
        const float4 v = w[(int64_t)z * n4 + i];
        s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    const int64_t e = i * 4, n1 = e / N2, n2 = e - n1 * N2;
    *reinterpret_cast<float4*>(out + n1 * ldo + n2) = s;
}

// ---------------------------------------------------------------------------------
// Classifier head backward (one workgroup, B clips in order: deterministic).
// Forward per clip: y = LN(x[b*S]) (final layernorm on the CLS row), logits = Wc y + bc.
// Given dlogits: dWc += dl (x) y, dbc += dl, dy = Wc^T dl, dgamma += dy*xhat, dbeta += dy,
// dx[b*S] = LN backward of dy (written; the dx rows of other tokens are left untouched).
// D <= 1024 (4 columns per thread).
// ---------------------------------------------------------------------------------
__device__ __forceinline__ float block_sum(float v, float* red) {
    v = wave_sum(v);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) red[w] = v;
    __syncthreads();
    return (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ void __launch_bounds__(256) cls_head_bwd_kernel(const float* __restrict__ x, int64_t ldx, int B, int64_t S,
                                                           int D, const float* __restrict__ gamma,
                                                           const float* __restrict__ beta, float eps,
                                                           const float* __restrict__ Wc, int nl,
                                                           const float* __restrict__ dlogits, float* __restrict__ dx,
                                                           int64_t lddx, uint16_t* __restrict__ dxb, int64_t lddxb,
                                                           float* __restrict__ dWc, float* __restrict__ dbc,
                                                           float* __restrict__ dgamma, float* __restrict__ dbeta) {
    __shared__ float red[4];
    const int tid = threadIdx.x;
    float dg[4] = {0.f, 0.f, 0.f, 0.f}, dbt[4] = {0.f, 0.f, 0.f, 0.f};
    for (int c = 0; c < nl; ++c)
        for (int k = 0; k < 4; ++k) {
            const int n = tid + 256 * k;
            if (n < D) dWc[c * D + n] = 0.f;
        }
    for (int b = 0; b < B; ++b) {
        const float* xr = x + (int64_t)b * S * ldx;
        float xv[4];
        float s = 0.f;
        for (int k = 0; k < 4; ++k) {
            const int n = tid + 256 * k;
            xv[k] = n < D ? xr[n] : 0.f;
            s += xv[k];
        }
        const float mean = block_sum(s, red) / (float)D;
        float q = 0.f;
        for (int k = 0; k < 4; ++k) {
            const int n = tid + 256 * k;
            if (n < D) q += (xv[k] - mean) * (xv[k] - mean);
        }
        const float rstd = rsqrtf(block_sum(q, red) / (float)D + eps);
        float gdy[4], s1 = 0.f, s2 = 0.f;
        for (int k = 0; k < 4; ++k) {
            const int n = tid + 256 * k;
            gdy[k] = 0.f;
            if (n < D) {
                xv[k] = (xv[k] - mean) * rstd;  // xhat
                const float y = xv[k] * gamma[n] + beta[n];
                float dy = 0.f;
                for (int c = 0; c < nl; ++c) {
                    const float dl = dlogits[b * nl + c];
                    dWc[c * D + n] += dl * y;
                    dy += dl * Wc[c * D + n];
                }
                dg[k] += dy * xv[k];
                dbt[k] += dy;
                gdy[k] = dy * gamma[n];
                s1 += gdy[k];
                s2 += gdy[k] * xv[k];
            }
        }
        const float c1 = block_sum(s1, red) / (float)D;
        const float c2 = block_sum(s2, red) / (float)D;
        for (int k = 0; k < 4; ++k) {
            const int n = tid + 256 * k;
            if (n < D) {
                const float v = rstd * (gdy[k] - c1 - xv[k] * c2);
                dx[(int64_t)b * S * lddx + n] = v;
                dxb[(int64_t)b * S * lddxb + n] = f2bf(v);
            }
        }
    }
    for (int k = 0; k < 4; ++k) {
        const int n = tid + 256 * k;
        if (n < D) { dgamma[n] = dg[k]; dbeta[n] = dbt[k]; }
    }
    if (tid < nl) {
        float s = 0.f;
        for (int b = 0; b < B; ++b) s += dlogits[b * nl + tid];
        dbc[tid] = s;
    }
}

// ---------------------------------------------------------------------------------
// Embedding backward: dpos[s] = sum_b dx[b*S + s]; dcls = dpos[0];
// demb[b*(S-1) + p] = bf16(dx[b*S + 1 + p]) (the patch rows, for the embed weight gradient).
// ---------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) embed_bwd_kernel(const float* __restrict__ dx, int64_t lddx, int B, int64_t S,
                                                        int D, float* __restrict__ dpos, float* __restrict__ dcls,
                                                        uint16_t* __restrict__ demb, int64_t ldde) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int d4 = D / 4;
    if (i >= S * d4) return;
    const int64_t s = i / d4;
    const int c = (int)(i - s * d4) * 4;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int b = 0; b < B; ++b) {
        const float4 v = *reinterpret_cast<const float4*>(dx + ((int64_t)b * S + s) * lddx + c);
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
        if (s >= 1) {
            uint2 o;
            o.x = pack2bf(v.x, v.y);
            o.y = pack2bf(v.z, v.w);
            *reinterpret_cast<uint2*>(demb + ((int64_t)b * (S - 1) + s - 1) * ldde + c) = o;
        }
    }
    *reinterpret_cast<float4*>(dpos + s * D + c) = acc;
    if (s == 0) *reinterpret_cast<float4*>(dcls + c) = acc;
}

// ---------------------------------------------------------------------------------
// AdamW over flat fp32 buffers, the arithmetic of torch.optim.AdamW (decoupled decay):
//   p *= 1 - lr*wd;  m += (1-b1)(g - m);  v = b2 v + (1-b2) g^2;
//   p -= (lr / bc1) * m / (sqrt(v) / sqrt(bc2) + eps)
// ---------------------------------------------------------------------------------
// one element of torch.optim.AdamW's update (shared by the single- and multi-tensor kernels, no
// FMA contraction, so both give the same bits)
__device__ __forceinline__ void adamw_elem(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                                           float* __restrict__ v, int64_t i, float lr, float b1, float b2, float eps,
                                           float wd, float step_size, float bc2_sqrt, float gscale) {
#pragma clang fp contract(off)  // plain IEEE mul / add in this order: the same bits in every caller
    const float gg = g[i] * gscale;
    float pp = p[i] * (1.0f - lr * wd);
    float mm = m[i];
    mm = mm + (1.0f - b1) * (gg - mm);
    const float vv = v[i] * b2 + (1.0f - b2) * gg * gg;
    const float denom = sqrtf(vv) / bc2_sqrt + eps;
    pp = pp - step_size * (mm / denom);
    p[i] = pp;
    m[i] = mm;
    v[i] = vv;
}

__global__ void __launch_bounds__(256) adamw_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                    float* __restrict__ m, float* __restrict__ v, int64_t n, float lr,
                                                    float b1, float b2, float eps, float wd, float step_size,
                                                    float bc2_sqrt, float gscale) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride)
        adamw_elem(p, g, m, v, i, lr, b1, b2, eps, wd, step_size, bc2_sqrt, gscale);
}

// The same update with the step taken on the device (a captured train-step graph replays one launch for
// every step): step = *counter + 1, its bias-correction constants (lr / bc1, sqrt(bc2)) read from a host-built
// table (the values vc_adamw derives for that step, so both paths give the same bits); vc_adamw_step_tick
// advances the counter after the update.
__global__ void __launch_bounds__(256) adamw_tab_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                        float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                        float lr, float b1, float b2, float eps, float wd,
                                                        const float* __restrict__ tab, const int64_t* __restrict__ counter,
                                                        int64_t tab_len, float gscale) {
    int64_t t = *counter;  // steps done
    if (t >= tab_len) t = tab_len - 1;  // beyond the table: the host refuses to replay (vc checks), clamp anyway
    const float step_size = tab[2 * t], bc2_sqrt = tab[2 * t + 1];
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride)
        adamw_elem(p, g, m, v, i, lr, b1, b2, eps, wd, step_size, bc2_sqrt, gscale);
}

__global__ void adamw_step_tick_kernel(int64_t* __restrict__ counter) {
    if (threadIdx.x == 0) *counter += 1;
}

// Multi-tensor AdamW: tab[i] = {p, g, m, v (addresses), n, chunk0}, chunk0 = the entry's first
// 1024-element chunk (prefix sum over the entries); one workgroup per chunk finds its entry by
// binary search over the (uniform, scalar-loaded) table; the element arithmetic is adamw_kernel's.
__global__ void __launch_bounds__(256) adamw_multi_kernel(const int64_t* __restrict__ tab, int ntab, float lr, float b1,
                                                          float b2, float eps, float wd, float step_size,
                                                          float bc2_sqrt, float gscale) {
    const int64_t c = blockIdx.x;
    int lo = 0, hi = ntab - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (tab[(int64_t)mid * 6 + 5] <= c) lo = mid;
        else hi = mid - 1;
    }
    const int64_t* e = tab + (int64_t)lo * 6;
    float* __restrict__ p = reinterpret_cast<float*>(e[0]);
    const float* __restrict__ g = reinterpret_cast<const float*>(e[1]);
    float* __restrict__ m = reinterpret_cast<float*>(e[2]);
    float* __restrict__ v = reinterpret_cast<float*>(e[3]);
    const int64_t n = e[4], base = (c - e[5]) * 1024;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int64_t i = base + k * 256 + threadIdx.x;
        if (i < n) adamw_elem(p, g, m, v, i, lr, b1, b2, eps, wd, step_size, bc2_sqrt, gscale);
    }
}

// ---------------------------------------------------------------------------------
// Weight packing after each optimizer step: fp32 master [N][K] -> bf16 [N][K] and/or
// bf16 [K][N] (the dgrad GEMMs' operand), rows < nscaled multiplied by `scale` (the
// softmax scale * log2 e folded into the q projection).  64 x 64 tiles through LDS.
// ---------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) pack_weight_kernel(const float* __restrict__ src, int64_t N, int64_t K,
                                                          int64_t nscaled, float scale, uint16_t* __restrict__ dst,
                                                          uint16_t* __restrict__ dstT) {
    // 64 x 64 tile; each thread moves 4 consecutive elements per pass (float4 in, 8-B bf16 out),
    // the transposed write goes through LDS as 4 consecutive n per thread (host: N, K % 4 == 0)
    __shared__ float tile[64][65];
    const int64_t n0 = (int64_t)blockIdx.y * 64, k0 = (int64_t)blockIdx.x * 64;
    const int t = threadIdx.x, rr0 = t >> 4, c4 = (t & 15) * 4;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const int rr = rr0 + p * 16;
        const int64_t n = n0 + rr, k = k0 + c4;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (n < N && k < K) {
            v = *reinterpret_cast<const float4*>(src + n * K + k);
            if (n < nscaled) { v.x *= scale; v.y *= scale; v.z *= scale; v.w *= scale; }
            if (dst) *reinterpret_cast<uint2*>(dst + n * K + k) = make_uint2(pack2bf(v.x, v.y), pack2bf(v.z, v.w));
        }
        tile[rr][c4 + 0] = v.x;
        tile[rr][c4 + 1] = v.y;
        tile[rr][c4 + 2] = v.z;
        tile[rr][c4 + 3] = v.w;
    }
    if (!dstT) return;
    __syncthreads();
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const int kr = rr0 + p * 16;  // k within the tile; c4: 4 consecutive n
        const int64_t k = k0 + kr, n = n0 + c4;
        if (n < N && k < K)
            *reinterpret_cast<uint2*>(dstT + k * N + n) =
                make_uint2(pack2bf(tile[c4][kr], tile[c4 + 1][kr]), pack2bf(tile[c4 + 2][kr], tile[c4 + 3][kr]));
    }
}

}  // namespace trn
}  // namespace vc

using namespace vc;
using namespace vc::trn;

extern "C" {

int vc_layernorm_bwd(const float* dy, int64_t lddy, const float* x, int64_t ldx, int64_t M, int64_t D,
                     const float* gamma, float eps, float* dx, int64_t lddx, uint16_t* dxb, int64_t lddxb,
                     float* dgamma, float* dbeta, float* dsum_in, float* dsum_out, float* work, int64_t work_elems,
                     hipStream_t stream) {
    if (!dy || !x || !gamma || !dx || !dxb || !dgamma || !dbeta || !work)
        return fail(VC_ERR_INVALID_ARG, "vc_layernorm_bwd: null pointer");
    if (D <= 0 || D % 4 || D > 1536)
        return fail(VC_ERR_UNSUPPORTED, "vc_layernorm_bwd: D must be a multiple of 4, at most 1536");
    if (lddy % 4 || ldx % 4 || lddx % 4 || lddxb % 4 || M <= 0)
        return fail(VC_ERR_INVALID_ARG, "vc_layernorm_bwd: leading dimensions must be multiples of 4");
    if ((dsum_in == nullptr) != (dsum_out == nullptr))
        return fail(VC_ERR_INVALID_ARG, "vc_layernorm_bwd: dsum_in and dsum_out go together");
    const bool sums = dsum_in != nullptr;
    const int np = sums ? 4 : 2;
    int64_t nb = (M + 3) / 4;
    if (nb > 512) nb = 512;
    const int64_t nsp = (nb + 31) / 32;  // row splits of the partial reduction
    const int64_t need = (nb + nsp) * np * D;
    if (work_elems < need) return fail(VC_ERR_INVALID_ARG, "vc_layernorm_bwd: work too small (need " + std::to_string(need) + ")");
#define VC_LNB(V)                                                                                                   \
    (sums ? (ln_bwd_kernel<V, true><<<(unsigned)nb, 256, 0, stream>>>(dy, lddy, x, ldx, gamma, eps, M, dx, lddx, dxb,  \
                                                                      lddxb, work), 0)                             \
          : (ln_bwd_kernel<V, false><<<(unsigned)nb, 256, 0, stream>>>(dy, lddy, x, ldx, gamma, eps, M, dx, lddx, dxb, \
                                                                       lddxb, work), 0))
#define VC_LNBM(V)                                                                                                  \
    (sums ? (ln_bwd_kernel<V, true, true><<<(unsigned)nb, 256, 0, stream>>>(dy, lddy, x, ldx, gamma, eps, M, dx, lddx,  \
                                                                            dxb, lddxb, work, (int)D), 0)              \
          : (ln_bwd_kernel<V, false, true><<<(unsigned)nb, 256, 0, stream>>>(dy, lddy, x, ldx, gamma, eps, M, dx, lddx, \
                                                                             dxb, lddxb, work, (int)D), 0))
    switch (D) {
        case 256: VC_LNB(1); break;
        case 512: VC_LNB(2); break;
        case 768: VC_LNB(3); break;
        case 1024: VC_LNB(4); break;
        default:
            if (D <= 256) VC_LNBM(1);
            else if (D <= 512) VC_LNBM(2);
            else if (D <= 768) VC_LNBM(3);
            else if (D <= 1024) VC_LNBM(4);
            else VC_LNBM(6);
    }
#undef VC_LNB
#undef VC_LNBM
    // partials [nb][np*D] -> [nsp][np*D] (32 rows per block) -> the np outputs
    float* tmp = work + nb * np * D;
    colsum_kernel<float><<<dim3((unsigned)((np * D + 255) / 256), (unsigned)nsp), 256, 0, stream>>>(
        work, np * D, nb, np * D, 32, tmp, np * D, nullptr, 0, 1.0f);
    Outs4 o{{dgamma, dbeta, dsum_in, dsum_out}};
    seg_colsum_kernel<<<(unsigned)((np * D + 63) / 64), 256, 0, stream>>>(tmp, nsp, D, np, o);
    return check_launch("vc_layernorm_bwd");
}

int vc_colsum(const void* in, int dtype, int64_t ld, int64_t R, int64_t N, int64_t nscaled, float scale, float* out,
              float* work, int64_t work_elems, hipStream_t stream) {
    if (!in || !out) return fail(VC_ERR_INVALID_ARG, "vc_colsum: null pointer");
    if (R <= 0 || N <= 0 || ld < N) return fail(VC_ERR_INVALID_ARG, "vc_colsum: bad shape");
    if (!work) work_elems = 0;
    if (dtype == 0)
        colsum_launch<float>((const float*)in, ld, R, N, out, N, nullptr, nscaled, scale, work, work_elems, stream);
    else if (dtype == 1)
        colsum_launch<uint16_t>((const uint16_t*)in, ld, R, N, out, N, nullptr, nscaled, scale, work, work_elems, stream);
    else
        return fail(VC_ERR_INVALID_ARG, "vc_colsum: dtype must be 0 (f32) or 1 (bf16)");
    return check_launch("vc_colsum");
}

// VCLIP_WGRAD_PP=0 in the environment: the weight gradients on wgrad_big_kernel (A/B of the schedules;
// read once per process)
static bool wgrad_pp_enabled() {
    static int v = -1;
    if (v < 0) {
        const char* e = getenv("VCLIP_WGRAD_PP");
        v = (e && e[0] == '0') ? 0 : 1;
    }
    return v == 1;
}

// The 256 x 256 weight-gradient schedule for M rows of reduction: split count sp (fewest workgroup rounds x
// half-tiles per workgroup over 1 .. ceil(CUs / tiles) splits, capped by the scratch), rows per split mch,
// and whether every split is long enough for the ping-pong kernel.  Shared by vc_wgrad_bf16 and
// vc_wgrad_pick (the host-side label query), so the two cannot disagree.
struct WgradPlan {
    int64_t sp, mch;
    bool pp;
};
static WgradPlan wgrad_plan(int64_t M, int64_t N1, int64_t N2, bool have_work, int64_t work_elems) {
    const int64_t nt2 = (N1 / 256) * (N2 / 256);
    const int64_t kt2 = M / 32;
    // round 5: ceil(256 / tiles) alone gave 270 / 261 / 288 workgroups for the ViViT-B q|k|v / o_proj / fc1
    // weights -- a second round of 14 / 5 / 32 (floor: 243 / 252 / 252 workgroups in one round)
    static int ncu_s = 0;
    if (!ncu_s) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&ncu_s, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu_s <= 0)
            ncu_s = 256;
    }
    const int64_t ncu = ncu_s;
    int64_t sp = 1, best = -1;
    for (int64_t c = 1; c <= (ncu + nt2 - 1) / nt2 && c <= (kt2 / 4 > 0 ? kt2 / 4 : 1); ++c) {
        const int64_t cost = ((nt2 * c + ncu - 1) / ncu) * ((kt2 + c - 1) / c);
        if (best < 0 || cost <= best) { best = cost; sp = c; }
    }
    if (!have_work || work_elems < 2 * N1 * N2) sp = 1;
    else if (sp * N1 * N2 > work_elems) sp = work_elems / (N1 * N2);
    if (sp < 1) sp = 1;
    WgradPlan p;
    p.mch = (kt2 + sp - 1) / sp * 32;
    p.sp = (M + p.mch - 1) / p.mch;
    // the ping-pong schedule when every split has >= 3 half-tiles (the last split is the shortest)
    p.pp = (M - (p.sp - 1) * p.mch) / 32 >= 3 && wgrad_pp_enabled();
    return p;
}

int vc_wgrad_pick(int64_t M, int64_t N1, int64_t N2, int64_t work_elems) {
    if (M <= 0 || N1 <= 0 || N2 <= 0) return fail(VC_ERR_INVALID_ARG, "vc_wgrad_pick: need M, N1, N2 > 0");
    if (N1 % 256 || N2 % 256) return 0;
    const WgradPlan p = wgrad_plan(M, N1, N2, work_elems > 0, work_elems);
    return (p.pp ? 2 : 1) | (int)(p.sp << 4);
}

int vc_wgrad_bf16(const uint16_t* G, int64_t ldg, const uint16_t* X, int64_t ldx, int64_t M, int64_t N1, int64_t N2,
                  int64_t nscaled, float scale, float* out, int64_t ldo, float* work, int64_t work_elems,
                  hipStream_t stream) {
    if (!G || !X || !out) return fail(VC_ERR_INVALID_ARG, "vc_wgrad_bf16: null pointer");
    const bool big = N1 % 256 == 0 && N2 % 256 == 0;
    if (M <= 0 || M % (big ? 32 : 64) || N1 % 128 || N2 % 128 || N1 <= 0 || N2 <= 0)
        return fail(VC_ERR_INVALID_ARG, "vc_wgrad_bf16: need N1 % 128 == 0, N2 % 128 == 0, M % 64 == 0 "
                                        "(M % 32 when N1, N2 % 256 == 0)");
    if (ldg % 8 || ldx % 8 || ldo % 4 || ldg < N1 || ldx < N2 || ldo < N2 ||
        ((((uintptr_t)G) | ((uintptr_t)X) | ((uintptr_t)out)) & 15))
        return fail(VC_ERR_INVALID_ARG, "vc_wgrad_bf16: bad leading dimension / alignment");
    if (big) {
        // 256 x 256 LDS-DMA kernel, split-K sized for ~one workgroup per CU
        const int nJ2 = (int)(N2 / 256);
        const int nt2 = (int)(N1 / 256) * nJ2;
        const WgradPlan plan = wgrad_plan(M, N1, N2, work != nullptr, work_elems);
        const int64_t sp = plan.sp, mch = plan.mch;
        static bool attr = false;
        if (!attr) {
            hipError_t e = hipFuncSetAttribute((const void*)wgrad_big_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                               WBNS * WBSLOT);
            if (e == hipSuccess)
                e = hipFuncSetAttribute((const void*)wgrad_pp_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                        WBNS * WBSLOT);
            if (e != hipSuccess) return fail((int)e, std::string("vc_wgrad_bf16: hipFuncSetAttribute: ") + hipGetErrorString(e));
            attr = true;
        }
        auto kern = plan.pp ? wgrad_pp_kernel : wgrad_big_kernel;
        if (sp == 1) {
            kern<<<dim3((unsigned)nt2, 1), 512, WBNS * WBSLOT, stream>>>(G, ldg, X, ldx, M, nJ2, mch, out, ldo, 0, nscaled,
                                                                         scale);
        } else {
            kern<<<dim3((unsigned)nt2, (unsigned)sp), 512, WBNS * WBSLOT, stream>>>(G, ldg, X, ldx, M, nJ2, mch, work, N2,
                                                                                    N1 * N2, nscaled, scale);
            const int64_t n4 = N1 * N2 / 4;
            wgrad_reduce_kernel<<<(unsigned)((n4 + 255) / 256), 256, 0, stream>>>(work, n4, (int)sp, N2, out, ldo);
        }
        return check_launch("vc_wgrad_bf16");
    }
    const int nI = (int)(N1 / 128), nJ = (int)(N2 / 128);
    const int ntiles = nI * nJ;
    const int64_t kt = M / 64;
    int64_t splits = (512 + ntiles - 1) / ntiles;
    if (splits > kt / 2) splits = kt / 2;
    if (!work || work_elems < 2 * N1 * N2) splits = 1;
    else if (splits * N1 * N2 > work_elems) splits = work_elems / (N1 * N2);
    if (splits < 1) splits = 1;
    const int64_t mchunk = (kt + splits - 1) / splits * 64;
    splits = (M + mchunk - 1) / mchunk;
    if (splits == 1) {
        wgrad_kernel<<<dim3((unsigned)ntiles, 1), 256, 0, stream>>>(G, ldg, X, ldx, M, nJ, mchunk, out, ldo, 0, nscaled,
                                                                  scale);
    } else {
        wgrad_kernel<<<dim3((unsigned)ntiles, (unsigned)splits), 256, 0, stream>>>(G, ldg, X, ldx, M, nJ, mchunk, work,
                                                                                 N2, N1 * N2, nscaled, scale);
        const int64_t n4 = N1 * N2 / 4;
        wgrad_reduce_kernel<<<(unsigned)((n4 + 255) / 256), 256, 0, stream>>>(work, n4, (int)splits, N2, out, ldo);
    }
    return check_launch("vc_wgrad_bf16");
}

int vc_cls_head_bwd(const float* x, int64_t ldx, int64_t B, int64_t S, int64_t D, const float* gamma, const float* beta,
                    float eps, const float* Wc, int64_t num_labels, const float* dlogits, float* dx, int64_t lddx,
                    uint16_t* dxb, int64_t lddxb, float* dWc, float* dbc, float* dgamma, float* dbeta,
                    hipStream_t stream) {
    if (!x || !gamma || !beta || !Wc || !dlogits || !dx || !dxb || !dWc || !dbc || !dgamma || !dbeta)
        return fail(VC_ERR_INVALID_ARG, "vc_cls_head_bwd: null pointer");
    if (D > 1024 || num_labels > 256 || B <= 0) return fail(VC_ERR_UNSUPPORTED, "vc_cls_head_bwd: D <= 1024, labels <= 256");
    cls_head_bwd_kernel<<<1, 256, 0, stream>>>(x, ldx, (int)B, S, (int)D, gamma, beta, eps, Wc, (int)num_labels, dlogits,
                                               dx, lddx, dxb, lddxb, dWc, dbc, dgamma, dbeta);
    return check_launch("vc_cls_head_bwd");
}

int vc_embed_bwd(const float* dx, int64_t lddx, int64_t B, int64_t S, int64_t D, float* dpos, float* dcls,
                 uint16_t* demb, int64_t ldde, hipStream_t stream) {
    if (!dx || !dpos || !dcls || !demb) return fail(VC_ERR_INVALID_ARG, "vc_embed_bwd: null pointer");
    if (D % 4 || lddx % 4 || ldde % 4 || S < 2 || ((uintptr_t)dx & 15) || ((uintptr_t)dpos & 15) || ((uintptr_t)dcls & 15))
        return fail(VC_ERR_INVALID_ARG, "vc_embed_bwd: D % 4, alignment");
    const int64_t n = S * (D / 4);
    embed_bwd_kernel<<<(unsigned)((n + 255) / 256), 256, 0, stream>>>(dx, lddx, (int)B, S, (int)D, dpos, dcls, demb, ldde);
    return check_launch("vc_embed_bwd");
}

int vc_adamw(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n, float lr, float beta1,
             float beta2, float eps, float weight_decay, int64_t step, float grad_scale, hipStream_t stream) {
    if (!param || !grad || !exp_avg || !exp_avg_sq) return fail(VC_ERR_INVALID_ARG, "vc_adamw: null pointer");
    if (n <= 0 || step <= 0) return fail(VC_ERR_INVALID_ARG, "vc_adamw: n > 0, step >= 1");
    const double bc1 = 1.0 - std::pow((double)beta1, (double)step);
    const double bc2 = 1.0 - std::pow((double)beta2, (double)step);
    const float step_size = (float)(lr / bc1);
    const float bc2_sqrt = (float)std::sqrt(bc2);
    int64_t nb = (n + 255) / 256;
    if (nb > 8192) nb = 8192;
    adamw_kernel<<<(unsigned)nb, 256, 0, stream>>>(param, grad, exp_avg, exp_avg_sq, n, lr, beta1, beta2, eps,
                                                   weight_decay, step_size, bc2_sqrt, grad_scale);
    return check_launch("vc_adamw");
}

int vc_adamw_step_table(float beta1, float beta2, float lr, int64_t steps, float* out) {
    if (!out || steps <= 0) return fail(VC_ERR_INVALID_ARG, "vc_adamw_step_table: null output / steps <= 0");
    for (int64_t t = 1; t <= steps; ++t) {  // exactly vc_adamw's arithmetic for step t
        const double bc1 = 1.0 - std::pow((double)beta1, (double)t);
        const double bc2 = 1.0 - std::pow((double)beta2, (double)t);
        out[2 * (t - 1)] = (float)(lr / bc1);
        out[2 * (t - 1) + 1] = (float)std::sqrt(bc2);
    }
    return 0;
}

int vc_adamw_tab(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n, float lr, float beta1,
                 float beta2, float eps, float weight_decay, const float* tab, const int64_t* counter, int64_t tab_len,
                 float grad_scale, hipStream_t stream) {
    if (!param || !grad || !exp_avg || !exp_avg_sq || !tab || !counter)
        return fail(VC_ERR_INVALID_ARG, "vc_adamw_tab: null pointer");
    if (n <= 0 || tab_len <= 0) return fail(VC_ERR_INVALID_ARG, "vc_adamw_tab: n > 0, tab_len > 0");
    int64_t nb = (n + 255) / 256;
    if (nb > 8192) nb = 8192;
    adamw_tab_kernel<<<(unsigned)nb, 256, 0, stream>>>(param, grad, exp_avg, exp_avg_sq, n, lr, beta1, beta2, eps,
                                                       weight_decay, tab, counter, tab_len, grad_scale);
    return check_launch("vc_adamw_tab");
}

int vc_adamw_step_tick(int64_t* counter, hipStream_t stream) {
    if (!counter) return fail(VC_ERR_INVALID_ARG, "vc_adamw_step_tick: null counter");
    adamw_step_tick_kernel<<<1, 64, 0, stream>>>(counter);
    return check_launch("vc_adamw_step_tick");
}

int vc_adamw_multi(const int64_t* table, int64_t ntab, int64_t nchunks, float lr, float beta1, float beta2, float eps,
                   float weight_decay, int64_t step, float grad_scale, hipStream_t stream) {
    if (!table) return fail(VC_ERR_INVALID_ARG, "vc_adamw_multi: null table");
    if (ntab <= 0 || ntab > (1 << 24) || nchunks <= 0 || nchunks > 0x7fffffff || step <= 0)
        return fail(VC_ERR_INVALID_ARG, "vc_adamw_multi: ntab, nchunks > 0, step >= 1");
    if ((uintptr_t)table & 7) return fail(VC_ERR_INVALID_ARG, "vc_adamw_multi: table must be 8-byte aligned");
    const double bc1 = 1.0 - std::pow((double)beta1, (double)step);
    const double bc2 = 1.0 - std::pow((double)beta2, (double)step);
    adamw_multi_kernel<<<(unsigned)nchunks, 256, 0, stream>>>(table, (int)ntab, lr, beta1, beta2, eps, weight_decay,
                                                              (float)(lr / bc1), (float)std::sqrt(bc2), grad_scale);
    return check_launch("vc_adamw_multi");
}

int vc_pack_weight(const float* src, int64_t N, int64_t K, int64_t nscaled, float scale, uint16_t* dst, uint16_t* dstT,
                   hipStream_t stream) {
    if (!src || (!dst && !dstT)) return fail(VC_ERR_INVALID_ARG, "vc_pack_weight: null pointer");
    if (N <= 0 || K <= 0 || N % 4 || K % 4) return fail(VC_ERR_INVALID_ARG, "vc_pack_weight: need N, K % 4 == 0");
    if ((((uintptr_t)src) & 15) || (((uintptr_t)dst) & 7) || (((uintptr_t)dstT) & 7))
        return fail(VC_ERR_INVALID_ARG, "vc_pack_weight: src 16-B / dst 8-B alignment");
    dim3 grid((unsigned)((K + 63) / 64), (unsigned)((N + 63) / 64));
    pack_weight_kernel<<<grid, 256, 0, stream>>>(src, N, K, nscaled, scale, dst, dstT);
    return check_launch("vc_pack_weight");
}

}  // extern "C"
