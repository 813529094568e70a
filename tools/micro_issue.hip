// Microbenchmark (tools only, not part of libvclip.so): how VALU work of one wave and the
// MFMAs of another wave on the same SIMD share the SIMD.  Each wave stamps s_memtime around
// its loop; we report cycles per loop iteration for several pairings.
//   hipcc -O3 --offload-arch=gfx950 tools/micro_issue.hip -o tools/micro_issue && ./tools/micro_issue
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>

typedef __bf16 v8bf __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

constexpr int ITERS = 2000;

// role: 0 = idle, 1 = 32 v_exp_f32, 2 = 32 v_add_f32, 3 = 16 MFMA 32x32x16 (2 chains),
//       4 = softmax mix (32 exp + 31 add + 16 cvt_pk)
template <int ROLE>
__device__ void body(float* x, v16f* acc, v8bf a, v8bf b) {
    if constexpr (ROLE == 1) {
#pragma unroll
        for (int i = 0; i < 32; ++i) asm volatile("v_exp_f32 %0, %0" : "+v"(x[i]));
    } else if constexpr (ROLE == 2) {
#pragma unroll
        for (int i = 0; i < 32; ++i) asm volatile("v_add_f32 %0, 1.0, %0" : "+v"(x[i]));
    } else if constexpr (ROLE == 3) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[0], 0, 0, 0);
            acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[1], 0, 0, 0);
        }
    } else if constexpr (ROLE == 5) {  // 16 MFMA, one accumulator chain
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[0], 0, 0, 0);
    } else if constexpr (ROLE == 6) {  // 16 MFMA, four chains
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[0], 0, 0, 0);
            acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[1], 0, 0, 0);
            acc[2] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[2], 0, 0, 0);
            acc[3] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[3], 0, 0, 0);
        }
    } else if constexpr (ROLE == 7) {  // 16 MFMA 16x16x32 (four chains)
        typedef float v4f __attribute__((ext_vector_type(4)));
        v4f* a4 = reinterpret_cast<v4f*>(acc);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int c = 0; c < 4; ++c) a4[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, a4[c], 0, 0, 0);
    } else if constexpr (ROLE == 8) {  // 32 v_exp_f16 (low halves)
#pragma unroll
        for (int i = 0; i < 32; ++i) asm volatile("v_exp_f16 %0, %0" : "+v"(x[i]));
    } else if constexpr (ROLE == 9) {  // 32 f16 exps on 16 packed registers: low half + high half (SDWA)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            asm volatile("v_exp_f16 %0, %0" : "+v"(x[i]));
            asm volatile("v_exp_f16_sdwa %0, %0 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1" : "+v"(x[i]));
        }
    } else if constexpr (ROLE == 10) {  // f16 softmax step for 32 scores: 16 cvt_pk_f16 + 32 f16 exps
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            unsigned pk;
            asm volatile("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(pk) : "v"(x[2 * i]), "v"(x[2 * i + 1]));
            asm volatile("v_exp_f16 %0, %0" : "+v"(pk));
            asm volatile("v_exp_f16_sdwa %0, %0 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1" : "+v"(pk));
            x[2 * i] = __builtin_bit_cast(float, pk);
        }
    } else if constexpr (ROLE == 11) {  // bf16 softmax step for 32 scores: 32 exp_f32 + 16 cvt_pk_bf16
#pragma unroll
        for (int i = 0; i < 32; ++i) asm volatile("v_exp_f32 %0, %0" : "+v"(x[i]));
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            unsigned pk;
            asm volatile("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(pk) : "v"(x[2 * i]), "v"(x[2 * i + 1]));
            x[2 * i] = __builtin_bit_cast(float, pk);
        }
    } else if constexpr (ROLE == 4) {
#pragma unroll
        for (int i = 0; i < 32; ++i) asm volatile("v_exp_f32 %0, %0" : "+v"(x[i]));
        float s = x[0];
#pragma unroll
        for (int i = 1; i < 32; ++i) asm volatile("v_add_f32 %0, %0, %1" : "+v"(s) : "v"(x[i]));
        unsigned pk;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            asm volatile("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(pk) : "v"(x[2 * i]), "v"(x[2 * i + 1]));
            x[2 * i] = __builtin_bit_cast(float, pk);
        }
        x[0] += s;
    }
}

template <int RA, int RB>
__global__ void __launch_bounds__(512, 1) pair_kernel(unsigned long long* out, float seed) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    float x[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) x[i] = seed * (i + lane) * 1e-3f;
    v16f acc[4];
#pragma unroll
    for (int e = 0; e < 16; ++e) { acc[0][e] = 0.f; acc[1][e] = 0.f; acc[2][e] = 0.f; acc[3][e] = 0.f; }
    v8bf a, b;
#pragma unroll
    for (int i = 0; i < 8; ++i) { a[i] = (__bf16)(seed * i); b[i] = (__bf16)(seed + i); }
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < ITERS; ++it) {
        if (wave < 4) body<RA>(x, acc, a, b);
        else body<RB>(x, acc, a, b);
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 32; ++i) s += x[i];
#pragma unroll
    for (int e = 0; e < 16; ++e) s += acc[0][e] + acc[1][e] + acc[2][e] + acc[3][e];
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) {
        out[blockIdx.x * 8 + wave] = (t1 - t0) + (s == 12345.f ? 1 : 0);
        out[2048 + blockIdx.x * 8 + wave] = r1 - r0;
    }
}

template <int RA, int RB>
static void run(const char* name, int nthreads) {
    unsigned long long* d;
    hipMalloc(&d, 4096 * sizeof(unsigned long long));
    hipMemset(d, 0, 4096 * sizeof(unsigned long long));
    for (int rep = 0; rep < 3; ++rep) pair_kernel<RA, RB><<<256, nthreads>>>(d, 1.0f);
    hipDeviceSynchronize();
    std::vector<unsigned long long> h(4096);
    hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
    double sa = 0, sb = 0;
    int na = 0, nb = 0;
    for (int blk = 0; blk < 256; ++blk)
        for (int w = 0; w < nthreads / 64; ++w) {
            if (w < 4) { sa += h[blk * 8 + w]; ++na; }
            else { sb += h[blk * 8 + w]; ++nb; }
        }
    double rt = 0;
    for (int i = 0; i < 256 * 8; ++i) rt += h[2048 + i];
    double tt = 0;
    for (int i = 0; i < 256 * 8; ++i) tt += h[i];
    printf("%-44s groupA %8.1f tick/iter   groupB %8.1f tick/iter   (tick rate %.2f GHz)\n", name, sa / na / ITERS,
           nb ? sb / nb / ITERS : 0.0, tt / rt * 0.1);
    hipFree(d);
}

int main() {
    run<1, 0>("A: 32 exp_f32 alone (1 wave/SIMD)", 256);
    run<8, 0>("A: 32 exp_f16 alone", 256);
    run<9, 0>("A: 32 exp_f16 lo+hi(sdwa) alone", 256);
    run<11, 0>("A: bf16 softmax 32 exp_f32 + 16 cvt alone", 256);
    run<10, 0>("A: f16 softmax 16 cvt + 32 exp_f16 alone", 256);
    run<1, 1>("A: 32 exp_f32 | B: 32 exp_f32", 512);
    run<8, 8>("A: 32 exp_f16 | B: 32 exp_f16", 512);
    run<3, 11>("A: 16 MFMA | B: bf16 softmax", 512);
    run<3, 10>("A: 16 MFMA | B: f16 softmax", 512);
    run<3, 0>("A: 16 MFMA alone", 256);
    return 0;
}
