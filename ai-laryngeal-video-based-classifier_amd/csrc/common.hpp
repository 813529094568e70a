// Shared helpers for the gfx950 kernels of libvclip.so.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "vclip.h"

namespace vc {

typedef short v4s __attribute__((ext_vector_type(4)));
typedef short v8s __attribute__((ext_vector_type(8)));
typedef __bf16 v8bf __attribute__((ext_vector_type(8)));
typedef float v2f __attribute__((ext_vector_type(2)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef unsigned int v2u __attribute__((ext_vector_type(2)));

typedef __attribute__((address_space(3))) v4s lds_v4s;

// error state (thread-local, set by host entry points)
void set_error(const std::string& msg);
int fail(int code, const std::string& msg);
int check_launch(const char* what);

// f32 -> bf16 round-to-nearest-even (hipcc lowers the scalar cast to v_cvt_pk_bf16_f32)
__device__ __forceinline__ unsigned short f2bf(float x) {
    __bf16 b = (__bf16)x;
    return __builtin_bit_cast(unsigned short, b);
}
// two f32 -> packed bf16 pair in ONE v_cvt_pk_bf16_f32 (RNE; the scalar casts + shift/or
// form costs four VALU ops)
typedef __bf16 v2bf __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned int pack2bf(float lo, float hi) {
    const v2f x = {lo, hi};
    return __builtin_bit_cast(unsigned int, __builtin_convertvector(x, v2bf));
}
__device__ __forceinline__ float bf2f(unsigned short u) {
    return __builtin_bit_cast(float, ((unsigned int)u) << 16);
}

// ---- 16-bit operand type of the inference forward (VC_ELEM_BF16 / VC_ELEM_F16).  Both run
// the same 32x32x16 MFMA rate; fp16 trades exponent range for 3 more mantissa bits (the
// ViViT-B logits move from ~4e-3 to ~7e-4 of the fp32 reference).  Kernels
// templated on ET keep their operands as raw 16-bit lanes (v8s) and go through these.
typedef _Float16 v2h __attribute__((ext_vector_type(2)));
typedef _Float16 v8h __attribute__((ext_vector_type(8)));
// two f32 -> one packed 16-bit pair (v_cvt_pk_bf16_f32 / v_cvt_pk_f16_f32, RNE)
template <int ET>
__device__ __forceinline__ unsigned int pack2(float lo, float hi) {
    const v2f x = {lo, hi};
    if constexpr (ET == VC_ELEM_F16) return __builtin_bit_cast(unsigned int, __builtin_convertvector(x, v2h));
    else return __builtin_bit_cast(unsigned int, __builtin_convertvector(x, v2bf));
}
template <int ET>
__device__ __forceinline__ unsigned short to16(float x) {
    if constexpr (ET == VC_ELEM_F16) return __builtin_bit_cast(unsigned short, (_Float16)x);
    else return f2bf(x);
}
template <int ET>
__device__ __forceinline__ float from16(unsigned short u) {
    if constexpr (ET == VC_ELEM_F16) return (float)__builtin_bit_cast(_Float16, u);
    else return bf2f(u);
}
// D = A.B + C over one 32x32x16 block, operands as raw 16-bit lanes
template <int ET>
__device__ __forceinline__ v16f mfma32x16(v8s a, v8s b, v16f c) {
    if constexpr (ET == VC_ELEM_F16)
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(v8h, a), __builtin_bit_cast(v8h, b), c, 0, 0, 0);
    else
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(v8bf, a), __builtin_bit_cast(v8bf, b), c, 0, 0, 0);
}
// D = A.B + C over one 16x16x32 block: lane l holds A[l & 15][8(l >> 4) .. +7], B likewise,
// and D[4(l >> 4) + e][l & 15] in c[e]
template <int ET>
__device__ __forceinline__ v4f mfma16x32(v8s a, v8s b, v4f c) {
    if constexpr (ET == VC_ELEM_F16)
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(v8h, a), __builtin_bit_cast(v8h, b), c, 0, 0, 0);
    else
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(v8bf, a), __builtin_bit_cast(v8bf, b), c, 0, 0, 0);
}

__device__ __forceinline__ float gelu_tanh(float x) {
    // gelu_fast: 0.5x(1+tanh(u)), u = 0.7978845608 x (1 + 0.044715 x^2)  (TF5/activations.py)
    // evaluated as x * sigmoid(2u) = x / (1 + 2^(-2u log2 e)): one v_exp_f32 + one v_rcp_f32
    // instead of libm tanhf (rel. error ~1e-7, far below the bf16 rounding of the output).
    // constants folded: -2 log2(e) u = x (k1 + k2 x^2), k1 = -2 log2(e) 0.7978845608, k2 = k1 0.044715
    // (5 VALU + 2 transcendental per element in the fc1 epilogue)
    const float z = x * __builtin_fmaf(-0.10294324f, x * x, -2.3022082f);
    return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(z));
}
// d/dx gelu_fast = 0.5(1 + tanh u) + 0.5 x (1 - tanh^2 u) * 0.7978845608 (1 + 3*0.044715 x^2)
__device__ __forceinline__ float dgelu_tanh(float x) {
    const float u = 0.7978845608f * x * (1.0f + 0.044715f * x * x);
    // tanh(u) = 1 - 2 / (exp(2u) + 1): one v_exp_f32 + one v_rcp_f32 (libm tanhf is a long
    // branchy sequence in the epilogue); exp -> inf / 0 gives the +-1 limits exactly
    const float t = 1.0f - 2.0f * __builtin_amdgcn_rcpf(__builtin_amdgcn_exp2f(2.8853900817779268f * u) + 1.0f);
    return 0.5f * (1.0f + t) + 0.5f * x * (1.0f - t * t) * 0.7978845608f * (1.0f + 0.134145f * x * x);
}
// exact GELU x * Phi(x), Phi(x) = 1 - h (x >= 0) or h (x < 0), h = erfc(|x|/sqrt 2) / 2 from
// Abramowitz-Stegun 7.1.26 (|erfc error| <= 1.5e-7): h = t P(t) exp(-x^2/2), t = 1/(1 + p|x|/sqrt 2).
// One v_rcp_f32 + one v_exp_f32 + ~11 VALU, no branches, instead of ocml's erff (two
// polynomial ranges, both evaluated under divergence).  Max |gelu error| 4.2e-7 over
// [-12, 12] vs an fp64 GELU (checked in numpy), far below the bf16 rounding of the output.
__device__ __forceinline__ float gelu_erf(float x) {
    const float t = __builtin_amdgcn_rcpf(__builtin_fmaf(0.23164189f, __builtin_fabsf(x), 1.0f));
    float p = __builtin_fmaf(t, 0.5307027145f, -0.7265760135f);
    p = __builtin_fmaf(t, p, 0.7107068705f);
    p = __builtin_fmaf(t, p, -0.142248368f);
    p = __builtin_fmaf(t, p, 0.127414796f);
    const float h = t * p * __builtin_amdgcn_exp2f(x * x * -0.72134752044448170f);
    return x * (x >= 0.0f ? 1.0f - h : h);
}

// sum over aligned groups of L lanes (L a power of two <= 64): every lane gets its group's sum
template <int L>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
    for (int o = L / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

}  // namespace vc
