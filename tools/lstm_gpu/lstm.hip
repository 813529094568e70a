// ResNet50-LSTM pieces (resnet50-2d-lstm/src/models/model.py:5-60): the
// per-frame global average pool of the ResNet-50 features, the LSTM recurrence (the input
// projections of all T steps run before it as one MFMA GEMM) and the 256 -> 64 -> 1 head.
#include "common.hpp"
#include "lstm.h"

// Out-of-scope experiment (the ResNet50-LSTM is BASELINE configs[0], a CPU
// reference path): built by tools/lstm_gpu/build.py into tools/lstm_gpu/liblstm.so, NOT part of
// libvclip.so.  It carries its own copy of the error helpers common.hpp declares.
namespace vc {
static thread_local std::string g_lstm_err;
void set_error(const std::string& msg) { g_lstm_err = msg; }
int fail(int code, const std::string& msg) {
    g_lstm_err = msg;
    return code;
}
int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        g_lstm_err = std::string(what) + ": " + hipGetErrorString(e);
        return (int)e;
    }
    return 0;
}
}  // namespace vc

namespace vc {

// features[n][c] = mean_p x[n*P + p][c] (channels-last bf16 in, bf16 out for the next GEMM)
__global__ void __launch_bounds__(256) global_avgpool_kernel(const uint16_t* __restrict__ x, int64_t ldx, int P, int C,
                                                             uint16_t* __restrict__ out, int64_t ldo) {
    const int64_t n = blockIdx.x;
    const int c = blockIdx.y * 256 + threadIdx.x;
    if (c >= C) return;
    float s = 0.f;
    for (int p = 0; p < P; ++p) s += bf2f(x[(n * P + p) * ldx + c]);
    out[n * ldo + c] = f2bf(s / (float)P);
}

__device__ __forceinline__ float sigmoidf_(float v) { return 1.0f / (1.0f + __expf(-v)); }

// One workgroup per sequence; thread j owns hidden unit j (Hs <= 256 threads... up to 1024 via
// a loop) and its four gate rows j, Hs+j, 2Hs+j, 3Hs+j (torch order i, f, g, o).
// pre[b*T + t][4Hs] = x_t . W_ih^T + b_ih + b_hh (f32); h_{t-1} is broadcast through LDS.
__global__ void __launch_bounds__(256) lstm_recurrence_kernel(const float* __restrict__ pre, int64_t ldpre, int T, int Hs,
                                                              const float* __restrict__ Whh, uint16_t* __restrict__ hout,
                                                              int64_t ldh, float* __restrict__ hlast) {
    extern __shared__ float hsh[];  // [Hs]
    const int b = blockIdx.x;
    float cst[4] = {0.f, 0.f, 0.f, 0.f};
    for (int j = threadIdx.x; j < Hs; j += 256) hsh[j] = 0.f;
    __syncthreads();
    for (int t = 0; t < T; ++t) {
        const float* pr = pre + ((int64_t)b * T + t) * ldpre;
        float hnew[4];
        int q = 0;
        for (int j = threadIdx.x; j < Hs; j += 256, ++q) {
            float g4[4];
#pragma unroll
            for (int gi = 0; gi < 4; ++gi) {
                const float* w = Whh + (int64_t)(gi * Hs + j) * Hs;
                float a = pr[gi * Hs + j];
                for (int k = 0; k < Hs; k += 4) {
                    const float4 wv = *reinterpret_cast<const float4*>(w + k);
                    a += wv.x * hsh[k] + wv.y * hsh[k + 1] + wv.z * hsh[k + 2] + wv.w * hsh[k + 3];
                }
                g4[gi] = a;
            }
            const float ig = sigmoidf_(g4[0]), fg = sigmoidf_(g4[1]), gg = tanhf(g4[2]), og = sigmoidf_(g4[3]);
            cst[q] = fg * cst[q] + ig * gg;
            hnew[q] = og * tanhf(cst[q]);
        }
        __syncthreads();  // every thread has read h_{t-1}
        q = 0;
        for (int j = threadIdx.x; j < Hs; j += 256, ++q) {
            hsh[j] = hnew[q];
            hout[((int64_t)b * T + t) * ldh + j] = f2bf(hnew[q]);
            if (t == T - 1) hlast[(int64_t)b * Hs + j] = hnew[q];
        }
        __syncthreads();
    }
}

// logits[b] = W2 . relu(W1 . h[b] + b1) + b2  (classifier: Linear, ReLU, Dropout(eval), Linear)
__global__ void __launch_bounds__(256) mlp_head_kernel(const float* __restrict__ h, int Hs, const float* __restrict__ W1,
                                                       const float* __restrict__ b1, int H1, const float* __restrict__ W2,
                                                       const float* __restrict__ b2, int nl, float* __restrict__ logits) {
    __shared__ float hid[1024];
    const int b = blockIdx.x;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int r = w; r < H1; r += 4) {
        float a = 0.f;
        for (int k = lane; k < Hs; k += 64) a += W1[(int64_t)r * Hs + k] * h[(int64_t)b * Hs + k];
        a = wave_sum(a);
        if (lane == 0) hid[r] = fmaxf(a + b1[r], 0.f);
    }
    __syncthreads();
    for (int c = w; c < nl; c += 4) {
        float a = 0.f;
        for (int k = lane; k < H1; k += 64) a += W2[(int64_t)c * H1 + k] * hid[k];
        a = wave_sum(a);
        if (lane == 0) logits[(int64_t)b * nl + c] = a + b2[c];
    }
}

}  // namespace vc

using namespace vc;

extern "C" {

int vc_global_avgpool(const uint16_t* x, int64_t ldx, int64_t N, int64_t P, int64_t C, uint16_t* out, int64_t ldo,
                      hipStream_t stream) {
    if (!x || !out) return fail(VC_ERR_INVALID_ARG, "vc_global_avgpool: null pointer");
    if (N <= 0 || P <= 0 || C <= 0 || ldx < C || ldo < C) return fail(VC_ERR_INVALID_ARG, "vc_global_avgpool: bad shape");
    global_avgpool_kernel<<<dim3((unsigned)N, (unsigned)((C + 255) / 256)), 256, 0, stream>>>(x, ldx, (int)P, (int)C, out, ldo);
    return check_launch("vc_global_avgpool");
}

int vc_lstm_recurrence(const float* pre, int64_t ldpre, int64_t B, int64_t T, int64_t hidden, const float* W_hh,
                       uint16_t* h_out, int64_t ldh, float* h_last, hipStream_t stream) {
    if (!pre || !W_hh || !h_out || !h_last) return fail(VC_ERR_INVALID_ARG, "vc_lstm_recurrence: null pointer");
    if (B <= 0 || T <= 0 || hidden <= 0 || hidden > 1024 || hidden % 4 || ldpre < 4 * hidden || ldh < hidden ||
        ((uintptr_t)W_hh & 15))
        return fail(VC_ERR_INVALID_ARG, "vc_lstm_recurrence: bad shape (hidden % 4 == 0, <= 1024)");
    lstm_recurrence_kernel<<<(unsigned)B, 256, hidden * sizeof(float), stream>>>(pre, ldpre, (int)T, (int)hidden, W_hh,
                                                                                 h_out, ldh, h_last);
    return check_launch("vc_lstm_recurrence");
}

int vc_mlp_head(const float* h, int64_t B, int64_t hidden, const float* W1, const float* b1, int64_t H1, const float* W2,
                const float* b2, int64_t num_labels, float* logits, hipStream_t stream) {
    if (!h || !W1 || !b1 || !W2 || !b2 || !logits) return fail(VC_ERR_INVALID_ARG, "vc_mlp_head: null pointer");
    if (H1 <= 0 || H1 > 1024) return fail(VC_ERR_INVALID_ARG, "vc_mlp_head: H1 in (0, 1024]");
    mlp_head_kernel<<<(unsigned)B, 256, 0, stream>>>(h, (int)hidden, W1, b1, (int)H1, W2, b2, (int)num_labels, logits);
    return check_launch("vc_mlp_head");
}

const char* lstm_last_error(void) { return vc::g_lstm_err.c_str(); }

}  // extern "C"
