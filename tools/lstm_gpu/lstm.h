/* ResNet50-LSTM on the GPU: an out-of-scope experiment kept under tools/ (SURVEY.md §2 row 13 makes
 * the ResNet50-LSTM a CPU reference path, BASELINE configs[0]); not part of libvclip.so. */
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif
/* ---- ResNet50-LSTM (resnet50-2d-lstm/src/models/model.py:5-60) -----------
 * The per-frame ResNet-50 runs on the 3D conv path with kt = 1 kernels. */

/* out[n][c] = mean over p < P of x[n*P + p][c] (channels-last bf16 -> bf16): AdaptiveAvgPool2d(1). */
int vc_global_avgpool(const uint16_t* x, int64_t ldx, int64_t N, int64_t P, int64_t C, uint16_t* out, int64_t ldo,
                      hipStream_t stream);

/*
 * One nn.LSTM layer's recurrence (batch_first, zero initial state, torch gate order i, f, g, o):
 * pre[b*T + t][0:4H] = x_t . W_ih^T + b_ih + b_hh (f32, from the GEMM), W_hh f32 [4H][H];
 * h_out[b*T + t][0:H] = h_t (bf16, the next layer's GEMM input), h_last[b][0:H] = h_{T-1} (f32).
 * One workgroup per sequence, fp32 state.  H % 4 == 0, H <= 1024.
 */
int vc_lstm_recurrence(const float* pre, int64_t ldpre, int64_t B, int64_t T, int64_t hidden, const float* W_hh,
                       uint16_t* h_out, int64_t ldh, float* h_last, hipStream_t stream);

/* logits[b] = W2 . relu(W1 . h[b] + b1) + b2 (fp32): the reference's classifier Sequential. */
int vc_mlp_head(const float* h, int64_t B, int64_t hidden, const float* W1, const float* b1, int64_t H1, const float* W2,
                const float* b2, int64_t num_labels, float* logits, hipStream_t stream);

const char* lstm_last_error(void);
#ifdef __cplusplus
}
#endif
