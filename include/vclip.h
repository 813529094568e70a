/*
 * vclip.h — C-ABI of libvclip.so, the MI355X (gfx950) kernels of the video-clip
 * classification hot path.  Plain pointers, sizes and a hipStream_t; no torch types.
 *
 * The reference has no FFI: its arithmetic runs inside torch modules built by its model
 * factories.  Each entry point below replaces one piece of that arithmetic; the
 * reference interface it stands in for is cited per function.
 *
 * Conventions (SURVEY.md §8b "C-ABI"):
 *   - every pointer is a DEVICE pointer owned by the caller (the library never frees
 *     caller memory and never allocates in a launch: graph-capture safe);
 *   - work is enqueued asynchronously on `stream` (pass the caller's current stream);
 *   - return 0 on success, otherwise a hipError_t or VC_ERR_* code; the message is
 *     available from vc_last_error() (thread-local);  no exception crosses the ABI;
 *   - bf16 tensors are passed as uint16_t* (raw bfloat16 bits);
 *   - single host thread per process, one process per GPU; re-entrant, no global
 *     mutable device state.
 */
#ifndef VCLIP_H_
#define VCLIP_H_

#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VC_ERR_INVALID_ARG (-1)
#define VC_ERR_UNSUPPORTED (-2)

/* Library identity: returns a static string "vclip <version> gfx950". */
const char* vc_version(void);

/* Thread-local message of the last failing call ("" if none). */
const char* vc_last_error(void);

/* Output element types of vc_frame_gather. */
#define VC_GATHER_U8_NHWC   0  /* out u8  [nclips][T][H][W][C]: exact copy of the sampled frames      */
#define VC_GATHER_F32_NCHW  1  /* out f32 [nclips][T][C][H][W] = x*scale + shift                       */
#define VC_GATHER_BF16_NCHW 2  /* out bf16[nclips][T][C][H][W] = bf16(x*scale + shift)                 */

/*
 * Frame-index gather (+ normalise + layout permute).
 * Replaces: the per-clip frame gather `frames[idx - start_idx]` of
 *   vivit_transformer/vivit_classifier/data_config/dataset.py:248-265 (u8 mode), and the
 *   processor affine x/63.75-3 with the [T,H,W,C]->[T,C,H,W] stack of
 *   vivit_transformer/vivit_classifier/trainers/trainer.py:62-95 (float modes).
 * frames: u8 [nclips][F][H][W][C] (decoded frames of each clip, F per clip);
 * idx:    int64 [nclips][T] frame indices, clamped to [0, F-1] like dataset.py:252-253.
 */
int vc_frame_gather(const uint8_t* frames, int64_t nclips, int64_t F, int64_t H, int64_t W, int64_t C,
                    const int64_t* idx, int64_t T, int out_kind, float scale, float shift,
                    void* out, hipStream_t stream);

/*
 * Tubelet im2col: pixel_values f32 [B][T][C][H][W] -> A bf16 [B*nt*nh*nw][C*kt*kh*kw]
 * (row = token in t,h,w order; column = (c,kt,kh,kw) = Conv3d weight order).
 * Replaces the input side of VivitTubeletEmbeddings (TF5/models/vivit/modeling_vivit.py:64-67).
 */
int vc_tubelet_im2col(const float* pixel_values, int64_t B, int64_t T, int64_t C, int64_t H, int64_t W,
                      int kt, int kh, int kw, uint16_t* A, int64_t lda, hipStream_t stream);

/* Token orders of vc_patch_im2col. */
#define VC_TOKENS_TIME_MAJOR  0  /* row = ((b*nt + t')*nh + hp)*nw + wp   (ViViT, modeling_vivit.py:64-67)          */
#define VC_TOKENS_PATCH_MAJOR 1  /* row = ((b*nh + hp)*nw + wp)*nt + t'   (TimeSformer, modeling_timesformer.py:121-143) */

/* Input layouts of vc_patch_im2col. */
#define VC_VIDEO_BTCHW 0  /* [B][T][C][H][W]: HF pixel_values (ViViT, TimeSformer)                   */
#define VC_VIDEO_BCTHW 1  /* [B][C][T][H][W]: torchvision video models (Swin3D, ResNet3D; trainer.py:116) */

/*
 * vc_tubelet_im2col with an explicit token order and input layout; kw % 4 == 0.
 * kt = 1 + VC_TOKENS_PATCH_MAJOR: the input side of TimeSformer's per-frame Conv2d patch
 * embedding re-ordered patch-major / time-minor (TF5/models/timesformer/modeling_timesformer.py:
 * 45-60, 121-143).  (2,4,4) + VC_VIDEO_BCTHW: torchvision PatchEmbed3d's Conv3d (Swin3D-T).
 */
int vc_patch_im2col(const float* pixel_values, int64_t B, int64_t T, int64_t C, int64_t H, int64_t W,
                    int kt, int kh, int kw, int token_order, int layout, uint16_t* A, int64_t lda,
                    hipStream_t stream);

/* GEMM epilogues for vc_gemm_bf16. */
#define VC_EPI_BIAS_BF16        0  /* out bf16[m][n]  = acc + bias[n]                               */
#define VC_EPI_BIAS_GELU_TANH   1  /* out bf16[m][n]  = gelu_fast(acc + bias[n])  (ViViT MLP fc1)    */
#define VC_EPI_BIAS_GELU_ERF    2  /* out bf16[m][n]  = gelu_erf(acc + bias[n])   (TimeSformer/Swin) */
#define VC_EPI_BIAS_RESID_F32   3  /* out f32 [m][n] += acc + bias[n]             (o_proj, fc2)       */
#define VC_EPI_EMBED_F32        4  /* out f32 [r(m)][n] = acc + bias[n] + aux[m % G][n],
                                       r(m) = (m / G) * group_stride + group_offset (tubelet -> tokens) */
#define VC_EPI_BIAS_F32         5  /* out f32 [m][n]  = acc + bias[n]             (Swin embed / merge)  */
#define VC_EPI_BIAS_RELU_BF16   6  /* out bf16[m][n]  = relu(acc + bias[n])       (conv + BN + ReLU)    */
#define VC_EPI_BIAS_RESID_RELU_BF16 7 /* out bf16[m][n] = relu(acc + bias[n] + res[m][n]), res = (const
                                       uint16_t*)aux bf16 with row stride ldaux (bottleneck conv_c + skip) */
/* Training epilogues (ViViT train step; block configs 0-3): */
#define VC_EPI_BIAS_ADD_F32     8  /* out f32 [m][n]  = aux[m][n] + acc + bias[n]  (residual into a new buffer,
                                       so the layer input stays saved for the backward)                    */
#define VC_EPI_BIAS_GELU_TANH_SAVE 9 /* out bf16[m][n] = gelu_fast(acc + bias[n]); (uint16_t*)aux[m][n] =
                                       bf16(acc + bias[n]), the pre-activation kept for the backward      */
#define VC_EPI_DGELU_TANH      10  /* out bf16[m][n]  = (acc + bias[n]) * gelu_fast'((uint16_t*)aux[m][n]):
                                       the fc2 dgrad fused with the gelu backward                          */

/*
 * C[M][N] = A[M][K] . W[N][K]^T  (bf16 inputs, fp32 accumulate on MFMA), fused epilogue.
 * Replaces torch nn.Linear (cuBLAS addmm) of every q/k/v/o/fc1/fc2 projection
 * (TF5/models/vivit/modeling_vivit.py:186-189, 229-237) and, with VC_EPI_EMBED_F32, the
 * Conv3d GEMM + CLS/position add of TF5/.../modeling_vivit.py:64-67,126-146.
 * Requirements: M % 128 == 0 (callers pad rows), N % 128 == 0, K % 64 == 0,
 * lda/ldw multiples of 8 elements, 16-byte aligned pointers.
 */
int vc_gemm_bf16(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw,
                 int64_t M, int64_t N, int64_t K, const float* bias, int epilogue,
                 void* out, int64_t ldo, const float* aux, int64_t ldaux,
                 int64_t G, int64_t group_stride, int64_t group_offset, hipStream_t stream);

/*
 * Same as vc_gemm_bf16 with an explicit block-tile configuration (tuning hook):
 *   cfg 0: 256x128, cfg 1: 128x128, cfg 2: 128x256, cfg 3: 256x256, cfg 4: 256x256 persistent
 *   (bf16-output epilogues 0/1/2/6 only), cfg 5: 128x128 with a 2-tile LDS ring (two workgroups
 *   per CU), cfg 7: 64x128 (two workgroups per CU); -1 = automatic (measured choice, gemm.hip pick_cfg).
 */
int vc_gemm_bf16_cfg(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw,
                     int64_t M, int64_t N, int64_t K, const float* bias, int epilogue,
                     void* out, int64_t ldo, const float* aux, int64_t ldaux,
                     int64_t G, int64_t group_stride, int64_t group_offset, int cfg, hipStream_t stream);

/*
 * Row LayerNorm: y bf16[m][:] = (x[m]-mean)/sqrt(var+eps)*gamma + beta, x f32, stats f32.
 * Replaces nn.LayerNorm layernorm_before/after (TF5/.../modeling_vivit.py:245-246, 258, 266).
 */
int vc_layernorm_f32_bf16(const float* x, int64_t ldx, int64_t M, int64_t D,
                          const float* gamma, const float* beta, float eps,
                          uint16_t* y, int64_t ldy, hipStream_t stream);

/*
 * Fused joint (non-causal) attention forward, head_dim 64, flash-style online softmax
 * in fp32, MFMA bf16 for Q.K^T and P.V.
 * qkv: bf16 rows of `ld` elements, row (b*S + s); head h's q at column h*64,
 *      k at H*64 + h*64, v at 2*H*64 + h*64 (the fused q|k|v projection output).
 * out: bf16 rows of `ldo` elements, head h at column h*64 (the o_proj input layout).
 * softmax(scale * q.k) with `scale` = head_dim^-0.5 in ViViT.  The kernel evaluates
 * exp2(q'.k - running max) with q' = q * scale * log2(e): if q_prescaled != 0 the
 * producer already stored q' (e.g. folded into the q projection weights and bias, one
 * rounding), otherwise the kernel forms q' in fp32 and re-rounds it to bf16.
 * Rows of qkv must be readable up to (B-1)*S + roundup(S, 64) - 1 (callers pad).
 * Replaces eager_attention_forward / SDPA (TF5/.../modeling_vivit.py:149-174, 177-223).
 */
int vc_attention_fwd(const uint16_t* qkv, int64_t ld, int64_t B, int64_t S, int64_t H, int64_t head_dim,
                     float scale, int q_prescaled, uint16_t* out, int64_t ldo, hipStream_t stream);

/* Test build of vc_attention_fwd's deferred running max (q not prescaled): re-bases the max on
 * EVERY key tile instead of only when a lane's partial row sum exceeds 2^8.  Must agree with
 * vc_attention_fwd to rounding (tests/test_kernels_gpu.py threshold sweep). */
int vc_attention_fwd_rebase_always(const uint16_t* qkv, int64_t ld, int64_t B, int64_t S, int64_t H, float scale,
                                   uint16_t* out, int64_t ldo, hipStream_t stream);

/*
 * 16-bit operand type of the inference forward (`elem` of the *_h16 entry points below).
 * VC_ELEM_BF16 is the benchmarked configuration (north_star: "ViViT-B ... forward bf16");
 * VC_ELEM_F16 runs the same kernels at the same MFMA rate with fp16 operands — 3 more
 * mantissa bits, 5 fewer exponent bits — for logits within 1e-3 of the fp32 reference
 * (DESIGN.md §6).  Accumulation, softmax statistics, LayerNorm statistics and the residual
 * stream stay fp32 in both.
 */
#define VC_ELEM_BF16 0
#define VC_ELEM_F16  1

/* vc_patch_im2col with the output element type as an argument. */
int vc_patch_im2col_h16(const float* pixel_values, int64_t B, int64_t T, int64_t C, int64_t H, int64_t W,
                        int kt, int kh, int kw, int token_order, int layout, int elem, uint16_t* A, int64_t lda,
                        hipStream_t stream);

/* The tile config (kCfgs index) that vc_gemm_bf16 / vc_gemm_h16 pick with cfg = -1 for this shape,
 * epilogue and output / aux layout (host-only query: no launch; instrumentation labels launches
 * with it). */
int vc_gemm_pick(int64_t M, int64_t N, int64_t K, int epilogue, int64_t ldo, int64_t ldaux, const void* aux);

/* vc_gemm_bf16_cfg with the operand type as an argument: A, W and the 16-bit outputs are `elem`;
 * fp16 supports epilogues 0-4 (the inference forward's), bf16 all of them. */
int vc_gemm_h16(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw,
                int64_t M, int64_t N, int64_t K, const float* bias, int epilogue,
                void* out, int64_t ldo, const float* aux, int64_t ldaux,
                int64_t G, int64_t group_stride, int64_t group_offset, int elem, int cfg, hipStream_t stream);

/* vc_gemm_h16 on the 256x256 ping-pong kernel with A's columns wrapping at ka (ka % 64 == 0,
 * ka <= K <= 2 ka, M % 256 == N % 256 == 0, epilogues 0-4): W = [W1 | W2] against A [M][ka] sums
 * A.W1 + A.W2 in one fp32 accumulation chain.  With W1 / W2 the high / low 16-bit parts of fp32
 * weights (and, for the patch embedding, A = [A_hi | A_lo] from vc_patch_im2col_split_h16 against
 * W = [W_hi | W_hi | W_lo]) this is the split-operand product of the fp16 build's first layers
 * (VivitForVideoClassification.precise_layers). */
int vc_gemm_h16_wrap(const uint16_t* A, int64_t lda, int64_t ka, const uint16_t* W, int64_t ldw, int64_t M,
                     int64_t N, int64_t K, const float* bias, int epilogue, void* out, int64_t ldo, const float* aux,
                     int64_t ldaux, int64_t G, int64_t group_stride, int64_t group_offset, int elem,
                     hipStream_t stream);
/* vc_patch_im2col_h16 writing [A_hi | A_lo] (2K columns, K = C kt kh kw; 8-wide patches): the 16-bit
 * pixel values and their rounding residuals. */
int vc_patch_im2col_split_h16(const float* pixel_values, int64_t B, int64_t T, int64_t C, int64_t H, int64_t W,
                              int kt, int kh, int kw, int token_order, int layout, int elem, uint16_t* A, int64_t lda,
                              hipStream_t stream);

/* vc_layernorm_f32_bf16 with the output type as an argument (same widths and kernels). */
int vc_layernorm_f32_h16(const float* x, int64_t ldx, int64_t M, int64_t D, const float* gamma, const float* beta,
                         float eps, int elem, uint16_t* y, int64_t ldy, hipStream_t stream);

/* vc_attention_fwd with the operand type of q|k|v, P and out as an argument. */
int vc_attention_fwd_h16(const uint16_t* qkv, int64_t ld, int64_t B, int64_t S, int64_t H, int64_t head_dim,
                         float scale, int q_prescaled, int elem, uint16_t* out, int64_t ldo, hipStream_t stream);

/* LayerNorm f32 -> f32 (any D; y may alias nothing of x).  Swin's patch_embed.norm (torchvision
 * PatchEmbed3d, eps 1e-5) whose output is the fp32 residual stream. */
int vc_layernorm_f32(const float* x, int64_t ldx, int64_t M, int64_t D, const float* gamma, const float* beta,
                     float eps, float* y, int64_t ldy, hipStream_t stream);

/* `blocks` one-wave workgroups, each sleeping iters x s_sleep 127, on `stream` (no memory traffic): the
 * hardware-queue probe of vclip_amd.streams.pick_streams.  No reference counterpart (the reference
 * runs one CUDA stream). */
int vc_spin(int64_t iters, int64_t blocks, hipStream_t stream);

/* CLS rows: x[b*S][:] = cls[:] + pos[0][:]   (TF5/.../modeling_vivit.py:131-142). */
int vc_cls_init(const float* cls, const float* pos, float* x, int64_t ldx, int64_t B, int64_t S, int64_t D,
                hipStream_t stream);

/*
 * Classifier head on the CLS rows: logits[b][c] = LN(x[b*S])[:] . Wc[c][:] + bc[c] (fp32).
 * Replaces the final LayerNorm + classifier of TF5/.../modeling_vivit.py:427, 556
 * (only the CLS row feeds the logits, so only it is normalised).
 */
int vc_cls_head(const float* x, int64_t ldx, int64_t B, int64_t S, int64_t D,
                const float* gamma, const float* beta, float eps,
                const float* Wc, const float* bc, int64_t num_labels, float* logits, hipStream_t stream);

/* ---- Clip preprocessing ------------------------------------------- */

/*
 * One axis of Pillow's BILINEAR resize of uint8 images [N][H][W][C] (C <= 4), bit-exact:
 * axis 0 resizes W -> out_size, axis 1 resizes H -> out_size.  bounds (int32 [out_size][2]:
 * first source index, tap count) and coeffs (int32 [out_size][ksize], 22 fraction bits) are
 * DEVICE tables built on the host exactly as Pillow's precompute_coeffs + normalize_coeffs_8bpc
 * (vclip_amd/preprocess.py); each pass rounds to uint8 as Pillow's clip8 does.  Two passes
 * (horizontal, then vertical) = PIL Image.resize(..., BILINEAR), which the ViViT processor
 * applies per frame (VivitImageProcessor, vivit_transformer/.../trainers/trainer.py:22-26).
 */
int vc_resample_u8(const uint8_t* src, int64_t N, int64_t H, int64_t W, int64_t C, int axis, int64_t out_size,
                   const int* bounds, const int* coeffs, int64_t ksize, uint8_t* dst, hipStream_t stream);

/*
 * OpenCV cv2.resize(frame, (w, h)) with INTER_LINEAR on N uint8 frames [N][H][W][C] -> [N][h][w][C]
 * (C <= 4): the reference's resize of decoded frames to 224x224 (vivit_transformer/vivit_classifier/
 * data_config/dataset.py:271-277, :348; vivit_transformer/inference.py:155).  tables: int32
 * xofs[w] | xa0[w] | xa1[w] | yofs[h] | yb0[h] | yb1[h] (11-bit coefficients, vclip_amd/resize.py
 * linear_tables); columns >= xlim copy the last source column.  area2x != 0: an exact 2x
 * downscale, INTER_AREA's fast 2x2 average (tables may be null).
 */
int vc_resize_linear_u8(const uint8_t* src, int64_t N, int64_t H, int64_t W, int64_t C, int64_t h, int64_t w,
                        const int* tables, int64_t xlim, int area2x, uint8_t* dst, hipStream_t stream);

/*
 * frames u8 [nclips][F][H][W][3] -> out[clip][t] = affine(crop(resize(frames[clip][idx[clip][t]]))):
 * idx int64 [nclips][T] (clamped to [0, F-1]); resize to (resize_h, resize_w) with torch
 * F.interpolate bilinear, align_corners=False semantics (skipped when equal to (H, W)); crop
 * (top, left, crop_h, crop_w); per-channel out = v * scale3[c] + shift3[c] (scale3 / shift3 are
 * HOST float[3]); layout 0: [clip][T][3][h][w] (HF pixel_values), 1: [clip][3][T][h][w]
 * (torchvision video models); f32 or (out_bf16) bf16.  Replaces pytorchvideo
 * UniformTemporalSubsample + ShortSideScale + CenterCrop + Normalize (videoswintransformer/.../
 * dataset.py:162-170, resnet50-3d-video/.../dataset.py:186-192), the inference scripts' /255 +
 * normalise (resnet50-3d-video/inference.py:382-394) and, after vc_resample_u8, the ViViT affine.
 */
int vc_video_transform(const uint8_t* frames, int64_t nclips, int64_t F, int64_t H, int64_t W, const int64_t* idx,
                       int64_t T, int64_t resize_h, int64_t resize_w, int64_t top, int64_t left, int64_t crop_h,
                       int64_t crop_w, const float* scale3, const float* shift3, int layout, int out_bf16, void* out,
                       hipStream_t stream);

/*
 * Train-time variant (videoswintransformer/.../data_config/dataset.py:151-163 train chain:
 * UniformTemporalSubsample -> RandomShortSideScale(256, 320) -> RandomCrop(224) ->
 * RandomHorizontalFlip(0.5) -> Normalize): clip_params = device int32 [nclips][5]
 * {resize_h, resize_w, top, left, flip} drawn on the host (vclip_amd/preprocess.py
 * video_train_transform, torch's RNG in the reference's draw order); each clip is resized, cropped
 * to crop_h x crop_w at (top, left), mirrored when flip != 0, and normalised.  The caller keeps
 * every crop window inside its resized frame.
 */
int vc_video_transform_clips(const uint8_t* frames, int64_t nclips, int64_t F, int64_t H, int64_t W, const int64_t* idx,
                             int64_t T, const int* clip_params, int64_t crop_h, int64_t crop_w, const float* scale3,
                             const float* shift3, int layout, int out_bf16, void* out, hipStream_t stream);

/* ---- TimeSformer divided space-time attention ------------------------
 * Clip layout: rows b*S + r, S = 1 + P*T, r = 0 (CLS) or 1 + p*T + t (patch-major, time-minor).
 * Frame layout: rows (b*T + t)*(1 + P) + j, j = 0 (CLS copy) or 1 + p (the spatial sequences). */

/*
 * Temporal attention: for each clip b, patch p and head, softmax(scale * q.k) v over the T
 * rows 1 + p*T + t of the clip layout (one head_dim-64 slice per head of the fused q|k|v
 * rows, as vc_attention_fwd).  out gets the same rows; CLS rows are not written.
 * q_prescaled: q already carries scale*log2(e) (then exp2 is used), else q is scaled in fp32.
 * Replaces TimesformerLayer's temporal branch attention (TF5/models/timesformer/
 * modeling_timesformer.py:337-347 with TimesformerSelfAttention :148-180).  T <= 32.
 */
int vc_temporal_attention(const uint16_t* qkv, int64_t ld, int64_t B, int64_t P, int64_t T, int64_t H,
                          int64_t head_dim, float scale, int q_prescaled, uint16_t* out, int64_t ldo,
                          hipStream_t stream);

#define VC_DIVIDED_TEMPORAL_TO_SPATIAL 0
#define VC_DIVIDED_SPATIAL_TO_MLP      1
/*
 * Residual add + LayerNorm across the two layouts, fp32 residual x (clip layout), bf16 y, h.
 *  mode 0: x[patch rows] += y[same rows] (y clip layout, the temporal_dense output) ->
 *          h (frame layout) = LN(x) with each clip's CLS row LN-ed and copied to its T frames
 *          (modeling_timesformer.py:349-366: temporal residual, CLS repeat, layernorm_before);
 *  mode 1: x[patch row] += y[its frame-layout row]; x[CLS] += mean over t of y[(b*T+t)*(1+P)]
 *          -> h (clip layout) = LN(x)   (modeling_timesformer.py:371-391: CLS mean, residual,
 *          layernorm_after).
 * D % 4 == 0, D <= 1024.
 */
int vc_divided_add_layernorm(float* x, int64_t ldx, const uint16_t* y, int64_t ldy, int64_t B, int64_t P, int64_t T,
                             int64_t D, const float* gamma, const float* beta, float eps, int mode, uint16_t* h,
                             int64_t ldh, hipStream_t stream);

/* ---- 3D convolutions (ResNet3D-50, pytorchvideo create_resnet) ------------
 * A Conv3d is vc_conv3d_im2col + vc_gemm_bf16 with the BatchNorm folded into W / bias and ReLU
 * (+ the residual) in the epilogue.  Channels-last activations: rows ((b*T + t)*H + h)*W + w. */
#define VC_CONV_IN_NCTHW_F32 0  /* the f32 [B][C][T][H][W] clip (stem); columns (c, kt, kh, kw)      */
#define VC_CONV_IN_CL_BF16   1  /* channels-last bf16 rows (ld = ldx), C % 8 == 0; columns (kt, kh, kw, c) */
/*
 * A[m][col] for output position m = ((b*To + to)*Ho + ho)*Wo + wo, zero padding, with
 * To = (T + 2p_t - k_t)/s_t + 1 (etc.); kernel/stride/pad are int[3] host arrays (t, h, w).
 * Replaces the input side of torch.nn.Conv3d in pytorchvideo's stem / bottleneck blocks.
 */
int vc_conv3d_im2col(const void* x, int64_t ldx, int input_kind, int64_t B, int64_t T, int64_t H, int64_t W,
                     int64_t C, const int* kernel, const int* stride, const int* pad, uint16_t* A, int64_t lda,
                     hipStream_t stream);

/* Implicit-GEMM Conv3d on channels-last bf16 activations (no im2col buffer): out[m][n] =
 * epilogue(sum over (tap, c) of x[in(m, tap)][c] * Wt[n][tap*C + c] + bias[n]) with the
 * vc_conv3d_im2col column order (kt, kh, kw, c); epilogue VC_EPI_BIAS_BF16 / _RELU_BF16 /
 * _RESID_RELU_BF16 (aux = the bf16 residual).  C % 64 == 0, N % 128 == 0 (zero-padded output
 * channels); `zero_row` points to >= 64 zero bf16 (the padding taps' source); the output rows
 * up to the next multiple of 128 are written (the caller's buffer holds them).  Replaces
 * vc_conv3d_im2col + vc_gemm_bf16 for pytorchvideo's conv_a / conv_b / strided branch1
 * (resnet50-3d-video/video_classifier/models/resnet3d.py:4-48). */
int vc_conv3d_gemm_bf16(const uint16_t* x, int64_t ldx, int64_t B, int64_t T, int64_t H, int64_t W, int64_t C,
                        const int* kernel, const int* stride, const int* pad, const uint16_t* zero_row,
                        const uint16_t* Wt, int64_t ldw, int64_t N, const float* bias, int epilogue, void* out,
                        int64_t ldo, const void* aux, int64_t ldaux, hipStream_t stream);
/* The same with the LDS ring depth chosen by the caller (a tuning entry, as vc_gemm_bf16_cfg):
 * ring 0 = automatic (what vc_conv3d_gemm_bf16 runs: 3 k-tiles when the grid has fewer than two
 * tiles per CU, else 2), 2, or 3 (one more k-tile in flight, one workgroup per CU except at 64 x 128
 * tiles).  Results are bit-identical for every ring. */
int vc_conv3d_gemm_bf16_ring(const uint16_t* x, int64_t ldx, int64_t B, int64_t T, int64_t H, int64_t W, int64_t C,
                             const int* kernel, const int* stride, const int* pad, const uint16_t* zero_row,
                             const uint16_t* Wt, int64_t ldw, int64_t N, const float* bias, int epilogue, void* out,
                             int64_t ldo, const void* aux, int64_t ldaux, int ring, hipStream_t stream);
/* The same with the tile chosen by the caller too (a tuning entry): tile 0 = automatic (what
 * vc_conv3d_gemm_bf16 runs: 256 x 64 for N % 128 != 0, 64 x 128 when 128 x 128 tiles would be fewer
 * than the CUs, else 128 x 128), 1 = 64 x 128, 2 = 128 x 128 (N % 128 == 0, bias / bias_relu for
 * tile 1); ring 0, 2, 3 or 4 (4: one workgroup per CU; 3 on 256 x 64 tiles).  Bit-identical for every
 * tile and ring. */
int vc_conv3d_gemm_bf16_cfg(const uint16_t* x, int64_t ldx, int64_t B, int64_t T, int64_t H, int64_t W, int64_t C,
                            const int* kernel, const int* stride, const int* pad, const uint16_t* zero_row,
                            const uint16_t* Wt, int64_t ldw, int64_t N, const float* bias, int epilogue, void* out,
                            int64_t ldo, const void* aux, int64_t ldaux, int ring, int tile, hipStream_t stream);

/* The stem Conv3d (3 input channels, kernel (kt, kh, kw <= 8), even w stride) as an implicit GEMM:
 * vc_conv3d_stem_pack writes the f32 [B][C][T][H][W] clip (C <= 4) as zero-padded channels-last
 * bf16 [B][T+2pt][H+2ph][W+2pw][4]; vc_conv3d_stem_gemm_bf16 reads one (kt, kh) tap row of 8
 * pixels x 4 channels as a 32-column segment, K = 64 * ceil(kt*kh / 2), Wt column
 * seg*32 + kw_i*4 + c for seg = kt_i*kh + kh_i (zero for kw_i >= kw, c >= C, seg >= kt*kh).
 * Replaces vc_conv3d_im2col (VC_CONV_IN_NCTHW_F32) + vc_gemm_bf16 for pytorchvideo's stem. */
int vc_conv3d_stem_pack(const float* x, int64_t B, int64_t C, int64_t T, int64_t H, int64_t W, const int* pad,
                        uint16_t* xp, hipStream_t stream);
int vc_conv3d_stem_gemm_bf16(const uint16_t* xp, int64_t B, int64_t T, int64_t H, int64_t W, const int* kernel,
                             const int* stride, const int* pad, const uint16_t* zero_row, const uint16_t* Wt,
                             int64_t ldw, int64_t N, const float* bias, int epilogue, void* out, int64_t ldo,
                             hipStream_t stream);

/* MaxPool3d on channels-last bf16 (padding counts as -inf): pytorchvideo's stem pool. */
int vc_maxpool3d(const uint16_t* x, int64_t ldx, int64_t B, int64_t T, int64_t H, int64_t W, int64_t C,
                 const int* kernel, const int* stride, const int* pad, uint16_t* y, int64_t ldy, hipStream_t stream);

/*
 * ResNetBasicHead (AvgPool3d(pool_kernel, stride 1) -> Linear -> AdaptiveAvgPool3d(1)) on
 * channels-last bf16 x: logits[b] = Wc . pooled[b] + bc, pooled = the position-weighted mean
 * (the Linear commutes with both averages).  work: caller scratch f32 [B * C * 33] (pooled + 32
 * fixed-order partial sums: deterministic).
 */
int vc_avgpool_head(const uint16_t* x, int64_t ldx, int64_t B, int64_t T, int64_t H, int64_t W, int64_t C,
                    const int* pool_kernel, const float* Wc, const float* bc, int64_t num_labels, float* work,
                    float* logits, hipStream_t stream);

/* ---- ResNet3D train step (conv3d_bwd.hip; resnet50-3d-video/.../trainers/trainer.py:106-123) ---- */

/* Backward of vc_conv3d_im2col (channels-last bf16 input): dx f32 [B*T*H*W][C] (row stride lddx)
 * = the sum of the dA [M_out][kt*kh*kw*C] entries that copied each input element (gather order
 * fixed: deterministic). */
int vc_col2im_cl(const uint16_t* dA, int64_t lda, int64_t B, int64_t T, int64_t H, int64_t W, int64_t C,
                 const int* kernel, const int* stride, const int* pad, float* dx, int64_t lddx, hipStream_t stream);

/* Backward of vc_maxpool3d: each output gradient (dy f32, or bf16 when dy_bf16) goes to the first
 * maximum of its window in (t, h, w) scan order (torch's max_pool3d indices); dx f32. */
int vc_maxpool3d_bwd(const uint16_t* x, int64_t ldx, const void* dy, int dy_bf16, int64_t lddy, int64_t B, int64_t T,
                     int64_t H, int64_t W, int64_t C, const int* kernel, const int* stride, const int* pad, float* dx,
                     int64_t lddx, hipStream_t stream);

/* nn.BatchNorm3d in training mode on channels-last rows y f32 [M][C] (C % 4 == 0): batch mean /
 * biased variance (two passes, fixed-order reductions) -> stat f32 [2][C] = {mean, rstd}; the
 * running statistics (if given) updated with `momentum` and the unbiased variance; z bf16 =
 * relu?(gamma * (y - mean) * rstd + beta (+ res: bf16 if res_bf16 else f32)).  work >= 2*C*splits
 * floats (splits = clamp(ceil(M / 128), 1, 4096)). */
int vc_batchnorm_train_fwd(const float* y, int64_t ldy, int64_t M, int64_t C, const float* gamma, const float* beta,
                           float eps, float momentum, float* running_mean, float* running_var, const void* res,
                           int res_bf16, int64_t ldr, int relu, uint16_t* z, int64_t ldz, float* stat, float* work,
                           int64_t work_elems, hipStream_t stream);

/* Its backward: g = dz (masked by z > 0 when relu); dbeta = sum g, dgamma = sum g * xhat;
 * dy = gamma * rstd * (g - dbeta / M - xhat * dgamma / M); dres (optional) = g. */
int vc_batchnorm_train_bwd(const float* y, int64_t ldy, int64_t M, int64_t C, const float* stat, const float* gamma,
                           const float* dz, int64_t lddz, const uint16_t* z, int64_t ldz, int relu, float* dy,
                           int64_t lddy, float* dres, int64_t lddr, float* dgamma, float* dbeta, float* work,
                           int64_t work_elems, hipStream_t stream);

/* pytorchvideo ResNetBasicHead in training mode on the final map x bf16 [B*T*HW][C] (one spatial
 * pool window = the whole HW): u f32 [B][C] = the AdaptiveAvgPool of the per-position inputs of
 * the Linear after AvgPool3d((pool_t, ., .), stride 1) and Dropout (keep f32 [B][T-pool_t+1][C] =
 * 0 or 1/(1-p)); logits = Wc . u + bc (fp32).  Backward: vc_pool_head_bwd (scale 1) gives du, dWc,
 * dbc; vc_resnet_head_train_bwd spreads du over x. */
int vc_resnet_head_train(const uint16_t* x, int64_t ldx, int64_t B, int64_t T, int64_t HW, int64_t C, int pool_t,
                         const float* keep, const float* Wc, const float* bc, int64_t num_labels, float* u,
                         float* logits, hipStream_t stream);
int vc_resnet_head_train_bwd(const float* du, int64_t B, int64_t T, int64_t HW, int64_t C, int pool_t, const float* keep,
                             float* dx, int64_t lddx, hipStream_t stream);

/* ---- Video Swin 3D (torchvision swin3d_t) -------------------------------
 * Token layout: rows ((b*T + t)*H + h)*W + w (channels-last [B][T][H][W][C]). */

/*
 * Shifted-window attention core, head_dim 32: for every window of (wt,wh,ww) tokens of the grid
 * rolled by -(st,sh,sw), softmax(q'.k + bias [+ shift mask]) v per head.  qkv: bf16 rows of the
 * fused q|k|v projection (head h: q at h*32, k at C + h*32, v at 2C + h*32, C = heads*32), with
 * q' = q * d^-1/2 * log2(e) (folded into the projection).  biasF: f32, the log2(e)-scaled
 * relative-position bias in accumulator-fragment order [heads][np/32][np/64][2][64][16]:
 * element [h][qb][t][kb][lane][e] = log2(e) * bias[h][q][k] with q = 32qb + lane%32,
 * k = 64t + 32kb + (e&3) + 8(e>>2) + 4(lane/32); -inf for k >= vol (np = roundup(vol, 64) <= 448).
 * The shift mask (tokens of different shift regions, torchvision's -100) is applied as -inf.
 * out: bf16 rows (head h at h*32), every token written once.  T, H, W must be whole windows.
 * Replaces shifted_window_attention_3d (torchvision.models.video.swin_transformer) between its
 * qkv and proj Linears.
 */
int vc_window_attention3d(const uint16_t* qkv, int64_t ld, int64_t B, int64_t T, int64_t H, int64_t W, int64_t heads,
                          int64_t head_dim, int wt, int wh, int ww, int st, int sh, int sw, const float* biasF,
                          int64_t np, uint16_t* out, int64_t ldo, hipStream_t stream);

/*
 * vc_window_attention3d with the bias and the shift mask on the matrix pipe (the inference path):
 * biasB: fp16, the log2(e)-scaled bias as MFMA B-operand fragments [heads][np/32][np/64][2][2][64][8]:
 * element [h][qb][t][kb][s][lane][m] = log2(e) * bias[h][q][k] with q = 32qb + lane%32,
 * k = 64t + 32kb + 16s + 8(lane/32) + m; -16384 for k >= vol, 0 for q >= vol (swin3d.expand_bias_mb).
 * The kernel adds it as S^T += I . Bias^T (identity A fragments) and the mask as a one-hot product
 * (-16384 between shift regions; exp2 -> 0 as the f32 kernel's -inf).  Same arguments otherwise.
 */
int vc_window_attention3d_mb(const uint16_t* qkv, int64_t ld, int64_t B, int64_t T, int64_t H, int64_t W,
                             int64_t heads, int64_t head_dim, int wt, int wh, int ww, int st, int sh, int sw,
                             const uint16_t* biasB, int64_t np, uint16_t* out, int64_t ldo, hipStream_t stream);

/* Train-step forward: vc_window_attention3d plus lse[row * heads + head] = base-2 log-sum-exp of
 * each query's scores (row = its global token row), kept for the backward. */
int vc_window_attention3d_lse(const uint16_t* qkv, int64_t ld, int64_t B, int64_t T, int64_t H, int64_t W,
                              int64_t heads, int64_t head_dim, int wt, int wh, int ww, int st, int sh, int sw,
                              const float* biasF, int64_t np, uint16_t* out, int64_t ldo, float* lse,
                              hipStream_t stream);

/*
 * Backward of vc_window_attention3d (the Swin3D train step; autograd of torchvision
 * shifted_window_attention_3d as videoswintransformer/.../trainers/trainer.py:105-122 runs it):
 * dqkv rows (d q', dk, dv, bf16; every row of the token grid written once) from q|k|v, the
 * forward output `out`, its gradient `dout` and lse; full_t/h/w = the model's window_size, on
 * which the relative-position index is defined; table = the f32 bias table [(2ft-1)(2fh-1)(2fw-1)]
 * [heads] (torchvision layout, natural units).  dtable_part = f32 [B * nwindows][heads][ntab]:
 * each (window, head)'s bias-table gradient, to be summed over windows by the caller (vc_colsum).
 */
int vc_window_attention3d_bwd(const uint16_t* qkv, int64_t ld, const uint16_t* out, int64_t ldo,
                              const uint16_t* dout, int64_t lddo, const float* lse, int64_t B, int64_t T,
                              int64_t H, int64_t W, int64_t heads, int64_t head_dim, int wt, int wh, int ww,
                              int st, int sh, int sw, int full_t, int full_h, int full_w, const float* table,
                              uint16_t* dqkv, int64_t lddq, float* dtable_part, hipStream_t stream);

/*
 * PatchMerging gather + LayerNorm(4C): y[(b,t,i,j)] = LN(cat(x[2i,2j], x[2i+1,2j], x[2i,2j+1],
 * x[2i+1,2j+1])) in bf16 (zero rows past an odd edge); the Linear(4C, 2C) follows as a GEMM.
 * Replaces torchvision PatchMerging's _patch_merging_pad + norm.  4C <= 4096.
 */
int vc_patch_merge_layernorm(const float* x, int64_t ldx, int64_t B, int64_t T, int64_t H, int64_t W, int64_t C,
                             const float* gamma, const float* beta, float eps, uint16_t* y, int64_t ldy,
                             hipStream_t stream);

/*
 * logits[b] = Wc . mean_n LN(x[b*ntok + n]) + bc (fp32): final norm, AdaptiveAvgPool3d(1) and
 * head of torchvision SwinTransformer3d.forward (head replaced by the reference, swin3d.py:43-44).
 * work: caller scratch f32 [B * 64 * D] (fixed-order partial sums: deterministic).  D <= 1024.
 */
int vc_pool_head(const float* x, int64_t ldx, int64_t B, int64_t ntok, int64_t D, const float* gamma,
                 const float* beta, float eps, const float* Wc, const float* bc, int64_t num_labels, float* logits,
                 float* work, hipStream_t stream);

/* vc_pool_head that also stores the pooled features pooled[B][D] (train step: the head's input). */
int vc_pool_head_pooled(const float* x, int64_t ldx, int64_t B, int64_t ntok, int64_t D, const float* gamma,
                        const float* beta, float eps, const float* Wc, const float* bc, int64_t num_labels, float* logits,
                        float* work, float* pooled, hipStream_t stream);

/* Backward of vc_pool_head's classifier (fp32): dpooled = scale * dlogits . Wc (scale = 1/ntok folds
 * the mean's backward), dWc = dlogits^T . pooled, dbc = column sums of dlogits.  The LayerNorm
 * backward of the pooled tokens is vc_layernorm_bwd. */
int vc_pool_head_bwd(const float* pooled, const float* dlogits, const float* Wc, int64_t B, int64_t D, int64_t num_labels,
                     float scale, float* dpooled, float* dWc, float* dbc, hipStream_t stream);

/* ---- ViViT train step: trainers/trainer.py:140-146 — forward, CE loss,
 * loss.backward(), AdamW.step() — and its data-parallel gradient all-reduce (§8e) ----------- */

/*
 * vc_attention_fwd + lse[(b*H + h)*S + q] = base-2 log-sum-exp of q's scaled scores (f32), kept
 * for the backward.  Requires the same row padding as vc_attention_fwd.
 */
int vc_attention_fwd_lse(const uint16_t* qkv, int64_t ld, int64_t B, int64_t S, int64_t H, int64_t head_dim,
                         float scale, int q_prescaled, uint16_t* out, int64_t ldo, float* lse, hipStream_t stream);

/*
 * Attention backward (autograd of eager_attention_forward, TF5/models/vivit/modeling_vivit.py:
 * 149-174).  qkv: the forward's q'|k|v rows (q' = q*scale*log2 e, q_prescaled); out: the forward
 * output O; dout: dL/dO (same layout as out); lse from vc_attention_fwd_lse; delta: caller
 * scratch f32 [B*H*S].  Writes dqkv (layout of qkv): the q part is dL/dq' (the gradient of the
 * STORED q'), then dL/dk, dL/dv; rows of a clip past S are not written.  dout rows must be
 * readable to (B-1)*S + roundup(S,64) - 1, as qkv.  Deterministic (no atomics).
 */
int vc_attention_bwd(const uint16_t* qkv, int64_t ld, const uint16_t* out, int64_t ldo, const uint16_t* dout,
                     int64_t lddo, const float* lse, float* delta, int64_t B, int64_t S, int64_t H, int64_t head_dim,
                     uint16_t* dqkv, int64_t lddq, hipStream_t stream);
/* The same with the dQ kernel on a second stream beside dK/dV (disjoint outputs, same inputs);
 * `stream` waits for it before the call returns, so later work on `stream` sees all of dqkv.
 * stream2 NULL or == stream: vc_attention_bwd. */
int vc_attention_bwd_2s(const uint16_t* qkv, int64_t ld, const uint16_t* out, int64_t ldo, const uint16_t* dout,
                        int64_t lddo, const float* lse, float* delta, int64_t B, int64_t S, int64_t H,
                        int64_t head_dim, uint16_t* dqkv, int64_t lddq, hipStream_t stream, hipStream_t stream2);

/*
 * LayerNorm backward fused with the residual-gradient add (nn.LayerNorm layernorm_before /
 * layernorm_after backward, TF5/.../modeling_vivit.py:245-266):
 * dx[m] += LN'(x[m]) . dy[m] (f32, in place), dxb[m] = bf16(dx[m]); dgamma / dbeta = column
 * sums over the M rows (overwritten).  Optional (both or neither): dsum_in / dsum_out = column
 * sums of dx before / after the update — the bias gradients of the Linear layers whose outputs
 * these residual gradients are (fc2 and o_proj around layernorm_after).  D in {256, 512, 768,
 * 1024}; work: f32 scratch of >= (nb + ceil(nb/32)) * 4D elements, nb = min(512, ceil(M/4)).
 */
int vc_layernorm_bwd(const float* dy, int64_t lddy, const float* x, int64_t ldx, int64_t M, int64_t D,
                     const float* gamma, float eps, float* dx, int64_t lddx, uint16_t* dxb, int64_t lddxb,
                     float* dgamma, float* dbeta, float* dsum_in, float* dsum_out, float* work, int64_t work_elems,
                     hipStream_t stream);

/*
 * out[n] = (n < nscaled ? scale : 1) * sum over R rows of in[r][n]; dtype 0 = f32, 1 = bf16
 * (bias gradients of nn.Linear).  work: optional f32 scratch for fixed-order row-split partials
 * (deterministic): S1 = min(2048, ceil(R / 64)) partial rows, then S2 = ceil(S1 / 64); (S1 + S2) * N
 * floats take the full split, less halves S1, none = one pass.
 */
int vc_colsum(const void* in, int dtype, int64_t ld, int64_t R, int64_t N, int64_t nscaled, float scale, float* out,
              float* work, int64_t work_elems, hipStream_t stream);

/*
 * Weight gradient of nn.Linear / the tubelet Conv3d: out[n1][n2] = s(n1) * sum_m G[m][n1] X[m][n2]
 * (G = output gradient, X = layer input, bf16 [M][*] row-major; fp32 out, overwritten),
 * s(n1) = scale for n1 < nscaled (the q-scale fold), else 1.  N1 % 128 == 0, N2 % 128 == 0,
 * M % 64 == 0 (M % 32 when N1 and N2 are multiples of 256: the 256 x 256 kernel).  work: f32 scratch
 * for split-K partials, splits * N1 * N2 floats (>= 2 * N1 * N2 enables splitting); the kernel aims
 * at ~512 (128 x 128 tiles) or ~256 (256 x 256 tiles) workgroups: splits = ceil(512 / tiles)
 * bounded by M / 128 (ceil(256 / tiles) bounded by M / 128 for the 256 x 256 kernel), fewer when
 * work is smaller (ops.wgrad_work sizes it).
 */
int vc_wgrad_bf16(const uint16_t* G, int64_t ldg, const uint16_t* X, int64_t ldx, int64_t M, int64_t N1, int64_t N2,
                  int64_t nscaled, float scale, float* out, int64_t ldo, float* work, int64_t work_elems,
                  hipStream_t stream);

/* The weight-gradient schedule vc_wgrad_bf16 runs for (M, N1, N2) with `work_elems` floats of split-K
 * scratch (host-only query, no launch; instrumentation labels launches with it): bits 0-3 = kernel
 * (0 wgrad_kernel 128 x 128, 1 wgrad_big_kernel, 2 wgrad_pp_kernel), bits 4.. = split count. */
int vc_wgrad_pick(int64_t M, int64_t N1, int64_t N2, int64_t work_elems);

/*
 * Backward of the final LayerNorm on the CLS rows + classifier (TF5/.../modeling_vivit.py:427,556)
 * given dlogits f32 [B][num_labels]: writes dx / dxb of the B CLS rows (row b*S; other rows are
 * not touched), dWc [num_labels][D], dbc, dgamma, dbeta (all overwritten).  D <= 1024.
 */
int vc_cls_head_bwd(const float* x, int64_t ldx, int64_t B, int64_t S, int64_t D, const float* gamma, const float* beta,
                    float eps, const float* Wc, int64_t num_labels, const float* dlogits, float* dx, int64_t lddx,
                    uint16_t* dxb, int64_t lddxb, float* dWc, float* dbc, float* dgamma, float* dbeta,
                    hipStream_t stream);

/*
 * Embedding backward (VivitEmbeddings, TF5/.../modeling_vivit.py:126-146): dpos[s] = sum_b dx[b*S+s],
 * dcls = dpos[0], demb[b*(S-1) + p] = bf16(dx[b*S + 1 + p]) (input of the tubelet weight gradient).
 */
int vc_embed_bwd(const float* dx, int64_t lddx, int64_t B, int64_t S, int64_t D, float* dpos, float* dcls,
                 uint16_t* demb, int64_t ldde, hipStream_t stream);

/* ---- TimeSformer train step (timesformer/.../trainers/trainer.py:139-174) ---- */

/*
 * Temporal self-attention backward (TimesformerSelfAttention over the T frames of a patch,
 * TF5/models/timesformer/modeling_timesformer.py:148-180, 332-349), on the clip layout of
 * vc_temporal_attention: rows b*(1 + P*T) + 1 + p*T + t of qkv (q' = q * scale * log2 e | k | v,
 * head h at column h*64 of each third), dout (dL/dO) and dqkv (written: dL/dq' | dL/dk | dL/dv;
 * CLS rows untouched).  T <= 32.  Deterministic.
 */
int vc_temporal_attention_bwd(const uint16_t* qkv, int64_t ld, const uint16_t* dout, int64_t lddo, int64_t B, int64_t P,
                              int64_t T, int64_t H, int64_t head_dim, uint16_t* dqkv, int64_t lddq, hipStream_t stream);

/* Exact GELU x * Phi(x) on bf16 rows [M][N] (N % 8 == 0): TimeSformer / Swin hidden_act "gelu". */
int vc_gelu_erf(const uint16_t* x, int64_t ldx, int64_t M, int64_t N, uint16_t* y, int64_t ldy, hipStream_t stream);

/* Its backward: dx = dy * (Phi(x) + x phi(x)), x = the bf16 pre-activation, dy f32 (dy_bf16 = 0) or
 * bf16 (dy_bf16 = 1), dx bf16. */
int vc_gelu_erf_bwd(const void* dy, int dy_bf16, int64_t lddy, const uint16_t* x, int64_t ldx, int64_t M, int64_t N,
                    uint16_t* dx, int64_t lddx, hipStream_t stream);

/*
 * torch.optim.AdamW step (decoupled weight decay, bias-corrected) over flat f32 buffers, with the
 * gradient multiplied by grad_scale first (1/world_size after a SUM all-reduce).  step >= 1.
 * Replaces optimizer.step() of trainer.py:146 (AdamW, vivit_transformer/main.py:150-155).
 */
int vc_adamw(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n, float lr, float beta1,
             float beta2, float eps, float weight_decay, int64_t step, float grad_scale, hipStream_t stream);

/* vc_adamw with the step on the device, for a train step captured into a hipGraph and replayed: the step is
 * *counter + 1 (counter = device int64, steps done), its constants (lr / (1 - beta1^t), sqrt(1 - beta2^t))
 * are row t - 1 of `tab` (device f32 [tab_len][2], filled by vc_adamw_step_table with vc_adamw's own
 * double-precision arithmetic, so both paths give the same bits); vc_adamw_step_tick adds 1 to the counter
 * (launched after the update).  vc_adamw_step_table writes the host table for steps 1 .. steps. */
int vc_adamw_step_table(float beta1, float beta2, float lr, int64_t steps, float* out);
int vc_adamw_tab(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n, float lr, float beta1,
                 float beta2, float eps, float weight_decay, const float* tab, const int64_t* counter, int64_t tab_len,
                 float grad_scale, hipStream_t stream);
int vc_adamw_step_tick(int64_t* counter, hipStream_t stream);

/* Multi-tensor vc_adamw in one launch (the per-tensor optimizer path of the autograd families):
 * table = device int64 [ntab][6] = {param, grad, exp_avg, exp_avg_sq (f32 device addresses),
 * numel, chunk0}, chunk0 = prefix sum of ceil(numel / 1024) over the preceding entries, nchunks =
 * the total; every tensor takes the same step (bias corrections) and hyper-parameters. */
int vc_adamw_multi(const int64_t* table, int64_t ntab, int64_t nchunks, float lr, float beta1, float beta2, float eps,
                   float weight_decay, int64_t step, float grad_scale, hipStream_t stream);

/*
 * fp32 master weight [N][K] -> bf16 [N][K] (dst) and/or bf16 [K][N] (dstT, the dgrad operand);
 * rows < nscaled are multiplied by scale first (q projection * softmax scale * log2 e).
 * N, K % 4 == 0; src 16-byte, dst / dstT 8-byte aligned.
 */
int vc_pack_weight(const float* src, int64_t N, int64_t K, int64_t nscaled, float scale, uint16_t* dst, uint16_t* dstT,
                   hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* VCLIP_H_ */
