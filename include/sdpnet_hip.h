/*
 * sdpnet_hip.h — C ABI of libsdpnet_hip.so, the MI355X (gfx950) kernels of the
 * SdP-Net forward hot path (y-akbal/SdP-Net @ 2025-06-14).
 *
 * The reference is pure Python on stock ATen ops; it has no FFI of its own.
 * Each entry point below replaces the ATen call(s) a reference forward makes at
 * the cited file:line; the Python host side (sdp-net_amd/sdpnet_hip.py, bound with
 * ctypes) mirrors the reference's nn.Module surface on top of these.
 *
 * Conventions (all entry points):
 *   - dtype codes: 0 = fp32, 1 = bf16 (uint16 bit pattern).  Arithmetic is fp32.
 *   - Every buffer is caller-owned device memory; kernels never allocate.
 *   - `stream` is a hipStream_t; launches are asynchronous on it, no host sync.
 *     Everything is graph-capturable.
 *   - Return value: 0 on success, else a hipError_t code (1 = invalid argument).
 *   - Row maps.  Row-addressed operands take (grp, gstride, off): logical row m
 *     lives at physical row (m / grp) * gstride + off + (m % grp), times the row
 *     stride `ld` (in elements).  grp <= 0 means "dense" (physical = logical).
 *     This addresses the image rows of the persistent [B, R+P, C] token buffer
 *     (grp = P, gstride = R+P, off = R) without gather/scatter copies.
 *   - Activation codes: 0 none, 1 gelu, 2 relu, 3 tanh, 4 sigmoid,
 *     5 leaky_relu (0.01), 6 selu, 7 kelu (model.py:13-24,
 *     training_utilities.py:91-92).  GELU is the erf form x * Phi(x) everywhere except
 *     the bf16 fast-GEMM epilogue (Phi through erfc by Abramowitz & Stegun 7.1.26: |diff|
 *     <= 4.2e-7 against double-precision erf, below the 4.5e-7 of the fp32 formula with
 *     erff), which uses the tanh form which uses the tanh form
 *     x * sigmoid(sqrt(2/pi) (x + 0.044715 x^3)) (|diff| <= 4.7e-4, about one bf16
 *     rounding of the output; a DECLARED deviation from nn.GELU(), model.py:15) unless
 *     sdp_gemm_set_exact_gelu(1) is set.
 */
#ifndef SDPNET_HIP_H
#define SDPNET_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Version string of the library build. */
const char* sdp_version(void);

/*
 * Y[m, n] = epi( sum_k X[m, k] * W[n, k] ),  W stored [N][K] (torch Linear /
 * 1x1-conv layout).  epi: v = acc + bias[n]; if (resid_pre) v += R[m, n];
 * v = act(v); if (!resid_pre) v += R[m, n].  bias fp32 or NULL, R or NULL.
 * Replaces: nn.Conv2d 1x1 of ConvMixer (layers.py:79-91), q/k/v/o_proj and
 * ff_linear1/2 (layers.py:242-249, :282-284, :301, :308), the patch conv as a
 * GEMM on im2col rows (layers.py:34-42) with the positional add of
 * EmbeddingLayer fused (layers.py:162-163), the head Linears (layers.py:445-459).
 * bf16 with K % 64 == 0 runs the 256x256x64 MFMA kernel; everything else the
 * masked generic kernel (fp32 uses exact v_mfma_f32_16x16x4_f32).
 */
int sdp_gemm(int dtype, const void* X, int64_t ldx, int x_grp, int64_t x_gstride, int x_off,
             const void* W, int64_t ldw, const float* bias, const void* R, int64_t ldr,
             int r_grp, int64_t r_gstride, int r_off, void* Y, int64_t ldy, int y_grp,
             int64_t y_gstride, int y_off, int M, int N, int K, int act, int resid_pre,
             void* stream);
/*
 * sdp_gemm with a LayerNorm folded in and/or the output rows' LayerNorm
 * statistics emitted (replaces nn.LayerNorm / channel LayerNorm + the following
 * Linear / 1x1 conv: layers.py:12-24 -> :83-88, :280 -> :282-284, :307 -> :308).
 *   ln_stats (float2 per logical row of X: mean, rstd) and ln_colsum ([N], 16-B
 *   aligned) together, or both NULL: W holds W_orig * gamma (per input column),
 *   bias holds beta . W_orig^T (+ the Linear bias), ln_colsum[n] = sum_k W[n][k];
 *   the epilogue computes rstd * acc - rstd * mean * ln_colsum[n] + bias[n]
 *   before activation / residual.
 *   part != NULL: part[(phys_out_row * ceil(N/64) + c) * 2 + {0,1}] = {mean, M2}
 *   of the stored output row's columns [64c, 64c+64) (combine with sdp_ln_stats).
 */
/* Training GEMM epilogues on the fast kernel (bf16, dense rows; training_tools.py:77-103 with
 * layers.py:83-91 / :306-309): mode 1: Y = X W^T + bias and Y2 = dropout_p(act(Y)) (the
 * ConvMixer up-projection / FFN first layer with sdp_act_fwd fused); mode 2: Y = dropout_p(X W^T)
 * * act'(Z) (the input gradient of the next layer with sdp_act_bwd fused; no bias).  Masks as
 * sdp_act_fwd / sdp_act_bwd (index m * N + n, same seed).  Returns hipErrorNotSupported
 * without launching when the fast kernel does not take the shape or alignment. */
int sdp_gemm_train_epi(int mode, const void* X, int64_t ldx, const void* W, int64_t ldw, const float* bias,
                       const void* Z, int64_t ldz, void* Y, int64_t ldy, void* Y2, int64_t ldy2, int M, int N, int K,
                       int act, float p, uint64_t seed, void* stream);
int sdp_gemm_ln(int dtype, const void* X, int64_t ldx, int x_grp, int64_t x_gstride, int x_off,
                const void* W, int64_t ldw, const float* bias, const void* R, int64_t ldr,
                int r_grp, int64_t r_gstride, int r_off, void* Y, int64_t ldy, int y_grp,
                int64_t y_gstride, int y_off, int M, int N, int K, int act, int resid_pre,
                const float* ln_stats, const float* ln_colsum, float* part, void* stream);
/* Which kernel sdp_gemm picks for a shape: 1 = 256x256 MFMA, 0 = generic. */
int sdp_gemm_variant(int dtype, int M, int N, int K);
/* Test hook: force the generic kernel (returns the previous setting). */
int sdp_gemm_force_generic(int on);
/* Select the bf16 fast kernel: 14 = 8-phase ping-pong 256x256x64 with the
 * whole-line (LDS-staged) epilogue, all row groups staged before the first store
 * (default); 9 = same main loop, permlane-paired 16-B register epilogue (also the
 * automatic fallback for unaligned rows and resid_pre with an activation).  0 queries;
 * any other value returns -1 and leaves the selection unchanged.  Returns the previous selection. */
int sdp_gemm_set_fast_kernel(int k);

/* Output store policy of the whole-line GEMM epilogue: 1 = non-temporal (streaming)
 * stores, 0 = default.  Returns the previous value.  The product library offers only 0 (a
 * request for 1 returns -1); the diagnostic build (make stamps) keeps the A/B arm. */
int sdp_gemm_set_store_policy(int nt);

/* Epilogue specialisation of the whole-line fast-GEMM epilogue: 1 (default) = the model's
 * flag combinations (plain; bias; LN fold + bias; residual + LN partials [+ bias]) with no / GELU
 * activation run an instantiation with the flags fixed at compile time (packed residual add,
 * dot2 partial sums); 0 = the run-time-flag epilogue for every call.  Outputs are
 * bit-identical; the emitted LN partials agree to fp32 rounding.  Returns the previous value.
 * The product library offers only 1 (a request for 0 returns -1; diagnostic build: both). */
int sdp_gemm_set_epi_spec(int on);

/* Phases per K-tile of the fast GEMM's data-parallel main loop: 2 (default, 32 MFMAs per
 * wave-group section, half the group-to-group hand-overs) or 4 (16 MFMAs per section; diagnostic
 * build only).  Same arithmetic order, bit-identical outputs.  Also selects the weight-gradient
 * kernel's loop (sdp_gemm_wgrad).  Returns the previous value; 0 queries it; a value the loaded
 * library does not offer returns -1. */
int sdp_gemm_set_kloop_phases(int n);

/* Launch timeline of the bf16 fast GEMM (measurement only; bench.py's roofline inside a replayed
 * HIP graph, where events cannot be recorded).  sdp_gemm_set_timeline(buf, slots): while buf
 * (device memory, 2 x u64 per slot, caller-initialised to {UINT64_MAX, 0}) is set, fast-GEMM
 * launch i (host launch order) atomically folds its first workgroup's start and its last
 * workgroup's end (after that workgroup's stores drained) into slot i, in s_memrealtime ticks
 * (100 MHz); launches beyond `slots` are not timed.  buf = NULL stops; returns the number of
 * slots the previous timeline took.  sdp_gemm_timeline_count() = slots taken so far.  Replaces
 * nothing in the reference. */
int sdp_gemm_set_timeline(void* buf, int slots);

/* Cross-tile bf16 GEMM kernel (gemm_bf16_ct): `tiles` 256 x 256 pair tiles per workgroup (0 = off,
 * -1 = one row of pair tiles), `re` row groups per epilogue step (1 or 2), taken by the
 * specialised-epilogue calls with K <= kmax and N <= nmax.  The two 4-wave groups of a workgroup own
 * different 128 x 256 tiles and run an epilogue's length apart, so one group's epilogue runs under
 * the other's MFMAs.  Bit-identical to the 8-phase kernel.  Returns the previous tile count, -2 for
 * invalid arguments. */
int sdp_gemm_set_ct(int tiles, int re, int kmax, int nmax);
int sdp_gemm_timeline_count(void);

/* Timing experiments only, diagnostic library (`make stamps`, -DSDP_DIAG): bit 0 makes sdp_dwconv,
 * bit 1 sdp_attention, bit 2 sdp_ln_stats return without launching (results WRONG) -- bounds what a
 * faster kernel could give the step.  Returns the previous mask.  The product library has no skip
 * paths: the mask stays 0 and a non-zero request returns -1.  Replaces nothing in the reference. */
int sdp_debug_skip(int mask);

/* Build flags of the loaded library: bit 0 = kernel skipping compiled in (SDP_DIAG), bit 1 = GEMM
 * wall-clock stamps compiled in (SDP_GEMM_STAMPS); 0 = the product library (the only one bench.py
 * times).  Replaces nothing in the reference. */
int sdp_build_info(void);

/* Tile raster of the 8-phase GEMM: M-blocks per group (consecutive blocks walk a group of
 * gm M-blocks before the next N-tile).  1 = row-major, -1 = auto (since round 6: 2 below 9 N-tiles, else 4).
 * Results do not depend on it.  Returns the previous value. */
int sdp_gemm_set_group_m(int gm);

/* GELU form of the bf16 fast-GEMM epilogue: 0 = tanh form (default, one v_exp + one
 * v_rcp per element), 1 = erf form (nn.GELU(), model.py:15; runtime-activation epilogue).
 * Used to bound the tanh form's share of the bf16 logits error.  Returns the previous value. */
int sdp_gemm_set_exact_gelu(int on);

/*
 * LayerNorm statistics by parts: sdp_row_partials writes {mean, M2} of every
 * 64-column chunk of the logical rows of X to part[(phys_row * ceil(C/64) + c) * 2];
 * sdp_ln_stats combines a row's chunks exactly (pairwise mean / M2 update) into
 * stats[m] = (mean, 1 / sqrt(M2 / C + eps)) for logical row m of the given map.
 */
int sdp_row_partials(int dtype, const void* X, int64_t ldx, int x_grp, int64_t x_gstride, int x_off,
                     int M, int C, float* part, void* stream);
int sdp_ln_stats(const float* part, int x_grp, int64_t x_gstride, int x_off, int M, int C, float eps,
                 float* stats, void* stream);

/*
 * Row LayerNorm over C contiguous channels, fp32 statistics, biased variance.
 * Replaces: channel LayerNorm of ConvMixer (layers.py:12-24, eps 1e-6) on the
 * token layout; nn.LayerNorm norm1/norm2 (layers.py:252-253, eps 1e-5); the
 * head LayerNorm (layers.py:445, :449).
 */
int sdp_layernorm(int dtype, const void* X, int64_t ldx, int x_grp, int64_t x_gstride, int x_off,
                  const float* gamma, const float* beta, float eps, void* Y, int64_t ldy,
                  int y_grp, int64_t y_gstride, int y_off, int M, int C, void* stream);

/*
 * In-place LayerNorm over each head_dim segment of the q and k thirds of the
 * fused QKV rows [rows, ld >= 3C]: q_norm / k_norm (layers.py:236-237, :286).
 */
int sdp_qk_headnorm(int dtype, void* QKV, int64_t ld, int64_t rows, int n_head, int head_dim,
                    const float* q_gamma, const float* q_beta, const float* k_gamma,
                    const float* k_beta, float eps, void* stream);

/*
 * Per-row LayerNorm statistics: stats[2m] = mean, stats[2m+1] = 1/sqrt(var+eps)
 * (biased variance) of logical row m; C % 4 == 0, C <= 2048.  Feeds the LN that
 * sdp_dwconv applies on load (ConvMixer layer_norm_1, layers.py:12-24, :102).
 */
int sdp_rowstats(int dtype, const void* X, int64_t ldx, int x_grp, int64_t x_gstride, int x_off,
                 float eps, float* stats, int M, int C, void* stream);

/*
 * Depthwise k x k conv, zero "same" padding, NHWC token rows (pixel (b,h,w) is
 * logical row b*H*W + h*W + w).  weight fp32 [C][k][k], bias fp32 [C] or NULL.
 * If stats != NULL the conv input is the LayerNorm (x - mean) * rstd * ln_gamma +
 * ln_beta computed while staging (fused layer_norm_1 of ConvMixer).
 * Replaces: layer_norm_1 + nn.Conv2d(C, C, k, groups=C, padding="same")
 * (layers.py:73-78, :102).  k in {1,3,5,7,9}.
 */
int sdp_dwconv(int dtype, const void* X, int64_t ldx, int x_grp, int64_t x_gstride, int x_off,
               const float* stats, const float* ln_gamma, const float* ln_beta,
               const float* weight, const float* bias, void* Y, int64_t ldy, int y_grp,
               int64_t y_gstride, int y_off, int B, int H, int W, int C, int k, void* stream);
/* Select the depthwise kernel: 3 (default) = MFMA Toeplitz form
 * (bf16, C % 32 == 0, H, W <= 16, k in {3,5,7}), 2 = 64-channel x band blocks with an fp32 LDS tile
 * (C % 8 == 0, k in {3,5,7}, 16-B aligned rows), 1 = 32-channel blocks with a
 * bf16 tile (any shape); each falls back to the next where it does not apply.  0 queries; any other
 * value returns -1 and leaves the selection unchanged.  Returns the previous selection. */
int sdp_dwconv_set_kernel(int k);

/*
 * softmax(LN_q(Q) LN_k(K)^T / sqrt(hd) + mask) V per (batch, head) from fused QKV
 * rows [B*N, ld_qkv] (q | k | v thirds), output rows [B*N, ld_o] (heads
 * concatenated).  q/k LayerNorm (q_norm / k_norm, shared across heads, eps) is
 * applied when q_gamma != NULL (then all four must be given); the generic path
 * applies it in place on the QKV rows.  mask: optional fp32 additive [.., N, N]
 * with batch / head strides (0 = broadcast).  Replaces q_norm/k_norm and
 * F.scaled_dot_product_attention (layers.py:286-291) and the manual softmax path
 * (layers.py:292-298).
 */
int sdp_attention(int dtype, const void* QKV, int64_t ld_qkv, void* O, int64_t ld_o, int B, int N,
                  int n_head, int head_dim, const float* q_gamma, const float* q_beta,
                  const float* k_gamma, const float* k_beta, float eps, const float* mask,
                  int64_t mask_sb, int64_t mask_sh, void* stream);
/* Kernel sdp_attention takes for this shape: 6 = attn_fa5, one double-buffered 8-wave workgroup per
 * CU (diagnostic build only, opt-in, hd % 32 == 0, N <= 224), 4 = two persistent 4-wave flash workgroups per CU, one LDS-DMA
 * K/V buffer each (hd % 32 == 0, N <= 256), 3 = whole-head flash kernels (hd % 32 == 0, head within
 * 160 KiB of LDS; at 9 key tiles the persistent attn_fa6 with three rotating K / V images where they
 * fit, else attn_fa2), 5 = streaming flash kernel (hd % 32 == 0, any N),
 * 2 = one-workgroup flash kernel, 0 = generic. */
int sdp_attention_variant(int dtype, int N, int n_head, int head_dim, int has_mask);
/* Select the bf16 flash kernel tier: 4 (default) = attn_fa4, 3 = attn_fa2 (both falling back to the
 * streaming attn_fs for heads that do not fit LDS), 5 = force attn_fs (each where it applies, else the
 * next lower one; attn_fa stays the path for hd % 32 != 0).  Diagnostic build only: 6 = allow attn_fa5,
 * 2 = attn_fa only.  0 queries; an unavailable value returns -1 and leaves the selection unchanged.
 * Returns the previous selection. */
int sdp_attention_set_kernel(int k);
/* Workgroups per CU of the persistent fa4 kernel (0 = as many as LDS and registers allow, at
 * most 4); returns the previous setting. */
int sdp_attn_set_per_cu(int n);

/*
 * im2col of the patch conv: image [B,3,Hi,Wi] -> rows [B*(Hi/p)*(Wi/p), Kpad],
 * column c*p*p + i*p + j, zero padded to Kpad.  (ConvPatcher, layers.py:34-42.)
 */
int sdp_patchify(int dtype_in, const void* img, int dtype_out, void* out, int B, int Hi, int Wi,
                 int p, int Kpad, void* stream);

/* Adjoint of sdp_patchify (the ConvPatcher input gradient, layers.py:34-42 in training):
 * image [B,3,Hi,Wi] <- rows [B*(Hi/p)*(Wi/p), Kpad]; pixels no patch covers get 0. */
int sdp_unpatchify(int dtype_in, const void* rows, int dtype_out, void* img, int B, int Hi, int Wi,
                   int p, int Kpad, void* stream);

/* T[h*W + w][c] = Eh[h][c] + Ew[w][c]   (EmbeddingLayer, layers.py:157-163). */
int sdp_pos_table(const float* eh, const float* ew, float* out, int H, int W, int C, void* stream);

/* T[h*W + w][c] = mean_{k x k} bone[c][h+i][w+j]  (ConvEmbedding, layers.py:205). */
int sdp_avgpool_table(const float* bone, int BH, int BW, float* out, int H, int W, int C, int k,
                      void* stream);
/* Its adjoint (trainable bone in train mode, layers.py:189-190): dbone [C, BH, BW] fp32 from
 * dtable [H*W, C] fp32. */
int sdp_avgpool_table_bwd(const float* dtable, int H, int W, int C, int k, float* dbone, int BH, int BW,
                          void* stream);

/* dst[b*gstride + r*ldd + c] = src[b*sgstride + r*lds + c]; sgstride = 0 expands
 * the register table over the batch (layers.py:166, :208), otherwise it copies
 * the register rows in/out of the token buffer (layers.py:275, :311). */
int sdp_copy_rows(int dtype_src, const void* src, int64_t lds, int64_t sgstride, int dtype_dst,
                  void* dst, int64_t ldd, int64_t gstride, int B, int R, int C, void* stream);

/* In place x[b][c][hw] += table[hw][c] on NCHW (standalone EmbeddingLayer.forward,
 * layers.py:162-163), and y = act(x) elementwise (its activation, :168). */
int sdp_nchw_add_table(int dtype, void* X, const float* table, int B, int C, int HW, void* stream);
int sdp_act(int dtype, const void* X, void* Y, int64_t n, int act, void* stream);

/* out[g][c] = mean over `rows` consecutive logical rows of X: registers.mean(-2)
 * (layers.py:464) and AdaptiveAvgPool2d((1,1)) + Flatten (layers.py:457-458). */
int sdp_group_mean(int dtype_in, const void* X, int64_t ldx, int x_grp, int64_t x_gstride, int x_off,
                   int dtype_out, void* out, int64_t ldo, int G, int rows, int C, void* stream);

/* NCHW [B,C,HW] <-> token rows (layers.py:271, :314). */
int sdp_nchw_to_rows(int dtype_in, const void* X, int dtype_out, void* Y, int64_t ldy, int y_grp,
                     int64_t y_gstride, int y_off, int B, int C, int HW, void* stream);
int sdp_rows_to_nchw(int dtype_in, const void* X, int64_t ldx, int x_grp, int64_t x_gstride,
                     int x_off, int dtype_out, void* Y, int B, int C, int HW, void* stream);

/* Element cast fp32 <-> bf16 (weight cache preparation, output conversion). */
int sdp_cast(int dtype_in, const void* X, int dtype_out, void* Y, int64_t n, void* stream);
/* LayerNorm folding of the Linear that consumes LN(x) (weight preparation for
 * sdp_gemm_ln): Wf[n][k] = W[n][k] * gamma[k] (dtype_out), colsum[n] = sum_k Wf[n][k],
 * cvec[n] = sum_k beta[k] * W[n][k] + bias[n] (bias may be NULL).  W, gamma, beta,
 * bias fp32; W [N][K] row-major. */
int sdp_fold_ln_weight(const float* W, const float* gamma, const float* beta, const float* bias, int N,
                       int K, int dtype_out, void* Wf, float* colsum, float* cvec, void* stream);

/* ---- Evaluation: either side of the forward path ---- */

/* Validation transform of hf_dataset_generator.py:27-41 (val_transforms, used by
 * model_test.py:50-52): RGB -> Resize((RH, RW), BICUBIC) -> CenterCrop((CH, CW)) ->
 * ToDtype(float32, scale=True) -> Normalize(mean3, std3), on B decoded uint8 RGB HWC
 * images of any sizes, bit-exact to Pillow 12.2.0's 8-bit resampler (the PIL path the
 * reference's torchvision transforms take) up to the uint8 crop.
 *   pix, offs[B] (int64 byte offsets), hw[B][2] (H, W): device; image b is
 *   pix[offs[b] .. + H*W*3).  top/left: the crop origin inside the RH x RW resize
 *   (torchvision: round((RH - CH) / 2), round((RW - CW) / 2)).
 *   KMAX: the largest tap count over the batch, ceil(2 * max(1, In / Out)) * 2 + 1 over
 *   both axes of every image (<= 160).  ws: B * (CW + CH) * (2 + KMAX) int32 of
 *   device workspace; tmp: B * tmp_stride bytes, tmp_stride >= max_H * CW * 4 (the
 *   horizontal pass's RGBX words).  max_w: the widest image of the batch (<= 40960; its
 *   RGBX row is staged in LDS).
 *   out: [B][3][CH][CW] fp32 (dtype_out 0) or bf16 (1); out_u8 (optional, may be NULL):
 *   the cropped uint8 HWC image [B][CH][CW][3].  mean3 / std3: host arrays. */
int sdp_val_preprocess(const uint8_t* pix, const int64_t* offs, const int* hw, int B, int RH, int RW,
                       int top, int left, int CH, int CW, int KMAX, const float* mean3, const float* std3,
                       void* ws, uint8_t* tmp, int64_t tmp_stride, int max_w, int dtype_out,
                       void* out, uint8_t* out_u8, void* stream);

/* Per-row evaluation metrics of run_test (model_test.py:69-82): for logits X [B][C]
 * (row stride ld, fp32 or bf16) and int64 labels [B]:
 *   out[3b] = logsumexp(X[b]) - X[b][label]     (nn.CrossEntropyLoss before the mean)
 *   out[3b+1] = sum_j BCE-with-logits(X[b][j], onehot * (1 - ls) + ls / C)
 *               (training_utilities.py:95-107 before the mean over B*C)
 *   out[3b+2] = 1 if the first maximal index equals the label (outputs.argmax(1) == labels)
 * A label outside [0, C) gives NaN. */
int sdp_logits_metrics(int dtype, const void* X, int64_t ld, const int64_t* labels, int B, int C,
                       float label_smoothing, float* out, void* stream);

/* ======================================================================================
 * Training step (BASELINE.json configs[4]).  Replaces the autograd
 * backward of the modules above under training_tools.py:85-99 (bf16 autocast forward,
 * scaler.scale(loss).backward(), unscale_ + clip_grad_norm_(5), AdamW step), the train-mode
 * StochasticDepth (utility_layers.py:16-27) and the dropouts (layers.py:291, :301-308).
 * ====================================================================================== */

/* Batched GEMM with either operand transposed (no transposed copies in HBM):
 *   C[z](i, j) = alpha * sum_k A[z](i, k) B[z](k, j)  (+ C[z](i, j) if accum)
 *   A(i, k) = ta ? A[k * lda + i] : A[i * lda + k];  B(k, j) = tb ? B[j * ldb + k] : B[k * ldb + j]
 *   batch z < Z: operand offset (z / zdiv) * s1 + (z % zdiv) * s2 elements.
 *   splits > 1: K is split into `splits` ranges (multiples of 32), range s writes its fp32
 *   partial to C + s * split_stride (reduce with sdp_seg_colsum); accum must be 0 then.
 * dtype 1 (bf16 operands, fp32 accumulate; out_dtype 0 fp32 / 1 bf16; 16-B vector loads where
 * leading dims, batch strides and bases are 8-element aligned, element loads otherwise) or
 * 0 (fp32, exact f32 MFMA).
 * Used for dW = dY^T X of every Linear / 1x1 conv (layers.py:79-91, :242-249, :308), the
 * patch-conv weight gradient (layers.py:34-42), dX = dY W, and the attention products of
 * the train-mode forward and backward (layers.py:289-298). */
int sdp_gemm_flex(int dtype, int out_dtype, int ta, int tb, const void* A, int64_t lda, int64_t sa1, int64_t sa2,
                  const void* B, int64_t ldb, int64_t sb1, int64_t sb2, void* C, int64_t ldc, int64_t sc1,
                  int64_t sc2, int M, int N, int K, int Z, int zdiv, int splits, int64_t split_stride, float alpha,
                  int accum, void* stream);

/* Y[c][r] = X[r][c] (X [R][C], row strides ldx / ldy): the weight transposes that let the
 * input-gradient GEMMs dX = dY W run on the 256x256 MFMA kernel. */
int sdp_transpose(int dtype, const void* X, int64_t ldx, void* Y, int64_t ldy, int R, int C, void* stream);

/* out[g * ldo + c] = scale * sum_{e < len} X[(g * gstride + e * estride) * ldx + c] (+ out if
 * accum), fp32 out: bias / LayerNorm-affine / embedding-table gradients and split-K reduction. */
int sdp_seg_colsum(int dtype, const void* X, int64_t ldx, int G, int len, int64_t gstride, int64_t estride, int C,
                   float* out, int64_t ldo, float scale, int accum, void* stream);

/* Y = act(Z) with dropout p (keep iff hash(seed, m * N + n) >= p, kept values / (1 - p));
 * backward DZ = DY * mask / (1 - p) * act'(Z).  Erf-form GELU.  p = 0: no mask.
 * (layers.py:83-88 activation, :308 FFN dropouts, :445-454 head dropout.) */
int sdp_act_fwd(int dtype, const void* Z, int64_t ldz, void* Y, int64_t ldy, int M, int N, int act, float p,
                uint64_t seed, void* stream);
int sdp_act_bwd(int dtype, const void* Z, int64_t ldz, const void* DY, int64_t lddy, void* DZ, int64_t lddz, int M,
                int N, int act, float p, uint64_t seed, void* stream);

/* Y[m] = X[m] * scale[m / sgrp] (+ R[m]) over row maps: per-sample drop path
 * (StochasticDepth, utility_layers.py:16-27) on a residual branch; scale may be NULL. */
int sdp_rowscale_add(int dtype, const void* X, int64_t ldx, int x_grp, int64_t x_gstride, int x_off,
                     const float* scale, int sgrp, const void* R, int64_t ldr, int r_grp, int64_t r_gstride, int r_off,
                     void* Y, int64_t ldy, int y_grp, int64_t y_gstride, int y_off, int M, int N, void* stream);
/* Y[m] = act(X[m]) * scale[m / sgrp] + R[m] (act's output rounded to dtype first, as sdp_act_fwd
 * stores it): the activation + drop path + residual add of a ConvMixer branch
 * (layers.py:83-104, utility_layers.py:16-27) in one pass, without the activation buffer. */
int sdp_act_rowscale_add(int dtype, int act, const void* X, int64_t ldx, int x_grp, int64_t x_gstride, int x_off,
                         const float* scale, int sgrp, const void* R, int64_t ldr, int r_grp, int64_t r_gstride,
                         int r_off, void* Y, int64_t ldy, int y_grp, int64_t y_gstride, int y_off, int M, int N,
                         void* stream);
/* Mixed-dtype form of the two above (act 0 = none): X in x_dtype, R and Y in y_dtype, 16-B
 * aligned rows and N % 8 == 0 when the dtypes differ.  The fp32 residual stream of bf16 training
 * (training_tools.py:85 autocast keeps x + branch in fp32): y32 = act(x16) * s + r32, and the
 * stream gradient cast into a bf16 branch, y16 = x32 * s. */
int sdp_rowscale_add_mixed(int x_dtype, int y_dtype, int act, const void* X, int64_t ldx, int x_grp,
                           int64_t x_gstride, int x_off, const float* scale, int sgrp, const void* R, int64_t ldr,
                           int r_grp, int64_t r_gstride, int r_off, void* Y, int64_t ldy, int y_grp,
                           int64_t y_gstride, int y_off, int M, int N, void* stream);

/* LayerNorm from given statistics (stats[2m] = mean, stats[2m+1] = rstd, from sdp_rowstats):
 * Y = (X - mean) * rstd * gamma + beta; and its backward
 * DX = rstd * (g.DY - mean(g.DY) - xhat * mean(g.DY * xhat)) (+ ADD), per-block partials
 * part[b][0][c] = sum DY * xhat, part[b][1][c] = sum DY for b < sdp_ln_bwd_blocks(M) (C <= 2048).
 * (layers.py:12-24 channel LN, :252-253 / :236-237 nn.LayerNorm, :445 head LN.) */
int sdp_ln_apply(int dtype, const void* X, int64_t ldx, int x_grp, int64_t x_gstride, int x_off,
                 const float* stats, const float* gamma, const float* beta, void* Y, int64_t ldy, int y_grp,
                 int64_t y_gstride, int y_off, int M, int C, void* stream);
int sdp_ln_bwd_blocks(int M);
/* Training-forward LayerNorm in one pass: stats[m] = (mean, rstd) and Y = LN(X) (C % 8 == 0,
 * C <= 2048, 16-B aligned rows). */
int sdp_ln_fwd(int dtype, const void* X, int64_t ldx, int x_grp, int64_t x_gstride, int x_off, float eps,
               const float* gamma, const float* beta, float* stats, void* Y, int64_t ldy, int y_grp,
               int64_t y_gstride, int y_off, int M, int C, void* stream);
int sdp_ln_bwd(int dtype, const void* X, int64_t ldx, int x_grp, int64_t x_gstride, int x_off, const float* stats,
               const float* gamma, const void* DY, int64_t lddy, int dy_grp, int64_t dy_gstride, int dy_off,
               const void* ADD, int64_t ldadd, int a_grp, int64_t a_gstride, int a_off, void* DX, int64_t lddx,
               int dx_grp, int64_t dx_gstride, int dx_off, int M, int C, float* part, void* stream);
/* Mixed-dtype LayerNorm (fp32 residual stream, bf16 GEMM operands; vector path only):
 * sdp_ln_fwd_mixed reads X in x_dtype and writes Y in y_dtype; sdp_ln_bwd_mixed reads X, ADD
 * and writes DX in x_dtype, DY in dy_dtype. */
int sdp_ln_fwd_mixed(int x_dtype, int y_dtype, const void* X, int64_t ldx, int x_grp, int64_t x_gstride, int x_off,
                     float eps, const float* gamma, const float* beta, float* stats, void* Y, int64_t ldy, int y_grp,
                     int64_t y_gstride, int y_off, int M, int C, void* stream);

/* Residual add + LayerNorm forward in one pass (training forward): y = act / dropout(x) * scale[m / sgrp]
 * + r (sdp_rowscale_add_mixed / sdp_rowscale_add_dropout mode 1 arithmetic; x in x_dtype, r and y in
 * y_dtype) and a = LN(y) with its (mean, rstd) statistics (sdp_ln_fwd_mixed; a in a_dtype), bit-identical
 * to the two passes.  reg_src != NULL: the register rows b * reg_n + i (i < reg_r, b < reg_b) of reg_src
 * (y_dtype, row stride ldy) are copied to reg_dst0 (and reg_dst1) by extra workgroups of the same launch
 * (a ConvMixer leaves them unchanged, layers.py:99-104).
 * hipErrorNotSupported where the one-pass form does not apply (C % 8, C <= 128, C > 2048,
 * unaligned rows, dropout mode 2).  Replaces the branch add + LayerNorm pairs of layers.py:99-103
 * (ConvMixer, x + drop_path(act(PW(.))) then layer_norm_2) and :300-306 (EncoderLayer, x +
 * drop_path(dropout(o_proj(.))) then norm2) in the training step. */
int sdp_add_ln_fwd(int x_dtype, int y_dtype, int a_dtype, int act, const void* X, int64_t ldx, int x_grp,
                   int64_t x_gstride, int x_off, const float* scale, int sgrp, const void* R, int64_t ldr, int r_grp,
                   int64_t r_gstride, int r_off, void* Y, int64_t ldy, int y_grp, int64_t y_gstride, int y_off,
                   float p, uint64_t seed, int dmode, float eps, const float* gamma, const float* beta, float* stats,
                   void* A, int64_t lda, int a_grp, int64_t a_gstride, int a_off, int M, int C,
                   const void* reg_src, void* reg_dst0, void* reg_dst1, int reg_b, int reg_r, int reg_n, void* stream);
int sdp_ln_bwd_mixed(int x_dtype, int dy_dtype, const void* X, int64_t ldx, int x_grp, int64_t x_gstride, int x_off,
                     const float* stats, const float* gamma, const void* DY, int64_t lddy, int dy_grp,
                     int64_t dy_gstride, int dy_off, const void* ADD, int64_t ldadd, int a_grp, int64_t a_gstride,
                     int a_off, void* DX, int64_t lddx, int dx_grp, int64_t dx_gstride, int dx_off, int M, int C,
                     float* part, void* stream);
/* sdp_ln_bwd_mixed in one launch (training backward), with
 *  (a) the affine sums finished in the kernel (ticket != NULL): part [sdp_ln_bwd_blocks(M)][2C] and
 *      gpart [ceil(blocks / 32)][2C] are scratch, aff [2C] receives {dgamma, dbeta}; ticket points
 *      at ceil(blocks / 32) + 1 zeroed ints, which the kernel leaves zeroed (one buffer per stream).
 *      Fixed summation order: deterministic, whichever block finishes last.  Opt-in
 *      (SDPNET_LN_TICKET=1): the device-scope fences it needs across the XCDs' L2s made the XL
 *      training step ~20 % slower (profiles/r06_ln_bwd_fused_ab.md);
 *  (b) optionally (O2 != NULL) the gradient of the branch that fed the LayerNorm input, bf16 dense
 *      rows: O2 = bf16(DX * scale[m / sgrp]); dmode 2: dropout on the rounded value (keep iff
 *      hash(seed, m * C + c) >= p, kept / (1 - p)); act != 0: O2 = bf16(O2 * act'(Z)), Z bf16 dense
 *      rows -- bit-identical to sdp_rowscale_add_mixed (+ _dropout mode 2) then sdp_act_bwd on DX.
 * (c) reg_src != NULL: register rows b * reg_n + i (i < reg_r, b < reg_b) of reg_src copied to reg_dst
 *     (x_dtype, row stride lddx) -- the rows a ConvMixer passes through unchanged.
 * hipErrorNotSupported where the one-launch form does not apply (C <= 128, C % 8, unaligned rows,
 * dmode 1): the caller runs sdp_ln_bwd_mixed and the passes.  Replaces, per ConvMixer backward,
 * LN2 backward + drop_path_2 scale + act' (layers.py:99-103) and, per EncoderLayer backward, norm2
 * backward + drop_path1 / dropout of the attention branch (:300-306). */
int sdp_ln_bwd_fused(int x_dtype, int dy_dtype, const void* X, int64_t ldx, int x_grp, int64_t x_gstride, int x_off,
                     const float* stats, const float* gamma, const void* DY, int64_t lddy, int dy_grp,
                     int64_t dy_gstride, int dy_off, const void* ADD, int64_t ldadd, int a_grp, int64_t a_gstride,
                     int a_off, void* DX, int64_t lddx, int dx_grp, int64_t dx_gstride, int dx_off, int M, int C,
                     float* part, float* gpart, float* aff, int* ticket, const float* scale, int sgrp, const void* Z,
                     int64_t ldz, int act, float p, uint64_t seed, int dmode, void* O2, int64_t ldo2,
                     const void* reg_src, void* reg_dst, int reg_b, int reg_r, int reg_n, void* stream);

/* Attention rows (layers.py:289-298, SDPA dropout_p in training): P = softmax(scale * S[:, :N])
 * (S fp32), Pd = P with dropout p (may be NULL), columns [N, Npad) zeroed; backward
 * DS = P * (DPm - sum(DPm * P)), DPm = DPd with the same mask. */
int sdp_softmax_fwd(int dtype, const float* S, int64_t lds, void* P, void* Pd, int64_t ldp, int rows, int N, int Npad,
                    float scale, float p, uint64_t seed, void* stream);
/* The same with an additive fp32 mask before the softmax (the masked attention of EncoderLayer in
 * train mode, layers.py:291 SDPA attn_mask / :294-295 masked_fill(mask == 0, -inf)): row r = z * N + i
 * of S adds mask[(z / mask_zdiv) * mask_sb + (z % mask_zdiv) * mask_sh + i * N + c] (strides 0
 * broadcast over batch / head; -inf gives exact zeros, a fully masked row NaN as torch). */
int sdp_softmax_fwd_mask(int dtype, const float* S, int64_t lds, void* P, void* Pd, int64_t ldp, int rows, int N,
                         int Npad, float scale, float p, uint64_t seed, const float* mask, int64_t mask_sb,
                         int64_t mask_sh, int mask_zdiv, void* stream);
int sdp_softmax_bwd(int dtype, const void* P, int64_t ldp, const void* DPd, int64_t lddp, void* DS, int64_t ldds,
                    int rows, int N, int Npad, float p, uint64_t seed, void* stream);

/* Depthwise-conv weight gradient (layers.py:73-78): part[chunk][c][t] = sum over the chunk's
 * images of DY[b, h, w, c] * A[b, h + ty - k/2, w + tx - k/2, c] (zero padded), NHWC rows,
 * chunk < sdp_dw_wgrad_chunks(B); H * W <= 640 (both planes staged as fp32), any W, odd k <= 9.  The input gradient is
 * sdp_dwconv with the kernel flipped. */
int sdp_dw_wgrad_chunks(int B);
int sdp_dw_wgrad(int dtype, const void* A, int64_t lda, int a_grp, int64_t a_gstride, int a_off, const void* DY,
                 int64_t lddy, int dy_grp, int64_t dy_gstride, int dy_off, int B, int H, int W, int C, int k,
                 float* part, void* stream);

/* Label-smoothed cross entropy, mean over the rows whose label is not ignore_index
 * (nn.CrossEntropyLoss(label_smoothing), training_tools.py:76, :88, with torch's default
 * ignore_index = -100): *loss += mean loss (fp32, atomic); dlogits = grad_scale / n * (softmax -
 * ((1 - eps) onehot + eps / K)) for the n counted rows, 0 for ignored rows (may be NULL); all rows
 * ignored gives a NaN loss (torch: 0 / 0).  sdp_ce_loss_ignore takes any ignore_index. */
int sdp_ce_loss(int dtype, const void* logits, int64_t ldl, const int64_t* labels, int B, int K, float eps,
                float grad_scale, void* dlogits, int64_t ldd, float* loss, void* stream);
int sdp_ce_loss_ignore(int dtype, const void* logits, int64_t ldl, const int64_t* labels, int B, int K, float eps,
                       float grad_scale, int64_t ignore_index, void* dlogits, int64_t ldd, float* loss, void* stream);
/* Row count of a hard-label cross entropy: n[0] = #{i : labels[i] != ignore_index} as float, one
 * pass over the labels (B >= 0).  Feeds sdp_ce_loss_counted.  Replaces the count inside
 * nn.CrossEntropyLoss's 'mean' reduction (training_tools.py:76). */
int sdp_ce_count(const int64_t* labels, int B, int64_t ignore_index, float* n, void* stream);

/* sdp_ce_loss_ignore with the row count taken from nrows (device float, sdp_ce_count on the same
 * stream) instead of every wave counting the labels: O(B) label reads in all, for per-token or
 * per-pixel losses.  Same arithmetic and results. */
int sdp_ce_loss_counted(int dtype, const void* logits, int64_t ldl, const int64_t* labels, int B, int K, float eps,
                        float grad_scale, int64_t ignore_index, const float* nrows, void* dlogits, int64_t ldd,
                        float* loss, void* stream);

/* The same loss on probability targets (fp32 rows [B][ldt], the CutMix / MixUp targets of
 * dataset_generator.py:105-110 fed to nn.CrossEntropyLoss): t' = (1 - eps) t + eps / K,
 * loss = mean_i -sum_k t'_ik log p_ik, dlogits = grad_scale / B * (p sum_k t' - t').  A hard
 * label outside [0, K) other than ignore_index makes its row's loss and gradient NaN instead of
 * reading out of bounds. */
int sdp_ce_loss_soft(int dtype, const void* logits, int64_t ldl, const float* targets, int64_t ldt, int B, int K,
                     float eps, float grad_scale, void* dlogits, int64_t ldd, float* loss, void* stream);

/* Multi-tensor optimizer step over fp32 tensors (device arrays of pointers / sizes and a
 * block table of sdp_mt_block_bytes()-sized {int tensor; int64 start} entries, 4096
 * elements per block):
 *   sdp_grad_sumsq: state[0] += sum g^2, state[1] (int) = 1 on any non-finite g;
 *   sdp_adamw: unless state[1] != 0 (GradScaler skip), g = grad * inv_scale * min(1,
 *     max_norm / (sqrt(state[0]) * inv_scale + 1e-6)) (clip_grad_norm_, max_norm <= 0: off),
 *     then torch.optim.AdamW (decoupled decay, bias corrections of step);
 *   sdp_scaler_update: GradScaler.update on sc[0] = scale, sc[1] = growth tracker, resets state.
 *   sdp_adamw_dev: sdp_adamw with the step counts on the device: steps[t] (fp32) = optimizer
 *     steps tensor t has taken; the bias corrections use steps[t] + 1 (double precision).
 *     scale != NULL: the grads are unscaled by 1 / scale[0] (device GradScaler scale; the loss
 *     is multiplied by the same device value, so a backoff needs no host sync).
 *   sdp_adamw_finish: if the step was taken (state[1] == 0) steps[0..nsteps) += 1; with
 *     scale_tracker != NULL the GradScaler update as sdp_scaler_update; always resets state.
 *     Together: torch.amp.GradScaler + torch.optim.AdamW semantics, where a skipped step
 *     advances neither the parameters, the moments nor the step count.
 * (training_tools.py:91-99, :235.) */
int sdp_mt_block_bytes(void);
int sdp_grad_sumsq(float* const* grads, const int64_t* sizes, const void* blocks, int nblocks, float* state,
                   void* stream);
int sdp_adamw(float* const* params, float* const* grads, float* const* exp_avg, float* const* exp_avg_sq,
              const int64_t* sizes, const void* blocks, int nblocks, const float* state, float lr, float beta1,
              float beta2, float eps, float weight_decay, int step, float inv_scale, float max_norm, void* stream);
int sdp_scaler_update(float* state, float* scale_tracker, float growth, float backoff, int interval, void* stream);
int sdp_adamw_dev(float* const* params, float* const* grads, float* const* exp_avg, float* const* exp_avg_sq,
                  const int64_t* sizes, const void* blocks, int nblocks, const float* state, float lr, float beta1,
                  float beta2, float eps, float weight_decay, const float* steps, const float* scale,
                  float inv_scale, float max_norm, void* stream);
int sdp_adamw_finish(float* state, float* scale_tracker, float growth, float backoff, int interval, float* steps,
                     int nsteps, void* stream);
/* Bit-reproducible gradient norm: sdp_grad_sumsq_parts writes block b's sum of squares to
 * partials[b] (and flags non-finite values in state[1]); sdp_sum_partials adds partials[0..n)
 * in a fixed order into state[0].  Same result as sdp_grad_sumsq without float atomics. */
/*
 * Flash-style training attention (layers.py:289-291, F.scaled_dot_product_attention with
 * dropout_p; bf16 only, hd % 16 == 0, hd <= 128, any N: every kernel streams 32-row tiles of the
 * head through a double-buffered LDS ring filled by a producer wave).
 * q, k, v of head h are columns h*hd, C + h*hd, 2C + h*hd of the [B*N, ldq] rows (C = H*hd).
 *   sdp_attn_train_fwd: O = dropout(softmax(scale Q K^T)) V into [B*N, ldo] rows; lse[(b*H+h)*N+q]
 *     = log2 sum_k exp2(scale log2(e) q.k) (fp32).  S and P are never stored.
 *   sdp_attn_train_bwd: dQ, dK, dV (bf16 rows, head h at column h*hd of each) from dO, O, lse;
 *     P recomputed; `delta` is caller scratch of B*H*N floats.  The dropout mask is a counter hash
 *     of (seed, b*H + h, q, k) -- the same in both directions; sdp_attn_dropout_mask writes it as
 *     bytes [B*H][N][N] (keep = 1) for tests.
 *   sdp_attn_train_applies(dtype, N, hd): 1 if the shape takes these kernels.
 */
int sdp_attn_train_applies(int dtype, int N, int hd);
int sdp_attn_train_fwd(int dtype, const void* qkv, int64_t ldq, void* o, int64_t ldo, float* lse, int B, int N, int H,
                       int hd, float scale, float p, uint64_t seed, void* stream);
int sdp_attn_train_bwd(int dtype, const void* qkv, int64_t ldq, const void* o, int64_t ldo, const void* dO,
                       int64_t lddo, const float* lse, float* delta, void* dq, int64_t lddq, void* dk, int64_t lddk,
                       void* dv, int64_t lddv, int B, int N, int H, int hd, float scale, float p, uint64_t seed,
                       void* stream);
int sdp_attn_dropout_mask(uint8_t* out, int Z, int N, float p, uint64_t seed, void* stream);
int sdp_grad_sumsq_parts(float* const* grads, const int64_t* sizes, const void* blocks, int nblocks,
                         float* partials, float* state, void* stream);
int sdp_sum_partials(const float* partials, int n, float* state, void* stream);

/* Weight gradient on the 8-phase MFMA main loop (training backward of every Linear / 1x1 conv,
 * the adjoint of layers.py:79-91, :242-249, :282-284, :308): C + s * split_stride = sum over
 * the token rows of split s of A[k][i] * B[k][j] (fp32), A = dY [ktok][lda], B = X [ktok][ldb]
 * bf16 token-major.  Split s covers K-tiles [s * kchunk_tiles, (s + 1) * kchunk_tiles) of 64
 * tokens; the caller reduces the slabs.  A last K-tile past ktok reads `zrow` (>= max(ni, nj)
 * zero bf16, 16-B aligned; may be NULL when ktok % 64 == 0) for the missing rows.  ni % 256 ==
 * 0, nj % 256 == 0, 16-B aligned operands (hipErrorNotSupported otherwise: use sdp_gemm_flex). */
int sdp_gemm_wgrad(const void* A, int64_t lda, const void* B, int64_t ldb, float* C, int64_t ldc,
                   int64_t split_stride, int ni, int nj, int ktok, int kchunk_tiles, const void* zrow,
                   void* stream);

/* Y = dropout(X) * scale[m / sgrp] (+ R) (mode 1) or Y = dropout(round(X * scale)) (mode 2), the
 * counter-hash mask of sdp_act_fwd (index m * N + n): the dropout of EncoderLayer's output
 * projections fused into the drop-path / residual pass (layers.py:301-309) and, mode 2, into the
 * cast of the stream gradient into that branch.  X in x_dtype, R / Y in y_dtype; 16-B aligned
 * rows, N % 8 == 0 (hipErrorNotSupported otherwise). */
int sdp_rowscale_add_dropout(int x_dtype, int y_dtype, const void* X, int64_t ldx, int x_grp, int64_t x_gstride,
                             int x_off, const float* scale, int sgrp, const void* R, int64_t ldr, int r_grp,
                             int64_t r_gstride, int r_off, void* Y, int64_t ldy, int y_grp, int64_t y_gstride,
                             int y_off, int M, int N, float p, uint64_t seed, int mode, void* stream);

/* Per-step weight preparation of the bf16 training step in one launch: entries is a device
 * array of sdp_mt_cast_transpose_entry_bytes()-sized records {const float* src; uint16_t* dst;
 * uint16_t* dstT; int64 ldd; int64 ldt; int R; int C} (fp32 [R][C] row-major in; bf16 copy
 * dst[r * ldd + c] and transposed copy dstT[c * ldt + r] out, either may be NULL); tiles is a
 * device array of int4 {entry, r0, c0, 0}, one 64 x 64 tile per workgroup. */
int sdp_mt_cast_transpose_entry_bytes(void);
int sdp_mt_cast_transpose(const void* entries, const void* tiles, int ntiles, void* stream);


#ifdef __cplusplus
}
#endif
#endif /* SDPNET_HIP_H */
