// Layout / embedding kernels around the SdP-Net hot path.
//
//  * sdp_patchify   — im2col for the stride = kernel = p patch conv
//                     (ConvPatcher, layers.py:34-42): image [B,3,Hi,Wi] ->
//                     rows [B*Hp*Wp, Kpad], column c*p*p + i*p + j (the flattened
//                     conv weight order), zero pad to Kpad (multiple of 64).
//  * sdp_pos_table  — EmbeddingLayer positional table (layers.py:157-163):
//                     T[h*W + w] = Eh[h] + Ew[w]  ('horizontal' table by row h,
//                     'vertical' by column w).
//  * sdp_avgpool_table — ConvEmbedding (layers.py:205): T[h*W+w][c] =
//                     mean_{k x k} bone[c][h+i][w+j].
//  * sdp_copy_rows  — strided row copy; with a zero source batch stride it is the
//                     register expansion over the batch (layers.py:166, :208)
//                     into token rows 0..R-1, else the register split (:311).
//  * sdp_nchw_add_table / sdp_act — standalone EmbeddingLayer.forward
//                     (in-place positional add on NCHW, layers.py:162-163, then
//                     the embedding activation) outside the fused model path.
//  * sdp_group_mean — mean over groups of rows: registers.mean(-2) of the head
//                     (layers.py:464) and the AdaptiveAvgPool2d((1,1)) head (:457).
//  * sdp_nchw_to_rows / sdp_rows_to_nchw — NCHW <-> token rows (the
//                     flatten/transpose of layers.py:271, :314), LDS-tiled.
//  * sdp_cast       — fp32 <-> bf16 element cast.
#include "common.h"

static RowMap mk_map3(int grp, int64_t gstride, int off) {
  RowMap r;
  r.grp = grp > 0 ? grp : 0x7fffffff;
  r.gstride = grp > 0 ? gstride : 0;
  r.off = grp > 0 ? off : 0;
  return r;
}

template <typename TI, typename TO>
__global__ void patchify_k(const TI* __restrict__ img, TO* __restrict__ out, int B, int Hi, int Wi, int p, int Hp,
                           int Wp, int Kpad) {
  const int64_t total = (int64_t)B * Hp * Wp * Kpad;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int col = (int)(idx % Kpad);
    const int64_t row = idx / Kpad;
    float v = 0.f;
    if (col < 3 * p * p) {
      const int c = col / (p * p), ij = col % (p * p), i = ij / p, j = ij % p;
      const int pw = (int)(row % Wp);
      const int64_t t = row / Wp;
      const int ph = (int)(t % Hp);
      const int b = (int)(t / Hp);
      v = to_f<TI>(img[(((int64_t)b * 3 + c) * Hi + ph * p + i) * Wi + pw * p + j]);
    }
    out[idx] = from_f<TO>(v);
  }
}

// One workgroup per patch row (b, ph, pw): the row's (b, ph, pw) decomposition is uniform and the
// per-column image offset is 32-bit arithmetic on the column alone (the grid-stride form above
// divides a 64-bit index five times per element).  Column-fastest threads: the loads walk the
// patch's pixel rows (p contiguous floats each), the stores are one contiguous row.
template <typename TI, typename TO>
__global__ __launch_bounds__(256) void patchify_rows_k(const TI* __restrict__ img, TO* __restrict__ out, int Hi,
                                                       int Wi, int p, int Hp, int Wp, int Kpad) {
  const int row = blockIdx.x;
  const int pw = row % Wp, t = row / Wp, ph = t % Hp, b = t / Hp;
  const TI* src = img + (int64_t)b * 3 * Hi * Wi + (int64_t)(ph * p) * Wi + pw * p;
  TO* dst = out + (int64_t)row * Kpad;
  const int pp = p * p;
  for (int col = threadIdx.x; col < Kpad; col += 256) {
    float v = 0.f;
    if (col < 3 * pp) {
      const int c = col / pp, ij = col - c * pp, i = ij / p, j = ij - i * p;
      v = to_f<TI>(src[(c * Hi + i) * Wi + j]);
    }
    dst[col] = from_f<TO>(v);
  }
}

// One workgroup per patch-row strip (b, ph): the strip's 3 x p image rows are read as pixel pairs in
// image order (coalesced rows of Wp p pixels per channel), each pair lands in one patch row (p even),
// and the Kpad - 3 p p padding columns of the strip's Wp patch rows are zeroed.  The per-patch-row
// kernel above walked each patch's p-pixel segments in its own workgroup, so the image lines shared by
// neighbouring patches were fetched once per patch (XL, p = 14: 2.4x the algorithmic bytes).
template <typename TI, typename TO>
__global__ __launch_bounds__(256) void patchify_strip_k(const TI* __restrict__ img, TO* __restrict__ out, int Hi,
                                                        int Wi, int p, int Hp, int Wp, int Kpad) {
  const int strip = blockIdx.x;  // b * Hp + ph
  const int ph = strip % Hp, b = strip / Hp;
  const int pp = p * p, W2 = Wp * p / 2;  // pixel pairs per image row segment
  const int n = 3 * p * W2;
  const TI* base = img + (int64_t)b * 3 * Hi * Wi + (int64_t)(ph * p) * Wi;
  TO* obase = out + (int64_t)strip * Wp * Kpad;
  for (int t = threadIdx.x; t < n; t += 256) {
    const int w2 = t % W2, ci = t / W2, c = ci / p, i = ci - c * p;
    const int w = 2 * w2, pw = w / p, j = w - pw * p;
    const TI* src = base + ((int64_t)c * Hi + i) * Wi + w;
    float v0, v1;
    if constexpr (sizeof(TI) == 4) {
      const float2 f = *(const float2*)src;
      v0 = f.x;
      v1 = f.y;
    } else {
      const uint32_t u = *(const uint32_t*)src;
      v0 = bf2f((bf16_t)(u & 0xffffu));
      v1 = bf2f((bf16_t)(u >> 16));
    }
    TO* dst = obase + (int64_t)pw * Kpad + c * pp + i * p + j;
    if constexpr (sizeof(TO) == 2) {
      *(uint32_t*)dst = (uint32_t)f2bf(v0) | ((uint32_t)f2bf(v1) << 16);
    } else {
      *(float2*)dst = float2{v0, v1};
    }
  }
  const int padc = Kpad - 3 * pp;
  for (int t = threadIdx.x; t < Wp * padc; t += 256) {
    const int pw = t / padc;
    obase[(int64_t)pw * Kpad + 3 * pp + (t - pw * padc)] = from_f<TO>(0.f);
  }
}

extern "C" int sdp_patchify(int dtype_in, const void* img, int dtype_out, void* out, int B, int Hi, int Wi, int p,
                            int Kpad, void* stream) {
  if (!img || !out || p <= 0 || Kpad < 3 * p * p) return (int)hipErrorInvalidValue;
  const int Hp = Hi / p, Wp = Wi / p;
  const int64_t total = (int64_t)B * Hp * Wp * Kpad;
  if (total == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const int64_t rows = (int64_t)B * Hp * Wp;
  // pixel pairs: p and Wi even, the pairs 4-B (bf16 in) / 8-B (fp32 in) aligned
  const int ein = dtype_in == 0 ? 4 : 2;
  if (p % 2 == 0 && Wi % 2 == 0 && Kpad % 2 == 0 && (uintptr_t)img % (2 * ein) == 0 &&
      (uintptr_t)out % (dtype_out == 0 ? 8 : 4) == 0 && (int64_t)B * Hp < (1ll << 31) &&
      (int64_t)3 * Hi * Wi < (1ll << 31)) {
#define SDP_PATCH_STRIP(TI, TO)                                                                                     \
  hipLaunchKernelGGL((patchify_strip_k<TI, TO>), dim3((unsigned)(B * Hp)), dim3(256), 0, s, (const TI*)img,        \
                     (TO*)out, Hi, Wi, p, Hp, Wp, Kpad)
    if (dtype_in == 0 && dtype_out == 1) SDP_PATCH_STRIP(float, bf16_t);
    else if (dtype_in == 0 && dtype_out == 0) SDP_PATCH_STRIP(float, float);
    else if (dtype_in == 1 && dtype_out == 1) SDP_PATCH_STRIP(bf16_t, bf16_t);
    else if (dtype_in == 1 && dtype_out == 0) SDP_PATCH_STRIP(bf16_t, float);
    else return (int)hipErrorInvalidValue;
#undef SDP_PATCH_STRIP
    return SDP_CHECK_LAUNCH();
  }
  if (rows < (1ll << 31) && (int64_t)3 * Hi * Wi < (1ll << 31)) {
#define SDP_PATCH_ROWS(TI, TO)                                                                                   \
  hipLaunchKernelGGL((patchify_rows_k<TI, TO>), dim3((unsigned)rows), dim3(256), 0, s, (const TI*)img, (TO*)out, \
                     Hi, Wi, p, Hp, Wp, Kpad)
    if (dtype_in == 0 && dtype_out == 1) SDP_PATCH_ROWS(float, bf16_t);
    else if (dtype_in == 0 && dtype_out == 0) SDP_PATCH_ROWS(float, float);
    else if (dtype_in == 1 && dtype_out == 1) SDP_PATCH_ROWS(bf16_t, bf16_t);
    else if (dtype_in == 1 && dtype_out == 0) SDP_PATCH_ROWS(bf16_t, float);
    else return (int)hipErrorInvalidValue;
#undef SDP_PATCH_ROWS
    return SDP_CHECK_LAUNCH();
  }
  const int blocks = (int)std::min<int64_t>((total + 255) / 256, 8192);
  if (dtype_in == 0 && dtype_out == 1)
    hipLaunchKernelGGL((patchify_k<float, bf16_t>), dim3(blocks), dim3(256), 0, s, (const float*)img, (bf16_t*)out, B, Hi, Wi, p, Hp, Wp, Kpad);
  else if (dtype_in == 0 && dtype_out == 0)
    hipLaunchKernelGGL((patchify_k<float, float>), dim3(blocks), dim3(256), 0, s, (const float*)img, (float*)out, B, Hi, Wi, p, Hp, Wp, Kpad);
  else if (dtype_in == 1 && dtype_out == 1)
    hipLaunchKernelGGL((patchify_k<bf16_t, bf16_t>), dim3(blocks), dim3(256), 0, s, (const bf16_t*)img, (bf16_t*)out, B, Hi, Wi, p, Hp, Wp, Kpad);
  else if (dtype_in == 1 && dtype_out == 0)
    hipLaunchKernelGGL((patchify_k<bf16_t, float>), dim3(blocks), dim3(256), 0, s, (const bf16_t*)img, (float*)out, B, Hi, Wi, p, Hp, Wp, Kpad);
  else
    return (int)hipErrorInvalidValue;
  return SDP_CHECK_LAUNCH();
}

// adjoint of patchify_k: image gradient [B,3,Hi,Wi] from the patch-row gradient [B*Hp*Wp, Kpad]
// (stride = kernel: every pixel belongs to at most one patch; the rows / columns past Hp*p / Wp*p
// that the stride-p convolution drops get 0).  One thread per image element.
template <typename TI, typename TO>
__global__ void unpatchify_k(const TI* __restrict__ rows, TO* __restrict__ img, int B, int Hi, int Wi, int p, int Hp,
                             int Wp, int Kpad) {
  const int64_t total = (int64_t)B * 3 * Hi * Wi;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int x = (int)(idx % Wi);
    const int64_t t = idx / Wi;
    const int y = (int)(t % Hi);
    const int64_t bc = t / Hi;
    const int c = (int)(bc % 3), b = (int)(bc / 3);
    float v = 0.f;
    if (y < Hp * p && x < Wp * p) {
      const int ph = y / p, i = y - ph * p, pw = x / p, j = x - pw * p;
      v = to_f<TI>(rows[(((int64_t)b * Hp + ph) * Wp + pw) * Kpad + c * p * p + i * p + j]);
    }
    img[idx] = from_f<TO>(v);
  }
}

extern "C" int sdp_unpatchify(int dtype_in, const void* rows, int dtype_out, void* img, int B, int Hi, int Wi, int p,
                              int Kpad, void* stream) {
  if (!rows || !img || p <= 0 || Kpad < 3 * p * p || B < 0 || Hi < 0 || Wi < 0) return (int)hipErrorInvalidValue;
  const int Hp = Hi / p, Wp = Wi / p;
  const int64_t total = (int64_t)B * 3 * Hi * Wi;
  if (total == 0) return 0;
  const int blocks = (int)std::min<int64_t>((total + 255) / 256, 8192);
  hipStream_t s = (hipStream_t)stream;
  if (dtype_in == 1 && dtype_out == 0)
    hipLaunchKernelGGL((unpatchify_k<bf16_t, float>), dim3(blocks), dim3(256), 0, s, (const bf16_t*)rows, (float*)img, B, Hi, Wi, p, Hp, Wp, Kpad);
  else if (dtype_in == 0 && dtype_out == 0)
    hipLaunchKernelGGL((unpatchify_k<float, float>), dim3(blocks), dim3(256), 0, s, (const float*)rows, (float*)img, B, Hi, Wi, p, Hp, Wp, Kpad);
  else if (dtype_in == 1 && dtype_out == 1)
    hipLaunchKernelGGL((unpatchify_k<bf16_t, bf16_t>), dim3(blocks), dim3(256), 0, s, (const bf16_t*)rows, (bf16_t*)img, B, Hi, Wi, p, Hp, Wp, Kpad);
  else if (dtype_in == 0 && dtype_out == 1)
    hipLaunchKernelGGL((unpatchify_k<float, bf16_t>), dim3(blocks), dim3(256), 0, s, (const float*)rows, (bf16_t*)img, B, Hi, Wi, p, Hp, Wp, Kpad);
  else
    return (int)hipErrorInvalidValue;
  return SDP_CHECK_LAUNCH();
}

__global__ void pos_table_k(const float* __restrict__ eh, const float* __restrict__ ew, float* __restrict__ out, int H,
                            int W, int C) {
  const int64_t total = (int64_t)H * W * C;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(idx % C);
    const int64_t hw = idx / C;
    const int h = (int)(hw / W), w = (int)(hw % W);
    out[idx] = eh[(int64_t)h * C + c] + ew[(int64_t)w * C + c];
  }
}

extern "C" int sdp_pos_table(const float* eh, const float* ew, float* out, int H, int W, int C, void* stream) {
  if (!eh || !ew || !out || H <= 0 || W <= 0 || C <= 0) return (int)hipErrorInvalidValue;
  const int64_t total = (int64_t)H * W * C;
  hipLaunchKernelGGL(pos_table_k, dim3((unsigned)std::min<int64_t>((total + 255) / 256, 4096)), dim3(256), 0,
                     (hipStream_t)stream, eh, ew, out, H, W, C);
  return SDP_CHECK_LAUNCH();
}

__global__ void avgpool_table_k(const float* __restrict__ bone, int BH, int BW, float* __restrict__ out, int H, int W,
                                int C, int k) {
  const int64_t total = (int64_t)H * W * C;
  const float inv = 1.0f / (float)(k * k);
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(idx % C);
    const int64_t hw = idx / C;
    const int h = (int)(hw / W), w = (int)(hw % W);
    float s = 0.f;
    for (int i = 0; i < k; ++i)
      for (int j = 0; j < k; ++j) s += bone[((int64_t)c * BH + h + i) * BW + w + j];
    out[idx] = s * inv;
  }
}

extern "C" int sdp_avgpool_table(const float* bone, int BH, int BW, float* out, int H, int W, int C, int k,
                                 void* stream) {
  if (!bone || !out || H + k - 1 > BH || W + k - 1 > BW) return (int)hipErrorInvalidValue;
  const int64_t total = (int64_t)H * W * C;
  hipLaunchKernelGGL(avgpool_table_k, dim3((unsigned)std::min<int64_t>((total + 255) / 256, 4096)), dim3(256), 0,
                     (hipStream_t)stream, bone, BH, BW, out, H, W, C, k);
  return SDP_CHECK_LAUNCH();
}

// Adjoint of sdp_avgpool_table (trainable bone, layers.py:189-190): dbone[c, i, j] =
// 1/k^2 * sum of dtable[h * W + w, c] over the windows (h, w) covering (i, j); the whole
// [C, BH, BW] gradient is written (zeros outside the used region).
__global__ void avgpool_table_bwd_k(const float* __restrict__ dt, int H, int W, int C, int k, float* __restrict__ dbone,
                                    int BH, int BW) {
  const int64_t total = (int64_t)C * BH * BW;
  const float inv = 1.0f / (float)(k * k);
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int j = (int)(idx % BW), i = (int)((idx / BW) % BH), c = (int)(idx / ((int64_t)BW * BH));
    float s = 0.f;
    for (int h = max(0, i - k + 1); h <= min(H - 1, i); ++h)
      for (int w = max(0, j - k + 1); w <= min(W - 1, j); ++w) s += dt[((int64_t)h * W + w) * C + c];
    dbone[idx] = s * inv;
  }
}

extern "C" int sdp_avgpool_table_bwd(const float* dtable, int H, int W, int C, int k, float* dbone, int BH, int BW,
                                     void* stream) {
  if (!dtable || !dbone || H <= 0 || W <= 0 || C <= 0 || k <= 0 || H + k - 1 > BH || W + k - 1 > BW)
    return (int)hipErrorInvalidValue;
  const int64_t total = (int64_t)C * BH * BW;
  hipLaunchKernelGGL(avgpool_table_bwd_k, dim3((unsigned)std::min<int64_t>((total + 255) / 256, 4096)), dim3(256), 0,
                     (hipStream_t)stream, dtable, H, W, C, k, dbone, BH, BW);
  return SDP_CHECK_LAUNCH();
}

template <typename TI, typename TO>
__global__ void broadcast_rows_k(const TI* __restrict__ src, int64_t lds, int64_t sgstride, TO* __restrict__ dst,
                                 int64_t ldd, int64_t gstride, int B, int R, int C) {
  const int64_t total = (int64_t)B * R * C;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(idx % C);
    const int64_t br = idx / C;
    const int r = (int)(br % R), b = (int)(br / R);
    dst[b * gstride + (int64_t)r * ldd + c] = from_f<TO>(to_f<TI>(src[b * sgstride + (int64_t)r * lds + c]));
  }
}

// Same-dtype copy, 16 B per work item (rows of 16-B multiples, 16-B aligned bases / strides).
__global__ void copy_rows16_k(const uint4* __restrict__ src, int64_t lds, int64_t sgstride, uint4* __restrict__ dst,
                              int64_t ldd, int64_t gstride, int B, int R, int C16) {
  const int64_t total = (int64_t)B * R * C16;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(idx % C16);
    const int64_t br = idx / C16;
    const int r = (int)(br % R), b = (int)(br / R);
    dst[b * gstride + (int64_t)r * ldd + c] = src[b * sgstride + (int64_t)r * lds + c];
  }
}

// dst[b*gstride + r*ldd + c] = src[b*sgstride + r*lds + c]  (sgstride 0 = broadcast)
extern "C" int sdp_copy_rows(int dtype_src, const void* src, int64_t lds, int64_t sgstride, int dtype_dst, void* dst,
                             int64_t ldd, int64_t gstride, int B, int R, int C, void* stream) {
  if (!src || !dst || B < 0 || R < 0 || C <= 0) return (int)hipErrorInvalidValue;
  const int64_t total = (int64_t)B * R * C;
  if (total == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  if (dtype_src == dtype_dst && (dtype_src == 0 || dtype_src == 1)) {
    const int64_t es = dtype_src == 1 ? 2 : 4, per = 16 / es;  // elements per 16 B
    if (C % per == 0 && lds % per == 0 && ldd % per == 0 && sgstride % per == 0 && gstride % per == 0 &&
        (uintptr_t)src % 16 == 0 && (uintptr_t)dst % 16 == 0) {
      const int C16 = (int)(C / per);
      const int64_t t16 = (int64_t)B * R * C16;
      dim3 g16((unsigned)std::min<int64_t>((t16 + 255) / 256, 8192));
      hipLaunchKernelGGL(copy_rows16_k, g16, dim3(256), 0, s, (const uint4*)src, lds / per, sgstride / per,
                         (uint4*)dst, ldd / per, gstride / per, B, R, C16);
      return SDP_CHECK_LAUNCH();
    }
  }
  dim3 grid((unsigned)std::min<int64_t>((total + 255) / 256, 4096));
  if (dtype_src == 0 && dtype_dst == 1)
    hipLaunchKernelGGL((broadcast_rows_k<float, bf16_t>), grid, dim3(256), 0, s, (const float*)src, lds, sgstride, (bf16_t*)dst, ldd, gstride, B, R, C);
  else if (dtype_src == 0 && dtype_dst == 0)
    hipLaunchKernelGGL((broadcast_rows_k<float, float>), grid, dim3(256), 0, s, (const float*)src, lds, sgstride, (float*)dst, ldd, gstride, B, R, C);
  else if (dtype_src == 1 && dtype_dst == 1)
    hipLaunchKernelGGL((broadcast_rows_k<bf16_t, bf16_t>), grid, dim3(256), 0, s, (const bf16_t*)src, lds, sgstride, (bf16_t*)dst, ldd, gstride, B, R, C);
  else if (dtype_src == 1 && dtype_dst == 0)
    hipLaunchKernelGGL((broadcast_rows_k<bf16_t, float>), grid, dim3(256), 0, s, (const bf16_t*)src, lds, sgstride, (float*)dst, ldd, gstride, B, R, C);
  else
    return (int)hipErrorInvalidValue;
  return SDP_CHECK_LAUNCH();
}

// out[g][c] = mean_{i < rows} X[xm(g*rows + i)][c]
template <typename TI, typename TO>
__global__ void group_mean_k(const TI* __restrict__ X, int64_t ldx, RowMap xm, TO* __restrict__ out, int64_t ldo,
                             int G, int rows, int C) {
  const int g = blockIdx.y;
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C || g >= G) return;
  float s = 0.f;
  for (int i = 0; i < rows; ++i) s += to_f<TI>(X[xm((int64_t)g * rows + i) * ldx + c]);
  out[(int64_t)g * ldo + c] = from_f<TO>(s / (float)rows);
}

extern "C" int sdp_group_mean(int dtype_in, const void* X, int64_t ldx, int x_grp, int64_t x_gstride, int x_off,
                              int dtype_out, void* out, int64_t ldo, int G, int rows, int C, void* stream) {
  if (!X || !out || G < 0 || rows <= 0 || C <= 0) return (int)hipErrorInvalidValue;
  if (G == 0) return 0;
  const RowMap xm = mk_map3(x_grp, x_gstride, x_off);
  dim3 grid((C + 255) / 256, G);
  hipStream_t s = (hipStream_t)stream;
  if (dtype_in == 1 && dtype_out == 1)
    hipLaunchKernelGGL((group_mean_k<bf16_t, bf16_t>), grid, dim3(256), 0, s, (const bf16_t*)X, ldx, xm, (bf16_t*)out, ldo, G, rows, C);
  else if (dtype_in == 1 && dtype_out == 0)
    hipLaunchKernelGGL((group_mean_k<bf16_t, float>), grid, dim3(256), 0, s, (const bf16_t*)X, ldx, xm, (float*)out, ldo, G, rows, C);
  else if (dtype_in == 0 && dtype_out == 0)
    hipLaunchKernelGGL((group_mean_k<float, float>), grid, dim3(256), 0, s, (const float*)X, ldx, xm, (float*)out, ldo, G, rows, C);
  else if (dtype_in == 0 && dtype_out == 1)
    hipLaunchKernelGGL((group_mean_k<float, bf16_t>), grid, dim3(256), 0, s, (const float*)X, ldx, xm, (bf16_t*)out, ldo, G, rows, C);
  else
    return (int)hipErrorInvalidValue;
  return SDP_CHECK_LAUNCH();
}

// NCHW [B, C, HW] <-> rows: row (b, hw) -> ym(b*HW + hw), element c.  64x64 LDS tile.
template <typename TI, typename TO, bool TO_ROWS>
__global__ __launch_bounds__(256) void transpose_k(const TI* __restrict__ src, TO* __restrict__ dst, int64_t ld,
                                                   RowMap rm, int C, int HW) {
  __shared__ float tile[64][65];
  const int b = blockIdx.z;
  const int c0 = blockIdx.y * 64, p0 = blockIdx.x * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  if (TO_ROWS) {
    // read NCHW: consecutive threads -> consecutive hw
    for (int i = ty; i < 64; i += 4) {
      const int c = c0 + i, p = p0 + tx;
      tile[i][tx] = (c < C && p < HW) ? to_f<TI>(src[((int64_t)b * C + c) * HW + p]) : 0.f;
    }
    __syncthreads();
    for (int i = ty; i < 64; i += 4) {
      const int p = p0 + i, c = c0 + tx;
      if (c < C && p < HW) dst[rm((int64_t)b * HW + p) * ld + c] = from_f<TO>(tile[tx][i]);
    }
  } else {
    for (int i = ty; i < 64; i += 4) {
      const int p = p0 + i, c = c0 + tx;
      tile[tx][i] = (c < C && p < HW) ? to_f<TI>(src[rm((int64_t)b * HW + p) * ld + c]) : 0.f;
    }
    __syncthreads();
    for (int i = ty; i < 64; i += 4) {
      const int c = c0 + i, p = p0 + tx;
      if (c < C && p < HW) dst[((int64_t)b * C + c) * HW + p] = from_f<TO>(tile[i][tx]);
    }
  }
}

template <bool TO_ROWS>
static int launch_transpose(int dti, const void* src, int dto, void* dst, int64_t ld, RowMap rm, int B, int C,
                            int HW, hipStream_t s) {
  dim3 grid((HW + 63) / 64, (C + 63) / 64, B);
#define SDP_T(TI, TO) hipLaunchKernelGGL((transpose_k<TI, TO, TO_ROWS>), grid, dim3(256), 0, s, (const TI*)src, (TO*)dst, ld, rm, C, HW)
  if (dti == 0 && dto == 0) SDP_T(float, float);
  else if (dti == 0 && dto == 1) SDP_T(float, bf16_t);
  else if (dti == 1 && dto == 0) SDP_T(bf16_t, float);
  else if (dti == 1 && dto == 1) SDP_T(bf16_t, bf16_t);
  else return (int)hipErrorInvalidValue;
#undef SDP_T
  return SDP_CHECK_LAUNCH();
}

extern "C" int sdp_nchw_to_rows(int dtype_in, const void* X, int dtype_out, void* Y, int64_t ldy, int y_grp,
                                int64_t y_gstride, int y_off, int B, int C, int HW, void* stream) {
  if (!X || !Y || B < 0 || C <= 0 || HW <= 0) return (int)hipErrorInvalidValue;
  if (B == 0) return 0;
  return launch_transpose<true>(dtype_in, X, dtype_out, Y, ldy, mk_map3(y_grp, y_gstride, y_off), B, C, HW,
                                (hipStream_t)stream);
}

extern "C" int sdp_rows_to_nchw(int dtype_in, const void* X, int64_t ldx, int x_grp, int64_t x_gstride, int x_off,
                                int dtype_out, void* Y, int B, int C, int HW, void* stream) {
  if (!X || !Y || B < 0 || C <= 0 || HW <= 0) return (int)hipErrorInvalidValue;
  if (B == 0) return 0;
  return launch_transpose<false>(dtype_in, X, dtype_out, Y, ldx, mk_map3(x_grp, x_gstride, x_off), B, C, HW,
                                 (hipStream_t)stream);
}

template <typename TI, typename TO>
__global__ void cast_k(const TI* __restrict__ x, TO* __restrict__ y, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    y[i] = from_f<TO>(to_f<TI>(x[i]));
}

extern "C" int sdp_cast(int dtype_in, const void* X, int dtype_out, void* Y, int64_t n, void* stream) {
  if (!X || !Y || n < 0) return (int)hipErrorInvalidValue;
  if (n == 0) return 0;
  dim3 grid((unsigned)std::min<int64_t>((n + 255) / 256, 8192));
  hipStream_t s = (hipStream_t)stream;
  if (dtype_in == 0 && dtype_out == 1) hipLaunchKernelGGL((cast_k<float, bf16_t>), grid, dim3(256), 0, s, (const float*)X, (bf16_t*)Y, n);
  else if (dtype_in == 1 && dtype_out == 0) hipLaunchKernelGGL((cast_k<bf16_t, float>), grid, dim3(256), 0, s, (const bf16_t*)X, (float*)Y, n);
  else if (dtype_in == 0 && dtype_out == 0) hipLaunchKernelGGL((cast_k<float, float>), grid, dim3(256), 0, s, (const float*)X, (float*)Y, n);
  else if (dtype_in == 1 && dtype_out == 1) hipLaunchKernelGGL((cast_k<bf16_t, bf16_t>), grid, dim3(256), 0, s, (const bf16_t*)X, (bf16_t*)Y, n);
  else return (int)hipErrorInvalidValue;
  return SDP_CHECK_LAUNCH();
}

// x[b][c][hw] += table[hw][c]  (in place, NCHW)
template <typename T>
__global__ void nchw_add_table_k(T* __restrict__ x, const float* __restrict__ table, int B, int C, int HW) {
  const int64_t total = (int64_t)B * C * HW;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int hw = (int)(i % HW);
    const int c = (int)((i / HW) % C);
    x[i] = from_f<T>(to_f<T>(x[i]) + table[(int64_t)hw * C + c]);
  }
}

extern "C" int sdp_nchw_add_table(int dtype, void* X, const float* table, int B, int C, int HW, void* stream) {
  if (!X || !table || B < 0 || C <= 0 || HW <= 0) return (int)hipErrorInvalidValue;
  const int64_t n = (int64_t)B * C * HW;
  if (n == 0) return 0;
  dim3 grid((unsigned)std::min<int64_t>((n + 255) / 256, 8192));
  hipStream_t s = (hipStream_t)stream;
  if (dtype == 1) hipLaunchKernelGGL(nchw_add_table_k<bf16_t>, grid, dim3(256), 0, s, (bf16_t*)X, table, B, C, HW);
  else if (dtype == 0) hipLaunchKernelGGL(nchw_add_table_k<float>, grid, dim3(256), 0, s, (float*)X, table, B, C, HW);
  else return (int)hipErrorInvalidValue;
  return SDP_CHECK_LAUNCH();
}

template <typename T>
__global__ void act_k(const T* __restrict__ x, T* __restrict__ y, int64_t n, int act) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    y[i] = from_f<T>(apply_act(act, to_f<T>(x[i])));
}

extern "C" int sdp_act(int dtype, const void* X, void* Y, int64_t n, int act, void* stream) {
  if (!X || !Y || n < 0) return (int)hipErrorInvalidValue;
  if (n == 0) return 0;
  dim3 grid((unsigned)std::min<int64_t>((n + 255) / 256, 8192));
  hipStream_t s = (hipStream_t)stream;
  if (dtype == 1) hipLaunchKernelGGL(act_k<bf16_t>, grid, dim3(256), 0, s, (const bf16_t*)X, (bf16_t*)Y, n, act);
  else if (dtype == 0) hipLaunchKernelGGL(act_k<float>, grid, dim3(256), 0, s, (const float*)X, (float*)Y, n, act);
  else return (int)hipErrorInvalidValue;
  return SDP_CHECK_LAUNCH();
}

extern "C" const char* sdp_version(void) { return "sdpnet-hip gfx950 r1"; }

// ---------------------------------------------------------------------------
// LayerNorm folding of a Linear / 1x1 conv that consumes LN(x) (layers.py:83-88
// after :102-103's layer_norm_2, :282-284 after norm1, :308 after norm2):
//   LN(x) . W^T + b = rstd * (x . (W*gamma)^T) - rstd * mean * colsum + (beta . W^T + b)
// One workgroup per output row n: Wf[n][k] = cast(W[n][k] * gamma[k]),
// colsum[n] = sum_k Wf[n][k] (of the stored, rounded values), cvec[n] = sum_k beta[k] W[n][k]
// (+ bias[n]).  W, gamma, beta, bias fp32.  Run once per weight version.
// ---------------------------------------------------------------------------
template <typename TO>
__global__ __launch_bounds__(256) void fold_ln_k(const float* __restrict__ W, const float* __restrict__ g,
                                                 const float* __restrict__ be, const float* __restrict__ bias,
                                                 TO* __restrict__ Wf, float* __restrict__ colsum,
                                                 float* __restrict__ cvec, int K) {
  const int n = blockIdx.x;
  const float* w = W + (int64_t)n * K;
  float s = 0.f, c = 0.f;
  for (int k = threadIdx.x; k < K; k += 256) {
    const TO v = from_f<TO>(w[k] * g[k]);
    Wf[(int64_t)n * K + k] = v;
    s += to_f<TO>(v);
    c = fmaf(be[k], w[k], c);
  }
  __shared__ float red[2][4];
  s = wave_sum(s);
  c = wave_sum(c);
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = s;
    red[1][threadIdx.x >> 6] = c;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    colsum[n] = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    cvec[n] = red[1][0] + red[1][1] + red[1][2] + red[1][3] + (bias ? bias[n] : 0.f);
  }
}

extern "C" int sdp_fold_ln_weight(const float* W, const float* gamma, const float* beta, const float* bias, int N,
                                  int K, int dtype_out, void* Wf, float* colsum, float* cvec, void* stream) {
  if (!W || !gamma || !beta || !Wf || !colsum || !cvec || N <= 0 || K <= 0) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  if (dtype_out == 1)
    hipLaunchKernelGGL(fold_ln_k<bf16_t>, dim3(N), dim3(256), 0, s, W, gamma, beta, bias, (bf16_t*)Wf, colsum, cvec, K);
  else if (dtype_out == 0)
    hipLaunchKernelGGL(fold_ln_k<float>, dim3(N), dim3(256), 0, s, W, gamma, beta, bias, (float*)Wf, colsum, cvec, K);
  else
    return (int)hipErrorInvalidValue;
  return SDP_CHECK_LAUNCH();
}


// Timing experiments only (tools/r4_skip.sh, diagnostic build): bit 0 skips sdp_dwconv, bit 1
// sdp_attention, bit 2 sdp_ln_stats -- the results are then WRONG; it bounds what a faster kernel
// could give the step.  Returns the previous mask.  The product library has no skip paths: it keeps
// the mask at 0 and returns -1 for any non-zero request (sdp_build_info() tells the builds apart).
#ifdef SDP_DIAG
int g_sdp_debug_skip = 0;
extern "C" int sdp_debug_skip(int mask) {
  const int old = g_sdp_debug_skip;
  g_sdp_debug_skip = mask;
  return old;
}
#else
extern "C" int sdp_debug_skip(int mask) { return mask ? -1 : 0; }
#endif

// Build flags of this library: bit 0 = diagnostic kernel skipping compiled in (SDP_DIAG), bit 1 =
// GEMM wall-clock stamps compiled in (SDP_GEMM_STAMPS).  0 for the product library; bench.py
// refuses to time anything else.
extern "C" int sdp_build_info(void) {
  int f = 0;
#ifdef SDP_DIAG
  f |= 1;
#endif
#ifdef SDP_GEMM_STAMPS
  f |= 2;
#endif
  return f;
}
