// Row LayerNorm and the depthwise k x k convolution, token-major (NHWC) layout.
//
//  * sdp_layernorm — per-row LN over the contiguous channel dim.  Serves
//      - channel LayerNorm of ConvMixer (layers.py:12-24, eps 1e-6, biased var)
//        which on the token layout is a row LN over C;
//      - nn.LayerNorm norm1/norm2 of EncoderLayer (layers.py:252-253, eps 1e-5)
//      - the head LayerNorm (layers.py:445-453).
//    One wave per row, row cached in registers, two-pass mean / centred
//    variance (fp32), 8-16 B vector loads.
//  * sdp_qk_headnorm — q_norm / k_norm (layers.py:236-237, :286): LayerNorm over
//    each head_dim segment of the q and k thirds of the fused QKV rows, in place.
//  * sdp_rowstats — per-row (mean, rstd) for a LayerNorm applied by its consumer.
//  * sdp_dwconv — depthwise conv (layers.py:73-78: groups=C, padding="same",
//    zeros, optional bias) on image rows of a token-major buffer, optionally on
//    LN(x) computed while staging (ConvMixer layer_norm_1, layers.py:102).
#include "common.h"
#include <type_traits>

// ---------------------------------------------------------------------------
// Row LayerNorm
// ---------------------------------------------------------------------------
template <typename T, int VPL>  // VPL: 4-element vectors per lane held in registers
__global__ __launch_bounds__(256) void layernorm_rows(const T* __restrict__ X, int64_t ldx, RowMap xm,
                                                      const float* __restrict__ g,
                                                      const float* __restrict__ bta, float eps,
                                                      T* __restrict__ Y, int64_t ldy, RowMap ym, int M,
                                                      int C) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const T* xp = X + xm(row) * ldx;
  T* yp = Y + ym(row) * ldy;
  const int nv = C >> 2;  // C % 4 == 0 enforced by the launcher
  float v[VPL][4];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c4 = lane + i * 64;
    if (c4 < nv) {
      if constexpr (sizeof(T) == 2) {
        bf16x4 t = *(const bf16x4*)(xp + c4 * 4);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[i][r] = bf2f((bf16_t)t[r]);
      } else {
        f32x4 t = *(const f32x4*)(xp + c4 * 4);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[i][r] = t[r];
      }
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) v[i][r] = 0.f;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) s += v[i][r];
  }
  const float mean = wave_sum(s) / (float)C;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c4 = lane + i * 64;
    if (c4 < nv) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float d = v[i][r] - mean;
        ss += d * d;
      }
    }
  }
  const float var = wave_sum(ss) / (float)C;
  const float rstd = 1.0f / sqrtf(var + eps);
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c4 = lane + i * 64;
    if (c4 < nv) {
      const f32x4 gg = *(const f32x4*)(g + c4 * 4);
      const f32x4 bb = *(const f32x4*)(bta + c4 * 4);
      float o[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = (v[i][r] - mean) * rstd * gg[r] + bb[r];
      if constexpr (sizeof(T) == 2) {
        bf16x4 t;
#pragma unroll
        for (int r = 0; r < 4; ++r) t[r] = (short)f2bf(o[r]);
        *(bf16x4*)(yp + c4 * 4) = t;
      } else {
        *(f32x4*)(yp + c4 * 4) = f32x4{o[0], o[1], o[2], o[3]};
      }
    }
  }
}

// Scalar fallback for C % 4 != 0 or very wide rows: three passes over global.
template <typename T>
__global__ __launch_bounds__(256) void layernorm_rows_scalar(const T* __restrict__ X, int64_t ldx, RowMap xm,
                                                             const float* __restrict__ g,
                                                             const float* __restrict__ bta, float eps,
                                                             T* __restrict__ Y, int64_t ldy, RowMap ym,
                                                             int M, int C) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const T* xp = X + xm(row) * ldx;
  T* yp = Y + ym(row) * ldy;
  float s = 0.f;
  for (int c = lane; c < C; c += 64) s += to_f<T>(xp[c]);
  const float mean = wave_sum(s) / (float)C;
  float ss = 0.f;
  for (int c = lane; c < C; c += 64) {
    const float d = to_f<T>(xp[c]) - mean;
    ss += d * d;
  }
  const float rstd = 1.0f / sqrtf(wave_sum(ss) / (float)C + eps);
  for (int c = lane; c < C; c += 64) yp[c] = from_f<T>((to_f<T>(xp[c]) - mean) * rstd * g[c] + bta[c]);
}

static RowMap mk_rmap(int grp, int64_t gstride, int off) {
  RowMap r;
  r.grp = grp > 0 ? grp : 0x7fffffff;
  r.gstride = grp > 0 ? gstride : 0;
  r.off = grp > 0 ? off : 0;
  return r;
}

template <typename T>
static int launch_ln(const void* X, int64_t ldx, RowMap xm, const float* g, const float* b, float eps, void* Y,
                     int64_t ldy, RowMap ym, int M, int C, hipStream_t s) {
  dim3 grid((M + 3) / 4), blk(256);
  const bool vec_ok = (C % 4 == 0) && (ldx % 4 == 0) && (ldy % 4 == 0) &&
                      ((uintptr_t)X % 16 == 0) && ((uintptr_t)Y % 16 == 0);
  const int nv = C / 4;
  if (vec_ok && nv <= 64)
    hipLaunchKernelGGL((layernorm_rows<T, 1>), grid, blk, 0, s, (const T*)X, ldx, xm, g, b, eps, (T*)Y, ldy, ym, M, C);
  else if (vec_ok && nv <= 256)
    hipLaunchKernelGGL((layernorm_rows<T, 4>), grid, blk, 0, s, (const T*)X, ldx, xm, g, b, eps, (T*)Y, ldy, ym, M, C);
  else if (vec_ok && nv <= 1024)
    hipLaunchKernelGGL((layernorm_rows<T, 16>), grid, blk, 0, s, (const T*)X, ldx, xm, g, b, eps, (T*)Y, ldy, ym, M, C);
  else
    hipLaunchKernelGGL(layernorm_rows_scalar<T>, grid, blk, 0, s, (const T*)X, ldx, xm, g, b, eps, (T*)Y, ldy, ym, M, C);
  return SDP_CHECK_LAUNCH();
}

extern "C" int sdp_layernorm(int dtype, const void* X, int64_t ldx, int x_grp, int64_t x_gstride, int x_off,
                             const float* gamma, const float* beta, float eps, void* Y, int64_t ldy, int y_grp,
                             int64_t y_gstride, int y_off, int M, int C, void* stream) {
  if (M < 0 || C <= 0 || !X || !Y || !gamma || !beta) return (int)hipErrorInvalidValue;
  if (M == 0) return 0;
  const RowMap xm = mk_rmap(x_grp, x_gstride, x_off), ym = mk_rmap(y_grp, y_gstride, y_off);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == 1) return launch_ln<bf16_t>(X, ldx, xm, gamma, beta, eps, Y, ldy, ym, M, C, s);
  if (dtype == 0) return launch_ln<float>(X, ldx, xm, gamma, beta, eps, Y, ldy, ym, M, C, s);
  return (int)hipErrorInvalidValue;
}

// ---------------------------------------------------------------------------
// q/k head LayerNorm, in place on the fused QKV rows [T, 3C]:
// segment s (0..2H-1) of row t = columns s*hd .. s*hd+hd-1; s <  H -> q_norm,
// s >= H -> k_norm (γ, β shared across heads, layers.py:236-237).
// 16 lanes per segment, 4 segments per wave.
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void qk_headnorm(T* __restrict__ QKV, int64_t ld, int64_t T_rows, int H, int hd,
                                                   const float* __restrict__ gq, const float* __restrict__ bq,
                                                   const float* __restrict__ gk, const float* __restrict__ bk,
                                                   float eps) {
  const int sub = threadIdx.x & 15;
  const int64_t seg = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4);
  const int64_t nseg = T_rows * 2 * H;
  const bool valid = seg < nseg;
  const int64_t t = valid ? seg / (2 * H) : 0;
  const int s = valid ? (int)(seg % (2 * H)) : 0;
  T* p = QKV + t * ld + (int64_t)s * hd;
  const float* g = s < H ? gq : gk;
  const float* b = s < H ? bq : bk;
  float v[8];
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int c = sub + i * 16;
    v[i] = (valid && c < hd) ? to_f<T>(p[c]) : 0.f;
    sum += v[i];
  }
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
  const float mean = sum / (float)hd;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int c = sub + i * 16;
    const float d = (c < hd) ? v[i] - mean : 0.f;
    ss += d * d;
  }
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
  const float rstd = 1.0f / sqrtf(ss / (float)hd + eps);
  if (!valid) return;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int c = sub + i * 16;
    if (c < hd) p[c] = from_f<T>((v[i] - mean) * rstd * g[c] + b[c]);
  }
}

extern "C" int sdp_qk_headnorm(int dtype, void* QKV, int64_t ld, int64_t rows, int n_head, int head_dim,
                               const float* gq, const float* bq, const float* gk, const float* bk, float eps,
                               void* stream) {
  if (!QKV || head_dim <= 0 || head_dim > 128 || n_head <= 0 || rows < 0) return (int)hipErrorInvalidValue;
  if (rows == 0) return 0;
  const int64_t nseg = rows * 2 * n_head;
  dim3 grid((unsigned)((nseg + 15) / 16)), blk(256);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == 1)
    hipLaunchKernelGGL(qk_headnorm<bf16_t>, grid, blk, 0, s, (bf16_t*)QKV, ld, rows, n_head, head_dim, gq, bq, gk, bk, eps);
  else if (dtype == 0)
    hipLaunchKernelGGL(qk_headnorm<float>, grid, blk, 0, s, (float*)QKV, ld, rows, n_head, head_dim, gq, bq, gk, bk, eps);
  else
    return (int)hipErrorInvalidValue;
  return SDP_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------
// Row statistics (mean, rstd) for a LayerNorm applied by the consumer kernel.
// stats[2m] = mean, stats[2m+1] = 1/sqrt(var + eps) of logical row m.
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void rowstats_k(const T* __restrict__ X, int64_t ldx, RowMap xm, float eps,
                                                  float* __restrict__ stats, int M, int C) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const T* xp = X + xm(row) * ldx;
  constexpr int VPL = 8;  // C <= 64 * 4 * 8 = 2048 in registers
  float v[VPL][4];
  float s = 0.f;
  const int nv = C >> 2;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c4 = lane + i * 64;
    if (c4 < nv) {
      if constexpr (sizeof(T) == 2) {
        bf16x4 t = *(const bf16x4*)(xp + c4 * 4);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[i][r] = bf2f((bf16_t)t[r]);
      } else {
        f32x4 t = *(const f32x4*)(xp + c4 * 4);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[i][r] = t[r];
      }
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) v[i][r] = 0.f;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) s += v[i][r];
  }
  const float mean = wave_sum(s) / (float)C;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    if (lane + i * 64 < nv) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float d = v[i][r] - mean;
        ss += d * d;
      }
    }
  }
  const float rstd = 1.0f / sqrtf(wave_sum(ss) / (float)C + eps);
  if (lane == 0) {
    stats[2 * row] = mean;
    stats[2 * row + 1] = rstd;
  }
}

extern "C" int sdp_rowstats(int dtype, const void* X, int64_t ldx, int x_grp, int64_t x_gstride, int x_off, float eps,
                            float* stats, int M, int C, void* stream) {
  if (!X || !stats || M < 0 || C <= 0 || C % 4 || C > 2048 || ldx % 4) return (int)hipErrorInvalidValue;
  if (M == 0) return 0;
  const RowMap xm = mk_rmap(x_grp, x_gstride, x_off);
  hipStream_t s = (hipStream_t)stream;
  dim3 grid((M + 3) / 4), blk(256);
  if (dtype == 1) hipLaunchKernelGGL(rowstats_k<bf16_t>, grid, blk, 0, s, (const bf16_t*)X, ldx, xm, eps, stats, M, C);
  else if (dtype == 0) hipLaunchKernelGGL(rowstats_k<float>, grid, blk, 0, s, (const float*)X, ldx, xm, eps, stats, M, C);
  else return (int)hipErrorInvalidValue;
  return SDP_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------
// LayerNorm statistics by parts.  A token row's LN statistics are carried as
// per-64-column partials {mean, M2} (written by the producing GEMM's whole-line
// epilogue, or by sdp_row_partials), combined exactly (Chan et al. pairwise
// formula) by sdp_ln_stats into (mean, rstd) for the consumer: the LN-folded GEMM
// or the depthwise conv.  Replaces the separate LayerNorm / row-statistics passes
// over the token buffer (layers.py:12-24, :252-253).
//   part[(phys_row * nch + c) * 2 + {0,1}] = {mean, M2} of columns [64c, 64c+64)
//   (the last chunk may be shorter when C % 64 != 0), nch = ceil(C / 64).
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void row_partials_k(const T* __restrict__ X, int64_t ldx, RowMap xm, int M, int C,
                                                      float* __restrict__ part) {
  // 8 lanes per 64-column chunk, 8 columns per lane
  const int64_t g = (int64_t)blockIdx.x * 32 + (threadIdx.x >> 3);  // (row, chunk) index
  const int nch = (C + 63) / 64;
  const int64_t row = g / nch;
  const int c = (int)(g - row * nch);
  const int sub = threadIdx.x & 7;
  const bool ok = row < M;
  const int64_t pr = ok ? xm(row) : 0;
  const int col = c * 64 + sub * 8;
  const int n = min(64, C - c * 64);
  float f[8], sum = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    f[e] = (ok && col + e < C) ? to_f<T>(X[pr * ldx + col + e]) : 0.f;
    sum += f[e];
  }
  sum += __shfl_xor(sum, 1, 64);
  sum += __shfl_xor(sum, 2, 64);
  sum += __shfl_xor(sum, 4, 64);
  const float mean = sum / (float)n;
  float m2 = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e)
    if (col + e < C) m2 = fmaf(f[e] - mean, f[e] - mean, m2);
  m2 += __shfl_xor(m2, 1, 64);
  m2 += __shfl_xor(m2, 2, 64);
  m2 += __shfl_xor(m2, 4, 64);
  if (ok && sub == 0) *(float2*)(part + (pr * nch + c) * 2) = float2{mean, m2};
}

extern "C" int sdp_row_partials(int dtype, const void* X, int64_t ldx, int x_grp, int64_t x_gstride, int x_off, int M,
                                int C, float* part, void* stream) {
  if (!X || !part || M < 0 || C <= 0) return (int)hipErrorInvalidValue;
  if (M == 0) return 0;
  const RowMap xm = mk_rmap(x_grp, x_gstride, x_off);
  const int64_t units = (int64_t)M * ((C + 63) / 64);
  dim3 grid((unsigned)((units + 31) / 32)), blk(256);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == 1) hipLaunchKernelGGL(row_partials_k<bf16_t>, grid, blk, 0, s, (const bf16_t*)X, ldx, xm, M, C, part);
  else if (dtype == 0) hipLaunchKernelGGL(row_partials_k<float>, grid, blk, 0, s, (const float*)X, ldx, xm, M, C, part);
  else return (int)hipErrorInvalidValue;
  return SDP_CHECK_LAUNCH();
}

// one thread per logical row: combine the nch partials of physical row xm(m)
__global__ __launch_bounds__(256) void ln_stats_k(const float* __restrict__ part, RowMap xm, int M, int C, float eps,
                                                  float* __restrict__ stats) {
  const int64_t m = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (m >= M) return;
  const int nch = (C + 63) / 64;
  const float* p = part + xm(m) * nch * 2;
  float na = 0.f, mean = 0.f, m2 = 0.f;
  for (int c = 0; c < nch; ++c) {
    const float2 q = *(const float2*)(p + 2 * c);
    const float nb = (float)min(64, C - c * 64);
    const float n = na + nb;
    const float d = q.x - mean;
    mean = fmaf(d, nb / n, mean);
    m2 += q.y + d * d * (na * nb / n);
    na = n;
  }
  *(float2*)(stats + 2 * m) = float2{mean, rsqrtf(m2 / (float)C + eps)};
}

extern "C" int sdp_ln_stats(const float* part, int x_grp, int64_t x_gstride, int x_off, int M, int C, float eps,
                            float* stats, void* stream) {
  if (SDP_DIAG_SKIP(4)) return 0;  // timing experiment, diagnostic build only (misc.hip)
  if (!part || !stats || M < 0 || C <= 0) return (int)hipErrorInvalidValue;
  if (M == 0) return 0;
  const RowMap xm = mk_rmap(x_grp, x_gstride, x_off);
  hipLaunchKernelGGL(ln_stats_k, dim3((M + 255) / 256), dim3(256), 0, (hipStream_t)stream, part, xm, M, C, eps, stats);
  return SDP_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------
// Depthwise conv, NHWC token rows, with the channel LayerNorm applied on load.
// X: pixel (b, h, w) at physical row xm(b*H*W + h*W + w).  Y: same with ym.
// If stats != null the conv input is LN(x) = (x - mean) * rstd * g + be (the
// ConvMixer's layer_norm_1, layers.py:102 + :20-24); the zero "same" padding is
// applied to that normalised input, as in the reference.
// Block = 32 channels x a band of output rows (+ halo) of one image, 128 threads.
// The band is staged in LDS (storage type T, rows padded with zeros to an odd
// pixel pitch -> conflict-free 8-B reads, no bounds checks in the inner loop);
// thread = 4 channels x a STRIP-pixel output strip: per kernel row it loads the
// STRIP+k-1 window into registers and accumulates STRIP independent outputs.
// ---------------------------------------------------------------------------
constexpr int DW_CB = 32;
constexpr int DW_THREADS = 128;
constexpr int DW_LDS_BYTES = 64 * 1024;       // preferred (several blocks per CU)
constexpr int DW_LDS_MAX = 160 * 1024;        // fallback for wide images

// Row maps used here are dense or group whole images (grp % (H*W) == 0), so the
// physical row of pixel `local` of image b is xm(b*H*W) + local: one map
// evaluation per block instead of a 64-bit division per pixel.
template <typename T, int KS, int STRIP>
__global__ __launch_bounds__(DW_THREADS) void dwconv_ln_nhwc(
    const T* __restrict__ X, int64_t ldx, RowMap xm, const float* __restrict__ stats, const float* __restrict__ lg,
    const float* __restrict__ lb, const float* __restrict__ Wt, const float* __restrict__ bias, T* __restrict__ Y,
    int64_t ldy, RowMap ym, int H, int W, int C, int band, int pitch, int vec_in) {
  constexpr int PAD = KS / 2;
  extern __shared__ __attribute__((aligned(16))) char dsm[];
  T* tile = (T*)dsm;  // [TH][pitch][32]; columns >= W + KS - 1 are zero
  const int b = blockIdx.z;
  const int h0 = blockIdx.y * band;
  const int c0 = blockIdx.x * DW_CB;
  const int hb = min(band, H - h0);
  const int TH = hb + KS - 1;
  float* wts = (float*)(dsm + (((size_t)band + KS - 1) * pitch * DW_CB * sizeof(T) + 15) / 16 * 16);  // [KS*KS][32]
  const int64_t img0 = (int64_t)b * H * W;
  const int64_t xrow0 = xm(img0), yrow0 = ym(img0);
  const int tid = threadIdx.x;

  for (int i = tid; i < KS * KS * DW_CB; i += DW_THREADS) {
    const int tap = i / DW_CB, cc = i % DW_CB;
    wts[i] = (c0 + cc < C) ? Wt[(int64_t)(c0 + cc) * KS * KS + tap] : 0.f;
  }
  // ---- stage LN(x) for the band + halo (zero outside the image / channel range) ----
  constexpr int EPL = 16 / sizeof(T);   // elements per 16-B lane load
  constexpr int LPP = DW_CB / EPL;      // lanes per pixel
  constexpr int SLOTS = DW_THREADS / LPP;
  const int part = tid % LPP, slot = tid / LPP;
  const int c = c0 + part * EPL;
  float g8[EPL], b8[EPL];
#pragma unroll
  for (int e = 0; e < EPL; ++e) {
    g8[e] = (stats && c + e < C) ? lg[c + e] : 1.f;
    b8[e] = (stats && c + e < C) ? lb[c + e] : 0.f;
  }
  // All loads of a batch of 8 items are issued before any is consumed (the loop
  // is HBM-latency-bound otherwise: one dependent round trip per pixel row).
  const int nitems = TH * pitch;  // pixels of the padded band, SLOTS per pass
  const float inv_pitch = 1.0f / (float)pitch;
  constexpr int UNR = 8;
  for (int base = slot; base < nitems; base += SLOTS * UNR) {
    f32x4 raw[UNR];
    float2 st[UNR];
    bool inb[UNR];
    int local[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int pix = base + u * SLOTS;
      const int th = (int)(((float)pix + 0.5f) * inv_pitch);
      const int tw = pix - th * pitch;
      const int h = h0 + th - PAD, w = tw - PAD;
      inb[u] = pix < nitems && h >= 0 && h < H && w >= 0 && w < W;
      local[u] = h * W + w;
      raw[u] = f32x4{0.f, 0.f, 0.f, 0.f};
      st[u] = float2{0.f, 1.f};
      if (inb[u]) {
        const T* src = X + (xrow0 + local[u]) * ldx + c;
        if (vec_in && c + EPL <= C) {
          raw[u] = *(const f32x4*)src;
        } else {
          T* rv = (T*)&raw[u];
#pragma unroll
          for (int e = 0; e < EPL; ++e) rv[e] = (c + e < C) ? src[e] : from_f<T>(0.f);
        }
        if (stats) st[u] = *(const float2*)(stats + 2 * (img0 + local[u]));
      }
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int pix = base + u * SLOTS;
      if (pix >= nitems) break;
      float v[EPL];
      const T* rv = (const T*)&raw[u];
#pragma unroll
      for (int e = 0; e < EPL; ++e) {
        v[e] = inb[u] ? to_f<T>(rv[e]) : 0.f;
        if (stats && inb[u]) v[e] = (v[e] - st[u].x) * st[u].y * g8[e] + b8[e];
        if (c + e >= C) v[e] = 0.f;
      }
      T* dst = tile + (size_t)pix * DW_CB + part * EPL;
      if constexpr (sizeof(T) == 2) {
        bf16x8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = (short)f2bf(v[e]);
        *(bf16x8*)dst = o;
      } else {
        *(f32x4*)dst = f32x4{v[0], v[1], v[2], v[3]};
      }
    }
  }
  __syncthreads();

  const int cq = tid & 7;    // channels 4cq .. 4cq+3 of the block
  const int grp = tid >> 3;  // 16 strip workers
  const int cg = c0 + cq * 4;
  const f32x4 bv = (bias && cg + 3 < C) ? *(const f32x4*)(bias + cg) : f32x4{0.f, 0.f, 0.f, 0.f};
  const int nstrip = (W + STRIP - 1) / STRIP;
  for (int job = grp; job < hb * nstrip; job += DW_THREADS / 8) {
    const int oh = job / nstrip;
    const int w0 = (job - oh * nstrip) * STRIP;
    f32x4 acc[STRIP];
#pragma unroll
    for (int o = 0; o < STRIP; ++o) acc[o] = bv;
    for (int ky = 0; ky < KS; ++ky) {
      const T* trow = tile + ((size_t)(oh + ky) * pitch + w0) * DW_CB + cq * 4;
      f32x4 win[STRIP + KS - 1];
#pragma unroll
      for (int ix = 0; ix < STRIP + KS - 1; ++ix) {
        if constexpr (sizeof(T) == 2) {
          const bf16x4 t = *(const bf16x4*)(trow + ix * DW_CB);
          win[ix] = f32x4{bf2f((bf16_t)t[0]), bf2f((bf16_t)t[1]), bf2f((bf16_t)t[2]), bf2f((bf16_t)t[3])};
        } else {
          win[ix] = *(const f32x4*)(trow + ix * DW_CB);
        }
      }
#pragma unroll
      for (int kx = 0; kx < KS; ++kx) {
        const f32x4 wv = *(const f32x4*)&wts[(ky * KS + kx) * DW_CB + cq * 4];
#pragma unroll
        for (int o = 0; o < STRIP; ++o) acc[o] += win[o + kx] * wv;
      }
    }
    const int gh = h0 + oh;
#pragma unroll
    for (int o = 0; o < STRIP; ++o) {
      const int w = w0 + o;
      if (w < W) {
        T* dst = Y + (yrow0 + (int64_t)gh * W + w) * ldy + cg;
        if (cg + 3 < C) {
          if constexpr (sizeof(T) == 2) {
            bf16x4 t;
#pragma unroll
            for (int r = 0; r < 4; ++r) t[r] = (short)f2bf(acc[o][r]);
            *(bf16x4*)dst = t;
          } else {
            *(f32x4*)dst = acc[o];
          }
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) if (cg + r < C) dst[r] = from_f<T>(acc[o][r]);
        }
      }
    }
  }
}

template <typename T, int KS, int STRIP>
static int launch_dw(const void* X, int64_t ldx, RowMap xm, const float* stats, const float* lg, const float* lb,
                     const float* Wt, const float* bias, void* Y, int64_t ldy, RowMap ym, int B, int H, int W, int C,
                     hipStream_t s) {
  const int nstrip = (W + STRIP - 1) / STRIP;
  const int TWp = nstrip * STRIP + KS - 1;  // widest column a strip window touches
  const int pitch = TWp | 1;                // odd pixel pitch: rows land on different LDS banks
  const size_t row_bytes = (size_t)pitch * DW_CB * sizeof(T);
  const size_t wbytes = (size_t)KS * KS * DW_CB * 4 + 16;
  int band = (int)((DW_LDS_BYTES - wbytes) / row_bytes) - (KS - 1);
  if (band < 1) band = (int)((DW_LDS_MAX - wbytes) / row_bytes) - (KS - 1);
  if (band < 1) return (int)hipErrorInvalidValue;  // image too wide for the LDS band
  band = band > H ? H : band;
  const int nb = (H + band - 1) / band;
  const size_t lds = ((size_t)(band + KS - 1) * row_bytes + 15) / 16 * 16 + (size_t)KS * KS * DW_CB * 4;
  dim3 grid((C + DW_CB - 1) / DW_CB, nb, B);
  const int vec_in = ((ldx * (int64_t)sizeof(T)) % 16 == 0) && ((uintptr_t)X % 16 == 0);
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute((const void*)dwconv_ln_nhwc<T, KS, STRIP>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
  }
  hipLaunchKernelGGL((dwconv_ln_nhwc<T, KS, STRIP>), grid, dim3(DW_THREADS), lds, s, (const T*)X, ldx, xm, stats, lg,
                     lb, Wt, bias, (T*)Y, ldy, ym, H, W, C, band, pitch, vec_in);
  return SDP_CHECK_LAUNCH();
}

template <typename T, int KS>
static int dw_strip(int W, const void* X, int64_t ldx, RowMap xm, const float* stats, const float* lg,
                    const float* lb, const float* Wt, const float* bias, void* Y, int64_t ldy, RowMap ym, int B, int H,
                    int C, hipStream_t s) {
  if (W % 14 == 0)  // SdP-Net-M (14x14): no wasted strip columns
    return launch_dw<T, KS, 14>(X, ldx, xm, stats, lg, lb, Wt, bias, Y, ldy, ym, B, H, W, C, s);
  return launch_dw<T, KS, 16>(X, ldx, xm, stats, lg, lb, Wt, bias, Y, ldy, ym, B, H, W, C, s);
}

template <typename T>
static int dw_dispatch(int k, const void* X, int64_t ldx, RowMap xm, const float* stats, const float* lg,
                       const float* lb, const float* Wt, const float* bias, void* Y, int64_t ldy, RowMap ym, int B,
                       int H, int W, int C, hipStream_t s) {
  switch (k) {
    case 1: return dw_strip<T, 1>(W, X, ldx, xm, stats, lg, lb, Wt, bias, Y, ldy, ym, B, H, C, s);
    case 3: return dw_strip<T, 3>(W, X, ldx, xm, stats, lg, lb, Wt, bias, Y, ldy, ym, B, H, C, s);
    case 5: return dw_strip<T, 5>(W, X, ldx, xm, stats, lg, lb, Wt, bias, Y, ldy, ym, B, H, C, s);
    case 7: return dw_strip<T, 7>(W, X, ldx, xm, stats, lg, lb, Wt, bias, Y, ldy, ym, B, H, C, s);
    case 9: return dw_strip<T, 9>(W, X, ldx, xm, stats, lg, lb, Wt, bias, Y, ldy, ym, B, H, C, s);
    default: return (int)hipErrorInvalidValue;
  }
}

// ---------------------------------------------------------------------------
// dwconv2_nhwc — the default depthwise kernel (C % 8 == 0, image width <= 57).
// Block = 64 channels (one full 128-B bf16 line per pixel) x a band of output
// rows of one image, 256 threads; two blocks per CU (<= 80 KiB LDS each).
//  * The band + halo is staged ONCE as fp32 in LDS (LN applied, zero padding
//    materialised), so the inner loop is ds_read_b128 + packed fp32 FMA only.
//    A pixel is 256 B = all 64 banks: every b128 lane group is conflict-free.
//  * thread = 4 channels x a STRIP of output pixels of one row; per kernel row it
//    reads the STRIP+KS-1 window once and accumulates STRIP outputs.
//  * block order: the bands of one (image, channel group) are consecutive blocks
//    of one XCD, so the halo rows they share are read from HBM once (L2).
// ---------------------------------------------------------------------------
constexpr int DW2_CB = 64;
constexpr int DW2_LDS = 80 * 1024;

template <typename T, int KS, int STRIP>
__global__ __launch_bounds__(256) void dwconv2_nhwc(
    const T* __restrict__ X, int64_t ldx, RowMap xm, const float* __restrict__ stats, const float* __restrict__ lg,
    const float* __restrict__ lb, const float* __restrict__ Wt, const float* __restrict__ bias, T* __restrict__ Y,
    int64_t ldy, RowMap ym, int B, int H, int W, int C, int band, int nband, int ncg, int pitch) {
  constexpr int PAD = KS / 2;
  extern __shared__ __attribute__((aligned(16))) float dsm2[];
  const int TH = band + KS - 1;
  float* tile = dsm2;                              // [TH][pitch][64]
  float* wts = dsm2 + (size_t)TH * pitch * DW2_CB;  // [KS*KS][64]
  // block -> (unit = (image, channel group), band): XCD x takes units x, x+8, ...
  const int bx = blockIdx.x, xcd = bx & 7, k = bx >> 3;
  const int unit = xcd + 8 * (k / nband), bnd = k - (k / nband) * nband;
  if (unit >= B * ncg) return;
  const int b = unit / ncg, cg = unit - b * ncg;
  const int c0 = cg * DW2_CB, h0 = bnd * band;
  const int hb = min(band, H - h0);
  const int tid = threadIdx.x;
  const int64_t img0 = (int64_t)b * H * W;
  const int64_t xrow0 = xm(img0), yrow0 = ym(img0);

  bool wdone = false;
  // ---- stage LN(x) of rows h0-PAD .. h0+hb+PAD-1 as fp32 (8 lanes x 8 channels per pixel) ----
  const int part = tid & 7;
  const int c = c0 + part * 8;
  const bool cok = c < C;  // C % 8 == 0: a part is all in or all out
  float g8[8], b8[8];
  const int npix = (hb + KS - 1) * pitch;
  // all of a thread's pixel loads are issued before any is consumed (one HBM round
  // trip per block: the staging is latency-bound otherwise)
  constexpr int UNR = 10;  // 32 pixels per pass: (7 + 6) x 20 = 260 pixels in one pass
  for (int base = tid >> 3; base < npix; base += 32 * UNR) {
    float v[UNR][8];
    float2 st[UNR];
    bool inb[UNR];
    // unconditional loads from clamped (valid) addresses, masked afterwards: a
    // load under a divergent branch makes hipcc wait for it at the branch join
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int pix = base + 32 * u;
      const int th = pix / pitch, tw = pix - th * pitch;
      const int h = h0 - PAD + th, w = tw - PAD;
      inb[u] = pix < npix && cok && h >= 0 && h < H && w >= 0 && w < W;
      const int hc = min(max(h, 0), H - 1), wc = min(max(w, 0), W - 1);
      const int64_t local = (int64_t)hc * W + wc;
      const T* src = X + (xrow0 + local) * ldx + (cok ? c : c0);
      if constexpr (sizeof(T) == 2) {
        const bf16x8 r = *(const bf16x8*)src;
#pragma unroll
        for (int e = 0; e < 8; ++e) v[u][e] = bf2f((bf16_t)r[e]);
      } else {
        const f32x4 r0 = *(const f32x4*)src, r1 = *(const f32x4*)(src + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[u][e] = r0[e];
          v[u][4 + e] = r1[e];
        }
      }
      st[u] = stats ? *(const float2*)(stats + 2 * (img0 + local)) : float2{0.f, 1.f};
    }
    if (!wdone) {  // weights and LN parameters: loaded behind the pixel loads (one round trip)
      wdone = true;
      for (int i = tid; i < KS * KS * DW2_CB; i += 256) {
        const int tap = i / DW2_CB, cc = i - tap * DW2_CB;
        wts[i] = (c0 + cc < C) ? Wt[(int64_t)(c0 + cc) * KS * KS + tap] : 0.f;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        g8[e] = (stats && cok) ? lg[c + e] : 1.f;
        b8[e] = (stats && cok) ? lb[c + e] : 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int pix = base + 32 * u;
      f32x4 o0, o1;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float a0 = stats ? (v[u][e] - st[u].x) * st[u].y * g8[e] + b8[e] : v[u][e];
        const float a1 = stats ? (v[u][4 + e] - st[u].x) * st[u].y * g8[4 + e] + b8[4 + e] : v[u][4 + e];
        o0[e] = inb[u] ? a0 : 0.f;
        o1[e] = inb[u] ? a1 : 0.f;
      }
      if (pix < npix) {
        float* dst = tile + (size_t)pix * DW2_CB + part * 8;
        *(f32x4*)dst = o0;
        *(f32x4*)(dst + 4) = o1;
      }
    }
  }
  __syncthreads();

  const int q = tid & 15;   // channels c0 + 4q .. +3
  const int cg4 = c0 + q * 4;
  const f32x4 bv = (bias && cg4 < C) ? *(const f32x4*)(bias + cg4) : f32x4{0.f, 0.f, 0.f, 0.f};
  const int nstrip = (W + STRIP - 1) / STRIP;
  for (int job = tid >> 4; job < hb * nstrip; job += 16) {
    const int oh = job / nstrip;
    const int w0 = (job - oh * nstrip) * STRIP;
    f32x4 acc[STRIP];
#pragma unroll
    for (int o = 0; o < STRIP; ++o) acc[o] = bv;
#pragma unroll 1
    for (int ky = 0; ky < KS; ++ky) {
      const float* trow = tile + ((size_t)(oh + ky) * pitch + w0) * DW2_CB + q * 4;
      f32x4 win[STRIP + KS - 1];
#pragma unroll
      for (int ix = 0; ix < STRIP + KS - 1; ++ix) win[ix] = *(const f32x4*)(trow + ix * DW2_CB);
#pragma unroll
      for (int kx = 0; kx < KS; ++kx) {
        const f32x4 wv = *(const f32x4*)&wts[(ky * KS + kx) * DW2_CB + q * 4];
#pragma unroll
        for (int o = 0; o < STRIP; ++o) acc[o] += win[o + kx] * wv;
      }
    }
    if (cg4 < C) {
      const int gh = h0 + oh;
#pragma unroll
      for (int o = 0; o < STRIP; ++o) {
        const int w = w0 + o;
        if (w < W) {
          T* dst = Y + (yrow0 + (int64_t)gh * W + w) * ldy + cg4;
          if constexpr (sizeof(T) == 2) {
            bf16x4 t;
#pragma unroll
            for (int r = 0; r < 4; ++r) t[r] = (short)f2bf(acc[o][r]);
            *(bf16x4*)dst = t;
          } else {
            *(f32x4*)dst = acc[o];
          }
        }
      }
    }
  }
}

template <typename T, int KS, int STRIP>
static int launch_dw2(const void* X, int64_t ldx, RowMap xm, const float* stats, const float* lg, const float* lb,
                      const float* Wt, const float* bias, void* Y, int64_t ldy, RowMap ym, int B, int H, int W, int C,
                      hipStream_t s) {
  const int nstrip = (W + STRIP - 1) / STRIP;
  const int pitch = nstrip * STRIP + KS - 1;
  const size_t row_bytes = (size_t)pitch * DW2_CB * 4;
  const size_t wbytes = (size_t)KS * KS * DW2_CB * 4;
  int maxband = (int)((DW2_LDS - wbytes) / row_bytes) - (KS - 1);
  if (maxband < 1) return -1;  // caller falls back
  const int nband = (H + maxband - 1) / maxband;
  const int band = (H + nband - 1) / nband;
  const size_t lds = (size_t)(band + KS - 1) * row_bytes + wbytes;
  const int ncg = (C + DW2_CB - 1) / DW2_CB;
  const int units = B * ncg;
  const int grid = ((units + 7) / 8) * 8 * nband;
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute((const void*)dwconv2_nhwc<T, KS, STRIP>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
  }
  hipLaunchKernelGGL((dwconv2_nhwc<T, KS, STRIP>), dim3(grid), dim3(256), lds, s, (const T*)X, ldx, xm, stats, lg, lb,
                     Wt, bias, (T*)Y, ldy, ym, B, H, W, C, band, nband, ncg, pitch);
  return SDP_CHECK_LAUNCH();
}

template <typename T>
static int dw2_dispatch(int k, const void* X, int64_t ldx, RowMap xm, const float* stats, const float* lg,
                        const float* lb, const float* Wt, const float* bias, void* Y, int64_t ldy, RowMap ym, int B,
                        int H, int W, int C, hipStream_t s) {
#define SDP_DW2(KS) \
  return (W % 8 == 0) ? launch_dw2<T, KS, 8>(X, ldx, xm, stats, lg, lb, Wt, bias, Y, ldy, ym, B, H, W, C, s) \
                      : launch_dw2<T, KS, 7>(X, ldx, xm, stats, lg, lb, Wt, bias, Y, ldy, ym, B, H, W, C, s)
  switch (k) {
    case 3: SDP_DW2(3);
    case 5: SDP_DW2(5);
    case 7: SDP_DW2(7);
    default: return -1;
  }
#undef SDP_DW2
}

// ---------------------------------------------------------------------------
// dwconv3_mfma — depthwise conv on the matrix cores (bf16, H, W <= 16,
// W + KS - 1 <= 32, C % 32 == 0).  Per (image, channel) the conv is 16x16 D
// tile (rows h, cols w) = sum over ky of A_ky (16 x 32) . B_ky (32 x 16):
//   A_ky[h][q] = LN(x)[h + ky - PAD][q - PAD] (zero padded; q = padded column),
//   B_ky[q][w] = W[c][ky][q - w] for 0 <= q - w < KS, else 0 (a Toeplitz band),
// i.e. KS v_mfma_f32_16x16x32_bf16 per (image, channel).  B depends only on the
// channel: each wave owns 2 channels and keeps their KS B fragments in registers
// for all the images its persistent workgroup walks.
// Workgroup = 32 channels (one 64-B half line per pixel; the other half is the
// neighbouring workgroup on the same XCD, same image order) x a chunk of images,
// 16 waves.  Per image: the 32 channel planes [22 rows][32 cols] bf16 are written
// to LDS transposed from the NHWC rows (LN applied; the zero padding is written
// once), the waves run their MFMAs, the D tiles go through an LDS [pixel][32]
// image back to NHWC 64-B row stores.  The next image's loads are in flight
// (registers) while the current one computes.
// ---------------------------------------------------------------------------
typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
SDP_DEV uint32_t pack_bf16x2(float a, float b) {
  const bf16x2v v = __builtin_convertvector((f32x2){a, b}, bf16x2v);
  return __builtin_bit_cast(uint32_t, v);
}
// plane rows are 48 elements (96 B) apart although only 32 are used: with 64-B rows a
// ds_read_b128 lane group (16 rows of one 16-B chunk) hit every bank twice
// (SQ_LDS_BANK_CONFLICT was 42 % of the kernel's LDS cycles)
constexpr int DW3_CB = 32, DW3_ROWS = 22, DW3_RS = 48;
constexpr int DW3_PLANE = DW3_ROWS * DW3_RS;  // elements per channel plane


template <int KS, int NT, bool LN, int PF>
__global__ __launch_bounds__(NT) void dwconv3_mfma(
    const bf16_t* __restrict__ X, int64_t ldx, RowMap xm, const float* __restrict__ stats,
    const float* __restrict__ lg, const float* __restrict__ lb, const float* __restrict__ Wt,
    const float* __restrict__ bias, bf16_t* __restrict__ Y, int64_t ldy, RowMap ym, int B, int H, int W, int C,
    int ncg, int ipb, int nunits) {
  constexpr int PAD = KS / 2;
  constexpr int CPW = DW3_CB / (NT / 64);  // channels per wave
  constexpr int NIT = 1024 / NT;            // staging items per thread (256 pixels x 4 parts)
  // channel plane cl at cl * DW3_PLANE + 16 * (cl >> 3): the +32 B skew per group of 8
  // puts the 4 planes a staging instruction writes (channels 8q + e) on distinct banks
  __shared__ __attribute__((aligned(16))) bf16_t planes[DW3_CB * DW3_PLANE + 48];  // 67,680 B
  __shared__ __attribute__((aligned(16))) bf16_t outs[256 * DW3_CB];          // [pixel][32]  16,384 B
  __shared__ __attribute__((aligned(16))) float lnp[2 * DW3_CB];              // gamma | beta of the block's channels
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // block -> (unit, half): blocks x and x+8 (same XCD) take the two 32-channel
  // halves of one 64-channel group for the same images
  const int xb = blockIdx.x, xcd = xb & 7, k = xb >> 3;
  const int unit = xcd + 8 * (k >> 1), half = k & 1;
  if (unit >= nunits) return;
  const int cgp = unit % ((ncg + 1) / 2), chunk = unit / ((ncg + 1) / 2);
  const int cg = 2 * cgp + half;
  if (cg >= ncg) return;
  const int c0 = cg * DW3_CB;
  const int b0 = chunk * ipb, b1 = min(B, b0 + ipb);
  if (b0 >= b1) return;
  const int P = H * W;

  // zero the planes once: the padding ring is never written again; the block's
  // weights (bf16, zero-padded rows [KS][32] per channel) go to the outs buffer
  for (int i = tid; i < (DW3_CB * DW3_PLANE + 48) / 8; i += NT) ((bf16x8*)planes)[i] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
  if (LN && tid < 2 * DW3_CB) lnp[tid] = tid < DW3_CB ? lg[c0 + tid] : lb[c0 + tid - DW3_CB];
  bf16_t* wl = outs;  // [32 ch][KS][32], tap kx at column kx + 16
  for (int i = tid; i < DW3_CB * KS * 32; i += NT) {
    const int cl = i / (KS * 32), r = i - cl * KS * 32, ky = r >> 5, col = r & 31;
    const int kx = col - 16;
    wl[i] = (kx >= 0 && kx < KS) ? f2bf(Wt[(int64_t)(c0 + cl) * KS * KS + ky * KS + kx]) : (bf16_t)0;
  }
  __syncthreads();
  // B fragments of this wave's channels: lane (n = lane % 16, j = lane / 16) holds
  // B_ky[8j + i][n] = W[c][ky][8j + i - n], i = 0..7 = row ky of the padded weights
  // from column 8j - n + 16 (2-byte granular: assembled from halfword LDS reads)
  const int n = lane & 15, j = lane >> 4;
  bf16x8 bfr[CPW][KS];
#pragma unroll
  for (int cc = 0; cc < CPW; ++cc) {
    const int cl = CPW * wave + cc;
#pragma unroll
    for (int ky = 0; ky < KS; ++ky) {
      // padded row: tap t at column 16 + t, columns outside [16, 16+KS) hold zeros,
      // so the window 16 + 8j - n + i (in [1, 47]) needs no masking: clamp into the row
      const bf16_t* row = wl + (cl * KS + ky) * 32;
      u32x4 o;
#pragma unroll
      for (int i = 0; i < 8; i += 2) {
        const int c0i = min(16 + 8 * j - n + i, 31), c1i = min(16 + 8 * j - n + i + 1, 31);
        o[i >> 1] = (uint32_t)row[c0i] | ((uint32_t)row[c1i] << 16);
      }
      bfr[cc][ky] = __builtin_bit_cast(bf16x8, o);
      asm volatile("" : "+v"(bfr[cc][ky]));  // build the fragments one at a time
    }
  }
  __syncthreads();  // weights consumed before outs is reused

  // staging role: item t (NIT per thread) -> pixel t / 4 (of up to 256), channels 8 * (t & 3) .. +7.
  // Pixel / plane offsets are image-independent (computed once); a group of the row maps holds whole
  // images (host check), so image b's rows are xm(b P) + pixel: one row-map evaluation per image.
  int pixo[NIT], dsto[NIT], outo[NIT];
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int t = tid + NT * it, pix = t >> 2, q = t & 3;
    const int h = pix / W, w = pix - (pix / W) * W;
    pixo[it] = pix < P ? pix : 0;
    dsto[it] = pix < P ? (8 * q) * DW3_PLANE + 16 * q + (h + PAD) * DW3_RS + (w + PAD) : -1;
    outo[it] = pix * DW3_CB + ((q ^ ((pix >> 2) & 3)) << 3);
  }
  const int q8 = 8 * (tid & 3);  // NT % 4 == 0: the same channel octet for every item
  auto load = [&](int b, int it, bf16x8& v, float2& st) {
    const int64_t r0 = xm((int64_t)b * P);
    v = *(const bf16x8*)(X + (r0 + pixo[it]) * ldx + c0 + q8);
    if constexpr (LN) st = *(const float2*)(stats + 2 * ((int64_t)b * P + pixo[it]));
  };
  auto put = [&](int it, const bf16x8& v, const float2& st) {  // LN + transpose into the planes
    if (dsto[it] < 0) return;
    bf16_t* dst = planes + dsto[it];
    if constexpr (LN) {  // gamma / beta from LDS (a global load here would drain the prefetch ring)
      const f32x4 g0 = *(const f32x4*)(lnp + q8), g1 = *(const f32x4*)(lnp + q8 + 4);
      const f32x4 e0 = *(const f32x4*)(lnp + DW3_CB + q8), e1 = *(const f32x4*)(lnp + DW3_CB + q8 + 4);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float x = (bf2f((bf16_t)v[e]) - st.x) * st.y;
        dst[e * DW3_PLANE] = f2bf(e < 4 ? fmaf(x, g0[e], e0[e]) : fmaf(x, g1[e - 4], e1[e - 4]));
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) dst[e * DW3_PLANE] = (bf16_t)v[e];
    }
  };
  // PF images of loads in flight (HBM latency x bandwidth needs tens of KiB per CU):
  // slot u of the register ring holds image b0 + u (mod PF); the loop is unrolled by
  // PF so the ring index is static
  float bch[CPW];
#pragma unroll
  for (int cc = 0; cc < CPW; ++cc) bch[cc] = bias ? bias[c0 + CPW * wave + cc] : 0.f;
  bf16x8 pv[PF][NIT];
  float2 ps[PF][NIT];
#pragma unroll
  for (int u = 0; u < PF; ++u)
#pragma unroll
    for (int it = 0; it < NIT; ++it) load(min(b0 + u, b1 - 1), it, pv[u][it], ps[u][it]);
#pragma unroll
  for (int it = 0; it < NIT; ++it) put(it, pv[0][it], ps[0][it]);
  for (int bb = b0; bb < b1; bb += PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const int b = bb + u;
      if (b >= b1) break;  // uniform
      __syncthreads();  // planes of image b complete
      // slot u is free (image b is in the planes): refill it with image b + PF
      // (unconditional, clamped to the last image: a static count of loads in flight lets
      //  the compiler wait for exactly the slot it needs)
#pragma unroll
      for (int it = 0; it < NIT; ++it) load(min(b + PF, b1 - 1), it, pv[u][it], ps[u][it]);
#pragma unroll
      for (int pp = 0; pp < CPW / 2; ++pp) {  // channel pairs: one packed dword per output pixel
        f32x4 d[2];
#pragma unroll
        for (int c2 = 0; c2 < 2; ++c2) {
          const int cc = 2 * pp + c2, cl = CPW * wave + cc;
          const bf16_t* pl = planes + (size_t)cl * DW3_PLANE + 16 * (cl >> 3);
          d[c2] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ky = 0; ky < KS; ++ky) {
              const bf16x8 a = *(const bf16x8*)(pl + (n + ky) * DW3_RS + 8 * j);  // A_ky[h = n][8j ..]
              d[c2] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bfr[cc][ky], d[c2], 0, 0, 0);
            }
        }
        // D[h = 4j + i][w = n] -> outs[pixel][32], 16-B chunk c of pixel p at c ^ ((p >> 2) & 3)
        const int cl0 = CPW * wave + 2 * pp;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int h = 4 * j + i;
          if (h < H && n < W) {
            const int p = h * W + n;
            *(uint32_t*)(outs + p * DW3_CB + (((cl0 >> 3) ^ ((p >> 2) & 3)) << 3) + (cl0 & 7)) =
                pack_bf16x2(d[0][i] + bch[2 * pp], d[1][i] + bch[2 * pp + 1]);
          }
        }
        asm volatile("" ::: "memory");  // one channel pair's A fragments live at a time
      }
      __syncthreads();  // outs complete; everyone done reading the planes
      const int64_t yr0 = ym((int64_t)b * P);
#pragma unroll
      for (int it = 0; it < NIT; ++it)
        if (dsto[it] >= 0) *(bf16x8*)(Y + (yr0 + pixo[it]) * ldy + c0 + q8) = *(const bf16x8*)(outs + outo[it]);
      if (b + 1 < b1) {
        const int un = (u + 1) % PF;  // static after unrolling
#pragma unroll
        for (int it = 0; it < NIT; ++it) put(it, pv[un][it], ps[un][it]);
      }
    }
  }
}

static int launch_dw3(int k, const void* X, int64_t ldx, RowMap xm, const float* stats, const float* lg,
                      const float* lb, const float* Wt, const float* bias, void* Y, int64_t ldy, RowMap ym, int B,
                      int H, int W, int C, hipStream_t s) {
  const int ncg = C / DW3_CB;
  int dev = 0, ncu = 256;
  (void)hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0) ncu = 256;
  const int npairs = (ncg + 1) / 2;
  // one workgroup per CU (16 waves at ~122 VGPRs fill a CU): at most ncu workgroups, or
  // the few left over would run as a second round after the rest had finished
  int nchunk = (ncu / 2) / npairs;
  if (nchunk < 1) nchunk = 1;
  if (nchunk > B) nchunk = B;
  const int ipb = (B + nchunk - 1) / nchunk;
  nchunk = (B + ipb - 1) / ipb;
  const int nunits = npairs * nchunk;
  const int grid = ((nunits + 7) / 8) * 16;
#define SDP_DW3(KS, NT, PF)                                                                                    \
  if (stats)                                                                                                        \
    hipLaunchKernelGGL((dwconv3_mfma<KS, NT, true, PF>), dim3(grid), dim3(NT), 0, s, (const bf16_t*)X, ldx, xm,     \
                       stats, lg, lb, Wt, bias, (bf16_t*)Y, ldy, ym, B, H, W, C, ncg, ipb, nunits);                \
  else                                                                                                              \
    hipLaunchKernelGGL((dwconv3_mfma<KS, NT, false, PF>), dim3(grid), dim3(NT), 0, s, (const bf16_t*)X, ldx, xm,    \
                       stats, lg, lb, Wt, bias, (bf16_t*)Y, ldy, ym, B, H, W, C, ncg, ipb, nunits)
  // 16 waves x 2 channels, 2 images in flight (k = 7 at the M shape: 1 / 2 / 3 / 4 images give
  // 53.4 / 51.2-51.5 / 54.4 / 55.2 us alone and M forward 10,212 / 10,255 / 10,213 / 10,201 img/s,
  // interleaved means, tools/r4_pf.sh)
  switch (k) {
    case 3: SDP_DW3(3, 1024, 2); break;
    case 5: SDP_DW3(5, 1024, 2); break;
    case 7: SDP_DW3(7, 1024, 2); break;
    default: return -1;
  }
#undef SDP_DW3
  return SDP_CHECK_LAUNCH();
}

// Highest kernel tier allowed (each tier falls back to the next lower one per shape):
// 3 (default) = dwconv3_mfma where it applies (bf16, H, W <= 16, C % 32 == 0, k in {3,5,7}),
// 2 = dwconv2_nhwc (C % 8 == 0, 16-B rows), 1 = dwconv_ln_nhwc (any shape)
// An unknown tier returns -1 and leaves the selection unchanged (0 queries it).
static int g_dw_kernel = 3;
extern "C" int sdp_dwconv_set_kernel(int k) {
  const int old = g_dw_kernel;
  if (k == 0) return old;
  if (k < 1 || k > 3) return -1;
  g_dw_kernel = k;
  return old;
}

extern "C" int sdp_dwconv(int dtype, const void* X, int64_t ldx, int x_grp, int64_t x_gstride, int x_off,
                          const float* stats, const float* ln_gamma, const float* ln_beta, const float* weight,
                          const float* bias, void* Y, int64_t ldy, int y_grp, int64_t y_gstride, int y_off, int B,
                          int H, int W, int C, int k, void* stream) {
  if (SDP_DIAG_SKIP(1)) return 0;  // timing experiment, diagnostic build only (misc.hip)
  if (!X || !Y || !weight || B < 0 || H <= 0 || W <= 0 || C <= 0) return (int)hipErrorInvalidValue;
  if (stats && (!ln_gamma || !ln_beta)) return (int)hipErrorInvalidValue;
  const int esz = dtype == 1 ? 2 : 4;
  if ((ldy * esz) % 8 || ((uintptr_t)Y % 8) || ((uintptr_t)X % esz)) return (int)hipErrorInvalidValue;
  if (bias && ((uintptr_t)bias % 16)) return (int)hipErrorInvalidValue;
  if (B == 0) return 0;
  // row maps must be dense or group whole images (see dwconv_ln_nhwc)
  if ((x_grp > 0 && x_grp % (H * W)) || (y_grp > 0 && y_grp % (H * W))) return (int)hipErrorInvalidValue;
  const RowMap xm = mk_rmap(x_grp, x_gstride, x_off), ym = mk_rmap(y_grp, y_gstride, y_off);
  hipStream_t s = (hipStream_t)stream;
  const bool v16 = ((ldx * esz) % 16 == 0) && ((uintptr_t)X % 16 == 0) && ((ldy * esz) % 16 == 0) &&
                   ((uintptr_t)Y % 16 == 0) && (!stats || ((uintptr_t)stats % 8 == 0));
  if (g_dw_kernel >= 3 && dtype == 1 && C % 32 == 0 && H <= 16 && W <= 16 && v16 && (k == 3 || k == 5 || k == 7) &&
      ((uintptr_t)weight % 4 == 0)) {
    const int rc = launch_dw3(k, X, ldx, xm, stats, ln_gamma, ln_beta, weight, bias, Y, ldy, ym, B, H, W, C, s);
    if (rc != -1) return rc;
  }
  if (g_dw_kernel >= 2 && C % 8 == 0 && v16 && (k == 3 || k == 5 || k == 7)) {
    const int rc = dtype == 1 ? dw2_dispatch<bf16_t>(k, X, ldx, xm, stats, ln_gamma, ln_beta, weight, bias, Y, ldy, ym, B, H, W, C, s)
                              : dw2_dispatch<float>(k, X, ldx, xm, stats, ln_gamma, ln_beta, weight, bias, Y, ldy, ym, B, H, W, C, s);
    if (rc != -1) return rc;  // -1: image too wide for the dw2 LDS band -> original kernel
  }
  if (dtype == 1) return dw_dispatch<bf16_t>(k, X, ldx, xm, stats, ln_gamma, ln_beta, weight, bias, Y, ldy, ym, B, H, W, C, s);
  if (dtype == 0) return dw_dispatch<float>(k, X, ldx, xm, stats, ln_gamma, ln_beta, weight, bias, Y, ldy, ym, B, H, W, C, s);
  return (int)hipErrorInvalidValue;
}
