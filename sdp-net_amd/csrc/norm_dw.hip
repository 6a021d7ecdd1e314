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
// Depthwise conv, NHWC token rows, with the channel LayerNorm applied on load.
// X: pixel (b, h, w) at physical row xm(b*H*W + h*W + w).  Y: same with ym.
// If stats != null the conv input is LN(x) = (x - mean) * rstd * g + be (the
// ConvMixer's layer_norm_1, layers.py:102 + :20-24); the zero "same" padding is
// applied to that normalised input, as in the reference.
// Block = 32 channels x a band of output rows (+ halo) of one image, 128 threads.
// The band is staged in LDS (storage type T, rows padded to an odd pixel pitch
// -> conflict-free 8/16-B reads); thread = 4 channels x a 16-pixel output strip,
// sliding the k-wide window along the row with the k*k taps read from LDS.
// ---------------------------------------------------------------------------
constexpr int DW_CB = 32;
constexpr int DW_STRIP = 16;
constexpr int DW_THREADS = 128;
constexpr int DW_LDS_BYTES = 64 * 1024;

template <typename T, int KS>
__global__ __launch_bounds__(DW_THREADS) void dwconv_ln_nhwc(
    const T* __restrict__ X, int64_t ldx, RowMap xm, const float* __restrict__ stats, const float* __restrict__ lg,
    const float* __restrict__ lb, const float* __restrict__ Wt, const float* __restrict__ bias, T* __restrict__ Y,
    int64_t ldy, RowMap ym, int H, int W, int C, int band, int pitch, int vec_in) {
  constexpr int PAD = KS / 2;
  extern __shared__ __attribute__((aligned(16))) char dsm[];
  T* tile = (T*)dsm;                                                         // [TH][pitch][32]
  const int b = blockIdx.z;
  const int h0 = blockIdx.y * band;
  const int c0 = blockIdx.x * DW_CB;
  const int hb = min(band, H - h0);
  const int TH = hb + KS - 1, TW = W + KS - 1;
  float* wts = (float*)(dsm + (((size_t)band + KS - 1) * pitch * DW_CB * sizeof(T) + 15) / 16 * 16);  // [KS*KS][32]
  const int64_t img0 = (int64_t)b * H * W;
  const int tid = threadIdx.x;

  for (int i = tid; i < KS * KS * DW_CB; i += DW_THREADS) {
    const int tap = i / DW_CB, cc = i % DW_CB;
    wts[i] = (c0 + cc < C) ? Wt[(int64_t)(c0 + cc) * KS * KS + tap] : 0.f;
  }
  // ---- stage LN(x) for the band + halo ----
  constexpr int EPL = 16 / sizeof(T);   // elements per 16-B lane load
  constexpr int LPP = DW_CB / EPL;      // lanes per pixel
  for (int idx = tid; idx < TH * TW * LPP; idx += DW_THREADS) {
    const int pix = idx / LPP, part = idx % LPP;
    const int th = pix / TW, tw = pix % TW;
    const int h = h0 + th - PAD, w = tw - PAD;
    const int c = c0 + part * EPL;
    float v[EPL];
#pragma unroll
    for (int e = 0; e < EPL; ++e) v[e] = 0.f;
    if (h >= 0 && h < H && w >= 0 && w < W) {
      const int64_t m = img0 + (int64_t)h * W + w;
      const T* src = X + xm(m) * ldx + c;
      if (vec_in && c + EPL <= C) {
        const f32x4 raw = *(const f32x4*)src;
        const T* rv = (const T*)&raw;
#pragma unroll
        for (int e = 0; e < EPL; ++e) v[e] = to_f<T>(rv[e]);
      } else {
#pragma unroll
        for (int e = 0; e < EPL; ++e) if (c + e < C) v[e] = to_f<T>(src[e]);
      }
      if (stats) {
        const float mean = stats[2 * m], rstd = stats[2 * m + 1];
#pragma unroll
        for (int e = 0; e < EPL; ++e)
          if (c + e < C) v[e] = (v[e] - mean) * rstd * lg[c + e] + lb[c + e];
      }
    }
    T* dst = tile + ((size_t)th * pitch + tw) * DW_CB + part * EPL;
    if constexpr (sizeof(T) == 2) {
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (short)f2bf(v[e]);
      *(bf16x8*)dst = o;
    } else {
      *(f32x4*)dst = f32x4{v[0], v[1], v[2], v[3]};
    }
  }
  __syncthreads();

  const int cq = tid & 7;          // channels 4cq .. 4cq+3 of the block
  const int grp = tid >> 3;        // 16 strip workers
  const int cg = c0 + cq * 4;
  const f32x4 bv = (bias && cg + 3 < C) ? *(const f32x4*)(bias + cg) : f32x4{0.f, 0.f, 0.f, 0.f};
  const int nstrip = (W + DW_STRIP - 1) / DW_STRIP;
  for (int job = grp; job < hb * nstrip; job += DW_THREADS / 8) {
    const int oh = job / nstrip;
    const int w0 = (job % nstrip) * DW_STRIP;
    f32x4 acc[DW_STRIP];
#pragma unroll
    for (int o = 0; o < DW_STRIP; ++o) acc[o] = bv;
    for (int ky = 0; ky < KS; ++ky) {
      f32x4 wk[KS];
#pragma unroll
      for (int kx = 0; kx < KS; ++kx) wk[kx] = *(const f32x4*)&wts[(ky * KS + kx) * DW_CB + cq * 4];
      const T* trow = tile + ((size_t)(oh + ky) * pitch + w0) * DW_CB + cq * 4;
#pragma unroll
      for (int ix = 0; ix < DW_STRIP + KS - 1; ++ix) {
        f32x4 v;
        if (w0 + ix < TW) {
          if constexpr (sizeof(T) == 2) {
            const bf16x4 t = *(const bf16x4*)(trow + ix * DW_CB);
            v = f32x4{bf2f((bf16_t)t[0]), bf2f((bf16_t)t[1]), bf2f((bf16_t)t[2]), bf2f((bf16_t)t[3])};
          } else {
            v = *(const f32x4*)(trow + ix * DW_CB);
          }
        } else {
          v = f32x4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int kx = 0; kx < KS; ++kx) {
          const int o = ix - kx;
          if (o >= 0 && o < DW_STRIP) {
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[o][r] = fmaf(v[r], wk[kx][r], acc[o][r]);
          }
        }
      }
    }
    const int gh = h0 + oh;
#pragma unroll
    for (int o = 0; o < DW_STRIP; ++o) {
      const int w = w0 + o;
      if (w < W) {
        T* dst = Y + ym(img0 + (int64_t)gh * W + w) * ldy + cg;
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

template <typename T, int KS>
static int launch_dw(const void* X, int64_t ldx, RowMap xm, const float* stats, const float* lg, const float* lb,
                     const float* Wt, const float* bias, void* Y, int64_t ldy, RowMap ym, int B, int H, int W, int C,
                     hipStream_t s) {
  const int TW = W + KS - 1;
  const int pitch = TW | 1;  // odd pixel pitch: rows land on different LDS banks
  const size_t row_bytes = (size_t)pitch * DW_CB * sizeof(T);
  const size_t wbytes = (size_t)KS * KS * DW_CB * 4 + 16;
  int band = (int)((DW_LDS_BYTES - wbytes) / row_bytes) - (KS - 1);
  if (band < 1) return (int)hipErrorInvalidValue;  // image too wide for the LDS band
  band = band > H ? H : band;
  const int nb = (H + band - 1) / band;
  const size_t lds = ((size_t)(band + KS - 1) * row_bytes + 15) / 16 * 16 + (size_t)KS * KS * DW_CB * 4;
  dim3 grid((C + DW_CB - 1) / DW_CB, nb, B);
  const int vec_in = ((ldx * (int64_t)sizeof(T)) % 16 == 0) && ((uintptr_t)X % 16 == 0);
  hipLaunchKernelGGL((dwconv_ln_nhwc<T, KS>), grid, dim3(DW_THREADS), lds, s, (const T*)X, ldx, xm, stats, lg, lb,
                     Wt, bias, (T*)Y, ldy, ym, H, W, C, band, pitch, vec_in);
  return SDP_CHECK_LAUNCH();
}

template <typename T>
static int dw_dispatch(int k, const void* X, int64_t ldx, RowMap xm, const float* stats, const float* lg,
                       const float* lb, const float* Wt, const float* bias, void* Y, int64_t ldy, RowMap ym, int B,
                       int H, int W, int C, hipStream_t s) {
  switch (k) {
    case 1: return launch_dw<T, 1>(X, ldx, xm, stats, lg, lb, Wt, bias, Y, ldy, ym, B, H, W, C, s);
    case 3: return launch_dw<T, 3>(X, ldx, xm, stats, lg, lb, Wt, bias, Y, ldy, ym, B, H, W, C, s);
    case 5: return launch_dw<T, 5>(X, ldx, xm, stats, lg, lb, Wt, bias, Y, ldy, ym, B, H, W, C, s);
    case 7: return launch_dw<T, 7>(X, ldx, xm, stats, lg, lb, Wt, bias, Y, ldy, ym, B, H, W, C, s);
    case 9: return launch_dw<T, 9>(X, ldx, xm, stats, lg, lb, Wt, bias, Y, ldy, ym, B, H, W, C, s);
    default: return (int)hipErrorInvalidValue;
  }
}

extern "C" int sdp_dwconv(int dtype, const void* X, int64_t ldx, int x_grp, int64_t x_gstride, int x_off,
                          const float* stats, const float* ln_gamma, const float* ln_beta, const float* weight,
                          const float* bias, void* Y, int64_t ldy, int y_grp, int64_t y_gstride, int y_off, int B,
                          int H, int W, int C, int k, void* stream) {
  if (!X || !Y || !weight || B < 0 || H <= 0 || W <= 0 || C <= 0) return (int)hipErrorInvalidValue;
  if (stats && (!ln_gamma || !ln_beta)) return (int)hipErrorInvalidValue;
  const int esz = dtype == 1 ? 2 : 4;
  if ((ldy * esz) % 8 || ((uintptr_t)Y % 8) || ((uintptr_t)X % esz)) return (int)hipErrorInvalidValue;
  if (bias && ((uintptr_t)bias % 16)) return (int)hipErrorInvalidValue;
  if (B == 0) return 0;
  const RowMap xm = mk_rmap(x_grp, x_gstride, x_off), ym = mk_rmap(y_grp, y_gstride, y_off);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == 1) return dw_dispatch<bf16_t>(k, X, ldx, xm, stats, ln_gamma, ln_beta, weight, bias, Y, ldy, ym, B, H, W, C, s);
  if (dtype == 0) return dw_dispatch<float>(k, X, ldx, xm, stats, ln_gamma, ln_beta, weight, bias, Y, ldy, ym, B, H, W, C, s);
  return (int)hipErrorInvalidValue;
}
