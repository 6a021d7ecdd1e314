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
//  * sdp_dwconv — depthwise conv (layers.py:73-78: groups=C, padding="same",
//    zeros, optional bias) on image rows of a token-major buffer.  One block =
//    one image x row band x 128 B of channels; the band + halo is staged in LDS
//    (zero-filled border), each thread owns one channel and slides a k-wide
//    window along 16-pixel output strips with its k*k taps in registers.
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
// Depthwise conv, NHWC token rows.
// X: image pixel (b, h, w) at physical row xm(b*H*W + h*W + w) (stride ldx)
// Y: same with ym.  Weight fp32 [C][k][k], bias fp32 [C] or null.
// ---------------------------------------------------------------------------
constexpr int DW_STRIP = 16;   // output pixels per sliding window
constexpr int DW_LDS_BYTES = 64 * 1024;

template <typename T, int KS>
__global__ __launch_bounds__(256) void dwconv_nhwc(const T* __restrict__ X, int64_t ldx, RowMap xm,
                                                   const float* __restrict__ Wt, const float* __restrict__ bias,
                                                   T* __restrict__ Y, int64_t ldy, RowMap ym, int H, int W, int C,
                                                   int band) {
  constexpr int CB = 128 / sizeof(T);  // channels per block (128 B per pixel)
  constexpr int PADK = KS / 2;
  extern __shared__ __attribute__((aligned(16))) char dsm[];
  T* tile = (T*)dsm;  // [(band+KS-1)][(W+KS-1)][CB]

  const int b = blockIdx.z;
  const int h0 = blockIdx.y * band;
  const int c0 = blockIdx.x * CB;
  const int hb = min(band, H - h0);
  const int TH = hb + KS - 1, TW = W + KS - 1;
  const int64_t img0 = (int64_t)b * H * W;

  // stage band + halo: 8 lanes x 16 B per pixel
  constexpr int LPP = 8;                // lanes per pixel
  constexpr int EPL = 16 / sizeof(T);   // elements per lane
  const int npix = TH * TW;
  for (int idx = threadIdx.x; idx < npix * LPP; idx += 256) {
    const int pix = idx / LPP, part = idx % LPP;
    const int th = pix / TW, tw = pix % TW;
    const int h = h0 + th - PADK, w = tw - PADK;
    const int c = c0 + part * EPL;
    T* dst = tile + (int64_t)pix * CB + part * EPL;
    if (h >= 0 && h < H && w >= 0 && w < W && c + EPL <= C) {
      const T* src = X + xm(img0 + (int64_t)h * W + w) * ldx + c;
      *(f32x4*)dst = *(const f32x4*)src;
    } else {
#pragma unroll
      for (int e = 0; e < EPL; ++e) {
        const bool ok = (h >= 0 && h < H && w >= 0 && w < W && c + e < C);
        dst[e] = ok ? X[xm(img0 + (int64_t)h * W + w) * ldx + c + e] : from_f<T>(0.f);
      }
    }
  }
  __syncthreads();

  const int cl = threadIdx.x % CB;
  const int grp = threadIdx.x / CB;
  constexpr int NGRP = 256 / CB;
  const int c = c0 + cl;
  if (c >= C) return;
  float wk[KS * KS];
#pragma unroll
  for (int i = 0; i < KS * KS; ++i) wk[i] = Wt[(int64_t)c * KS * KS + i];
  const float bv = bias ? bias[c] : 0.f;

  const int nstrip = (W + DW_STRIP - 1) / DW_STRIP;
  for (int job = grp; job < hb * nstrip; job += NGRP) {
    const int oh = job / nstrip;
    const int w0 = (job % nstrip) * DW_STRIP;
    float acc[DW_STRIP];
#pragma unroll
    for (int i = 0; i < DW_STRIP; ++i) acc[i] = bv;
#pragma unroll
    for (int ky = 0; ky < KS; ++ky) {
      const T* trow = tile + ((int64_t)(oh + ky) * TW + w0) * CB + cl;
      float win[DW_STRIP + KS - 1];
#pragma unroll
      for (int i = 0; i < DW_STRIP + KS - 1; ++i)
        win[i] = (w0 + i < TW) ? to_f<T>(trow[i * CB]) : 0.f;
#pragma unroll
      for (int kx = 0; kx < KS; ++kx) {
        const float wv = wk[ky * KS + kx];
#pragma unroll
        for (int i = 0; i < DW_STRIP; ++i) acc[i] = fmaf(win[i + kx], wv, acc[i]);
      }
    }
    const int gh = h0 + oh;
#pragma unroll
    for (int i = 0; i < DW_STRIP; ++i) {
      const int w = w0 + i;
      if (w < W) Y[ym(img0 + (int64_t)gh * W + w) * ldy + c] = from_f<T>(acc[i]);
    }
  }
}

template <typename T, int KS>
static int launch_dw(const void* X, int64_t ldx, RowMap xm, const float* Wt, const float* bias, void* Y,
                     int64_t ldy, RowMap ym, int B, int H, int W, int C, hipStream_t s) {
  constexpr int CB = 128 / sizeof(T);
  const int TW = W + KS - 1;
  int band = DW_LDS_BYTES / (TW * 128) - (KS - 1);
  if (band < 1) return (int)hipErrorInvalidValue;  // image too wide for the LDS band
  band = band > H ? H : band;
  const int nb = (H + band - 1) / band;
  const size_t lds = (size_t)(band + KS - 1) * TW * 128;
  dim3 grid((C + CB - 1) / CB, nb, B);
  hipLaunchKernelGGL((dwconv_nhwc<T, KS>), grid, dim3(256), lds, s, (const T*)X, ldx, xm, Wt, bias, (T*)Y, ldy,
                     ym, H, W, C, band);
  return SDP_CHECK_LAUNCH();
}

template <typename T>
static int dw_dispatch(int k, const void* X, int64_t ldx, RowMap xm, const float* Wt, const float* bias, void* Y,
                       int64_t ldy, RowMap ym, int B, int H, int W, int C, hipStream_t s) {
  switch (k) {
    case 1: return launch_dw<T, 1>(X, ldx, xm, Wt, bias, Y, ldy, ym, B, H, W, C, s);
    case 3: return launch_dw<T, 3>(X, ldx, xm, Wt, bias, Y, ldy, ym, B, H, W, C, s);
    case 5: return launch_dw<T, 5>(X, ldx, xm, Wt, bias, Y, ldy, ym, B, H, W, C, s);
    case 7: return launch_dw<T, 7>(X, ldx, xm, Wt, bias, Y, ldy, ym, B, H, W, C, s);
    case 9: return launch_dw<T, 9>(X, ldx, xm, Wt, bias, Y, ldy, ym, B, H, W, C, s);
    default: return (int)hipErrorInvalidValue;
  }
}

extern "C" int sdp_dwconv(int dtype, const void* X, int64_t ldx, int x_grp, int64_t x_gstride, int x_off,
                          const float* weight, const float* bias, void* Y, int64_t ldy, int y_grp,
                          int64_t y_gstride, int y_off, int B, int H, int W, int C, int k, void* stream) {
  if (!X || !Y || !weight || B < 0 || H <= 0 || W <= 0 || C <= 0) return (int)hipErrorInvalidValue;
  if ((ldx * (dtype == 1 ? 2 : 4)) % 16 || ((uintptr_t)X % 16)) return (int)hipErrorInvalidValue;
  if (B == 0) return 0;
  const RowMap xm = mk_rmap(x_grp, x_gstride, x_off), ym = mk_rmap(y_grp, y_gstride, y_off);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == 1) return dw_dispatch<bf16_t>(k, X, ldx, xm, weight, bias, Y, ldy, ym, B, H, W, C, s);
  if (dtype == 0) return dw_dispatch<float>(k, X, ldx, xm, weight, bias, Y, ldy, ym, B, H, W, C, s);
  return (int)hipErrorInvalidValue;
}
