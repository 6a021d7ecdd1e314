// Kernels on either side of the forward path for evaluation.
//
//  * sdp_val_preprocess — the reference's validation transform (hf_dataset_generator.py:27-41,
//    model_test.py:50-52): RGB -> Resize((RH, RW), BICUBIC) -> CenterCrop((CH, CW)) ->
//    ToDtype(float32, scale=True) -> Normalize(mean, std), on a batch of decoded uint8 HWC
//    images of different sizes, straight into the model's NCHW input.  The resize is
//    Pillow's 8-bit two-pass separable convolution (the PIL path torchvision takes for
//    PIL images; Pillow 12.2.0 libImaging/Resample.c): a Keys cubic with a = -0.5,
//    support 2 x max(scale, 1), double-precision taps normalised to 22-bit fixed point,
//    int32 accumulation from 1 << 21, clamp(v >> 22, 0, 255) after each pass, the
//    horizontal pass first, a pass skipped when its axis keeps its size.  Only the
//    cropped window is produced (each output pixel depends on its own taps only, so the
//    crop commutes with the resize bit for bit).
//  * sdp_logits_metrics — per-row cross-entropy, BCE-with-logits against the smoothed
//    one-hot target and top-1 hit (model_test.py:69-82, training_utilities.py:95-107).
#include "common.h"

namespace pre {
constexpr int PREC = 22;  // Pillow PRECISION_BITS = 32 - 8 - 2

// Pillow's coefficient arithmetic is plain IEEE double; the pragmas keep the compiler
// from contracting it into FMAs so the taps round exactly as on the host.
__device__ double bicubic(double x) {
#pragma clang fp contract(off)
  const double a = -0.5;
  if (x < 0.0) x = -x;
  if (x < 1.0) return ((a + 2.0) * x - (a + 3.0)) * x * x + 1;
  if (x < 2.0) return (((x - 5) * x + 8) * x - 4) * a;
  return 0.0;
}

// Workspace per image: for the CW cropped output columns then the CH cropped output
// rows: bounds {first tap, tap count} and KMAX fixed-point taps, tap-major so that the
// lanes of a wave (consecutive output columns) read one tap with one coalesced load.
struct Tab {
  int* bounds;  // [B][CW + CH][2]
  int* coef;    // [B][KMAX][CW + CH]
};
SDP_DEV int64_t tap_at(int b, int x, int t, int CW, int CH, int KMAX) {
  return ((int64_t)b * KMAX + x) * (CW + CH) + t;
}

__global__ void coef_k(const int* __restrict__ hw, int B, int RH, int RW, int top, int left, int CH, int CW, int KMAX,
                       Tab tab) {
#pragma clang fp contract(off)
  const int b = blockIdx.y;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= CW + CH) return;
  const bool horiz = t < CW;
  const int inSize = horiz ? hw[2 * b + 1] : hw[2 * b];
  const int outSize = horiz ? RW : RH;
  const int xx = horiz ? left + t : top + (t - CW);
  // precompute_coeffs(inSize, 0, inSize, outSize, bicubic)
  double filterscale, scale;
  filterscale = scale = (double)inSize / outSize;
  if (filterscale < 1.0) filterscale = 1.0;
  const double support = 2.0 * filterscale;
  const double center = (xx + 0.5) * scale;
  const double ss = 1.0 / filterscale;
  int xmin = (int)(center - support + 0.5);
  if (xmin < 0) xmin = 0;
  int xmax = (int)(center + support + 0.5);
  if (xmax > inSize) xmax = inSize;
  xmax -= xmin;
  if (xmax > KMAX) xmax = KMAX;  // host sizes KMAX to the largest ksize: never taken
  const int n = xmax;
  double ww = 0.0;
  for (int x = 0; x < n; ++x) ww += bicubic((x + xmin - center + 0.5) * ss);
  for (int x = 0; x < n; ++x) {  // the same taps again (deterministic), normalised
    double v = bicubic((x + xmin - center + 0.5) * ss);
    if (ww != 0.0) v /= ww;
    // normalize_coeffs_8bpc
    tab.coef[tap_at(b, x, t, CW, CH, KMAX)] = v < 0 ? (int)(-0.5 + v * (1 << PREC)) : (int)(0.5 + v * (1 << PREC));
  }
  for (int x = n; x < KMAX; ++x) tab.coef[tap_at(b, x, t, CW, CH, KMAX)] = 0;
  int* bd = tab.bounds + ((int64_t)b * (CW + CH) + t) * 2;
  bd[0] = xmin;
  bd[1] = n;
}

SDP_DEV uint8_t clip8(int v) {
  v >>= PREC;
  return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

// Source rows the vertical pass reads for the cropped rows.
SDP_DEV void rows_needed(const Tab& tab, int b, int CH, int CW, bool need_v, int top, int& y0, int& y1) {
  if (!need_v) {
    y0 = top;
    y1 = top + CH;
    return;
  }
  const int* bd = tab.bounds + (int64_t)b * (CW + CH) * 2;
  y0 = bd[2 * CW];
  y1 = bd[2 * (CW + CH - 1)] + bd[2 * (CW + CH - 1) + 1];
}

// Horizontal pass over the needed source rows, cropped columns only.  Each wave owns
// one source row at a time: it stages the packed RGB row into its private LDS slot as
// RGBX words (coalesced byte loads, ds_write_b8 into the padded slot; no workgroup
// barrier, a wave's LDS accesses execute in order), then every output column reads
// its taps as one 32-bit word each.  Output: tmp[b][y][j] RGBX uint32 (row stride CW
// words, image stride tmp_stride bytes).
__global__ __launch_bounds__(256) void hpass_k(const uint8_t* __restrict__ pix, const int64_t* __restrict__ offs,
                                               const int* __restrict__ hw, int RH, int RW, int top, int left, int CH,
                                               int CW, int KMAX, Tab tab, uint8_t* __restrict__ tmp,
                                               int64_t tmp_stride, int max_w) {
  extern __shared__ uint32_t lds_rows[];  // [waves][max_w] RGBX
  const int b = blockIdx.y;
  const int H = hw[2 * b], W = hw[2 * b + 1];
  const bool need_h = W != RW, need_v = H != RH;
  int y0, y1;
  rows_needed(tab, b, CH, CW, need_v, top, y0, y1);
  const uint8_t* img = pix + offs[b];
  uint32_t* out = (uint32_t*)(tmp + (int64_t)b * tmp_stride);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  uint32_t* srow = lds_rows + (int64_t)wave * max_w;
  for (int y = y0 + blockIdx.x * nw + wave; y < y1; y += gridDim.x * nw) {
    const uint8_t* row = img + (int64_t)y * W * 3;
    __builtin_amdgcn_wave_barrier();  // previous row's tap reads precede the overwrite
    for (int i = lane; i < W * 3; i += 64) ((uint8_t*)srow)[(i / 3) * 4 + (i % 3)] = row[i];
    __builtin_amdgcn_wave_barrier();
    for (int j = lane; j < CW; j += 64) {
      uint32_t o;
      if (!need_h) {
        o = srow[left + j] & 0x00ffffffu;
      } else {
        const int* bd = tab.bounds + ((int64_t)b * (CW + CH) + j) * 2;
        const int* k = tab.coef + tap_at(b, 0, j, CW, CH, KMAX);
        const int xmin = bd[0], n = bd[1];
        int s0 = 1 << (PREC - 1), s1 = s0, s2 = s0;
        for (int x = 0; x < n; ++x) {
          const int w = k[(int64_t)x * (CW + CH)];
          const uint32_t px = srow[xmin + x];
          s0 += (int)(px & 0xff) * w;
          s1 += (int)((px >> 8) & 0xff) * w;
          s2 += (int)((px >> 16) & 0xff) * w;
        }
        o = (uint32_t)clip8(s0) | ((uint32_t)clip8(s1) << 8) | ((uint32_t)clip8(s2) << 16);
      }
      out[(int64_t)y * CW + j] = o;
    }
  }
}

struct Norm {
  float mean[3], std[3];
};

// Vertical pass over the cropped rows + ToDtype(scale) + Normalize into NCHW.
template <typename TO>
__global__ void vpass_k(const int* __restrict__ hw, int RH, int top, int CH, int CW, int KMAX, Tab tab,
                        const uint8_t* __restrict__ tmp, int64_t tmp_stride, Norm nm, TO* __restrict__ out,
                        uint8_t* __restrict__ out_u8) {
  const int b = blockIdx.y;
  const int H = hw[2 * b];
  const bool need_v = H != RH;
  const uint32_t* src = (const uint32_t*)(tmp + (int64_t)b * tmp_stride);
  const int64_t total = (int64_t)CH * CW;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int i = (int)(idx / CW), j = (int)(idx % CW);
    uint8_t u[3];
    if (!need_v) {
      const uint32_t px = src[(int64_t)(top + i) * CW + j];
      u[0] = px & 0xff;
      u[1] = (px >> 8) & 0xff;
      u[2] = (px >> 16) & 0xff;
    } else {
      const int* bd = tab.bounds + ((int64_t)b * (CW + CH) + CW + i) * 2;
      const int* k = tab.coef + tap_at(b, 0, CW + i, CW, CH, KMAX);
      const int ymin = bd[0], n = bd[1];
      int s0 = 1 << (PREC - 1), s1 = s0, s2 = s0;
      const uint32_t* p = src + (int64_t)ymin * CW + j;
      for (int y = 0; y < n; ++y) {
        const int w = k[(int64_t)y * (CW + CH)];
        const uint32_t px = p[(int64_t)y * CW];
        s0 += (int)(px & 0xff) * w;
        s1 += (int)((px >> 8) & 0xff) * w;
        s2 += (int)((px >> 16) & 0xff) * w;
      }
      u[0] = clip8(s0);
      u[1] = clip8(s1);
      u[2] = clip8(s2);
    }
    if (out_u8) {
      uint8_t* o = out_u8 + (((int64_t)b * CH + i) * CW + j) * 3;
      o[0] = u[0];
      o[1] = u[1];
      o[2] = u[2];
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float v = ((float)u[c] / 255.0f - nm.mean[c]) / nm.std[c];
      out[(((int64_t)b * 3 + c) * CH + i) * CW + j] = from_f<TO>(v);
    }
  }
}
}  // namespace pre

extern "C" int sdp_val_preprocess(const uint8_t* pix, const int64_t* offs, const int* hw, int B, int RH, int RW,
                                  int top, int left, int CH, int CW, int KMAX, const float* mean3, const float* std3,
                                  void* ws, uint8_t* tmp, int64_t tmp_stride, int max_w, int dtype_out,
                                  void* out, uint8_t* out_u8, void* stream) {
  if (B < 0 || RH <= 0 || RW <= 0 || CH <= 0 || CW <= 0 || top < 0 || left < 0 || top + CH > RH ||
      left + CW > RW || KMAX <= 0 || KMAX > 160 || !mean3 || !std3 || max_w <= 0 || max_w > 40960)
    return (int)hipErrorInvalidValue;
  if (B == 0) return 0;
  if (!pix || !offs || !hw || !ws || !tmp || !out) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  pre::Tab tab{(int*)ws, (int*)ws + (int64_t)B * (CW + CH) * 2};
  pre::Norm nm;
  for (int c = 0; c < 3; ++c) {
    nm.mean[c] = mean3[c];
    nm.std[c] = std3[c];
  }
  hipLaunchKernelGGL(pre::coef_k, dim3((CW + CH + 63) / 64, B), dim3(64), 0, s, hw, B, RH, RW, top, left, CH, CW,
                     KMAX, tab);
  // one RGBX source row per wave in LDS: 4 waves per block while they fit in 64 KiB
  int nw = 4;
  while (nw > 1 && (size_t)nw * max_w * 4 > 65536) nw >>= 1;
  const size_t lds = (size_t)nw * max_w * 4;
  if (lds > 65536) {
    static bool raised = false;
    if (!raised) {
      (void)hipFuncSetAttribute((const void*)pre::hpass_k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      raised = true;
    }
  }
  hipLaunchKernelGGL(pre::hpass_k, dim3(64, B), dim3(64 * nw), lds, s, pix, offs, hw, RH, RW, top, left, CH, CW,
                     KMAX, tab, tmp, tmp_stride, max_w);
  if (dtype_out == 0)
    hipLaunchKernelGGL(pre::vpass_k<float>, dim3(64, B), dim3(256), 0, s, hw, RH, top, CH, CW, KMAX, tab,
                       (const uint8_t*)tmp, tmp_stride, nm, (float*)out, out_u8);
  else if (dtype_out == 1)
    hipLaunchKernelGGL(pre::vpass_k<bf16_t>, dim3(64, B), dim3(256), 0, s, hw, RH, top, CH, CW, KMAX, tab,
                       (const uint8_t*)tmp, tmp_stride, nm, (bf16_t*)out, out_u8);
  else
    return (int)hipErrorInvalidValue;
  return SDP_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------
// Per-row evaluation metrics on logits [B][C] (row stride ld), one wave per row:
//   out[3b+0] = logsumexp(x) - x[label]                      (nn.CrossEntropyLoss, per row)
//   out[3b+1] = sum_j bce(x_j, t_j), t = onehot(1-ls) + ls/C  (BCEWithLogitsLoss, row sum)
//   out[3b+2] = 1 if argmax(x) == label (first maximal index) else 0
// bce(x, t) = (1 - t) x + m + log(exp(-m) + exp(-x - m)), m = max(-x, 0) (ATen's form).
// A label outside [0, C) yields NaN in all three.
template <typename T>
__global__ __launch_bounds__(256) void metrics_k(const T* __restrict__ X, int64_t ld, const int64_t* __restrict__ labels,
                                                 int B, int C, float ls, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  const T* x = X + (int64_t)b * ld;
  const int64_t lab = labels[b];
  float mx = -INFINITY;
  int arg = 0x7fffffff;
  for (int j = lane; j < C; j += 64) {
    const float v = to_f<T>(x[j]);
    if (v > mx) {
      mx = v;
      arg = j;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(mx, o, 64);
    const int a2 = __shfl_xor(arg, o, 64);
    if (m2 > mx || (m2 == mx && a2 < arg)) {
      mx = m2;
      arg = a2;
    }
  }
  const float t_off = ls / C, t_on = (1.0f - ls) + ls / C;
  float se = 0.f, bce = 0.f;
  for (int j = lane; j < C; j += 64) {
    const float v = to_f<T>(x[j]);
    se += expf(v - mx);
    const float t = (j == lab) ? t_on : t_off;
    const float m = fmaxf(-v, 0.f);
    bce += (1.f - t) * v + m + logf(expf(-m) + expf(-v - m));
  }
  for (int o = 32; o > 0; o >>= 1) {
    se += __shfl_xor(se, o, 64);
    bce += __shfl_xor(bce, o, 64);
  }
  if (lane == 0) {
    const bool ok = lab >= 0 && lab < C;
    const float nan = __int_as_float(0x7fc00000);
    out[3 * b + 0] = ok ? (mx + logf(se)) - to_f<T>(x[lab]) : nan;
    out[3 * b + 1] = ok ? bce : nan;
    out[3 * b + 2] = ok ? (arg == lab ? 1.f : 0.f) : nan;
  }
}

extern "C" int sdp_logits_metrics(int dtype, const void* X, int64_t ld, const int64_t* labels, int B, int C,
                                  float label_smoothing, float* out, void* stream) {
  if (B < 0 || C <= 0 || ld < C) return (int)hipErrorInvalidValue;
  if (B == 0) return 0;
  if (!X || !labels || !out) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid((B + 3) / 4);
  if (dtype == 0)
    hipLaunchKernelGGL(metrics_k<float>, grid, dim3(256), 0, s, (const float*)X, ld, labels, B, C, label_smoothing, out);
  else if (dtype == 1)
    hipLaunchKernelGGL(metrics_k<bf16_t>, grid, dim3(256), 0, s, (const bf16_t*)X, ld, labels, B, C, label_smoothing,
                       out);
  else
    return (int)hipErrorInvalidValue;
  return SDP_CHECK_LAUNCH();
}
