// Scaled-dot-product attention of EncoderLayer (layers.py:289-298):
//     O = softmax(Q K^T / sqrt(hd) + bias) V      per (batch, head), no dropout (eval)
// Q, K, V are read straight out of the fused QKV projection rows
// [B*N, 3C] (q | k | v, head h at columns h*hd..h*hd+hd-1 of each third), already
// q/k-normalised here.  O is written as [B*N, C] rows (heads
// concatenated), i.e. the layout o_proj consumes (layers.py:300-301).
//
//  * attn_fa_bf16 — bf16 hot path: flash-style, swapped-operand 32x32x16 MFMA with
//    P kept in registers, q/k LayerNorm fused into the loads (see below).
//  * attn_generic<T> — fp32 path / any shape / optional additive mask: 4 lanes per
//    query, online softmax over keys (fp32 throughout); q/k norms are applied
//    first, in place on the QKV rows, by sdp_qk_headnorm.
#include "common.h"

// ---------------------------------------------------------------------------
// generic
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void attn_generic(const T* __restrict__ QKV, int64_t ldq, T* __restrict__ O,
                                                    int64_t ldo, const float* __restrict__ mask,
                                                    int64_t mask_sb, int64_t mask_sh, int N, int H, int hd,
                                                    float scale) {
  const int b = blockIdx.z, h = blockIdx.y;
  const int q = blockIdx.x * 64 + (threadIdx.x >> 2);
  const int part = threadIdx.x & 3;
  const int C = H * hd;
  const bool qvalid = q < N;
  const int qq = qvalid ? q : N - 1;
  const T* qrow = QKV + ((int64_t)b * N + qq) * ldq + h * hd;
  const T* kbase = QKV + (int64_t)b * N * ldq + C + h * hd;
  const T* vbase = QKV + (int64_t)b * N * ldq + 2 * C + h * hd;
  const float* mrow = mask ? mask + b * mask_sb + h * mask_sh + (int64_t)qq * N : nullptr;
  constexpr int MAXD = 32;  // hd <= 128 -> <= 32 dims per lane
  float qv[MAXD], ov[MAXD];
  const int dpl = (hd + 3) / 4;
#pragma unroll
  for (int i = 0; i < MAXD; ++i) {
    const int d = part + 4 * i;
    qv[i] = (i < dpl && d < hd) ? to_f<T>(qrow[d]) * scale : 0.f;
    ov[i] = 0.f;
  }
  float m = -INFINITY, l = 0.f;
  for (int j = 0; j < N; ++j) {
    const T* kr = kbase + (int64_t)j * ldq;
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < MAXD; ++i) {
      const int d = part + 4 * i;
      if (i < dpl && d < hd) s = fmaf(qv[i], to_f<T>(kr[d]), s);
    }
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);
    if (mrow) s += mrow[j];
    const float mn = fmaxf(m, s);
    if (mn == -INFINITY) continue;  // all masked so far
    const float alpha = expf(m - mn);
    const float p = expf(s - mn);
    l = l * alpha + p;
    const T* vr = vbase + (int64_t)j * ldq;
#pragma unroll
    for (int i = 0; i < MAXD; ++i) {
      const int d = part + 4 * i;
      if (i < dpl && d < hd) ov[i] = ov[i] * alpha + p * to_f<T>(vr[d]);
    }
    m = mn;
  }
  if (!qvalid) return;
  const float inv = 1.0f / l;  // fully masked row -> NaN, like SDPA
  T* orow = O + ((int64_t)b * N + q) * ldo + h * hd;
#pragma unroll
  for (int i = 0; i < MAXD; ++i) {
    const int d = part + 4 * i;
    if (i < dpl && d < hd) orow[d] = from_f<T>(ov[i] * inv);
  }
}

// ---------------------------------------------------------------------------
// Flash-style MFMA attention, one workgroup per (b, h), one wave per 32-query
// tile, v_mfma_f32_32x32x16_bf16 in the "swapped" form:
//   S^T[key][q] = K Q^T       (A = K rows from LDS, B = Q fragment in registers)
//   O^T[d][q]  += V^T P^T     (A = V^T read transposed from the row-major V tile
//                             with ds_read_b64_tr_b16, B = the S^T accumulator)
// The S^T accumulator has the query on the lane and 16 keys in registers, so the
// softmax is in-lane + one cross-half shuffle and P never leaves registers
// (cdna_hip_programming.md §3 "An accumulator tile as the next MFMA's operand").
// Online softmax over 32-key tiles (running max m, partial sum l per lane half).
// q_norm / k_norm (layers.py:236-237, :286) are applied while loading Q and
// staging K; the 1/sqrt(hd) scale (and log2 e) is applied to S in fp32.
// ---------------------------------------------------------------------------
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

template <int HDT>  // O d-tiles of 32 (hd <= 32 * HDT)
__global__ __launch_bounds__(640) void attn_fa_bf16(const bf16_t* __restrict__ QKV, int64_t ldq,
                                                     bf16_t* __restrict__ O, int64_t ldo, int N, int H, int hd,
                                                     const float* __restrict__ gq, const float* __restrict__ bq,
                                                     const float* __restrict__ gk, const float* __restrict__ bk,
                                                     float eps, float scale_log2, int ldk, int ldv) {
  extern __shared__ __attribute__((aligned(16))) char sm[];
  const int NP = (N + 31) / 32 * 32;
  bf16_t* Ks = (bf16_t*)sm;            // [NP][ldk]  k-normed K rows
  bf16_t* Vs = Ks + (size_t)NP * ldk;  // [NP][ldv]  V rows (read transposed by ds_read_b64_tr_b16)
  const int b = blockIdx.x / H, hh = blockIdx.x % H;
  const int C = H * hd;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nwaves = blockDim.x >> 6;
  const bf16_t* base = QKV + (int64_t)b * N * ldq + hh * hd;

  // ---- stage K (k-normed) and V: 16 lanes per key row, 8 elements per lane.
  // Loads of up to 8 rows per thread are issued before any is consumed. ----
  {
    const int sub = tid & 15;
    const int c8 = sub * 8;
    const int rstep = blockDim.x >> 4;
    constexpr int UNR = 8;
    for (int j0 = tid >> 4; j0 < NP; j0 += rstep * UNR) {
      bf16x8 kr[UNR], vr[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const int j = j0 + u * rstep;
        kr[u] = vr[u] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
        if (j < N && c8 < hd) {
          kr[u] = *(const bf16x8*)(base + (int64_t)j * ldq + C + c8);
          vr[u] = *(const bf16x8*)(base + (int64_t)j * ldq + 2 * C + c8);
        }
      }
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const int j = j0 + u * rstep;
        if (j >= NP) break;  // uniform per 16-lane group
        const bool ok = (j < N) && (c8 < hd);
        if (gk) {
          float kv[8];
          float s = 0.f;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            kv[e] = bf2f((bf16_t)kr[u][e]);
            s += kv[e];
          }
#pragma unroll
          for (int o = 8; o > 0; o >>= 1) s += __shfl_xor(s, o, 16);
          const float mean = s / (float)hd;
          float ss = 0.f;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float d = ok ? kv[e] - mean : 0.f;
            ss += d * d;
          }
#pragma unroll
          for (int o = 8; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 16);
          const float rstd = 1.0f / sqrtf(ss / (float)hd + eps);
          if (ok) {
#pragma unroll
            for (int e = 0; e < 8; ++e) kr[u][e] = (short)f2bf((kv[e] - mean) * rstd * gk[c8 + e] + bk[c8 + e]);
          }
        }
        if (c8 < hd) *(bf16x8*)&Ks[(size_t)j * ldk + c8] = kr[u];
        if (c8 < ldv) *(bf16x8*)&Vs[(size_t)j * ldv + c8] = vr[u];  // also zeroes the d-padding
      }
    }
  }
  __syncthreads();

  const int r = lane & 31, hf = lane >> 5;
  const int nds = hd / 16;          // k-steps of 16 over the head dim
  const int nqt = NP / 32;
  for (int qt = wave; qt < nqt; qt += nwaves) {
    const int q = qt * 32 + r;
    const bool qok = q < N;
    // ---- Q fragments (B operand): Q[q][16s + 8hf + j], q-normed and pre-scaled ----
    constexpr int NDS_MAX = 2 * HDT;  // hd <= 32 * HDT -> at most 2*HDT k-steps of 16
    bf16x8 qf[NDS_MAX];
    float qsum = 0.f;
#pragma unroll
    for (int s = 0; s < NDS_MAX; ++s) {
      qf[s] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
      if (s < nds && qok) qf[s] = *(const bf16x8*)(base + (int64_t)q * ldq + 16 * s + 8 * hf);
#pragma unroll
      for (int e = 0; e < 8; ++e) qsum += bf2f((bf16_t)qf[s][e]);
    }
    float qmean = 0.f, qrstd = 1.f;
    if (gq) {
      qsum += __shfl_xor(qsum, 32, 64);
      qmean = qsum / (float)hd;
      float ss = 0.f;
#pragma unroll
      for (int s = 0; s < NDS_MAX; ++s) {
        if (s < nds) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float d = bf2f((bf16_t)qf[s][e]) - qmean;
            ss += d * d;
          }
        }
      }
      ss += __shfl_xor(ss, 32, 64);
      qrstd = 1.0f / sqrtf(ss / (float)hd + eps);
    }
#pragma unroll
    for (int s = 0; s < NDS_MAX; ++s) {
      if (s < nds) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int d = 16 * s + 8 * hf + e;
          float x = bf2f((bf16_t)qf[s][e]);
          if (gq) x = (x - qmean) * qrstd * gq[d] + bq[d];
          qf[s][e] = (short)f2bf(qok ? x : 0.f);
        }
      }
    }

    f32x16 acc[HDT];
#pragma unroll
    for (int dt = 0; dt < HDT; ++dt)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[dt][i] = 0.f;
    float m = -INFINITY, l = 0.f;
    for (int kt = 0; kt < nqt; ++kt) {
      f32x16 st;
#pragma unroll
      for (int i = 0; i < 16; ++i) st[i] = 0.f;
      const bf16_t* krow = Ks + (size_t)(kt * 32 + r) * ldk + 8 * hf;
#pragma unroll
      for (int s = 0; s < NDS_MAX; ++s) {
        if (s < nds) {
          const bf16x8 kf = *(const bf16x8*)(krow + 16 * s);
          st = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[s], st, 0, 0, 0);
        }
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) st[i] *= scale_log2;  // fp32 scale (bf16 Q stays unscaled)
      if (kt * 32 + 32 > N) {  // mask padded keys of the last tile
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int key = kt * 32 + (i & 3) + 8 * (i >> 2) + 4 * hf;
          if (key >= N) st[i] = -INFINITY;
        }
      }
      float tmax = st[0];
#pragma unroll
      for (int i = 1; i < 16; ++i) tmax = fmaxf(tmax, st[i]);
      tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
      const float mn = fmaxf(m, tmax);
      if (__any(mn > m)) {  // wave-uniform: rescale only when some running max moved
        const float alpha = __builtin_amdgcn_exp2f(m - mn);
        l *= alpha;
#pragma unroll
        for (int dt = 0; dt < HDT; ++dt)
#pragma unroll
          for (int i = 0; i < 16; ++i) acc[dt][i] *= alpha;
        m = mn;
      }
      float p[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        p[i] = __builtin_amdgcn_exp2f(st[i] - m);
        l += p[i];
      }
      // A = V^T fragment via transposed LDS reads of the row-major V tile: the
      // 16-lane group g = lane/16 reads the 4-key x 16-d block (keys key0..key0+3,
      // d = 32*dt + 16*(g&1) ..+15); lane 4q+p addresses key key0+q, d +4p..+4p+3,
      // and receives d = its own column for the 4 keys (= fragment elements 0..3;
      // the +8-key read gives elements 4..7, matching P^T's register order).
      const int gi = lane & 15, tq = gi >> 2, tp = gi & 3;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        bf16x8 pb;
#pragma unroll
        for (int j = 0; j < 8; ++j) pb[j] = (short)f2bf(p[8 * s2 + j]);
        const int key0 = kt * 32 + 16 * s2 + 4 * hf;
#pragma unroll
        for (int dt = 0; dt < HDT; ++dt) {
          const bf16_t* vb = Vs + (size_t)(key0 + tq) * ldv + dt * 32 + 16 * ((lane >> 4) & 1) + 4 * tp;
          const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)vb);
          const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(vb + 8 * ldv));
          const bf16x8 vf = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          acc[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pb, acc[dt], 0, 0, 0);
        }
      }
    }
    l += __shfl_xor(l, 32, 64);
    const float inv = 1.0f / l;
    if (qok) {
      bf16_t* orow = O + ((int64_t)b * N + q) * ldo + hh * hd;
#pragma unroll
      for (int dt = 0; dt < HDT; ++dt) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int d = dt * 32 + 8 * g + 4 * hf;
          if (d < hd) {
            bf16x4 o;
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = (short)f2bf(acc[dt][4 * g + e] * inv);
            *(bf16x4*)(orow + d) = o;
          }
        }
      }
    }
  }
}

template <int HDT>
static int launch_attn_fa(const void* QKV, int64_t ldq, void* O, int64_t ldo, int B, int N, int H, int hd,
                          const float* gq, const float* bq, const float* gk, const float* bk, float eps, float scale,
                          hipStream_t s) {
  const int NP = (N + 31) / 32 * 32;
  const int ldk = hd + 8, ldv = 32 * HDT + 8;
  const size_t bytes = ((size_t)NP * ldk + (size_t)NP * ldv) * 2;
  if (bytes > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute((const void*)attn_fa_bf16<HDT>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)bytes);
    if (e != hipSuccess) return (int)e;
  }
  int waves = NP / 32;
  if (waves > 10) waves = 10;  // __launch_bounds__(640): <= 168 VGPRs
  hipLaunchKernelGGL(attn_fa_bf16<HDT>, dim3(B * H), dim3(64 * waves), bytes, s, (const bf16_t*)QKV, ldq,
                     (bf16_t*)O, ldo, N, H, hd, gq, bq, gk, bk, eps, scale * 1.4426950408889634f, ldk, ldv);
  return SDP_CHECK_LAUNCH();
}

static size_t attn_fa_bytes(int N, int hd) {
  const int NP = (N + 31) / 32 * 32;
  const int HDT = (hd + 31) / 32;
  return ((size_t)NP * (hd + 8) + (size_t)NP * (32 * HDT + 8)) * 2;
}

extern "C" int sdp_attention_variant(int dtype, int N, int n_head, int head_dim, int has_mask) {
  if (dtype != 1 || has_mask || head_dim > 128 || head_dim % 16 != 0) return 0;
  if (attn_fa_bytes(N, head_dim) > 160 * 1024) return 0;
  return 2;
}

int sdp_qk_headnorm(int dtype, void* QKV, int64_t ld, int64_t rows, int n_head, int head_dim, const float* gq,
                    const float* bq, const float* gk, const float* bk, float eps, void* stream);

extern "C" int sdp_attention(int dtype, const void* QKV, int64_t ldq, void* O, int64_t ldo, int B, int N,
                             int n_head, int head_dim, const float* q_gamma, const float* q_beta,
                             const float* k_gamma, const float* k_beta, float eps, const float* mask, int64_t mask_sb,
                             int64_t mask_sh, void* stream) {
  if (!QKV || !O || B < 0 || N <= 0 || n_head <= 0 || head_dim <= 0 || head_dim > 128)
    return (int)hipErrorInvalidValue;
  const bool norm = q_gamma != nullptr;
  if (norm && (!q_beta || !k_gamma || !k_beta)) return (int)hipErrorInvalidValue;
  if (B == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const float scale = 1.0f / sqrtf((float)head_dim);
  if (sdp_attention_variant(dtype, N, n_head, head_dim, mask != nullptr) == 2 && (ldq % 8 == 0) && (ldo % 4 == 0) &&
      ((uintptr_t)QKV % 16 == 0) && ((uintptr_t)O % 8 == 0)) {
    const int HDT = (head_dim + 31) / 32;
    const float *gq = norm ? q_gamma : nullptr, *bq = norm ? q_beta : nullptr;
    const float *gk = norm ? k_gamma : nullptr, *bk = norm ? k_beta : nullptr;
    switch (HDT) {
      case 1: return launch_attn_fa<1>(QKV, ldq, O, ldo, B, N, n_head, head_dim, gq, bq, gk, bk, eps, scale, s);
      case 2: return launch_attn_fa<2>(QKV, ldq, O, ldo, B, N, n_head, head_dim, gq, bq, gk, bk, eps, scale, s);
      case 3: return launch_attn_fa<3>(QKV, ldq, O, ldo, B, N, n_head, head_dim, gq, bq, gk, bk, eps, scale, s);
      default: return launch_attn_fa<4>(QKV, ldq, O, ldo, B, N, n_head, head_dim, gq, bq, gk, bk, eps, scale, s);
    }
  }
  // generic path: head norms in place on the QKV rows, then the VALU kernel
  if (norm) {
    const int rc = sdp_qk_headnorm(dtype, (void*)QKV, ldq, (int64_t)B * N, n_head, head_dim, q_gamma, q_beta, k_gamma,
                                   k_beta, eps, stream);
    if (rc) return rc;
  }
  dim3 grid((N + 63) / 64, n_head, B);
  if (dtype == 1)
    hipLaunchKernelGGL(attn_generic<bf16_t>, grid, dim3(256), 0, s, (const bf16_t*)QKV, ldq, (bf16_t*)O, ldo,
                       mask, mask_sb, mask_sh, N, n_head, head_dim, scale);
  else if (dtype == 0)
    hipLaunchKernelGGL(attn_generic<float>, grid, dim3(256), 0, s, (const float*)QKV, ldq, (float*)O, ldo, mask,
                       mask_sb, mask_sh, N, n_head, head_dim, scale);
  else
    return (int)hipErrorInvalidValue;
  return SDP_CHECK_LAUNCH();
}
