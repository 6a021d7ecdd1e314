// Scaled-dot-product attention of EncoderLayer (layers.py:289-298):
//     O = softmax(Q K^T / sqrt(hd) + bias) V      per (batch, head), no dropout (eval)
// Q, K, V are read straight out of the fused QKV projection rows
// [B*N, 3C] (q | k | v, head h at columns h*hd..h*hd+hd-1 of each third), already
// q/k-normalised (sdp_qk_headnorm).  O is written as [B*N, C] rows (heads
// concatenated), i.e. the layout o_proj consumes (layers.py:300-301).
//
//  * attn_mfma_bf16 — one workgroup per (b, h), 4 waves.  The whole K (row-major)
//    and V^T of the head are staged in LDS (N <= ~320 fits), each wave walks
//    16-query tiles: S = Q K^T with v_mfma_f32_16x16x32_bf16 (Q fragments loaded
//    straight from HBM), row softmax with in-lane + 16-lane shuffle reductions,
//    P (bf16) through a per-wave LDS tile, O = P V with the same MFMA, O staged
//    through LDS and stored as 16-B row chunks.  Row strides are padded by 16 B so
//    every 16-row ds_read_b128 fragment read is bank-conflict free.
//  * attn_generic<T> — fp32 path / any shape / optional additive mask: 4 lanes per
//    query, online softmax over keys (fp32 throughout).
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
// MFMA bf16
// ---------------------------------------------------------------------------
struct AttnGeom {
  int N, H, hd, HDP, NP;   // HDP: hd padded to 32; NP: N padded to 32
  int ldk, ldv, ldp;       // LDS row strides (elements), each = multiple of 8 + 8 pad
  int k_off, v_off, p_off, p_wave;  // byte offsets
  int bytes;
};

static AttnGeom attn_geom(int N, int H, int hd) {
  AttnGeom g;
  g.N = N; g.H = H; g.hd = hd;
  g.HDP = (hd + 31) / 32 * 32;
  g.NP = (N + 31) / 32 * 32;
  g.ldk = g.HDP + 8;
  g.ldv = g.NP + 8;
  g.ldp = g.NP + 8;
  g.k_off = 0;
  g.v_off = g.NP * g.ldk * 2;
  g.p_off = g.v_off + g.HDP * g.ldv * 2;
  const int ptile = 16 * g.ldp * 2;
  const int otile = 16 * (g.HDP + 8) * 2;
  g.p_wave = ptile > otile ? ptile : otile;
  g.bytes = g.p_off + 4 * g.p_wave;
  return g;
}

template <int NKT>  // number of 16-key tiles = NP / 16 (compile time: the score row lives in registers)
__global__ __launch_bounds__(256) void attn_mfma_bf16(const bf16_t* __restrict__ QKV, int64_t ldq,
                                                      bf16_t* __restrict__ O, int64_t ldo, AttnGeom g,
                                                      float scale_log2) {
  extern __shared__ __attribute__((aligned(16))) char sm[];
  bf16_t* Ks = (bf16_t*)(sm + g.k_off);   // [NP][ldk]   K rows (zero pad)
  bf16_t* Vt = (bf16_t*)(sm + g.v_off);   // [HDP][ldv]  V transposed (zero pad)
  const int b = blockIdx.x / g.H, h = blockIdx.x % g.H;
  const int N = g.N, hd = g.hd, HDP = g.HDP, NP = g.NP;
  const int C = g.H * hd;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bf16_t* base = QKV + (int64_t)b * N * ldq + h * hd;

  // ---- stage K (row-major) and V^T, 8 elements (16 B) per load ----
  const int cpr = HDP / 8;  // chunks per padded row
  for (int idx = tid; idx < NP * cpr; idx += 256) {
    const int j = idx / cpr, c8 = (idx % cpr) * 8;
    bf16x8 kv = {0, 0, 0, 0, 0, 0, 0, 0}, vv = {0, 0, 0, 0, 0, 0, 0, 0};
    if (j < N) {
      const bf16_t* kr = base + (int64_t)j * ldq + C + c8;
      const bf16_t* vr = base + (int64_t)j * ldq + 2 * C + c8;
      if (c8 + 8 <= hd) {
        kv = *(const bf16x8*)kr;
        vv = *(const bf16x8*)vr;
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          if (c8 + e < hd) {
            kv[e] = (short)kr[e];
            vv[e] = (short)vr[e];
          }
        }
      }
    }
    *(bf16x8*)&Ks[j * g.ldk + c8] = kv;
#pragma unroll
    for (int e = 0; e < 8; ++e) Vt[(c8 + e) * g.ldv + j] = (bf16_t)vv[e];
  }
  __syncthreads();

  bf16_t* Ps = (bf16_t*)(sm + g.p_off + wave * g.p_wave);  // [16][ldp], reused for O
  const int fr = lane & 15, fq = lane >> 4;
  const int nqt = (N + 15) / 16;
  constexpr int MAXKT = NKT;
  const int nkt = NKT;
  const int nks = HDP / 32;  // k-steps over head dim
  for (int qt = wave; qt < nqt; qt += 4) {
    // Q fragments (A operand): Q[q = qt*16 + fr][d = 32*ks + 8*fq .. +7]
    bf16x8 qf[4];
    const int qrow = qt * 16 + fr;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      qf[ks] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
      if (ks < nks && qrow < N) {
        const int d0 = ks * 32 + fq * 8;
        const bf16_t* qp = base + (int64_t)qrow * ldq + d0;
        if (d0 + 8 <= hd) {
          qf[ks] = *(const bf16x8*)qp;
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) if (d0 + e < hd) qf[ks][e] = (short)qp[e];
        }
      }
    }
    // S = Q K^T: D[q][key], lane holds rows 4*fq + r of column key = 16*t + fr
    f32x4 s[MAXKT];
#pragma unroll
    for (int t = 0; t < MAXKT; ++t) {
      s[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (t < nkt) {
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
          if (ks < nks) {
            const bf16x8 kf = *(const bf16x8*)&Ks[(t * 16 + fr) * g.ldk + ks * 32 + fq * 8];
            s[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qf[ks], kf, s[t], 0, 0, 0);
          }
        }
      }
    }
    // softmax over keys (mask padded keys)
    float mx[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
    for (int t = 0; t < MAXKT; ++t) {
      if (t < nkt) {
        const bool kv = (t * 16 + fr) < N;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          s[t][r] = kv ? s[t][r] * scale_log2 : -INFINITY;
          mx[r] = fmaxf(mx[r], s[t][r]);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) mx[r] = fmaxf(mx[r], __shfl_xor(mx[r], o, 64));
    float sum[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < MAXKT; ++t) {
      if (t < nkt) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = exp2f(s[t][r] - mx[r]);
          sum[r] += p;
          Ps[(fq * 4 + r) * g.ldp + t * 16 + fr] = f2bf(p);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) sum[r] += __shfl_xor(sum[r], o, 64);
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): P writes landed (single wave owns Ps)
    __builtin_amdgcn_wave_barrier();

    // O = P V: D[q][d], A = P[q][key], B = V[key][d] read from V^T[d][key]
    f32x4 o[8];
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int kk = 0; kk < NP / 32; ++kk) {
      const bf16x8 pf = *(const bf16x8*)&Ps[fr * g.ldp + kk * 32 + fq * 8];
#pragma unroll
      for (int dt = 0; dt < 8; ++dt) {
        if (dt * 16 < HDP) {
          const bf16x8 vf = *(const bf16x8*)&Vt[(dt * 16 + fr) * g.ldv + kk * 32 + fq * 8];
          o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pf, vf, o[dt], 0, 0, 0);
        }
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    // normalise, stage O tile [16][HDP+8] in the P region, store 16-B chunks
    const int ldo_s = HDP + 8;
    float inv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) inv[r] = 1.0f / sum[r];
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) {
      if (dt * 16 < HDP) {
#pragma unroll
        for (int r = 0; r < 4; ++r) Ps[(fq * 4 + r) * ldo_s + dt * 16 + fr] = f2bf(o[dt][r] * inv[r]);
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    const int cpr_o = HDP / 8;
    for (int idx = lane; idx < 16 * cpr_o; idx += 64) {
      const int r = idx / cpr_o, c8 = (idx % cpr_o) * 8;
      const int q = qt * 16 + r;
      if (q < N && c8 < hd) {
        bf16_t* op = O + ((int64_t)b * N + q) * ldo + h * hd + c8;
        const bf16x8 v = *(const bf16x8*)&Ps[r * ldo_s + c8];
        if (c8 + 8 <= hd) {
          *(bf16x8*)op = v;
        } else {
          for (int e = 0; e < 8 && c8 + e < hd; ++e) op[e] = (bf16_t)v[e];
        }
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
  }
}

template <int NKT>
static int launch_attn_mfma(const void* QKV, int64_t ldq, void* O, int64_t ldo, int B, const AttnGeom& g,
                            float scale, hipStream_t s) {
  if (g.bytes > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute((const void*)attn_mfma_bf16<NKT>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, g.bytes);
    if (e != hipSuccess) return (int)e;
  }
  hipLaunchKernelGGL(attn_mfma_bf16<NKT>, dim3(B * g.H), dim3(256), g.bytes, s, (const bf16_t*)QKV, ldq,
                     (bf16_t*)O, ldo, g, scale * 1.4426950408889634f);
  return SDP_CHECK_LAUNCH();
}

extern "C" int sdp_attention_variant(int dtype, int N, int n_head, int head_dim, int has_mask) {
  if (dtype != 1 || has_mask || head_dim > 128 || head_dim % 8 != 0) return 0;
  const AttnGeom g = attn_geom(N, n_head, head_dim);
  if (g.NP > 384 || g.bytes > 160 * 1024) return 0;
  return 1;
}

extern "C" int sdp_attention(int dtype, const void* QKV, int64_t ldq, void* O, int64_t ldo, int B, int N,
                             int n_head, int head_dim, const float* mask, int64_t mask_sb, int64_t mask_sh,
                             void* stream) {
  if (!QKV || !O || B < 0 || N <= 0 || n_head <= 0 || head_dim <= 0 || head_dim > 128)
    return (int)hipErrorInvalidValue;
  if (B == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const float scale = 1.0f / sqrtf((float)head_dim);
  if (sdp_attention_variant(dtype, N, n_head, head_dim, mask != nullptr) == 1 && (ldq % 8 == 0) &&
      (ldo % 8 == 0) && ((uintptr_t)QKV % 16 == 0) && ((uintptr_t)O % 16 == 0)) {
    const AttnGeom g = attn_geom(N, n_head, head_dim);
    switch (g.NP / 16) {
#define SDP_ATT(NKT) case NKT: return launch_attn_mfma<NKT>(QKV, ldq, O, ldo, B, g, scale, s);
      SDP_ATT(2) SDP_ATT(4) SDP_ATT(6) SDP_ATT(8) SDP_ATT(10) SDP_ATT(12)
      SDP_ATT(14) SDP_ATT(16) SDP_ATT(18) SDP_ATT(20) SDP_ATT(22) SDP_ATT(24)
#undef SDP_ATT
      default: return (int)hipErrorInvalidValue;
    }
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
