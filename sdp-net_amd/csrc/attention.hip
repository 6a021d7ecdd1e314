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

#ifndef ATTN_CH
// key tiles per softmax chunk of attn_qtile_chunked for hd <= 96: 7 = the whole key range at
// N <= 224 in one chunk (one max, no rescale of O), N <= 256 in two; 111.7 vs 117.5 us at the M
// shape with 4 (tools/r4_ch.sh).  hd = 128 keeps 4 (register budget).
#define ATTN_CH 7
#endif

// K and V of one (image, head) pair -> LDS by buffer LDS-DMA (K chunk c of row r at c ^ ((r >> 2) & 3),
// V row-major, NP16 rows each), in units of 16 rows = HDT instructions of 64 x 16 B.  A 16-row unit
// keeps the K swizzle phase, so the per-lane byte offsets within a unit are the same for every unit
// and pair: computed once (2 HDT registers); a unit's loads differ only by the scalar offset, and
// no per-load address arithmetic is left (it was ~40 VALU per load, a quarter of the kernel's VALU).
// The buffer resource ends at row N-1 of the pair's image, so rows N .. NP16-1 read as 0 (the
// hardware's range check): finite, masked scores, P = 0, and nothing read from another image.
template <int HDT>
struct AttnKV {
  uint32_t ko[HDT], vo[HDT];
  SDP_DEV AttnKV(int lane, int64_t ldq, int C) {
    constexpr int CPR = 4 * HDT;
#pragma unroll
    for (int r = 0; r < HDT; ++r) {
      const int g = r * 64 + lane, row = g / CPR, pc = g - (g / CPR) * CPR;
      ko[r] = (uint32_t)(((int64_t)row * ldq + C + 8 * (pc ^ ((row >> 2) & 3))) * 2);
      vo[r] = (uint32_t)(((int64_t)row * ldq + 2 * C + 8 * pc) * 2);
    }
  }
  // base: row 0 / column hh * HD of the pair; bytes: extent of the image's QKV rows from base.
  // DK / DV: stage K / V (attn_fa6 stages them at different times).
  template <bool DK = true, bool DV = true>
  SDP_DEV void issue(const bf16_t* base, uint64_t bytes, char* Ks, char* Vs, int NP16, int64_t ldq, int wave,
                     int nwaves) const {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)base, 0, (int)(bytes < 0xffffffffull ? bytes : 0xffffffffull), 0x00020000);
    const int U = NP16 >> 4, w0 = __builtin_amdgcn_readfirstlane(wave);  // wave-uniform unit index
    const uint32_t ustep = (uint32_t)(16 * ldq * 2);
    if constexpr (DK)
      for (int u = w0; u < U; u += nwaves)
#pragma unroll
        for (int r = 0; r < HDT; ++r)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (AS3 void*)(Ks + (u * HDT + r) * 1024), 16, (int)ko[r], (int)(u * ustep), 0, 0);
    if constexpr (DV)
      for (int u = w0; u < U; u += nwaves)
#pragma unroll
        for (int r = 0; r < HDT; ++r)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (AS3 void*)(Vs + (u * HDT + r) * 1024), 16, (int)vo[r], (int)(u * ustep), 0, 0);
  }
};
// ---------------------------------------------------------------------------
// Per-wave pieces of the two-workgroup / persistent flash kernels (hd = 32*HDT).
// Lane (r = lane & 31, hf = lane >> 5) owns query r of a 32-query tile and, in
// every fragment, the 8 head dims 16s + 8hf .. +7 (k-step s).
// ---------------------------------------------------------------------------
// qrow must be a valid row (callers clamp padded queries to row N-1: their
// fragments are finite and their outputs are never stored).  Unconditional loads,
// so a prefetch into qf is not waited for until qf is used.
template <int HDT>
SDP_DEV void attn_load_q(const bf16_t* qrow, int hf, bf16x8 (&qf)[2 * HDT]) {
#pragma unroll
  for (int s = 0; s < 2 * HDT; ++s) qf[s] = *(const bf16x8*)(qrow + 16 * s + 8 * hf);
}

// q_norm (layers.py:236, :286) on the fragments: mean / biased var over the head
// dim (the two halves of a query meet through one cross-half shuffle).
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
// two fp32 -> one dword of two bf16 (RNE), a single v_cvt_pk_bf16_f32
SDP_DEV uint32_t pack_bf16x2(float a, float b) {
  const bf16x2v v = __builtin_convertvector((f32x2){a, b}, bf16x2v);
  return __builtin_bit_cast(uint32_t, v);
}
typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;

// Partial LayerNorm statistics of one 8 x bf16 fragment: {sum x, sum x^2} with
// v_dot2_f32_bf16 (fp32 accumulation), 8 instructions per fragment.
typedef __bf16 bf16x8v __attribute__((ext_vector_type(8)));
SDP_DEV f32x2 frag_stats(const bf16x8& v, f32x2 acc) {
  // (element-wise pairs: bit-casting a u32x4 lane to bf16x2 miscompiles in ROCm 7.2 hipcc,
  // every pair then reads dword 0)
  const bf16x8v v8 = __builtin_bit_cast(bf16x8v, v);
  const bf16x2v one = __builtin_bit_cast(bf16x2v, 0x3F803F80u);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const bf16x2v x = {v8[2 * k], v8[2 * k + 1]};
    acc.x = __builtin_amdgcn_fdot2_f32_bf16(x, one, acc.x, false);
    acc.y = __builtin_amdgcn_fdot2_f32_bf16(x, x, acc.y, false);
  }
  return acc;
}
// y = (x - mean) * rstd * g + b on one fragment (g, b: its 8 columns), packed f32
// math: y = x * t + (b - mean * t) with t = rstd * g.
SDP_DEV bf16x8 frag_norm(const bf16x8& v, float mean, float rstd, const float* g, const float* b) {
  const u32x4 w = __builtin_bit_cast(u32x4, v);
  const f32x4 g0 = *(const f32x4*)g, g1 = *(const f32x4*)(g + 4);
  const f32x4 b0 = *(const f32x4*)b, b1 = *(const f32x4*)(b + 4);
  const f32x2 r2 = {rstd, rstd}, m2 = {-mean, -mean};
  u32x4 o;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const f32x2 x = {__uint_as_float(w[k] << 16), __uint_as_float(w[k] & 0xFFFF0000u)};
    const f32x2 gg = k < 2 ? f32x2{g0[2 * k], g0[2 * k + 1]} : f32x2{g1[2 * k - 4], g1[2 * k - 3]};
    const f32x2 bb = k < 2 ? f32x2{b0[2 * k], b0[2 * k + 1]} : f32x2{b1[2 * k - 4], b1[2 * k - 3]};
    const f32x2 t = gg * r2;
    const f32x2 c = t * m2 + bb;
    const f32x2 y = x * t + c;
    o[k] = pack_bf16x2(y.x, y.y);
  }
  return __builtin_bit_cast(bf16x8, o);
}

template <int HDT>
SDP_DEV void attn_norm_q(bf16x8 (&qf)[2 * HDT], bool qok, int hf, const float* gq, const float* bq, float eps) {
  constexpr int HD = 32 * HDT;
  f32x2 st = {0.f, 0.f};
#pragma unroll
  for (int s = 0; s < 2 * HDT; ++s) st = frag_stats(qf[s], st);
  st.x += __shfl_xor(st.x, 32, 64);
  st.y += __shfl_xor(st.y, 32, 64);
  const float qmean = st.x * (1.0f / HD);
  const float qrstd = rsqrtf(fmaxf(st.y * (1.0f / HD) - qmean * qmean, 0.f) + eps);
#pragma unroll
  for (int s = 0; s < 2 * HDT; ++s) {
    const int d = 16 * s + 8 * hf;
    qf[s] = qok ? frag_norm(qf[s], qmean, qrstd, gq + d, bq + d) : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
  }
}

// One 32-query tile against all keys: K rows in Ks ([.][HD], 16-B chunk c of row
// r at c ^ ((r >> 2) & 3)), V rows in Vs ([NP16][HD] row-major).  Online softmax
// over 32-key tiles; O row written (bf16) to orow unless null.
template <int HDT>
SDP_DEV void attn_qtile(const bf16_t* Ks, const bf16_t* Vs, const bf16x8 (&qf)[2 * HDT], int N, int nkt,
                        float scale_log2, int lane, bf16_t* orow) {
  constexpr int HD = 32 * HDT;
  constexpr int NDS = HD / 16;
  const int r = lane & 31, hf = lane >> 5;
  f32x16 acc[HDT];
#pragma unroll
  for (int dt = 0; dt < HDT; ++dt)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[dt][i] = 0.f;
  float m = -INFINITY, l = 0.f;
  const int kswz = (r >> 2) & 3;  // K row (kt*32 + r) swizzle
  const int gi = lane & 15, tq = gi >> 2, tp = gi & 3;
  for (int kt = 0; kt < nkt; ++kt) {
    f32x16 st;
#pragma unroll
    for (int i = 0; i < 16; ++i) st[i] = 0.f;
    const bf16x8* krow = (const bf16x8*)(Ks + (size_t)(kt * 32 + r) * HD);
#pragma unroll
    for (int s = 0; s < NDS; ++s) st = __builtin_amdgcn_mfma_f32_32x32x16_bf16(krow[(2 * s + hf) ^ kswz], qf[s], st, 0, 0, 0);
    if (kt * 32 + 32 > N) {  // mask padded keys of the last tile
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int key = kt * 32 + (i & 3) + 8 * (i >> 2) + 4 * hf;
        if (key >= N) st[i] = -INFINITY;
      }
    }
    float tmax = fmaxf(fmaxf(st[0], st[1]), st[2]);
#pragma unroll
    for (int i = 3; i < 15; i += 2) tmax = fmaxf(fmaxf(tmax, st[i]), st[i + 1]);
    tmax = fmaxf(tmax, st[15]);
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    const float mn = fmaxf(m, tmax);
    if (__any(mn > m)) {  // wave-uniform: rescale only when some running max moved
      const float alpha = __builtin_amdgcn_exp2f((m - mn) * scale_log2);
      l *= alpha;
#pragma unroll
      for (int dt = 0; dt < HDT; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[dt][i] *= alpha;
      m = mn;
    }
    const float msc = -m * scale_log2;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      if (kt * 32 + 16 * s2 >= N) break;  // whole half past the keys (wave-uniform)
      float p[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        p[j] = __builtin_amdgcn_exp2f(fmaf(st[8 * s2 + j], scale_log2, msc));
        l += p[j];
      }
      bf16x8 pb;
#pragma unroll
      for (int j = 0; j < 8; ++j) pb[j] = (short)f2bf(p[j]);
      const int key0 = kt * 32 + 16 * s2 + 4 * hf;
      // V^T fragments by inline-asm ds_read_b64_tr_b16: the builtin makes hipcc wait
      // vmcnt(0) (an in-flight LDS-DMA might alias), which would drain the next
      // pair's prefetch here; the reads' own completion is waited for explicitly.
      bf16x4 lo[HDT], hi[HDT];
#pragma unroll
      for (int dt = 0; dt < HDT; ++dt) {
        const uint32_t va = (uint32_t)(uintptr_t)(const AS3 bf16_t*)(Vs + (size_t)(key0 + tq) * HD + dt * 32 +
                                                                     16 * ((lane >> 4) & 1) + 4 * tp);
        asm volatile("ds_read_b64_tr_b16 %0, %2\n\tds_read_b64_tr_b16 %1, %2 offset:%3"
                     : "=&v"(lo[dt]), "=&v"(hi[dt])
                     : "v"(va), "i"(16 * HD)
                     : "memory");
      }
#pragma unroll
      for (int dt = 0; dt < HDT; ++dt) asm volatile("" : "+v"(lo[dt]), "+v"(hi[dt]));
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int dt = 0; dt < HDT; ++dt) {
        asm volatile("" : "+v"(lo[dt]), "+v"(hi[dt]));
        const bf16x8 vf = {lo[dt][0], lo[dt][1], lo[dt][2], lo[dt][3], hi[dt][0], hi[dt][1], hi[dt][2], hi[dt][3]};
        acc[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pb, acc[dt], 0, 0, 0);
      }
    }
  }
  l += __shfl_xor(l, 32, 64);
  const float inv = 1.0f / l;
  if (orow) {
#pragma unroll
    for (int dt = 0; dt < HDT; ++dt) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        bf16x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = (short)f2bf(acc[dt][4 * g + e] * inv);
        *(bf16x4*)(orow + dt * 32 + 8 * g + 4 * hf) = o;
      }
    }
  }
}

// Software-pipelined form of attn_qtile for the 256-VGPR persistent kernel: the
// QK^T MFMAs of key tile kt+1 are issued before the softmax of tile kt (the MFMA
// pipe works while the VALU exponentiates), the V^T fragments of tile kt are
// read before its softmax, and the cross-half max uses v_permlane32_swap.
template <int HDT>
SDP_DEV f32x16 attn_qk(const bf16_t* Ks, const bf16x8 (&qf)[2 * HDT], int kt, int r, int hf) {
  constexpr int HD = 32 * HDT;
  const int kswz = (r >> 2) & 3;
  const bf16x8* krow = (const bf16x8*)(Ks + (size_t)(kt * 32 + r) * HD);
  f32x16 st;
#pragma unroll
  for (int i = 0; i < 16; ++i) st[i] = 0.f;
#pragma unroll
  for (int s = 0; s < 2 * HDT; ++s)
    st = __builtin_amdgcn_mfma_f32_32x32x16_bf16(krow[(2 * s + hf) ^ kswz], qf[s], st, 0, 0, 0);
  return st;
}

// Same with the K row reads addressed from two per-lane bases: chunk (2s + hf) ^ kswz
// = 4 (s >> 1) + ((2 (s & 1) + hf) ^ kswz), so k-steps s and s + 2 differ by an
// immediate 64 B and key tiles by an immediate 32 * HD * 2 B.
template <int HDT>
SDP_DEV f32x16 attn_qk2(const char* k0, const char* k1, const bf16x8 (&qf)[2 * HDT], int kt) {
  constexpr int HD = 32 * HDT;
  f32x16 st;
#pragma unroll
  for (int i = 0; i < 16; ++i) st[i] = 0.f;
#pragma unroll
  for (int s = 0; s < 2 * HDT; ++s) {
    const char* a = ((s & 1) ? k1 : k0) + kt * 32 * HD * 2 + 64 * (s >> 1);
    st = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*(const bf16x8*)a, qf[s], st, 0, 0, 0);
  }
  return st;
}

SDP_DEV float xhalf_max(float v) {
  const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
}
SDP_DEV float xhalf_sum(float v) {
  const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
}

template <int HDT>
SDP_DEV void attn_qtile_pipe(const bf16_t* Ks, const bf16_t* Vs, const bf16x8 (&qf)[2 * HDT], int N, int nkt,
                             float scale_log2, int lane, bf16_t* orow) {
  constexpr int HD = 32 * HDT;
  const int r = lane & 31, hf = lane >> 5;
  f32x16 acc[HDT];
#pragma unroll
  for (int dt = 0; dt < HDT; ++dt)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[dt][i] = 0.f;
  float m = -INFINITY, l = 0.f;
  const int gi = lane & 15, tq = gi >> 2, tp = gi & 3;
  const uint32_t vbase = (uint32_t)(uintptr_t)(const AS3 bf16_t*)(Vs + (size_t)(4 * hf + tq) * HD +
                                                                  16 * ((lane >> 4) & 1) + 4 * tp);
  f32x16 st = attn_qk<HDT>(Ks, qf, 0, r, hf);
  for (int kt = 0; kt < nkt; ++kt) {
    f32x16 stn;
    if (kt + 1 < nkt) stn = attn_qk<HDT>(Ks, qf, kt + 1, r, hf);
    const bool h1 = kt * 32 + 16 < N;  // second 16-key half has keys (wave-uniform)
    // V^T fragments of tile kt (inline asm: see attn_qtile)
    bf16x4 lo[2][HDT], hi[2][HDT];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      if (s2 == 1 && !h1) break;
#pragma unroll
      for (int dt = 0; dt < HDT; ++dt) {
        const uint32_t va = vbase + (uint32_t)(((kt * 32 + 16 * s2) * HD + dt * 32) * 2);
        asm volatile("ds_read_b64_tr_b16 %0, %2\n\tds_read_b64_tr_b16 %1, %2 offset:%3"
                     : "=&v"(lo[s2][dt]), "=&v"(hi[s2][dt])
                     : "v"(va), "i"(16 * HD)
                     : "memory");
      }
    }
    if (kt * 32 + 32 > N) {  // mask padded keys of the last tile
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int key = kt * 32 + (i & 3) + 8 * (i >> 2) + 4 * hf;
        if (key >= N) st[i] = -INFINITY;
      }
    }
    float tmax = fmaxf(fmaxf(st[0], st[1]), st[2]);
#pragma unroll
    for (int i = 3; i < 15; i += 2) tmax = fmaxf(fmaxf(tmax, st[i]), st[i + 1]);
    tmax = xhalf_max(fmaxf(tmax, st[15]));
    const float mn = fmaxf(m, tmax);
    if (__any(mn > m)) {  // wave-uniform: rescale only when some running max moved
      const float alpha = __builtin_amdgcn_exp2f((m - mn) * scale_log2);
      l *= alpha;
#pragma unroll
      for (int dt = 0; dt < HDT; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[dt][i] *= alpha;
      m = mn;
    }
    const float msc = -m * scale_log2;
    bf16x8 pb[2];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float p = __builtin_amdgcn_exp2f(fmaf(st[8 * s2 + j], scale_log2, msc));
        l += p;
        pb[s2][j] = (short)f2bf(p);
      }
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int dt = 0; dt < HDT; ++dt) asm volatile("" : "+v"(lo[s2][dt]), "+v"(hi[s2][dt]));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      if (s2 == 1 && !h1) break;
#pragma unroll
      for (int dt = 0; dt < HDT; ++dt) {
        asm volatile("" : "+v"(lo[s2][dt]), "+v"(hi[s2][dt]));
        const bf16x8 vf = {lo[s2][dt][0], lo[s2][dt][1], lo[s2][dt][2], lo[s2][dt][3],
                           hi[s2][dt][0], hi[s2][dt][1], hi[s2][dt][2], hi[s2][dt][3]};
        acc[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pb[s2], acc[dt], 0, 0, 0);
      }
    }
    st = stn;
  }
  l = xhalf_sum(l);
  const float inv = 1.0f / l;
  if (orow) {
#pragma unroll
    for (int dt = 0; dt < HDT; ++dt) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        bf16x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = (short)f2bf(acc[dt][4 * g + e] * inv);
        *(bf16x4*)(orow + dt * 32 + 8 * g + 4 * hf) = o;
      }
    }
  }
}

// Chunked form for N <= 32 * NKT keys, used by the persistent kernel: the key
// tiles are taken CH at a time; a chunk's CH S^T tiles are computed first (CH
// independent MFMA chains), then one max over the chunk (one rescale of O per
// chunk after the first), one pass of exp2 / row sums / bf16 packing, then P V^T.
// Few, long MFMA and VALU phases per wave instead of one short chain per key
// tile, so the two waves of a SIMD overlap each other's phases.
// The next Q tile (qnext) is loaded into qn after the last chunk's
// exponentials, when the S^T registers are free: the loads overlap the P V^T phase.
// KT0 / KT1: the key tiles this call covers (default all NKT).  part != nullptr: instead of the
// normalised O row, store the unnormalised partial of row r -- part[0] = running max (raw score),
// part[1] = row sum, part[4 + d] = O numerator of head dim d -- for a later merge over key ranges.
template <int HDT, int NKT, int CH, bool PF = true, int KT0 = 0, int KT1 = NKT>
SDP_DEV void attn_qtile_chunked(const bf16_t* Ks, const bf16_t* Vs, const bf16x8 (&qf)[2 * HDT], int N,
                                float scale_log2, int lane, bf16_t* orow, const bf16_t* qnext,
                                bf16x8 (&qn)[2 * HDT], float* part = nullptr) {
  constexpr int HD = 32 * HDT;
  const int r = lane & 31, hf = lane >> 5;
  f32x16 acc[HDT];  // first written by the first P V^T MFMA (zero C operand): not live before
  float m = -INFINITY;
  f32x2 l2 = {0.f, 0.f};  // row sum, two partial sums
  const int gi = lane & 15, tq = gi >> 2, tp = gi & 3;
  const uint32_t vbase = (uint32_t)(uintptr_t)(const AS3 bf16_t*)(Vs + (size_t)(4 * hf + tq) * HD +
                                                                  16 * ((lane >> 4) & 1) + 4 * tp);
  const int kswz = (r >> 2) & 3;
  const char* kb0 = (const char*)(Ks + (size_t)r * HD) + 16 * ((hf) ^ kswz);
  const char* kb1 = (const char*)(Ks + (size_t)r * HD) + 16 * ((2 + hf) ^ kswz);
#pragma unroll
  for (int c0 = KT0; c0 < KT1; c0 += CH) {
    const int n = KT1 - c0 < CH ? KT1 - c0 : CH;  // compile-time after unrolling
    f32x16 st[CH];
#pragma unroll
    for (int t = 0; t < CH; ++t)
      if (t < n) {
        st[t] = attn_qk2<HDT>(kb0, kb1, qf, c0 + t);
        // pin the phase order (IR passes would otherwise sink work to its uses and
        // interleave the phases, multiplying the live registers)
        asm volatile("" : "+v"(st[t]));
      }
    if (c0 + n == NKT && NKT * 32 > N) {  // mask padded keys of the last tile
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int key = (NKT - 1) * 32 + (i & 3) + 8 * (i >> 2) + 4 * hf;
        if (key >= N) st[n - 1][i] = -INFINITY;
      }
    }
    float mx = -INFINITY;
#pragma unroll
    for (int t = 0; t < CH; ++t)
      if (t < n)
#pragma unroll
        for (int i = 0; i < 16; i += 2) mx = fmaxf(fmaxf(mx, st[t][i]), st[t][i + 1]);
    mx = xhalf_max(mx);
    if (c0 > KT0) {  // acc holds earlier chunks
      const float mn = fmaxf(m, mx);
      const float alpha = __builtin_amdgcn_exp2f((m - mn) * scale_log2);
      l2 *= alpha;
#pragma unroll
      for (int dt = 0; dt < HDT; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[dt][i] *= alpha;
      m = mn;
    } else {
      m = mx;
    }
    const float msc = -m * scale_log2;
    const f32x2 sl2 = {scale_log2, scale_log2}, msc2 = {msc, msc};
    bf16x8 pb[CH][2];
#pragma unroll
    for (int t = 0; t < CH; ++t)
      if (t < n) {
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          u32x4 pk;
#pragma unroll
          for (int j = 0; j < 8; j += 2) {
            // packed scale-and-subtract and packed row sum: 5 VALU per 2 elements
            const f32x2 a = f32x2{st[t][8 * s2 + j], st[t][8 * s2 + j + 1]} * sl2 + msc2;
            const f32x2 p2 = {__builtin_amdgcn_exp2f(a.x), __builtin_amdgcn_exp2f(a.y)};
            l2 += p2;
            pk[j >> 1] = pack_bf16x2(p2.x, p2.y);
          }
          pb[t][s2] = __builtin_bit_cast(bf16x8, pk);
        }
        asm volatile("" : "+v"(pb[t][0]), "+v"(pb[t][1]), "+v"(l2));  // one tile's exponentials at a time
      }
    if (PF && c0 + n == KT1) {
      asm volatile("" ::: "memory");
      attn_load_q<HDT>(qnext, hf, qn);
    }  // P complete before P V^T (bounds the live registers)
#pragma unroll
    for (int t = 0; t < CH; ++t) {
      if (t >= n) break;
      const int kt = c0 + t;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        if (kt == NKT - 1 && s2 == 1 && kt * 32 + 16 >= N) break;  // half past the keys (uniform)
        bf16x4 lo[HDT], hi[HDT];
#pragma unroll
        for (int dt = 0; dt < HDT; ++dt) {
          const uint32_t va = vbase + (uint32_t)(((kt * 32 + 16 * s2) * HD + dt * 32) * 2);
          asm volatile("ds_read_b64_tr_b16 %0, %2\n\tds_read_b64_tr_b16 %1, %2 offset:%3"
                       : "=&v"(lo[dt]), "=&v"(hi[dt])
                       : "v"(va), "i"(16 * HD)
                       : "memory");
        }
#pragma unroll
        for (int dt = 0; dt < HDT; ++dt) asm volatile("" : "+v"(lo[dt]), "+v"(hi[dt]));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int dt = 0; dt < HDT; ++dt) {
          asm volatile("" : "+v"(lo[dt]), "+v"(hi[dt]));
          const bf16x8 vf = {lo[dt][0], lo[dt][1], lo[dt][2], lo[dt][3], hi[dt][0], hi[dt][1], hi[dt][2], hi[dt][3]};
          if (kt == KT0 && s2 == 0) {
            const f32x16 z = {};
            acc[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pb[t][s2], z, 0, 0, 0);
          } else {
            acc[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pb[t][s2], acc[dt], 0, 0, 0);
          }
        }
      }
    }
  }
  const float l = xhalf_sum(l2.x + l2.y);
  if (part) {
    if (hf == 0) {
      part[0] = m;
      part[1] = l;
    }
#pragma unroll
    for (int dt = 0; dt < HDT; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *(f32x4*)(part + 4 + dt * 32 + 8 * g + 4 * hf) =
            f32x4{acc[dt][4 * g], acc[dt][4 * g + 1], acc[dt][4 * g + 2], acc[dt][4 * g + 3]};
    return;
  }
  const float inv = 1.0f / l;
  if (orow) {
#pragma unroll
    for (int dt = 0; dt < HDT; ++dt) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        bf16x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = (short)f2bf(acc[dt][4 * g + e] * inv);
        *(bf16x4*)(orow + dt * 32 + 8 * g + 4 * hf) = o;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// attn_fa2_bf16 — same math and MFMA forms as attn_fa_bf16, laid out so that TWO
// workgroups fit on a CU (one stages while the other computes):
//   * LDS holds K and V unpadded, NP16 = ceil(N/16)*16 rows each (N = 200, hd = 96:
//     2 x 39,936 B <= 80 KiB); both are filled by LDS-DMA (global_load_lds_dwordx4,
//     no VGPR staging).  K's 16-B chunk c of row r sits at c ^ ((r >> 2) & 3):
//     with a 192-B row pitch every ds_read_b128 lane group of the QK^T A-operand
//     read hits 16 distinct 4-bank slots; V's 192-B pitch is already conflict-free
//     for the 4-key x 32-d transposed reads.
//   * k_norm runs in place over the staged K rows (one LDS read + write), q_norm
//     on the Q fragments in registers.
//   * the 1/sqrt(hd) * log2(e) scale is folded into the exponent's FMA.
//   * keys >= NP16 are never read as V (the second 16-key half of a tile past N is
//     skipped); K rows in [NP16, NP32) alias the start of V (finite, masked).
//   * register budget 128 (4 waves / SIMD) for the 7-wave workgroups.
// Needs hd % 32 == 0 (whole 4-chunk swizzle groups).
// ---------------------------------------------------------------------------
// NKT > 0: each query tile runs the chunked single-max softmax of attn_fa4 over NKT key tiles
// (N <= 32 NKT; ATTN_CH2 tiles per chunk, no next-tile Q prefetch: one tile per wave) instead of
// the per-key-tile online softmax (NKT = 0, any N).
#ifndef ATTN_CH2
#define ATTN_CH2 3  // at 168 VGPRs (three waves on a SIMD): 4 spills at hd 96
#endif
template <int HDT, int NKT = 0>
__global__ __launch_bounds__(NKT > 0 ? 64 * (NKT + 2) : 576) __attribute__((amdgpu_waves_per_eu(NKT > 0 ? 3 : (HDT <= 3 ? 4 : 2)))) void attn_fa2_bf16(
    const bf16_t* __restrict__ QKV, int64_t ldq, bf16_t* __restrict__ O, int64_t ldo, int B, int N, int H,
    const float* __restrict__ gq, const float* __restrict__ bq, const float* __restrict__ gk,
    const float* __restrict__ bk, float eps, float scale_log2) {
  extern __shared__ __attribute__((aligned(16))) char sm[];
  constexpr int HD = 32 * HDT;  // head dim (hd % 32 == 0 on this path)
  constexpr int CPR = HD / 8;   // 16-B chunks per row
  const int NP16 = (N + 15) / 16 * 16;
  const int NP32 = (N + 31) / 32 * 32;
  bf16_t* Ks = (bf16_t*)sm;               // [NP16][HD] swizzled chunks
  bf16_t* Vs = Ks + (size_t)NP16 * HD;    // [NP16][HD] row-major
  // XCD-aware pair order: consecutive (b, h) pairs (which share QKV cache lines)
  // run on one XCD
  const int nwg = B * H, x = blockIdx.x;
  const int xcd = x & 7, qd = nwg >> 3, rem = nwg & 7;
  const int pair = (xcd < rem ? xcd * (qd + 1) : rem * (qd + 1) + (xcd - rem) * qd) + (x >> 3);
  const int b = pair / H, hh = pair % H;
  const int C = H * HD;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nwaves = blockDim.x >> 6;
  const bf16_t* base = QKV + (int64_t)b * N * ldq + hh * HD;

  // ---- K and V -> LDS by DMA ----
  {
    const AttnKV<HDT> kv(lane, ldq, C);
    kv.issue(base, (uint64_t)((int64_t)(N - 1) * ldq + 3 * C - hh * HD) * 2, (char*)Ks, (char*)Vs, NP16, ldq,
             wave, nwaves);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // ---- k_norm in place: 16 lanes per row (CPR <= 16 active) ----
  if (gk) {
    const int sub = tid & 15;
    const bool act = sub < CPR;
    for (int row = tid >> 4; row < NP16; row += nwaves * 4) {
      bf16x8* p = (bf16x8*)(Ks + (size_t)row * HD) + (act ? sub : 0);
      const bf16x8 raw = *p;
      float kv[8];
      float s = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        kv[e] = act ? bf2f((bf16_t)raw[e]) : 0.f;
        s += kv[e];
      }
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) s += __shfl_xor(s, o, 16);
      const float mean = s * (1.0f / HD);
      float ss = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float d = act ? kv[e] - mean : 0.f;
        ss += d * d;
      }
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 16);
      const float rstd = 1.0f / sqrtf(ss * (1.0f / HD) + eps);
      if (act) {
        const int c8 = (sub ^ ((row >> 2) & 3)) * 8;  // logical columns of this chunk
        bf16x8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = (short)f2bf((kv[e] - mean) * rstd * gk[c8 + e] + bk[c8 + e]);
        *p = o;
      }
    }
    __syncthreads();
  }

  const int r = lane & 31, hf = lane >> 5;
  const int nqt = NP32 / 32;
  if constexpr (NKT > 0) {
    // NKT + 2 waves: waves 0 .. NKT-2 one full query tile each; the last (partial) query tile's keys
    // split in three chunk-aligned ranges over waves NKT-1 .. NKT+1, so each SIMD runs ~2.3 tiles of
    // work instead of one SIMD running three; the three unnormalised partials meet in LDS.
    static_assert(NKT == 9 && ATTN_CH2 == 3, "key-split last tile assumes 9 key tiles in 3 chunks");
    constexpr int PP = HD + 4;  // partial row pitch (floats): m, l, pad, pad, O numerator
    const int nlast = N - (NKT - 1) * 32;  // rows of the last query tile
    float* part = (float*)(Vs + (size_t)NP16 * HD);  // [3][nlast][PP]
    const int qt = wave < NKT - 1 ? wave : NKT - 1;
    const int q = qt * 32 + r;
    const bool qok = q < N;
    bf16x8 qf[2 * HDT];
    attn_load_q<HDT>(base + (int64_t)(qok ? q : N - 1) * ldq, hf, qf);
    if (gq) attn_norm_q<HDT>(qf, qok, hf, gq, bq, eps);
    if (wave < NKT - 1) {
      bf16_t* orow = O + ((int64_t)b * N + q) * ldo + hh * HD;
      attn_qtile_chunked<HDT, NKT, ATTN_CH2, false>(Ks, Vs, qf, N, scale_log2, lane, orow, nullptr, qf);
    } else {
      const int sl = wave - (NKT - 1);
      float* pr = qok ? part + ((size_t)sl * nlast + r) * PP : nullptr;
      if (sl == 0)
        attn_qtile_chunked<HDT, NKT, ATTN_CH2, false, 0, 3>(Ks, Vs, qf, N, scale_log2, lane, nullptr, nullptr, qf, pr);
      else if (sl == 1)
        attn_qtile_chunked<HDT, NKT, ATTN_CH2, false, 3, 6>(Ks, Vs, qf, N, scale_log2, lane, nullptr, nullptr, qf, pr);
      else
        attn_qtile_chunked<HDT, NKT, ATTN_CH2, false, 6, 9>(Ks, Vs, qf, N, scale_log2, lane, nullptr, nullptr, qf, pr);
    }
    __syncthreads();
    if (wave == NKT - 1) {  // merge: O = sum_i 2^((m_i - M) s) acc_i / sum_i 2^((m_i - M) s) l_i
      constexpr int D4 = HD / 4;
      for (int i = lane; i < nlast * D4; i += 64) {
        const int row = i / D4, d4 = i - row * D4;
        const float* p0 = part + (size_t)row * PP;
        const float* p1 = p0 + (size_t)nlast * PP;
        const float* p2 = p1 + (size_t)nlast * PP;
        const float mx = fmaxf(fmaxf(p0[0], p1[0]), p2[0]);
        const float w0 = __builtin_amdgcn_exp2f((p0[0] - mx) * scale_log2);
        const float w1 = __builtin_amdgcn_exp2f((p1[0] - mx) * scale_log2);
        const float w2 = __builtin_amdgcn_exp2f((p2[0] - mx) * scale_log2);
        const float inv = 1.0f / (w0 * p0[1] + w1 * p1[1] + w2 * p2[1]);
        const f32x4 a0 = *(const f32x4*)(p0 + 4 + 4 * d4), a1 = *(const f32x4*)(p1 + 4 + 4 * d4),
                    a2 = *(const f32x4*)(p2 + 4 + 4 * d4);
        bf16x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = (short)f2bf((w0 * a0[e] + w1 * a1[e] + w2 * a2[e]) * inv);
        *(bf16x4*)(O + ((int64_t)b * N + (NKT - 1) * 32 + row) * ldo + hh * HD + 4 * d4) = o;
      }
    }
  } else {
    for (int qt = wave; qt < nqt; qt += nwaves) {
      const int q = qt * 32 + r;
      const bool qok = q < N;
      bf16x8 qf[2 * HDT];
      attn_load_q<HDT>(base + (int64_t)(qok ? q : N - 1) * ldq, hf, qf);
      if (gq) attn_norm_q<HDT>(qf, qok, hf, gq, bq, eps);
      bf16_t* orow = qok ? O + ((int64_t)b * N + q) * ldo + hh * HD : nullptr;
      attn_qtile<HDT>(Ks, Vs, qf, N, nqt, scale_log2, lane, orow);
    }
  }
}

static size_t attn_fa2_bytes(int N, int hd) { return (size_t)2 * ((N + 15) / 16 * 16) * hd * 2; }

static size_t attn_fa6_bytes(int N, int hd);
template <int HDT>
static int launch_attn_fa6(const void* QKV, int64_t ldq, void* O, int64_t ldo, int B, int N, int H,
                           const float* gq, const float* bq, const float* gk, const float* bk, float eps, float scale,
                           hipStream_t s);

template <int HDT>
static int launch_attn_fa2(const void* QKV, int64_t ldq, void* O, int64_t ldo, int B, int N, int H,
                           const float* gq, const float* bq, const float* gk, const float* bk, float eps, float scale,
                           hipStream_t s) {
  size_t bytes = attn_fa2_bytes(N, 32 * HDT);
  // one query tile per wave up to 9 tiles (N <= 288: XL's 260 tokens are 8 full tiles + 4 rows;
  // with 8 waves one wave did two tiles and set the block's time), else 8 waves looping; at exactly
  // 9 key tiles (XL) the chunked single-max softmax (hd <= 96: hd 128 would spill at 168 VGPRs)
  // with the last query tile's keys split over three more waves (11 in all)
  int waves = (N + 31) / 32;
  if (waves > 9) waves = 8;
  const bool split = waves == 9 && HDT <= 3;
  const void* fn = split ? (const void*)attn_fa2_bf16<HDT, HDT <= 3 ? 9 : 0> : (const void*)attn_fa2_bf16<HDT, 0>;
  if constexpr (HDT <= 3)
    if (split && attn_fa6_bytes(N, 32 * HDT) <= 160 * 1024)  // persistent form, K / V staging hidden
      return launch_attn_fa6<HDT>(QKV, ldq, O, ldo, B, N, H, gq, bq, gk, bk, eps, scale, s);
  if (split) {
    waves = 11;
    bytes += (size_t)3 * (N - 256) * (32 * HDT + 4) * 4;
  }
  if (bytes > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e != hipSuccess) return (int)e;
  }
  const float sl = scale * 1.4426950408889634f;
  const bf16_t* q = (const bf16_t*)QKV;
  bf16_t* o = (bf16_t*)O;
  void* args[] = {(void*)&q, (void*)&ldq, (void*)&o, (void*)&ldo, (void*)&B, (void*)&N, (void*)&H, (void*)&gq,
                  (void*)&bq, (void*)&gk, (void*)&bk, (void*)&eps, (void*)&sl};
  const hipError_t e = hipLaunchKernel(fn, dim3(B * H), dim3(64 * waves), args, bytes, s);
  if (e != hipSuccess) return (int)e;
  return SDP_CHECK_LAUNCH();
}

// k_norm (layers.py:237, :286) in place on 32 staged K rows row0 .. row0+31
// (swizzled image, see attn_qtile): lane (r, hf) normalises head dims
// [HD/2 * hf, HD/2 * (hf+1)) of row row0 + r; the halves meet by one permlane32
// swap.  g / be: k_norm gamma / beta (LDS).
template <int HDT>
SDP_DEV void attn_knorm32(bf16_t* Kd, int row0, int NP16, int lane, const float* g, const float* be, float eps) {
  constexpr int HD = 32 * HDT, NDS = HD / 16;
  const int r = lane & 31, hf = lane >> 5;
  const int row = row0 + r;
  const bool ok = row < NP16;  // same for both halves of a row
  bf16x8* kr = (bf16x8*)(Kd + (size_t)(ok ? row : 0) * HD);
  const int sw = (row >> 2) & 3;
  bf16x8 kv[NDS];
  f32x2 st = {0.f, 0.f};
#pragma unroll
  for (int i = 0; i < NDS; ++i) {
    kv[i] = kr[(NDS * hf + i) ^ sw];
    st = frag_stats(kv[i], st);
  }
  st.x = xhalf_sum(st.x);
  st.y = xhalf_sum(st.y);
  const float mean = st.x * (1.0f / HD);
  const float rstd = rsqrtf(fmaxf(st.y * (1.0f / HD) - mean * mean, 0.f) + eps);
  if (ok) {
#pragma unroll
    for (int i = 0; i < NDS; ++i) {
      const int c8 = (NDS * hf + i) * 8;
      kr[(NDS * hf + i) ^ sw] = frag_norm(kv[i], mean, rstd, g + c8, be + c8);
    }
  }
}

// ---------------------------------------------------------------------------
// attn_fa4_bf16 — two persistent 4-wave workgroups per CU, each with ONE K/V
// buffer (80 KiB): a workgroup loads a pair (LDS-DMA), k-norms it and computes it
// while the other workgroup of the CU is in a different phase, so the two waves
// of a SIMD (one per workgroup) are not in lockstep and one's MFMA phase overlaps
// the other's VALU or load phase.  Wave w computes query tiles w and w + 4
// (slots 0, 1) with the chunked whole-tile softmax; each slot prefetches the
// next slot's Q fragments (the next pair's slot 0 after slot 1).
// LDS: (K + V) x NP16 x HD x 2 B + 4 x HD x 4 B  (N = 200, hd = 96: 81,408 B).
// ---------------------------------------------------------------------------
#ifdef SDP_GEMM_STAMPS
// Diagnostic build only (tools/attn_stamps.py): per workgroup, per pair j < 8, the shader clock
// (s_memtime) of waves 0 and 3 at: pair start, K/V landed (after the barrier), k-norm done,
// slot 0 done, slot 1 done.  [wg][wave 0|3][j][5]
__device__ unsigned long long g_attn_stamps[1024 * 2 * 8 * 5];
#define SDP_ASTAMP(j, k)                                                                               \
  do {                                                                                                 \
    if ((wave == 0 || wave == 3) && lane == 0 && (j) < 8 && blockIdx.x < 1024)                         \
      g_attn_stamps[(((int64_t)blockIdx.x * 2 + (wave == 3)) * 8 + (j)) * 5 + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
// attn_fa5: waves 0 (a compute wave) and 7 (the producer) in the same slots
#define SDP_ASTAMP5(j, k)                                                                              \
  do {                                                                                                 \
    if ((wave == 0 || wave == 7) && lane == 0 && (j) < 8 && blockIdx.x < 1024)                         \
      g_attn_stamps[(((int64_t)blockIdx.x * 2 + (wave == 7)) * 8 + (j)) * 5 + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
// attn_fa6: waves 0 (a compute wave) and 11 (the producer)
#define SDP_ASTAMP6(j, k)                                                                              \
  do {                                                                                                 \
    if ((wave == 0 || wave == 11) && lane == 0 && (j) < 8 && blockIdx.x < 1024)                        \
      g_attn_stamps[(((int64_t)blockIdx.x * 2 + (wave == 11)) * 8 + (j)) * 5 + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define SDP_ASTAMP(j, k) do {} while (0)
#define SDP_ASTAMP5(j, k) do {} while (0)
#define SDP_ASTAMP6(j, k) do {} while (0)
#endif
template <int HDT, int NKT>
__global__ __launch_bounds__(256, 2) void attn_fa4_bf16(const bf16_t* __restrict__ QKV, int64_t ldq,
                                                     bf16_t* __restrict__ O, int64_t ldo, int B, int N, int H,
                                                     const float* __restrict__ gq, const float* __restrict__ bq,
                                                     const float* __restrict__ gk, const float* __restrict__ bk,
                                                     float eps, float scale_log2) {
  extern __shared__ __attribute__((aligned(16))) char sm[];
  constexpr int HD = 32 * HDT;
  const int NP16 = (N + 15) / 16 * 16;
  bf16_t* const Ks = (bf16_t*)sm;
  bf16_t* const Vs = Ks + (size_t)NP16 * HD;
  float* const prm = (float*)(sm + (size_t)2 * NP16 * HD * sizeof(bf16_t));  // gq | bq | gk | bk
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int npairs = B * H, G = gridDim.x, x = blockIdx.x;
  const int nj = (npairs - x + G - 1) / G;
  if (nj <= 0) return;
  const int C = H * HD;
  const bool norm = gq != nullptr;
  if (norm) {
    for (int i = tid; i < 4 * HD; i += 256) {
      const int k = i / HD, d = i - k * HD;
      prm[i] = (k == 0 ? gq : k == 1 ? bq : k == 2 ? gk : bk)[d];
    }
  }
  // pair order: virtual id x + jG through the XCD-contiguous remap (G % 8 == 0)
  auto pair_of = [&](int j) {
    const int v = x + j * G;
    const int xcd = v & 7, qd = npairs >> 3, rem = npairs & 7;
    return (xcd < rem ? xcd * (qd + 1) : rem * (qd + 1) + (xcd - rem) * qd) + (v >> 3);
  };
  auto qkv_base = [&](int pair) {
    const int b = pair / H, hh = pair - (pair / H) * H;
    return QKV + (int64_t)b * N * ldq + hh * HD;
  };
  const AttnKV<HDT> kv(lane, ldq, C);
  auto stage = [&](int pair) {
    const int hh = pair - (pair / H) * H;
    kv.issue(qkv_base(pair), (uint64_t)((int64_t)(N - 1) * ldq + 3 * C - hh * HD) * 2, (char*)Ks, (char*)Vs, NP16,
             ldq, wave, 4);
  };
  const int r = lane & 31, hf = lane >> 5;
  // Every wave computes two query-tile slots per pair; a slot past the last tile
  // (e.g. tile 7 at N = 200) is computed on row N-1 and not stored: it sits on a
  // SIMD whose partner slots are real, so it costs no time on the critical path,
  // and it keeps the Q prefetch unconditional (no register merges that would make
  // the compiler wait for the loads).
  const int q0 = wave * 32 + r, q1 = (wave + 4) * 32 + r;
  const bool ok0 = q0 < N, ok1 = q1 < N;
  const int64_t off0 = (int64_t)(ok0 ? q0 : N - 1) * ldq, off1 = (int64_t)(ok1 ? q1 : N - 1) * ldq;
  bf16x8 qa[2 * HDT], qb[2 * HDT];
  int pair = pair_of(0);
  attn_load_q<HDT>(qkv_base(pair) + off0, hf, qa);
  for (int j = 0; j < nj; ++j) {
    const int nxt = j + 1 < nj ? pair_of(j + 1) : pair;  // last pair: a harmless re-load
    SDP_ASTAMP(j, 0);
    stage(pair);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    SDP_ASTAMP(j, 1);
    if (norm) {
#pragma unroll
      for (int rr = 0; rr < 2; ++rr)
        if (32 * (wave + 4 * rr) < NP16) attn_knorm32<HDT>(Ks, 32 * (wave + 4 * rr), NP16, lane, prm + 2 * HD, prm + 3 * HD, eps);
      __syncthreads();
    }
    SDP_ASTAMP(j, 2);
    const int b = pair / H, hh = pair - (pair / H) * H;
    bf16_t* obase = O + (int64_t)b * N * ldo + hh * HD;
    // slot 0 (query tile w), prefetching slot 1's Q
    if (norm) attn_norm_q<HDT>(qa, ok0, hf, prm, prm + HD, eps);
    attn_qtile_chunked<HDT, NKT, (HDT <= 3 ? ATTN_CH : 4)>(Ks, Vs, qa, N, scale_log2, lane, ok0 ? obase + q0 * ldo : nullptr,
                                          qkv_base(pair) + off1, qb);
    SDP_ASTAMP(j, 3);
    // slot 1 (query tile w + 4), prefetching the next pair's slot 0
    if (norm) attn_norm_q<HDT>(qb, ok1, hf, prm, prm + HD, eps);
    attn_qtile_chunked<HDT, NKT, (HDT <= 3 ? ATTN_CH : 4)>(Ks, Vs, qb, N, scale_log2, lane, ok1 ? obase + q1 * ldo : nullptr,
                                          qkv_base(nxt) + off0, qa);
    SDP_ASTAMP(j, 4);
    pair = nxt;
    __syncthreads();  // every wave is done with K / V before the next pair's DMA
  }
}

#ifdef SDP_DIAG  // attn_fa5: opt-in tier 6, slower in the model than fa4 (round 5); diagnostic build only
// ---------------------------------------------------------------------------
// attn_fa5_bf16 — one persistent 8-wave workgroup per CU with K / V double-buffered in LDS
// (2 x (K + V) x NP16 x HD x 2 B + gamma / beta; N = 200, hd = 96: 161,280 of 163,840 B).
// Waves 0..6 own query tiles 0..6 (N <= 224: one 32-row tile each, none of them padding -- fa4
// computes 8 slots for 7 tiles) and compute pair j out of buffer j & 1 with the chunked
// whole-tile softmax, prefetching their next Q tile.  Wave 7 is the producer: it stages pair j + 1
// into the other buffer (buffer LDS-DMA, K then V) while pair j computes, so the staging latency
// hides behind a whole pair.  After the pair's barrier all eight waves k-normalise the next K (32
// rows each, ~2.2k cycles) before a second barrier (fa4: stage -> barrier -> k-norm -> barrier ->
// compute, per pair, two workgroups per CU).  The producer k-normalising alone (one barrier per
// pair) measured 129 vs 91-97 us: one wave's k-norm of 208 rows outlasts the compute.
// ---------------------------------------------------------------------------
template <int HDT, int NKT>
__global__ __launch_bounds__(512) void attn_fa5_bf16(const bf16_t* __restrict__ QKV, int64_t ldq,
                                                  bf16_t* __restrict__ O, int64_t ldo, int B, int N, int H,
                                                  const float* __restrict__ gq, const float* __restrict__ bq,
                                                  const float* __restrict__ gk, const float* __restrict__ bk,
                                                  float eps, float scale_log2) {
  extern __shared__ __attribute__((aligned(16))) char sm[];
  constexpr int HD = 32 * HDT;
  const int NP16 = (N + 15) / 16 * 16;
  const size_t kvb = (size_t)NP16 * HD * sizeof(bf16_t);  // bytes of one K (or V) image
  float* const prm = (float*)(sm + 4 * kvb);              // gq | bq | gk | bk
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int npairs = B * H, G = gridDim.x, x = blockIdx.x;
  const int nj = (npairs - x + G - 1) / G;
  if (nj <= 0) return;
  const int C = H * HD;
  const bool norm = gq != nullptr;
  if (norm) {
    for (int i = tid; i < 4 * HD; i += 512) {
      const int k = i / HD, d = i - k * HD;
      prm[i] = (k == 0 ? gq : k == 1 ? bq : k == 2 ? gk : bk)[d];
    }
  }
  auto pair_of = [&](int j) {  // XCD-contiguous pair order, as attn_fa4 (G % 8 == 0)
    const int v = x + j * G;
    const int xcd = v & 7, qd = npairs >> 3, rem = npairs & 7;
    return (xcd < rem ? xcd * (qd + 1) : rem * (qd + 1) + (xcd - rem) * qd) + (v >> 3);
  };
  auto qkv_base = [&](int pair) {
    const int b = pair / H, hh = pair - (pair / H) * H;
    return QKV + (int64_t)b * N * ldq + hh * HD;
  };
  auto kbuf = [&](int i) { return (bf16_t*)(sm + (size_t)(2 * i) * kvb); };
  auto vbuf = [&](int i) { return (bf16_t*)(sm + (size_t)(2 * i + 1) * kvb); };
  const bool producer = wave == 7;
  const AttnKV<HDT> kv(lane, ldq, C);
  // producer: pair -> buffer i (K units, then V units), all landed before it joins the barrier
  auto produce = [&](int pair, int i) {
    const int hh = pair - (pair / H) * H;
    kv.issue(qkv_base(pair), (uint64_t)((int64_t)(N - 1) * ldq + 3 * C - hh * HD) * 2, (char*)kbuf(i), (char*)vbuf(i),
             NP16, ldq, 0, 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };
  const int r = lane & 31, hf = lane >> 5;
  const bool has_tile = !producer && wave * 32 < N;
  const int q0 = wave * 32 + r;
  const bool ok0 = q0 < N;
  const int64_t off0 = (int64_t)(ok0 ? q0 : N - 1) * ldq;
  bf16x8 qa[2 * HDT], qb[2 * HDT];
  int pair = pair_of(0);
  // barrier without the vmcnt(0) of __syncthreads: a compute wave's O stores and Q prefetch
  // stay in flight across it (the producer has waited for its DMA; LDS accesses are retired)
  auto barrier = [] {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  // k-norm of buffer i by all eight waves, 32 rows each, between two barriers
  auto knorm_all = [&](int i) {
    if (32 * wave < NP16) attn_knorm32<HDT>(kbuf(i), 32 * wave, NP16, lane, prm + 2 * HD, prm + 3 * HD, eps);
  };
  if (producer) produce(pair, 0);
  else if (has_tile) attn_load_q<HDT>(qkv_base(pair) + off0, hf, qa);
  __syncthreads();
  if (norm) {
    knorm_all(0);
    barrier();
  }
  for (int j = 0; j < nj; ++j) {
    const int nxt = j + 1 < nj ? pair_of(j + 1) : pair;  // last pair: a harmless re-load
    SDP_ASTAMP5(j, 0);
    if (producer) {
      if (j + 1 < nj) produce(nxt, (j + 1) & 1);
    } else if (has_tile) {
      const int b = pair / H, hh = pair - (pair / H) * H;
      bf16_t* obase = O + (int64_t)b * N * ldo + hh * HD;
      if (norm) attn_norm_q<HDT>(qa, ok0, hf, prm, prm + HD, eps);
      attn_qtile_chunked<HDT, NKT, (HDT <= 3 ? ATTN_CH : 4)>(kbuf(j & 1), vbuf(j & 1), qa, N, scale_log2, lane,
                                                             ok0 ? obase + q0 * ldo : nullptr, qkv_base(nxt) + off0, qb);
#pragma unroll
      for (int s = 0; s < 2 * HDT; ++s) qa[s] = qb[s];
    }
    pair = nxt;
    SDP_ASTAMP5(j, 1);
    barrier();  // pair j's buffer free, pair j + 1's staged
    SDP_ASTAMP5(j, 2);
    if (norm && j + 1 < nj) {
      knorm_all((j + 1) & 1);
      SDP_ASTAMP5(j, 3);
      barrier();
    }
    SDP_ASTAMP5(j, 4);
  }
}

#endif  // SDP_DIAG (attn_fa5)
// ---------------------------------------------------------------------------
// attn_fa6_bf16 — the XL shape (256 < N <= 288, 9 key tiles, hd <= 96): one persistent 12-wave
// workgroup per CU.  A whole head does not fit twice in LDS (N = 260, hd = 96: K or V 52,224 B),
// but three K / V images do, so the head is staged in two halves that each hide behind a phase:
//   phase 1: waves 0..8 k-normalise K_j (32 rows each) while V_j lands (DMA issued at the end of
//            pair j-1), waves 9..10 merge pair j-1's last-tile partials, every compute wave loads
//            its Q fragments;
//   phase 2: waves 0..7 compute query tiles 0..7 and waves 8..10 the last (partial) tile over key
//            tiles 0-2 / 3-5 / 6-8 (attn_fa2's split), while the producer (wave 11) stages K_{j+1}
//            into the spare image.
// The three images rotate (K_j's image takes V_{j+1}, V_j's becomes the spare): two barriers per
// pair, no staging or launch on the critical path except V's DMA behind the k-norm.
// LDS: 3 x NP16 x HD x 2 B + gamma / beta + 3 x nlast x (HD + 4) x 4 B (N = 260, hd = 96: 163,008 B).
// ---------------------------------------------------------------------------
template <int HDT>
__global__ __launch_bounds__(768) __attribute__((amdgpu_waves_per_eu(3))) void attn_fa6_bf16(
    const bf16_t* __restrict__ QKV, int64_t ldq, bf16_t* __restrict__ O, int64_t ldo, int B, int N, int H,
    const float* __restrict__ gq, const float* __restrict__ bq, const float* __restrict__ gk,
    const float* __restrict__ bk, float eps, float scale_log2) {
  extern __shared__ __attribute__((aligned(16))) char sm[];
  constexpr int NKT = 9, HD = 32 * HDT, PP = HD + 4, D4 = HD / 4;
  static_assert(ATTN_CH2 == 3, "the last tile's key ranges are whole chunks of 3 key tiles");
  const int NP16 = (N + 15) / 16 * 16;
  const size_t kvb = (size_t)NP16 * HD * sizeof(bf16_t);  // bytes of one K (or V) image
  float* const prm = (float*)(sm + 3 * kvb);              // gq | bq | gk | bk
  float* const part = prm + 4 * HD;                       // [3][nlast][PP]
  const int nlast = N - (NKT - 1) * 32;
  // wave index made scalar: the producer / compute / merge branches are then uniform to the
  // compiler, and nothing staged under them needs a waterfall loop
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int npairs = B * H, G = gridDim.x, x = blockIdx.x;
  const int nj = (npairs - x + G - 1) / G;
  if (nj <= 0) return;
  const int C = H * HD;
  const bool norm = gq != nullptr;
  if (norm) {
    for (int i = tid; i < 4 * HD; i += 768) {
      const int k = i / HD, d = i - k * HD;
      prm[i] = (k == 0 ? gq : k == 1 ? bq : k == 2 ? gk : bk)[d];
    }
  }
  auto pair_of = [&](int j) {  // XCD-contiguous pair order, as attn_fa4
    const int v = x + j * G;
    const int xcd = v & 7, qd = npairs >> 3, rem = npairs & 7;
    return (xcd < rem ? xcd * (qd + 1) : rem * (qd + 1) + (xcd - rem) * qd) + (v >> 3);
  };
  auto qkv_base = [&](int pair) {
    const int b = pair / H, hh = pair - (pair / H) * H;
    return QKV + (int64_t)b * N * ldq + hh * HD;
  };
  auto img = [&](int i) { return (bf16_t*)(sm + (size_t)i * kvb); };
  const bool producer = wave == NKT + 2;
  // (the DMA offsets are rebuilt per stage: kept live they cost the compute waves registers)
  auto stage_k = [&](int pair_, int i_) {
    // pair / image are wave-uniform; say so, or the DMA's resource and M0 get waterfall loops
    const int pair = __builtin_amdgcn_readfirstlane(pair_), i = __builtin_amdgcn_readfirstlane(i_);
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const AttnKV<HDT> kv(ln, ldq, C);
    const int hh = pair - (pair / H) * H;
    kv.template issue<true, false>(qkv_base(pair), (uint64_t)((int64_t)(N - 1) * ldq + 3 * C - hh * HD) * 2,
                                   (char*)img(i), nullptr, NP16, ldq, 0, 1);
  };
  auto stage_v = [&](int pair_, int i_) {
    // pair / image are wave-uniform; say so, or the DMA's resource and M0 get waterfall loops
    const int pair = __builtin_amdgcn_readfirstlane(pair_), i = __builtin_amdgcn_readfirstlane(i_);
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const AttnKV<HDT> kv(ln, ldq, C);
    const int hh = pair - (pair / H) * H;
    kv.template issue<false, true>(qkv_base(pair), (uint64_t)((int64_t)(N - 1) * ldq + 3 * C - hh * HD) * 2,
                                   nullptr, (char*)img(i), NP16, ldq, 0, 1);
  };
  // barrier without the vmcnt(0) of __syncthreads (as attn_fa5: the producer waits for its DMA)
  auto barrier = [] {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  // last tile of `pair` from the three partials: O = sum 2^((m_i - M) s) acc_i / sum 2^((m_i - M) s) l_i;
  // waves 9 and 10 share the nlast x HD outputs
  auto merge = [&](int pair) {
    const int b = pair / H, hh = pair - (pair / H) * H;
    int ln = lane;
    asm volatile("" : "+v"(ln));
    for (int i = ln + 64 * (wave - NKT); i < nlast * D4; i += 128) {
      const int row = i / D4, d4 = i - row * D4;
      const float* p0 = part + (size_t)row * PP;
      const float* p1 = p0 + (size_t)nlast * PP;
      const float* p2 = p1 + (size_t)nlast * PP;
      const float mx = fmaxf(fmaxf(p0[0], p1[0]), p2[0]);
      const float w0 = __builtin_amdgcn_exp2f((p0[0] - mx) * scale_log2);
      const float w1 = __builtin_amdgcn_exp2f((p1[0] - mx) * scale_log2);
      const float w2 = __builtin_amdgcn_exp2f((p2[0] - mx) * scale_log2);
      const float inv = 1.0f / (w0 * p0[1] + w1 * p1[1] + w2 * p2[1]);
      const f32x4 a0 = *(const f32x4*)(p0 + 4 + 4 * d4), a1 = *(const f32x4*)(p1 + 4 + 4 * d4),
                  a2 = *(const f32x4*)(p2 + 4 + 4 * d4);
      bf16x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = (short)f2bf((w0 * a0[e] + w1 * a1[e] + w2 * a2[e]) * inv);
      *(bf16x4*)(O + ((int64_t)b * N + (NKT - 1) * 32 + row) * ldo + hh * HD + 4 * d4) = o;
    }
  };
  const int r = lane & 31;
  const int qt = wave < NKT - 1 ? wave : NKT - 1;  // waves 8..10: the last tile
  const int q0 = qt * 32 + r;
  const bool ok0 = q0 < N;
  const int64_t off0 = (int64_t)(ok0 ? q0 : N - 1) * ldq;
  bf16x8 qa[2 * HDT];
  int ik = 0, iv = 1, is = 2;  // images holding K_j, V_j and the spare
  int pair = pair_of(0), prev = pair;
  if (producer) {
    stage_k(pair, ik);
    stage_v(pair, iv);
  }
  for (int j = 0; j < nj; ++j) {
    const int nxt = j + 1 < nj ? pair_of(j + 1) : pair;
    SDP_ASTAMP6(j, 0);
    if (producer) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // V_j (and at j = 0, K_0) landed
      SDP_ASTAMP6(j, 1);
      if (j == 0) barrier();                             // K_0 and gamma / beta visible
    } else {
      if (j == 0) barrier();
      if (j > 0 && wave >= NKT) merge(prev);
      if (norm && 32 * wave < NP16) attn_knorm32<HDT>(img(ik), 32 * wave, NP16, lane, prm + 2 * HD, prm + 3 * HD, eps);
      SDP_ASTAMP6(j, 1);
    }
    barrier();  // K_j normalised, V_j landed, pair j-1's partials consumed
    SDP_ASTAMP6(j, 2);
    if (producer) {
      if (j + 1 < nj) {
        stage_k(nxt, is);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      SDP_ASTAMP6(j, 3);
    } else {
      // lane-derived values re-made opaque each pair: hoisted out of the loop they stay live
      // through the compute (masks, LDS lane offsets) and push it past 168 VGPRs
      int ln = lane;
      asm volatile("" : "+v"(ln));
      const int b = pair / H, hh = pair - (pair / H) * H;
      attn_load_q<HDT>(qkv_base(pair) + off0, ln >> 5, qa);
      if (norm) attn_norm_q<HDT>(qa, ok0, ln >> 5, prm, prm + HD, eps);
      if (wave < NKT - 1) {
        bf16_t* orow = O + ((int64_t)b * N + q0) * ldo + hh * HD;
        attn_qtile_chunked<HDT, NKT, ATTN_CH2, false>(img(ik), img(iv), qa, N, scale_log2, ln, orow, nullptr, qa);
      } else {
        const int sl = wave - (NKT - 1);
        float* pr = ok0 ? part + ((size_t)sl * nlast + (ln & 31)) * PP : nullptr;
        if (sl == 0)
          attn_qtile_chunked<HDT, NKT, ATTN_CH2, false, 0, 3>(img(ik), img(iv), qa, N, scale_log2, ln, nullptr, nullptr, qa, pr);
        else if (sl == 1)
          attn_qtile_chunked<HDT, NKT, ATTN_CH2, false, 3, 6>(img(ik), img(iv), qa, N, scale_log2, ln, nullptr, nullptr, qa, pr);
        else
          attn_qtile_chunked<HDT, NKT, ATTN_CH2, false, 6, 9>(img(ik), img(iv), qa, N, scale_log2, ln, nullptr, nullptr, qa, pr);
      }
    }
    if (!producer) SDP_ASTAMP6(j, 3);
    barrier();  // K_j / V_j images free, K_{j+1} landed, pair j's partials written
    SDP_ASTAMP6(j, 4);
    if (producer && j + 1 < nj) stage_v(nxt, ik);
    const int t = ik;
    ik = is;
    is = iv;
    iv = t;
    prev = pair;
    pair = nxt;
  }
  if (!producer && wave >= NKT) merge(prev);
}

static size_t attn_fa6_bytes(int N, int hd) {
  const size_t np16 = (size_t)(N + 15) / 16 * 16;
  return 3 * np16 * hd * 2 + (size_t)16 * hd + (size_t)3 * (N > 256 ? N - 256 : 0) * (hd + 4) * 4;
}

template <int HDT>
static int launch_attn_fa6(const void* QKV, int64_t ldq, void* O, int64_t ldo, int B, int N, int H,
                           const float* gq, const float* bq, const float* gk, const float* bk, float eps, float scale,
                           hipStream_t s) {
  if (N <= 256 || N > 288) return (int)hipErrorInvalidValue;  // 9 key tiles only
  const size_t bytes = attn_fa6_bytes(N, 32 * HDT);
  const void* fn = (const void*)attn_fa6_bf16<HDT>;
  hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
  if (e != hipSuccess) return (int)e;
  int dev = 0, ncu = 256;
  (void)hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0) ncu = 256;
  int grid = ncu / 8 * 8;  // one workgroup per CU (LDS)
  if (grid < 8) grid = 8;
  if (grid > B * H) grid = B * H;
  const float sl = scale * 1.4426950408889634f;
  const bf16_t* q = (const bf16_t*)QKV;
  bf16_t* o = (bf16_t*)O;
  void* args[] = {(void*)&q, (void*)&ldq, (void*)&o, (void*)&ldo, (void*)&B, (void*)&N, (void*)&H, (void*)&gq,
                  (void*)&bq, (void*)&gk, (void*)&bk, (void*)&eps, (void*)&sl};
  e = hipLaunchKernel(fn, dim3(grid), dim3(768), args, bytes, s);
  if (e != hipSuccess) return (int)e;
  return SDP_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------
// attn_fs_bf16 — streaming flash attention (the training kernels' structure, csrc/attn_train.hip):
// workgroup = (b, h, <= 3 query tiles) + one producer wave.  The producer streams the head's
// 32-row K / V tiles through a double-buffered LDS ring (padded rows, LD = HD + 8): lane l loads
// row l & 31 of K (l < 32) or V, all CPR 16-B chunks in flight at once, k-normalises its K row in
// registers (one-pass fp32 statistics, as attn_knorm32) and stores it; one barrier per key tile.
// Compute wave w owns query tile grp * qtw + w: q-norm on its fragments, then the online softmax
// over the key tiles as they arrive (S^T = K Q^T and O^T += V^T P^T in the swapped 32x32x16 form,
// exp2 argument folded into one FMA).  LDS 26 KiB per workgroup at hd = 96, so several workgroups
// share a CU and no K / V staging phase stands alone (attn_fa2 stages the whole head first).
// ---------------------------------------------------------------------------
template <int HDT>
__global__ __launch_bounds__(256, 2) void attn_fs_bf16(const bf16_t* __restrict__ QKV, int64_t ldq,
                                                    bf16_t* __restrict__ O, int64_t ldo, int N, int H, int qtw,
                                                    int groups, const float* __restrict__ gq,
                                                    const float* __restrict__ bq, const float* __restrict__ gk,
                                                    const float* __restrict__ bk, float eps, float scale_log2) {
  constexpr int HD = 32 * HDT, LD = HD + 8, CPR = HD / 8, NDS = HD / 16;
  __shared__ __attribute__((aligned(16))) bf16_t Kr[2][32 * LD];
  __shared__ __attribute__((aligned(16))) bf16_t Vr[2][32 * LD];
  __shared__ __attribute__((aligned(16))) float prm[2 * HD];  // k_norm gamma | beta
  const int bh = blockIdx.x / groups, grp = blockIdx.x - bh * groups;
  const int b = bh / H, hh = bh - b * H;
  const int C = H * HD;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nkt = (N + 31) / 32;
  const bf16_t* base = QKV + (int64_t)b * N * ldq + hh * HD;
  const bool norm = gq != nullptr;
  if (wave == qtw) {  // producer
    if (norm)
      for (int i = lane; i < 2 * HD; i += 64) prm[i] = i < HD ? gk[i] : bk[i - HD];
    const int mtx = lane >> 5, row = lane & 31;
    bf16x8 pv[CPR];
    auto p_load = [&](int kt) {
      const int kr = kt * 32 + row;
      const bf16_t* src = base + (int64_t)(kr < N ? kr : N - 1) * ldq + (mtx + 1) * C;
#pragma unroll
      for (int u = 0; u < CPR; ++u) pv[u] = *(const bf16x8*)(src + 8 * u);
      if (kr >= N)
#pragma unroll
        for (int u = 0; u < CPR; ++u) pv[u] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    };
    auto p_store = [&](int buf) {
      if (norm && mtx == 0) {
        f32x2 st = {0.f, 0.f};
#pragma unroll
        for (int u = 0; u < CPR; ++u) st = frag_stats(pv[u], st);
        const float mean = st.x * (1.0f / HD);
        const float rstd = rsqrtf(fmaxf(st.y * (1.0f / HD) - mean * mean, 0.f) + eps);
#pragma unroll
        for (int u = 0; u < CPR; ++u) pv[u] = frag_norm(pv[u], mean, rstd, prm + 8 * u, prm + HD + 8 * u);
      }
      bf16_t* dst = (mtx == 0 ? &Kr[buf][0] : &Vr[buf][0]) + row * LD;
#pragma unroll
      for (int u = 0; u < CPR; ++u) *(bf16x8*)(dst + 8 * u) = pv[u];
    };
    p_load(0);
    p_store(0);  // (prm was written by this wave: its LDS accesses are in order)
    __syncthreads();
    for (int kt = 0; kt < nkt; ++kt) {
      if (kt + 1 < nkt) {
        p_load(kt + 1);
        p_store((kt & 1) ^ 1);  // last read in iteration kt - 1, whose barrier has passed
      }
      __syncthreads();
    }
    return;
  }
  const int r = lane & 31, hf = lane >> 5;
  const int qt = grp * qtw + wave;
  const bool active = qt < nkt;
  const int q = qt * 32 + r;
  const bool qok = active && q < N;
  bf16x8 qf[2 * HDT];
  attn_load_q<HDT>(base + (int64_t)(q < N ? q : N - 1) * ldq, hf, qf);
  if (norm) attn_norm_q<HDT>(qf, qok, hf, gq, bq, eps);
  f32x16 acc[HDT];
#pragma unroll
  for (int dt = 0; dt < HDT; ++dt)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[dt][i] = 0.f;
  float m = -INFINITY;
  f32x2 l2 = {0.f, 0.f};
  const f32x2 sl2 = {scale_log2, scale_log2};
  const int gi = lane & 15, tq = gi >> 2, tp = gi & 3;
  __syncthreads();
  for (int kt = 0; kt < nkt; ++kt) {
    if (active) {
      const bf16_t* Kt = Kr[kt & 1];
      const bf16_t* Vt = Vr[kt & 1];
      f32x16 st;
#pragma unroll
      for (int i = 0; i < 16; ++i) st[i] = 0.f;
      const bf16_t* krow = Kt + (size_t)r * LD + 8 * hf;
#pragma unroll
      for (int s2 = 0; s2 < NDS; ++s2)
        st = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*(const bf16x8*)(krow + 16 * s2), qf[s2], st, 0, 0, 0);
      if (kt * 32 + 32 > N) {  // padded keys of the last tile
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if (kt * 32 + (i & 3) + 8 * (i >> 2) + 4 * hf >= N) st[i] = -INFINITY;
      }
      float tmax = fmaxf(fmaxf(st[0], st[1]), st[2]);
#pragma unroll
      for (int i = 3; i < 15; i += 2) tmax = fmaxf(fmaxf(tmax, st[i]), st[i + 1]);
      tmax = xhalf_max(fmaxf(tmax, st[15]));
      const float mn = fmaxf(m, tmax);
      if (__any(mn > m)) {  // wave-uniform: rescale only when some running max moved
        const float alpha = __builtin_amdgcn_exp2f((m - mn) * scale_log2);
        l2 *= alpha;
#pragma unroll
        for (int dt = 0; dt < HDT; ++dt)
#pragma unroll
          for (int i = 0; i < 16; ++i) acc[dt][i] *= alpha;
        m = mn;
      }
      const float msc = -m * scale_log2;
      const f32x2 msc2 = {msc, msc};
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        u32x4 pk;
#pragma unroll
        for (int j = 0; j < 8; j += 2) {
          const f32x2 a = f32x2{st[8 * s2 + j], st[8 * s2 + j + 1]} * sl2 + msc2;
          const f32x2 p2 = {__builtin_amdgcn_exp2f(a.x), __builtin_amdgcn_exp2f(a.y)};
          l2 += p2;
          pk[j >> 1] = pack_bf16x2(p2.x, p2.y);
        }
        const bf16x8 pb = __builtin_bit_cast(bf16x8, pk);
#pragma unroll
        for (int dt = 0; dt < HDT; ++dt) {
          const bf16_t* vb = Vt + (size_t)(16 * s2 + 4 * hf + tq) * LD + dt * 32 + 16 * ((lane >> 4) & 1) + 4 * tp;
          const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)vb);
          const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(vb + 8 * LD));
          const bf16x8 vf = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          acc[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pb, acc[dt], 0, 0, 0);
        }
      }
    }
    __syncthreads();
  }
  if (!qok) return;
  const float inv = 1.0f / xhalf_sum(l2.x + l2.y);
  bf16_t* orow = O + ((int64_t)b * N + q) * ldo + hh * HD;
#pragma unroll
  for (int dt = 0; dt < HDT; ++dt)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      bf16x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = (short)f2bf(acc[dt][4 * g + e] * inv);
      *(bf16x4*)(orow + dt * 32 + 8 * g + 4 * hf) = o;
    }
}

template <int HDT>
static int launch_attn_fs(const void* QKV, int64_t ldq, void* O, int64_t ldo, int B, int N, int H,
                          const float* gq, const float* bq, const float* gk, const float* bk, float eps, float scale,
                          hipStream_t s) {
  // at most 3 compute waves + the producer per workgroup (launch bound 256)
  const int nqt = (N + 31) / 32;
  const int groups = (nqt + 2) / 3, qtw = (nqt + groups - 1) / groups;
  hipLaunchKernelGGL(attn_fs_bf16<HDT>, dim3(B * H * groups), dim3(64 * (qtw + 1)), 0, s, (const bf16_t*)QKV, ldq,
                     (bf16_t*)O, ldo, N, H, qtw, groups, gq, bq, gk, bk, eps, scale * 1.4426950408889634f);
  return SDP_CHECK_LAUNCH();
}

static int g_attn_per_cu = 0;  // fa4 workgroups per CU (0 = as many as LDS and registers allow)

// Set the fa4 workgroups per CU (0 = occupancy-derived); returns the old value.
extern "C" int sdp_attn_set_per_cu(int n) {
  const int old = g_attn_per_cu;
  if (n >= 0 && n <= 8) g_attn_per_cu = n;
  return old;
}

#ifdef SDP_GEMM_STAMPS
extern "C" int sdp_attn_stamps(void* dst, int64_t bytes) {
  hipError_t rc = hipDeviceSynchronize();
  if (rc == hipSuccess && bytes >= (int64_t)sizeof(g_attn_stamps))
    rc = hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_attn_stamps), sizeof(g_attn_stamps));
  return (int)rc;
}
#endif
static size_t attn_fa4_bytes(int N, int hd) { return (size_t)2 * ((N + 15) / 16 * 16) * hd * 2 + 16 * (size_t)hd; }

template <int HDT>
static int launch_attn_fa4(const void* QKV, int64_t ldq, void* O, int64_t ldo, int B, int N, int H,
                           const float* gq, const float* bq, const float* gk, const float* bk, float eps, float scale,
                           hipStream_t s) {
  const size_t bytes = attn_fa4_bytes(N, 32 * HDT);
  const void* fn;
  switch ((N + 31) / 32) {
    case 1: fn = (const void*)attn_fa4_bf16<HDT, 1>; break;
    case 2: fn = (const void*)attn_fa4_bf16<HDT, 2>; break;
    case 3: fn = (const void*)attn_fa4_bf16<HDT, 3>; break;
    case 4: fn = (const void*)attn_fa4_bf16<HDT, 4>; break;
    case 5: fn = (const void*)attn_fa4_bf16<HDT, 5>; break;
    case 6: fn = (const void*)attn_fa4_bf16<HDT, 6>; break;
    case 7: fn = (const void*)attn_fa4_bf16<HDT, 7>; break;
    case 8: fn = (const void*)attn_fa4_bf16<HDT, 8>; break;
    default: return (int)hipErrorInvalidValue;
  }
  hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
  if (e != hipSuccess) return (int)e;
  int dev = 0, ncu = 256;
  (void)hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0) ncu = 256;
  // persistent grid: as many workgroups per CU as LDS and registers allow (N = 200, hd = 64:
  // 54 KiB and 160 VGPRs -> 3), so each SIMD interleaves up to three waves' MFMA / softmax phases
  int per_cu = g_attn_per_cu;
  if (per_cu <= 0) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, 256, bytes) != hipSuccess || nb <= 0)
      nb = bytes <= 80 * 1024 ? 2 : 1;
    per_cu = nb < 4 ? nb : 4;
  }
  int grid = per_cu * ncu;
  grid = grid / 8 * 8;
  if (grid < 8) grid = 8;
  if (grid > B * H) grid = B * H;
  const float sl = scale * 1.4426950408889634f;
  const bf16_t* q = (const bf16_t*)QKV;
  bf16_t* o = (bf16_t*)O;
  void* args[] = {(void*)&q, (void*)&ldq, (void*)&o, (void*)&ldo, (void*)&B, (void*)&N, (void*)&H, (void*)&gq,
                  (void*)&bq, (void*)&gk, (void*)&bk, (void*)&eps, (void*)&sl};
  e = hipLaunchKernel(fn, dim3(grid), dim3(256), args, bytes, s);
  if (e != hipSuccess) return (int)e;
  return SDP_CHECK_LAUNCH();
}

#ifdef SDP_DIAG
static size_t attn_fa5_bytes(int N, int hd) { return (size_t)4 * ((N + 15) / 16 * 16) * hd * 2 + 16 * (size_t)hd; }

template <int HDT>
static int launch_attn_fa5(const void* QKV, int64_t ldq, void* O, int64_t ldo, int B, int N, int H,
                           const float* gq, const float* bq, const float* gk, const float* bk, float eps, float scale,
                           hipStream_t s) {
  const size_t bytes = attn_fa5_bytes(N, 32 * HDT);
  const void* fn = nullptr;
  switch ((N + 31) / 32) {
    case 1: fn = (const void*)attn_fa5_bf16<HDT, 1>; break;
    case 2: fn = (const void*)attn_fa5_bf16<HDT, 2>; break;
    case 3: fn = (const void*)attn_fa5_bf16<HDT, 3>; break;
    case 4: fn = (const void*)attn_fa5_bf16<HDT, 4>; break;
    case 5: fn = (const void*)attn_fa5_bf16<HDT, 5>; break;
    case 6: fn = (const void*)attn_fa5_bf16<HDT, 6>; break;
    case 7: fn = (const void*)attn_fa5_bf16<HDT, 7>; break;
    default: return (int)hipErrorInvalidValue;
  }
  hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
  if (e != hipSuccess) return (int)e;
  int dev = 0, ncu = 256;
  (void)hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0) ncu = 256;
  int grid = ncu / 8 * 8;  // one workgroup per CU (LDS); pair order needs grid % 8 == 0
  if (grid < 8) grid = 8;
  if (grid > B * H) grid = B * H;
  const float sl = scale * 1.4426950408889634f;
  const bf16_t* q = (const bf16_t*)QKV;
  bf16_t* o = (bf16_t*)O;
  void* args[] = {(void*)&q, (void*)&ldq, (void*)&o, (void*)&ldo, (void*)&B, (void*)&N, (void*)&H, (void*)&gq,
                  (void*)&bq, (void*)&gk, (void*)&bk, (void*)&eps, (void*)&sl};
  e = hipLaunchKernel(fn, dim3(grid), dim3(512), args, bytes, s);
  if (e != hipSuccess) return (int)e;
  return SDP_CHECK_LAUNCH();
}

#endif  // SDP_DIAG

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

// bf16 flash kernel selection (highest tier allowed; each applies where it fits, else the next):
//   6 attn_fa5_bf16: N <= 224, K / V double-buffered within 160 KiB (M: 91-102 vs fa4's 103-109 us
//     alone, but the M forward 0.25 % slower than with fa4 over 8 interleaved runs -- opt-in);
//   4 (default) attn_fa4_bf16: N <= 256, two workgroups per CU;
//   3 attn_fa2_bf16: the whole head staged; at 9 key tiles (XL, N = 260) attn_fa6_bf16, persistent
//     with three rotating K / V images, where those fit 160 KiB;
//   then attn_fs_bf16 (5), the streaming kernel, for any longer N (hd % 32 == 0), and attn_fa_bf16
//   (2) for hd % 32 != 0.  Setting 5 forces attn_fs_bf16; 2 allows only attn_fa_bf16.
// The product library accepts tiers 3, 4 and 5; tier 2 (attn_fa for every shape) and 6 (attn_fa5)
// exist only in the diagnostic build (make stamps).  An unknown or unavailable tier returns -1 and
// leaves the selection unchanged; 0 queries it.
static int g_attn_kernel = 4;
extern "C" int sdp_attention_set_kernel(int k) {
  const int old = g_attn_kernel;
  if (k == 0) return old;
#ifdef SDP_DIAG
  if (k >= 2 && k <= 6) { g_attn_kernel = k; return old; }
#else
  if (k >= 3 && k <= 5) { g_attn_kernel = k; return old; }
#endif
  return -1;
}

extern "C" int sdp_attention_variant(int dtype, int N, int n_head, int head_dim, int has_mask) {
  if (dtype != 1 || has_mask || head_dim > 128 || head_dim % 16 != 0) return 0;
  const bool hd32 = head_dim % 32 == 0;
  if (g_attn_kernel == 5 && hd32) return 5;
#ifdef SDP_DIAG
  if (g_attn_kernel == 6 && hd32 && N <= 224 && attn_fa5_bytes(N, head_dim) <= 160 * 1024) return 6;
#endif
  if (g_attn_kernel >= 4 && g_attn_kernel != 5 && hd32 && N <= 256 && attn_fa4_bytes(N, head_dim) <= 160 * 1024)
    return 4;
  if (g_attn_kernel >= 3 && hd32 && attn_fa2_bytes(N, head_dim) <= 160 * 1024) return 3;
  if (g_attn_kernel >= 3 && hd32) return 5;  // longer heads: streamed K / V tiles, any N
  if (attn_fa_bytes(N, head_dim) > 160 * 1024) return 0;
  return 2;
}

int sdp_qk_headnorm(int dtype, void* QKV, int64_t ld, int64_t rows, int n_head, int head_dim, const float* gq,
                    const float* bq, const float* gk, const float* bk, float eps, void* stream);

extern "C" int sdp_attention(int dtype, const void* QKV, int64_t ldq, void* O, int64_t ldo, int B, int N,
                             int n_head, int head_dim, const float* q_gamma, const float* q_beta,
                             const float* k_gamma, const float* k_beta, float eps, const float* mask, int64_t mask_sb,
                             int64_t mask_sh, void* stream) {
  if (SDP_DIAG_SKIP(2)) return 0;  // timing experiment, diagnostic build only (misc.hip)
  if (!QKV || !O || B < 0 || N <= 0 || n_head <= 0 || head_dim <= 0 || head_dim > 128)
    return (int)hipErrorInvalidValue;
  const bool norm = q_gamma != nullptr;
  if (norm && (!q_beta || !k_gamma || !k_beta)) return (int)hipErrorInvalidValue;
  if (B == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const float scale = 1.0f / sqrtf((float)head_dim);
  const bool al = (ldq % 8 == 0) && (ldo % 4 == 0) && ((uintptr_t)QKV % 16 == 0) && ((uintptr_t)O % 8 == 0);
  const int variant = al ? sdp_attention_variant(dtype, N, n_head, head_dim, mask != nullptr) : 0;
  if (variant == 5) {
    const float *gq = norm ? q_gamma : nullptr, *bq = norm ? q_beta : nullptr;
    const float *gk = norm ? k_gamma : nullptr, *bk = norm ? k_beta : nullptr;
    switch (head_dim / 32) {
      case 1: return launch_attn_fs<1>(QKV, ldq, O, ldo, B, N, n_head, gq, bq, gk, bk, eps, scale, s);
      case 2: return launch_attn_fs<2>(QKV, ldq, O, ldo, B, N, n_head, gq, bq, gk, bk, eps, scale, s);
      case 3: return launch_attn_fs<3>(QKV, ldq, O, ldo, B, N, n_head, gq, bq, gk, bk, eps, scale, s);
      default: return launch_attn_fs<4>(QKV, ldq, O, ldo, B, N, n_head, gq, bq, gk, bk, eps, scale, s);
    }
  }
#ifdef SDP_DIAG
  if (variant == 6) {
    const float *gq = norm ? q_gamma : nullptr, *bq = norm ? q_beta : nullptr;
    const float *gk = norm ? k_gamma : nullptr, *bk = norm ? k_beta : nullptr;
    switch (head_dim / 32) {
      case 1: return launch_attn_fa5<1>(QKV, ldq, O, ldo, B, N, n_head, gq, bq, gk, bk, eps, scale, s);
      case 2: return launch_attn_fa5<2>(QKV, ldq, O, ldo, B, N, n_head, gq, bq, gk, bk, eps, scale, s);
      case 3: return launch_attn_fa5<3>(QKV, ldq, O, ldo, B, N, n_head, gq, bq, gk, bk, eps, scale, s);
      default: return launch_attn_fa5<4>(QKV, ldq, O, ldo, B, N, n_head, gq, bq, gk, bk, eps, scale, s);
    }
  }
#endif
  if (variant == 4) {
    const float *gq = norm ? q_gamma : nullptr, *bq = norm ? q_beta : nullptr;
    const float *gk = norm ? k_gamma : nullptr, *bk = norm ? k_beta : nullptr;
    switch (head_dim / 32) {
      case 1: return launch_attn_fa4<1>(QKV, ldq, O, ldo, B, N, n_head, gq, bq, gk, bk, eps, scale, s);
      case 2: return launch_attn_fa4<2>(QKV, ldq, O, ldo, B, N, n_head, gq, bq, gk, bk, eps, scale, s);
      case 3: return launch_attn_fa4<3>(QKV, ldq, O, ldo, B, N, n_head, gq, bq, gk, bk, eps, scale, s);
      default: return launch_attn_fa4<4>(QKV, ldq, O, ldo, B, N, n_head, gq, bq, gk, bk, eps, scale, s);
    }
  }
  if (variant == 3) {
    const float *gq = norm ? q_gamma : nullptr, *bq = norm ? q_beta : nullptr;
    const float *gk = norm ? k_gamma : nullptr, *bk = norm ? k_beta : nullptr;
    switch (head_dim / 32) {
      case 1: return launch_attn_fa2<1>(QKV, ldq, O, ldo, B, N, n_head, gq, bq, gk, bk, eps, scale, s);
      case 2: return launch_attn_fa2<2>(QKV, ldq, O, ldo, B, N, n_head, gq, bq, gk, bk, eps, scale, s);
      case 3: return launch_attn_fa2<3>(QKV, ldq, O, ldo, B, N, n_head, gq, bq, gk, bk, eps, scale, s);
      default: return launch_attn_fa2<4>(QKV, ldq, O, ldo, B, N, n_head, gq, bq, gk, bk, eps, scale, s);
    }
  }
  if (variant == 2) {
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
