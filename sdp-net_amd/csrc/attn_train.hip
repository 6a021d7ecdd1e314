// Training attention of EncoderLayer (layers.py:289-291: F.scaled_dot_product_attention with
// dropout_p = att_dropout under sdpa_kernel([MATH, FLASH_ATTENTION]); the manual path :292-298
// is the same math), flash-style on gfx950 MFMA, bf16 operands / fp32 accumulation:
//
//   forward   O = dropout(P) V,  P = softmax(S),  S = Q K^T / sqrt(hd)       (per batch, head)
//             saves O and the row log-sum-exp (base 2) -- never S or P
//   backward  dQ = scale * dS K, D = rowsum(dO o O)                (attn_bwd_q_k,  wave = query tile)
//             dV = Pd^T dO,  dK = scale * dS^T Q                   (attn_bwd_kv_k, wave = key tile)
//             with P recomputed from Q, K and the saved LSE, Pd = P o M / (1 - p),
//             dP = (dO V^T) o M / (1 - p),  dS = P o (dP - D)
//
// Q, K, V are read straight from the fused (q/k-normalised) projection rows [B*N, 3C]; O and
// dO are [B*N, C] rows; dQ, dK, dV are written to caller-given row blocks (the three thirds of
// the QKV gradient).  The dropout mask M is a counter hash of (seed, batch*H + head, query,
// key): regenerated, never stored, identical in the three kernels (sdp_attn_dropout_mask
// materialises it for tests).
//
// MFMA: v_mfma_f32_32x32x16_bf16.  D[i][j] = sum_k A[i][k] B[k][j]; lane l holds A row l%32 /
// B column l%32 with k = 8 (l/32) .. +7, and D column l%32, rows (i&3) + 8 (i>>2) + 4 (l/32)
// for register i.  An accumulator used as the next B operand keeps that row order as its k
// order, so the matching A operand is read transposed from a row-major LDS tile with
// ds_read_b64_tr_b16 in the same order (4 rows at +0, 4 at +8) -- the eval kernel's P V trick.
#include "common.h"

namespace attn_train {

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

SDP_DEV uint32_t hash4(uint64_t seed, uint32_t bh, uint32_t q, uint32_t k) {
  uint32_t x = (uint32_t)seed ^ (bh * 0x9E3779B9u);
  x ^= q * 0x85EBCA6Bu;
  x = (x << 13) | (x >> 19);
  x ^= k * 0xC2B2AE35u;
  x ^= (uint32_t)(seed >> 32);
  x ^= x >> 16;
  x *= 0x85EBCA6Bu;
  x ^= x >> 13;
  x *= 0xC2B2AE35u;
  x ^= x >> 16;
  return x;
}

// dropout keep factor: 0 or 1 / (1 - p)
SDP_DEV float keepf(uint64_t seed, uint32_t bh, int q, int k, uint32_t thresh, float inv_keep) {
  return hash4(seed, bh, (uint32_t)q, (uint32_t)k) >= thresh ? inv_keep : 0.f;
}

// row of register i of a 32x32 accumulator held by lane half hf
SDP_DEV int acc_row(int i, int hf) { return (i & 3) + 8 * (i >> 2) + 4 * hf; }

// A operand [32 rows x 16 k] = T^T of a row-major LDS tile T [k rows][ld] restricted to columns
// c0 .. c0+31, k rows taken in accumulator order starting at row k0 (k0 = 16 s2 + 4 hf):
// rows k0..k0+3 and k0+8..k0+11 (the eval kernel's V^T read).
SDP_DEV bf16x8 tr_frag(const bf16_t* T, int ld, int k0, int c0, int lane) {
  const int gi = lane & 15, tq = gi >> 2, tp = gi & 3;
  const bf16_t* p = T + (size_t)(k0 + tq) * ld + c0 + 16 * ((lane >> 4) & 1) + 4 * tp;
  const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)p);
  const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(p + 8 * ld));
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// ---------------------------------------------------------------------------
// Producer wave of the streaming kernels: key tile kt of the head (K and V rows, hd columns,
// zero padding) -> Kb / Vb + buf * 32 * LD, for kt = 0 .. nkt-1 into alternate buffers.  Its
// barrier sequence (one after tile 0, then one per tile) matches the compute waves' (one before
// their loop, one per tile): tile kt + 1 is loaded while the compute waves consume tile kt, and
// written to the buffer they finished reading in iteration kt - 1.
// ---------------------------------------------------------------------------
template <int HDT>
SDP_DEV void kv_ring_producer(const bf16_t* base, int64_t ldq, int C, int N, int hd, int nkt, bf16_t* Kb,
                              bf16_t* Vb, int lane) {
  constexpr int LD = 32 * HDT + 8;
  constexpr int CPR = 4 * HDT;  // 16-B chunks per staged row
  constexpr int NCH = (2 * 32 * CPR + 63) / 64;
  bf16x8 pv[NCH];
  auto p_load = [&](int kt) {
    const int k0 = kt * 32, valid = min(32, N - k0);
#pragma unroll
    for (int u = 0; u < NCH; ++u) {
      const int idx = u * 64 + lane;  // [matrix][row][chunk]
      const int mtx = idx / (32 * CPR), rem = idx - mtx * 32 * CPR;
      const int rr = rem / CPR, c8 = (rem - rr * CPR) * 8;
      pv[u] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
      if (mtx < 2 && rr < valid && c8 < hd) pv[u] = *(const bf16x8*)(base + (int64_t)(k0 + rr) * ldq + (mtx + 1) * C + c8);
    }
  };
  auto p_store = [&](int buf) {
#pragma unroll
    for (int u = 0; u < NCH; ++u) {
      const int idx = u * 64 + lane;
      const int mtx = idx / (32 * CPR), rem = idx - mtx * 32 * CPR;
      const int rr = rem / CPR, c8 = (rem - rr * CPR) * 8;
      if (mtx < 2) *(bf16x8*)((mtx == 0 ? Kb : Vb) + buf * 32 * LD + rr * LD + c8) = pv[u];
    }
  };
  p_load(0);
  p_store(0);
  __syncthreads();
  for (int kt = 0; kt < nkt; ++kt) {
    if (kt + 1 < nkt) {
      p_load(kt + 1);
      p_store((kt & 1) ^ 1);
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// Forward: workgroup = (b, h, group of qtw query tiles) + one producer wave streaming the key
// tiles (K, V rows) through a double-buffered LDS ring; compute wave w owns the 32-query tile
// grp * qtw + w and runs the online softmax over the key tiles as they arrive.
// ---------------------------------------------------------------------------
template <int HDT>
__global__ __launch_bounds__(256, 2) void attn_fwd_k(const bf16_t* __restrict__ QKV, int64_t ldq,
                                                  bf16_t* __restrict__ O, int64_t ldo, float* __restrict__ lse,
                                                  int N, int H, int hd, int qtw, int groups, float scale_log2,
                                                  uint32_t thresh, float inv_keep, uint64_t seed) {
  constexpr int LD = 32 * HDT + 8;
  __shared__ __attribute__((aligned(16))) bf16_t Kr[2][32 * LD];
  __shared__ __attribute__((aligned(16))) bf16_t Vr[2][32 * LD];
  const int bh = blockIdx.x / groups, grp = blockIdx.x - bh * groups;
  const int b = bh / H, hh = bh % H;
  const int C = H * hd;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int NP = (N + 31) / 32 * 32, nqt = NP / 32;
  const bf16_t* base = QKV + (int64_t)b * N * ldq + hh * hd;
  if (wave == qtw) {
    kv_ring_producer<HDT>(base, ldq, C, N, hd, nqt, &Kr[0][0], &Vr[0][0], lane);
    return;
  }
  const int r = lane & 31, hf = lane >> 5;
  const int nds = hd / 16;
  {
    const int qt = grp * qtw + wave;
    const bool active = qt < nqt;
    const int q = qt * 32 + r;
    const bool qok = active && q < N;
    bf16x8 qf[2 * HDT];
#pragma unroll
    for (int s = 0; s < 2 * HDT; ++s) {
      qf[s] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
      if (s < nds && qok) qf[s] = *(const bf16x8*)(base + (int64_t)q * ldq + 16 * s + 8 * hf);
    }
    f32x16 acc[HDT];
#pragma unroll
    for (int dt = 0; dt < HDT; ++dt)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[dt][i] = 0.f;
    float m = -INFINITY, l = 0.f;
    __syncthreads();
    for (int kt = 0; kt < nqt; ++kt) {
      if (!active) {
        __syncthreads();
        continue;
      }
      const bf16_t* Kt = Kr[kt & 1];
      const bf16_t* Vt = Vr[kt & 1];
      f32x16 st;
#pragma unroll
      for (int i = 0; i < 16; ++i) st[i] = 0.f;
      const bf16_t* krow = Kt + (size_t)r * LD + 8 * hf;
#pragma unroll
      for (int s = 0; s < 2 * HDT; ++s)
        if (s < nds) st = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*(const bf16x8*)(krow + 16 * s), qf[s], st, 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        st[i] *= scale_log2;
        if (kt * 32 + acc_row(i, hf) >= N) st[i] = -INFINITY;  // padded keys
      }
      float tmax = st[0];
#pragma unroll
      for (int i = 1; i < 16; ++i) tmax = fmaxf(tmax, st[i]);
      tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
      const float mn = fmaxf(m, tmax);
      if (__any(mn > m)) {
        const float alpha = __builtin_amdgcn_exp2f(m - mn);
        l *= alpha;
#pragma unroll
        for (int dt = 0; dt < HDT; ++dt)
#pragma unroll
          for (int i = 0; i < 16; ++i) acc[dt][i] *= alpha;
        m = mn;
      }
      float pv[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        pv[i] = __builtin_amdgcn_exp2f(st[i] - m);
        l += pv[i];  // the softmax normaliser sums the undropped P
      }
      if (thresh) {
#pragma unroll
        for (int i = 0; i < 16; ++i) pv[i] *= keepf(seed, bh, q, kt * 32 + acc_row(i, hf), thresh, inv_keep);
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        bf16x8 pb;
#pragma unroll
        for (int j = 0; j < 8; ++j) pb[j] = (short)f2bf(pv[8 * s2 + j]);
#pragma unroll
        for (int dt = 0; dt < HDT; ++dt)
          acc[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_frag(Vt, LD, 16 * s2 + 4 * hf, dt * 32, lane),
                                                            pb, acc[dt], 0, 0, 0);
      }
      __syncthreads();
    }
    l += __shfl_xor(l, 32, 64);
    if (qok) {
      const float inv = 1.0f / l;
      bf16_t* orow = O + ((int64_t)b * N + q) * ldo + hh * hd;
#pragma unroll
      for (int dt = 0; dt < HDT; ++dt)
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
      if (hf == 0) lse[(int64_t)bh * N + q] = m + __builtin_amdgcn_logf(l);  // log2 of the sum, base-2 units
    }
  }
}

// ---------------------------------------------------------------------------
// dK, dV: workgroup = (b, h, group of ktw key tiles) + one producer wave.  Compute wave w owns
// the 32-key tile grp * ktw + w (K, V fragments of its keys in registers, dK^T / dV^T
// accumulators); the query tiles stream through a double-buffered LDS ring filled by the last
// wave of the workgroup: while the compute waves work on query tile qt, the producer loads tile
// qt + 1 (Q rows, dO rows, LSE, D: 12 KiB of 16-B loads, all in flight at once) and writes it to
// the other buffer -- one barrier per query tile, the global-load latency off the compute path.
// ---------------------------------------------------------------------------
template <int HDT>
__global__ __launch_bounds__(256, 2) void attn_bwd_kv_k(const bf16_t* __restrict__ QKV, int64_t ldq,
                                                     const bf16_t* __restrict__ dO, int64_t lddo,
                                                     const float* __restrict__ lse, const float* __restrict__ D,
                                                     bf16_t* __restrict__ dK, int64_t lddk, bf16_t* __restrict__ dV,
                                                     int64_t lddv, int N, int H, int hd, int ktw, int groups,
                                                     float scale_log2, float scale, uint32_t thresh, float inv_keep,
                                                     uint64_t seed) {
  constexpr int LD = 32 * HDT + 8;
  constexpr int CPR = 4 * HDT;  // 16-B chunks per staged row (32 * HDT columns)
  __shared__ __attribute__((aligned(16))) bf16_t Qs[2][32 * LD];
  __shared__ __attribute__((aligned(16))) bf16_t Gs[2][32 * LD];  // dO tiles
  __shared__ __attribute__((aligned(16))) float Ls[2][32], Ds[2][32];
  const int bh = blockIdx.x / groups, grp = blockIdx.x - bh * groups;
  const int b = bh / H, hh = bh % H;
  const int C = H * hd;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, hf = lane >> 5;
  const int nds = hd / 16;
  const int NP = (N + 31) / 32 * 32, nqt = NP / 32;
  const bool producer = wave == ktw;  // wave-uniform
  const int kt = grp * ktw + wave;
  const bool active = !producer && kt < nqt;  // (the last group may hold fewer key tiles)
  const bf16_t* base = QKV + (int64_t)b * N * ldq + hh * hd;
  const bf16_t* gbase = dO + (int64_t)b * N * lddo + hh * hd;

  // producer: query tile qt -> registers (12 chunks of Q + dO rows per lane, LSE / D)
  constexpr int NCH = (2 * 32 * CPR + 63) / 64;
  bf16x8 pv[NCH];
  float pl = 0.f, pd = 0.f;
  auto p_load = [&](int qt) {
    const int q0 = qt * 32, valid = min(32, N - q0);
#pragma unroll
    for (int u = 0; u < NCH; ++u) {
      const int idx = u * 64 + lane;  // [matrix][row][chunk]
      const int mtx = idx / (32 * CPR), rem = idx - mtx * 32 * CPR;
      const int rr = rem / CPR, c8 = (rem - rr * CPR) * 8;
      pv[u] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
      if (mtx < 2 && rr < valid && c8 < hd)
        pv[u] = mtx == 0 ? *(const bf16x8*)(base + (int64_t)(q0 + rr) * ldq + c8)
                         : *(const bf16x8*)(gbase + (int64_t)(q0 + rr) * lddo + c8);
    }
    if (lane < 32) {
      pl = lane < valid ? lse[(int64_t)bh * N + q0 + lane] : INFINITY;  // padded queries: P = 0
      pd = lane < valid ? D[(int64_t)bh * N + q0 + lane] : 0.f;
    }
  };
  auto p_store = [&](int buf) {
#pragma unroll
    for (int u = 0; u < NCH; ++u) {
      const int idx = u * 64 + lane;
      const int mtx = idx / (32 * CPR), rem = idx - mtx * 32 * CPR;
      const int rr = rem / CPR, c8 = (rem - rr * CPR) * 8;
      if (mtx < 2) *(bf16x8*)((mtx == 0 ? Qs[buf] : Gs[buf]) + rr * LD + c8) = pv[u];
    }
    if (lane < 32) {
      Ls[buf][lane] = pl;
      Ds[buf][lane] = pd;
    }
  };

  // the producer and the compute waves run separate loops with the same barrier sequence
  // (nqt + 1 barriers), so neither keeps the other's registers live
  if (producer) {
    p_load(0);
    p_store(0);
    __syncthreads();
    for (int qt = 0; qt < nqt; ++qt) {
      if (qt + 1 < nqt) {
        p_load(qt + 1);
        p_store((qt & 1) ^ 1);  // last read in iteration qt - 1, whose barrier has passed
      }
      __syncthreads();
    }
    return;
  }
  bf16x8 kf[2 * HDT], vf[2 * HDT];
  f32x16 adk[HDT], adv[HDT];
  const int key = kt * 32 + r;
#pragma unroll
  for (int s = 0; s < 2 * HDT; ++s) {
    kf[s] = vf[s] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    if (active && s < nds && key < N) {
      kf[s] = *(const bf16x8*)(base + (int64_t)key * ldq + C + 16 * s + 8 * hf);
      vf[s] = *(const bf16x8*)(base + (int64_t)key * ldq + 2 * C + 16 * s + 8 * hf);
    }
  }
#pragma unroll
  for (int dt = 0; dt < HDT; ++dt)
#pragma unroll
    for (int i = 0; i < 16; ++i) adk[dt][i] = adv[dt][i] = 0.f;
  __syncthreads();
  for (int qt = 0; qt < nqt; ++qt) {
    const int cur = qt & 1;
    if (active) {
      const bf16_t* Q = Qs[cur];
      const bf16_t* G = Gs[cur];
      const int q0 = qt * 32;
      // S[q][key] and dPd[q][key] (lane = key, registers = queries)
      f32x16 st, dp;
#pragma unroll
      for (int i = 0; i < 16; ++i) st[i] = dp[i] = 0.f;
#pragma unroll
      for (int s = 0; s < 2 * HDT; ++s) {
        if (s < nds) {
          const bf16x8 qa = *(const bf16x8*)(Q + (size_t)r * LD + 16 * s + 8 * hf);
          const bf16x8 ga = *(const bf16x8*)(G + (size_t)r * LD + 16 * s + 8 * hf);
          st = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qa, kf[s], st, 0, 0, 0);
          dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ga, vf[s], dp, 0, 0, 0);
        }
      }
      // LSE / D of the 16 queries this lane holds: rows (i & 3) + 8 (i >> 2) + 4 hf
      f32x4 lq[4], dq4[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        lq[g] = *(const f32x4*)(&Ls[cur][8 * g + 4 * hf]);
        dq4[g] = *(const f32x4*)(&Ds[cur][8 * g + 4 * hf]);
      }
      float pdv[16], ds[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int qi = acc_row(i, hf);
        const float pr = key < N ? __builtin_amdgcn_exp2f(st[i] * scale_log2 - lq[i >> 2][i & 3]) : 0.f;
        const float kp = thresh ? keepf(seed, bh, q0 + qi, key, thresh, inv_keep) : 1.f;
        pdv[i] = pr * kp;                                // dropout(P)
        ds[i] = pr * (dp[i] * kp - dq4[i >> 2][i & 3]);  // P o (dP - D)
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        bf16x8 pb, sb;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          pb[j] = (short)f2bf(pdv[8 * s2 + j]);
          sb[j] = (short)f2bf(ds[8 * s2 + j]);
        }
#pragma unroll
        for (int dt = 0; dt < HDT; ++dt) {
          adv[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_frag(G, LD, 16 * s2 + 4 * hf, dt * 32, lane), pb,
                                                            adv[dt], 0, 0, 0);
          adk[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_frag(Q, LD, 16 * s2 + 4 * hf, dt * 32, lane), sb,
                                                            adk[dt], 0, 0, 0);
        }
      }
    }
    __syncthreads();
  }
  if (!active || key >= N) return;
  bf16_t* krow = dK + ((int64_t)b * N + key) * lddk + hh * hd;
  bf16_t* vrow = dV + ((int64_t)b * N + key) * lddv + hh * hd;
#pragma unroll
  for (int dt = 0; dt < HDT; ++dt)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d = dt * 32 + 8 * g + 4 * hf;
      if (d < hd) {
        bf16x4 ok, ov;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          ok[e] = (short)f2bf(adk[dt][4 * g + e] * scale);
          ov[e] = (short)f2bf(adv[dt][4 * g + e]);
        }
        *(bf16x4*)(krow + d) = ok;
        *(bf16x4*)(vrow + d) = ov;
      }
    }
}

// ---------------------------------------------------------------------------
// dQ (and D = rowsum(dO o O)): workgroup = (b, h, group of qtw query tiles) + one producer wave;
// compute wave w owns the 32-query tile grp * qtw + w (lane = query, registers = keys: the
// forward's layout) and loops over the key tiles, which the producer streams through a
// double-buffered LDS ring (K and V rows of tile kt + 1 loaded while tile kt is consumed; one
// barrier per key tile) -- the dK / dV kernel's structure with the roles of queries and keys
// swapped.
// ---------------------------------------------------------------------------
template <int HDT>
__global__ __launch_bounds__(256, 2) void attn_bwd_q_k(const bf16_t* __restrict__ QKV, int64_t ldq,
                                                    const bf16_t* __restrict__ O, int64_t ldo,
                                                    const bf16_t* __restrict__ dO, int64_t lddo,
                                                    const float* __restrict__ lse, float* __restrict__ D,
                                                    bf16_t* __restrict__ dQ, int64_t lddq, int N, int H, int hd,
                                                    int qtw, int groups, float scale_log2, float scale,
                                                    uint32_t thresh, float inv_keep, uint64_t seed) {
  constexpr int LD = 32 * HDT + 8;
  __shared__ __attribute__((aligned(16))) bf16_t Ks[2][32 * LD];
  __shared__ __attribute__((aligned(16))) bf16_t Vs[2][32 * LD];
  const int bh = blockIdx.x / groups, grp = blockIdx.x - bh * groups;
  const int b = bh / H, hh = bh % H;
  const int C = H * hd;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, hf = lane >> 5;
  const int nds = hd / 16;
  const int NP = (N + 31) / 32 * 32, nkt = NP / 32;
  const bf16_t* base = QKV + (int64_t)b * N * ldq + hh * hd;
  if (wave == qtw) {
    kv_ring_producer<HDT>(base, ldq, C, N, hd, nkt, &Ks[0][0], &Vs[0][0], lane);
    return;
  }
  const int qt = grp * qtw + wave;
  const bool active = qt < nkt;
  const int q = qt * 32 + r;
  const bool qok = active && q < N;
  const bf16_t* gbase = dO + (int64_t)b * N * lddo + hh * hd;
  bf16x8 qf[2 * HDT], gf[2 * HDT];
#pragma unroll
  for (int s = 0; s < 2 * HDT; ++s) {
    qf[s] = gf[s] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    if (s < nds && qok) {
      qf[s] = *(const bf16x8*)(base + (int64_t)q * ldq + 16 * s + 8 * hf);
      gf[s] = *(const bf16x8*)(gbase + (int64_t)q * lddo + 16 * s + 8 * hf);
    }
  }
  const float lq = qok ? lse[(int64_t)bh * N + q] : INFINITY;
  // D = rowsum(dO o O) for this query (its two lane halves hold the two halves of every
  // 16-wide d step); written for attn_bwd_kv_k, which runs next
  float dq_ = 0.f;
  if (qok) {
    const bf16_t* orow = O + ((int64_t)b * N + q) * ldo + hh * hd;
#pragma unroll
    for (int s = 0; s < 2 * HDT; ++s) {
      if (s < nds) {
        const bf16x8 ov = *(const bf16x8*)(orow + 16 * s + 8 * hf);
#pragma unroll
        for (int e = 0; e < 8; ++e) dq_ = fmaf(bf2f((bf16_t)ov[e]), bf2f((bf16_t)gf[s][e]), dq_);
      }
    }
  }
  dq_ += __shfl_xor(dq_, 32, 64);
  if (qok && hf == 0) D[(int64_t)bh * N + q] = dq_;
  f32x16 acc[HDT];
#pragma unroll
  for (int dt = 0; dt < HDT; ++dt)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[dt][i] = 0.f;
  __syncthreads();
  for (int kt = 0; kt < nkt; ++kt) {
    const int cur = kt & 1;
    if (active) {
      const bf16_t* Kt = Ks[cur];
      const bf16_t* Vt = Vs[cur];
      f32x16 st, dp;
#pragma unroll
      for (int i = 0; i < 16; ++i) st[i] = dp[i] = 0.f;
      const bf16_t* krow = Kt + (size_t)r * LD + 8 * hf;
      const bf16_t* vrow = Vt + (size_t)r * LD + 8 * hf;
#pragma unroll
      for (int s = 0; s < 2 * HDT; ++s) {
        if (s < nds) {
          st = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*(const bf16x8*)(krow + 16 * s), qf[s], st, 0, 0, 0);
          dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*(const bf16x8*)(vrow + 16 * s), gf[s], dp, 0, 0, 0);
        }
      }
      float ds[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int kk = kt * 32 + acc_row(i, hf);
        const float pr = kk < N ? __builtin_amdgcn_exp2f(st[i] * scale_log2 - lq) : 0.f;
        const float kp = thresh ? keepf(seed, bh, q, kk, thresh, inv_keep) : 1.f;
        ds[i] = pr * (dp[i] * kp - dq_);
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        bf16x8 sb;
#pragma unroll
        for (int j = 0; j < 8; ++j) sb[j] = (short)f2bf(ds[8 * s2 + j]);
#pragma unroll
        for (int dt = 0; dt < HDT; ++dt)
          acc[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_frag(Kt, LD, 16 * s2 + 4 * hf, dt * 32, lane), sb,
                                                            acc[dt], 0, 0, 0);
      }
    }
    __syncthreads();
  }
  if (qok) {
    bf16_t* row = dQ + ((int64_t)b * N + q) * lddq + hh * hd;
#pragma unroll
    for (int dt = 0; dt < HDT; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = dt * 32 + 8 * g + 4 * hf;
        if (d < hd) {
          bf16x4 o;
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = (short)f2bf(acc[dt][4 * g + e] * scale);
          *(bf16x4*)(row + d) = o;
        }
      }
  }
}

__global__ __launch_bounds__(256) void dropout_mask_k(uint8_t* __restrict__ out, int Z, int N, uint32_t thresh,
                                                      uint64_t seed) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t total = (int64_t)Z * N * N;
  if (idx >= total) return;
  const int k = (int)(idx % N);
  const int64_t t = idx / N;
  const int q = (int)(t % N), z = (int)(t / N);
  out[idx] = hash4(seed, (uint32_t)z, (uint32_t)q, (uint32_t)k) >= thresh ? 1 : 0;
}

}  // namespace attn_train

using namespace attn_train;

static void drop_params(float p, uint32_t* thresh, float* inv_keep) {
  const double t = (double)p * 4294967296.0;
  *thresh = p <= 0.f ? 0u : (t >= 4294967295.0 ? 4294967295u : (uint32_t)t);
  *inv_keep = p < 1.f ? 1.0f / (1.0f - p) : 0.f;
}

// every kernel streams the key / query tiles through a fixed 2-buffer LDS ring: any N
extern "C" int sdp_attn_train_applies(int dtype, int N, int hd) {
  return (dtype == 1 && N >= 1 && hd >= 16 && hd <= 128 && hd % 16 == 0) ? 1 : 0;
}

#define SDP_HDT_DISPATCH(hd, KERN, ...)                                    \
  do {                                                                      \
    const int hdt_ = ((hd) + 31) / 32;                                      \
    if (hdt_ == 1) KERN<1>(__VA_ARGS__);                                    \
    else if (hdt_ == 2) KERN<2>(__VA_ARGS__);                               \
    else if (hdt_ == 3) KERN<3>(__VA_ARGS__);                               \
    else KERN<4>(__VA_ARGS__);                                              \
  } while (0)

template <int HDT>
static int launch_fwd(const void* qkv, int64_t ldq, void* o, int64_t ldo, float* lse, int B, int N, int H, int hd,
                      float scale, uint32_t thresh, float inv_keep, uint64_t seed, hipStream_t s) {
  // at most 3 compute waves + the producer per workgroup (launch bound 256)
  const int nqt = (N + 31) / 32;
  const int groups = (nqt + 2) / 3, qtw = (nqt + groups - 1) / groups;
  hipLaunchKernelGGL(attn_fwd_k<HDT>, dim3(B * H * groups), dim3(64 * (qtw + 1)), 0, s, (const bf16_t*)qkv, ldq,
                     (bf16_t*)o, ldo, lse, N, H, hd, qtw, groups, scale * 1.4426950408889634f, thresh, inv_keep, seed);
  return SDP_CHECK_LAUNCH();
}

template <int HDT>
static int launch_bwd(const void* qkv, int64_t ldq, const void* o, int64_t ldo, const void* dO, int64_t lddo,
                      const float* lse, float* D, void* dq, int64_t lddq, void* dk, int64_t lddk, void* dv,
                      int64_t lddv, int B, int N, int H, int hd, float scale, uint32_t thresh, float inv_keep,
                      uint64_t seed, hipStream_t s) {
  const int nkt = (N + 31) / 32;
  // dQ (and D = rowsum(dO o O)) first: the dK / dV kernel reads D.  Both: at most 3 compute
  // waves + the producer per workgroup (launch bound 256)
  const int groups = (nkt + 2) / 3, ktw = (nkt + groups - 1) / groups;
  hipLaunchKernelGGL(attn_bwd_q_k<HDT>, dim3(B * H * groups), dim3(64 * (ktw + 1)), 0, s, (const bf16_t*)qkv, ldq,
                     (const bf16_t*)o, ldo, (const bf16_t*)dO, lddo, lse, D, (bf16_t*)dq, lddq, N, H, hd, ktw,
                     groups, scale * 1.4426950408889634f, scale, thresh, inv_keep, seed);
  int rc = SDP_CHECK_LAUNCH();
  if (rc) return rc;
  hipLaunchKernelGGL(attn_bwd_kv_k<HDT>, dim3(B * H * groups), dim3(64 * (ktw + 1)), 0, s, (const bf16_t*)qkv, ldq,
                     (const bf16_t*)dO, lddo, lse, (const float*)D, (bf16_t*)dk, lddk, (bf16_t*)dv, lddv, N, H, hd,
                     ktw, groups, scale * 1.4426950408889634f, scale, thresh, inv_keep, seed);
  return SDP_CHECK_LAUNCH();
}

extern "C" int sdp_attn_train_fwd(int dtype, const void* qkv, int64_t ldq, void* o, int64_t ldo, float* lse, int B,
                                  int N, int H, int hd, float scale, float p, uint64_t seed, void* stream) {
  // bf16x8 loads of the qkv rows, bf16x4 stores of O rows
  if (!sdp_attn_train_applies(dtype, N, hd) || !qkv || !o || !lse || B < 0 || H <= 0 || p < 0.f || p >= 1.f ||
      ldq % 8 || ldo % 8 || ldq < 3 * (int64_t)H * hd || ldo < (int64_t)H * hd || (uintptr_t)qkv % 16 ||
      (uintptr_t)o % 8)
    return (int)hipErrorInvalidValue;
  if (B == 0) return 0;
  uint32_t thresh;
  float inv_keep;
  drop_params(p, &thresh, &inv_keep);
  int rc = 0;
  SDP_HDT_DISPATCH(hd, rc = launch_fwd, qkv, ldq, o, ldo, lse, B, N, H, hd, scale, thresh, inv_keep, seed,
                   (hipStream_t)stream);
  return rc;
}

extern "C" int sdp_attn_train_bwd(int dtype, const void* qkv, int64_t ldq, const void* o, int64_t ldo,
                                  const void* dO, int64_t lddo, const float* lse, float* delta, void* dq,
                                  int64_t lddq, void* dk, int64_t lddk, void* dv, int64_t lddv, int B, int N, int H,
                                  int hd, float scale, float p, uint64_t seed, void* stream) {
  // the same leading-dimension checks as the forward, plus the row widths of dq / dk / dv and the
  // base alignments the kernels' vector accesses need (bf16x8 loads of qkv / o / dO, 8-B stores)
  const int64_t hw = (int64_t)H * hd;
  auto al = [](const void* q, uintptr_t a) { return ((uintptr_t)q % a) == 0; };
  if (!sdp_attn_train_applies(dtype, N, hd) || !qkv || !o || !dO || !lse || !delta || !dq || !dk || !dv || B < 0 ||
      H <= 0 || p < 0.f || p >= 1.f || ldq % 8 || ldo % 8 || lddo % 8 || lddq % 4 || lddk % 4 || lddv % 4 ||
      ldq < 3 * hw || ldo < hw || lddo < hw || lddq < hw || lddk < hw || lddv < hw || !al(qkv, 16) || !al(o, 16) ||
      !al(dO, 16) || !al(dq, 8) || !al(dk, 8) || !al(dv, 8))
    return (int)hipErrorInvalidValue;
  if (B == 0) return 0;
  uint32_t thresh;
  float inv_keep;
  drop_params(p, &thresh, &inv_keep);
  hipStream_t s = (hipStream_t)stream;
  int rc = 0;
  SDP_HDT_DISPATCH(hd, rc = launch_bwd, qkv, ldq, o, ldo, dO, lddo, lse, delta, dq, lddq, dk, lddk, dv, lddv, B, N,
                   H, hd, scale, thresh, inv_keep, seed, s);
  return rc;
}

extern "C" int sdp_attn_dropout_mask(uint8_t* out, int Z, int N, float p, uint64_t seed, void* stream) {
  if (!out || Z < 0 || N < 0 || p < 0.f || p >= 1.f) return (int)hipErrorInvalidValue;
  const int64_t total = (int64_t)Z * N * N;
  if (total == 0) return 0;
  uint32_t thresh;
  float inv_keep;
  drop_params(p, &thresh, &inv_keep);
  hipLaunchKernelGGL(dropout_mask_k, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream, out, Z,
                     N, thresh, seed);
  return SDP_CHECK_LAUNCH();
}
