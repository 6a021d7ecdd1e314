// Training-step kernels of the SdP-Net path on gfx950 (BASELINE.json configs[4]: fwd + bwd +
// AdamW).  Reference: the bf16-autocast forward + backward,
// GradScaler, clip_grad_norm_(5) and AdamW of training_tools.py:77-103 / :230-259, the
// train-mode StochasticDepth of utility_layers.py:16-27 and the dropouts of layers.py:291,
// :301-308.
//
//  * gemm_flex — batched MFMA GEMM with either operand transposed, split-K partial slabs:
//      C[z](i, j) = alpha * sum_k A[z](i, k) * B[z](k, j)
//      A(i, k) = TA ? A[k * lda + i] : A[i * lda + k];  B(k, j) = TB ? B[j * ldb + k] : B[k * ldb + j]
//    bf16: 128x128x32 tiles, 4 waves (64x64 each, v_mfma_f32_16x16x32_bf16).  An operand
//    whose K runs along its rows ([i][k], [j][k]) is staged as [row][32] 64-B rows and read
//    with ds_read_b128; one whose K runs down its columns ([k][i], [k][j]) is staged as it
//    lies ([32][128] 256-B rows) and read with ds_read_b64_tr_b16, the hardware transpose
//    (no transposed copy in HBM).  fp32: v_mfma_f32_16x16x4_f32 (exact f32), scalar LDS reads.
//    Covers dW = dY^T X (both operands k-major), the attention products of the backward
//    (S = QK^T, O = PV, dV = P^T dO, dP = dO V^T, dQ = dS K, dK = dS^T Q) and dX = dY W.
//  * seg_colsum — out[g][c] = sum over a strided segment of rows (bias / LayerNorm-affine /
//    embedding-table gradients, split-K slab reduction).
//  * act_fwd / act_bwd with a counter-hash dropout mask (regenerated, never stored).
//  * ln_apply (LayerNorm with given statistics), ln_bwd (dx + per-block dgamma/dbeta partials).
//  * softmax_fwd / softmax_bwd over attention rows (with attention dropout).
//  * dw_wgrad — depthwise-conv weight gradient (per-channel correlation).
//  * ce_loss — label-smoothed cross entropy (training_tools.py:76) loss and dlogits.
//  * sumsq / adamw — fused gradient norm (clip_grad_norm_, unscale, inf check) and the
//    multi-tensor AdamW update (torch.optim.AdamW semantics), no host synchronisation.
#include "common.h"

static RowMap mk_tmap(int grp, int64_t gstride, int off) {
  RowMap r;
  r.grp = grp > 0 ? grp : 0x7fffffff;
  r.gstride = grp > 0 ? gstride : 0;
  r.off = grp > 0 ? off : 0;
  return r;
}


// ---------------------------------------------------------------------------
// gemm_flex
// ---------------------------------------------------------------------------
namespace flex {
constexpr int BI = 128, BJ = 128, BK = 32, NT = 256;
constexpr int TILE = 8192;  // bytes per operand tile (bf16: 128 x 32 x 2)

// [128][32] bf16, 64-B rows: 16-B chunk c of row r at c ^ H[(r >> 2) & 3], H = {0, 2, 3, 1}
// (conflict-free ds_read_b128 for the 16x16x32 operand map: lane -> row l & 15, chunk l >> 4)
SDP_DEV int rr_off(int r, int c) { return r * 64 + ((c ^ ((0x78 >> (2 * ((r >> 2) & 3))) & 3)) << 4); }
// [32][128] bf16, 256-B rows, XOR image for ds_read_b64_tr_b16 (one image serves row and
// transposed reads; cdna_hip_programming.md T10 layout (b))
SDP_DEV int tr_off(int r, int ch) { return r * 256 + ((ch ^ (((r & 3) << 2) | ((r >> 2) & 3))) << 4); }

struct Op {
  const void* p;
  int64_t ld;
  int64_t s1, s2;  // batch strides: z -> (z / zdiv) * s1 + (z % zdiv) * s2
  int vec;         // rows 16-B aligned: 8-element vector loads (else element loads)
};

SDP_DEV int64_t zoff(const Op& o, int z, int zdiv) { return (int64_t)(z / zdiv) * o.s1 + (int64_t)(z % zdiv) * o.s2; }

// Load 8 consecutive bf16 (along the contiguous axis) of logical row `row`, starting at
// contiguous index `c0`; zero outside [0, nrow) x [0, ncol).
SDP_DEV bf16x8 load8(const bf16_t* base, int64_t ld, int row, int nrow, int c0, int ncol, int vec) {
  bf16x8 v = {0, 0, 0, 0, 0, 0, 0, 0};
  if (row >= nrow) return v;
  const bf16_t* p = base + (int64_t)row * ld + c0;
  if (vec && c0 + 8 <= ncol) return *(const bf16x8*)p;
#pragma unroll
  for (int e = 0; e < 8; ++e)
    if (c0 + e < ncol) v[e] = (short)p[e];
  return v;
}

typedef short v4i16 __attribute__((ext_vector_type(4)));

template <bool TR>
SDP_DEV bf16x8 frag(const char* tile, int rbase, int lane) {
  if constexpr (!TR) {
    return *(const bf16x8*)(tile + rr_off(rbase + (lane & 15), lane >> 4));
  } else {
    // rbase = first column (multiple of 16) of the 16-wide block; K rows 8g .. 8g+7
    const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
    const int ch = (rbase >> 3) + (p >> 1);
    const char* a0 = tile + tr_off(8 * g + q, ch) + 8 * (p & 1);
    const char* a1 = tile + tr_off(8 * g + 4 + q, ch) + 8 * (p & 1);
    v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((AS3 v4i16*)(a0));
    v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((AS3 v4i16*)(a1));
    return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  }
}

// Stage one operand tile (128 along i/j, 32 along k) into LDS; the loads for the NEXT
// k-step are issued into registers first (reg), then written after the MFMAs.
template <bool KMAJ>  // KMAJ: the operand's k runs down its rows ([k][i]) -> [32][128] image
SDP_DEV void gload(bf16x8 (&reg)[2], const bf16_t* base, int64_t ld, int r0, int nr, int k0, int K, int tid,
                   int vec) {
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int idx = tid + s * NT;
    if constexpr (!KMAJ) {
      const int row = idx >> 2, c = idx & 3;  // row of 128, chunk of 8 k
      reg[s] = load8(base, ld, r0 + row, nr, k0 + 8 * c, K, vec);
    } else {
      const int kr = idx >> 4, ch = idx & 15;  // k row of 32, chunk of 8 along i
      reg[s] = load8(base, ld, k0 + kr, K, r0 + 8 * ch, nr, vec);
    }
  }
}
template <bool KMAJ>
SDP_DEV void lstore(const bf16x8 (&reg)[2], char* tile, int tid) {
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int idx = tid + s * NT;
    if constexpr (!KMAJ) *(bf16x8*)(tile + rr_off(idx >> 2, idx & 3)) = reg[s];
    else *(bf16x8*)(tile + tr_off(idx >> 4, idx & 15)) = reg[s];
  }
}

template <typename TO>
SDP_DEV void cstore(TO* C, int64_t ldc, int i, int j, int Mi, int Nj, float v, bool accum) {
  if (i >= Mi || j >= Nj) return;
  TO* p = C + (int64_t)i * ldc + j;
  if (accum) v += to_f<TO>(*p);
  *p = from_f<TO>(v);
}

// TA: A stored [k][i] (else [i][k]); TB: B stored [j][k] (else [k][j])
template <bool TA, bool TB, typename TO>
__global__ __launch_bounds__(NT) void gemm_flex_bf16(Op A, Op B, Op Cc, int Mi, int Nj, int K, int zdiv,
                                                     int splits, int kchunk, int64_t split_stride, float alpha,
                                                     int accum) {
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * TILE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wi = wave >> 1, wj = wave & 1;
  // XCD-contiguous tile order (consecutive block ids go to different XCDs): the tiles one XCD
  // runs together share their column blocks in its L2 (XL training step +1 %)
  int bx, by, bz;
  {
    const int gx = gridDim.x, gy = gridDim.y, nwg = gx * gy * gridDim.z;
    const int b = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
    const int xcd = b & 7, q = nwg >> 3, rem = nwg & 7;
    const int w = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + (b >> 3);
    bx = w % gx;
    by = (w / gx) % gy;
    bz = w / (gx * gy);
  }
  const int i0 = by * BI, j0 = bx * BJ;
  const int z = bz / splits, sk = bz % splits;
  const int kb = sk * kchunk, ke = min(K, kb + kchunk);
  const bf16_t* Ap = (const bf16_t*)A.p + zoff(A, z, zdiv);
  const bf16_t* Bp = (const bf16_t*)B.p + zoff(B, z, zdiv);
  TO* Cp = (TO*)Cc.p + zoff(Cc, z, zdiv) + (int64_t)sk * split_stride;
  // A operand: rows i (KMAJ = TA); B operand: rows j (KMAJ = !TB)
  f32x4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 ra[2], rb[2];
  if (kb < ke) {
    gload<TA>(ra, Ap, A.ld, i0, Mi, kb, ke, tid, A.vec);
    gload<!TB>(rb, Bp, B.ld, j0, Nj, kb, ke, tid, B.vec);
    lstore<TA>(ra, smem, tid);
    lstore<!TB>(rb, smem + TILE, tid);
  }
  __syncthreads();
  int buf = 0;
  for (int k0 = kb; k0 < ke; k0 += BK) {
    const bool more = k0 + BK < ke;
    if (more) {
      gload<TA>(ra, Ap, A.ld, i0, Mi, k0 + BK, ke, tid, A.vec);
      gload<!TB>(rb, Bp, B.ld, j0, Nj, k0 + BK, ke, tid, B.vec);
    }
    const char* at = smem + buf * 2 * TILE;
    const char* bt = at + TILE;
    bf16x8 fa[4], fb[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) fa[t] = frag<TA>(at, wi * 64 + t * 16, lane);
#pragma unroll
    for (int t = 0; t < 4; ++t) fb[t] = frag<!TB>(bt, wj * 64 + t * 16, lane);
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[a], fb[b], acc[a][b], 0, 0, 0);
    if (more) {
      char* nt = smem + (buf ^ 1) * 2 * TILE;
      lstore<TA>(ra, nt, tid);
      lstore<!TB>(rb, nt + TILE, tid);
    }
    __syncthreads();
    buf ^= 1;
  }
  // D[i][j]: lane holds i = 4 * (lane >> 4) + r, j = lane & 15 of each 16x16 tile
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = i0 + wi * 64 + a * 16 + 4 * (lane >> 4) + r;
        const int j = j0 + wj * 64 + b * 16 + (lane & 15);
        cstore<TO>(Cp, Cc.ld, i, j, Mi, Nj, alpha * acc[a][b][r], accum != 0);
      }
}

// fp32 (exact f32 MFMA): operands staged in their stored orientation, scalar LDS reads
constexpr int FK = 16;
template <bool TA, bool TB>
__global__ __launch_bounds__(NT) void gemm_flex_f32(Op A, Op B, Op Cc, int Mi, int Nj, int K, int zdiv, int splits,
                                                    int kchunk, int64_t split_stride, float alpha, int accum) {
  // [i][k] pitch 17 or [k][i] pitch 132 floats (both 2176 / 2112 floats, <= 2176)
  __shared__ float as[2176], bs[2176];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wi = wave >> 1, wj = wave & 1;
  const int i0 = blockIdx.y * BI, j0 = blockIdx.x * BJ;
  const int z = blockIdx.z / splits, sk = blockIdx.z % splits;
  const int kb = sk * kchunk, ke = min(K, kb + kchunk);
  const float* Ap = (const float*)A.p + zoff(A, z, zdiv);
  const float* Bp = (const float*)B.p + zoff(B, z, zdiv);
  float* Cp = (float*)Cc.p + zoff(Cc, z, zdiv) + (int64_t)sk * split_stride;
  f32x4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  // logical element (r in 0..127 along i/j, k in 0..15)
  auto stage = [&](float* s, const float* base, int64_t ld, int r0, int nr, int k0, bool kmaj) {
    for (int e = tid; e < 128 * FK; e += NT) {
      int r, k;
      if (kmaj) { k = e >> 7; r = e & 127; } else { r = e >> 4; k = e & 15; }
      const int gr = r0 + r, gk = k0 + k;
      float v = 0.f;
      if (gr < nr && gk < ke) v = kmaj ? base[(int64_t)gk * ld + gr] : base[(int64_t)gr * ld + gk];
      if (kmaj) s[k * 132 + r] = v; else s[r * 17 + k] = v;
    }
  };
  for (int k0 = kb; k0 < ke; k0 += FK) {
    stage(as, Ap, A.ld, i0, Mi, k0, TA);
    stage(bs, Bp, B.ld, j0, Nj, k0, !TB);
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < FK; kk += 4) {
      float fa[4], fb[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int i = wi * 64 + t * 16 + (lane & 15), k = kk + (lane >> 4);
        fa[t] = TA ? as[k * 132 + i] : as[i * 17 + k];
        const int j = wj * 64 + t * 16 + (lane & 15);
        fb[t] = !TB ? bs[k * 132 + j] : bs[j * 17 + k];
      }
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[a], fb[b], acc[a][b], 0, 0, 0);
    }
    __syncthreads();
  }
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = i0 + wi * 64 + a * 16 + 4 * (lane >> 4) + r;
        const int j = j0 + wj * 64 + b * 16 + (lane & 15);
        cstore<float>(Cp, Cc.ld, i, j, Mi, Nj, alpha * acc[a][b][r], accum != 0);
      }
}
}  // namespace flex

extern "C" int sdp_gemm_flex(int dtype, int out_dtype, int ta, int tb, const void* A, int64_t lda, int64_t sa1,
                             int64_t sa2, const void* B, int64_t ldb, int64_t sb1, int64_t sb2, void* C, int64_t ldc,
                             int64_t sc1, int64_t sc2, int M, int N, int K, int Z, int zdiv, int splits,
                             int64_t split_stride, float alpha, int accum, void* stream) {
  if (!A || !B || !C || M < 0 || N < 0 || K < 0 || Z < 0 || zdiv <= 0 || splits <= 0) return (int)hipErrorInvalidValue;
  if (M == 0 || N == 0 || Z == 0) return 0;
  if (dtype == 1) {
    if (out_dtype != 0 && out_dtype != 1) return (int)hipErrorInvalidValue;
  } else if (dtype == 0) {
    if (out_dtype != 0) return (int)hipErrorInvalidValue;
  } else {
    return (int)hipErrorInvalidValue;
  }
  if (splits > 1 && accum) return (int)hipErrorInvalidValue;
  int kchunk = (K + splits - 1) / splits;
  const int kq = dtype == 1 ? flex::BK : flex::FK;
  kchunk = (kchunk + kq - 1) / kq * kq;
  // 16-B vector loads where leading dimensions, batch strides and bases are 8-element aligned
  const int va = !(lda % 8 || sa1 % 8 || sa2 % 8 || ((uintptr_t)A % 16));
  const int vb = !(ldb % 8 || sb1 % 8 || sb2 % 8 || ((uintptr_t)B % 16));
  flex::Op a{A, lda, sa1, sa2, va}, b{B, ldb, sb1, sb2, vb}, c{C, ldc, sc1, sc2, 0};
  dim3 grid((N + flex::BJ - 1) / flex::BJ, (M + flex::BI - 1) / flex::BI, Z * splits);
  hipStream_t s = (hipStream_t)stream;
#define SDP_FLEX(KN, TA_, TB_, ...)                                                                                 \
  hipLaunchKernelGGL((flex::KN<TA_, TB_, ##__VA_ARGS__>), grid, dim3(flex::NT), 0, s, a, b, c, M, N, K, zdiv, splits, \
                     kchunk, split_stride, alpha, accum)
  if (dtype == 1) {
    if (out_dtype == 0) {
      if (!ta && !tb) SDP_FLEX(gemm_flex_bf16, false, false, float);
      else if (!ta && tb) SDP_FLEX(gemm_flex_bf16, false, true, float);
      else if (ta && !tb) SDP_FLEX(gemm_flex_bf16, true, false, float);
      else SDP_FLEX(gemm_flex_bf16, true, true, float);
    } else {
      if (!ta && !tb) SDP_FLEX(gemm_flex_bf16, false, false, bf16_t);
      else if (!ta && tb) SDP_FLEX(gemm_flex_bf16, false, true, bf16_t);
      else if (ta && !tb) SDP_FLEX(gemm_flex_bf16, true, false, bf16_t);
      else SDP_FLEX(gemm_flex_bf16, true, true, bf16_t);
    }
  } else {
    if (!ta && !tb) SDP_FLEX(gemm_flex_f32, false, false);
    else if (!ta && tb) SDP_FLEX(gemm_flex_f32, false, true);
    else if (ta && !tb) SDP_FLEX(gemm_flex_f32, true, false);
    else SDP_FLEX(gemm_flex_f32, true, true);
  }
#undef SDP_FLEX
  return SDP_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------
// seg_colsum: out[g * ldo + c] (+)= sum_{e < len} X[row(g, e) * ldx + c],
// row(g, e) = g * gstride + e * estride (in rows).  fp32 accumulation.
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void seg_colsum_k(const T* __restrict__ X, int64_t ldx, int G, int len,
                                                    int64_t gstride, int64_t estride, int C, float* __restrict__ out,
                                                    int64_t ldo, float scale, int accum) {
  // block: 64 columns x 4 row slices; grid (ceil(C/64), G)
  __shared__ float red[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63), sl = threadIdx.x >> 6, g = blockIdx.y;
  float s = 0.f;
  if (c < C) {
    const T* p = X + (int64_t)g * gstride * ldx + c;
    for (int e = sl; e < len; e += 4) s += to_f<T>(p[(int64_t)e * estride * ldx]);
  }
  red[sl][threadIdx.x & 63] = s;
  __syncthreads();
  if (sl == 0 && c < C) {
    const float v = scale * (red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x]);
    float* o = out + (int64_t)g * ldo + c;
    *o = accum ? *o + v : v;
  }
}

// 4 consecutive columns per thread (16-B fp32 / 8-B bf16 loads): block = 256 columns x 4 row
// slices (C % 4 == 0, aligned rows).
template <typename T>
__global__ __launch_bounds__(256) void seg_colsum_v4(const T* __restrict__ X, int64_t ldx, int G, int len,
                                                     int64_t gstride, int64_t estride, int C, float* __restrict__ out,
                                                     int64_t ldo, float scale, int accum) {
  __shared__ f32x4 red[4][64];
  const int c = (blockIdx.x * 64 + (threadIdx.x & 63)) * 4, sl = threadIdx.x >> 6, g = blockIdx.y;
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  auto ld = [&](const T* q) -> f32x4 {
    if constexpr (sizeof(T) == 2) {
      const bf16x4 t = *(const bf16x4*)q;
      return f32x4{bf2f((bf16_t)t[0]), bf2f((bf16_t)t[1]), bf2f((bf16_t)t[2]), bf2f((bf16_t)t[3])};
    } else {
      return *(const f32x4*)q;
    }
  };
  if (c < C) {
    const T* p = X + (int64_t)g * gstride * ldx + c;
    const int64_t rs = estride * ldx;
    int e = sl;
    // eight of the slice's rows loaded before any is added (the rows are independent; one load in
    // flight per thread made the long, narrow reductions -- bias / LN-affine sums over token
    // segments, the second level over 256-row partials -- latency-bound); the adds keep the
    // row order, so the sums are bit-identical to the one-row loop
    for (; e + 28 < len; e += 32) {
      f32x4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = ld(p + (int64_t)(e + 4 * u) * rs);
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; e + 12 < len; e += 16) {
      f32x4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = ld(p + (int64_t)(e + 4 * u) * rs);
#pragma unroll
      for (int u = 0; u < 4; ++u) s += v[u];
    }
    for (; e < len; e += 4) s += ld(p + (int64_t)e * rs);
  }
  red[sl][threadIdx.x & 63] = s;
  __syncthreads();
  if (sl == 0 && c < C) {
    const f32x4 v = scale * (red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x]);
    f32x4* o = (f32x4*)(out + (int64_t)g * ldo + c);
    *o = accum ? *o + v : v;
  }
}

// Wide, short sums (the weight-gradient slab reduction: G = 1, len = split count <= 64, C = N x K):
// each thread owns 8 consecutive columns and walks all len rows itself, eight rows (16 loads) in
// flight at a time, adding them in row order -- out[c] = ((x_0 + x_1) + x_2) + ... exactly.
// seg_colsum_v4's 4-row slices give such a sum only len / 4 loads per thread.
__global__ __launch_bounds__(256) void colsum_wide_f32(const float* __restrict__ X, int64_t rs, int len, int C,
                                                       float* __restrict__ out, float scale, int accum) {
  const int c = (blockIdx.x * 256 + threadIdx.x) * 8;
  if (c >= C) return;
  const float* p = X + c;
  f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = s0;
  int e = 0;
  for (; e + 8 <= len; e += 8) {
    f32x4 a[8], b[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      a[u] = *(const f32x4*)(p + (int64_t)(e + u) * rs);
      b[u] = *(const f32x4*)(p + (int64_t)(e + u) * rs + 4);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      s0 += a[u];
      s1 += b[u];
    }
  }
  for (; e < len; ++e) {
    s0 += *(const f32x4*)(p + (int64_t)e * rs);
    s1 += *(const f32x4*)(p + (int64_t)e * rs + 4);
  }
  f32x4* o = (f32x4*)(out + c);
  const f32x4 v0 = scale * s0, v1 = scale * s1;
  if (accum) {
    o[0] += v0;
    o[1] += v1;
  } else {
    o[0] = v0;
    o[1] = v1;
  }
}

extern "C" int sdp_seg_colsum(int dtype, const void* X, int64_t ldx, int G, int len, int64_t gstride,
                              int64_t estride, int C, float* out, int64_t ldo, float scale, int accum, void* stream) {
  if (!X || !out || G < 0 || len < 0 || C < 0) return (int)hipErrorInvalidValue;
  if (G == 0 || C == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const int es = dtype == 1 ? 2 : 4;
  if (dtype == 0 && G == 1 && len <= 64 && C >= 65536 && C % 8 == 0 && (estride * ldx) % 4 == 0 &&
      (uintptr_t)X % 16 == 0 && (uintptr_t)out % 16 == 0) {
    hipLaunchKernelGGL(colsum_wide_f32, dim3((C / 8 + 255) / 256), dim3(256), 0, s, (const float*)X, estride * ldx, len,
                       C, out, scale, accum);
    return SDP_CHECK_LAUNCH();
  }
  if (C % 4 == 0 && ldx % 4 == 0 && ldo % 4 == 0 && (uintptr_t)X % (4 * es) == 0 && (uintptr_t)out % 16 == 0) {
    dim3 g4((C / 4 + 63) / 64, G);
    if (dtype == 1)
      hipLaunchKernelGGL(seg_colsum_v4<bf16_t>, g4, dim3(256), 0, s, (const bf16_t*)X, ldx, G, len, gstride, estride, C,
                         out, ldo, scale, accum);
    else if (dtype == 0)
      hipLaunchKernelGGL(seg_colsum_v4<float>, g4, dim3(256), 0, s, (const float*)X, ldx, G, len, gstride, estride, C,
                         out, ldo, scale, accum);
    else
      return (int)hipErrorInvalidValue;
    return SDP_CHECK_LAUNCH();
  }
  dim3 grid((C + 63) / 64, G);
  if (dtype == 1)
    hipLaunchKernelGGL(seg_colsum_k<bf16_t>, grid, dim3(256), 0, s, (const bf16_t*)X, ldx, G, len, gstride, estride, C,
                       out, ldo, scale, accum);
  else if (dtype == 0)
    hipLaunchKernelGGL(seg_colsum_k<float>, grid, dim3(256), 0, s, (const float*)X, ldx, G, len, gstride, estride, C,
                       out, ldo, scale, accum);
  else
    return (int)hipErrorInvalidValue;
  return SDP_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------
// activation forward / backward with dropout (rows of a [M, N] matrix, row stride ld)
//   fwd: y = act(z) * (keep ? 1 / (1 - p) : 0)           (p = 0: no mask)
//   bwd: dz = dy * (keep ? 1 / (1 - p) : 0) * act'(z)
// keep = uniform01(seed, m * N + n) >= p.  Erf-form GELU (nn.GELU(), model.py:15; common.h gelu_erf).
// ---------------------------------------------------------------------------

// 8 consecutive elements of a row per work item (16-B bf16 / 2 x 16-B fp32 accesses); the
// host takes this form when N % 8 == 0 and every row stride / base is 8-element aligned.
template <typename T>
struct V8 {
  float v[8];
  SDP_DEV void load(const T* p) {
    if constexpr (sizeof(T) == 2) {
      const bf16x8 t = *(const bf16x8*)p;
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = bf2f((bf16_t)t[q]);
    } else {
      const f32x4 a = *(const f32x4*)p, b = *(const f32x4*)(p + 4);
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = a[q], v[4 + q] = b[q];
    }
  }
  SDP_DEV void store(T* p) const {
    if constexpr (sizeof(T) == 2) {
      bf16x8 t;
#pragma unroll
      for (int q = 0; q < 8; ++q) t[q] = (short)f2bf(v[q]);
      *(bf16x8*)p = t;
    } else {
      *(f32x4*)p = f32x4{v[0], v[1], v[2], v[3]};
      *(f32x4*)(p + 4) = f32x4{v[4], v[5], v[6], v[7]};
    }
  }
};
// 8 consecutive elements as loaded (bf16 stays packed: 4 registers instead of 8 until used)
template <typename T>
struct Raw8 {
  typename std::conditional<sizeof(T) == 2, bf16x8, f32x4[2]>::type r;
  SDP_DEV void load(const T* p) {
    if constexpr (sizeof(T) == 2) {
      r = *(const bf16x8*)p;
    } else {
      r[0] = *(const f32x4*)p;
      r[1] = *(const f32x4*)(p + 4);
    }
  }
  SDP_DEV float operator[](int q) const {
    if constexpr (sizeof(T) == 2) return bf2f((bf16_t)r[q]);
    else return r[q >> 2][q & 3];
  }
};

// ACT >= 0: the activation fixed at compile time (the model's GELU / ReLU), -1: the run-time code.
// Work items are indexed in 32 bits (the host takes this form for M * N / 8 < 2^31); the dropout
// hash keys once per 8-element run (drop_key), one mix32 per element after that.
template <typename T, int ACT>
__global__ __launch_bounds__(256) void act_fwd_v8(const T* __restrict__ Z, int64_t ldz, T* __restrict__ Y,
                                                  int64_t ldy, int M, int N, int act, float p, uint64_t seed) {
  const uint32_t n8 = (uint32_t)N >> 3;
  const uint32_t total = (uint32_t)M * n8;
  const float inv = p > 0.f ? 1.0f / (1.0f - p) : 1.0f;
  const uint32_t thr = drop_thresh(p);
  const int a = ACT >= 0 ? ACT : act;
  for (uint32_t e = blockIdx.x * 256u + threadIdx.x; e < total; e += gridDim.x * 256u) {
    const uint32_t m = e / n8;
    const uint32_t n = (e - m * n8) * 8u;
    V8<T> x;
    x.load(Z + (int64_t)m * ldz + n);
#pragma unroll
    for (int q = 0; q < 8; ++q) x.v[q] = apply_act(a, x.v[q]);
    if (p > 0.f) {
      const uint64_t base = (uint64_t)m * (uint32_t)N + n;
      const uint32_t key = drop_key(seed, base);
#pragma unroll
      for (int q = 0; q < 8; ++q) x.v[q] = drop_keep(key, (uint32_t)base + q, thr) ? x.v[q] * inv : 0.f;
    }
    x.store(Y + (int64_t)m * ldy + n);
  }
}

template <typename T, int ACT>
__global__ __launch_bounds__(256) void act_bwd_v8(const T* __restrict__ Z, int64_t ldz, const T* __restrict__ DY,
                                                  int64_t lddy, T* __restrict__ DZ, int64_t lddz, int M, int N,
                                                  int act, float p, uint64_t seed) {
  const uint32_t n8 = (uint32_t)N >> 3;
  const uint32_t total = (uint32_t)M * n8;
  const float inv = p > 0.f ? 1.0f / (1.0f - p) : 1.0f;
  const uint32_t thr = drop_thresh(p);
  const int a = ACT >= 0 ? ACT : act;
  for (uint32_t e = blockIdx.x * 256u + threadIdx.x; e < total; e += gridDim.x * 256u) {
    const uint32_t m = e / n8;
    const uint32_t n = (e - m * n8) * 8u;
    V8<T> z, g;
    z.load(Z + (int64_t)m * ldz + n);
    g.load(DY + (int64_t)m * lddy + n);
    if (p > 0.f) {
      const uint64_t base = (uint64_t)m * (uint32_t)N + n;
      const uint32_t key = drop_key(seed, base);
#pragma unroll
      for (int q = 0; q < 8; ++q) g.v[q] = drop_keep(key, (uint32_t)base + q, thr) ? g.v[q] * inv : 0.f;
    }
    if (a != ACT_NONE) {
#pragma unroll
      for (int q = 0; q < 8; ++q) g.v[q] *= act_grad(a, z.v[q]);
    }
    g.store(DZ + (int64_t)m * lddz + n);
  }
}

// X in TX; the residual R and the output Y in TY (TX = bf16 branch, TY = fp32 residual stream
// in the fp32-stream training mode; the reverse for a stream gradient cast into a branch).
template <typename TX, typename TY, int ACT>
__global__ __launch_bounds__(256) void rowscale_v8(const TX* __restrict__ X, int64_t ldx, RowMap xm,
                                                   const float* __restrict__ sc, int sgrp, const TY* __restrict__ R,
                                                   int64_t ldr, RowMap rm, TY* __restrict__ Y, int64_t ldy, RowMap ym,
                                                   int M, int N, int act, float p, uint64_t seed, int dmode) {
  const int n8 = N >> 3;
  const int64_t total = (int64_t)M * n8;
  const float inv = p > 0.f ? 1.0f / (1.0f - p) : 1.0f;
  const uint32_t thr = drop_thresh(p);
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int64_t m = e / n8;
    const int n = (int)(e - m * n8) * 8;
    V8<TX> x;
    x.load(X + xm(m) * ldx + n);
    const int a = ACT >= 0 ? ACT : act;
    if (a != ACT_NONE) {  // = sdp_act_fwd's stored output (rounded to TX) without the round trip
#pragma unroll
      for (int q = 0; q < 8; ++q) x.v[q] = to_f<TX>(from_f<TX>(apply_act(a, x.v[q])));
    }
    const uint64_t base = (uint64_t)m * N + n;
    const uint32_t key = dmode ? drop_key(seed, base) : 0u;
    if (dmode == 1) {  // dropout on the branch (= sdp_act_fwd / sdp_act_bwd with no activation, rounded to TX)
#pragma unroll
      for (int q = 0; q < 8; ++q)
        x.v[q] = to_f<TX>(from_f<TX>(drop_keep(key, (uint32_t)base + q, thr) ? x.v[q] * inv : 0.f));
    }
    const float s_ = sc ? sc[m / sgrp] : 1.0f;
    V8<TY> y;
    if (R) {
      y.load(R + rm(m) * ldr + n);
#pragma unroll
      for (int q = 0; q < 8; ++q) y.v[q] = fmaf(x.v[q], s_, y.v[q]);
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q) y.v[q] = x.v[q] * s_;
    }
    if (dmode == 2) {  // dropout on the rounded output (a stream gradient cast into a dropout branch)
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float r = to_f<TY>(from_f<TY>(y.v[q]));
        y.v[q] = drop_keep(key, (uint32_t)base + q, thr) ? r * inv : 0.f;
      }
    }
    y.store(Y + ym(m) * ldy + n);
  }
}

template <typename T>
struct DTag {
  using type = T;
};

// Calls f(DTag<A>{}, DTag<B>{}) for the (a, b) dtype codes (0 fp32, 1 bf16).
template <typename F>
static int by_dtypes(int a, int b, F&& f) {
  if (a == 1 && b == 1) return f(DTag<bf16_t>{}, DTag<bf16_t>{});
  if (a == 0 && b == 0) return f(DTag<float>{}, DTag<float>{});
  if (a == 0 && b == 1) return f(DTag<float>{}, DTag<bf16_t>{});
  if (a == 1 && b == 0) return f(DTag<bf16_t>{}, DTag<float>{});
  return (int)hipErrorInvalidValue;
}

template <typename T>
__global__ __launch_bounds__(256) void act_fwd_k(const T* __restrict__ Z, int64_t ldz, T* __restrict__ Y, int64_t ldy,
                                                 int M, int N, int act, float p, uint64_t seed) {
  const int64_t total = (int64_t)M * N;
  const float inv = p > 0.f ? 1.0f / (1.0f - p) : 1.0f;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int64_t m = e / N, n = e % N;
    float v = apply_act(act, to_f<T>(Z[m * ldz + n]));
    if (p > 0.f) v = uniform01(seed, e) >= p ? v * inv : 0.f;
    Y[m * ldy + n] = from_f<T>(v);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void act_bwd_k(const T* __restrict__ Z, int64_t ldz, const T* __restrict__ DY,
                                                 int64_t lddy, T* __restrict__ DZ, int64_t lddz, int M, int N, int act,
                                                 float p, uint64_t seed) {
  const int64_t total = (int64_t)M * N;
  const float inv = p > 0.f ? 1.0f / (1.0f - p) : 1.0f;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int64_t m = e / N, n = e % N;
    float g = to_f<T>(DY[m * lddy + n]);
    if (p > 0.f) g = uniform01(seed, e) >= p ? g * inv : 0.f;
    DZ[m * lddz + n] = from_f<T>(g * act_grad(act, to_f<T>(Z[m * ldz + n])));
  }
}

static int ew_grid(int64_t total) {
  int64_t g = (total + 255) / 256;
  return (int)(g < 16384 ? (g > 0 ? g : 1) : 16384);
}

extern "C" int sdp_act_fwd(int dtype, const void* Z, int64_t ldz, void* Y, int64_t ldy, int M, int N, int act, float p,
                           uint64_t seed, void* stream) {
  if (!Z || !Y || M < 0 || N < 0 || p < 0.f || p >= 1.f) return (int)hipErrorInvalidValue;
  if ((int64_t)M * N == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const int es = dtype == 1 ? 2 : 4;
  if (N % 8 == 0 && ldz % 8 == 0 && ldy % 8 == 0 && (uintptr_t)Z % 16 == 0 && (uintptr_t)Y % 16 == 0 && (es == 2 || es == 4) &&
      (int64_t)M * (N / 8) < (1ll << 31)) {
    const int gv = ew_grid((int64_t)M * (N / 8));
    auto go = [&](auto tag) {
      using T = typename decltype(tag)::type;
#define SDP_AF(A) hipLaunchKernelGGL((act_fwd_v8<T, A>), dim3(gv), dim3(256), 0, s, (const T*)Z, ldz, (T*)Y, ldy, M, N, act, p, seed)
      if (act == ACT_GELU) SDP_AF(ACT_GELU);
      else if (act == ACT_NONE) SDP_AF(ACT_NONE);
      else SDP_AF(-1);
#undef SDP_AF
      return SDP_CHECK_LAUNCH();
    };
    if (dtype == 1) return go(DTag<bf16_t>{});
    if (dtype == 0) return go(DTag<float>{});
    return (int)hipErrorInvalidValue;
  }
  const int g = ew_grid((int64_t)M * N);
  if (dtype == 1)
    hipLaunchKernelGGL(act_fwd_k<bf16_t>, dim3(g), dim3(256), 0, s, (const bf16_t*)Z, ldz, (bf16_t*)Y, ldy, M, N, act, p, seed);
  else if (dtype == 0)
    hipLaunchKernelGGL(act_fwd_k<float>, dim3(g), dim3(256), 0, s, (const float*)Z, ldz, (float*)Y, ldy, M, N, act, p, seed);
  else
    return (int)hipErrorInvalidValue;
  return SDP_CHECK_LAUNCH();
}

extern "C" int sdp_act_bwd(int dtype, const void* Z, int64_t ldz, const void* DY, int64_t lddy, void* DZ, int64_t lddz,
                           int M, int N, int act, float p, uint64_t seed, void* stream) {
  if (!Z || !DY || !DZ || M < 0 || N < 0 || p < 0.f || p >= 1.f) return (int)hipErrorInvalidValue;
  if ((int64_t)M * N == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  if (N % 8 == 0 && ldz % 8 == 0 && lddy % 8 == 0 && lddz % 8 == 0 && (uintptr_t)Z % 16 == 0 &&
      (uintptr_t)DY % 16 == 0 && (uintptr_t)DZ % 16 == 0 && (int64_t)M * (N / 8) < (1ll << 31)) {
    const int gv = ew_grid((int64_t)M * (N / 8));
    auto go = [&](auto tag) {
      using T = typename decltype(tag)::type;
#define SDP_AB(A)                                                                                                  \
  hipLaunchKernelGGL((act_bwd_v8<T, A>), dim3(gv), dim3(256), 0, s, (const T*)Z, ldz, (const T*)DY, lddy, (T*)DZ, lddz, \
                     M, N, act, p, seed)
      if (act == ACT_GELU) SDP_AB(ACT_GELU);
      else if (act == ACT_NONE) SDP_AB(ACT_NONE);
      else SDP_AB(-1);
#undef SDP_AB
      return SDP_CHECK_LAUNCH();
    };
    if (dtype == 1) return go(DTag<bf16_t>{});
    if (dtype == 0) return go(DTag<float>{});
    return (int)hipErrorInvalidValue;
  }
  const int g = ew_grid((int64_t)M * N);
  if (dtype == 1)
    hipLaunchKernelGGL(act_bwd_k<bf16_t>, dim3(g), dim3(256), 0, s, (const bf16_t*)Z, ldz, (const bf16_t*)DY, lddy,
                       (bf16_t*)DZ, lddz, M, N, act, p, seed);
  else if (dtype == 0)
    hipLaunchKernelGGL(act_bwd_k<float>, dim3(g), dim3(256), 0, s, (const float*)Z, ldz, (const float*)DY, lddy,
                       (float*)DZ, lddz, M, N, act, p, seed);
  else
    return (int)hipErrorInvalidValue;
  return SDP_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------
// Per-sample row scaling (drop path, utility_layers.py:16-27): y[m] = x[m] * scale[m / grp]
// plus an optional residual: y = x * s + r.  In place allowed (y == x).
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void rowscale_k(const T* __restrict__ X, int64_t ldx, RowMap xm,
                                                  const float* __restrict__ sc, int sgrp, const T* __restrict__ R,
                                                  int64_t ldr, RowMap rm, T* __restrict__ Y, int64_t ldy, RowMap ym,
                                                  int M, int N, int act) {
  const int64_t total = (int64_t)M * N;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int64_t m = e / N, n = e % N;
    float x = to_f<T>(X[xm(m) * ldx + n]);
    if (act != ACT_NONE) x = to_f<T>(from_f<T>(apply_act(act, x)));
    float v = x * (sc ? sc[m / sgrp] : 1.0f);
    if (R) v += to_f<T>(R[rm(m) * ldr + n]);
    Y[ym(m) * ldy + n] = from_f<T>(v);
  }
}

static int rowscale_impl(int xdt, int ydt, int act, const void* X, int64_t ldx, int x_grp, int64_t x_gstride,
                         int x_off, const float* scale, int sgrp, const void* R, int64_t ldr, int r_grp,
                         int64_t r_gstride, int r_off, void* Y, int64_t ldy, int y_grp, int64_t y_gstride, int y_off,
                         int M, int N, void* stream, float p = 0.f, uint64_t seed = 0, int dmode = 0) {
  if (!X || !Y || M < 0 || N < 0 || (scale && sgrp <= 0) || act < 0 || act > ACT_KELU) return (int)hipErrorInvalidValue;
  if (p < 0.f || p >= 1.f || dmode < 0 || dmode > 2) return (int)hipErrorInvalidValue;
  if (p == 0.f) dmode = 0;
  if ((int64_t)M * N == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const RowMap xm = mk_tmap(x_grp, x_gstride, x_off), rm = mk_tmap(r_grp, r_gstride, r_off),
               ym = mk_tmap(y_grp, y_gstride, y_off);
  if (N % 8 == 0 && ldx % 8 == 0 && ldy % 8 == 0 && (!R || (ldr % 8 == 0 && (uintptr_t)R % 16 == 0)) &&
      (uintptr_t)X % 16 == 0 && (uintptr_t)Y % 16 == 0) {
    const int gv = ew_grid((int64_t)M * (N / 8));
    return by_dtypes(xdt, ydt, [&](auto tx, auto ty) {
      using TX = typename decltype(tx)::type;
      using TY = typename decltype(ty)::type;
      if (act == ACT_GELU)
        hipLaunchKernelGGL((rowscale_v8<TX, TY, ACT_GELU>), dim3(gv), dim3(256), 0, s, (const TX*)X, ldx, xm, scale,
                           sgrp, (const TY*)R, ldr, rm, (TY*)Y, ldy, ym, M, N, act, p, seed, dmode);
      else
        hipLaunchKernelGGL((rowscale_v8<TX, TY, -1>), dim3(gv), dim3(256), 0, s, (const TX*)X, ldx, xm, scale, sgrp,
                           (const TY*)R, ldr, rm, (TY*)Y, ldy, ym, M, N, act, p, seed, dmode);
      return SDP_CHECK_LAUNCH();
    });
  }
  if (xdt != ydt) return (int)hipErrorInvalidValue;  // mixed dtypes: 16-B aligned rows, N % 8 == 0 only
  if (dmode) return (int)hipErrorNotSupported;       // fused dropout: the vector path only
  const int g = ew_grid((int64_t)M * N);
  if (xdt == 1)
    hipLaunchKernelGGL(rowscale_k<bf16_t>, dim3(g), dim3(256), 0, s, (const bf16_t*)X, ldx, xm, scale, sgrp,
                       (const bf16_t*)R, ldr, rm, (bf16_t*)Y, ldy, ym, M, N, act);
  else if (xdt == 0)
    hipLaunchKernelGGL(rowscale_k<float>, dim3(g), dim3(256), 0, s, (const float*)X, ldx, xm, scale, sgrp,
                       (const float*)R, ldr, rm, (float*)Y, ldy, ym, M, N, act);
  else
    return (int)hipErrorInvalidValue;
  return SDP_CHECK_LAUNCH();
}

extern "C" int sdp_rowscale_add(int dtype, const void* X, int64_t ldx, int x_grp, int64_t x_gstride, int x_off,
                                const float* scale, int sgrp, const void* R, int64_t ldr, int r_grp, int64_t r_gstride,
                                int r_off, void* Y, int64_t ldy, int y_grp, int64_t y_gstride, int y_off, int M, int N,
                                void* stream) {
  return rowscale_impl(dtype, dtype, ACT_NONE, X, ldx, x_grp, x_gstride, x_off, scale, sgrp, R, ldr, r_grp, r_gstride,
                       r_off, Y, ldy, y_grp, y_gstride, y_off, M, N, stream);
}

// Y = act(X) * scale + R: activation, drop path and residual add of a ConvMixer branch in one
// pass (the activation output itself is not needed by the backward).
extern "C" int sdp_act_rowscale_add(int dtype, int act, const void* X, int64_t ldx, int x_grp, int64_t x_gstride,
                                    int x_off, const float* scale, int sgrp, const void* R, int64_t ldr, int r_grp,
                                    int64_t r_gstride, int r_off, void* Y, int64_t ldy, int y_grp, int64_t y_gstride,
                                    int y_off, int M, int N, void* stream) {
  return rowscale_impl(dtype, dtype, act, X, ldx, x_grp, x_gstride, x_off, scale, sgrp, R, ldr, r_grp, r_gstride,
                       r_off, Y, ldy, y_grp, y_gstride, y_off, M, N, stream);
}

// Mixed-dtype form: X in x_dtype, R and Y in y_dtype (fp32 residual stream of bf16 training:
// y32 = act(x16) * scale + r32, or a stream gradient cast into a branch, y16 = x32 * scale).
extern "C" int sdp_rowscale_add_mixed(int x_dtype, int y_dtype, int act, const void* X, int64_t ldx, int x_grp,
                                      int64_t x_gstride, int x_off, const float* scale, int sgrp, const void* R,
                                      int64_t ldr, int r_grp, int64_t r_gstride, int r_off, void* Y, int64_t ldy,
                                      int y_grp, int64_t y_gstride, int y_off, int M, int N, void* stream) {
  return rowscale_impl(x_dtype, y_dtype, act, X, ldx, x_grp, x_gstride, x_off, scale, sgrp, R, ldr, r_grp, r_gstride,
                       r_off, Y, ldy, y_grp, y_gstride, y_off, M, N, stream);
}

// The same with a dropout mask (the counter hash of sdp_act_fwd / sdp_act_bwd, index m * N + n
// over the logical rows): mode 1 drops the branch X before the scale and the residual add,
// y = dropout(X) * scale + R (EncoderLayer's x + drop_path(dropout(proj(.))), layers.py:301-309);
// mode 2 drops the rounded output, y = dropout(round(X * scale)) (its gradient cast into the
// branch).  Bit-identical to sdp_act_fwd / sdp_act_bwd followed by sdp_rowscale_add[_mixed] and
// the reverse; 16-B aligned rows and N % 8 == 0 only (hipErrorNotSupported otherwise).
extern "C" int sdp_rowscale_add_dropout(int x_dtype, int y_dtype, const void* X, int64_t ldx, int x_grp,
                                        int64_t x_gstride, int x_off, const float* scale, int sgrp, const void* R,
                                        int64_t ldr, int r_grp, int64_t r_gstride, int r_off, void* Y, int64_t ldy,
                                        int y_grp, int64_t y_gstride, int y_off, int M, int N, float p, uint64_t seed,
                                        int mode, void* stream) {
  if (mode != 1 && mode != 2) return (int)hipErrorInvalidValue;
  return rowscale_impl(x_dtype, y_dtype, ACT_NONE, X, ldx, x_grp, x_gstride, x_off, scale, sgrp, R, ldr, r_grp,
                       r_gstride, r_off, Y, ldy, y_grp, y_gstride, y_off, M, N, stream, p, seed, mode);
}

// ---------------------------------------------------------------------------
// LayerNorm with given statistics (stats[2m] = mean, stats[2m+1] = rstd): y = (x - mean) * rstd * g + b
// and its backward.  One wave per row, any C.
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void ln_apply_k(const T* __restrict__ X, int64_t ldx, RowMap xm,
                                                  const float* __restrict__ st, const float* __restrict__ g,
                                                  const float* __restrict__ b, T* __restrict__ Y, int64_t ldy,
                                                  RowMap ym, int M, int C) {
  const int lane = threadIdx.x & 63;
  const int64_t m = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= M) return;
  const float mean = st[2 * m], rstd = st[2 * m + 1];
  const T* xp = X + xm(m) * ldx;
  T* yp = Y + ym(m) * ldy;
  for (int c = lane; c < C; c += 64) yp[c] = from_f<T>((to_f<T>(xp[c]) - mean) * rstd * g[c] + b[c]);
}

// dx = rstd * (gdy - mean(gdy) - xhat * mean(gdy * xhat)) [+ add];  per-block partials of
// dgamma = sum dy * xhat, dbeta = sum dy in part[blockIdx.x][2][C].  V = ceil(C / 64) values
// per lane (compile time, so the per-row arrays stay in registers).
template <typename T, int V>
__global__ __launch_bounds__(256) void ln_bwd_k(const T* __restrict__ X, int64_t ldx, RowMap xm,
                                                const float* __restrict__ st, const float* __restrict__ g,
                                                const T* __restrict__ DY, int64_t lddy, RowMap dym,
                                                const T* __restrict__ ADD, int64_t ldadd, RowMap am,
                                                T* __restrict__ DX, int64_t lddx, RowMap dxm, int M, int C,
                                                float* __restrict__ part) {
  extern __shared__ float red[];  // [2][4][C]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float dg[V], db[V], gv[V];
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const int c = lane + 64 * i;
    dg[i] = db[i] = 0.f;
    gv[i] = c < C ? g[c] : 0.f;
  }
  for (int64_t m = (int64_t)blockIdx.x * 4 + w; m < M; m += (int64_t)gridDim.x * 4) {
    const float mean = st[2 * m], rstd = st[2 * m + 1];
    const T* xp = X + xm(m) * ldx;
    const T* dyp = DY + dym(m) * lddy;
    float xh[V], gd[V];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < V; ++i) {
      const int c = lane + 64 * i;
      xh[i] = gd[i] = 0.f;
      if (c < C) {
        const float dy = to_f<T>(dyp[c]);
        xh[i] = (to_f<T>(xp[c]) - mean) * rstd;
        gd[i] = dy * gv[i];
        dg[i] += dy * xh[i];
        db[i] += dy;
        s1 += gd[i];
        s2 += gd[i] * xh[i];
      }
    }
    s1 = wave_sum(s1) / (float)C;
    s2 = wave_sum(s2) / (float)C;
    T* dxp = DX + dxm(m) * lddx;
    const T* ap = ADD ? ADD + am(m) * ldadd : nullptr;
#pragma unroll
    for (int i = 0; i < V; ++i) {
      const int c = lane + 64 * i;
      if (c < C) {
        float v = rstd * (gd[i] - s1 - xh[i] * s2);
        if (ap) v += to_f<T>(ap[c]);
        dxp[c] = from_f<T>(v);
      }
    }
  }
  if (!part) return;
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const int c = lane + 64 * i;
    if (c < C) {
      red[(0 * 4 + w) * C + c] = dg[i];
      red[(1 * 4 + w) * C + c] = db[i];
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    part[(int64_t)blockIdx.x * 2 * C + c] = red[0 * C + c] + red[1 * C + c] + red[2 * C + c] + red[3 * C + c];
    part[(int64_t)blockIdx.x * 2 * C + C + c] =
        red[4 * C + c] + red[5 * C + c] + red[6 * C + c] + red[7 * C + c];
  }
}

// Register rows carried past a ConvMixer (layers.py:99-104 transforms the image rows only): rows
// b * N + i (i < R, b < B) of src copied to dst0 (and dst1), row pitch ld bytes, `bytes` per row
// (a multiple of 16, 16-B aligned).  One wave per row, folded into a row kernel the layer runs anyway
// instead of a copy launch per buffer.
struct RegCopy {
  const char* src;
  char* dst0;
  char* dst1;
  int64_t ld;
  int B, R, N, bytes;
};
SDP_DEV void reg_copy_row(const RegCopy& rc, int w, int lane) {
  if (!rc.src || w >= rc.B * rc.R) return;
  const int b = w / rc.R, i = w - b * rc.R;
  const int64_t off = ((int64_t)b * rc.N + i) * rc.ld;
  for (int o = lane * 16; o < rc.bytes; o += 64 * 16) {
    const int4 v = *(const int4*)(rc.src + off + o);
    *(int4*)(rc.dst0 + off + o) = v;
    if (rc.dst1) *(int4*)(rc.dst1 + off + o) = v;
  }
}
static bool reg_copy_ok(const RegCopy& rc) {
  auto a16 = [](const void* q) { return (uintptr_t)q % 16 == 0; };
  return !rc.src || (rc.dst0 && a16(rc.src) && a16(rc.dst0) && (!rc.dst1 || a16(rc.dst1)) && rc.ld % 16 == 0 &&
                     rc.bytes % 16 == 0 && rc.bytes <= rc.ld && rc.B >= 0 && rc.R >= 0 && rc.N >= rc.R);
}

// What a LayerNorm backward can hand on in the same pass (training, fp32 residual stream): the
// gradient of the branch that fed the LayerNorm input, in the branch dtype (bf16, dense rows), as the
// two passes after it computed it from the stored dX:
//   h = bf16(dX * scale[m / sgrp])                          (sdp_rowscale_add, drop path)
//   dmode 2: h = bf16(keep(seed, m * C + c) ? h / (1 - p) : 0)  (the branch's dropout, on the rounded h)
//   act:     h = bf16(h * act'(Z))                          (sdp_act_bwd: the branch activation)
struct LnBwdEmit {
  const float* sc;
  int sgrp;
  const bf16_t* z;
  int64_t ldz;
  int act;
  float p;
  uint64_t seed;
  int dmode;
  bf16_t* o2;
  int64_t ldo2;
};

// Deterministic in-kernel reduction of per-block column partials (part[b][0 .. n)): blocks are
// grouped GS at a time; the last block of a group to finish (device-scope ticket) sums the group's
// partials in block order into gpart[g], the last group to finish sums gpart in group order into
// out.  The sums' order never depends on which block arrives last; tickets are reset by their last
// user, so a buffer serves any number of launches on one stream.
template <int NT>
SDP_DEV void ticket_colsum(const float* part, int nb, int n, int gs, float* gpart, float* out, int* ticket) {
  __shared__ int s_last;
  __threadfence();  // this block's partials visible device-wide before its ticket
  __syncthreads();
  const int g = blockIdx.x / gs, ng = (nb + gs - 1) / gs;
  const int b0 = g * gs, nin = min(gs, nb - b0);
  if (threadIdx.x == 0) s_last = atomicAdd(&ticket[g], 1) == nin - 1;
  __syncthreads();
  if (!s_last) return;
  __threadfence();
  for (int c = threadIdx.x * 4; c < n; c += NT * 4) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    int r = 0;
    for (; r + 8 <= nin; r += 8) {
      f32x4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = *(const f32x4*)(part + (int64_t)(b0 + r + u) * n + c);
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; r < nin; ++r) acc += *(const f32x4*)(part + (int64_t)(b0 + r) * n + c);
    *(f32x4*)(gpart + (int64_t)g * n + c) = acc;
  }
  __threadfence();
  __syncthreads();
  if (threadIdx.x == 0) {
    ticket[g] = 0;
    s_last = atomicAdd(&ticket[ng], 1) == ng - 1;
  }
  __syncthreads();
  if (!s_last) return;
  __threadfence();
  for (int c = threadIdx.x * 4; c < n; c += NT * 4) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    int r = 0;
    for (; r + 8 <= ng; r += 8) {
      f32x4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = *(const f32x4*)(gpart + (int64_t)(r + u) * n + c);
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; r < ng; ++r) acc += *(const f32x4*)(gpart + (int64_t)r * n + c);
    *(f32x4*)(out + c) = acc;
  }
  if (threadIdx.x == 0) ticket[ng] = 0;
}

// Same backward, 8 consecutive channels per lane (16-B accesses; C % 8 == 0, aligned rows):
// lane covers channels 8 * lane + 512 * i, i < V.  EA != LNB_NOEMIT: also writes the branch gradient
// (LnBwdEmit) with activation EA (the model's GELU / none at compile time, -1: em.act at run time);
// ticket != nullptr: the affine partials are reduced in the same launch (ticket_colsum).
constexpr int LNB_NOEMIT = -100;  // EA of a LayerNorm backward without the branch-gradient output

template <typename T, typename TD, int V, int EA>
__global__ __launch_bounds__(256) void ln_bwd_v8(const T* __restrict__ X, int64_t ldx, RowMap xm,
                                                 const float* __restrict__ st, const float* __restrict__ g,
                                                 const TD* __restrict__ DY, int64_t lddy, RowMap dym,
                                                 const T* __restrict__ ADD, int64_t ldadd, RowMap am,
                                                 T* __restrict__ DX, int64_t lddx, RowMap dxm, int M, int C,
                                                 float* __restrict__ part, float* gpart, float* aff, int* ticket,
                                                 LnBwdEmit em, RegCopy rc) {
  constexpr bool EM = EA != LNB_NOEMIT;
  [[maybe_unused]] const int ea = EA >= 0 ? EA : em.act;  // the emitted gradient's activation
  extern __shared__ float red[];  // [2][4][C]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (rc.src)
    for (int gw = blockIdx.x * 4 + w; gw < rc.B * rc.R; gw += gridDim.x * 4) reg_copy_row(rc, gw, lane);
  float dg[V][8], db[V][8];
#pragma unroll
  for (int i = 0; i < V; ++i)
#pragma unroll
    for (int q = 0; q < 8; ++q) dg[i][q] = db[i][q] = 0.f;
  // software-pipelined over the wave's rows: row m + stride's X / dY / addend loads are issued
  // before row m's reductions and stores, so each wave keeps one row of loads in flight while it
  // computes (one row at a time left every wave waiting a memory round trip per row)
  const int64_t stride = (int64_t)gridDim.x * 4;
  struct RowIn {
    Raw8<T> x[V], a[V];
    Raw8<TD> dy[V];
    Raw8<bf16_t> z[V];
    float mean, rstd;
  };
  auto fetch = [&](int64_t m, RowIn& r) {
    r.mean = st[2 * m];
    r.rstd = st[2 * m + 1];
    const T* xp = X + xm(m) * ldx;
    const TD* dyp = DY + dym(m) * lddy;
    const T* ap = ADD ? ADD + am(m) * ldadd : nullptr;
#pragma unroll
    for (int i = 0; i < V; ++i) {
      const int c = 8 * lane + 512 * i;
      if (c < C) {
        r.dy[i].load(dyp + c);
        r.x[i].load(xp + c);
        if (ap) r.a[i].load(ap + c);
        if constexpr (EM) {
          if (ea != ACT_NONE) r.z[i].load(em.z + m * em.ldz + c);
        }
      }
    }
  };
  [[maybe_unused]] const float inv2 = EM && em.p > 0.f ? 1.0f / (1.0f - em.p) : 1.0f;
  [[maybe_unused]] const uint32_t thr2 = EM ? drop_thresh(em.p) : 0u;
  int64_t m = (int64_t)blockIdx.x * 4 + w;
  RowIn cur, nxt;
  if (m < M) fetch(m, cur);
  for (; m < M; m += stride) {
    if (m + stride < M) fetch(m + stride, nxt);
    const float mean = cur.mean, rstd = cur.rstd;
    T* dxp = DX + dxm(m) * lddx;
    V8<T> xh[V], gd[V];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < V; ++i) {
      const int c = 8 * lane + 512 * i;
      if (c < C) {
        const f32x4 g0 = *(const f32x4*)(g + c), g1 = *(const f32x4*)(g + c + 4);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const float dyq = cur.dy[i][q];
          const float x_ = (cur.x[i][q] - mean) * rstd;
          xh[i].v[q] = x_;
          gd[i].v[q] = dyq * (q < 4 ? g0[q] : g1[q - 4]);
          dg[i][q] = fmaf(dyq, x_, dg[i][q]);
          db[i][q] += dyq;
          s1 += gd[i].v[q];
          s2 = fmaf(gd[i].v[q], x_, s2);
        }
      }
    }
    s1 = wave_sum(s1) / (float)C;
    s2 = wave_sum(s2) / (float)C;
    [[maybe_unused]] float s_ = 1.0f;
    if constexpr (EM) s_ = em.sc ? em.sc[m / em.sgrp] : 1.0f;
#pragma unroll
    for (int i = 0; i < V; ++i) {
      const int c = 8 * lane + 512 * i;
      if (c < C) {
        V8<T> o;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const float v = rstd * (gd[i].v[q] - s1 - xh[i].v[q] * s2);
          o.v[q] = ADD ? cur.a[i][q] + v : v;
        }
        o.store(dxp + c);
        if constexpr (EM) {  // the two passes that followed, on the stored value (rounded to T)
          const uint64_t base = (uint64_t)m * C + c;
          const uint32_t key = em.dmode == 2 ? drop_key(em.seed, base) : 0u;
          bf16x8 hv;
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            float h = to_f<T>(from_f<T>(o.v[q])) * s_;
            if (em.dmode == 2) {
              const float r = bf2f(f2bf(h));
              h = drop_keep(key, (uint32_t)base + q, thr2) ? r * inv2 : 0.f;
            }
            h = bf2f(f2bf(h));
            if (ea != ACT_NONE) h = h * act_grad(ea, cur.z[i][q]);
            hv[q] = (short)f2bf(h);
          }
          *(bf16x8*)(em.o2 + m * em.ldo2 + c) = hv;
        }
      }
    }
    cur = nxt;
  }
  if (!part) return;
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const int c = 8 * lane + 512 * i;
    if (c < C) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        red[(0 * 4 + w) * C + c + q] = dg[i][q];
        red[(1 * 4 + w) * C + c + q] = db[i][q];
      }
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    part[(int64_t)blockIdx.x * 2 * C + c] = red[0 * C + c] + red[1 * C + c] + red[2 * C + c] + red[3 * C + c];
    part[(int64_t)blockIdx.x * 2 * C + C + c] =
        red[4 * C + c] + red[5 * C + c] + red[6 * C + c] + red[7 * C + c];
  }
  if (ticket) ticket_colsum<256>(part, gridDim.x, 2 * C, 32, gpart, aff, ticket);
}

// LayerNorm forward that also writes its statistics (training forward keeps them for the
// backward): one wave per row, 8 consecutive channels per lane (C % 8 == 0, <= 2048).
template <typename T, typename TY, int V>
__global__ __launch_bounds__(256) void ln_fwd_v8(const T* __restrict__ X, int64_t ldx, RowMap xm, float eps,
                                                 const float* __restrict__ g, const float* __restrict__ b,
                                                 float* __restrict__ st, TY* __restrict__ Y, int64_t ldy, RowMap ym,
                                                 int M, int C) {
  const int lane = threadIdx.x & 63;
  const int64_t m = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= M) return;
  const T* xp = X + xm(m) * ldx;
  V8<T> x[V];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const int c = 8 * lane + 512 * i;
    if (c < C) {
      x[i].load(xp + c);
#pragma unroll
      for (int q = 0; q < 8; ++q) s += x[i].v[q];
    }
  }
  const float mean = wave_sum(s) / (float)C;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const int c = 8 * lane + 512 * i;
    if (c < C) {
#pragma unroll
      for (int q = 0; q < 8; ++q) ss = fmaf(x[i].v[q] - mean, x[i].v[q] - mean, ss);
    }
  }
  const float rstd = 1.0f / sqrtf(wave_sum(ss) / (float)C + eps);
  if (lane == 0) *(float2*)(st + 2 * m) = float2{mean, rstd};
  TY* yp = Y + ym(m) * ldy;
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const int c = 8 * lane + 512 * i;
    if (c < C) {
      const f32x4 g0 = *(const f32x4*)(g + c), g1 = *(const f32x4*)(g + c + 4);
      const f32x4 b0 = *(const f32x4*)(b + c), b1 = *(const f32x4*)(b + c + 4);
      V8<TY> y;
#pragma unroll
      for (int q = 0; q < 8; ++q)
        y.v[q] = (x[i].v[q] - mean) * rstd * (q < 4 ? g0[q] : g1[q - 4]) + (q < 4 ? b0[q] : b1[q - 4]);
      y.store(yp + c);
    }
  }
}

// Short rows (C <= 128, the per-head q/k LayerNorm of hd = 64..128): L = pow2 >= C / 8
// lanes per row, 64 / L rows per wave (one wave per row would leave 52 of 64 lanes idle
// at hd = 96); reductions stay inside each L-lane segment.
template <int L>
SDP_DEV float seg_sum(float v) {
#pragma unroll
  for (int o = 1; o < L; o <<= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <typename T, typename TY, int L>
__global__ __launch_bounds__(256) void ln_fwd_sm(const T* __restrict__ X, int64_t ldx, RowMap xm, float eps,
                                                 const float* __restrict__ g, const float* __restrict__ b,
                                                 float* __restrict__ st, TY* __restrict__ Y, int64_t ldy, RowMap ym,
                                                 int M, int C) {
  constexpr int R = 64 / L;
  const int lane = threadIdx.x & 63, seg = lane / L, sl = lane % L;
  const int64_t m = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * R + seg;
  const int c = 8 * sl;
  const bool act = m < M && c < C;
  V8<T> x;
  float s = 0.f;
  if (act) {
    x.load(X + xm(m) * ldx + c);
#pragma unroll
    for (int q = 0; q < 8; ++q) s += x.v[q];
  }
  const float mean = seg_sum<L>(s) / (float)C;
  float ss = 0.f;
  if (act) {
#pragma unroll
    for (int q = 0; q < 8; ++q) ss = fmaf(x.v[q] - mean, x.v[q] - mean, ss);
  }
  const float rstd = 1.0f / sqrtf(seg_sum<L>(ss) / (float)C + eps);
  if (m < M && sl == 0) *(float2*)(st + 2 * m) = float2{mean, rstd};
  if (act) {
    const f32x4 g0 = *(const f32x4*)(g + c), g1 = *(const f32x4*)(g + c + 4);
    const f32x4 b0 = *(const f32x4*)(b + c), b1 = *(const f32x4*)(b + c + 4);
    V8<TY> y;
#pragma unroll
    for (int q = 0; q < 8; ++q)
      y.v[q] = (x.v[q] - mean) * rstd * (q < 4 ? g0[q] : g1[q - 4]) + (q < 4 ? b0[q] : b1[q - 4]);
    y.store(Y + ym(m) * ldy + c);
  }
}

template <typename T, typename TD, int L>
__global__ __launch_bounds__(256) void ln_bwd_sm(const T* __restrict__ X, int64_t ldx, RowMap xm,
                                                 const float* __restrict__ st, const float* __restrict__ g,
                                                 const TD* __restrict__ DY, int64_t lddy, RowMap dym,
                                                 const T* __restrict__ ADD, int64_t ldadd, RowMap am,
                                                 T* __restrict__ DX, int64_t lddx, RowMap dxm, int M, int C,
                                                 float* __restrict__ part) {
  extern __shared__ float red[];  // [2][4][C]
  constexpr int R = 64 / L;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, seg = lane / L, sl = lane % L;
  const int c = 8 * sl;
  float dg[8], db[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) dg[q] = db[q] = 0.f;
  f32x4 g0 = {0.f, 0.f, 0.f, 0.f}, g1 = g0;
  if (c < C) {
    g0 = *(const f32x4*)(g + c);
    g1 = *(const f32x4*)(g + c + 4);
  }
  // the wave's first row decides the trip count (uniform: the segment sums shuffle)
  for (int64_t mb = ((int64_t)blockIdx.x * 4 + w) * R; mb < M; mb += (int64_t)gridDim.x * 4 * R) {
    const int64_t m = mb + seg;
    const bool act = m < M && c < C;
    float mean = 0.f, rstd = 0.f;
    V8<T> xh, gd;
    float s1 = 0.f, s2 = 0.f;
    if (act) {
      mean = st[2 * m];
      rstd = st[2 * m + 1];
      V8<TD> dy;
      dy.load(DY + dym(m) * lddy + c);
      xh.load(X + xm(m) * ldx + c);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float x_ = (xh.v[q] - mean) * rstd;
        xh.v[q] = x_;
        gd.v[q] = dy.v[q] * (q < 4 ? g0[q] : g1[q - 4]);
        dg[q] = fmaf(dy.v[q], x_, dg[q]);
        db[q] += dy.v[q];
        s1 += gd.v[q];
        s2 = fmaf(gd.v[q], x_, s2);
      }
    }
    s1 = seg_sum<L>(s1) / (float)C;
    s2 = seg_sum<L>(s2) / (float)C;
    if (act) {
      V8<T> o;
      const T* ap = ADD ? ADD + am(m) * ldadd : nullptr;
      if (ap) o.load(ap + c);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float v = rstd * (gd.v[q] - s1 - xh.v[q] * s2);
        o.v[q] = ap ? o.v[q] + v : v;
      }
      o.store(DX + dxm(m) * lddx + c);
    }
  }
  if (!part) return;
  // the R row segments of a wave hold the same channels: fold them onto segment 0
#pragma unroll
  for (int o = L; o < 64; o <<= 1)
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      dg[q] += __shfl_xor(dg[q], o, 64);
      db[q] += __shfl_xor(db[q], o, 64);
    }
  if (seg == 0 && c < C) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      red[(0 * 4 + w) * C + c + q] = dg[q];
      red[(1 * 4 + w) * C + c + q] = db[q];
    }
  }
  __syncthreads();
  for (int cc = threadIdx.x; cc < C; cc += 256) {
    part[(int64_t)blockIdx.x * 2 * C + cc] = red[0 * C + cc] + red[1 * C + cc] + red[2 * C + cc] + red[3 * C + cc];
    part[(int64_t)blockIdx.x * 2 * C + C + cc] =
        red[4 * C + cc] + red[5 * C + cc] + red[6 * C + cc] + red[7 * C + cc];
  }
}

static int ln_fwd_impl(int xdt, int ydt, const void* X, int64_t ldx, int x_grp, int64_t x_gstride, int x_off,
                       float eps, const float* gamma, const float* beta, float* stats, void* Y, int64_t ldy, int y_grp,
                       int64_t y_gstride, int y_off, int M, int C, void* stream) {
  if (!X || !Y || !stats || !gamma || !beta || M < 0 || C <= 0 || C > 2048 || C % 8) return (int)hipErrorInvalidValue;
  if (ldx % 8 || ldy % 8 || (uintptr_t)X % 16 || (uintptr_t)Y % 16 || (uintptr_t)gamma % 16 || (uintptr_t)beta % 16 ||
      (uintptr_t)stats % 8)
    return (int)hipErrorInvalidValue;
  if (M == 0) return 0;
  const RowMap xm = mk_tmap(x_grp, x_gstride, x_off), ym = mk_tmap(y_grp, y_gstride, y_off);
  hipStream_t s = (hipStream_t)stream;
  return by_dtypes(xdt, ydt, [&](auto tx, auto ty) {
    using TX = typename decltype(tx)::type;
    using TY = typename decltype(ty)::type;
    if (C <= 128) {  // several rows per wave
      const int L = C <= 64 ? 8 : 16, R = 64 / L;
      const dim3 gs((M + 4 * R - 1) / (4 * R));
      if (L == 8)
        hipLaunchKernelGGL((ln_fwd_sm<TX, TY, 8>), gs, dim3(256), 0, s, (const TX*)X, ldx, xm, eps, gamma, beta, stats,
                           (TY*)Y, ldy, ym, M, C);
      else
        hipLaunchKernelGGL((ln_fwd_sm<TX, TY, 16>), gs, dim3(256), 0, s, (const TX*)X, ldx, xm, eps, gamma, beta,
                           stats, (TY*)Y, ldy, ym, M, C);
      return SDP_CHECK_LAUNCH();
    }
    const dim3 grid((M + 3) / 4);
    const int v8 = (C + 511) / 512;
#define SDP_LNF(VV)                                                                                                \
  hipLaunchKernelGGL((ln_fwd_v8<TX, TY, VV>), grid, dim3(256), 0, s, (const TX*)X, ldx, xm, eps, gamma, beta, stats, \
                     (TY*)Y, ldy, ym, M, C)
    if (v8 <= 1) SDP_LNF(1); else if (v8 <= 2) SDP_LNF(2); else SDP_LNF(4);
#undef SDP_LNF
    return SDP_CHECK_LAUNCH();
  });
}

// Residual add + LayerNorm forward in one pass (training forward, the branch add that feeds the
// next LayerNorm inside one sub-layer: ConvMixer's x_ = x + drop_path(act(PW(..))) -> LN2,
// EncoderLayer's x + drop_path(dropout(o_proj(..))) -> norm2; layers.py:99-103, :300-306):
//   y = rowscale(act / dropout(x)) * scale[m / sgrp] + r   (sdp_rowscale_add[_mixed / _dropout] mode 1)
//   a = LN(y) with its (mean, rstd) statistics            (sdp_ln_fwd[_mixed])
// One wave per row; y is rounded to its dtype before the statistics, so both outputs and the
// statistics are bit-identical to the two separate passes (which stored y and re-read it).  Saves
// the re-read of y and one launch per sub-layer.
template <typename TX, typename TY, typename TA, int V, int ACT>
__global__ __launch_bounds__(256) void add_ln_fwd_v8(const TX* __restrict__ X, int64_t ldx, RowMap xm,
                                                     const float* __restrict__ sc, int sgrp, const TY* __restrict__ R,
                                                     int64_t ldr, RowMap rm, TY* __restrict__ Y, int64_t ldy,
                                                     RowMap ym, int act, float p, uint64_t seed, int dmode, float eps,
                                                     const float* __restrict__ g, const float* __restrict__ b,
                                                     float* __restrict__ st, TA* __restrict__ A, int64_t lda,
                                                     RowMap am, int M, int C, RegCopy rc) {
  const int lane = threadIdx.x & 63;
  const int nbm = (M + 3) >> 2;
  if ((int)blockIdx.x >= nbm) {  // register-row copy blocks after the row blocks
    reg_copy_row(rc, ((int)blockIdx.x - nbm) * 4 + (threadIdx.x >> 6), lane);
    return;
  }
  const int64_t m = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= M) return;
  const float inv = p > 0.f ? 1.0f / (1.0f - p) : 1.0f;
  const uint32_t thr = drop_thresh(p);
  const float s_ = sc ? sc[m / sgrp] : 1.0f;
  const TX* xp = X + xm(m) * ldx;
  const TY* rp = R + rm(m) * ldr;
  TY* yp = Y + ym(m) * ldy;
  V8<TY> y[V];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const int c = 8 * lane + 512 * i;
    if (c < C) {
      V8<TX> x;
      x.load(xp + c);
      const int a = ACT >= 0 ? ACT : act;
      if (a != ACT_NONE) {  // rowscale_v8's arithmetic, step by step
#pragma unroll
        for (int q = 0; q < 8; ++q) x.v[q] = to_f<TX>(from_f<TX>(apply_act(a, x.v[q])));
      }
      if (dmode == 1) {
        const uint64_t base = (uint64_t)m * C + c;
        const uint32_t key = drop_key(seed, base);
#pragma unroll
        for (int q = 0; q < 8; ++q)
          x.v[q] = to_f<TX>(from_f<TX>(drop_keep(key, (uint32_t)base + q, thr) ? x.v[q] * inv : 0.f));
      }
      y[i].load(rp + c);
#pragma unroll
      for (int q = 0; q < 8; ++q) y[i].v[q] = fmaf(x.v[q], s_, y[i].v[q]);
      y[i].store(yp + c);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        y[i].v[q] = to_f<TY>(from_f<TY>(y[i].v[q]));  // the stored value, as ln_fwd_v8 would load it
        s += y[i].v[q];
      }
    }
  }
  // ln_fwd_v8's statistics and output, same summation order
  const float mean = wave_sum(s) / (float)C;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const int c = 8 * lane + 512 * i;
    if (c < C) {
#pragma unroll
      for (int q = 0; q < 8; ++q) ss = fmaf(y[i].v[q] - mean, y[i].v[q] - mean, ss);
    }
  }
  const float rstd = 1.0f / sqrtf(wave_sum(ss) / (float)C + eps);
  if (lane == 0) *(float2*)(st + 2 * m) = float2{mean, rstd};
  TA* ap = A + am(m) * lda;
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const int c = 8 * lane + 512 * i;
    if (c < C) {
      const f32x4 g0 = *(const f32x4*)(g + c), g1 = *(const f32x4*)(g + c + 4);
      const f32x4 b0 = *(const f32x4*)(b + c), b1 = *(const f32x4*)(b + c + 4);
      V8<TA> o;
#pragma unroll
      for (int q = 0; q < 8; ++q)
        o.v[q] = (y[i].v[q] - mean) * rstd * (q < 4 ? g0[q] : g1[q - 4]) + (q < 4 ? b0[q] : b1[q - 4]);
      o.store(ap + c);
    }
  }
}

// C ABI of add_ln_fwd_v8: x in x_dtype; r, y in y_dtype (the residual stream); a in a_dtype (the
// next GEMM's operand).  hipErrorNotSupported where the one-pass form does not apply (C % 8 != 0,
// C > 2048, rows not 16-B aligned, dmode 2): the caller then runs the two passes.
extern "C" int sdp_add_ln_fwd(int x_dtype, int y_dtype, int a_dtype, int act, const void* X, int64_t ldx, int x_grp,
                              int64_t x_gstride, int x_off, const float* scale, int sgrp, const void* R, int64_t ldr,
                              int r_grp, int64_t r_gstride, int r_off, void* Y, int64_t ldy, int y_grp,
                              int64_t y_gstride, int y_off, float p, uint64_t seed, int dmode, float eps,
                              const float* gamma, const float* beta, float* stats, void* A, int64_t lda, int a_grp,
                              int64_t a_gstride, int a_off, int M, int C, const void* reg_src, void* reg_dst0,
                              void* reg_dst1, int reg_b, int reg_r, int reg_n, void* stream) {
  if (!X || !R || !Y || !A || !stats || !gamma || !beta || M < 0 || C <= 0 || (scale && sgrp <= 0) || act < 0 ||
      act > ACT_KELU || p < 0.f || p >= 1.f || dmode < 0 || dmode > 2 ||
      (reg_src && (!reg_dst0 || reg_b < 0 || reg_r < 0)))
    return (int)hipErrorInvalidValue;
  const int yes = y_dtype == 1 ? 2 : 4;
  const RegCopy rc{reg_b * reg_r > 0 ? (const char*)reg_src : nullptr, (char*)reg_dst0, (char*)reg_dst1, ldy * yes,
                   reg_b, reg_r, reg_n, C * yes};
  if (!reg_copy_ok(rc)) return (int)hipErrorNotSupported;
  if (p == 0.f) dmode = 0;
  // (C <= 128: sdp_ln_fwd takes the several-rows-per-wave kernel, whose sums run in another order)
  if (dmode == 2 || C % 8 || C <= 128 || C > 2048 || ldx % 8 || ldr % 8 || ldy % 8 || lda % 8 || (uintptr_t)X % 16 ||
      (uintptr_t)R % 16 || (uintptr_t)Y % 16 || (uintptr_t)A % 16 || (uintptr_t)gamma % 16 || (uintptr_t)beta % 16 ||
      (uintptr_t)stats % 8)
    return (int)hipErrorNotSupported;
  if ((x_dtype != 0 && x_dtype != 1) || (y_dtype != 0 && y_dtype != 1) || (a_dtype != 0 && a_dtype != 1))
    return (int)hipErrorInvalidValue;
  if (M == 0) return 0;
  const RowMap xm = mk_tmap(x_grp, x_gstride, x_off), rm = mk_tmap(r_grp, r_gstride, r_off),
               ym = mk_tmap(y_grp, y_gstride, y_off), am = mk_tmap(a_grp, a_gstride, a_off);
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid((M + 3) / 4 + (rc.src ? (rc.B * rc.R + 3) / 4 : 0));
  const int v8 = (C + 511) / 512;
  auto launch = [&](auto tx, auto ty, auto ta) {
    using TX = typename decltype(tx)::type;
    using TY = typename decltype(ty)::type;
    using TA = typename decltype(ta)::type;
#define SDP_ALN(VV, AA)                                                                                           \
  hipLaunchKernelGGL((add_ln_fwd_v8<TX, TY, TA, VV, AA>), grid, dim3(256), 0, s, (const TX*)X, ldx, xm, scale, sgrp, \
                     (const TY*)R, ldr, rm, (TY*)Y, ldy, ym, act, p, seed, dmode, eps, gamma, beta, stats, (TA*)A,  \
                     lda, am, M, C, rc)
    if (act == ACT_GELU) {
      if (v8 <= 1) SDP_ALN(1, ACT_GELU); else if (v8 <= 2) SDP_ALN(2, ACT_GELU); else SDP_ALN(4, ACT_GELU);
    } else {
      if (v8 <= 1) SDP_ALN(1, -1); else if (v8 <= 2) SDP_ALN(2, -1); else SDP_ALN(4, -1);
    }
#undef SDP_ALN
    return SDP_CHECK_LAUNCH();
  };
  return by_dtypes(x_dtype, y_dtype, [&](auto tx, auto ty) {
    return a_dtype == 1 ? launch(tx, ty, DTag<bf16_t>{}) : launch(tx, ty, DTag<float>{});
  });
}

extern "C" int sdp_ln_fwd(int dtype, const void* X, int64_t ldx, int x_grp, int64_t x_gstride, int x_off, float eps,
                          const float* gamma, const float* beta, float* stats, void* Y, int64_t ldy, int y_grp,
                          int64_t y_gstride, int y_off, int M, int C, void* stream) {
  return ln_fwd_impl(dtype, dtype, X, ldx, x_grp, x_gstride, x_off, eps, gamma, beta, stats, Y, ldy, y_grp, y_gstride,
                     y_off, M, C, stream);
}

// X in x_dtype, Y in y_dtype (fp32 residual stream -> bf16 GEMM operand).
extern "C" int sdp_ln_fwd_mixed(int x_dtype, int y_dtype, const void* X, int64_t ldx, int x_grp, int64_t x_gstride,
                                int x_off, float eps, const float* gamma, const float* beta, float* stats, void* Y,
                                int64_t ldy, int y_grp, int64_t y_gstride, int y_off, int M, int C, void* stream) {
  return ln_fwd_impl(x_dtype, y_dtype, X, ldx, x_grp, x_gstride, x_off, eps, gamma, beta, stats, Y, ldy, y_grp,
                     y_gstride, y_off, M, C, stream);
}

extern "C" int sdp_ln_apply(int dtype, const void* X, int64_t ldx, int x_grp, int64_t x_gstride, int x_off,
                            const float* stats, const float* gamma, const float* beta, void* Y, int64_t ldy, int y_grp,
                            int64_t y_gstride, int y_off, int M, int C, void* stream) {
  if (!X || !Y || !stats || !gamma || !beta || M < 0 || C <= 0) return (int)hipErrorInvalidValue;
  if (M == 0) return 0;
  const RowMap xm = mk_tmap(x_grp, x_gstride, x_off), ym = mk_tmap(y_grp, y_gstride, y_off);
  hipStream_t s = (hipStream_t)stream;
  dim3 grid((M + 3) / 4);
  if (dtype == 1)
    hipLaunchKernelGGL(ln_apply_k<bf16_t>, grid, dim3(256), 0, s, (const bf16_t*)X, ldx, xm, stats, gamma, beta,
                       (bf16_t*)Y, ldy, ym, M, C);
  else if (dtype == 0)
    hipLaunchKernelGGL(ln_apply_k<float>, grid, dim3(256), 0, s, (const float*)X, ldx, xm, stats, gamma, beta,
                       (float*)Y, ldy, ym, M, C);
  else
    return (int)hipErrorInvalidValue;
  return SDP_CHECK_LAUNCH();
}

// Number of partial blocks sdp_ln_bwd uses for M rows (part needs nblk * 2 * C floats).
extern "C" int sdp_ln_bwd_blocks(int M) {
  int b = (M + 3) / 4;
  return b < 1024 ? (b > 0 ? b : 1) : 1024;
}

static int ln_bwd_impl(int xdt, int dydt, const void* X, int64_t ldx, int x_grp, int64_t x_gstride, int x_off,
                       const float* stats, const float* gamma, const void* DY, int64_t lddy, int dy_grp,
                       int64_t dy_gstride, int dy_off, const void* ADD, int64_t ldadd, int a_grp, int64_t a_gstride,
                       int a_off, void* DX, int64_t lddx, int dx_grp, int64_t dx_gstride, int dx_off, int M, int C,
                       float* part, void* stream, float* gpart = nullptr, float* aff = nullptr, int* ticket = nullptr,
                       const LnBwdEmit* em = nullptr, const RegCopy* rcp = nullptr) {
  if (!X || !stats || !gamma || !DY || !DX || M < 0 || C <= 0 || C > 2048) return (int)hipErrorInvalidValue;
  if (ticket && (!part || !gpart || !aff)) return (int)hipErrorInvalidValue;
  if (M == 0) return 0;
  const RowMap xm = mk_tmap(x_grp, x_gstride, x_off), dym = mk_tmap(dy_grp, dy_gstride, dy_off),
               am = mk_tmap(a_grp, a_gstride, a_off), dxm = mk_tmap(dx_grp, dx_gstride, dx_off);
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid(sdp_ln_bwd_blocks(M));
  const size_t lds = (size_t)8 * C * sizeof(float);
  const bool vec = C % 8 == 0 && ldx % 8 == 0 && lddy % 8 == 0 && lddx % 8 == 0 && (!ADD || ldadd % 8 == 0) &&
                   (uintptr_t)X % 16 == 0 && (uintptr_t)DY % 16 == 0 && (uintptr_t)DX % 16 == 0 &&
                   (!ADD || (uintptr_t)ADD % 16 == 0) && (uintptr_t)gamma % 16 == 0;
  // the one-launch forms (branch-gradient output, in-kernel affine sums) exist for ln_bwd_v8 only
  const bool fused = ticket || em || (rcp && rcp->src);
  if (fused) {
    if (rcp && !reg_copy_ok(*rcp)) return (int)hipErrorNotSupported;
    auto a16 = [](const void* q) { return (uintptr_t)q % 16 == 0; };
    if (!vec || C <= 128 || (C * 2) % 4 || (ticket && (!a16(part) || !a16(gpart) || !a16(aff))))
      return (int)hipErrorNotSupported;
    if (em && (!em->o2 || em->ldo2 % 8 || !a16(em->o2) || (em->sc && em->sgrp <= 0) || em->dmode < 0 ||
               em->dmode > 2 || em->dmode == 1 || em->p < 0.f || em->p >= 1.f || em->act < 0 || em->act > ACT_KELU ||
               (em->act != ACT_NONE && (!em->z || em->ldz % 8 || !a16(em->z)))))
      return (int)hipErrorNotSupported;
  }
  const LnBwdEmit e0{};
  const RegCopy r0{};
  if (vec) {
    return by_dtypes(xdt, dydt, [&](auto tx, auto td) {
      using TX = typename decltype(tx)::type;
      using TD = typename decltype(td)::type;
      if (C <= 128) {  // several rows per wave
#define SDP_LNVS(LL)                                                                                            \
  hipLaunchKernelGGL((ln_bwd_sm<TX, TD, LL>), grid, dim3(256), lds, s, (const TX*)X, ldx, xm, stats, gamma,        \
                     (const TD*)DY, lddy, dym, (const TX*)ADD, ldadd, am, (TX*)DX, lddx, dxm, M, C, part)
        if (C <= 64) SDP_LNVS(8); else SDP_LNVS(16);
#undef SDP_LNVS
        return SDP_CHECK_LAUNCH();
      }
      const int v8 = (C + 511) / 512;
#define SDP_LNV(VV, EMV)                                                                                          \
  hipLaunchKernelGGL((ln_bwd_v8<TX, TD, VV, EMV>), grid, dim3(256), lds, s, (const TX*)X, ldx, xm, stats, gamma,   \
                     (const TD*)DY, lddy, dym, (const TX*)ADD, ldadd, am, (TX*)DX, lddx, dxm, M, C, part, gpart, aff, \
                     ticket, em ? *em : e0, rcp ? *rcp : r0)
#define SDP_LNVA(EA_)                                                                              \
  if (v8 <= 1) SDP_LNV(1, EA_); else if (v8 <= 2) SDP_LNV(2, EA_); else SDP_LNV(4, EA_);
      if (!em) { SDP_LNVA(LNB_NOEMIT) }
      else if (em->act == ACT_GELU) { SDP_LNVA(ACT_GELU) }
      else if (em->act == ACT_NONE) { SDP_LNVA(ACT_NONE) }
      else { SDP_LNVA(-1) }
#undef SDP_LNVA
#undef SDP_LNV
      return SDP_CHECK_LAUNCH();
    });
  }
  if (xdt != dydt) return (int)hipErrorInvalidValue;  // mixed dtypes: vector path only
  const int v = (C + 63) / 64;
#define SDP_LNB(TT, VV)                                                                                          \
  hipLaunchKernelGGL((ln_bwd_k<TT, VV>), grid, dim3(256), lds, s, (const TT*)X, ldx, xm, stats, gamma, (const TT*)DY, \
                     lddy, dym, (const TT*)ADD, ldadd, am, (TT*)DX, lddx, dxm, M, C, part)
#define SDP_LNB_T(TT)                                 \
  if (v <= 2) SDP_LNB(TT, 2);                         \
  else if (v <= 4) SDP_LNB(TT, 4);                    \
  else if (v <= 8) SDP_LNB(TT, 8);                    \
  else if (v <= 12) SDP_LNB(TT, 12);                  \
  else if (v <= 16) SDP_LNB(TT, 16);                  \
  else SDP_LNB(TT, 32)
  if (xdt == 1) {
    SDP_LNB_T(bf16_t);
  } else if (xdt == 0) {
    SDP_LNB_T(float);
  } else {
    return (int)hipErrorInvalidValue;
  }
#undef SDP_LNB_T
#undef SDP_LNB
  return SDP_CHECK_LAUNCH();
}

extern "C" int sdp_ln_bwd(int dtype, const void* X, int64_t ldx, int x_grp, int64_t x_gstride, int x_off,
                          const float* stats, const float* gamma, const void* DY, int64_t lddy, int dy_grp,
                          int64_t dy_gstride, int dy_off, const void* ADD, int64_t ldadd, int a_grp, int64_t a_gstride,
                          int a_off, void* DX, int64_t lddx, int dx_grp, int64_t dx_gstride, int dx_off, int M, int C,
                          float* part, void* stream) {
  return ln_bwd_impl(dtype, dtype, X, ldx, x_grp, x_gstride, x_off, stats, gamma, DY, lddy, dy_grp, dy_gstride, dy_off,
                     ADD, ldadd, a_grp, a_gstride, a_off, DX, lddx, dx_grp, dx_gstride, dx_off, M, C, part, stream);
}

// sdp_ln_bwd_mixed in one launch with (a) the affine sums finished in the kernel: part
// [sdp_ln_bwd_blocks(M)][2C] and gpart [ceil(blocks / 32)][2C] scratch, aff [2C] = {dgamma, dbeta},
// ticket[ceil(blocks / 32) + 1] zeroed ints (left zeroed), or ticket = nullptr for part only; and
// (b) optionally (O2 != nullptr) the branch gradient O2 (bf16, LnBwdEmit): bf16(DX * scale[m / sgrp]),
// dmode 2 dropout (p, seed, index m * C + c), times act'(Z) (act != 0; Z bf16).  hipErrorNotSupported
// where the one-launch form does not apply (C <= 128, C % 8, misaligned rows, dmode 1).
extern "C" int sdp_ln_bwd_fused(int x_dtype, int dy_dtype, const void* X, int64_t ldx, int x_grp, int64_t x_gstride,
                                int x_off, const float* stats, const float* gamma, const void* DY, int64_t lddy,
                                int dy_grp, int64_t dy_gstride, int dy_off, const void* ADD, int64_t ldadd, int a_grp,
                                int64_t a_gstride, int a_off, void* DX, int64_t lddx, int dx_grp, int64_t dx_gstride,
                                int dx_off, int M, int C, float* part, float* gpart, float* aff, int* ticket,
                                const float* scale, int sgrp, const void* Z, int64_t ldz, int act, float p,
                                uint64_t seed, int dmode, void* O2, int64_t ldo2, const void* reg_src, void* reg_dst,
                                int reg_b, int reg_r, int reg_n, void* stream) {
  const LnBwdEmit em{scale, sgrp, (const bf16_t*)Z, ldz, act, p, seed, dmode, (bf16_t*)O2, ldo2};
  const int es = x_dtype == 1 ? 2 : 4;
  const RegCopy rc{(const char*)reg_src, (char*)reg_dst, nullptr, lddx * es, reg_b, reg_r, reg_n, C * es};
  if (reg_src && (!reg_dst || reg_b < 0 || reg_r < 0)) return (int)hipErrorInvalidValue;
  return ln_bwd_impl(x_dtype, dy_dtype, X, ldx, x_grp, x_gstride, x_off, stats, gamma, DY, lddy, dy_grp, dy_gstride,
                     dy_off, ADD, ldadd, a_grp, a_gstride, a_off, DX, lddx, dx_grp, dx_gstride, dx_off, M, C, part,
                     stream, gpart, aff, ticket, O2 ? &em : nullptr, reg_src && reg_b * reg_r > 0 ? &rc : nullptr);
}

// X, ADD and DX in x_dtype (the residual stream and its gradient), DY in dy_dtype (the
// gradient of the LN output coming back from a bf16 GEMM operand).
extern "C" int sdp_ln_bwd_mixed(int x_dtype, int dy_dtype, const void* X, int64_t ldx, int x_grp, int64_t x_gstride,
                                int x_off, const float* stats, const float* gamma, const void* DY, int64_t lddy,
                                int dy_grp, int64_t dy_gstride, int dy_off, const void* ADD, int64_t ldadd, int a_grp,
                                int64_t a_gstride, int a_off, void* DX, int64_t lddx, int dx_grp, int64_t dx_gstride,
                                int dx_off, int M, int C, float* part, void* stream) {
  return ln_bwd_impl(x_dtype, dy_dtype, X, ldx, x_grp, x_gstride, x_off, stats, gamma, DY, lddy, dy_grp, dy_gstride,
                     dy_off, ADD, ldadd, a_grp, a_gstride, a_off, DX, lddx, dx_grp, dx_gstride, dx_off, M, C, part,
                     stream);
}

// ---------------------------------------------------------------------------
// Attention rows: P = softmax(scale * S) over the first N of each row (row stride ld),
// Pd = P with dropout (keep ? P / (1 - p) : 0), columns [N, ld) of P and Pd are zeroed
// (they feed the PV product as K padding).  Backward: dS = P * (dPm - sum(dPm * P)),
// dPm = dPd with the same dropout mask.  One wave per row; S fp32.
// ---------------------------------------------------------------------------
// Optional additive fp32 attention mask of the materialised softmax (the masked manual /
// SDPA attention of EncoderLayer, layers.py:289-298): row r = z * N + i of S (z = b * zdiv + h)
// adds mask[(z / zdiv) * sb + (z % zdiv) * sh + i * N + c] (batch / head strides 0 = broadcast)
// before the max; -inf entries give exact zeros.
struct SmMask {
  const float* m;
  int64_t sb, sh;
  int zdiv;
  SDP_DEV const float* row(int64_t r, int N) const {
    if (!m) return nullptr;
    const int64_t z = r / N, i = r - z * N;
    return m + (z / zdiv) * sb + (z % zdiv) * sh + i * N;
  }
};

template <typename T>
__global__ __launch_bounds__(256) void softmax_fwd_k(const float* __restrict__ S, int64_t lds, T* __restrict__ P,
                                                     T* __restrict__ Pd, int64_t ldp, int rows, int N, int Npad,
                                                     float scale, float p, uint64_t seed, SmMask mk) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const float* sp_ = S + r * lds;
  const float* mp = mk.row(r, N);
  auto val = [&](int c) { return mp ? fmaf(sp_[c], scale, mp[c]) : sp_[c] * scale; };
  float mx = -INFINITY;
  for (int c = lane; c < N; c += 64) mx = fmaxf(mx, val(c));
  mx = wave_max(mx);
  float sum = 0.f;
  for (int c = lane; c < N; c += 64) sum += expf(val(c) - mx);
  sum = wave_sum(sum);
  const float inv = 1.0f / sum, kp = p > 0.f ? 1.0f / (1.0f - p) : 1.0f;
  for (int c = lane; c < Npad; c += 64) {
    float v = c < N ? expf(val(c) - mx) * inv : 0.f;
    P[r * ldp + c] = from_f<T>(v);
    if (Pd) {
      float d = v;
      if (p > 0.f && c < N) d = uniform01(seed, (uint64_t)r * N + c) >= p ? v * kp : 0.f;
      Pd[r * ldp + c] = from_f<T>(d);
    }
  }
}

template <typename T>
__global__ __launch_bounds__(256) void softmax_bwd_k(const T* __restrict__ P, int64_t ldp, const T* __restrict__ DPd,
                                                     int64_t lddp, T* __restrict__ DS, int64_t ldds, int rows, int N,
                                                     int Npad, float p, uint64_t seed) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const float kp = p > 0.f ? 1.0f / (1.0f - p) : 1.0f;
  auto dpm = [&](int c) {
    float g = to_f<T>(DPd[r * lddp + c]);
    if (p > 0.f) g = uniform01(seed, (uint64_t)r * N + c) >= p ? g * kp : 0.f;
    return g;
  };
  float dot = 0.f;
  for (int c = lane; c < N; c += 64) dot += dpm(c) * to_f<T>(P[r * ldp + c]);
  dot = wave_sum(dot);
  for (int c = lane; c < Npad; c += 64) {
    const float v = c < N ? to_f<T>(P[r * ldp + c]) * (dpm(c) - dot) : 0.f;
    DS[r * ldds + c] = from_f<T>(v);
  }
}

// Register-resident rows (Npad <= 512, Npad % 4 == 0): lane holds 4-column chunks lane and
// lane + 64; one read of S, one write of P / Pd.
template <typename T>
SDP_DEV void store4(T* p, const float (&v)[4]) {
  if constexpr (sizeof(T) == 2) {
    bf16x4 t;
#pragma unroll
    for (int q = 0; q < 4; ++q) t[q] = (short)f2bf(v[q]);
    *(bf16x4*)p = t;
  } else {
    *(f32x4*)p = f32x4{v[0], v[1], v[2], v[3]};
  }
}
template <typename T>
SDP_DEV void load4(const T* p, float (&v)[4]) {
  if constexpr (sizeof(T) == 2) {
    const bf16x4 t = *(const bf16x4*)p;
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = bf2f((bf16_t)t[q]);
  } else {
    const f32x4 t = *(const f32x4*)p;
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = t[q];
  }
}

template <typename T>
__global__ __launch_bounds__(256) void softmax_fwd_r(const float* __restrict__ S, int64_t lds, T* __restrict__ P,
                                                     T* __restrict__ Pd, int64_t ldp, int rows, int N, int Npad,
                                                     float scale, float p, uint64_t seed, SmMask mk) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const float* sp_ = S + r * lds;
  const float* mp = mk.row(r, N);
  float v[2][4];
  float mx = -INFINITY;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = 4 * (lane + 64 * i);
    if (c < Npad) {
      const f32x4 t = *(const f32x4*)(sp_ + c);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        v[i][q] = c + q < N ? (mp ? fmaf(t[q], scale, mp[c + q]) : t[q] * scale) : -INFINITY;
        mx = fmaxf(mx, v[i][q]);
      }
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) v[i][q] = -INFINITY;
    }
  }
  mx = wave_max(mx);
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      v[i][q] = v[i][q] == -INFINITY ? 0.f : expf(v[i][q] - mx);
      sum += v[i][q];
    }
  const float inv = 1.0f / wave_sum(sum), kp = p > 0.f ? 1.0f / (1.0f - p) : 1.0f;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = 4 * (lane + 64 * i);
    if (c < Npad) {
      float o[4], d[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        o[q] = v[i][q] * inv;
        d[q] = o[q];
        if (p > 0.f && c + q < N) d[q] = uniform01(seed, (uint64_t)r * N + c + q) >= p ? o[q] * kp : 0.f;
      }
      store4<T>(P + r * ldp + c, o);
      if (Pd) store4<T>(Pd + r * ldp + c, d);
    }
  }
}

template <typename T>
__global__ __launch_bounds__(256) void softmax_bwd_r(const T* __restrict__ P, int64_t ldp, const T* __restrict__ DPd,
                                                     int64_t lddp, T* __restrict__ DS, int64_t ldds, int rows, int N,
                                                     int Npad, float p, uint64_t seed) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const float kp = p > 0.f ? 1.0f / (1.0f - p) : 1.0f;
  float pv[2][4], g[2][4];
  float dot = 0.f;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = 4 * (lane + 64 * i);
#pragma unroll
    for (int q = 0; q < 4; ++q) pv[i][q] = g[i][q] = 0.f;
    if (c < Npad) {
      load4<T>(P + r * ldp + c, pv[i]);
      load4<T>(DPd + r * lddp + c, g[i]);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (c + q >= N) { g[i][q] = 0.f; pv[i][q] = 0.f; }
        else if (p > 0.f) g[i][q] = uniform01(seed, (uint64_t)r * N + c + q) >= p ? g[i][q] * kp : 0.f;
        dot = fmaf(g[i][q], pv[i][q], dot);
      }
    }
  }
  dot = wave_sum(dot);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = 4 * (lane + 64 * i);
    if (c < Npad) {
      float o[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) o[q] = pv[i][q] * (g[i][q] - dot);
      store4<T>(DS + r * ldds + c, o);
    }
  }
}

extern "C" int sdp_softmax_fwd_mask(int dtype, const float* S, int64_t lds, void* P, void* Pd, int64_t ldp, int rows,
                                    int N, int Npad, float scale, float p, uint64_t seed, const float* mask,
                                    int64_t mask_sb, int64_t mask_sh, int mask_zdiv, void* stream);

extern "C" int sdp_softmax_fwd(int dtype, const float* S, int64_t lds, void* P, void* Pd, int64_t ldp, int rows, int N,
                               int Npad, float scale, float p, uint64_t seed, void* stream) {
  return sdp_softmax_fwd_mask(dtype, S, lds, P, Pd, ldp, rows, N, Npad, scale, p, seed, nullptr, 0, 0, 1, stream);
}

extern "C" int sdp_softmax_fwd_mask(int dtype, const float* S, int64_t lds, void* P, void* Pd, int64_t ldp, int rows,
                                    int N, int Npad, float scale, float p, uint64_t seed, const float* mask,
                                    int64_t mask_sb, int64_t mask_sh, int mask_zdiv, void* stream) {
  if (!S || !P || rows < 0 || N <= 0 || Npad < N || p < 0.f || p >= 1.f || mask_zdiv <= 0 || mask_sb < 0 ||
      mask_sh < 0)
    return (int)hipErrorInvalidValue;
  if (rows == 0) return 0;
  const SmMask mk{mask, mask_sb, mask_sh, mask_zdiv};
  hipStream_t s = (hipStream_t)stream;
  dim3 grid((rows + 3) / 4);
  if (Npad <= 512 && Npad % 4 == 0 && lds % 4 == 0 && ldp % 4 == 0 && (uintptr_t)S % 16 == 0 && (uintptr_t)P % 16 == 0 &&
      (!Pd || (uintptr_t)Pd % 16 == 0)) {
    if (dtype == 1)
      hipLaunchKernelGGL(softmax_fwd_r<bf16_t>, grid, dim3(256), 0, s, S, lds, (bf16_t*)P, (bf16_t*)Pd, ldp, rows, N,
                         Npad, scale, p, seed, mk);
    else if (dtype == 0)
      hipLaunchKernelGGL(softmax_fwd_r<float>, grid, dim3(256), 0, s, S, lds, (float*)P, (float*)Pd, ldp, rows, N,
                         Npad, scale, p, seed, mk);
    else
      return (int)hipErrorInvalidValue;
    return SDP_CHECK_LAUNCH();
  }
  if (dtype == 1)
    hipLaunchKernelGGL(softmax_fwd_k<bf16_t>, grid, dim3(256), 0, s, S, lds, (bf16_t*)P, (bf16_t*)Pd, ldp, rows, N,
                       Npad, scale, p, seed, mk);
  else if (dtype == 0)
    hipLaunchKernelGGL(softmax_fwd_k<float>, grid, dim3(256), 0, s, S, lds, (float*)P, (float*)Pd, ldp, rows, N, Npad,
                       scale, p, seed, mk);
  else
    return (int)hipErrorInvalidValue;
  return SDP_CHECK_LAUNCH();
}

extern "C" int sdp_softmax_bwd(int dtype, const void* P, int64_t ldp, const void* DPd, int64_t lddp, void* DS,
                               int64_t ldds, int rows, int N, int Npad, float p, uint64_t seed, void* stream) {
  if (!P || !DPd || !DS || rows < 0 || N <= 0 || Npad < N || p < 0.f || p >= 1.f) return (int)hipErrorInvalidValue;
  if (rows == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  dim3 grid((rows + 3) / 4);
  if (Npad <= 512 && Npad % 4 == 0 && ldp % 4 == 0 && lddp % 4 == 0 && ldds % 4 == 0 && (uintptr_t)P % 16 == 0 &&
      (uintptr_t)DPd % 16 == 0 && (uintptr_t)DS % 16 == 0) {
    if (dtype == 1)
      hipLaunchKernelGGL(softmax_bwd_r<bf16_t>, grid, dim3(256), 0, s, (const bf16_t*)P, ldp, (const bf16_t*)DPd, lddp,
                         (bf16_t*)DS, ldds, rows, N, Npad, p, seed);
    else if (dtype == 0)
      hipLaunchKernelGGL(softmax_bwd_r<float>, grid, dim3(256), 0, s, (const float*)P, ldp, (const float*)DPd, lddp,
                         (float*)DS, ldds, rows, N, Npad, p, seed);
    else
      return (int)hipErrorInvalidValue;
    return SDP_CHECK_LAUNCH();
  }
  if (dtype == 1)
    hipLaunchKernelGGL(softmax_bwd_k<bf16_t>, grid, dim3(256), 0, s, (const bf16_t*)P, ldp, (const bf16_t*)DPd, lddp,
                       (bf16_t*)DS, ldds, rows, N, Npad, p, seed);
  else if (dtype == 0)
    hipLaunchKernelGGL(softmax_bwd_k<float>, grid, dim3(256), 0, s, (const float*)P, ldp, (const float*)DPd, lddp,
                       (float*)DS, ldds, rows, N, Npad, p, seed);
  else
    return (int)hipErrorInvalidValue;
  return SDP_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------
// Depthwise-conv weight gradient (layers.py:73-78 backward):
//   part[chunk][c][t] = sum over the chunk's images and pixels of DY[b,h,w,c] * A[b,h+ty-P,w+tx-P,c]
// (zero padding), NHWC rows through row maps.  Block: 32 channels x (image chunk); both planes of
// one image staged in LDS as fp32 [pixel][32] (converted once at staging: every staged value is
// read by KS threads).  Reduce the chunk slabs with sdp_seg_colsum.
// ---------------------------------------------------------------------------
// Thread (channel pair cp = lane % 16, tap row ty = wave, output rows h = lane / 16 mod 4): for
// each of its rows (in 16-column segments) it loads the 16-wide DY row and the (16 + KS - 1)-wide
// zero-padded A row hh = h + ty - KS/2 of both channels into registers once (one 64-bit LDS read
// per pixel) and does the KS x 16 two-channel FMAs (v_pk_fma_f32) of that row pair from
// registers; the four row groups' sums are added at the end (lane ^ 16, lane ^ 32).  The planes
// take 2 x HW x 128 B = 64 KiB at 16 x 16, so two workgroups share a CU and one stages while the
// other computes; all of a thread's staging loads of an image are issued before its LDS stores.
template <typename T, int KS>
__global__ __launch_bounds__(64 * KS) void dw_wgrad_k(const T* __restrict__ A, int64_t lda, RowMap am,
                                                      const T* __restrict__ DY, int64_t lddy, RowMap dym, int B, int H,
                                                      int W, int C, int ipb, float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) char dw_sm[];
  constexpr int P = KS / 2, MW = 16, NT = 64 * KS, U = 4, CB = 32, NCP = CB / 2, NRG = 64 / NCP, CH = CB / 8;
  const int HW = H * W;
  float* ap = (float*)dw_sm;  // [HW][32]
  float* dp = ap + HW * CB;   // [HW][32]
  const int c0 = blockIdx.x * CB, chunk = blockIdx.y;
  const int cp = threadIdx.x % NCP, rg = (threadIdx.x & 63) / NCP, ty = threadIdx.x / 64;
  f32x2 acc[KS];
#pragma unroll
  for (int i = 0; i < KS; ++i) acc[i] = f32x2{0.f, 0.f};
  const int b0 = chunk * ipb, b1 = min(B, b0 + ipb);
  const bool v8 = (sizeof(T) == 2) && (c0 + CB <= C) && (lda % 8 == 0) && (lddy % 8 == 0) &&
                  (((uintptr_t)A & 15) == 0) && (((uintptr_t)DY & 15) == 0);
  for (int b = b0; b < b1; ++b) {
    __syncthreads();
    if (v8) {  // 16-B loads: CH chunks of 8 channels per pixel, U chunk pairs in flight per thread
      const int n = HW * CH;
      for (int e0 = threadIdx.x; e0 < n; e0 += NT * U) {
        bf16x8 va[U], vd[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int e = min(e0 + u * NT, n - 1);
          const int64_t m = (int64_t)b * HW + e / CH;
          va[u] = *(const bf16x8*)(A + am(m) * lda + c0 + (e % CH) * 8);
          vd[u] = *(const bf16x8*)(DY + dym(m) * lddy + c0 + (e % CH) * 8);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int e = e0 + u * NT;
          if (e < n) {
            f32x4* pa = (f32x4*)(ap + (e / CH) * CB + (e % CH) * 8);
            f32x4* pd = (f32x4*)(dp + (e / CH) * CB + (e % CH) * 8);
            pa[0] = f32x4{bf2f((bf16_t)va[u][0]), bf2f((bf16_t)va[u][1]), bf2f((bf16_t)va[u][2]), bf2f((bf16_t)va[u][3])};
            pa[1] = f32x4{bf2f((bf16_t)va[u][4]), bf2f((bf16_t)va[u][5]), bf2f((bf16_t)va[u][6]), bf2f((bf16_t)va[u][7])};
            pd[0] = f32x4{bf2f((bf16_t)vd[u][0]), bf2f((bf16_t)vd[u][1]), bf2f((bf16_t)vd[u][2]), bf2f((bf16_t)vd[u][3])};
            pd[1] = f32x4{bf2f((bf16_t)vd[u][4]), bf2f((bf16_t)vd[u][5]), bf2f((bf16_t)vd[u][6]), bf2f((bf16_t)vd[u][7])};
          }
        }
      }
    } else {
      for (int e = threadIdx.x; e < HW * CB; e += NT) {
        const int px = e / CB, c = c0 + (e % CB);
        const int64_t m = (int64_t)b * HW + px;
        ap[e] = c < C ? to_f<T>(A[am(m) * lda + c]) : 0.f;
        dp[e] = c < C ? to_f<T>(DY[dym(m) * lddy + c]) : 0.f;
      }
    }
    __syncthreads();
    for (int h = rg; h < H; h += NRG) {
      const int hh = h + ty - P;
      if (hh < 0 || hh >= H) continue;
      for (int w0 = 0; w0 < W; w0 += MW) {
        f32x2 ar[MW + KS - 1], dr[MW];
#pragma unroll
        for (int q = 0; q < MW + KS - 1; ++q) {
          const int ww = w0 + q - P;
          ar[q] = (ww >= 0 && ww < W) ? *(const f32x2*)(ap + (hh * W + ww) * CB + 2 * cp) : f32x2{0.f, 0.f};
        }
#pragma unroll
        for (int q = 0; q < MW; ++q)
          dr[q] = w0 + q < W ? *(const f32x2*)(dp + (h * W + w0 + q) * CB + 2 * cp) : f32x2{0.f, 0.f};
#pragma unroll
        for (int q = 0; q < MW; ++q)
#pragma unroll
          for (int tx = 0; tx < KS; ++tx) acc[tx] = __builtin_elementwise_fma(dr[q], ar[q + tx], acc[tx]);
      }
    }
  }
#pragma unroll
  for (int tx = 0; tx < KS; ++tx) {
#pragma unroll
    for (int sh = NCP; sh < 64; sh *= 2) {
      acc[tx].x += __shfl_xor(acc[tx].x, sh);
      acc[tx].y += __shfl_xor(acc[tx].y, sh);
    }
  }
  const int c = c0 + 2 * cp;
  if (rg || c >= C) return;
  float* o = part + ((int64_t)chunk * C + c) * (KS * KS) + ty * KS;
#pragma unroll
  for (int tx = 0; tx < KS; ++tx) o[tx] = acc[tx].x;
  if (c + 1 >= C) return;
#pragma unroll
  for (int tx = 0; tx < KS; ++tx) o[KS * KS + tx] = acc[tx].y;
}

extern "C" int sdp_dw_wgrad_chunks(int B) { return B < 64 ? (B > 0 ? B : 1) : 64; }

extern "C" int sdp_dw_wgrad(int dtype, const void* A, int64_t lda, int a_grp, int64_t a_gstride, int a_off,
                            const void* DY, int64_t lddy, int dy_grp, int64_t dy_gstride, int dy_off, int B, int H,
                            int W, int C, int k, float* part, void* stream) {
  if (!A || !DY || !part || B < 0 || H <= 0 || W <= 0 || C <= 0 || (k != 3 && k != 5 && k != 7 && k != 9))
    return (int)hipErrorInvalidValue;
  if (B == 0) return 0;
  const size_t lds = (size_t)H * W * 32 * 2 * 4;  // both planes, fp32 [HW][32]
  if (lds > 160 * 1024) return (int)hipErrorInvalidValue;
  if ((a_grp > 0 && a_grp % (H * W)) || (dy_grp > 0 && dy_grp % (H * W))) return (int)hipErrorInvalidValue;
  const RowMap am = mk_tmap(a_grp, a_gstride, a_off), dym = mk_tmap(dy_grp, dy_gstride, dy_off);
  const int nch = sdp_dw_wgrad_chunks(B), ipb = (B + nch - 1) / nch;
  dim3 grid((C + 31) / 32, nch);
  hipStream_t s = (hipStream_t)stream;
#define SDP_DWG(TT, KK)                                                                                              \
  do {                                                                                                               \
    (void)hipFuncSetAttribute((const void*)dw_wgrad_k<TT, KK>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds); \
    hipLaunchKernelGGL((dw_wgrad_k<TT, KK>), grid, dim3(64 * KK), lds, s, (const TT*)A, lda, am, (const TT*)DY, lddy, \
                       dym, B, H, W, C, ipb, part);                                                                  \
  } while (0)
#define SDP_DWG_T(TT)                  \
  switch (k) {                         \
    case 3: SDP_DWG(TT, 3); break;     \
    case 5: SDP_DWG(TT, 5); break;     \
    case 7: SDP_DWG(TT, 7); break;     \
    default: SDP_DWG(TT, 9); break;    \
  }
  if (dtype == 1) {
    SDP_DWG_T(bf16_t)
  } else if (dtype == 0) {
    SDP_DWG_T(float)
  } else {
    return (int)hipErrorInvalidValue;
  }
#undef SDP_DWG_T
#undef SDP_DWG
  return SDP_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------
// Label-smoothed cross entropy (nn.CrossEntropyLoss(label_smoothing=eps), mean over rows):
//   hard labels:  loss_i = -(1 - eps) log p_{y_i} - eps / K * sum_k log p_k
//                 dlogits_i = grad_scale / B * (softmax_i - ((1 - eps) onehot(y_i) + eps / K))
//   soft targets (probability rows t_i, the CutMix / MixUp targets of dataset_generator.py:105-110):
//                 t'_i = (1 - eps) t_i + eps / K,  loss_i = -sum_k t'_ik log p_ik,
//                 dlogits_i = grad_scale / B * (softmax_i * sum_k t'_ik - t'_i)
// loss_sum += sum_i loss_i / n (atomic, fp32), n = B for soft targets and the number of rows
// whose label is not ignore_index for hard labels (nn.CrossEntropyLoss's default
// ignore_index = -100, reduction 'mean': an ignored row adds nothing to the loss and gets a zero
// gradient row; every row ignored gives a NaN loss, as torch's 0 / 0).  One wave per row; the
// row count comes from sdp_ce_count (one pass over the labels, sdp_ce_loss_counted) or, in the
// older entry points, every wave counts the labels itself (B reads per row: fine at
// classification batch sizes, quadratic per token).  Any other hard label outside [0, K) is
// never dereferenced: the row's loss and gradient become NaN, so the bad batch shows in the loss
// instead of reading out of bounds (torch raises there).
// ---------------------------------------------------------------------------
template <typename T, bool SOFT>
__global__ __launch_bounds__(256) void ce_k(const T* __restrict__ L, int64_t ldl, const int64_t* __restrict__ y,
                                            const float* __restrict__ tg, int64_t ldt, int B, int K, float eps,
                                            float grad_scale, T* __restrict__ D, int64_t ldd,
                                            float* __restrict__ loss, int64_t ignore,
                                            const float* __restrict__ counted) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= B) return;
  float nrows = (float)B;
  if constexpr (!SOFT) {
    if (counted) {  // sdp_ce_count ran first (O(B) in all)
      nrows = *counted;
    } else {        // legacy entry points: every wave counts (B reads per row)
      float cnt = 0.f;
      for (int i = lane; i < B; i += 64) cnt += (y[i] != ignore) ? 1.f : 0.f;
      nrows = wave_sum(cnt);
    }
    if (y[r] == ignore) {  // no loss, zero gradient row
      if (r == 0 && lane == 0 && nrows == 0.f) atomicAdd(loss, NAN);
      if (D)
        for (int c = lane; c < K; c += 64) D[r * ldd + c] = from_f<T>(0.f);
      return;
    }
  }
  const T* lp = L + r * ldl;
  float mx = -INFINITY, sl = 0.f;
  for (int c = lane; c < K; c += 64) {
    const float v = to_f<T>(lp[c]);
    mx = fmaxf(mx, v);
    sl += v;
  }
  mx = wave_max(mx);
  sl = wave_sum(sl);
  float se = 0.f;
  for (int c = lane; c < K; c += 64) se += expf(to_f<T>(lp[c]) - mx);
  se = wave_sum(se);
  const float lse = mx + logf(se);
  int64_t lab = 0;
  float li, tsum = 1.0f;
  if constexpr (SOFT) {
    // -sum t'_k (l_k - lse) = lse * sum t' - sum t' l
    const float* tp = tg + r * ldt;
    float st = 0.f, stl = 0.f;
    for (int c = lane; c < K; c += 64) {
      const float t = fmaf(1.0f - eps, tp[c], eps / (float)K);
      st += t;
      stl = fmaf(t, to_f<T>(lp[c]), stl);
    }
    st = wave_sum(st);
    stl = wave_sum(stl);
    tsum = st;
    li = lse * st - stl;
  } else {
    lab = y[r];
    const bool ok = lab >= 0 && lab < K;
    const float ly = ok ? to_f<T>(lp[lab]) : NAN;
    li = (1.0f - eps) * (lse - ly) + eps * (lse - sl / (float)K);
  }
  if (lane == 0) atomicAdd(loss, li / nrows);
  if (!D) return;
  const float sc = grad_scale / nrows, inv = 1.0f / se;
  const float bad = (!SOFT && !(lab >= 0 && lab < K)) ? NAN : 0.0f;
  for (int c = lane; c < K; c += 64) {
    const float pr = expf(to_f<T>(lp[c]) - mx) * inv;
    float tgt;
    if constexpr (SOFT) tgt = fmaf(1.0f - eps, tg[r * ldt + c], eps / (float)K);
    else tgt = (c == lab ? (1.0f - eps) : 0.0f) + eps / (float)K;
    D[r * ldd + c] = from_f<T>(sc * (pr * tsum - tgt) + bad);
  }
}

template <bool SOFT>
static int ce_launch(int dtype, const void* logits, int64_t ldl, const int64_t* labels, const float* targets,
                     int64_t ldt, int B, int K, float eps, float grad_scale, void* dlogits, int64_t ldd, float* loss,
                     void* stream, int64_t ignore = -100, const float* counted = nullptr) {
  if (!logits || !loss || B < 0 || K <= 0) return (int)hipErrorInvalidValue;
  if (SOFT ? !targets : !labels) return (int)hipErrorInvalidValue;
  if (B == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  dim3 grid((B + 3) / 4);
  if (dtype == 1)
    hipLaunchKernelGGL((ce_k<bf16_t, SOFT>), grid, dim3(256), 0, s, (const bf16_t*)logits, ldl, labels, targets, ldt,
                       B, K, eps, grad_scale, (bf16_t*)dlogits, ldd, loss, ignore, counted);
  else if (dtype == 0)
    hipLaunchKernelGGL((ce_k<float, SOFT>), grid, dim3(256), 0, s, (const float*)logits, ldl, labels, targets, ldt, B,
                       K, eps, grad_scale, (float*)dlogits, ldd, loss, ignore, counted);
  else
    return (int)hipErrorInvalidValue;
  return SDP_CHECK_LAUNCH();
}

extern "C" int sdp_ce_loss(int dtype, const void* logits, int64_t ldl, const int64_t* labels, int B, int K, float eps,
                           float grad_scale, void* dlogits, int64_t ldd, float* loss, void* stream) {
  return ce_launch<false>(dtype, logits, ldl, labels, nullptr, 0, B, K, eps, grad_scale, dlogits, ldd, loss, stream);
}

extern "C" int sdp_ce_loss_ignore(int dtype, const void* logits, int64_t ldl, const int64_t* labels, int B, int K,
                                  float eps, float grad_scale, int64_t ignore_index, void* dlogits, int64_t ldd,
                                  float* loss, void* stream) {
  return ce_launch<false>(dtype, logits, ldl, labels, nullptr, 0, B, K, eps, grad_scale, dlogits, ldd, loss, stream,
                          ignore_index);
}

// n[0] = number of labels != ignore_index, one workgroup sweeping the labels once.  Counted in
// integers (exact for every B < 2^31, as torch's count) and converted to float once at the end.
__global__ __launch_bounds__(1024) void ce_count_k(const int64_t* __restrict__ y, int B, int64_t ignore,
                                                   float* __restrict__ n) {
  __shared__ unsigned ws[16];
  unsigned c = 0;
  for (int i = threadIdx.x; i < B; i += 1024) c += (y[i] != ignore) ? 1u : 0u;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += (unsigned)__shfl_xor((int)c, o, 64);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned t = 0;
    for (int w = 0; w < 16; ++w) t += ws[w];
    n[0] = (float)t;
  }
}

extern "C" int sdp_ce_count(const int64_t* labels, int B, int64_t ignore_index, float* n, void* stream) {
  if (!labels || !n || B < 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(ce_count_k, dim3(1), dim3(1024), 0, (hipStream_t)stream, labels, B, ignore_index, n);
  return SDP_CHECK_LAUNCH();
}

extern "C" int sdp_ce_loss_counted(int dtype, const void* logits, int64_t ldl, const int64_t* labels, int B, int K,
                                   float eps, float grad_scale, int64_t ignore_index, const float* nrows,
                                   void* dlogits, int64_t ldd, float* loss, void* stream) {
  if (!nrows) return (int)hipErrorInvalidValue;
  return ce_launch<false>(dtype, logits, ldl, labels, nullptr, 0, B, K, eps, grad_scale, dlogits, ldd, loss, stream,
                          ignore_index, nrows);
}

extern "C" int sdp_ce_loss_soft(int dtype, const void* logits, int64_t ldl, const float* targets, int64_t ldt, int B,
                                int K, float eps, float grad_scale, void* dlogits, int64_t ldd, float* loss,
                                void* stream) {
  return ce_launch<true>(dtype, logits, ldl, nullptr, targets, ldt, B, K, eps, grad_scale, dlogits, ldd, loss, stream);
}

// ---------------------------------------------------------------------------
// Multi-tensor gradient norm and AdamW.  Tensors are fp32; the work list is a table of
// (tensor, first element) per 4096-element block built once by the host.
//   sdp_grad_sumsq: state[0] += sum g^2 over every tensor, state[1] = 1 if any g is non-finite
//   sdp_adamw: if state[1] == 0:  g = grad * inv_scale * clip, clip = min(1, max_norm /
//     (sqrt(state[0]) * inv_scale + 1e-6)) (clip_grad_norm_ on the unscaled grads,
//     training_tools.py:95-97);  p *= 1 - lr * wd;  m = b1 m + (1 - b1) g;
//     v = b2 v + (1 - b2) g^2;  p -= lr / bc1 * m / (sqrt(v / bc2) + eps)   (torch AdamW)
// ---------------------------------------------------------------------------
struct MTBlock {
  int tensor;
  int64_t start;
};

__global__ __launch_bounds__(256) void sumsq_k(float* const* __restrict__ grads, const int64_t* __restrict__ sizes,
                                               const MTBlock* __restrict__ blocks, float* __restrict__ state) {
  const MTBlock bl = blocks[blockIdx.x];
  const float* g = grads[bl.tensor];
  const int64_t n = sizes[bl.tensor];
  float s = 0.f;
  int bad = 0;
  for (int64_t i = bl.start + threadIdx.x; i < min(n, bl.start + 4096); i += 256) {
    const float v = g[i];
    s = fmaf(v, v, s);
    bad |= !isfinite(v);
  }
  __shared__ float red[4];
  __shared__ int rb[4];
  s = wave_sum(s);
  const int wb = __ballot(bad) != 0ull ? 1 : 0;
  if ((threadIdx.x & 63) == 0) {
    red[threadIdx.x >> 6] = s;
    rb[threadIdx.x >> 6] = wb;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    atomicAdd(state, red[0] + red[1] + red[2] + red[3]);
    if (rb[0] | rb[1] | rb[2] | rb[3]) atomicMax((int*)(state + 1), 1);
  }
}

// steps (optional): per-tensor count of completed optimizer steps (fp32, exact to 2^24); the
// bias corrections of this step use steps[t] + 1, computed in double (torch AdamW computes
// 1 - beta ** step on the host in double).  dscale (optional): the device GradScaler scale;
// the grads are unscaled by 1 / dscale[0] instead of inv_scale.
// Deterministic form of sumsq_k: block b writes its sum of squares to partials[b] (the
// non-finite flag is an integer max, order-free), sum_partials_k adds them in a fixed order,
// so the clip coefficient -- and every parameter after the step -- is bit-reproducible.
__global__ __launch_bounds__(256) void sumsq_parts_k(float* const* __restrict__ grads,
                                                     const int64_t* __restrict__ sizes,
                                                     const MTBlock* __restrict__ blocks, float* __restrict__ partials,
                                                     float* __restrict__ state) {
  const MTBlock bl = blocks[blockIdx.x];
  const float* g = grads[bl.tensor];
  const int64_t n = sizes[bl.tensor];
  float s = 0.f;
  int bad = 0;
  for (int64_t i = bl.start + threadIdx.x; i < min(n, bl.start + 4096); i += 256) {
    const float v = g[i];
    s = fmaf(v, v, s);
    bad |= !isfinite(v);
  }
  __shared__ float red[4];
  __shared__ int rb[4];
  s = wave_sum(s);
  const int wb = __ballot(bad) != 0ull ? 1 : 0;
  if ((threadIdx.x & 63) == 0) {
    red[threadIdx.x >> 6] = s;
    rb[threadIdx.x >> 6] = wb;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    partials[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
    if (rb[0] | rb[1] | rb[2] | rb[3]) atomicMax((int*)(state + 1), 1);
  }
}

__global__ __launch_bounds__(1024) void sum_partials_k(const float* __restrict__ partials, int n,
                                                       float* __restrict__ state) {
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 1024) s += partials[i];  // fixed stride order
  __shared__ float red[16];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < 16; ++w) t += red[w];
    state[0] += t;
  }
}

extern "C" int sdp_grad_sumsq_parts(float* const* grads, const int64_t* sizes, const void* blocks, int nblocks,
                                    float* partials, float* state, void* stream) {
  if (!grads || !sizes || !blocks || !partials || !state || nblocks < 0) return (int)hipErrorInvalidValue;
  if (nblocks == 0) return 0;
  hipLaunchKernelGGL(sumsq_parts_k, dim3(nblocks), dim3(256), 0, (hipStream_t)stream, grads, sizes,
                     (const MTBlock*)blocks, partials, state);
  return SDP_CHECK_LAUNCH();
}

extern "C" int sdp_sum_partials(const float* partials, int n, float* state, void* stream) {
  if (!partials || !state || n < 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(sum_partials_k, dim3(1), dim3(1024), 0, (hipStream_t)stream, partials, n, state);
  return SDP_CHECK_LAUNCH();
}

__global__ __launch_bounds__(256) void adamw_k(float* const* __restrict__ params, float* const* __restrict__ grads,
                                               float* const* __restrict__ m1, float* const* __restrict__ m2,
                                               const int64_t* __restrict__ sizes, const MTBlock* __restrict__ blocks,
                                               const float* __restrict__ state, float lr, float b1, float b2,
                                               float eps, float wd, float bc1, float bc2, float inv_scale,
                                               float max_norm, const float* __restrict__ steps,
                                               const float* __restrict__ dscale) {
  if (((const int*)state)[1] != 0) return;  // inf / nan in the grads: skip the step (GradScaler)
  float sc = dscale ? 1.0f / dscale[0] : inv_scale;
  if (max_norm > 0.f) {
    const float norm = sqrtf(state[0]) * sc;
    const float clip = max_norm / (norm + 1e-6f);
    if (clip < 1.f) sc *= clip;
  }
  const MTBlock bl = blocks[blockIdx.x];
  if (steps) {
    const double st = (double)steps[bl.tensor] + 1.0;
    bc1 = (float)(1.0 - pow((double)b1, st));
    bc2 = (float)(1.0 - pow((double)b2, st));
  }
  float* p = params[bl.tensor];
  const float* g = grads[bl.tensor];
  float* a = m1[bl.tensor];
  float* v = m2[bl.tensor];
  const int64_t n = sizes[bl.tensor];
  const float step = lr / bc1, rb2 = 1.0f / sqrtf(bc2);
  for (int64_t i = bl.start + threadIdx.x; i < min(n, bl.start + 4096); i += 256) {
    const float gi = g[i] * sc;
    float pi = p[i] * (1.0f - lr * wd);
    const float mi = b1 * a[i] + (1.0f - b1) * gi;
    const float vi = b2 * v[i] + (1.0f - b2) * gi * gi;
    a[i] = mi;
    v[i] = vi;
    pi -= step * mi / (sqrtf(vi) * rb2 + eps);
    p[i] = pi;
  }
}

extern "C" int sdp_grad_sumsq(float* const* grads, const int64_t* sizes, const void* blocks, int nblocks, float* state,
                              void* stream) {
  if (!grads || !sizes || !blocks || !state || nblocks < 0) return (int)hipErrorInvalidValue;
  if (nblocks == 0) return 0;
  hipLaunchKernelGGL(sumsq_k, dim3(nblocks), dim3(256), 0, (hipStream_t)stream, grads, sizes,
                     (const MTBlock*)blocks, state);
  return SDP_CHECK_LAUNCH();
}

extern "C" int sdp_adamw(float* const* params, float* const* grads, float* const* exp_avg, float* const* exp_avg_sq,
                         const int64_t* sizes, const void* blocks, int nblocks, const float* state, float lr,
                         float beta1, float beta2, float eps, float weight_decay, int step, float inv_scale,
                         float max_norm, void* stream) {
  if (!params || !grads || !exp_avg || !exp_avg_sq || !sizes || !blocks || !state || nblocks < 0 || step <= 0)
    return (int)hipErrorInvalidValue;
  if (nblocks == 0) return 0;
  const float bc1 = 1.0f - powf(beta1, (float)step), bc2 = 1.0f - powf(beta2, (float)step);
  hipLaunchKernelGGL(adamw_k, dim3(nblocks), dim3(256), 0, (hipStream_t)stream, params, grads, exp_avg, exp_avg_sq,
                     sizes, (const MTBlock*)blocks, state, lr, beta1, beta2, eps, weight_decay, bc1, bc2, inv_scale,
                     max_norm, (const float*)nullptr, (const float*)nullptr);
  return SDP_CHECK_LAUNCH();
}

extern "C" int sdp_adamw_dev(float* const* params, float* const* grads, float* const* exp_avg,
                             float* const* exp_avg_sq, const int64_t* sizes, const void* blocks, int nblocks,
                             const float* state, float lr, float beta1, float beta2, float eps, float weight_decay,
                             const float* steps, const float* scale, float inv_scale, float max_norm, void* stream) {
  if (!params || !grads || !exp_avg || !exp_avg_sq || !sizes || !blocks || !state || !steps || nblocks < 0)
    return (int)hipErrorInvalidValue;
  if (nblocks == 0) return 0;
  hipLaunchKernelGGL(adamw_k, dim3(nblocks), dim3(256), 0, (hipStream_t)stream, params, grads, exp_avg, exp_avg_sq,
                     sizes, (const MTBlock*)blocks, state, lr, beta1, beta2, eps, weight_decay, 1.f, 1.f, inv_scale,
                     max_norm, steps, scale);
  return SDP_CHECK_LAUNCH();
}

// End of an optimizer step: when the step was taken (no inf / nan flagged in state[1]) every
// per-tensor step count advances; with sc != NULL the GradScaler scale updates (backoff on a
// skipped step, growth every `interval` clean steps); state is reset for the next step.
__global__ __launch_bounds__(256) void adamw_finish_k(float* __restrict__ state, float* __restrict__ sc, float growth,
                                                      float backoff, int interval, float* __restrict__ steps, int n) {
  const bool bad = ((const int*)state)[1] != 0;
  if (!bad && steps)
    for (int i = threadIdx.x; i < n; i += 256) steps[i] += 1.0f;
  __syncthreads();
  if (threadIdx.x == 0) {
    if (sc) {
      int* tr = (int*)(sc + 1);
      if (bad) {
        sc[0] *= backoff;
        *tr = 0;
      } else if (++*tr >= interval) {
        sc[0] *= growth;
        *tr = 0;
      }
    }
    state[0] = 0.f;
    ((int*)state)[1] = 0;
  }
}

extern "C" int sdp_adamw_finish(float* state, float* scale_tracker, float growth, float backoff, int interval,
                                float* steps, int nsteps, void* stream) {
  if (!state || nsteps < 0 || (scale_tracker && interval <= 0) || (nsteps > 0 && !steps))
    return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(adamw_finish_k, dim3(1), dim3(256), 0, (hipStream_t)stream, state, scale_tracker, growth,
                     backoff, interval, steps, nsteps);
  return SDP_CHECK_LAUNCH();
}

// Size of one work-list entry of sdp_grad_sumsq / sdp_adamw (host builds the table).
extern "C" int sdp_mt_block_bytes(void) { return (int)sizeof(MTBlock); }

// GradScaler.update (torch.amp.GradScaler semantics, training_tools.py:64, :99): scale *= backoff
// and the growth tracker resets when state[1] flags a non-finite gradient, else the tracker
// counts up and the scale grows by `growth` every `interval` clean steps.  Then state is reset
// for the next step.  sc[0] = scale (fp32), sc[1] = tracker (int bits).
__global__ void scaler_update_k(float* __restrict__ state, float* __restrict__ sc, float growth, float backoff,
                                int interval) {
  int* tr = (int*)(sc + 1);
  if (((int*)state)[1] != 0) {
    sc[0] *= backoff;
    *tr = 0;
  } else if (++*tr >= interval) {
    sc[0] *= growth;
    *tr = 0;
  }
  state[0] = 0.f;
  ((int*)state)[1] = 0;
}

extern "C" int sdp_scaler_update(float* state, float* scale_tracker, float growth, float backoff, int interval,
                                 void* stream) {
  if (!state || !scale_tracker || interval <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(scaler_update_k, dim3(1), dim3(1), 0, (hipStream_t)stream, state, scale_tracker, growth, backoff,
                     interval);
  return SDP_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------
// 2-D transpose through LDS (64 x 64 tiles): Y[c][r] = X[r][c], X [R][C] row stride ldx, Y row
// stride ldy.  Weight transposes for the input-gradient GEMMs (dX = dY W runs on the fast
// GEMM as dY . (W^T)^T).
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void transpose_k(const T* __restrict__ X, int64_t ldx, T* __restrict__ Y,
                                                   int64_t ldy, int R, int C) {
  __shared__ T tile[64][65];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int i = ty; i < 64; i += 4) {
    const int r = r0 + i, c = c0 + tx;
    if (r < R && c < C) tile[i][tx] = X[(int64_t)r * ldx + c];
  }
  __syncthreads();
  for (int i = ty; i < 64; i += 4) {
    const int c = c0 + i, r = r0 + tx;
    if (r < R && c < C) Y[(int64_t)c * ldy + r] = tile[tx][i];
  }
}

extern "C" int sdp_transpose(int dtype, const void* X, int64_t ldx, void* Y, int64_t ldy, int R, int C, void* stream) {
  if (!X || !Y || R < 0 || C < 0) return (int)hipErrorInvalidValue;
  if (R == 0 || C == 0) return 0;
  dim3 grid((C + 63) / 64, (R + 63) / 64);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == 1)
    hipLaunchKernelGGL(transpose_k<bf16_t>, grid, dim3(256), 0, s, (const bf16_t*)X, ldx, (bf16_t*)Y, ldy, R, C);
  else if (dtype == 0)
    hipLaunchKernelGGL(transpose_k<float>, grid, dim3(256), 0, s, (const float*)X, ldx, (float*)Y, ldy, R, C);
  else
    return (int)hipErrorInvalidValue;
  return SDP_CHECK_LAUNCH();
}
