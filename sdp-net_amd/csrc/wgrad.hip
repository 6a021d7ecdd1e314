// Weight gradient of every Linear / 1x1 conv of the training backward on the 8-phase MFMA
// main loop (the adjoint of layers.py:79-91, :242-249, :282-284, :308):
//
//     C_s[i][j] = sum_{k in split s} A[k][i] * B[k][j]        (dW = dY^T X, fp32 out)
//
// with A = dY [tokens][lda] and B = X [tokens][ldb], both bf16 and token-major, i.e. the
// reduction runs DOWN the rows of both operands.  Same 256x256x64 tile, 8 waves (2 along i x 4
// along j, 128x64 per wave), 4 MFMA phases per K-tile with the two wave groups ping-ponging and
// the same three LDS-DMA sub-stages as gemm_bf16_8ph (csrc/gemm.hip); only the LDS images and
// the fragment reads differ:
//   * a staged K-tile holds 64 token rows of each operand, cut into column blocks so that each
//     sub-stage is a set of whole blocks and every LDS-DMA piece (64 lanes x 16 B) is a
//     contiguous 1 KiB of one block: A = 4 blocks of 64 i-columns ([64 k][64 i], 128-B rows),
//     B = 8 blocks of 32 j-columns ([64 k][32 j], 64-B rows);
//   * the MFMA operands (16 columns x 32 k per fragment, 8 consecutive k per lane) are read
//     transposed with ds_read_b64_tr_b16 (two per fragment);
//   * 16-B chunks are XOR-swizzled per k-row (the swizzle applied on the DMA source address,
//     the LDS destination stays lane-linear) so that the 8 k-rows x 32 B each 32-lane half of
//     a transposed read touches land on 16 distinct 16-B bank slots.
// K (tokens) is split over workgroups into fp32 slabs C + s * split_stride that the caller
// reduces (sdp_seg_colsum) in a fixed order: results are bit-reproducible.
#include "common.h"

namespace wg {
constexpr int BM = 256, BN = 256, BK = 64, NTHREADS = 512;
constexpr int TILE_BYTES = BM * BK * 2;  // 32 KiB per operand per stage
constexpr int BUF = 2 * TILE_BYTES;

// physical 16-B chunk of logical chunk c in k-row r
SDP_DEV int swz_a(int r) { return 2 * (((r >> 1) & 1) | (((r >> 3) & 1) << 1)); }  // 8 chunks per row
SDP_DEV int swz_b(int r) { return 2 * ((r >> 3) & 1); }                            // 4 chunks per row

typedef short v4i16 __attribute__((ext_vector_type(4)));

#define SDP_VMCNT(n) asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory")

template <bool PH2>
__global__ __launch_bounds__(NTHREADS) void gemm_wgrad_8ph(const bf16_t* __restrict__ A, int64_t lda,
                                                         const bf16_t* __restrict__ B, int64_t ldb,
                                                         float* __restrict__ C, int64_t ldc, int64_t split_stride,
                                                         int tiles_i, int tiles_j, int nkt, int kchunk, int mtok,
                                                         const bf16_t* __restrict__ zrow) {
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const int fr = lane & 15, fq = lane >> 4;
  // XCD-contiguous logical order (blocks b, b + 8, ... share an XCD): an XCD runs consecutive
  // tiles of one split, which share their A / B token rows in its L2
  int split, ti, tj;
  {
    const int nwg = gridDim.x, b = blockIdx.x;
    const int xcd = b & 7, q = nwg >> 3, rem = nwg & 7;
    const int L = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + (b >> 3);
    const int ntiles = tiles_i * tiles_j;
    split = L / ntiles;
    const int t = L - split * ntiles;
    ti = t / tiles_j;
    tj = t - ti * tiles_j;
  }
  const int i0 = ti * BM, j0 = tj * BN;
  const int kt0 = split * kchunk;
  const int kn = min(kchunk, nkt - kt0);
  float* Cs = C + (int64_t)split * split_stride;

  f32x4 acc[4][8];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (kn > 0) {
    // ---- the wave's 8 DMA pieces per K-tile: [0,1] S1-A (blocks 0, 2), [2,3] S1-B (blocks
    // 0, 2, 4, 6), [4,5] S2-B (blocks 1, 3, 5, 7), [6,7] S3-A (blocks 1, 3)
    const bf16_t* src[8];
    int loff[8];
    int64_t kstep[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int idx = wave * 2 + (s & 1);  // 0..15
      const bool isa = s < 2 || s >= 6;
      if (isa) {
        const int blk = (idx < 8 ? 0 : 2) + (s >= 6 ? 1 : 0);
        const int kp = idx & 7;
        const int r = kp * 8 + (lane >> 3), pc = lane & 7;
        const int c = pc ^ swz_a(r);
        src[s] = A + ((int64_t)kt0 * BK + r) * lda + i0 + blk * 64 + c * 8;
        loff[s] = blk * 8192 + kp * 1024;
        kstep[s] = (int64_t)BK * lda;
      } else {
        const int blk = 2 * (idx >> 2) + (s >= 4 ? 1 : 0);
        const int kp = idx & 3;
        const int r = kp * 16 + (lane >> 2), pc = lane & 3;
        const int c = pc ^ swz_b(r);
        src[s] = B + ((int64_t)kt0 * BK + r) * ldb + j0 + blk * 32 + c * 8;
        loff[s] = TILE_BYTES + blk * 4096 + kp * 1024;
        kstep[s] = (int64_t)BK * ldb;
      }
    }
    // the global last K-tile may hold token rows past mtok: those lanes read the zero row
    const bool tail = (mtok & (BK - 1)) != 0 && kt0 + kn == nkt;
    auto dma = [&](int s, int kt) {
      const bf16_t* ptr = src[s] + kt * kstep[s];
      if (tail && kt == kn - 1) {  // wave-uniform
        const int idx = wave * 2 + (s & 1);
        const bool isa = s < 2 || s >= 6;
        int r, col;
        if (isa) {
          r = (idx & 7) * 8 + (lane >> 3);
          col = i0 + ((idx < 8 ? 0 : 2) + (s >= 6 ? 1 : 0)) * 64 + ((lane & 7) ^ swz_a(r)) * 8;
        } else {
          r = (idx & 3) * 16 + (lane >> 2);
          col = j0 + (2 * (idx >> 2) + (s >= 4 ? 1 : 0)) * 32 + ((lane & 3) ^ swz_b(r)) * 8;
        }
        if ((kt0 + kt) * BK + r >= mtok) ptr = zrow + col;
      }
      __builtin_amdgcn_global_load_lds((const AS1 void*)ptr, (AS3 void*)(smem + (kt & 1) * BUF + loff[s]), 16, 0, 0);
    };
    auto S1 = [&](int kt) { dma(0, kt); dma(1, kt); dma(2, kt); dma(3, kt); };
    auto S2 = [&](int kt) { dma(4, kt); dma(5, kt); };
    auto S3 = [&](int kt) { dma(6, kt); dma(7, kt); };

    // per-lane parts of the transposed fragment addresses: lane (g, q, p) reads k-row
    // 8 g + q (+4 for the upper half) and the 8-B piece p of the fragment's 16 columns
    const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
    const int swa = 2 * (((q >> 1) & 1) | ((g & 1) << 1));  // = swz_a of every row the lane reads
    const int swb = 2 * (g & 1);                            // = swz_b of every row the lane reads
    int offa[4], offb[2];
#pragma unroll
    for (int cbi = 0; cbi < 4; ++cbi) offa[cbi] = (8 * g + q) * 128 + ((((2 * cbi) ^ swa) | (p >> 1)) << 4) + 8 * (p & 1);
#pragma unroll
    for (int cbi = 0; cbi < 2; ++cbi) offb[cbi] = TILE_BYTES + (8 * g + q) * 64 + ((((2 * cbi) ^ swb) | (p >> 1)) << 4) + 8 * (p & 1);

    auto tr2 = [&](const char* a0, int hi_off) {
      const v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((AS3 v4i16*)(a0));
      const v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((AS3 v4i16*)(a0 + hi_off));
      return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    };
    bf16x8 xf[8], w0[4], w1[4];
    // A fragments (i columns wm*128 + jm*64 + j*16: block 2 wm + jm, column group j)
    auto read_x = [&](const char* buf, int jm) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          xf[j * 2 + ks] = tr2(buf + (2 * wm + jm) * 8192 + ks * 32 * 128 + offa[j], 4 * 128);
    };
    // B fragments (j columns wn*64 + in*32 + i*16: block 2 wn + in, column group i)
    auto read_w = [&](const char* buf, int in, bf16x8(&wf)[4]) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          wf[i * 2 + ks] = tr2(buf + (2 * wn + in) * 4096 + ks * 32 * 64 + offb[i], 4 * 64);
    };
    auto quad = [&](int jm, int in, const bf16x8(&wf)[4]) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[in * 2 + i][jm * 4 + j] =
                __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[i * 2 + ks], xf[j * 2 + ks], acc[in * 2 + i][jm * 4 + j], 0, 0, 0);
    };
    auto mfma_section = [&](auto&& body) {
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
      body();
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    };

    if constexpr (PH2) {
      // 2 phases per K-tile (32 MFMAs per section): the schedule and retire counts of
      // gemm_bf16_8ph's 2-phase loop (csrc/gemm.hip), which reads its staged regions in the same
      // phases (w0, w1, x half 0 in P0; x half 1 in P1)
#ifndef SDP_WGRAD_PH2_PRIO
// 1 (default): static priority for wave group 1, as gemm_bf16_8ph's PH2 loop; XL bs120 training
// 1,045 / 1,059 img/s (both kernels flipping per section) -> 1,054 / 1,063 (GEMM static) ->
// 1,064 / 1,059 (both static), interleaved on one box (tools/r4_prio2.sh); 0 = per-section flips
#define SDP_WGRAD_PH2_PRIO 1
#endif
      if (SDP_WGRAD_PH2_PRIO == 1 && __builtin_amdgcn_readfirstlane(wm) == 1) __builtin_amdgcn_s_setprio(1);
      auto section = [&](auto&& body) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        if (SDP_WGRAD_PH2_PRIO == 0) __builtin_amdgcn_s_setprio(1);
        body();
        if (SDP_WGRAD_PH2_PRIO == 0) __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
      };
      S1(0); S2(0); S3(0);
      if (kn > 1) { S1(1); S2(1); SDP_VMCNT(8); }
      else SDP_VMCNT(2);
      __builtin_amdgcn_s_barrier();
      if (wm == 1) __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      for (int t = 0; t < kn; ++t) {
        const char* buf = smem + (t & 1) * BUF;
        const bool more1 = t + 1 < kn, more2 = t + 2 < kn;
        read_w(buf, 0, w0);
        read_w(buf, 1, w1);
        read_x(buf, 0);
        if (more1) { S3(t + 1); SDP_VMCNT(8); } else SDP_VMCNT(0);
        section([&] { quad(0, 0, w0); quad(0, 1, w1); });
        read_x(buf, 1);
        if (more2) { S1(t + 2); S2(t + 2); SDP_VMCNT(8); }
        else if (more1) SDP_VMCNT(2);
        section([&] { quad(1, 1, w1); quad(1, 0, w0); });
      }
      if (wm == 0) __builtin_amdgcn_s_barrier();
    } else {
    // prologue / schedule / retire counts exactly as gemm_bf16_8ph (same pieces per sub-stage)
    S1(0); S2(0); S3(0);
    if (kn > 1) { S1(1); S2(1); SDP_VMCNT(10); }
    else SDP_VMCNT(4);
    __builtin_amdgcn_s_barrier();
    if (wm == 1) __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);

    for (int t = 0; t < kn; ++t) {
      const char* buf = smem + (t & 1) * BUF;
      const bool more1 = t + 1 < kn, more2 = t + 2 < kn;
      read_w(buf, 0, w0);
      read_x(buf, 0);
      if (more1) { S3(t + 1); SDP_VMCNT(10); } else SDP_VMCNT(2);
      mfma_section([&] { quad(0, 0, w0); });
      read_w(buf, 1, w1);
      if (more1) SDP_VMCNT(8); else SDP_VMCNT(0);
      mfma_section([&] { quad(0, 1, w1); });
      read_x(buf, 1);
      if (more2) S1(t + 2);
      mfma_section([&] { quad(1, 1, w1); });
      if (more2) { S2(t + 2); SDP_VMCNT(10); }
      else if (more1) SDP_VMCNT(4);
      mfma_section([&] { quad(1, 0, w0); });
    }
    if (wm == 0) __builtin_amdgcn_s_barrier();
    }  // !PH2
  }

  // ---- fp32 epilogue: D[j][i] per 16x16 block, lane (fr, fq) holds j = 4 fq + r, i = fr:
  // one 16-B store of C[i][j .. j+3] per block
#pragma unroll
  for (int in2 = 0; in2 < 4; ++in2)
#pragma unroll
    for (int jm4 = 0; jm4 < 8; ++jm4) {
      const int i = i0 + wm * 128 + jm4 * 16 + fr;
      const int j = j0 + wn * 64 + in2 * 16 + fq * 4;
      *(f32x4*)(Cs + (int64_t)i * ldc + j) = acc[in2][jm4];
    }
}

#undef SDP_VMCNT
}  // namespace wg

extern "C" int sdp_gemm_wgrad(const void* A, int64_t lda, const void* B, int64_t ldb, float* C, int64_t ldc,
                              int64_t split_stride, int ni, int nj, int ktok, int kchunk_tiles, const void* zrow,
                              void* stream) {
  if (!A || !B || !C || ni <= 0 || nj <= 0 || ktok <= 0 || kchunk_tiles <= 0) return (int)hipErrorInvalidValue;
  if (ni % wg::BM || nj % wg::BN || lda % 8 || ldb % 8 || ldc % 4 || (uintptr_t)A % 16 || (uintptr_t)B % 16 ||
      (uintptr_t)C % 16 || lda < ni || ldb < nj || ldc < nj)
    return (int)hipErrorNotSupported;
  if (ktok % wg::BK && (!zrow || (uintptr_t)zrow % 16)) return (int)hipErrorInvalidValue;
  const int nkt = (ktok + wg::BK - 1) / wg::BK;
  const int splits = (nkt + kchunk_tiles - 1) / kchunk_tiles;
  if (splits > 1 && split_stride < (int64_t)ni * ldc) return (int)hipErrorInvalidValue;
  const int ti = ni / wg::BM, tj = nj / wg::BN;
  const int64_t nwg = (int64_t)ti * tj * splits;
  if (nwg > (1 << 30)) return (int)hipErrorInvalidValue;
  // the main-loop phase count follows the forward GEMM's (sdp_gemm_set_kloop_phases; 0 = query)
  // (the 4-phase loop exists only in the diagnostic build)
#ifdef SDP_DIAG
  if (sdp_gemm_set_kloop_phases(0) != 2)
    hipLaunchKernelGGL(wg::gemm_wgrad_8ph<false>, dim3((unsigned)nwg), dim3(wg::NTHREADS), 0, (hipStream_t)stream,
                       (const bf16_t*)A, lda, (const bf16_t*)B, ldb, C, ldc, split_stride, ti, tj, nkt, kchunk_tiles,
                       ktok, (const bf16_t*)zrow);
  else
#endif
    hipLaunchKernelGGL(wg::gemm_wgrad_8ph<true>, dim3((unsigned)nwg), dim3(wg::NTHREADS), 0, (hipStream_t)stream,
                       (const bf16_t*)A, lda, (const bf16_t*)B, ldb, C, ldc, split_stride, ti, tj, nkt, kchunk_tiles,
                       ktok, (const bf16_t*)zrow);
  return SDP_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------
// Per-step weight preparation of the training forward / backward in one launch: every entry
// reads an fp32 weight [R][C] (row stride C) once and writes its bf16 copy dst[r * ldd + c]
// (the GEMM operand of the forward) and / or its transposed bf16 copy dstT[c * ldt + r] (the
// operand of the input-gradient GEMM dX = dY W); either output may be NULL.  64 x 64 tiles,
// transposed through LDS.  Replaces one cast and one transpose launch per weight and step.
// ---------------------------------------------------------------------------
struct MtCastT {
  const float* src;
  uint16_t* dst;
  uint16_t* dstT;
  int64_t ldd, ldt;
  int R, C;
};

extern "C" int sdp_mt_cast_transpose_entry_bytes(void) { return (int)sizeof(MtCastT); }

__global__ __launch_bounds__(256) void mt_cast_transpose_k(const MtCastT* __restrict__ ent,
                                                           const int4* __restrict__ tiles) {
  __shared__ uint16_t tl[64][72];
  const int4 t = tiles[blockIdx.x];
  const MtCastT e = ent[t.x];
  const int r0 = t.y, c0 = t.z, tid = threadIdx.x;
  const int cc = (tid & 15) * 4;
  const bool vec = (e.C & 3) == 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int rr = (tid >> 4) + 16 * i;
    const int r = r0 + rr, c = c0 + cc;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    if (r < e.R) {
      const float* p = e.src + (int64_t)r * e.C + c;
      if (vec && c + 3 < e.C) {
        const float4 q = *(const float4*)p;
        v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (c + k < e.C) v[k] = p[k];
      }
    }
    uint16_t b[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      b[k] = f2bf(v[k]);
      tl[rr][cc + k] = b[k];
    }
    if (e.dst && r < e.R) {
      uint16_t* q = e.dst + (int64_t)r * e.ldd + c;
      if (c + 3 < e.C && ((uintptr_t)q & 7) == 0) {
        *(uint2*)q = make_uint2((uint32_t)b[0] | ((uint32_t)b[1] << 16), (uint32_t)b[2] | ((uint32_t)b[3] << 16));
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (c + k < e.C) q[k] = b[k];
      }
    }
  }
  if (!e.dstT) return;
  __syncthreads();
  // transposed: lane -> column c0 + tc, rows r0 + tr .. tr + 15 (32 contiguous bytes)
  const int tc = tid >> 2, tr = (tid & 3) * 16;
  const int c = c0 + tc;
  if (c >= e.C) return;
  uint16_t* q = e.dstT + (int64_t)c * e.ldt + r0 + tr;
  uint32_t w[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) w[k] = (uint32_t)tl[tr + 2 * k][tc] | ((uint32_t)tl[tr + 2 * k + 1][tc] << 16);
  if (r0 + tr + 15 < e.R && ((uintptr_t)q & 15) == 0) {
    *(uint4*)q = make_uint4(w[0], w[1], w[2], w[3]);
    *(uint4*)(q + 8) = make_uint4(w[4], w[5], w[6], w[7]);
  } else {
#pragma unroll
    for (int k = 0; k < 16; ++k)
      if (r0 + tr + k < e.R) q[k] = tl[tr + k][tc];
  }
}

extern "C" int sdp_mt_cast_transpose(const void* entries, const void* tiles, int ntiles, void* stream) {
  if (!entries || !tiles || ntiles < 0) return (int)hipErrorInvalidValue;
  if (ntiles == 0) return 0;
  hipLaunchKernelGGL(mt_cast_transpose_k, dim3(ntiles), dim3(256), 0, (hipStream_t)stream, (const MtCastT*)entries,
                     (const int4*)tiles);
  return SDP_CHECK_LAUNCH();
}
