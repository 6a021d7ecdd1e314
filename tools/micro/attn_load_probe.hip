// Load-only probe of the attention access pattern (M forward: B 256, N 200, 12 heads of 64,
// QKV rows [B*N, 2304] bf16): each persistent workgroup walks (b, head-group) pairs and
// DMA-stages K and V of HG heads into LDS (global_load_lds, 16 B per lane), waits, barriers.
// Reports GB/s for HG = 1 (128-B row pieces, what attn_fa4 does) and HG = 2, 4 (256 / 512 B).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#define AS1 __attribute__((address_space(1)))
#define AS3 __attribute__((address_space(3)))

template <int HG>
__global__ __launch_bounds__(256) void probe(const unsigned short* __restrict__ qkv, int ldq, int B, int N, int H,
                                             int hd, int* sink) {
  extern __shared__ __attribute__((aligned(16))) char sm[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ngroups = H / HG, npairs = B * ngroups;
  const int C = H * hd;
  const int rowbytes = HG * hd * 2, cpr = rowbytes / 16;
  const int NP16 = (N + 15) / 16 * 16;
  const int nchunk = NP16 * cpr, ninst = (nchunk + 63) / 64;
  for (int pair = blockIdx.x; pair < npairs; pair += gridDim.x) {
    const int b = pair / ngroups, g = pair - b * ngroups;
    const unsigned short* base = qkv + (long)b * N * ldq + g * HG * hd;
    for (int i = wave; i < 2 * ninst; i += 4) {
      const bool isv = i >= ninst;
      const int ii = isv ? i - ninst : i;
      const int gg = ii * 64 + lane;
      const int row = gg / cpr, pc = gg - row * cpr;
      const int srow = row < N ? row : N - 1;
      const unsigned short* src = base + (long)srow * ldq + (isv ? 2 * C : C) + pc * 8;
      char* dst = sm + (isv ? nchunk * 16 : 0) + ii * 1024;
      if (gg < nchunk) __builtin_amdgcn_global_load_lds((const AS1 void*)src, (AS3 void*)dst, 16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if (tid == 0 && sm[5] == 123) sink[0] = 1;
}

template <int HG>
float run(const unsigned short* d, int B, int N, int H, int hd, int grid, int* sink) {
  const int NP16 = (N + 15) / 16 * 16;
  const size_t lds = (size_t)2 * NP16 * HG * hd * 2;
  hipFuncSetAttribute((const void*)probe<HG>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(probe<HG>, dim3(grid), dim3(256), lds, 0, d, 3 * H * hd, B, N, H, hd, sink);
  hipEventRecord(a);
  for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(probe<HG>, dim3(grid), dim3(256), lds, 0, d, 3 * H * hd, B, N, H, hd, sink);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  const double us = ms * 1e3 / 20;
  const double mb = 2.0 * B * N * H * hd * 2 / 1e6;
  printf("HG %d grid %5d lds %6zu B: %7.1f us  K+V %.0f MB -> %.2f TB/s\n", HG, grid, lds, us, mb, mb / us);
  return (float)us;
}

int main() {
  const int B = 256, N = 200, H = 12, hd = 64;
  unsigned short* d;
  int* sink;
  hipMalloc(&d, (size_t)B * N * 3 * H * hd * 2);
  hipMalloc(&sink, 4);
  hipMemset(d, 0, (size_t)B * N * 3 * H * hd * 2);
  for (int g : {256, 512, 768}) run<1>(d, B, N, H, hd, g, sink);
  for (int g : {256, 512}) run<2>(d, B, N, H, hd, g, sink);
  run<4>(d, B, N, H, hd, 256, sink);
  hipFree(d);
  return 0;
}
