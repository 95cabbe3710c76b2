// probe_ldsdma.hip -- the LDS-DMA issue / landing rate of a loader-only ring (GPU box, not part of
// the product), to size the persistent decode's loader (pds.hip):
//
//   hipcc -O3 --offload-arch=gfx950 tools/probe_ldsdma.hip -o exp/probe_ldsdma && exp/probe_ldsdma
//
// 256 workgroups (one per CU) of NL loader waves stream their own contiguous 4 MiB each in 16 KiB
// fills of 16 one-KiB pieces (64 lanes x 16 B) into an 8-slot LDS ring, loader w issuing pieces
// w, w + NL, ...; AHEAD fills in flight per wave (s_waitcnt vmcnt(AHEAD * 16 / NL)).  Variants:
//   MODE 0: inline asm with M0 saved / set / restored around each global_load_lds_dwordx4 ... nt (pds.hip)
//   MODE 1: __builtin_amdgcn_global_load_lds(..., 16, 0, aux = 2 (nt))
//   ALT:    pieces alternate between two regions (the attention's K / V pieces)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) {                                                                    \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));        \
      exit(1);                                                                                 \
    }                                                                                          \
  } while (0)

typedef const char __attribute__((address_space(1))) gchar;
typedef char __attribute__((address_space(3))) lchar;

template <int NL, int MODE, int AHEAD, bool ALT>
__global__ __launch_bounds__(NL * 64, 1) void dma_kernel(const char* buf, size_t per_wg, int nfill, int* sink) {
  extern __shared__ __attribute__((aligned(16))) char smem[];   // 8 slots x 16 KiB
  constexpr int PPL = 16 / NL;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const char* b0 = buf + (size_t)blockIdx.x * per_wg;
  const char* b1 = buf + (size_t)(gridDim.x + blockIdx.x) * per_wg;
  const uint32_t ring = (uint32_t)(uintptr_t)smem;
  for (int f = 0; f < nfill; ++f) {
    const uint32_t slot = (uint32_t)(f & 7) * 16384u;
#pragma unroll
    for (int jj = 0; jj < PPL; ++jj) {
      const int j = w + jj * NL;
      const char* src = ALT ? ((j & 1) ? b1 : b0) + ((size_t)f * 8 + (j >> 1)) * 1024 + lane * 16
                            : b0 + ((size_t)f * 16 + j) * 1024 + lane * 16;
      if constexpr (MODE == 0) {
        uint32_t keep;
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep)
                     : "v"(src), "s"(__builtin_amdgcn_readfirstlane(ring + slot + j * 1024))
                     : "memory");
      } else {
        __builtin_amdgcn_global_load_lds((gchar*)src, (lchar*)(smem + slot + j * 1024), 16, 0, 2);
      }
    }
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PPL * AHEAD) : "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane == 0 && smem[w] == 123 && smem[w + 1] == 45) sink[0] = 1;   // keep the loads
}

template <int NL, int MODE, int AHEAD, bool ALT>
static void run(const char* buf, size_t per_wg, int nfill, int* sink, const char* name) {
  auto fn = dma_kernel<NL, MODE, AHEAD, ALT>;
  CK(hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL(fn, dim3(256), dim3(NL * 64), 128 * 1024, 0, buf, per_wg, nfill, sink);   // warm
  CK(hipDeviceSynchronize());
  const int reps = 5;
  CK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(fn, dim3(256), dim3(NL * 64), 128 * 1024, 0, buf, per_wg, nfill, sink);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  const double us = ms * 1000.0 / reps, bytes = 256.0 * nfill * 16384.0;
  printf("%-34s %8.1f us  %7.2f TB/s  %6.2f GB/s per CU  %5.3f us per fill\n", name, us, bytes / us / 1e6,
         bytes / 256 / us / 1e3, us / nfill);
}

int main() {
  const int nfill = 256;                       // 4 MiB per workgroup
  const size_t per_wg = (size_t)nfill * 16384;
  char* buf;
  int* sink;
  CK(hipMalloc(&buf, per_wg * 512));          // two regions per workgroup (ALT)
  CK(hipMemset(buf, 1, per_wg * 512));
  CK(hipMalloc(&sink, 4));
  run<1, 0, 3, false>(buf, per_wg, nfill, sink, "1 loader asm(M0 save) ahead 3");
  run<1, 1, 3, false>(buf, per_wg, nfill, sink, "1 loader builtin ahead 3");
  run<2, 0, 3, false>(buf, per_wg, nfill, sink, "2 loaders asm ahead 3");
  run<2, 1, 3, false>(buf, per_wg, nfill, sink, "2 loaders builtin ahead 3");
  run<4, 0, 3, false>(buf, per_wg, nfill, sink, "4 loaders asm ahead 3");
  run<4, 1, 3, false>(buf, per_wg, nfill, sink, "4 loaders builtin ahead 3");
  run<4, 1, 5, false>(buf, per_wg, nfill, sink, "4 loaders builtin ahead 5");
  run<1, 0, 3, true>(buf, per_wg, nfill, sink, "1 loader asm ahead 3, K/V alternating");
  run<1, 1, 3, true>(buf, per_wg, nfill, sink, "1 loader builtin ahead 3, K/V alternating");
  run<4, 1, 3, true>(buf, per_wg, nfill, sink, "4 loaders builtin ahead 3, K/V alternating");
  CK(hipFree(buf));
  CK(hipFree(sink));
  return 0;
}
