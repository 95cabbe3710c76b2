// probe_coresident.hip -- when do a launch's workgroups share a CU with another launch's?
// (GPU box, diagnostic only.)
//
//   hipcc -std=c++20 -O3 --offload-arch=gfx950 tools/probe_coresident.hip -o tools/probe_coresident && tools/probe_coresident
//
// Spin kernels record s_memrealtime at start; reported relative to the first start of the
// first launch: (1) one launch of 2 workgroups per CU; (2) a 256-workgroup launch followed
// by a hipExtAnyOrderLaunch launch on the same stream, by block size and LDS of the second.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#define CK(x)                                                                           \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                          \
    }                                                                                   \
  } while (0)

template <int THREADS, int LDS>
__global__ __launch_bounds__(THREADS) void spin_kernel(unsigned long long* ts, int spin_ticks) {
  __shared__ float scratch[LDS / 4];
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) ts[blockIdx.x] = t0;
  scratch[threadIdx.x % (LDS / 4)] = (float)t0;
  while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)spin_ticks) __builtin_amdgcn_s_sleep(2);
  __syncthreads();
  if (threadIdx.x == 0 && scratch[(threadIdx.x + 1) % (LDS / 4)] == -1.0f) ts[0] = 0;
}

static void stats(const char* what, const std::vector<unsigned long long>& t, unsigned long long base) {
  unsigned long long lo = ~0ull, hi = 0;
  for (auto v : t) { lo = v < lo ? v : lo; hi = v > hi ? v : hi; }
  printf("  %-36s first start %7.2f us, last start %7.2f us\n", what, (lo - base) * 0.01, (hi - base) * 0.01);
}

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  unsigned long long *a, *b;
  CK(hipMalloc(&a, 4096 * 8));
  CK(hipMalloc(&b, 4096 * 8));
  std::vector<unsigned long long> ha, hb;
  auto get = [&](unsigned long long* d, int n, std::vector<unsigned long long>& h) {
    h.resize(n);
    CK(hipMemcpy(h.data(), d, n * 8, hipMemcpyDeviceToHost));
  };
  int spin = 3000;   // 30 us
  // (1) one launch, 512 and 1024 workgroups of 512 threads, 16 KiB LDS
  for (int grid : {256, 512, 1024}) {
    hipLaunchKernelGGL((spin_kernel<512, 16384>), dim3(grid), dim3(512), 0, s, a, spin);
    CK(hipStreamSynchronize(s));
    get(a, grid, ha);
    unsigned long long base = ~0ull;
    for (auto v : ha) base = v < base ? v : base;
    char buf[64];
    snprintf(buf, sizeof buf, "one launch, %d WG x 512 thr", grid);
    stats(buf, ha, base);
  }
  // (2) 256 WG (512 threads, 16 KiB) then any-order launch of 256 WG
  auto pair = [&](auto kb, int tb, const char* what, int flags) {
    void* aa[] = {(void*)&a, (void*)&spin};
    int spin_b = 500;
    void* ab[] = {(void*)&b, (void*)&spin_b};
    CK(hipExtLaunchKernel((const void*)spin_kernel<512, 16384>, dim3(256), dim3(512), aa, 0, s, nullptr, nullptr, 0));
    CK(hipExtLaunchKernel((const void*)kb, dim3(256), dim3(tb), ab, 0, s, nullptr, nullptr, flags));
    CK(hipStreamSynchronize(s));
    get(a, 256, ha);
    get(b, 256, hb);
    unsigned long long base = ~0ull;
    for (auto v : ha) base = v < base ? v : base;
    printf(" %s (flags %d):\n", what, flags);
    stats("A 256 x 512 thr, 16 KiB", ha, base);
    stats("B", hb, base);
  };
  for (int fl : {0, 1}) {
    pair(spin_kernel<512, 16384>, 512, "B = 256 x 512 thr, 16 KiB", fl);
    pair(spin_kernel<256, 16384>, 256, "B = 256 x 256 thr, 16 KiB", fl);
    pair(spin_kernel<64, 1024>, 64, "B = 256 x 64 thr, 1 KiB", fl);
  }
  return 0;
}
