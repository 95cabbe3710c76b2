// probe_waves.hip -- does a CU stream faster with more waves in flight? (GPU box, diagnostic)
//
//   hipcc -O3 --offload-arch=gfx950 tools/probe_waves.hip -o tools/probe_waves && tools/probe_waves
//
// Pure nt weight stream (no compute, no dependency) on the 7B INT4 decode byte counts, one
// workgroup per CU (grid 256), graph-replayed over a rotating 1 GiB buffer (cold), for
// workgroups of 4 / 8 / 16 waves and ring depths R (16-byte loads in flight per lane).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#define CK(x)                                                                               \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess) {                                                                 \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));     \
      exit(1);                                                                              \
    }                                                                                       \
  } while (0)

template <int R>
__global__ __launch_bounds__(1024, 1) void stream_kernel(const u32x4* __restrict__ w, size_t n_items, float* out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, waves = blockDim.x >> 6;
  const size_t i0 = (size_t)blockIdx.x * n_items / gridDim.x, i1 = (size_t)(blockIdx.x + 1) * n_items / gridDim.x;
  const u32x4* base = w + wave * 64 + lane;
  const size_t stride = (size_t)waves * 64;
  u32x4 ring[R];
  size_t j = i0;
#pragma unroll
  for (int s = 0; s < R; ++s) {
    const size_t jj = j + s < i1 ? j + s : i1 - 1;
    ring[s] = __builtin_nontemporal_load(base + jj * stride);
  }
  unsigned acc = 0;
  for (; j < i1; j += R) {
#pragma unroll
    for (int s = 0; s < R; ++s) {
      acc ^= ring[s][0] + ring[s][1] * 3 + ring[s][2] * 5 + ring[s][3] * 7;
      const size_t jj = j + R + s < i1 ? j + R + s : i1 - 1;
      ring[s] = __builtin_nontemporal_load(base + jj * stride);
    }
  }
  if (acc == 0x12345678u) out[threadIdx.x] = (float)acc;
}

template <class F>
static double time_graph(hipStream_t s, int reps, F f) {
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  for (int r = 0; r < reps; ++r) f();
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  CK(hipGraphLaunch(ge, s));
  CK(hipStreamSynchronize(s));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a, s));
  CK(hipGraphLaunch(ge, s));
  CK(hipEventRecord(b, s));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  return ms * 1e3 / reps;
}

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  float* out;
  CK(hipMalloc(&out, 4096 * 4));
  const size_t big = 1ull << 30;
  void* wbuf;
  CK(hipMalloc(&wbuf, big));
  CK(hipMemset(wbuf, 1, big));
  CK(hipDeviceSynchronize());
  const double sizes_mb[] = {8.66, 25.97, 46.51, 23.27, 67.6};
  const char* names[] = {"o", "qkv", "gate_up", "down", "lm_head"};
  for (int si = 0; si < 5; ++si) {
    const size_t bytes = (size_t)(sizes_mb[si] * 1e6) & ~(size_t)16383;
    const int nbuf = (int)(big / bytes);
    printf("%-8s %6.2f MB:", names[si], bytes / 1e6);
    for (int threads : {256, 512, 1024}) {
      const size_t items = bytes / (threads * 16);
      int rot = 0;
      auto next = [&]() { const u32x4* p = (const u32x4*)((char*)wbuf + (size_t)(rot % nbuf) * bytes); ++rot; return p; };
      const double t2 = time_graph(s, 64, [&] { stream_kernel<2><<<256, threads, 0, s>>>(next(), items, out); });
      const double t4 = time_graph(s, 64, [&] { stream_kernel<4><<<256, threads, 0, s>>>(next(), items, out); });
      const double t8 = time_graph(s, 64, [&] { stream_kernel<8><<<256, threads, 0, s>>>(next(), items, out); });
      const double t16 = time_graph(s, 64, [&] { stream_kernel<16><<<256, threads, 0, s>>>(next(), items, out); });
      printf(" | %2dw R2 %5.2f R4 %5.2f R8 %5.2f R16 %5.2f", threads / 64, t2, t4, t8, t16);
    }
    printf("  (us/launch)\n");
  }
  return 0;
}
