// probe_stream.hip -- ceiling probe for the decode GEMV design (GPU box, not part of the product).
//
//   hipcc -O3 --offload-arch=gfx950 tools/probe_stream.hip -o tools/probe_stream && tools/probe_stream
//
// Measures, per launch, on the byte counts of the Llama-2-7B INT4 decode projections:
//   * a trivial 256-WG kernel chain (the dependent-launch boundary),
//   * a pure weight stream with the GEMV's access pattern (8 waves per WG, 1 KiB per wave
//     instruction, contiguous per-WG range, R loads in flight per wave), default vs nt policy,
//     for several grid shapes,
// eager back-to-back and replayed from a hipGraph.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

__global__ void trivial_kernel(int* p) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && p[0] == 12345) p[1] = 1;
}

// Each WG streams items [i0, i1) of 8 KiB (8 waves x 1 KiB); wave w loads the w-th KiB.
template <int R, bool NT>
__global__ __launch_bounds__(512, 1) void stream_kernel(const u32x4* __restrict__ w, size_t n_items, float* out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, waves = blockDim.x >> 6;
  const size_t i0 = (size_t)blockIdx.x * n_items / gridDim.x, i1 = (size_t)(blockIdx.x + 1) * n_items / gridDim.x;
  const u32x4* base = w + wave * 64 + lane;
  const size_t stride = (size_t)waves * 64;
  u32x4 ring[R];
  size_t j = i0;
#pragma unroll
  for (int s = 0; s < R; ++s) {
    const size_t jj = j + s < i1 ? j + s : i1 - 1;
    ring[s] = NT ? __builtin_nontemporal_load(base + jj * stride) : base[jj * stride];
  }
  unsigned acc = 0;
  for (; j < i1; j += R) {
#pragma unroll
    for (int s = 0; s < R; ++s) {
      acc ^= ring[s][0] + ring[s][1] * 3 + ring[s][2] * 5 + ring[s][3] * 7;
      const size_t jj = j + R + s < i1 ? j + R + s : i1 - 1;
      ring[s] = NT ? __builtin_nontemporal_load(base + jj * stride) : base[jj * stride];
    }
  }
  if (acc == 0x12345678u) out[threadIdx.x] = (float)acc;
}

struct Timer {
  hipEvent_t a, b;
  Timer() { CK(hipEventCreate(&a)); CK(hipEventCreate(&b)); }
};

template <class F>
static double time_eager(hipStream_t s, int reps, F f) {
  Timer t;
  f();
  CK(hipStreamSynchronize(s));
  CK(hipEventRecord(t.a, s));
  for (int r = 0; r < reps; ++r) f();
  CK(hipEventRecord(t.b, s));
  CK(hipEventSynchronize(t.b));
  float ms;
  CK(hipEventElapsedTime(&ms, t.a, t.b));
  return ms * 1e3 / reps;
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
  Timer t;
  CK(hipEventRecord(t.a, s));
  CK(hipGraphLaunch(ge, s));
  CK(hipEventRecord(t.b, s));
  CK(hipEventSynchronize(t.b));
  float ms;
  CK(hipEventElapsedTime(&ms, t.a, t.b));
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  return ms * 1e3 / reps;
}

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  int* flag;
  CK(hipMalloc(&flag, 64));
  CK(hipMemset(flag, 0, 64));
  float* out;
  CK(hipMalloc(&out, 4096));
  const size_t big = 1ull << 30;   // rotate through 1 GiB so consecutive launches miss MALL
  void* wbuf;
  CK(hipMalloc(&wbuf, big));
  CK(hipMemset(wbuf, 1, big));
  CK(hipDeviceSynchronize());

  printf("trivial 256x256: eager %.2f us/launch, graph %.2f us/launch\n",
         time_eager(s, 200, [&] { trivial_kernel<<<256, 256, 0, s>>>(flag); }),
         time_graph(s, 200, [&] { trivial_kernel<<<256, 256, 0, s>>>(flag); }));

  const double sizes_mb[] = {8.66, 25.97, 46.51, 23.27, 67.6};
  const char* names[] = {"o", "qkv", "gate_up", "down", "lm_head"};
  const int grids[] = {256, 512};
  for (int si = 0; si < 5; ++si) {
    const size_t bytes = (size_t)(sizes_mb[si] * 1e6) & ~(size_t)8191;
    const size_t items = bytes / 8192;
    const int nbuf = (int)(big / bytes);
    for (int gi = 0; gi < 2; ++gi) {
      const int grid = grids[gi];
      int rot = 0;
      auto next = [&]() { const u32x4* p = (const u32x4*)((char*)wbuf + (size_t)(rot % nbuf) * bytes); ++rot; return p; };
      double t[4];
      t[0] = time_graph(s, 64, [&] { stream_kernel<16, false><<<grid, 512, 0, s>>>(next(), items, out); });
      t[1] = time_graph(s, 64, [&] { stream_kernel<16, true><<<grid, 512, 0, s>>>(next(), items, out); });
      t[2] = time_graph(s, 64, [&] { stream_kernel<8, true><<<grid, 512, 0, s>>>(next(), items, out); });
      rot = 0;
      t[3] = time_graph(s, 64, [&] { stream_kernel<16, true><<<grid, 512, 0, s>>>((const u32x4*)wbuf, items, out); });
      printf("%-8s %7.2f MB grid %4d: R16 %6.2f us (%5.0f GB/s) | R16 nt %6.2f us (%5.0f) | R8 nt %6.2f us (%5.0f) | "
             "same-buffer R16 nt %6.2f us (%5.0f)\n",
             names[si], bytes / 1e6, grid, t[0], bytes / t[0] / 1e3, t[1], bytes / t[1] / 1e3, t[2], bytes / t[2] / 1e3,
             t[3], bytes / t[3] / 1e3);
    }
  }
  return 0;
}
