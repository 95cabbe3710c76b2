// probe_mb.hip -- per-launch timing of the batched-rows GEMM (ti_gemm_wq_a16 at 17-32 fp16
// rows, gemv_mb_kernel) on the Llama-2-7B decode shapes, graph-replayed over rotating
// weights (cold), GPU box, diagnostic only:
//   for e in 0 8 32; do hipcc -std=c++20 -O3 -Iinclude -Iturboinfer_amd/csrc/kernels --offload-arch=gfx950 \
//     -DTI_GEMV_EXP=$e tools/probe_mb.hip -o tools/probe_mb_e$e; done
// TI_GEMV_EXP: 8 = no activation traffic after the first chunk, 32 = no weight traffic.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>

#include "../turboinfer_amd/csrc/kernels/gemv.hip"

int ti_set_error(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vfprintf(stderr, fmt, ap);
  va_end(ap);
  fprintf(stderr, "\n");
  return code;
}
int ti_check_hip(hipError_t e, const char* what) {
  if (e == hipSuccess) return 0;
  fprintf(stderr, "%s: %s\n", what, hipGetErrorString(e));
  exit(1);
}
#define CK(x) ti_check_hip((x), #x)

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 32;
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  struct Shape { const char* name; int K, N; } shapes[] = {
      {"qkv", 4096, 12288}, {"o", 4096, 4096}, {"gate_up", 4096, 22016}, {"down", 11008, 4096}, {"lm_head", 4096, 32000}};
  const size_t big = 1ull << 30;
  void* wbuf;
  CK(hipMalloc(&wbuf, big));
  CK(hipMemset(wbuf, 0x5a, big));
  void *x, *y;
  CK(hipMalloc(&x, 32 * 11008 * 2));
  CK(hipMemset(x, 0, 32 * 11008 * 2));
  CK(hipMalloc(&y, 32 * 32000 * 4));
  CK((hipError_t)(ti_gemm_prepare() ? hipErrorUnknown : hipSuccess));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  printf("TI_GEMV_EXP=%d\n", TI_GEMV_EXP);
  for (int M : {8, 16, 32}) {
    for (auto& sh : shapes) {
      const size_t tb = (size_t)sh.K * sh.N / 2, sb = (size_t)sh.K / 128 * sh.N * 2, per = (tb + sb + 4095) & ~(size_t)4095;
      const int nbuf = (int)(big / per);
      ti_epilogue ep{};
      ep.kind = TI_EPI_STORE_F32;
      ep.ldo = sh.N;
      ep.out = y;
      hipGraph_t g;
      hipGraphExec_t ge;
      CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
      for (int r = 0; r < reps; ++r) {
        char* base = (char*)wbuf + (size_t)(r % nbuf) * per;
        if (ti_gemm_wq_a16(base, (const uint16_t*)(base + tb), 4, x, TI_X_F16, sh.K, nullptr, 1e-5f, M, sh.N, sh.K, &ep, s))
          return 1;
      }
      CK(hipStreamEndCapture(s, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      CK(hipGraphLaunch(ge, s));
      CK(hipStreamSynchronize(s));
      CK(hipEventRecord(e0, s));
      CK(hipGraphLaunch(ge, s));
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double us = ms * 1e3 / reps;
      int ntl = 0;
      const int grid = ti::mb_grid(M > 16 ? 2 : 1, sh.N, sh.K, 256, &ntl);
      printf("M=%2d %-8s K=%5d N=%5d grid %4d ntl %d: %7.2f us  weights %6.0f GB/s  x %6.0f GB/s (L2)\n", M, sh.name,
             sh.K, sh.N, grid, ntl, us, (tb + sb) / us / 1e3, (double)grid * M * sh.K * 2 / us / 1e3);
      CK(hipGraphExecDestroy(ge));
      CK(hipGraphDestroy(g));
    }
  }
  return 0;
}
