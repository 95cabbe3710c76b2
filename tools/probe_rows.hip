// probe_rows.hip -- per-wave phase timestamps of the batched-rows GEMM (gemm_rows_kernel,
// TI_X_F16_PACKED) on the Llama-2-7B shapes at 32 / 64 rows, cold weights, GPU box, diagnostic:
//   hipcc -std=c++20 -O3 -Iinclude -Iturboinfer_amd/csrc/kernels --offload-arch=gfx950 \
//     -mllvm -amdgpu-kernarg-preload-count=16 -DTI_GEMV_EXP=4 tools/probe_rows.hip -o tools/probe_rows
// Phases (s_memrealtime, 100 MHz, relative to the earliest wave start of the launch):
// 0 start, 1 scales in LDS, 2 first item computed, 3 stream done, 4 loads drained, 5 epilogue done.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

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

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  struct Shape { const char* name; int K, N; } shapes[] = {
      {"qkv", 4096, 12288}, {"o", 4096, 4096}, {"gate_up", 4096, 22016}, {"down", 11008, 4096}};
  const size_t big = 1ull << 30;
  void* wbuf;
  CK(hipMalloc(&wbuf, big));
  CK(hipMemset(wbuf, 0x11, big));
  void *x, *y;
  CK(hipMalloc(&x, 64 * 11008 * 2));
  CK(hipMemset(x, 0, 64 * 11008 * 2));
  CK(hipMalloc(&y, 64 * 32000 * 4));
  if (ti_gemm_prepare()) return 1;
  static unsigned long long ts[4096 * 8 * 8];
  for (int M : {32, 64}) {
    for (auto& sh : shapes) {
      const size_t tb = (size_t)sh.K * sh.N / 2, sb = (size_t)sh.K / 128 * sh.N * 2, per = (tb + sb + 4095) & ~(size_t)4095;
      const int nbuf = (int)(big / per);
      ti_epilogue ep{};
      ep.kind = TI_EPI_STORE_F32;
      ep.ldo = sh.N;
      ep.out = y;
      for (int r = 0; r < 8; ++r) {   // warm up, rotating weights; the last launch is measured
        char* base = (char*)wbuf + (size_t)(r % nbuf) * per;
        if (ti_gemm_wq_a16(base, (const uint16_t*)(base + tb), 4, x, TI_X_F16_PACKED, sh.K, nullptr, 1e-5f, M, sh.N,
                           sh.K, &ep, s))
          return 1;
      }
      CK(hipStreamSynchronize(s));
      CK(hipMemcpyFromSymbol(ts, HIP_SYMBOL(ti::g_rows_ts), sizeof(ts)));
      int MB = 0, RG = 0, ntl = 0;
      ti::rows_on();
      ti::rows_shape(M, &MB, &RG);
      const int grid = ti::rows_grid(MB, sh.N, sh.K, 256, &ntl);
      unsigned long long t0 = ~0ull;
      for (int g = 0; g < grid; ++g)
        for (int w = 0; w < 8; ++w) t0 = std::min(t0, ts[(g * 8 + w) * 8 + 0]);
      double avg[6] = {0}, mx[6] = {0};
      for (int g = 0; g < grid; ++g)
        for (int w = 0; w < 8; ++w)
          for (int k = 0; k < 6; ++k) {
            const double v = (ts[(g * 8 + w) * 8 + k] - t0) * 0.01;   // us
            avg[k] += v / (grid * 8);
            mx[k] = std::max(mx[k], v);
          }
      printf("M=%2d %-8s grid %3d ntl %d MB %d RG %d | avg", M, sh.name, grid, ntl, MB, RG);
      for (int k = 0; k < 6; ++k) printf(" %6.2f", avg[k]);
      printf(" | max");
      for (int k = 0; k < 6; ++k) printf(" %6.2f", mx[k]);
      printf("\n");
    }
  }
  return 0;
}
