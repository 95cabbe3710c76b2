// probe_gemv.hip -- per-launch timing of ti_gemm_wq_a16 on the Llama-2-7B INT4 decode shapes,
// replayed from a hipGraph (GPU box, diagnostic only; not part of the product).
//
//   for e in 0 1 4 5 8 16 12 20; do hipcc -std=c++20 -O3 -Iinclude -Iturboinfer_amd/csrc/kernels --offload-arch=gfx950 \
//     -DTI_GEMV_EXP=$e tools/probe_gemv.hip -o tools/probe_gemv_e$e; done
//
// The kernel source is compiled into this TU with TI_GEMV_EXP:
//   0 product kernel, 1 stream only (no dequant/MFMA), +4 per-workgroup phase timestamps,
//   +8 no x / scale dependency (constants), +16 non-temporal weight loads.
// Weights are random bytes (timing does not depend on values); x is fp16 or f32+rmsnorm.
#include <hip/hip_runtime.h>
#include <algorithm>
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
  const int reps = argc > 1 ? atoi(argv[1]) : 64;
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  struct Shape { const char* name; int K, N; } shapes[] = {
      {"qkv", 4096, 12288}, {"o", 4096, 4096}, {"gate_up", 4096, 22016}, {"down", 11008, 4096}, {"lm_head", 4096, 32000}};
  const size_t big = 1ull << 30;
  void* wbuf;
  CK(hipMalloc(&wbuf, big));
  CK(hipMemset(wbuf, 0x5a, big));
  void *x, *y, *nw;
  CK(hipMalloc(&x, 16 * 11008 * 4));
  CK(hipMemset(x, 0, 16 * 11008 * 4));
  CK(hipMalloc(&y, 16 * 32000 * 4));
  CK(hipMalloc(&nw, 11008 * 4));
  CK(hipMemset(nw, 0, 11008 * 4));
  CK((hipError_t)(ti_gemm_prepare() ? hipErrorUnknown : hipSuccess));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  printf("TI_GEMV_EXP=%d\n", TI_GEMV_EXP);
  for (auto& sh : shapes) {
    const size_t tb = (size_t)sh.K * sh.N / 2, sb = (size_t)sh.K / 128 * sh.N * 2, per = (tb + sb + 4095) & ~(size_t)4095;
    const int nbuf = getenv("PROBE_HOT") ? 1 : (int)(big / per);   // PROBE_HOT: same weights every launch (Infinity-Cache hot)
    for (int xk : {TI_X_F16, TI_X_F32_RMSNORM}) {
      ti_epilogue ep{};
      ep.kind = TI_EPI_STORE_F32;
      ep.ldo = sh.N;
      ep.out = y;
      hipGraph_t g;
      hipGraphExec_t ge;
      CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
      for (int r = 0; r < reps; ++r) {
        char* base = (char*)wbuf + (size_t)(r % nbuf) * per;
        if (ti_gemm_wq_a16(base, (const uint16_t*)(base + tb), 4, x, xk, sh.K, (const float*)nw, 1e-5f, 1, sh.N, sh.K,
                           &ep, s))
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
      printf("%-8s K=%5d N=%5d x=%s %7.2f us %6.0f GB/s\n", sh.name, sh.K, sh.N, xk == TI_X_F16 ? "f16 " : "norm", us,
             (tb + sb) / us / 1e3);
      CK(hipGraphExecDestroy(ge));
      CK(hipGraphDestroy(g));
#if TI_GEMV_EXP & 4
      // one more launch on cold weights, then the per-workgroup phase timestamps
      {
        char* base = (char*)wbuf + (size_t)((reps + 1) % nbuf) * per;
        if (ti_gemm_wq_a16(base, (const uint16_t*)(base + tb), 4, x, xk, sh.K, (const float*)nw, 1e-5f, 1, sh.N, sh.K,
                           &ep, s))
          return 1;
        CK(hipStreamSynchronize(s));
        static unsigned long long ts[4096 * 8];
        CK(hipMemcpyFromSymbol(ts, HIP_SYMBOL(ti::g_gemv_ts), sizeof(ts)));
        const int grid = ti::gemv_grid(1, sh.N, sh.K, 256);
        unsigned long long t0 = ~0ull, tend = 0;
        double ph[4][3];
        for (int k = 0; k < 4; ++k) ph[k][0] = 1e30, ph[k][1] = 0, ph[k][2] = 0;
        for (int b = 0; b < grid; ++b) {
          t0 = ts[b * 8] < t0 ? ts[b * 8] : t0;
          tend = ts[b * 8 + 4] > tend ? ts[b * 8 + 4] : tend;
        }
        double start[3] = {1e30, 0, 0};
        for (int b = 0; b < grid; ++b) {
          const double st = (ts[b * 8] - t0) * 0.01;
          start[0] = st < start[0] ? st : start[0];
          start[1] += st / grid;
          start[2] = st > start[2] ? st : start[2];
          for (int k = 0; k < 4; ++k) {
            const double d = (double)(ts[b * 8 + k + 1] - ts[b * 8 + k]) * 0.01;   // us
            ph[k][0] = d < ph[k][0] ? d : ph[k][0];
            ph[k][1] += d / grid;
            ph[k][2] = d > ph[k][2] ? d : ph[k][2];
          }
        }
        static unsigned long long wts[4096 * 8];
        CK(hipMemcpyFromSymbol(wts, HIP_SYMBOL(ti::g_gemv_wts), sizeof(wts)));
        double skew = 0, w0late = 0, post = 0;
        for (int b = 0; b < grid; ++b) {
          unsigned long long lo = ~0ull, hi = 0;
          for (int w = 0; w < 8; ++w) {
            lo = wts[b * 8 + w] < lo ? wts[b * 8 + w] : lo;
            hi = wts[b * 8 + w] > hi ? wts[b * 8 + w] : hi;
          }
          skew += (hi - lo) * 0.01 / grid;
          w0late += (wts[b * 8] - lo) * 0.01 / grid;
          post += (double)(ts[b * 8 + 4] - ts[b * 8 + 5]) * 0.01 / grid;
        }
        printf("   waves: end skew %.2f us, wave0 after first %.2f us | barrier->end %.2f us\n", skew, w0late, post);
        {   // workgroup end times after the first start: how unbalanced the grid finishes
          static double ends[4096];
          for (int b = 0; b < grid; ++b) ends[b] = (ts[b * 8 + 4] - t0) * 0.01;
          std::sort(ends, ends + grid);
          printf("   workgroup end (us after first start): min %.2f p10 %.2f p50 %.2f p90 %.2f max %.2f\n", ends[0],
                 ends[grid / 10], ends[grid / 2], ends[grid * 9 / 10], ends[grid - 1]);
        }
        printf("   span %.2f us | start skew avg %.2f max %.2f | issue %.2f/%.2f/%.2f | stage %.2f/%.2f/%.2f | "
               "stream %.2f/%.2f/%.2f | epi %.2f/%.2f/%.2f (min/avg/max)\n",
               (tend - t0) * 0.01, start[1], start[2], ph[0][0], ph[0][1], ph[0][2], ph[1][0], ph[1][1], ph[1][2],
               ph[2][0], ph[2][1], ph[2][2], ph[3][0], ph[3][1], ph[3][2]);
      }
#endif
    }
  }
  return 0;
}
