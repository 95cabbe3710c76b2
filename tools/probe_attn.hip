// probe_attn.hip -- per-launch timing of ti_attn_decode (split-K decode attention) on the
// Llama-2-7B / Llama-3-8B decode shapes, replayed from a hipGraph with the KV cache rotating
// through 1 GiB (cold, as in a real decode step).  Diagnostic only; not part of the product.
//
//   hipcc -std=c++20 -O3 -Iinclude -Iturboinfer_amd/csrc/kernels --offload-arch=gfx950 \
//     tools/probe_attn.hip -o tools/probe_attn && tools/probe_attn
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>

#include "../turboinfer_amd/csrc/kernels/attention.hip"

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
  const size_t big = 1ull << 30;
  void* kvbuf;
  CK(hipMalloc(&kvbuf, big));
  CK(hipMemset(kvbuf, 0x11, big));
  float *q, *ws;
  uint16_t* out;
  int32_t* pos;
  CK(hipMalloc(&q, 64 * 128 * 4));
  CK(hipMemset(q, 0, 64 * 128 * 4));
  CK(hipMalloc(&out, 64 * 128 * 2));
  CK(hipMalloc(&ws, 64 << 20));
  CK(hipMemset(ws, 0, 64 << 20));
  CK(hipMalloc(&pos, 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  struct Shape { const char* name; int heads, kv, hd, L; } shapes[] = {
      {"llama2-7b", 32, 32, 128, 2048}, {"llama3-8b", 32, 8, 128, 2048}, {"tinyllama", 32, 4, 64, 2048}};
  for (auto& sh : shapes) {
    const int max_seq = sh.L;
    const size_t kv_bytes = (size_t)sh.kv * max_seq * sh.hd * 2;   // one of K or V
    const size_t per = 2 * kv_bytes;
    const int nbuf = (int)(big / per);
    const int p = sh.L - 1;
    CK(hipMemcpy(pos, &p, 4, hipMemcpyHostToDevice));
    for (int splits : {4, 8, 16, 22, 32, 64}) {
      hipGraph_t g;
      hipGraphExec_t ge;
      CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
      for (int r = 0; r < reps; ++r) {
        const uint16_t* kc = (const uint16_t*)((char*)kvbuf + (size_t)(r % nbuf) * per);
        if (ti_attn_decode(q, kc, kc + kv_bytes / 2, (int64_t)sh.kv * max_seq * sh.hd, max_seq, pos, 1, sh.heads, sh.kv,
                           sh.hd, splits, ws, out, s))
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
      printf("%-14s heads %2d kv %2d L %5d splits %3d (%5d WGs): %7.2f us %6.0f GB/s\n", sh.name, sh.heads, sh.kv, sh.L,
             splits, splits * sh.kv, us, 2.0 * kv_bytes * sh.L / max_seq / us / 1e3);
      CK(hipGraphExecDestroy(ge));
      CK(hipGraphDestroy(g));
#if TI_ATTN_EXP & 4
      {   // one more launch, then per-workgroup phases: 0 start, 1 stream done, 2 merged, 3 ticket, 4 end (last)
        const uint16_t* kc = (const uint16_t*)kvbuf;
        if (ti_attn_decode(q, kc, kc + kv_bytes / 2, (int64_t)sh.kv * max_seq * sh.hd, max_seq, pos, 1, sh.heads,
                           sh.kv, sh.hd, splits, ws, out, s))
          return 1;
        CK(hipStreamSynchronize(s));
        static unsigned long long ts[4096 * 8];
        CK(hipMemcpyFromSymbol(ts, HIP_SYMBOL(ti::g_attn_ts), sizeof(ts)));
        const int nwg = splits * sh.kv;
        unsigned long long t0 = ~0ull, tend = 0;
        double ph[3] = {0, 0, 0}, last_tail = 0;
        int nlast = 0;
        for (int b = 0; b < nwg; ++b) t0 = ts[b * 8] < t0 ? ts[b * 8] : t0;
        for (int b = 0; b < nwg; ++b) {
          for (int k = 0; k < 3; ++k) ph[k] += (double)(ts[b * 8 + k + 1] - ts[b * 8 + k]) * 0.01 / nwg;
          if (ts[b * 8 + 4] > ts[b * 8 + 3] && ts[b * 8 + 4] - ts[b * 8 + 3] < 100000) {
            last_tail += (double)(ts[b * 8 + 4] - ts[b * 8 + 3]) * 0.01;
            ++nlast;
            tend = ts[b * 8 + 4] > tend ? ts[b * 8 + 4] : tend;
          }
        }
        printf("   span %.2f us | stream %.2f | wave merge %.2f | publish+ticket %.2f | last-arriver merge %.2f (avg)\n",
               (tend - t0) * 0.01, ph[0], ph[1], ph[2], nlast ? last_tail / nlast : 0.0);
      }
#endif
    }
  }
  return 0;
}
