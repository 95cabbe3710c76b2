// probe_tile.hip -- where a tile-GEMM wave's cycles go, by loop phase (GPU box, diagnostic only;
// not part of the product).  The kernel source is compiled into this TU with TI_GEMV_EXP=16384,
// which stamps s_memtime around each step of the asm pipeline's group loop (x wait, barrier,
// issue, weight wait, compute) and the epilogue, accumulated per wave.
//
//   hipcc -std=c++20 -O3 -Iinclude -Iturboinfer_amd/csrc/kernels --offload-arch=gfx950 -ffp-contract=off \
//     -DTI_GEMV_EXP=16384 tools/probe_tile.hip -o tools/probe_tile
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

int main() {
  // kind: the epilogue the prefill runs (QKV: RoPE + KV append; gate/up: SiLU * up to fp16;
  // O / down: residual add), or plain fp32 stores
  struct Shape { const char* name; int M, K, N, kind; } shapes[] = {
      {"qkv", 512, 4096, 12288, TI_EPI_STORE_F32},   {"qkv", 512, 4096, 12288, TI_EPI_QKV_ROPE_KV},
      {"gate_up", 512, 4096, 22016, TI_EPI_STORE_F32}, {"gate_up", 512, 4096, 22016, TI_EPI_SILU_MUL_F16},
      {"down", 512, 11008, 4096, TI_EPI_STORE_F32},  {"down", 512, 11008, 4096, TI_EPI_RESID_F32},
      {"o", 512, 4096, 4096, TI_EPI_RESID_F32},      {"qkv", 256, 4096, 12288, TI_EPI_QKV_ROPE_KV}};
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const size_t wbytes = 64ull << 20;
  void *w, *x, *y;
  CK(hipMalloc(&w, wbytes));
  CK(hipMemset(w, 0x5a, wbytes));                 // int4 nibbles 5 / 10, fp16 scales 0x5a5a (finite)
  CK(hipMalloc(&x, 1024 * 11008 * 2));
  CK(hipMemset(x, 0x11, 1024 * 11008 * 2));       // fp16 0x1111 (finite, small)
  CK(hipMalloc(&y, 1024 * 32000 * 4));
  CK((hipError_t)(ti_gemm_prepare() ? hipErrorUnknown : hipSuccess));
  const int hd = 128, max_seq = 2048;
  int32_t* pos;
  float* cs;
  uint16_t *kc, *vc;
  CK(hipMalloc(&pos, 1024 * 4));
  CK(hipMalloc(&cs, (size_t)max_seq * hd * 4));
  CK(hipMemset(cs, 0, (size_t)max_seq * hd * 4));
  CK(hipMalloc(&kc, (size_t)32 * max_seq * hd * 2));
  CK(hipMalloc(&vc, (size_t)32 * max_seq * hd * 2));
  {
    static int32_t ph[1024];
    for (int i = 0; i < 1024; ++i) ph[i] = i;
    CK(hipMemcpy(pos, ph, sizeof(ph), hipMemcpyHostToDevice));
  }
  static unsigned long long cy[4096 * 8 * 8];
  for (auto& sh : shapes) {
    const size_t tb = (size_t)sh.K * sh.N / 2;
    ti_epilogue ep{};
    ep.kind = sh.kind;
    ep.ldo = sh.kind == TI_EPI_QKV_ROPE_KV ? sh.N / 3 : sh.kind == TI_EPI_SILU_MUL_F16 ? sh.N / 2 : sh.N;
    ep.out = y;
    if (sh.kind == TI_EPI_QKV_ROPE_KV) {
      ep.q_dim = ep.kv_dim = sh.N / 3;
      ep.head_dim = hd;
      ep.max_seq = max_seq;
      ep.pos = pos;
      ep.rope_cs = cs;
      ep.k_cache = kc;
      ep.v_cache = vc;
      ep.kv_stream_stride = 0;
    }
    for (int r = 0; r < 4; ++r)   // warm, then the stamped launch is the last one
      if (ti_gemm_wq_a16(w, (const uint16_t*)((char*)w + tb), 4, x, TI_X_F16, sh.K, nullptr, 1e-5f, sh.M, sh.N, sh.K,
                         &ep, s))
        return 1;
    CK(hipStreamSynchronize(s));
    CK(hipMemcpyFromSymbol(cy, HIP_SYMBOL(ti::g_tile_cy), sizeof(cy)));
    int wmr = 0, tpw = 0, ks = 0;
    ti::tile_plan(sh.M, sh.N, sh.K, false, 256, 0, &wmr, &tpw, &ks);
    const int cols = (8 / wmr) * tpw, n_cb = ((sh.N >> 4) + cols - 1) / cols, n_rb = (sh.M + 64 * wmr - 1) / (64 * wmr);
    const int grid = (n_cb + 7) / 8 * 8 * n_rb;
    double tot[6] = {0, 0, 0, 0, 0, 0};
    int n = 0;
    for (int b = 0; b < grid; ++b) {
      const int cb = (b >> 3) / n_rb * 8 + (b & 7);
      if (cb >= n_cb) continue;
      for (int wv = 0; wv < 8; ++wv, ++n)
        for (int i = 0; i < 6; ++i) tot[i] += (double)cy[((size_t)b * 8 + wv) * 8 + i];
    }
    const int groups = sh.K / 128 + 3;
    double all = 0;
    for (int i = 0; i < 6; ++i) all += tot[i];
    printf("%-8s epi %d M=%4d K=%5d N=%5d wmr%d tpw%d: %d waves, cycles per wave %.0f (per group %.0f):", sh.name, sh.kind,
           sh.M, sh.K, sh.N, wmr, tpw, n, all / n, (all - tot[5]) / n / groups);
    const char* nm[6] = {"x-wait", "barrier", "issue", "w-wait", "compute", "epilogue"};
    for (int i = 0; i < 6; ++i) printf(" %s %.1f%%", nm[i], 100.0 * tot[i] / all);
    printf("\n");
  }
  return 0;
}
