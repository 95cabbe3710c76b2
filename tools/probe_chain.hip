// probe_chain.hip -- can a persistent launch beat one launch per GEMV on a chain of
// weight-streaming stages with all-to-all edges?  (GPU box, diagnostic only.)
//
//   hipcc -std=c++20 -O3 --offload-arch=gfx950 tools/probe_chain.hip -o tools/probe_chain && tools/probe_chain
//
// One workgroup per CU: 8 stream waves + 1 edge wave.  Each stream wave owns a private LDS
// ring of D 1-KiB slots filled by LDS-DMA (global_load_lds_dwordx4, nt) and runs ahead across
// stage boundaries: the next stage's weights do not depend on data.  Per stage a wave
// consumes its items against x (LDS), writes its partial, and the last wave of the
// workgroup folds the partials into the workgroup's 16 outputs.  The edge wave publishes
// them (sc1 stores, vmcnt(0) of its own, agent atomic add to the stage's counter), polls the
// counter with sc1 loads, gathers the whole 4096-float vector with sc1 loads into the
// other x buffer and raises an LDS flag.  Every spin is bounded (abort flag).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
#define CK(x)                                                                               \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess) {                                                                 \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));     \
      exit(1);                                                                              \
    }                                                                                       \
  } while (0)

constexpr int kN = 4096;          // edge vector (floats)
constexpr int kSpin = 1 << 22;    // poll bound

__device__ __forceinline__ int lds_load_acquire(const int* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_store_release(int* p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ u32x4 ld_sc1(const void* base, int byte_off) {
  return __builtin_amdgcn_raw_buffer_load_b128(__builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000),
                                              byte_off, 0, 16);
}
__device__ __forceinline__ void st_sc1_f32(float* p, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v),
                                        __builtin_amdgcn_make_buffer_rsrc(p, 0, 0x7fffffff, 0x00020000), 0, 0, 16);
}

__device__ __forceinline__ void dma16(const u32x4* g, u32x4* l) {   // LDS-DMA, 1 KiB per wave, nt
  __builtin_amdgcn_global_load_lds(g, l, 16, 0, 2);
}
__device__ __forceinline__ int ld_sc1_i32(const int* p) {
  return __builtin_amdgcn_raw_buffer_load_b32(__builtin_amdgcn_make_buffer_rsrc(const_cast<int*>(p), 0, 0x7fffffff, 0x00020000), 0, 0, 16);
}

template <int D>
__global__ __launch_bounds__(576, 1) void chain_kernel(const u32x4* w, int stages, int ipw, float* vec,
                                                       int* counters, int* abort_flag, float* out,
                                                       unsigned long long* ts) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  u32x4* ring = (u32x4*)smem;                                   // [8][D][64]
  float* xb = (float*)(smem + 8 * D * 1024);                    // [2][kN]
  float* slab = xb + 2 * kN;                                    // [2][8][16]
  int* flags = (int*)(slab + 2 * 8 * 16);                       // done[2], outready, xready, abort
  float* out16 = (float*)(flags + 8);                           // [16]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int G = gridDim.x, b = blockIdx.x;
  if (tid < 8) flags[tid] = 0;
  for (int i = tid; i < kN; i += 576) xb[i] = 1.0f;
  __syncthreads();
  unsigned long long t0 = __builtin_amdgcn_s_memrealtime();

  if (wave == 8) {   // ---------------- edge wave
    for (int s = 0; s < stages; ++s) {
      int spins = 0;
      while (lds_load_acquire(flags + 2) < s + 1) {          // outputs of stage s folded
        if (++spins > kSpin) { atomicExch(abort_flag, 1); lds_store_release(flags + 4, 1); return; }
        __builtin_amdgcn_s_sleep(1);
      }
      float* dst = vec + (size_t)((s + 1) & 1) * kN;
      if (lane < 16) st_sc1_f32(dst + b * 16 + lane, out16[lane]);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) __hip_atomic_fetch_add(counters + s, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (s + 1 == stages) break;
      spins = 0;
      for (;;) {
        int c = 0;
        if (lane == 0) c = ld_sc1_i32(counters + s);
        c = __builtin_amdgcn_readfirstlane(c);
        if (c >= G) break;
        if (++spins > kSpin || *(volatile int*)abort_flag) { atomicExch(abort_flag, 1); lds_store_release(flags + 4, 1); return; }
        __builtin_amdgcn_s_sleep(1);
      }
      u32x4 g[kN / 256];
#pragma unroll
      for (int i = 0; i < kN / 256; ++i) g[i] = ld_sc1(dst, (i * 64 + lane) * 16);
      float* xd = xb + ((s + 1) & 1) * kN;
#pragma unroll
      for (int i = 0; i < kN / 256; ++i) *(u32x4*)(xd + (i * 64 + lane) * 4) = g[i];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      lds_store_release(flags + 3, s + 1);                     // x of stage s+1 ready
    }
    if (lane == 0) ts[b] = __builtin_amdgcn_s_memrealtime() - t0;
    return;
  }

  // ---------------- stream waves: item (stage s, i) of wave w of workgroup b
  auto src = [&](int j) -> const u32x4* {
    const int s = j / ipw, i = j - s * ipw;
    return w + (((size_t)s * G + b) * ipw + i) * 8 * 64 + wave * 64 + lane;
  };
  const int total = stages * ipw;
  u32x4* myring = ring + wave * D * 64;
#pragma unroll
  for (int d = 0; d < D; ++d) dma16(src(d < total ? d : total - 1), myring + d * 64);
  float acc = 0.0f;
  int j = 0;
  for (int s = 0; s < stages; ++s) {
    if (s > 0) {
      int spins = 0;
      while (lds_load_acquire(flags + 3) < s) {
        if (++spins > kSpin || lds_load_acquire(flags + 4)) { atomicExch(abort_flag, 1); return; }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    const float* x = xb + (s & 1) * kN;
    for (int i = 0; i < ipw; ++i, ++j) {
      const int slot = j % D;
      asm volatile("s_waitcnt vmcnt(%0)" :: "n"(D - 1) : "memory");
      const u32x4 v = myring[slot * 64 + lane];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      const int jn = j + D < total ? j + D : total - 1;
      dma16(src(jn), myring + slot * 64);
      acc = fmaf((float)(v[0] & 0xffu) + (float)(v[3] >> 24), x[(lane * 64 + i) & (kN - 1)], acc);
    }
    // partial of this wave for stage s; the last wave folds the workgroup's 16 outputs
    float* sl = slab + (s & 1) * 128;
    float p = acc;
    for (int o = 16; o < 64; o <<= 1) p += __shfl_xor(p, o, 64);
    if (lane < 16) sl[wave * 16 + lane] = p;
    acc = 0.0f;
    int last = 0;
    if (lane == 0) last = __hip_atomic_fetch_add(flags + (s & 1), 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP) == 8 * (s / 2 + 1) - 1;
    last = __builtin_amdgcn_readfirstlane(last);
    if (last) {
      if (lane < 16) {
        float v = 0.0f;
        for (int w2 = 0; w2 < 8; ++w2) v += sl[w2 * 16 + lane];
        out16[lane] = v * 1e-6f;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      lds_store_release(flags + 2, s + 1);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (acc == 12345.0f) out[0] = acc;
}

struct Ctx { hipStream_t st; u32x4* w; float *vec, *out; int *counters, *abort_flag; unsigned long long* ts; hipEvent_t e0, e1; };
template <int D>
static void run(const Ctx& c, int stages, int ipw) {
  const int G = 256;
  const int lds = 8 * D * 1024 + 2 * kN * 4 + 2 * 8 * 16 * 4 + 8 * 4 + 16 * 4;
  CK(hipFuncSetAttribute((const void*)chain_kernel<D>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  double best = 1e30;
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipMemsetAsync(c.counters, 0, 4096 * 4, c.st));
    CK(hipEventRecord(c.e0, c.st));
    hipLaunchKernelGGL(chain_kernel<D>, dim3(G), dim3(576), lds, c.st, c.w, stages, ipw, c.vec, c.counters, c.abort_flag, c.out, c.ts);
    CK(hipEventRecord(c.e1, c.st));
    CK(hipEventSynchronize(c.e1));
    float ms;
    CK(hipEventElapsedTime(&ms, c.e0, c.e1));
    int ab = 0;
    CK(hipMemcpy(&ab, c.abort_flag, 4, hipMemcpyDeviceToHost));
    if (ab) { printf("ABORTED (D %d stages %d ipw %d)\n", D, stages, ipw); exit(1); }
    best = ms * 1e3 < best ? ms * 1e3 : best;
  }
  const double mb = (double)G * 8 * ipw * 1024 / 1e6;
  printf("D %2d stages %3d x %6.2f MB: %8.2f us total, %6.2f us/stage, %6.0f GB/s\n", D, stages, mb, best,
         best / stages, mb * stages / best * 1e3);
}

int main(int argc, char** argv) {
  const int G = 256;
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  const size_t big = 3ull << 30;
  u32x4* w;
  CK(hipMalloc(&w, big));
  CK(hipMemset(w, 1, big));
  float *vec, *out;
  int *counters, *abort_flag;
  unsigned long long* ts;
  CK(hipMalloc(&vec, 2 * kN * 4));
  CK(hipMemset(vec, 0, 2 * kN * 4));
  CK(hipMalloc(&counters, 4096 * 4));
  CK(hipMalloc(&abort_flag, 4));
  CK(hipMemset(abort_flag, 0, 4));
  CK(hipMalloc(&out, 64));
  CK(hipMalloc(&ts, 8 * G));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  Ctx c{st, w, vec, out, counters, abort_flag, ts, e0, e1};
  for (int ipw : {0, 4, 13, 23}) {
    const int stages = ipw ? (int)(big / ((size_t)G * 8 * ipw * 1024)) - 1 : 128;
    const int S = stages > 128 ? 128 : stages;
    if (ipw == 0) { run<8>(c, S, 1); continue; }
    run<8>(c, S, ipw);
    run<12>(c, S, ipw);
  }
  return 0;
}
