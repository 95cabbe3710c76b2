// probe_engine.hip -- MI355X_MICROARCH.md `engine-vs-launches` (1 loader + 3 consumer waves per CU,
// nt LDS-DMA weight ring, 8-byte {data, tag} granule hand-offs gathered by one consumer wave that also
// publishes) on the bytes of the Llama-2-7B INT4 decode layer, against a graph of per-phase launches
// doing the same work (diagnostic only, not part of the product).
//
//   hipcc -std=c++20 -O3 --offload-arch=gfx950 -Iinclude -Iturboinfer_amd/csrc/kernels tools/probe_engine.hip \
//     -o /tmp/probe_engine && /tmp/probe_engine [layers] [thin]
//
// Phases per layer (QKV 26 MB, attention 33.6, O 8.66, gate/up 46.5, down 23.3), each CU its share of
// 1 KiB items; every item gets the product GEMV's int4 math (4 x (dequant + v_mfma_f32_16x16x32_f16) on
// x fragments read from LDS, one FMA per result) so the consumers pay what the real kernel's waves pay.
// x of each phase = the previous phase's outputs of all CUs (2048 words; 5504 for down).
//   graph:  one launch per phase (512 threads, every wave a 5-item register ring of nt loads: the
//           product's streaming shape), x staged from global, 16 outputs published per workgroup
//   engine: ONE launch, 256 threads per CU: wave 0 the loader (8 x 16 KiB LDS slots, 16 nt LDS-DMA
//           per fill, 3 fills in flight, a FULL word per slot published behind its vmcnt, a slot reused
//           once the 3 consumers counted it free), waves 1-3 the consumers (item i of a fill to consumer
//           i % 3); consumer 1 also reduces the phase, publishes the CU's slice of its output as 8-byte
//           sc1 granules {value, epoch} and gathers the next x (16-load sc1 passes, tag checks) into LDS;
//           with `thin` the loader keeps one fill in flight while its CU gathers.  Every spin is bounded.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "dequant.hpp"

using namespace ti;

#define CK(x)                                                                           \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                          \
    }                                                                                   \
  } while (0)

constexpr int kPh = 5, kXMax = 5504, kS = 8, kFill = 16, kD = 3, kConsMax = 7;
struct Chain {
  const u32x4* w[kPh];
  int items[kPh];   // 1 KiB items per CU
  int xw[kPh];      // x words (fp16 pairs) of the phase
  size_t layer_u4;  // u32x4 per layer
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ uint64_t ld_sc1_b64(const uint64_t* p, int i) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b64(rsrc(p), i * 8, 0, 16);
  return __builtin_bit_cast(uint64_t, v);
}
__device__ __forceinline__ void st_sc1_b64(uint64_t* p, int i, uint64_t v) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, v), rsrc(p),
                                        i * 8, 0, 16);
}
// 64 lanes x 16 B -> LDS at the wave-uniform byte address lds (hidden from the waitcnt pass)
__device__ __forceinline__ void dma_1k(const void* src_lane, uint32_t lds) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src_lane), "s"(lds)
               : "memory");
}

// the product's int4 item: 4 x (dequant + MFMA) against x fragments of k-tile kt, one FMA per result
__device__ __forceinline__ void item_math(const u32x4 w, const uint16_t* xs16, int kt, f32x4& acc, uint32_t magic) {
  const int lane = threadIdx.x & 63, kq = lane >> 4, r = lane & 15;
  f32x4 t = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int s4 = 0; s4 < 4; ++s4) {
    const f16x8 bf = deq_int4_raw(w[s4], magic);
    const f16x8 af = *(const f16x8*)(xs16 + (kt & 31) * 128 + kq * 32 + s4 * 8 + 0 * r);
    t = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, bf, t, 0, 0, 0);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i] = fmaf(0.5f, acc[i], t[i]);
}

// ---------------------------------------------------------------- graph: one launch per phase
constexpr int kR = 5;
__global__ __launch_bounds__(512, 1) void phase_kernel(const u32x4* w, int items, int xw, const unsigned* xin,
                                                       unsigned* xout) {
  __shared__ __attribute__((aligned(16))) unsigned xs[kXMax];
  __shared__ float red[8];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  unsigned xr[11];
#pragma unroll
  for (int q = 0; q < 11; ++q) xr[q] = xin[(tid + q * 512) % xw];
  const int ipw = items / 8;
  const u32x4* p = w + ((size_t)blockIdx.x * items + (size_t)wave * ipw) * 64 + lane;
  u32x4 ring[kR];
#pragma unroll
  for (int s = 0; s < kR; ++s) ring[s] = __builtin_nontemporal_load(p + (s < ipw ? s : ipw - 1) * 64);
#pragma unroll
  for (int q = 0; q < 11; ++q)
    if (tid + q * 512 < xw) xs[tid + q * 512] = xr[q];
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  uint32_t magic;
  asm volatile("v_mov_b32 %0, 0x64006400" : "=v"(magic));
  f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
  const uint16_t* xs16 = (const uint16_t*)xs;
  int j = 0;
  for (; j + kR <= ipw; j += kR) {
#pragma unroll
    for (int s = 0; s < kR; ++s) {
      item_math(ring[s], xs16, j + s, acc, magic);
      const int nj = j + s + kR;
      ring[s] = __builtin_nontemporal_load(p + (nj < ipw ? nj : ipw - 1) * 64);
    }
  }
#pragma unroll
  for (int s = 0; s < kR; ++s)
    if (j + s < ipw) item_math(ring[s], xs16, j + s, acc, magic);
  float a = acc[0] + acc[1] + acc[2] + acc[3];
  for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o);
  if (lane == 0) red[wave] = a;
  __syncthreads();
  if (tid < 16) {
    float s = 0.f;
    for (int q = 0; q < 8; ++q) s += red[q];
    xout[(blockIdx.x * 16 + tid) % kXMax] = __builtin_bit_cast(unsigned, s * 1e-30f);
  }
}

// ---------------------------------------------------------------- engine: one persistent launch
struct EngLds {
  u32x4 ring[kS][kFill][64];   // 128 KiB
  unsigned xs[kXMax];
  unsigned full[kS], freec[kS], xs_ready, arrive, dead, gathering;
  float red[kConsMax];
};

__device__ __forceinline__ unsigned lds_ld(const unsigned& x) {
  return __hip_atomic_load(&x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// MODE bit 1: no gathers (consumers never wait for x: the ring and the math alone); bit 2: no math
// (consumers only wait for a fill and release it: the loader ring alone).  kCons consumer waves.
template <bool THIN, int kCons, int MODE>
__global__ __launch_bounds__(64 * (kCons + 1), 1) void engine_kernel(Chain c, int layers, uint64_t* gran, unsigned* abort_flag,
                                                        unsigned long long* ts) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  EngLds& L = *(EngLds*)smem;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int G = gridDim.x, cu = blockIdx.x;
  if (tid < kS) {
    L.full[tid] = 0;
    L.freec[tid] = 0;
  }
  if (tid == 0) {
    L.xs_ready = 0;
    L.arrive = 0;
    L.dead = 0;
    L.gathering = 0;
    if (cu == 0) ts[0] = __builtin_amdgcn_s_memrealtime();
  }
  for (int i = tid; i < kXMax; i += 64 * (kCons + 1)) L.xs[i] = 0;
  __syncthreads();   // (the only workgroup barrier: roles never meet at one again)
  constexpr unsigned kSpin = 1u << 22;
  if (wave == 0) {
    // ---- loader
    const uint32_t ring0 = (uint32_t)(uintptr_t)&L.ring[0][0][0];
    unsigned f = 0;   // fills issued
    auto publish = [&](unsigned upto) {   // fills [.., upto) have landed
      if (lane == 0)
        for (unsigned g = upto > kD + 1 ? upto - kD - 1 : 0; g < upto; ++g) __hip_atomic_store(&L.full[g % kS], g + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    for (int l = 0; l < layers && !lds_ld(L.dead); ++l)
      for (int k = 0; k < kPh; ++k) {
        const int items = c.items[k], F = (items + kFill - 1) / kFill;
        const u32x4* base = c.w[k] + (size_t)l * c.layer_u4 + (size_t)cu * items * 64 + lane;
        for (int fi = 0; fi < F; ++fi, ++f) {
          const unsigned slot = f % kS;
          if (f >= kS) {   // the slot's previous fill released by the 3 consumers
            const unsigned need = kCons * (f / kS);
            unsigned n = 0;
            while (__hip_atomic_load(&L.freec[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < need) {
              __builtin_amdgcn_s_sleep(1);
              if (++n > kSpin || lds_ld(L.dead)) { L.dead = 1; break; }
            }
          }
          const uint32_t dst = __builtin_amdgcn_readfirstlane(ring0 + slot * kFill * 1024);
#pragma unroll
          for (int i = 0; i < kFill; ++i) {
            const int it = fi * kFill + i < items ? fi * kFill + i : items - 1;
            dma_1k(base + (size_t)it * 64, dst + i * 1024);
          }
          // keep kD fills in flight (one while this CU gathers, THIN): publish what landed
          if (THIN && lds_ld(L.gathering)) {
            asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
            publish(f);
          } else if (f + 1 > kD) {
            asm volatile("s_waitcnt vmcnt(32)" ::: "memory");   // 16 x (kD - 1): fill f - 2 landed
            publish(f - 1);
          }
        }
      }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    publish(f);
  } else {
    // ---- consumers
    const int cn = wave - 1;
    uint32_t magic;
    asm volatile("v_mov_b32 %0, 0x64006400" : "=v"(magic));
    const uint16_t* xs16 = (const uint16_t*)L.xs;
    f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
    unsigned f = 0;
    int n = 0;
    for (int l = 0; l < layers; ++l)
      for (int k = 0; k < kPh; ++k, ++n) {
        if (n > 0 && !(MODE & 1)) {   // edge: x of phase n = the outputs of phase n - 1 (epoch n) of every CU
          if (cn == 0) {
            if (lane == 0) __hip_atomic_store(&L.gathering, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            const uint64_t* g = gran + ((n - 1) & 1) * kXMax;
            const int xw = c.xw[k];
            for (int b = 0; b < xw; b += 64 * 16) {   // passes of 16 sc1 loads per lane
              uint64_t v[16];
#pragma unroll
              for (int q = 0; q < 16; ++q) v[q] = ld_sc1_b64(g, b + q * 64 + lane < xw ? b + q * 64 + lane : 0);
#pragma unroll
              for (int q = 0; q < 16; ++q) {
                const int idx = b + q * 64 + lane;
                unsigned sp = 0;
                while (idx < xw && (unsigned)(v[q] >> 32) != (unsigned)n && !lds_ld(L.dead)) {
                  __builtin_amdgcn_s_sleep(1);
                  v[q] = ld_sc1_b64(g, idx);
                  if (++sp > kSpin) L.dead = 1;
                }
                if (idx < xw) L.xs[idx] = (unsigned)v[q];
              }
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (lane == 0) __hip_atomic_store(&L.gathering, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (lane == 0) __hip_atomic_store(&L.xs_ready, (unsigned)n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          } else {
            unsigned sp = 0;
            while (lds_ld(L.xs_ready) < (unsigned)n && !lds_ld(L.dead)) {
              __builtin_amdgcn_s_sleep(1);
              if (++sp > kSpin) L.dead = 1;
            }
          }
        }
        const int items = c.items[k], F = (items + kFill - 1) / kFill;
        for (int fi = 0; fi < F; ++fi, ++f) {
          const unsigned slot = f % kS;
          unsigned sp = 0;
          while (lds_ld(L.full[slot]) < f + 1 && !lds_ld(L.dead)) {
            __builtin_amdgcn_s_sleep(1);
            if (++sp > kSpin) L.dead = 1;
          }
          if (!(MODE & 2))
            for (int i = cn; i < kFill; i += kCons)
              if (fi * kFill + i < items) item_math(L.ring[slot][i][lane], xs16, fi * kFill + i, acc, magic);
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          if (lane == 0) __hip_atomic_fetch_add(&L.freec[slot], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        // phase end: the 3 consumers' sums, published by consumer 0 as granules of epoch n + 1
        float a = acc[0] + acc[1] + acc[2] + acc[3];
        for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o);
        if (MODE & 1) continue;
        if (lane == 0) {
          L.red[cn] = a;
          __hip_atomic_fetch_add(&L.arrive, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        if (cn == 0) {
          unsigned sp = 0;
          while (lds_ld(L.arrive) < (unsigned)(kCons * (n + 1)) && !lds_ld(L.dead)) {
            __builtin_amdgcn_s_sleep(1);
            if (++sp > kSpin) L.dead = 1;
          }
          float s = 0.0f;
          for (int q = 0; q < kCons; ++q) s += L.red[q];
          const int xw_next = c.xw[(k + 1) % kPh], per = (xw_next + G - 1) / G;
          uint64_t* g = gran + (n & 1) * kXMax;
          for (int j = lane; j < per; j += 64) {
            const int idx = cu * per + j;
            if (idx < xw_next)
              st_sc1_b64(g, idx, ((uint64_t)(unsigned)(n + 1) << 32) | __builtin_bit_cast(unsigned, s * 1e-30f + (float)j));
          }
        }
      }
  }
  if (lds_ld(L.dead) && lane == 0) atomicOr(abort_flag, 1u);
  if (lane == 0) atomicMax(ts + 1, __builtin_amdgcn_s_memrealtime());   // every wave: the last one's end
}

int main(int argc, char** argv) {
  const int layers = argc > 1 ? atoi(argv[1]) : 32;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int G = prop.multiProcessorCount;
  const double mb[kPh] = {26.0, 33.6, 8.66, 46.5, 23.3};
  const int xw[kPh] = {2048, 2048, 2048, 2048, 5504};
  Chain c;
  size_t per_layer = 0, off[kPh];
  for (int k = 0; k < kPh; ++k) {
    c.items[k] = 8 * (int)(mb[k] * 1e6 / (G * 8 * 1024.0) + 0.5);
    c.xw[k] = xw[k];
    off[k] = per_layer;
    per_layer += (size_t)c.items[k] * G * 1024;
  }
  c.layer_u4 = per_layer / 16;
  const size_t total = per_layer * layers;
  char* w;
  CK(hipMalloc(&w, total));
  CK(hipMemset(w, 0x11, total));
  for (int k = 0; k < kPh; ++k) c.w[k] = (const u32x4*)(w + off[k]);
  unsigned *xbuf, *abort_flag;
  uint64_t* gran;
  unsigned long long* ts;
  CK(hipMalloc(&xbuf, 2 * kXMax * 4));
  CK(hipMemset(xbuf, 0, 2 * kXMax * 4));
  CK(hipMalloc(&gran, 2 * kXMax * 8));
  CK(hipMalloc(&abort_flag, 4));
  CK(hipMemset(abort_flag, 0, 4));
  CK(hipMalloc(&ts, 16));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  printf("CUs %d, layers %d, %.1f MB per layer, items per CU %d %d %d %d %d, LDS %zu B\n", G, layers, per_layer / 1e6,
         c.items[0], c.items[1], c.items[2], c.items[3], c.items[4], sizeof(EngLds));
  {   // graph of launches
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int l = 0; l < layers; ++l)
      for (int k = 0; k < kPh; ++k) {
        const int n = l * kPh + k;
        hipLaunchKernelGGL(phase_kernel, dim3(G), dim3(512), 0, s, (const u32x4*)(w + l * per_layer + off[k]), c.items[k],
                           c.xw[k], xbuf + (n & 1) * kXMax, xbuf + ((n + 1) & 1) * kXMax);
      }
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    float best = 1e30f;
    for (int r = 0; r < 8; ++r) {
      float ms;
      CK(hipEventRecord(e0, s));
      CK(hipGraphLaunch(ge, s));
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (r > 0 && ms < best) best = ms;
    }
    printf("graph (%d launches): %.1f us, %.2f us per layer\n", layers * kPh, best * 1e3, best * 1e3 / layers);
  }
  auto run = [&](const void* fn, int threads, const char* what) -> int {
    CK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, sizeof(EngLds)));
    float best = 1e30f, span_best = 1e30f;
    for (int r = 0; r < 4; ++r) {
      CK(hipMemsetAsync(gran, 0, 2 * kXMax * 8, s));
      CK(hipMemsetAsync(ts, 0, 16, s));
      float ms;
      CK(hipEventRecord(e0, s));
      void* args[] = {&c, (void*)&layers, &gran, &abort_flag, &ts};
      CK(hipLaunchKernel(fn, dim3(G), dim3(threads), args, sizeof(EngLds), s));
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      unsigned long long h[2];
      CK(hipMemcpy(h, ts, 16, hipMemcpyDeviceToHost));
      unsigned ab = 0;
      CK(hipMemcpy(&ab, abort_flag, 4, hipMemcpyDeviceToHost));
      if (ab) {
        printf("engine %s: ABORTED (bounded spin expired)\n", what);
        return 1;
      }
      const float span = (h[1] - h[0]) * 0.01f;
      if (r > 0 && ms < best) best = ms;
      if (r > 0 && span < span_best) span_best = span;
    }
    printf("engine %-44s %8.1f us (in-kernel %8.1f), %6.2f us per layer\n", what, best * 1e3, span_best, span_best / layers);
    return 0;
  };
  int rc = 0;
  rc |= run((const void*)engine_kernel<false, 3, 0>, 256, "1 loader + 3 consumers");
  rc |= run((const void*)engine_kernel<true, 3, 0>, 256, "1 loader + 3 consumers, thinned loader");
  rc |= run((const void*)engine_kernel<false, 3, 1>, 256, "1 + 3, no gathers (ring + math)");
  rc |= run((const void*)engine_kernel<false, 3, 3>, 256, "1 + 3, no gathers, no math (ring alone)");
  rc |= run((const void*)engine_kernel<false, 7, 0>, 512, "1 loader + 7 consumers");
  rc |= run((const void*)engine_kernel<false, 7, 1>, 512, "1 + 7, no gathers (ring + math)");
  return rc;
}
