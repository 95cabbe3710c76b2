// probe_persist.hip -- decode-layer chain as graph launches vs ONE persistent launch whose phases
// stream weights exactly as gemv_wq_kernel does (every wave its own register ring of 1 KiB items),
// with the all-to-all edges done in-kernel (diagnostic only, not part of the product).
//
//   hipcc -std=c++20 -O3 --offload-arch=gfx950 tools/probe_persist.hip -o /tmp/probe_persist && /tmp/probe_persist
//
// Phases per layer (bytes of the Llama-2-7B INT4 layer): QKV 26 MB, attention 33.6, O 8.66, gate/up
// 46.5, down 23.3; x of each phase = the previous phase's output vector (fp16 words: 4096 / 4096 /
// 4096 / 4096 / 11008).  Each workgroup (512 threads, one per CU) stages x in LDS, streams its items
// (xor-folded into the accumulator against x: no dequant, no MFMA), sums the 8 waves and publishes 16
// floats.  Modes:
//   0  one launch per phase, captured into a hipGraph (today's engine structure)
//   1  one persistent launch; edge = sc1 output stores, the storing wave's vmcnt(0), one agent atomic
//      add per workgroup on its shard (blockIdx & 7) of an 8-way counter; lane 0 of the polling wave
//      sums the 8 shards (sc1 loads, s_sleep between polls); the next phase's ring is issued BEFORE the
//      wait by every wave but the poller
//   2  as 1, ring issued after x is staged (the edge alone, no prefetch)
//   3  as 1 with one unsharded counter
//   4  as 1, every wave prefetches (the poller too: its poll waits behind its own ring)
//   5  as 1, and before the wait every wave but the poller also DMAs the first kPF items of its
//      next phase into LDS (global_load_lds_dwordx4 nt, 1 KiB each), consumed from LDS after the edge
//   6  as 5 with half as many items in LDS
//   7  as 1, x loaded and staged by the poller wave alone, right after its poll (before its own ring)
//   8  as 7 with the LDS prefetch of 5
// Every spin is bounded (abort flag).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#define CK(x)                                                                           \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                          \
    }                                                                                   \
  } while (0)

constexpr int kThreads = 512, kR = 5, kPh = 5, kXMax = 5504;   // x words (u32) max
struct Chain {
  const u32x4* w[kPh];
  int ipw[kPh];      // items (1 KiB) per wave
  int xw[kPh];       // x words (fp16 pairs) of the phase
  size_t layer_bytes;
};

__device__ __forceinline__ int rsrc_flags() { return 0x00020000; }
__device__ __forceinline__ unsigned ld_sc1_u32(const unsigned* p, int off) {
  return __builtin_amdgcn_raw_buffer_load_b32(
      __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned*>(p), 0, 0x7fffffff, rsrc_flags()), off * 4, 0, 16);
}
__device__ __forceinline__ u32x4 ld_sc1_b128(const unsigned* p, int off16) {
  return __builtin_amdgcn_raw_buffer_load_b128(
      __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned*>(p), 0, 0x7fffffff, rsrc_flags()), off16 * 16, 0, 16);
}
__device__ __forceinline__ void st_sc1_u32(unsigned* p, int off, unsigned v) {
  __builtin_amdgcn_raw_buffer_store_b32(v, __builtin_amdgcn_make_buffer_rsrc(p, 0, 0x7fffffff, rsrc_flags()), off * 4, 0, 16);
}
// 64 lanes x 16 B -> LDS at the wave-uniform byte address lds (hidden from the waitcnt pass)
__device__ __forceinline__ void dma_1k_asm(const void* src_lane, uint32_t lds) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src_lane), "s"(lds)
               : "memory");
}
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// One phase's body after x is staged: stream items j of this wave (ring already issued for j < kR).
__device__ __forceinline__ float stream_phase(const u32x4* p, int ipw, u32x4 (&ring)[kR], const unsigned* xs, int xw,
                                              int j0 = 0, const u32x4* pf = nullptr) {
  float acc = 0.0f;
  for (int j = 0; j < j0; ++j) {   // the items prefetched into LDS (this wave's region)
    const u32x4 v = pf[j * 64];
    acc = fmaf(__builtin_bit_cast(float, (v[0] ^ v[1] ^ v[2] ^ v[3]) & 0x3fffffffu), __builtin_bit_cast(float, xs[j % xw] & 0x3fffffffu), acc);
  }
  p += (size_t)j0 * 64;
  ipw -= j0;
  int j = 0;
  for (; j + kR <= ipw; j += kR) {
#pragma unroll
    for (int s = 0; s < kR; ++s) {
      const u32x4 v = ring[s];
      acc = fmaf(__builtin_bit_cast(float, (v[0] ^ v[1] ^ v[2] ^ v[3]) & 0x3fffffffu), __builtin_bit_cast(float, xs[(j + s) % xw] & 0x3fffffffu), acc);
      const int nj = j + s + kR;
      ring[s] = __builtin_nontemporal_load(p + (nj < ipw ? nj : ipw - 1) * 64);
    }
  }
#pragma unroll
  for (int s = 0; s < kR; ++s)
    if (j + s < ipw) acc += __builtin_bit_cast(float, ring[s][0] & 0x3fffffffu);
  return acc;
}

__device__ __forceinline__ void issue_ring(const u32x4* p, int ipw, u32x4 (&ring)[kR]) {
#pragma unroll
  for (int s = 0; s < kR; ++s) ring[s] = __builtin_nontemporal_load(p + (s < ipw ? s : ipw - 1) * 64);
}

// ---- mode 0: one launch per phase
__global__ __launch_bounds__(kThreads, 1) void phase_kernel(const u32x4* w, int ipw, int xw, const unsigned* xin,
                                                            unsigned* xout) {
  __shared__ __attribute__((aligned(16))) unsigned xs[kXMax];
  __shared__ float red[8];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  unsigned xr[11];
#pragma unroll
  for (int q = 0; q < 11; ++q) xr[q] = xin[(tid + q * kThreads) % xw];
  const u32x4* p = w + ((size_t)(blockIdx.x * 8 + wave) * ipw) * 64 + lane;
  u32x4 ring[kR];
  issue_ring(p, ipw, ring);
#pragma unroll
  for (int q = 0; q < 11; ++q)
    if (tid + q * kThreads < xw) xs[tid + q * kThreads] = xr[q];
  lds_barrier();
  float acc = stream_phase(p, ipw, ring, xs, xw);
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  if (lane == 0) red[wave] = acc;
  __syncthreads();
  if (tid < 16) {
    float s = 0.f;
    for (int q = 0; q < 8; ++q) s += red[q];
    xout[(blockIdx.x * 16 + tid) % kXMax] = __builtin_bit_cast(unsigned, s * 1e-30f);
  }
}

// ---- modes 1-4: one persistent launch
constexpr int kPF = 12;
template <int MODE>
__global__ __launch_bounds__(kThreads, 1) void persist_kernel(Chain c, int layers, unsigned* xbuf, unsigned* ctr,
                                                              unsigned* abort_flag, unsigned long long* ts) {
  __shared__ __attribute__((aligned(16))) unsigned xs[kXMax];
  __shared__ __attribute__((aligned(16))) u32x4 pfl[MODE >= 5 ? 8 * kPF * 64 : 1];   // [wave][item][lane]
  __shared__ float red[8];
  __shared__ unsigned dead;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int G = gridDim.x;
  constexpr int kPollWave = 0;
  const bool prefetch = MODE == 1 || MODE == 3 || MODE == 4 || MODE >= 5;
  const int npf_max = MODE == 5 || MODE == 8 ? kPF : MODE == 6 ? kPF / 2 : 0;
  constexpr bool kX0 = MODE >= 7;   // x staged by the poller wave alone, before its own ring
  const bool self_pf = MODE == 4 || wave != kPollWave;
  if (tid == 0) dead = 0;
  if (tid == 0 && blockIdx.x == 0) ts[0] = __builtin_amdgcn_s_memrealtime();
  __syncthreads();
  u32x4 ring[kR];
  int n = 0;   // phase index within the launch
  for (int l = 0; l < layers; ++l) {
    for (int ph = 0; ph < kPh; ++ph, ++n) {
      const int ipw = c.ipw[ph], xw = c.xw[ph];
      const u32x4* p = c.w[ph] + (size_t)l * (c.layer_bytes / 16) + ((size_t)(blockIdx.x * 8 + wave) * ipw) * 64 + lane;
      // items of this phase taken from LDS (prefetched by DMA before the edge), then the ring
      const int npf = self_pf && npf_max > 0 ? (ipw - kR < npf_max ? (ipw - kR > 0 ? ipw - kR : 0) : npf_max) : 0;
      if (npf > 0) {
        const uint32_t base = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(pfl + wave * kPF * 64));
        for (int j = 0; j < npf; ++j) dma_1k_asm(p + j * 64, base + j * 1024);
      }
      if (prefetch && self_pf) issue_ring(p + npf * 64, ipw - npf, ring);
      if (n > 0) {   // edge n-1: every workgroup published phase n-1
        if (wave == kPollWave && lane == 0 && !dead) {
          const unsigned target = (unsigned)G * n;
          unsigned k = 0;
          while (true) {
            unsigned s = 0;
            if (MODE == 3) {
              s = ld_sc1_u32(ctr, 0);
            } else {
#pragma unroll
              for (int q = 0; q < 8; ++q) s += ld_sc1_u32(ctr, q * 32);
            }
            if (s >= target) break;
            __builtin_amdgcn_s_sleep(1);
            if ((++k & 255) == 0 && ld_sc1_u32(abort_flag, 0)) { dead = 1; break; }
            if (k > (1u << 18)) { atomicOr(abort_flag, 1u); dead = 1; break; }
          }
        }
        lds_barrier();
      }
      const unsigned* xin = xbuf + (n & 1) * kXMax;
      if (kX0) {
        if (wave == kPollWave) {
          u32x4 xq[22];
#pragma unroll
          for (int q = 0; q < 22; ++q) xq[q] = ld_sc1_b128(xin, (lane + q * 64) % (xw >> 2));
          if (prefetch) issue_ring(p, ipw, ring);
#pragma unroll
          for (int q = 0; q < 22; ++q)
            if (lane + q * 64 < (xw >> 2)) *(u32x4*)(xs + 4 * (lane + q * 64)) = xq[q];
        }
      } else {
        if (prefetch && !self_pf) issue_ring(p, ipw, ring);
        unsigned xr[11];
#pragma unroll
        for (int q = 0; q < 11; ++q) xr[q] = ld_sc1_u32(xin, (tid + q * kThreads) % xw);
        if (!prefetch) issue_ring(p, ipw, ring);
#pragma unroll
        for (int q = 0; q < 11; ++q)
          if (tid + q * kThreads < xw) xs[tid + q * kThreads] = xr[q];
      }
      if (npf_max > 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the asm DMA (invisible to hipcc)
      lds_barrier();
      float acc = stream_phase(p, ipw, ring, xs, xw, npf, pfl + wave * kPF * 64 + lane);
      for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
      if (lane == 0) red[wave] = acc;
      lds_barrier();
      if (wave == 0) {
        if (tid < 16) {
          float s = 0.f;
          for (int q = 0; q < 8; ++q) s += red[q];
          st_sc1_u32(xbuf + ((n + 1) & 1) * kXMax, (blockIdx.x * 16 + tid) % kXMax, __builtin_bit_cast(unsigned, s * 1e-30f));
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) {
          const int shard = MODE == 3 ? 0 : (blockIdx.x & 7) * 32;
          __hip_atomic_fetch_add(ctr + shard, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
  }
  if (tid == 0) atomicMax(ts + 1, __builtin_amdgcn_s_memrealtime());
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
    c.ipw[k] = (int)(mb[k] * 1e6 / (G * 8 * 1024.0) + 0.5);
    c.xw[k] = xw[k];
    off[k] = per_layer;
    per_layer += (size_t)c.ipw[k] * G * 8 * 1024;
  }
  c.layer_bytes = per_layer;
  const size_t total = per_layer * layers;
  char* w;
  CK(hipMalloc(&w, total));
  CK(hipMemset(w, 0x11, total));
  for (int k = 0; k < kPh; ++k) c.w[k] = (const u32x4*)(w + off[k]);
  unsigned *xbuf, *ctr, *abort_flag;
  unsigned long long* ts;
  CK(hipMalloc(&xbuf, 2 * kXMax * 4));
  CK(hipMemset(xbuf, 0, 2 * kXMax * 4));
  CK(hipMalloc(&ctr, 256 * 4));
  CK(hipMalloc(&abort_flag, 4));
  CK(hipMemset(abort_flag, 0, 4));
  CK(hipMalloc(&ts, 16));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  printf("CUs %d, layers %d, %.1f MB per layer, items/wave %d %d %d %d %d\n", G, layers, per_layer / 1e6, c.ipw[0], c.ipw[1],
         c.ipw[2], c.ipw[3], c.ipw[4]);
  // mode 0: graph of launches
  {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int l = 0; l < layers; ++l)
      for (int k = 0; k < kPh; ++k) {
        const int n = l * kPh + k;
        hipLaunchKernelGGL(phase_kernel, dim3(G), dim3(kThreads), 0, s, (const u32x4*)(w + l * per_layer + off[k]), c.ipw[k],
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
    printf("mode 0 (graph of %d launches): %.1f us, %.2f us per layer\n", layers * kPh, best * 1e3, best * 1e3 / layers);
  }
  for (int mode : {1, 7, 8}) {
    float best = 1e30f, span_best = 1e30f;
    for (int r = 0; r < 8; ++r) {
      CK(hipMemsetAsync(ctr, 0, 256 * 4, s));
      CK(hipMemsetAsync(ts, 0, 16, s));
      float ms;
      CK(hipEventRecord(e0, s));
      if (mode == 1) hipLaunchKernelGGL(persist_kernel<1>, dim3(G), dim3(kThreads), 0, s, c, layers, xbuf, ctr, abort_flag, ts);
      if (mode == 2) hipLaunchKernelGGL(persist_kernel<2>, dim3(G), dim3(kThreads), 0, s, c, layers, xbuf, ctr, abort_flag, ts);
      if (mode == 3) hipLaunchKernelGGL(persist_kernel<3>, dim3(G), dim3(kThreads), 0, s, c, layers, xbuf, ctr, abort_flag, ts);
      if (mode == 4) hipLaunchKernelGGL(persist_kernel<4>, dim3(G), dim3(kThreads), 0, s, c, layers, xbuf, ctr, abort_flag, ts);
      if (mode == 5) hipLaunchKernelGGL(persist_kernel<5>, dim3(G), dim3(kThreads), 0, s, c, layers, xbuf, ctr, abort_flag, ts);
      if (mode == 7) hipLaunchKernelGGL(persist_kernel<7>, dim3(G), dim3(kThreads), 0, s, c, layers, xbuf, ctr, abort_flag, ts);
      if (mode == 8) hipLaunchKernelGGL(persist_kernel<8>, dim3(G), dim3(kThreads), 0, s, c, layers, xbuf, ctr, abort_flag, ts);
      if (mode == 6) hipLaunchKernelGGL(persist_kernel<6>, dim3(G), dim3(kThreads), 0, s, c, layers, xbuf, ctr, abort_flag, ts);
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      unsigned long long h[2];
      CK(hipMemcpy(h, ts, 16, hipMemcpyDeviceToHost));
      unsigned ab = 0;
      CK(hipMemcpy(&ab, abort_flag, 4, hipMemcpyDeviceToHost));
      if (ab) {
        printf("mode %d: ABORTED (bounded spin expired)\n", mode);
        return 1;
      }
      const float span = (h[1] - h[0]) * 0.01f;
      if (r > 0 && ms < best) best = ms;
      if (r > 0 && span < span_best) span_best = span;
    }
    printf("mode %d (persistent): %.1f us (in-kernel %.1f), %.2f us per layer\n", mode, best * 1e3, span_best,
           span_best / layers);
  }
  return 0;
}
