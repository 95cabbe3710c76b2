// probe_overlap.hip -- can dependent decode launches overlap?  (GPU box, diagnostic only.)
//
//   hipcc -std=c++20 -O3 --offload-arch=gfx950 tools/probe_overlap.hip -o tools/probe_overlap && tools/probe_overlap
//
// A chain of weight-streaming launches shaped like one Llama-2-7B INT4 decode layer
// (QKV 26 MB, attention 34 MB, O 8.7 MB, gate/up 46.5 MB, down 23.3 MB) x 32.  Each launch:
// 256 workgroups x 8 waves; every wave keeps R 1-KiB items of its weight slice in flight
// (nt dwordx4 loads into registers), consumes them against a small input vector and
// publishes 16 floats per workgroup.  Modes:
//   0  one stream, plain dependent launches (today's engine structure)
//   1  two streams, launches alternate; launch i waits IN-KERNEL for launch i-1 (after its
//      weight ring is issued): producer sc1 stores + vmcnt(0) + one agent atomic add per
//      workgroup, consumer polls the counter with sc1 loads, then reads the input with sc1 loads
//   2  one stream, hipExtAnyOrderLaunch + the same in-kernel waits
//   3  mode 1 captured into a hipGraph (fork/join only at the ends)
//   4  mode 2 captured into a hipGraph
//   5  mode 2 with the weight ring issued after the wait (the boundary overlap alone)
// Every spin is bounded (abort flag, reported).
#include <hip/hip_ext.h>
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

#ifndef POLL_SLEEP
#define POLL_SLEEP 1   // s_sleep immediate between polls (x 64 clocks)
#endif
constexpr int kWG = 256, kThreads = 512, kR = 5, kVec = 4096;

__device__ __forceinline__ int ld_sc1_i32(const unsigned* p) {
  return __builtin_amdgcn_raw_buffer_load_b32(
      __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned*>(p), 0, 0x7fffffff, 0x00020000), 0, 0, 16);
}
__device__ __forceinline__ float ld_sc1_f32(const float* p, int off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                       __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), 0, 0x7fffffff, 0x00020000),
                                       off * 4, 0, 16));
}
__device__ __forceinline__ void st_sc1_f32(float* p, int off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v),
                                        __builtin_amdgcn_make_buffer_rsrc(p, 0, 0x7fffffff, 0x00020000), off * 4, 0, 16);
}

__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4, 4)))
void link_kernel(const u32x4* w, int ipw, const float* xin, float* xout, unsigned* ctr, int idx, int wait,
                 unsigned* abort_flag, unsigned long long* ts, unsigned long long* ts2) {
  __shared__ float red[8];
  __shared__ float xs[kVec];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) {
    const unsigned long long t = __builtin_amdgcn_s_memrealtime();
    atomicMin(ts + 2 * idx, t);
    atomicMax(ts2 + 4 * idx + 0, t);   // last workgroup start
  }
  // this wave's slice: items j = 0..ipw-1, 1 KiB each, contiguous per wave
  const u32x4* p = w + ((size_t)(blockIdx.x * 8 + wave) * ipw) * 64 + lane;
  u32x4 ring[kR];
  if (wait != 2) {
#pragma unroll
    for (int s = 0; s < kR; ++s) ring[s] = __builtin_nontemporal_load(p + (s < ipw ? s : ipw - 1) * 64);
  }
  if (wait && idx > 0) {
    if (tid == 0) {
      int n = 0;
      while (ld_sc1_i32(ctr + idx - 1) < kWG) {
        __builtin_amdgcn_s_sleep(POLL_SLEEP);
        if (++n > (1 << 22)) { atomicOr(abort_flag, 1u); break; }
      }
    }
    __syncthreads();
  }
  if (wait == 2) {   // ring issued only after the dependency (what the overlap alone buys)
#pragma unroll
    for (int s = 0; s < kR; ++s) ring[s] = __builtin_nontemporal_load(p + (s < ipw ? s : ipw - 1) * 64);
  }
  // the input vector (the previous launch's output): sc1 loads
  for (int i = tid; i < kVec; i += kThreads) xs[i] = wait ? ld_sc1_f32(xin, i) : xin[i];
  __syncthreads();
  float acc = xs[(tid * 7) & (kVec - 1)];
  int j = 0;
  for (; j + kR <= ipw; j += kR) {
#pragma unroll
    for (int s = 0; s < kR; ++s) {
      const u32x4 v = ring[s];
      acc += __builtin_bit_cast(float, (v[0] ^ v[1] ^ v[2] ^ v[3]) & 0x3fffffffu) * xs[(j + s) & (kVec - 1)];
      const int nj = j + s + kR;
      ring[s] = __builtin_nontemporal_load(p + (nj < ipw ? nj : ipw - 1) * 64);
    }
  }
#pragma unroll
  for (int s = 0; s < kR; ++s)
    if (j + s < ipw) acc += __builtin_bit_cast(float, ring[s][0] & 0x3fffffffu);
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  if (lane == 0) red[wave] = acc;
  __syncthreads();
  if (tid < 16) {
    float s = 0.f;
    for (int q = 0; q < 8; ++q) s += red[q];
    const int o = (blockIdx.x * 16 + tid) & (kVec - 1);
    if (wait) st_sc1_f32(xout, o, s * 1e-30f + (float)idx); else xout[o] = s * 1e-30f + (float)idx;
  }
  if (wait) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) __hip_atomic_fetch_add(ctr + idx, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (tid == 0) {
    const unsigned long long t = __builtin_amdgcn_s_memrealtime();
    atomicMax(ts + 2 * idx + 1, t);
    atomicMin(ts2 + 4 * idx + 1, t);   // first workgroup end
  }
}

int main(int argc, char** argv) {
  const int layers = argc > 1 ? atoi(argv[1]) : 32;
  const double mb[5] = {26.0, 33.6, 8.66, 46.5, 23.3};
  const int n = layers * 5;
  int ipw[5];
  for (int k = 0; k < 5; ++k) ipw[k] = (int)(mb[k] * 1e6 / (kWG * 8 * 1024.0) + 0.5);
  size_t per_layer = 0;
  for (int k = 0; k < 5; ++k) per_layer += (size_t)ipw[k] * kWG * 8 * 1024;
  const size_t total = per_layer * layers;
  char* w;
  CK(hipMalloc(&w, total));
  CK(hipMemset(w, 0x11, total));
  float* vec;
  CK(hipMalloc(&vec, 2 * kVec * 4));
  CK(hipMemset(vec, 0, 2 * kVec * 4));
  unsigned* ctr;
  CK(hipMalloc(&ctr, 64 * n * 4));
  unsigned *abort_flag;
  CK(hipMalloc(&abort_flag, 4));
  unsigned long long* ts;
  CK(hipMalloc(&ts, 2 * n * 8));
  unsigned long long* ts2;
  CK(hipMalloc(&ts2, 4 * n * 8));
  hipStream_t s[2];
  CK(hipStreamCreateWithFlags(&s[0], hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s[1], hipStreamNonBlocking));
  hipEvent_t e0, e1, fork, join;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
  printf("layers %d, %d launches, %.1f MB per layer, items/wave %d %d %d %d %d\n", layers, n, per_layer / 1e6, ipw[0],
         ipw[1], ipw[2], ipw[3], ipw[4]);

  auto enqueue = [&](int mode, int round) {
    size_t off = 0;
    for (int i = 0; i < n; ++i) {
      const int k = i % 5;
      const u32x4* wp = (const u32x4*)(w + off);
      off += (size_t)ipw[k] * kWG * 8 * 1024;
      const float* xin = vec + (i & 1) * kVec;
      float* xout = vec + ((i + 1) & 1) * kVec;
      unsigned* c = ctr + (size_t)round * n;
      const int wait = mode == 0 ? 0 : mode == 5 ? 2 : 1;
      hipStream_t st = mode == 1 || mode == 3 ? s[i & 1] : s[0];
      void* args[] = {(void*)&wp, (void*)&ipw[k], (void*)&xin, (void*)&xout, (void*)&c, (void*)&i, (void*)&wait,
                      (void*)&abort_flag, (void*)&ts, (void*)&ts2};
      CK(hipExtLaunchKernel((const void*)link_kernel, dim3(kWG), dim3(kThreads), args, 0, st, nullptr, nullptr,
                            mode == 2 || mode >= 4 ? hipExtAnyOrderLaunch : 0));
    }
  };
  for (int mode : {0, 1, 2, 3}) {
    double best = 1e30;
    for (int round = 0; round < 6; ++round) {
      CK(hipMemset(ctr, 0, 64 * n * 4));
      CK(hipMemset(abort_flag, 0, 4));
      CK(hipMemset(ts, 0xff, 2 * n * 8));
      for (int i = 0; i < n; ++i) CK(hipMemset(ts + 2 * i + 1, 0, 8));
      CK(hipMemset(ts2, 0, 4 * n * 8));
      for (int i = 0; i < n; ++i) CK(hipMemset(ts2 + 4 * i + 1, 0xff, 8));
      CK(hipDeviceSynchronize());
      float ms = 0;
      if (mode == 3 || mode == 4) {
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s[0], hipStreamCaptureModeThreadLocal));
        CK(hipEventRecord(fork, s[0]));
        CK(hipStreamWaitEvent(s[1], fork, 0));
        enqueue(mode == 3 ? 1 : 2, 0);
        CK(hipEventRecord(join, s[1]));
        CK(hipStreamWaitEvent(s[0], join, 0));
        CK(hipStreamEndCapture(s[0], &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        CK(hipEventRecord(e0, s[0]));
        CK(hipGraphLaunch(ge, s[0]));
        CK(hipEventRecord(e1, s[0]));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
      } else {
        CK(hipEventRecord(e0, s[0]));
        CK(hipEventRecord(fork, s[0]));
        CK(hipStreamWaitEvent(s[1], fork, 0));
        enqueue(mode, 0);
        CK(hipEventRecord(join, s[1]));
        CK(hipStreamWaitEvent(s[0], join, 0));
        CK(hipEventRecord(e1, s[0]));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
      }
      unsigned ab = 0;
      CK(hipMemcpy(&ab, abort_flag, 4, hipMemcpyDeviceToHost));
      std::vector<unsigned long long> h(2 * n);
      CK(hipMemcpy(h.data(), ts, 2 * n * 8, hipMemcpyDeviceToHost));
      double span = (h[2 * n - 1] - h[0]) * 0.01, overl = 0;
      int nov = 0;
      for (int i = 1; i < n; ++i) {
        const double d = ((double)h[2 * i] - (double)h[2 * (i - 1) + 1]) * 0.01;   // start(i) - end(i-1)
        overl += d;
        nov += d < 0;
      }
      if (round > 0 && span < best) best = span;
      if (round == 5) {
        std::vector<unsigned long long> h2(4 * n);
        CK(hipMemcpy(h2.data(), ts2, 4 * n * 8, hipMemcpyDeviceToHost));
        for (int i = 20; i < 26; ++i)   // relative to kernel i-1's first start (us)
          printf("   k%d: prev [first start 0, last start %.2f, first end %.2f, last end %.2f] this [first start %.2f, last start %.2f]\n",
                 i, (h2[4 * (i - 1)] - h[2 * (i - 1)]) * 0.01, (h2[4 * (i - 1) + 1] - h[2 * (i - 1)]) * 0.01,
                 (h[2 * (i - 1) + 1] - h[2 * (i - 1)]) * 0.01, ((double)h[2 * i] - (double)h[2 * (i - 1)]) * 0.01,
                 ((double)h2[4 * i] - (double)h[2 * (i - 1)]) * 0.01);
      }
      if (round == 5)
        printf("mode %d: events %.1f us, device span %.1f us (best %.1f), %.2f us per layer, start(i)-end(i-1) avg %.2f us, "
               "%d of %d starts before predecessor end, abort %u\n",
               mode, ms * 1e3, span, best, best / layers, overl / (n - 1), nov, n - 1, ab);
    }
  }
  return 0;
}
