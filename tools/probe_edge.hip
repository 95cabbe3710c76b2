// probe_edge.hip -- cost of an all-to-all "granule" edge inside one persistent launch
// (diagnostic only, not part of the product).
//
//   hipcc -std=c++20 -O3 --offload-arch=gfx950 tools/probe_edge.hip -o tools/probe_edge && tools/probe_edge
//
// G workgroups (one per CU, 512 threads) run `rounds` rounds of: publish this WG's slice of an
// N-float vector as 8-byte {value, tag} granules (sc1 stores, no fence, no drain), then read
// the WHOLE vector back with sc1 loads until every tag equals the round's tag (two buffers,
// alternating by round).  Optionally a
// weight stream runs beside it (each wave keeps 16 KiB of loads in flight), as in a decode
// stage.  Every spin is bounded: a timeout sets a flag and the kernel exits.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

#define CK(x)                                                                               \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess) {                                                                 \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));     \
      exit(1);                                                                              \
    }                                                                                       \
  } while (0)

__device__ __forceinline__ void st_granule(u32x2* p, u32x2 v) {
  __builtin_amdgcn_raw_buffer_store_b64(v, __builtin_amdgcn_make_buffer_rsrc(p, 0, 0x7fffffff, 0x00020000), 0, 0, 16);
}
__device__ __forceinline__ u32x4 ld_granule2(const u32x2* p) {   // two granules, 16 B
  return __builtin_amdgcn_raw_buffer_load_b128(__builtin_amdgcn_make_buffer_rsrc(const_cast<u32x2*>(p), 0, 0x7fffffff, 0x00020000), 0, 0, 16);
}

template <bool STREAM>
__global__ __launch_bounds__(512, 1) void edge_kernel(u32x2* vec, int N, int rounds, unsigned tag0, const u32x4* w,
                                                      size_t w_items, int* abort_flag, float* out,
                                                      unsigned long long* ts) {
  __shared__ float xs[16384];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int per = N / gridDim.x;   // slice of this WG
  u32x4 ring[16];
  size_t wi = ((size_t)blockIdx.x * 8 + wave) * 64 + lane;
  const size_t wstride = (size_t)gridDim.x * 8 * 64;
  if (STREAM)
    for (int s = 0; s < 16; ++s) { ring[s] = w[wi % w_items]; wi += wstride; }
  float acc = 0.0f;
  unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
  for (int r = 0; r < rounds; ++r) {
    const unsigned tag = tag0 + r;
    // publish (double-buffered by round parity: a WG can only get here once every WG has
    // finished reading round r-1, whose buffer round r+1 overwrites)
    u32x2* buf = vec + (size_t)(r & 1) * 16384;
    for (int i = tid; i < per; i += 512) {
      const float v = (float)(blockIdx.x * per + i) + acc * 0.0f;
      st_granule(buf + (size_t)blockIdx.x * per + i, (u32x2){__float_as_uint(v), tag});
    }
    // consume the whole vector: every lane owns a fixed set of granule pairs, issues all of
    // its loads, then re-polls only its own stale ones (bounded), staging into LDS.
    {
      int spins = 0;
      const int npairs = N / 2;
      u32x4 g[8];
      int idx[8];
      unsigned pending = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        idx[k] = tid + k * 512;
        if (idx[k] < npairs) pending |= 1u << k;
        g[k] = ld_granule2(buf + 2 * (idx[k] < npairs ? idx[k] : 0));
      }
      while (pending) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          if (pending & (1u << k)) {
            if (g[k][1] == tag && g[k][3] == tag) {
              xs[2 * idx[k]] = __uint_as_float(g[k][0]);
              xs[2 * idx[k] + 1] = __uint_as_float(g[k][2]);
              pending &= ~(1u << k);
            }
          }
        }
        if (!pending) break;
        if (++spins > (1 << 22)) {
          atomicExch(abort_flag, 1);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
#pragma unroll
        for (int k = 0; k < 8; ++k)
          if (pending & (1u << k)) g[k] = ld_granule2(buf + 2 * idx[k]);
      }
      __syncthreads();
      if (*(volatile int*)abort_flag) return;
    }
    float s = 0.0f;
    for (int i = tid; i < N; i += 512) s += xs[i];
    acc += s;
    if (STREAM) {   // consume + refill the ring between edges, like a GEMV stage
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        acc += __uint_as_float(ring[k][0] & 0x00ffffffu) * 1e-30f;
        ring[k] = w[wi % w_items];
        wi += wstride;
      }
    }
    __syncthreads();
  }
  if (tid == 0) ts[blockIdx.x] = __builtin_amdgcn_s_memrealtime() - t_start;
  if (acc == 12345.0f) out[0] = acc;
}

int main() {
  const int G = 256, N = 4096;
  u32x2* vec;
  int* abort_flag;
  float* out;
  unsigned long long* ts;
  u32x4* w;
  const size_t wbytes = 512ull << 20;
  CK(hipMalloc(&vec, sizeof(u32x2) * 32768));
  CK(hipMemset(vec, 0xff, sizeof(u32x2) * 32768));
  CK(hipMalloc(&abort_flag, 4));
  CK(hipMemset(abort_flag, 0, 4));
  CK(hipMalloc(&out, 4));
  CK(hipMalloc(&ts, 8 * G));
  CK(hipMalloc(&w, wbytes));
  CK(hipMemset(w, 1, wbytes));
  unsigned tag = 1;
  for (int stream = 0; stream < 2; ++stream) {
    for (int n : {1024, 4096, 11008 / 8 * 8}) {
      for (int rounds : {1, 64}) {
        const int nn = (n / G) * G;
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        CK(hipEventRecord(a));
        if (stream)
          edge_kernel<true><<<G, 512>>>(vec, nn, rounds, tag, w, wbytes / 16, abort_flag, out, ts);
        else
          edge_kernel<false><<<G, 512>>>(vec, nn, rounds, tag, w, wbytes / 16, abort_flag, out, ts);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        tag += rounds;
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        int ab = 0;
        CK(hipMemcpy(&ab, abort_flag, 4, hipMemcpyDeviceToHost));
        unsigned long long t[256];
        CK(hipMemcpy(t, ts, 8 * G, hipMemcpyDeviceToHost));
        double mx = 0;
        for (int i = 0; i < G; ++i) mx = t[i] > mx ? t[i] : mx;
        printf("stream %d N %5d rounds %3d: launch %8.2f us, in-kernel %8.2f us -> %6.2f us per edge%s\n", stream, nn,
               rounds, ms * 1e3, mx * 0.01, mx * 0.01 / rounds, ab ? "  ABORTED" : "");
        if (ab) return 1;
      }
    }
  }
  return 0;
}
