// gemv.hip -- fused weight-dequant x fp16 decode GEMM for gfx950 (ti_gemm_wq_a16).
//
// Replaces the decode projections of the reference: TensorEngine::matmul ->
// matmul_3d_2d (src/core/tensor_engine.cpp:594-640, scalar fp32, one core) with the
// int weights' convert_dtype (:2218-2284), plus the neighbouring element-wise ops of
// TransformerLayer::forward (src/model/inference_engine.cpp:203-233, 376-401).
//
// Shape of the work (M <= 16 decode rows, N outputs, K inputs), one launch per projection:
//   * one 8-wave workgroup per CU streams a contiguous run of 16-row tiles; wave w owns
//     k-tiles w, w+8, ... of every tile and keeps R items (1 KiB each for int4) of packed
//     weights in flight as dwordx4 loads straight into VGPRs, refilled R items ahead across
//     tile boundaries (weights are read once: no LDS round trip, cdna_hip_programming.md
//     "GEMV / M <= 16").
//   * everything small the workgroup needs (group scales, the activation rows, the
//     epilogue's residual / position inputs) is loaded BEFORE the weight ring is issued,
//     so waiting for it never drains the ring (vmcnt retires in issue order).
//   * the activation row(s) are staged in LDS as fp16 (rms_norm fused), read back as MFMA
//     A fragments; per item 4 x v_mfma_f32_16x16x32_f16 on (x, dequantized W) then one
//     fp32 FMA by the group scale; int4 nibbles -> fp16 with the 0x6400 magic (exact), int8
//     with v_perm_b32 + the same magic.
//   * the stream loop has no branches and no barriers: each item's running partial is
//     written to its tile's LDS slab (or a dummy slab), so the compiler schedules R items
//     as one block; after the stream the 8 waves' partials are summed in a fixed order
//     (deterministic) and the epilogue (residual add, SiLU*up, RoPE + KV append, logits +
//     argmax) runs on the 16 x M results of each tile.
#include <math.h>
#include <atomic>
#include <stdlib.h>

#include "common.hpp"
#include "attention_body.hpp"
#include "dequant.hpp"

namespace ti {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#ifndef TI_GEMV_RING_VGPRS
// VGPRs per lane of packed weights in flight.  Deeper is slower: a CU accepts a bounded
// number of outstanding loads, and a wave whose refill cannot issue stalls before its next
// item's math (tools/probe_gemv.hip sweep: 16-24 best, 64 costs ~15 %).
#define TI_GEMV_RING_VGPRS 20
#endif
#ifndef TI_GEMV_SYNC
#define TI_GEMV_SYNC 0   // blocks of R items between workgroup barriers in the stream (0 = none)
#endif
#ifndef TI_GEMV_RING_DELAY
#define TI_GEMV_RING_DELAY 0
#endif
#ifndef TI_GEMV_EXP
#define TI_GEMV_EXP 0   // product build; tools/probe_gemv.hip compiles diagnostic variants
#endif
#if TI_GEMV_EXP & 4   // diagnostic: per-workgroup phase timestamps (s_memrealtime, 100 MHz)
__device__ unsigned long long g_gemv_ts[4096 * 8];
#define GEMV_TS(k) \
  do { if (threadIdx.x == 0) g_gemv_ts[blockIdx.x * 8 + (k)] = __builtin_amdgcn_s_memrealtime(); } while (0)
__device__ unsigned long long g_gemv_wts[4096 * 8];   // per-wave end of stream
#define GEMV_WTS() \
  do { if ((threadIdx.x & 63) == 0) g_gemv_wts[blockIdx.x * 8 + (threadIdx.x >> 6)] = __builtin_amdgcn_s_memrealtime(); } while (0)
__device__ unsigned long long g_rows_ts[4096 * 8 * 8];   // [wg][wave][phase] (gemm_rows_kernel)
#define ROWS_TS(k)                                                                                     \
  do {                                                                                                 \
    if ((threadIdx.x & 63) == 0)                                                                       \
      g_rows_ts[(blockIdx.x * 8 + (threadIdx.x >> 6)) * 8 + (k)] = __builtin_amdgcn_s_memrealtime();   \
  } while (0)
#else
#define GEMV_WTS() do { } while (0)
#define GEMV_TS(k) do { } while (0)
#define ROWS_TS(k) do { } while (0)
#endif

constexpr int kGemvWaves = 8;
constexpr int kGemvThreads = kGemvWaves * kWave;

struct GemvArgs {
  const u32x4* tiles;
  const uint16_t* scales;
  const void* x;
  const float* norm_w;
  float eps;
  int32_t x_kind, ldx, M, N, K;
  ti_epilogue epi;
  unsigned long long* stamp;   // in-step launch stamps (common.hpp stamp_end), NULL in product launches
};

__host__ __device__ constexpr int align16(int b) { return (b + 15) & ~15; }

// The GEMM's two remaining A/B knobs, read once per process (thread-safe static init).
struct GemmKnobs {
  bool splitk = true;       // TI_GEMM_SPLITK=0: no split-K for under-filled tile grids
  bool rows_split = true;   // TI_GEMM_ROWS_SPLIT=0: all rows in one batched-rows workgroup
};
__host__ inline const GemmKnobs& gemm_knobs() {
  static const GemmKnobs k = [] {
    GemmKnobs v;
    if (const char* e = getenv("TI_GEMM_SPLITK")) v.splitk = atoi(e) != 0;
    if (const char* e = getenv("TI_GEMM_ROWS_SPLIT")) v.rows_split = atoi(e) != 0;
    return v;
  }();
  return k;
}

// Workgroups per launch: one 8-wave workgroup per CU (a second workgroup per CU measured slower,
// DESIGN 4.1), never more than there are 16-row tiles.

__host__ __device__ inline int gemv_lds_bytes_tiles(int M, int K, int tiles_per_wg, bool g32 = false, bool aff = false);

// Tiles per workgroup are bounded by the LDS image (partial slabs and scales grow with
// them): very wide outputs (a 128k vocabulary) get more workgroups than CUs.
__host__ inline int gemv_grid(int M, int N, int K, int num_cus, bool g32 = false, bool aff = false) {
  const int NT = N >> 4;
  const int g = num_cus > 0 ? num_cus : 256;
  int grid = NT < g ? NT : g;
  while (grid < NT && gemv_lds_bytes_tiles(M, K, (NT + grid - 1) / grid, g32, aff) > 160 * 1024) grid += grid / 8 + 1;
  return grid < NT ? grid : NT;
}

// LDS image of one workgroup (bytes, each region 16-aligned):
//   x      [M][K + 8] fp16            activation rows (row pad breaks bank aliasing)
//   scales [ntl][K/128][16] fp16      group scales of the workgroup's tiles ([ntl][K/128][4][16]
//                                     with group-32 weights, TI_BITS_G32)
//   corr   [K/128][16] f32            int4: per (group, row) offset correction (see deq_int4_raw)
//                                     ([K/32][16] with group-32 weights)
//   slab   [ntl + 1][8][64] f32x4     per-wave partial tiles (+ one dummy slab)
//   es     epilogue inputs: residual [ntl][M][16] f32 (+ the fold weights of the same
//          outputs, TI_EPI_RESID_F32 with fold_x), or RoPE (cos, sin) [M][hd] + pos [M]
//   best   [16] u64                   argmax keys of the workgroup
//   (affine group-32, TI_BITS_AFF: + the block minimums [ntl][K/128][4][16] fp16 after the scales
//    and the blocks' sums of x [K/32][16] f32 after corr)
struct GemvLds {
  int x, sc, corr, slab, es, best, total, mins, bsum;
};
__host__ __device__ inline GemvLds gemv_lds_layout(int M, int K, int ntl, bool g32 = false, bool aff = false) {
  GemvLds l;
  const int gm = g32 ? 4 : 1;                  // scale / correction groups per 128 k
  l.x = 0;
  l.sc = l.x + align16(M * (K + 8) * 2);
  l.mins = l.sc + align16(ntl * (K >> 7) * 32 * gm);
  l.corr = l.mins + (aff ? align16(ntl * (K >> 7) * 32 * gm) : 0);
  l.bsum = l.corr + (K >> 7) * 16 * 4 * gm;
  l.slab = l.bsum + (aff ? (K >> 7) * 16 * 4 * gm : 0);   // int4 offset correction [K/128 (x4)][16 rows] f32
  l.es = l.slab + (ntl + 1) * kGemvWaves * kWave * 16;
  const int es_bytes = 2 * ntl * M * 16 * 4 > M * 128 * 4 + 64 ? 2 * ntl * M * 16 * 4 : M * 128 * 4 + 64;
  l.best = l.es + align16(es_bytes);
  l.total = l.best + 16 * 8;
  return l;
}
__host__ __device__ inline int gemv_lds_bytes_tiles(int M, int K, int tiles_per_wg, bool g32, bool aff) {
  return gemv_lds_layout(M, K, tiles_per_wg, g32, aff).total;
}

// ------------------------------------------------------------- x staging (LDS)
// x staging modes (chosen on the host): fp16 rows prefetched into registers; fp32 rows;
// rms_norm of ONE row of K <= 4096 held in registers; rms_norm of several / longer rows.
// XM_F16F: fp16 rows of h * nw (TI_X_F16_FOLDED, one row) staged like XM_F16; the rms comes
// from the producer's partial sums of squares and divides the outputs before the epilogue.
// XM_ATTN: the attention's split partials (TI_X_ATTN_SPLITS, one row), merged while staging.
enum { XM_F16 = 0, XM_F32 = 1, XM_NORM1 = 2, XM_NORM = 3, XM_F16F = 4, XM_ATTN = 5 };

// Generic staging (M > 1 with rms_norm, f32 rows, or rows longer than the register
// prefetch covers).  Runs after the ring is issued, so its loads wait behind the ring.
template <int XM>
__device__ __forceinline__ void stage_x_generic(const GemvArgs& a, f16* xl, float* red, int k8_from) {
  const int tid = threadIdx.x, K = a.K, xs = K + 8, K8 = K >> 3;
  if constexpr (XM == XM_NORM || XM == XM_NORM1) {
    // rms_norm (tensor_engine.cpp:1488-1505): y = (x / sqrt(sum(x^2)/K + eps)) * w.
    for (int m = 0; m < a.M; ++m) {
      const float* xr = (const float*)a.x + (size_t)m * a.ldx;
      float ss = 0.0f;
      for (int k8 = tid; k8 < K8; k8 += kGemvThreads) {
        const float4 v0 = *(const float4*)(xr + 8 * k8), v1 = *(const float4*)(xr + 8 * k8 + 4);
        ss = fmaf(v0.x, v0.x, ss); ss = fmaf(v0.y, v0.y, ss); ss = fmaf(v0.z, v0.z, ss); ss = fmaf(v0.w, v0.w, ss);
        ss = fmaf(v1.x, v1.x, ss); ss = fmaf(v1.y, v1.y, ss); ss = fmaf(v1.z, v1.z, ss); ss = fmaf(v1.w, v1.w, ss);
      }
      ss = group_sum<kWave>(ss);
      if ((tid & 63) == 0) red[tid >> 6] = ss;
      __syncthreads();
      float tot = 0.0f;
#pragma unroll
      for (int w = 0; w < kGemvWaves; ++w) tot += red[w];
      const float rms = sqrtf(tot / (float)K + a.eps);
      for (int k8 = tid; k8 < K8; k8 += kGemvThreads) {
        const float4 v0 = *(const float4*)(xr + 8 * k8), v1 = *(const float4*)(xr + 8 * k8 + 4);
        const float4 w0 = *(const float4*)(a.norm_w + 8 * k8), w1 = *(const float4*)(a.norm_w + 8 * k8 + 4);
        f16x8 h;
        h[0] = (f16)((v0.x / rms) * w0.x); h[1] = (f16)((v0.y / rms) * w0.y);
        h[2] = (f16)((v0.z / rms) * w0.z); h[3] = (f16)((v0.w / rms) * w0.w);
        h[4] = (f16)((v1.x / rms) * w1.x); h[5] = (f16)((v1.y / rms) * w1.y);
        h[6] = (f16)((v1.z / rms) * w1.z); h[7] = (f16)((v1.w / rms) * w1.w);
        *(f16x8*)(xl + m * xs + 8 * k8) = h;
      }
      __syncthreads();   // red reused by the next row
    }
  } else if constexpr (XM == XM_F32) {
    for (int i = tid; i < a.M * K8; i += kGemvThreads) {
      const int m = i / K8, k8 = i - m * K8;
      const float* xr = (const float*)a.x + (size_t)m * a.ldx + 8 * k8;
      const float4 v0 = *(const float4*)xr, v1 = *(const float4*)(xr + 4);
      f16x8 h;
      h[0] = (f16)v0.x; h[1] = (f16)v0.y; h[2] = (f16)v0.z; h[3] = (f16)v0.w;
      h[4] = (f16)v1.x; h[5] = (f16)v1.y; h[6] = (f16)v1.z; h[7] = (f16)v1.w;
      *(f16x8*)(xl + m * xs + 8 * k8) = h;
    }
  } else {
    for (int i = tid + k8_from; i < a.M * K8; i += kGemvThreads) {
      const int m = i / K8, k8 = i - m * K8;
      *(u32x4*)(xl + m * xs + 8 * k8) = *(const u32x4*)((const f16*)a.x + (size_t)m * a.ldx + 8 * k8);
    }
  }
}

// ------------------------------------------------------------------ epilogue
__device__ __forceinline__ uint32_t float_order_key(float v) {
  const uint32_t u = __builtin_bit_cast(uint32_t, v);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// Thread (l, i) holds y[m][n] of tile nt with m = 4*(l>>4) + i, n = l & 15 (the
// v_mfma_f32_16x16x32 C layout, reduced over the 8 waves); l is the lane or, for M <= 4,
// n alone.  Partners of the shuffles below (n ^ 1, n + 8) sit in the same 16-lane group.  `best` is the
// thread's running argmax key for LOGITS_ARGMAX.
// RESID with fold_x (M == 1): also the fp16 h * nw of the next projection's TI_X_F16_FOLDED input
// (fold weights pre-staged at fw) and this thread's running sum of h^2 (ssacc).
__device__ __forceinline__ void epilogue(const GemvArgs& a, int nt, int tl, int l, int i, float v, const float* es,
                                         unsigned long long& best, bool ok, const float* fw, float& ssacc) {
  const ti_epilogue& e = a.epi;
  const int m = 4 * (l >> 4) + i, n = l & 15, ng = nt * 16 + n;
  const bool live = ok && m < a.M;
  switch (e.kind) {
    case TI_EPI_STORE_F32:
      if (live) ((float*)e.out)[(size_t)m * e.ldo + ng] = v;
      break;
    case TI_EPI_STORE_F16:
      if (live) ((uint16_t*)e.out)[(size_t)m * e.ldo + ng] = f2h(v);
      break;
    case TI_EPI_RESID_F32:   // add(residual, y), tensor_engine.cpp:1626-1678; residual pre-staged in LDS
      if (live) {
        const float r = es[(tl * a.M + m) * 16 + n] + v;
        ((float*)e.out)[(size_t)m * e.ldo + ng] = r;
        if (e.fold_x) {
          e.fold_x[ng] = f2h(r * fw[tl * 16 + n]);
          ssacc = fmaf(r, r, ssacc);
        }
      }
      break;
    case TI_EPI_SILU_MUL_F16: {
      // compute_ffn (inference_engine.cpp:386-391): multiply(up, silu(gate)).
      const float up = lane_xor<8>(v);   // lanes n < 8: the up row n + 8 of the same tile
      const float s = v / (1.0f + expf(-v));
      if (live && n < 8) ((uint16_t*)e.out)[(size_t)m * e.ldo + nt * 8 + n] = f2h(up * s);
      break;
    }
    case TI_EPI_QKV_ROPE_KV: {
      const float partner = lane_xor<1>(v);
      const int hd = e.head_dim;
      const bool qk = ng < e.q_dim + e.kv_dim;
      float r = v;
      int p = 0;
      if (live) {
        p = ((const int*)(es + a.M * hd))[m];
        if (qk) {
          const int base = ng < e.q_dim ? 0 : e.q_dim;
          const int d = (ng - base) % hd;
          const float2 cs = *(const float2*)(es + m * hd + (d & ~1));   // (cos, sin) of pos[m], staged
          // apply_rope (tensor_engine.cpp:1602-1612): even = x*c - y*s, odd = x*s + y*c,
          // evaluated with the reference build's contraction pattern.
          r = (d & 1) == 0 ? fmaf(-partner, cs.y, v * cs.x) : fmaf(v, cs.x, partner * cs.y);
        }
      }
      if (!live) break;
      if (ng < e.q_dim) {
        ((float*)e.out)[(size_t)m * e.ldo + ng] = r;
      } else {
        const bool is_k = qk;
        const int c = ng - e.q_dim - (is_k ? 0 : e.kv_dim);
        const int kvh = c / hd, d = c - kvh * hd;
        uint16_t* cache = is_k ? e.k_cache : e.v_cache;
        cache[(size_t)m * e.kv_stream_stride + ((size_t)kvh * e.max_seq + p) * hd + d] = f2h(r);
      }
      break;
    }
    case TI_EPI_LOGITS_ARGMAX: {
      if (live) {
        ((float*)e.out)[(size_t)m * e.ldo + ng] = v;
        const unsigned long long key = ((unsigned long long)float_order_key(v) << 32) |
                                       (unsigned long long)(0xFFFFFFFFu - (uint32_t)ng);
        best = key > best ? key : best;
      }
      break;
    }
    default:
      break;
  }
}

// Weight stream load: read once per launch, so non-temporal where that pays (TI_GEMV_NT).
#ifndef TI_GEMV_NT
#define TI_GEMV_NT 1
#endif
__device__ __forceinline__ u32x4 ld_w(const u32x4* p) {
#if TI_GEMV_NT || (TI_GEMV_EXP & 16)
  return __builtin_nontemporal_load(p);
#else
  return *p;
#endif
}

// Offset-folded int4 input prep of one staged x piece (deq_int4_raw): the high-nibble slots scaled
// by 1/16 (exact in fp16) and the piece's share of corr[g][m] = 1032 * sum_lo x + 1152 * sum_hi x.
__device__ __forceinline__ float int4_x_prep(f16x8& h) {
  const f16 s16 = (f16)0.0625f;
  h[2] *= s16; h[3] *= s16; h[6] *= s16; h[7] *= s16;
  const float lo = ((float)h[0] + (float)h[1]) + ((float)h[4] + (float)h[5]);
  const float hi = ((float)h[2] + (float)h[3]) + ((float)h[6] + (float)h[7]);
  return 1032.0f * lo + 1152.0f * hi;
}

// --------------------------------------------------------------------- kernel
// LDS barrier that leaves the wave's outstanding global loads in flight (a plain
// __syncthreads() may drain vmcnt): LDS writes retired, then s_barrier.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// The fields on the prologue's critical path come first as separate arguments: gfx950 can
// preload leading kernel arguments into SGPRs before the waves start (compiled with
// -mllvm -amdgpu-kernarg-preload-count, see Makefile), so the first x / weight / epilogue-input
// loads do not wait for a kernarg s_load round trip (the grid size is passed too: gridDim
// comes from the hidden kernargs).  Everything read before the weight ring is issued sits in
// the 14 dwords the hardware preloads (s[2:15]; packed below); the struct carries the rest.
//   p_aux: the rms_norm weight (XM_NORM*), the producer's ss partials (XM_F16F), the splits'
//          (max, sum) pairs (XM_ATTN), else NULL
//   p_mgk: M | grid << 6 | epilogue kind << 18 | head_dim / 64 << 21 (XM_ATTN)
//   p_kx:  K | (ldx, or n_ss for XM_F16F, or splits for XM_ATTN) << 16
// Workgroup blockIdx.x runs over its contiguous tile range.
// G32: group-32 weights (TI_BITS_G32, GGUF Q4_0 / Q8_0 blocks): within a tile, lane l holds for
// MFMA step s4 the 8 k = 32 s4 + 8 (l >> 4) + e, so each v_mfma_f32_16x16x32 reduces exactly one
// 32-weight block; its scale (and, int4, its offset correction) is applied per step.
template <int BITS, int XM, bool G32 = false, bool AFF = false>
__global__ __launch_bounds__(kGemvThreads, 1) void gemv_wq_kernel(const u32x4* p_tiles, const uint16_t* p_scales,
                                                                   const void* p_x, const float* p_aux, int p_mgk,
                                                                   int p_N, int p_kx, int p_ldo, const float* p_pre,
                                                                   GemvArgs a) {
  const unsigned long long t_entry = stamp_now();
  const unsigned bid = blockIdx.x;
  a.tiles = p_tiles;
  a.scales = p_scales;
  a.x = p_x;
  a.norm_w = p_aux;
  a.M = p_mgk & 63;
  // p_N = q | r << 8: NT = q * grid + r 16-row tiles, workgroup b takes q (+1 for b < r) of them from
  // t0 = b q + min(b, r) (scalar arithmetic only; launch_gemv packs it)
  const int nt_q = p_N & 0xff, nt_r = (int)((unsigned)p_N >> 8);
  a.K = p_kx & 0xffff;
  a.ldx = XM == XM_F16F || XM == XM_ATTN ? a.K : (int)((unsigned)p_kx >> 16);
  const int p_grid = (p_mgk >> 6) & 0xfff;
  a.N = 16 * (nt_q * p_grid + nt_r);
  constexpr int C = TileFmt<BITS>::kChunks;
  constexpr int R = TI_GEMV_RING_VGPRS / (4 * C) > 2 ? TI_GEMV_RING_VGPRS / (4 * C) : 2;   // ring depth (items)
  constexpr int XPF = 3;                           // fp16 x: 16-byte pieces prefetched per thread
  extern __shared__ __attribute__((aligned(16))) char smem[];
  GEMV_TS(0);
  const int KT = a.K >> 7, xs = a.K + 8, NT = a.N >> 4, K8 = a.K >> 3;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: counters live in SGPRs
  const int t0 = (int)bid * nt_q + ((int)bid < nt_r ? (int)bid : nt_r);
  const int ntl = nt_q + ((int)bid < nt_r ? 1 : 0);
  constexpr bool kOneRow = XM == XM_F16F || XM == XM_ATTN || XM == XM_NORM1;   // (M == 1 by construction)
  const int KW = wave < KT ? (KT - wave + kGemvWaves - 1) / kGemvWaves : 0;   // k-tiles per tile, this wave
  const int total = ntl * KW;
  static_assert(!G32 || BITS != 16, "group-32 weights: int4 / int8");
  static_assert(!AFF || (G32 && BITS == 4), "affine blocks: group-32 int4");
  const GemvLds L = gemv_lds_layout(a.M, a.K, ntl, G32, AFF);
  uint16_t* ml = (uint16_t*)(smem + L.mins);       // AFF: block minimums, as sl
  float* bsum = (float*)(smem + L.bsum);           // AFF: [K/32][16] sums of x per block and row
  f16* xl = (f16*)(smem + L.x);
  uint16_t* sl = (uint16_t*)(smem + L.sc);
  float* corr = (float*)(smem + L.corr);           // [K/128][16] (int4 only)
  f32x4* slab = (f32x4*)(smem + L.slab);           // [ntl + 1][8][64]
  float* es = (float*)(smem + L.es);
  unsigned long long* best_l = (unsigned long long*)(smem + L.best);
  float* red = (float*)(smem + L.slab);            // norm reduction scratch (before the stream)

  // ---- 1. small inputs into registers, ahead of the ring
  const int n_sc = BITS == 16 ? 0 : ntl * KT * (G32 ? 8 : 2);  // u32x4 pieces of scales
  const u32x4* sg = (const u32x4*)(a.scales + (size_t)t0 * KT * (G32 ? 64 : 16));
  u32x4 sc_reg = {0u, 0u, 0u, 0u};
#if TI_GEMV_EXP & 8   // diagnostic: no dependency on x / scales (constants instead of loads)
  const int nx16 = a.M * K8;
  float4 v0 = {1.0f, 1.0f, 1.0f, 1.0f}, v1 = v0, w0 = v0, w1 = v0;
  u32x4 xr16[XPF];
  for (int q = 0; q < XPF; ++q) xr16[q] = (u32x4){0x3c003c00u, 0x3c003c00u, 0x3c003c00u, 0x3c003c00u};
  sc_reg = xr16[0];
  auto load_x = [&]() {};
  if (false) {
#else
  if constexpr (BITS != 16) sc_reg = ld_w(sg + (tid < n_sc ? tid : 0));

  const int nx16 = a.M * K8;
  float4 v0, v1, w0, w1;
  u32x4 xr16[XPF];
  // x rows and the epilogue input depend on the previous launch
  // XM_ATTN: this thread's 8 dims (one head) of every split, and the splits' (max, sum)
  constexpr int kPS = TI_ATTN_MAX_PART_SPLITS;
  u32x4 po[XM == XM_ATTN ? kPS : 1];
  float2 pml[XM == XM_ATTN ? kPS : 1];
  auto load_x = [&]() {
    if constexpr (XM == XM_ATTN) {
      const int S = (int)((unsigned)p_kx >> 16), hsh = ((p_mgk >> 21) & 3) == 2 ? 7 : 6;
      const int i = tid < K8 ? tid : K8 - 1, h = (8 * i) >> hsh, d = (8 * i) & ((1 << hsh) - 1);
#pragma unroll
      for (int sp = 0; sp < kPS; ++sp) {
        const int r = h * S + (sp < S ? sp : S - 1);
        po[sp] = *(const u32x4*)((const f16*)a.x + ((size_t)r << hsh) + d);
        pml[sp] = *(const float2*)(p_aux + 2 * r);
      }
    } else if constexpr (XM == XM_NORM1) {
      const int k8 = tid < K8 ? tid : K8 - 1;
      const float* xr = (const float*)a.x;
      v0 = *(const float4*)(xr + 8 * k8);
      v1 = *(const float4*)(xr + 8 * k8 + 4);
    } else if constexpr (XM == XM_F16 || XM == XM_F16F) {
#pragma unroll
      for (int q = 0; q < XPF; ++q) {
        const int i = tid + q * kGemvThreads < nx16 ? tid + q * kGemvThreads : nx16 - 1;
        const int m = kOneRow ? 0 : i / K8, k8 = i - m * K8;
        xr16[q] = *(const u32x4*)((const f16*)a.x + (size_t)m * a.ldx + 8 * k8);
      }
    }
  };
  if constexpr (XM == XM_NORM1) {
#endif
    const int k8 = tid < K8 ? tid : K8 - 1;
    w0 = *(const float4*)(a.norm_w + 8 * k8);
    w1 = *(const float4*)(a.norm_w + 8 * k8 + 4);
  }
  load_x();
  // Epilogue input, one word per thread, loaded unconditionally (a branch here would make
  // the compiler wait at the join): a residual element of our tiles, this step's position
  // of row tid, or a dummy word of x.
  // (p_pre / kind / ldo are preloaded: epi.out for RESID, epi.pos for QKV, else x)
  const int kind = (p_mgk >> 18) & 7, ldo = p_ldo;
  const int n_res = kind == TI_EPI_RESID_F32 ? ntl * a.M * 16 : 0;
  const float* pre_p;
  {
    const int idx = tid < n_res ? tid : 0;
    const int tl = kOneRow ? idx >> 4 : idx / (a.M * 16), rem = idx - tl * a.M * 16, m = rem >> 4, n = rem & 15;
    pre_p = kind == TI_EPI_RESID_F32 ? p_pre + (size_t)m * ldo + (t0 + tl) * 16 + n
            : kind == TI_EPI_QKV_ROPE_KV ? p_pre + (tid < a.M ? tid : 0) : p_pre;
  }
  const float pre = *pre_p;
  // RESID with fold_x: the fold weight of the same output (one row), consumed by the epilogue
  // (its pointer comes from the kernarg struct: loaded after the ring is issued, below)
  float fw_pre = 0.0f;
  // XM_F16F: this lane's share of the producer's partial sums of squares (up to 256 of them),
  // clamped loads; masked and summed after the stream
  float ss4[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  const int n_ss = (int)((unsigned)p_kx >> 16);
  if constexpr (XM == XM_F16F) {
#pragma unroll
    for (int j = 0; j < 4; ++j) ss4[j] = p_aux[lane + 64 * j < n_ss ? lane + 64 * j : 0];
  }

  // ---- 2. the weight ring.  Item j of this wave = (tile j / KW, k-tile wave + 8 * (j % KW));
  // items past the end re-load the last item (no branch around loads); coordinates advance
  // by counters (no integer division in the stream).
  const u32x4* tb = a.tiles + (size_t)t0 * KT * (kWave * C) + lane;
  const size_t last_off = total > 0 ? ((size_t)(ntl - 1) * KT + wave + kGemvWaves * (KW - 1)) * (kWave * C) : 0;
  int rt = 0, rk = 0, rj = 0;                      // refill cursor: tile, k index, item
  auto refill_off = [&]() -> size_t {
    const size_t o = rj < total ? ((size_t)rt * KT + wave + kGemvWaves * rk) * (kWave * C) : last_off;
    ++rj;
    if (++rk == KW) { rk = 0; ++rt; }
    return o;
  };
  // Only the first R0 slots go out before the staging barrier: a CU's memory pipe accepts a
  // limited number of outstanding loads, so a wave issuing all R slots blocks in issue for
  // microseconds, and the barrier (hence the first MFMA) would wait for the slowest wave's
  // whole burst.  The rest of the ring is issued right after the barrier.
  constexpr int R0 = R >= 8 ? 4 : R;
  u32x4 ring[R][C];
#if TI_GEMV_RING_DELAY > 0   // A/B knob: hold the ring back (x 64 clocks) behind the small loads
  __builtin_amdgcn_s_sleep(TI_GEMV_RING_DELAY);
#endif
#pragma unroll
  for (int s = 0; s < R0; ++s) {
    const size_t o = refill_off();
#pragma unroll
    for (int c = 0; c < C; ++c) ring[s][c] = ld_w(tb + o + c * kWave);
  }
  const bool fold = (XM == XM_F16 || XM == XM_ATTN) && kind == TI_EPI_RESID_F32 && a.epi.fold_x != nullptr;
  if constexpr (XM == XM_F16 || XM == XM_ATTN) {   // fold weight (consumed by the epilogue)
    const float* fw_p = fold ? a.epi.fold_w + (size_t)t0 * 16 + (tid < n_res ? tid : 0) : pre_p;
    fw_pre = *fw_p;
  }

  GEMV_TS(1);
  STAMP_MARK(ph_issued);
  // ---- 3. stage scales and x in LDS (waits only for the loads of step 1)
  if constexpr (BITS != 16) {
    if (tid < n_sc) ((u32x4*)sl)[tid] = sc_reg;
  }
  // int4 (group 128): the x pieces staged from registers get their 1/16 scaling and offset correction
  // here, before the staging barrier (no second LDS pass and barrier in front of the stream); every
  // piece of x must come from registers for that (rare long shapes take the pass below)
  constexpr bool kRegPrep = BITS == 4 && !G32 && (XM == XM_NORM1 || XM == XM_ATTN || XM == XM_F16 || XM == XM_F16F);
  const bool reg_prep = kRegPrep && (XM == XM_NORM1 || XM == XM_ATTN || nx16 <= XPF * kGemvThreads);
  if constexpr (XM == XM_NORM1) {
    // rms_norm (tensor_engine.cpp:1488-1505) of the single row, x and w held in registers.
    float ss = 0.0f;
    if (tid < K8) {
      ss = fmaf(v0.x, v0.x, ss); ss = fmaf(v0.y, v0.y, ss); ss = fmaf(v0.z, v0.z, ss); ss = fmaf(v0.w, v0.w, ss);
      ss = fmaf(v1.x, v1.x, ss); ss = fmaf(v1.y, v1.y, ss); ss = fmaf(v1.z, v1.z, ss); ss = fmaf(v1.w, v1.w, ss);
    }
    ss = group_sum<kWave>(ss);
    if (lane == 0) red[wave] = ss;
    lds_barrier();
    float tot = 0.0f;
#pragma unroll
    for (int w = 0; w < kGemvWaves; ++w) tot += red[w];
    const float rms = sqrtf(tot / (float)a.K + a.eps);
    float part = 0.0f;
    if (tid < K8) {
      f16x8 h;
      h[0] = (f16)((v0.x / rms) * w0.x); h[1] = (f16)((v0.y / rms) * w0.y);
      h[2] = (f16)((v0.z / rms) * w0.z); h[3] = (f16)((v0.w / rms) * w0.w);
      h[4] = (f16)((v1.x / rms) * w1.x); h[5] = (f16)((v1.y / rms) * w1.y);
      h[6] = (f16)((v1.z / rms) * w1.z); h[7] = (f16)((v1.w / rms) * w1.w);
      if constexpr (kRegPrep) part = int4_x_prep(h);
      *(f16x8*)(xl + 8 * tid) = h;
    }
    if constexpr (kRegPrep) {
      part = group_sum<16>(part);
      if (tid < K8 && (lane & 15) == 0) corr[(tid >> 4) * 16] = part;
    }
  } else if constexpr (XM == XM_ATTN) {
    // the attention's split merge (attention.hip last-arriver merge): weights
    // l_s * exp(m_s - max), normalised rows o_s, empty splits (m = -inf) weigh 0
    const int S = (int)((unsigned)p_kx >> 16);
    float mx = -INFINITY;
#pragma unroll
    for (int sp = 0; sp < kPS; ++sp) mx = sp < S ? fmaxf(mx, pml[sp].x) : mx;
    float num[8] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f}, den = 0.0f;
#pragma unroll
    for (int sp = 0; sp < kPS; ++sp) {
      const float f = sp < S && pml[sp].x != -INFINITY ? pml[sp].y * __expf(pml[sp].x - mx) : 0.0f;
      den += f;
      const f16x8 o = __builtin_bit_cast(f16x8, po[sp]);
#pragma unroll
      for (int e = 0; e < 8; ++e) num[e] = fmaf(f, (float)o[e], num[e]);
    }
    float part = 0.0f;
    if (tid < K8) {
      f16x8 hx;
#pragma unroll
      for (int e = 0; e < 8; ++e) hx[e] = (f16)(den > 0.0f ? num[e] / den : 0.0f);
      if constexpr (kRegPrep) part = int4_x_prep(hx);
      *(f16x8*)(xl + 8 * tid) = hx;
    }
    if constexpr (kRegPrep) {
      part = group_sum<16>(part);
      if (tid < K8 && (lane & 15) == 0) corr[(tid >> 4) * 16] = part;
    }
  } else if constexpr (XM == XM_F16 || XM == XM_F16F) {
#pragma unroll
    for (int q = 0; q < XPF; ++q) {
      const int i = tid + q * kGemvThreads;
      const int m = kOneRow || i >= nx16 ? 0 : i / K8, k8 = i - m * K8;
      float part = 0.0f;
      if (i < nx16) {
        if (kRegPrep && reg_prep) {
          f16x8 h = __builtin_bit_cast(f16x8, xr16[q]);
          part = int4_x_prep(h);
          *(f16x8*)(xl + m * xs + 8 * k8) = h;
        } else {
          *(u32x4*)(xl + m * xs + 8 * k8) = xr16[q];
        }
      }
      if (kRegPrep && reg_prep) {   // (uniform: every lane of a 16-lane group has the same q)
        part = group_sum<16>(part);
        if (i < nx16 && (lane & 15) == 0) corr[(k8 >> 4) * 16 + m] = part;
      }
    }
  }
  // rare shapes: what the register prefetch did not cover (these loads wait behind the ring)
  if constexpr (BITS != 16) {
    for (int i = tid + kGemvThreads; i < n_sc; i += kGemvThreads) ((u32x4*)sl)[i] = sg[i];
  }
  if constexpr (AFF) {   // the minimums follow all N/16 tiles' scales in the same buffer
    const u32x4* mg = (const u32x4*)(a.scales + (size_t)NT * KT * 64 + (size_t)t0 * KT * 64);
    for (int i = tid; i < n_sc; i += kGemvThreads) ((u32x4*)ml)[i] = mg[i];
  }
  if constexpr (XM == XM_F16 || XM == XM_F16F) {
    if (nx16 > XPF * kGemvThreads) stage_x_generic<XM>(a, xl, red, XPF * kGemvThreads);
  } else if constexpr (XM != XM_NORM1 && XM != XM_ATTN) {
    stage_x_generic<XM>(a, xl, red, 0);
  }
  if (a.epi.kind == TI_EPI_QKV_ROPE_KV && tid < a.M) ((int*)(es + a.M * a.epi.head_dim))[tid] = __builtin_bit_cast(int, pre);
  if (tid < 16) best_l[tid] = 0ull;
  lds_barrier();
  STAMP_MARK(ph_staged);
#pragma unroll
  for (int s = R0; s < R; ++s) {
    const size_t o = refill_off();
#pragma unroll
    for (int c = 0; c < C; ++c) ring[s][c] = ld_w(tb + o + c * kWave);
  }
  if constexpr (BITS == 4) if (!reg_prep) {
    // Offset-folded int4 (deq_int4_raw): scale the high-nibble slots of x by 1/16 (exact in
    // fp16) and build corr[g][m] = 1032 * sum_lo a + 1152 * sum_hi a per 128-k group.  A
    // group is 16 consecutive k8 pieces, i.e. 16 consecutive lanes (K8 % 16 == 0).
    const f16 s16 = (f16)0.0625f;
    for (int i0 = 0; i0 < a.M * K8; i0 += kGemvThreads) {
      const int idx = i0 + tid;
      float part = 0.0f, sx = 0.0f;
      int m = 0, k8 = 0;
      if (idx < a.M * K8) {
        m = idx / K8;
        k8 = idx - m * K8;
        f16x8 h = *(const f16x8*)(xl + m * xs + 8 * k8);
        h[2] *= s16; h[3] *= s16; h[6] *= s16; h[7] *= s16;
        *(f16x8*)(xl + m * xs + 8 * k8) = h;
        const float lo = ((float)h[0] + (float)h[1]) + ((float)h[4] + (float)h[5]);
        const float hi = ((float)h[2] + (float)h[3]) + ((float)h[6] + (float)h[7]);
        part = 1032.0f * lo + 1152.0f * hi;
        if constexpr (AFF) sx = lo + 16.0f * hi;   // the piece's sum of x (high slots were scaled by 1/16)
      }
      if constexpr (G32) {   // one 32-k block = 4 consecutive pieces
        part = group_sum<4>(part);
        if (idx < a.M * K8 && (lane & 3) == 0) corr[(k8 >> 2) * 16 + m] = part;
        if constexpr (AFF) {
          sx = group_sum<4>(sx);
          if (idx < a.M * K8 && (lane & 3) == 0) bsum[(k8 >> 2) * 16 + m] = sx;
        }
      } else {
        part = group_sum<16>(part);
        if (idx < a.M * K8 && (lane & 15) == 0) corr[(k8 >> 4) * 16 + m] = part;
      }
    }
    lds_barrier();
  }

  // RoPE (cos, sin) of each row's position: issued now, consumed after the stream.
  float cs_reg = 0.0f;
  const int n_cs = a.epi.kind == TI_EPI_QKV_ROPE_KV ? a.M * a.epi.head_dim : 0;
  if (n_cs > 0) {
    const int hd = a.epi.head_dim, idx = tid < n_cs ? tid : 0, m = idx / hd, j = idx - m * hd;
    cs_reg = a.epi.rope_cs[(size_t)((const int*)(es + a.M * hd))[m] * hd + j];
  }

  GEMV_TS(2);
  STAMP_MARK(ph_stream);
  // ---- 4. the stream: branch-free, R items per block
  const int r = lane & 15, kq = lane >> 4;
  const f16* xrow = xl + (r < a.M ? r : a.M - 1) * xs + kq * 32;
  f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
  uint32_t magic;   // 0x64006400 in a VGPR (see deq_int4_raw)
  asm volatile("v_mov_b32 %0, 0x64006400" : "=v"(magic));
  f32x4* my_slab = slab + wave * kWave + lane;     // + tile * 8 * 64
  constexpr int kSlabStride = kGemvWaves * kWave;
  int ct = 0, ck = 0;                              // compute cursor: tile, k index
  auto item = [&](const u32x4 (&w)[C]) {
    const int kt = wave + kGemvWaves * ck;
    f32x4 t = {0.0f, 0.0f, 0.0f, 0.0f};
    if constexpr (BITS == 16) t = acc;
    if constexpr (G32) {
      const f16* xr32 = xrow - kq * 32 + kq * 8;   // this lane's 8 k of each 32-k block
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        const f16x8 bf = dequant_step<BITS>(w, s4, magic);
        const f16x8 af = *(const f16x8*)(xr32 + kt * 128 + s4 * 32);
        f32x4 tb = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, bf, (f32x4){0.0f, 0.0f, 0.0f, 0.0f}, 0, 0, 0);
        if constexpr (BITS == 4) tb -= *(const f32x4*)(corr + (kt * 4 + s4) * 16 + 4 * kq);
        const float sc = h2f(sl[((ct * KT + kt) * 4 + s4) * 16 + r]);
        acc[0] = fmaf(sc, tb[0], acc[0]);
        acc[1] = fmaf(sc, tb[1], acc[1]);
        acc[2] = fmaf(sc, tb[2], acc[2]);
        acc[3] = fmaf(sc, tb[3], acc[3]);
        if constexpr (AFF) {   // weight = d (q - 8) + (8 d + m): the offset term times the block's sum of x
          const float mt = fmaf(8.0f, sc, h2f(ml[((ct * KT + kt) * 4 + s4) * 16 + r]));
          const f32x4 bs = *(const f32x4*)(bsum + (kt * 4 + s4) * 16 + 4 * kq);
          acc[0] = fmaf(mt, bs[0], acc[0]);
          acc[1] = fmaf(mt, bs[1], acc[1]);
          acc[2] = fmaf(mt, bs[2], acc[2]);
          acc[3] = fmaf(mt, bs[3], acc[3]);
        }
      }
    } else {
#if TI_GEMV_EXP & 1   // diagnostic build (tools/probe_gemv.hip): stream only, no dequant / MFMA
    t[0] += __builtin_bit_cast(float, w[0][0] ^ w[0][1] ^ w[0][2] ^ w[0][3]) + (float)xrow[kt];
#else
    (void)t;
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      const f16x8 bf = dequant_step<BITS>(w, s4, magic);
      const f16x8 af = *(const f16x8*)(xrow + kt * 128 + s4 * 8);
      t = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, bf, t, 0, 0, 0);
    }
#endif
    if constexpr (BITS == 16) {
      acc = t;
    } else {
      if constexpr (BITS == 4) {   // remove the folded offsets of this group (deq_int4_raw)
        const f32x4 cr = *(const f32x4*)(corr + kt * 16 + 4 * kq);
        t -= cr;
      }
      const float sc = h2f(sl[(ct * KT + kt) * 16 + r]);
      acc[0] = fmaf(sc, t[0], acc[0]);
      acc[1] = fmaf(sc, t[1], acc[1]);
      acc[2] = fmaf(sc, t[2], acc[2]);
      acc[3] = fmaf(sc, t[3], acc[3]);
    }
    }   // !G32
    // the tile's last item lands in its slab, every other item in the dummy slab
    const bool last = ++ck == KW;
    my_slab[(last ? ct : ntl) * kSlabStride] = acc;
    if (last) acc = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
    ck = last ? 0 : ck;
    ct += last ? 1 : 0;
  };
  int j0 = 0;
#if TI_GEMV_SYNC > 0
  // Waves of a CU drift apart (the oldest wins issue arbitration); a workgroup barrier every
  // TI_GEMV_SYNC blocks keeps them together while every wave still has blocks left (the
  // count of barriers is the same for all waves: blocks below the smallest wave total).
  const int common = ntl * (KT / kGemvWaves);
  int blk = 0;
  for (; j0 + R <= common; j0 += R) {
#pragma unroll
    for (int s = 0; s < R; ++s) {
      item(ring[s]);
      const size_t o = refill_off();
#pragma unroll
      for (int c = 0; c < C; ++c) ring[s][c] = ld_w(tb + o + c * kWave);
    }
    if (++blk == TI_GEMV_SYNC) {
      blk = 0;
      __builtin_amdgcn_s_barrier();
    }
  }
#endif
  for (; j0 + R <= total; j0 += R) {   // full blocks: no branches, R items scheduled together
#pragma unroll
    for (int s = 0; s < R; ++s) {
      item(ring[s]);
      const size_t o = refill_off();   // refill this slot R items ahead (clamped past the end)
#pragma unroll
      for (int c = 0; c < C; ++c) ring[s][c] = ld_w(tb + o + c * kWave);
    }
  }
#pragma unroll
  for (int s = 0; s < R; ++s)          // tail: the last total % R items, nothing refilled
    if (j0 + s < total) item(ring[s]);
  if (KW == 0)   // K < 8*128: this wave owns no k-tiles; its partials are zero
    for (int tl = 0; tl < ntl; ++tl) my_slab[tl * kSlabStride] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};

  GEMV_TS(3);
  GEMV_WTS();
  STAMP_MARK(ph_streamed);
  // ---- 5. epilogue inputs into LDS, reduce the 8 partials per tile, epilogue
  if (tid < n_res) es[tid] = pre;
  if (fold && tid < n_res) es[n_res + tid] = fw_pre;
  if (tid < n_cs) es[tid] = cs_reg;
  // inputs past the one-per-thread prefetch (ntl * M * 16 or M * head_dim > 512): loaded now
  for (int i = tid + kGemvThreads; i < n_res; i += kGemvThreads) {
    const int tl = i / (a.M * 16), rem = i - tl * a.M * 16, m = rem >> 4, n = rem & 15;
    es[i] = p_pre[(size_t)m * ldo + (t0 + tl) * 16 + n];
    if (fold) es[n_res + i] = a.epi.fold_w[(size_t)t0 * 16 + i];
  }
  // XM_F16F: rms of the row from the producer's partials, the same fixed-order sum in every
  // wave (rms_norm, tensor_engine.cpp:1488-1505, with the division moved behind the GEMM)
  float rms = 1.0f;
  if constexpr (XM == XM_F16F) {
    float t = 0.0f;
#pragma unroll
    for (int j = 0; j < 4; ++j) t += lane + 64 * j < n_ss ? ss4[j] : 0.0f;
    t = group_sum<kWave>(t);
    rms = sqrtf(t / (float)a.K + a.eps);
  }
  float ssacc = 0.0f;
  const float* fw_l = es + n_res;
  for (int i = tid + kGemvThreads; i < n_cs; i += kGemvThreads) {
    const int hd = a.epi.head_dim, m = i / hd, j = i - m * hd;
    es[i] = a.epi.rope_cs[(size_t)((const int*)(es + a.M * hd))[m] * hd + j];
  }
  lds_barrier();
  GEMV_TS(5);
  STAMP_MARK(ph_reduce);
  unsigned long long best[4] = {0ull, 0ull, 0ull, 0ull};
  if (a.M <= 4) {
    // rows m < 4 live in lanes 0-15 of each partial (C layout m = 4*(l>>4) + i): one thread per
    // (tile, n), all tiles in one pass over the workgroup, the M components of its f32x4.
    for (int tb0 = wave * kWave; tb0 < ntl * 16; tb0 += kGemvThreads) {
      const int t = tb0 + lane, ok = t < ntl * 16, tl = ok ? t >> 4 : 0, n = lane & 15;
      const f32x4* sp = slab + tl * kSlabStride + n;
      f32x4 v = sp[0];
#pragma unroll
      for (int w = 1; w < kGemvWaves; ++w) v += sp[w * kWave];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (i < a.M) epilogue(a, t0 + tl, tl, n, i, XM == XM_F16F ? v[i] / rms : v[i], es, best[i], ok, fw_l, ssacc);
    }
  } else {
    const int i4 = wave & 3;
    for (int tl = wave >> 2; tl < ntl; tl += 2) {
      const float* sp = (const float*)(slab + tl * kSlabStride + lane) + i4;
      float v = 0.0f;
#pragma unroll
      for (int w = 0; w < kGemvWaves; ++w) v += sp[w * kWave * 4];
      epilogue(a, t0 + tl, tl, lane, i4, v, es, best[0], true, fw_l, ssacc);
    }
  }
  STAMP_MARK(ph_epi);
  if (a.epi.kind == TI_EPI_LOGITS_ARGMAX) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        const unsigned long long other = __shfl_xor(best[i], o, kWave);
        best[i] = other > best[i] ? other : best[i];
      }
    }
    if (a.M <= 4) {
      if ((lane & 15) == 0)
#pragma unroll
        for (int i = 0; i < 4; ++i)   // constant bounds: best[] stays in registers
          if (i < a.M && best[i]) atomicMax(best_l + i, best[i]);
    } else {
      const int m = 4 * (lane >> 4) + (wave & 3);
      if ((lane & 15) == 0 && m < a.M && best[0]) atomicMax(best_l + m, best[0]);
    }
    lds_barrier();
    if (tid < a.M && best_l[tid])
      atomicMax(a.epi.argmax + (size_t)tid * TI_ARGMAX_SLOTS + (bid & (TI_ARGMAX_SLOTS - 1)), best_l[tid]);
    if (a.epi.step_ctr && bid == 0 && tid == 0) *a.epi.step_ctr += a.epi.advance;
  }
  if (fold && a.M <= 4 && ntl * 16 <= kWave) {
    // every output of the workgroup was wave 0's (the M <= 4 epilogue above): its sum alone, no
    // barrier -- the same value as the general form below, whose other terms are exact zeros
    if (wave == 0) {
      const float sw = group_sum<kWave>(ssacc);
      if (lane == 0) a.epi.fold_ss[bid] = sw;
    }
  } else if (fold) {   // this workgroup's sum of h^2, waves in a fixed order (best_l: unused by RESID)
    float* red2 = (float*)best_l;
    const float sw = group_sum<kWave>(ssacc);
    if (lane == 0) red2[wave] = sw;
    lds_barrier();
    if (tid == 0) {
      float t = 0.0f;
#pragma unroll
      for (int w = 0; w < kGemvWaves; ++w) t += red2[w];
      a.epi.fold_ss[bid] = t;
    }
  }
  GEMV_TS(4);
  stamp_end(a.stamp, t_entry, ph_issued, ph_staged, ph_stream, ph_streamed, ph_reduce, ph_epi, ph_streamed);
}

// ================================================================= batched rows
// gemv_mb_kernel<MB, NTL>: int4 weights x fp16 activations for M <= 16*MB rows (MB <= 2):
// the batched decode of generate_batch (inference_engine.cpp:804-828), and
// long-K projections whose activation rows no longer fit gemv_wq_kernel's LDS image.
// Weights are still read once per launch, straight into registers; the activations are
// staged in k-chunks of 1024 (8 k-tiles, one per wave):
//   * a chunk of all rows is copied by LDS-DMA (global_load_lds_dwordx4: every wave
//     instruction one contiguous KiB of a row) into one of two LDS buffers, one chunk ahead;
//   * item order per wave: chunk c (k-tile 8c + wave) x tile tl; the NTL tiles' weights of
//     chunk c + 1 are loaded into the other register buffer while chunk c computes (the chunk
//     loop unrolled by two), and one barrier per chunk hands the x buffers over;
//   * per 32-k step one dequantized weight fragment feeds MB MFMAs (one per 16-row block);
//     nibble offsets are removed in the dequant (x is used as staged);
//   * k-tiles past K (the last chunk) and the dummy tile of workgroups with NTL - 1 tiles use
//     clamped addresses and a zero scale.
// After the stream the waves' blocks are summed in a fixed order through LDS (the x buffers
// are reused) and the same epilogue kinds run, their inputs read from global.
constexpr int kMbChunkK = 1024;
constexpr int kMbXs = kMbChunkK + 8;   // LDS row (halfs): 516 dwords = 4 mod 64 banks, conflict-free A reads

__host__ __device__ inline int mb_xbuf_bytes(int MB) { return align16(2 * 16 * MB * kMbXs * 2); }
__host__ __device__ inline int mb_lds_bytes(int MB, int ntl, int K) {
  const int x = mb_xbuf_bytes(MB), slab = align16(ntl * MB * kGemvWaves * kWave * 16);
  return (x > slab ? x : slab) + align16(ntl * (K >> 7) * 32);
}

__device__ __forceinline__ f16x8 deq_int4_signed(uint32_t w, uint32_t magic) {
  const f16x8 r = deq_int4_raw(w, magic);   // lanes (1024 + n) and (1024 + 16 n)
  const f16x2 lo_off = {(f16)-1032.0f, (f16)-1032.0f}, hi_mul = {(f16)0.0625f, (f16)0.0625f},
              hi_off = {(f16)-72.0f, (f16)-72.0f};
  // (1024 + 16 n) / 16 - 72 = n - 8 exactly: one v_pk_fma_f16 (the build's -ffp-contract=off
  // would otherwise split it into a multiply and an add)
  const f16x2 a = (f16x2){r[0], r[1]} + lo_off, b = __builtin_elementwise_fma((f16x2){r[2], r[3]}, hi_mul, hi_off);
  const f16x2 c = (f16x2){r[4], r[5]} + lo_off, d = __builtin_elementwise_fma((f16x2){r[6], r[7]}, hi_mul, hi_off);
  return (f16x8){a[0], a[1], b[0], b[1], c[0], c[1], d[0], d[1]};
}

// Epilogue of one output y[m][nt*16 + n]; the inputs gemv_wq_kernel stages in LDS are read
// from global.  Shuffle partners (n ^ 1, n + 8) are lanes of the same 16-lane group.
__device__ __forceinline__ void epilogue_mb(const GemvArgs& a, int nt, int m, int n, float v, bool live) {
  const ti_epilogue& e = a.epi;
  const int ng = nt * 16 + n;
  switch (e.kind) {
    case TI_EPI_STORE_F32:
      if (live) ((float*)e.out)[(size_t)m * e.ldo + ng] = v;
      break;
    case TI_EPI_STORE_F16:
      if (live)
        ((uint16_t*)e.out)[e.out_packed ? TI_PACKED_INDEX(m, ng, e.ldo >> 7) : (size_t)m * e.ldo + ng] = f2h(v);
      break;
    case TI_EPI_RESID_F32:
      if (live) {
        float* o = (float*)e.out + (size_t)m * e.ldo + ng;
        *o = *o + v;
      }
      break;
    case TI_EPI_SILU_MUL_F16: {
      const float up = __shfl_down(v, 8, kWave);
      if (live && n < 8) {
        const float s = v / (1.0f + expf(-v));
        const int j = nt * 8 + n;
        ((uint16_t*)e.out)[e.out_packed ? TI_PACKED_INDEX(m, j, e.ldo >> 7) : (size_t)m * e.ldo + j] = f2h(up * s);
      }
      break;
    }
    case TI_EPI_QKV_ROPE_KV: {
      const float partner = __shfl_xor(v, 1, kWave);
      if (!live) break;
      const int hd = e.head_dim, p = e.pos[m];
      if (ng < e.q_dim + e.kv_dim) {
        const int base = ng < e.q_dim ? 0 : e.q_dim;
        const int d = (ng - base) % hd;
        const float2 cs = *(const float2*)(e.rope_cs + (size_t)p * hd + (d & ~1));
        const float r = (d & 1) == 0 ? fmaf(-partner, cs.y, v * cs.x) : fmaf(v, cs.x, partner * cs.y);
        if (ng < e.q_dim) {
          ((float*)e.out)[(size_t)m * e.ldo + ng] = r;
        } else {
          const int kvh = (ng - e.q_dim) / hd;
          e.k_cache[(size_t)m * e.kv_stream_stride + ((size_t)kvh * e.max_seq + p) * hd + d] = f2h(r);
        }
      } else {
        const int c = ng - e.q_dim - e.kv_dim;
        const int kvh = c / hd, d = c - kvh * hd;
        e.v_cache[(size_t)m * e.kv_stream_stride + ((size_t)kvh * e.max_seq + p) * hd + d] = f2h(v);
      }
      break;
    }
    case TI_EPI_LOGITS_ARGMAX: {
      unsigned long long key = 0ull;
      if (live) {
        ((float*)e.out)[(size_t)m * e.ldo + ng] = v;
        key = ((unsigned long long)float_order_key(v) << 32) | (unsigned long long)(0xFFFFFFFFu - (uint32_t)ng);
      }
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        const unsigned long long other = __shfl_xor(key, o, kWave);
        key = other > key ? other : key;
      }
      if (n == 0 && key) atomicMax(e.argmax + (size_t)m * TI_ARGMAX_SLOTS + (blockIdx.x & (TI_ARGMAX_SLOTS - 1)), key);
      break;
    }
    default:
      break;
  }
}

__device__ __forceinline__ void dma_1k(const void* src_lane, void* lds_wave) {   // 64 lanes x 16 B -> LDS
  __builtin_amdgcn_global_load_lds(src_lane, lds_wave, 16, 0, 0);
}

template <int MB, int NTL>
__device__ __forceinline__ void gemv_mb_body(const GemvArgs a, int grid);
template <int MB, int NTL>
__global__ __launch_bounds__(kGemvThreads, 1) void gemv_mb_kernel(const GemvArgs a, int grid) {
  const unsigned long long t_entry = stamp_now();
  gemv_mb_body<MB, NTL>(a, grid);
  stamp_end(a.stamp, t_entry);
}
template <int MB, int NTL>
__device__ __forceinline__ void gemv_mb_body(const GemvArgs a, int grid) {
  constexpr int XDMA = 2 * 16 * MB / kGemvWaves;   // x-chunk DMA instructions per wave (2 per row)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int KT = a.K >> 7, NT = a.N >> 4, NC = (KT + kGemvWaves - 1) / kGemvWaves;
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 15, kq = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int t0 = (int)(blockIdx.x * (unsigned)NT / (unsigned)grid);
  const int t1 = (int)((blockIdx.x + 1) * (unsigned)NT / (unsigned)grid);
  const int ntl = t1 - t0;                           // NTL or NTL - 1
  f16* xb = (f16*)smem;                              // [2][16 MB][kMbXs]
  const int xslab = mb_xbuf_bytes(MB) > align16(NTL * MB * kGemvWaves * kWave * 16)
                        ? mb_xbuf_bytes(MB) : align16(NTL * MB * kGemvWaves * kWave * 16);
  f32x4* slab = (f32x4*)smem;                        // after the stream: [NTL][MB][8][64]
  uint16_t* sl = (uint16_t*)(smem + xslab);          // [ntl][KT][16]

  // scales of our tiles first (two pieces per thread cover ntl * KT <= 512 groups)
  const int n_sc = ntl * KT * 2;
  const u32x4* sg = (const u32x4*)(a.scales + (size_t)t0 * KT * 16);
  const u32x4 sc0 = ld_w(sg + (tid < n_sc ? tid : 0));
  const u32x4 sc1 = ld_w(sg + (tid + kGemvThreads < n_sc ? tid + kGemvThreads : 0));

  const f16* xg = (const f16*)a.x;
  auto issue_x = [&](int c) {   // chunk c of every row into buffer c & 1 (rows >= M repeat row M-1)
#pragma unroll
    for (int q = 0; q < XDMA; ++q) {
      const int piece = wave * XDMA + q, row = piece >> 1, half = piece & 1;
      const int m = row < a.M ? row : a.M - 1;
      int k = c * kMbChunkK + half * 512 + lane * 8;
      k = k < a.K ? k : a.K - 8;
#if TI_GEMV_EXP & 8   // diagnostic: no activation traffic (the first chunk only)
      if (c > 0) continue;
#endif
      dma_1k(xg + (size_t)m * a.ldx + k, xb + ((c & 1) * 16 * MB + row) * kMbXs + half * 512);
    }
  };
  const u32x4* tb = a.tiles + lane;
  auto load = [&](u32x4 (&w)[NTL], int c) {
#if TI_GEMV_EXP & 32  // diagnostic: no weight traffic (the first chunk's weights re-used)
    c = 0;
#endif
    const int kt = min(c * kGemvWaves + wave, KT - 1);
#pragma unroll
    for (int tl = 0; tl < NTL; ++tl) w[tl] = ld_w(tb + ((size_t)(t0 + min(tl, ntl - 1)) * KT + kt) * kWave);
  };
  u32x4 B0[NTL], B1[NTL];
  issue_x(0);
  load(B0, 0);
  if (tid < n_sc) ((u32x4*)sl)[tid] = sc0;
  if (tid + kGemvThreads < n_sc) ((u32x4*)sl)[tid + kGemvThreads] = sc1;
  asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NTL) : "memory");   // x chunk 0 landed (B0 may fly)
  lds_barrier();

  f32x4 acc[NTL][MB];
#pragma unroll
  for (int t = 0; t < NTL; ++t)
#pragma unroll
    for (int b = 0; b < MB; ++b) acc[t][b] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
  uint32_t magic;
  asm volatile("v_mov_b32 %0, 0x64006400" : "=v"(magic));
  auto compute = [&](const u32x4 (&w)[NTL], int c) {
    const int kt = c * kGemvWaves + wave;
    const bool kvalid = kt < KT;
    const f16* xr = xb + ((c & 1) * 16 * MB + r) * kMbXs + wave * 128 + kq * 32;   // the tile's k order
    f16x8 xf[MB][4];
#pragma unroll
    for (int b = 0; b < MB; ++b)
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) xf[b][s4] = *(const f16x8*)(xr + b * 16 * kMbXs + s4 * 8);
#pragma unroll
    for (int tl = 0; tl < NTL; ++tl) {
      f32x4 t[MB];
#pragma unroll
      for (int b = 0; b < MB; ++b) t[b] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        const f16x8 bf = deq_int4_signed(w[tl][s4], magic);
#pragma unroll
        for (int b = 0; b < MB; ++b) t[b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xf[b][s4], bf, t[b], 0, 0, 0);
      }
      const float sc = kvalid ? h2f(sl[(min(tl, ntl - 1) * KT + kt) * 16 + r]) : 0.0f;
#pragma unroll
      for (int b = 0; b < MB; ++b) {
        acc[tl][b][0] = fmaf(sc, t[b][0], acc[tl][b][0]);
        acc[tl][b][1] = fmaf(sc, t[b][1], acc[tl][b][1]);
        acc[tl][b][2] = fmaf(sc, t[b][2], acc[tl][b][2]);
        acc[tl][b][3] = fmaf(sc, t[b][3], acc[tl][b][3]);
      }
    }
  };
  // Per chunk: DMA the next x chunk into the other buffer, load the next weights, compute,
  // wait for our DMA (the NTL weight loads after it may still fly), barrier.  Reloads past the
  // end are clamped and harmless; the tail computes load nothing.
  int c = 0;
  for (; c + 1 < NC; c += 2) {
    issue_x(c + 1);
    load(B1, c + 1);
    compute(B0, c);
    asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NTL) : "memory");
    lds_barrier();
    issue_x(c + 2 < NC ? c + 2 : NC - 1);
    load(B0, c + 2 < NC ? c + 2 : NC - 1);
    compute(B1, c + 1);
    asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NTL) : "memory");
    lds_barrier();
  }
  if (c < NC) compute(B0, c);

  // ---- sum the 8 waves' blocks in a fixed order, then the epilogue
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // clamped reloads / DMA done before the slab reuses LDS
  lds_barrier();
#pragma unroll
  for (int tl = 0; tl < NTL; ++tl)
#pragma unroll
    for (int b = 0; b < MB; ++b) slab[((tl * MB + b) * kGemvWaves + wave) * kWave + lane] = acc[tl][b];
  lds_barrier();
  const int n = lane & 15, nblk = ntl * MB * 4;
  const int nblk_pad = (nblk + kGemvWaves - 1) / kGemvWaves * kGemvWaves;
  for (int cb = wave; cb < nblk_pad; cb += kGemvWaves) {   // wave-uniform trip count (shuffles inside)
    const bool ok = cb < nblk;
    const int cbc = ok ? cb : 0, tl = cbc / (MB * 4), b = (cbc >> 2) % MB, i = cbc & 3;
    const float* sp = (const float*)(slab + (tl * MB + b) * kGemvWaves * kWave + lane) + i;
    float v = 0.0f;
#pragma unroll
    for (int w = 0; w < kGemvWaves; ++w) v += sp[w * kWave * 4];
    const int m = b * 16 + 4 * (lane >> 4) + i;
    epilogue_mb(a, t0 + tl, m, n, v, ok && m < a.M);
  }
  if (a.epi.kind == TI_EPI_LOGITS_ARGMAX && a.epi.step_ctr && blockIdx.x == 0 && tid == 0)
    *a.epi.step_ctr += a.epi.advance;
}

__host__ __device__ inline int mbr_slab_bytes(int MB, int ntl) { return align16(ntl * MB * kGemvWaves * kWave * 16); }
__host__ __device__ inline int mbr_lds_bytes(int MB, int ntl, int K) {
  return mbr_slab_bytes(MB, ntl) + align16(ntl * (K >> 7) * 32);
}

template <int MB, int NTL>
struct MbrChunk {       // one chunk's operands of one wave
  u32x4 w[NTL];        // packed int4 weights of (tile tl, this wave's k-tile)
  f16x8 x[MB][4];      // A fragments: rows 16 b + (lane & 15), k = kt*128 + 32 (lane >> 4) + 8 s4
};

// Register-fragment variant (one 16-row block): each wave loads the A fragments of its own
// k-tile straight into registers, one chunk ahead, so no barrier is needed until the end;
// at <= 16 rows this beats the LDS-staged kernel (bench.py --batch 8/16).
template <int MB, int NTL>
__device__ __forceinline__ void gemv_mbr_body(const GemvArgs a, int grid);
template <int MB, int NTL>
__global__ __launch_bounds__(kGemvThreads, 1) void gemv_mbr_kernel(const GemvArgs a, int grid) {
  const unsigned long long t_entry = stamp_now();
  gemv_mbr_body<MB, NTL>(a, grid);
  stamp_end(a.stamp, t_entry);
}
template <int MB, int NTL>
__device__ __forceinline__ void gemv_mbr_body(const GemvArgs a, int grid) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int KT = a.K >> 7, NT = a.N >> 4, NC = (KT + kGemvWaves - 1) / kGemvWaves;
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 15, kq = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int t0 = (int)(blockIdx.x * (unsigned)NT / (unsigned)grid);
  const int t1 = (int)((blockIdx.x + 1) * (unsigned)NT / (unsigned)grid);
  const int ntl = t1 - t0;                           // NTL or NTL - 1
  f32x4* slab = (f32x4*)smem;                        // after the stream: [NTL][MB][8][64]
  uint16_t* sl = (uint16_t*)(smem + mbr_slab_bytes(MB, NTL));   // [ntl][KT][16]

  // scales of our tiles: loaded first (two pieces per thread cover ntl * KT <= 512 groups)
  const int n_sc = ntl * KT * 2;
  const u32x4* sg = (const u32x4*)(a.scales + (size_t)t0 * KT * 16);
  const u32x4 sc0 = ld_w(sg + (tid < n_sc ? tid : 0));
  const u32x4 sc1 = ld_w(sg + (tid + kGemvThreads < n_sc ? tid + kGemvThreads : 0));

  const f16* xg = (const f16*)a.x;
  const u32x4* tb = a.tiles + lane;
  auto load = [&](MbrChunk<MB, NTL>& ch, int c) {
    const int kt = min(c * kGemvWaves + wave, KT - 1);
#pragma unroll
    for (int tl = 0; tl < NTL; ++tl) ch.w[tl] = ld_w(tb + ((size_t)(t0 + min(tl, ntl - 1)) * KT + kt) * kWave);
#pragma unroll
    for (int b = 0; b < MB; ++b) {
      const int m = min(b * 16 + r, a.M - 1);
      const f16* xr = xg + (size_t)m * a.ldx + kt * 128 + kq * 32;   // the tile's k order (B fragments)
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) ch.x[b][s4] = *(const f16x8*)(xr + s4 * 8);
    }
  };
  MbrChunk<MB, NTL> B0, B1;
  load(B0, 0);
  if (tid < n_sc) ((u32x4*)sl)[tid] = sc0;
  if (tid + kGemvThreads < n_sc) ((u32x4*)sl)[tid + kGemvThreads] = sc1;
  lds_barrier();

  f32x4 acc[NTL][MB];
#pragma unroll
  for (int t = 0; t < NTL; ++t)
#pragma unroll
    for (int b = 0; b < MB; ++b) acc[t][b] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
  uint32_t magic;
  asm volatile("v_mov_b32 %0, 0x64006400" : "=v"(magic));
  auto compute = [&](const MbrChunk<MB, NTL>& ch, int c) {
    const int kt = c * kGemvWaves + wave;
    const bool kvalid = kt < KT;
#pragma unroll
    for (int tl = 0; tl < NTL; ++tl) {
      f32x4 t[MB];
#pragma unroll
      for (int b = 0; b < MB; ++b) t[b] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        const f16x8 bf = deq_int4_signed(ch.w[tl][s4], magic);
#pragma unroll
        for (int b = 0; b < MB; ++b) t[b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ch.x[b][s4], bf, t[b], 0, 0, 0);
      }
      const float sc = kvalid ? h2f(sl[(min(tl, ntl - 1) * KT + kt) * 16 + r]) : 0.0f;
#pragma unroll
      for (int b = 0; b < MB; ++b) {
        acc[tl][b][0] = fmaf(sc, t[b][0], acc[tl][b][0]);
        acc[tl][b][1] = fmaf(sc, t[b][1], acc[tl][b][1]);
        acc[tl][b][2] = fmaf(sc, t[b][2], acc[tl][b][2]);
        acc[tl][b][3] = fmaf(sc, t[b][3], acc[tl][b][3]);
      }
    }
  };
  // chunks two at a time, each loaded one chunk ahead (the reload past the end is harmless)
  int c = 0;
  for (; c + 1 < NC; c += 2) {
    load(B1, c + 1);
    compute(B0, c);
    load(B0, c + 2 < NC ? c + 2 : NC - 1);
    compute(B1, c + 1);
  }
  if (c < NC) compute(B0, c);

  // ---- sum the 8 waves' blocks in a fixed order, then the epilogue
#pragma unroll
  for (int tl = 0; tl < NTL; ++tl)
#pragma unroll
    for (int b = 0; b < MB; ++b) slab[((tl * MB + b) * kGemvWaves + wave) * kWave + lane] = acc[tl][b];
  lds_barrier();
  const int n = lane & 15, nblk = ntl * MB * 4;
  const int nblk_pad = (nblk + kGemvWaves - 1) / kGemvWaves * kGemvWaves;
  for (int cb = wave; cb < nblk_pad; cb += kGemvWaves) {   // wave-uniform trip count (shuffles inside)
    const bool ok = cb < nblk;
    const int cbc = ok ? cb : 0, tl = cbc / (MB * 4), b = (cbc >> 2) % MB, i = cbc & 3;
    const float* sp = (const float*)(slab + (tl * MB + b) * kGemvWaves * kWave + lane) + i;
    float v = 0.0f;
#pragma unroll
    for (int w = 0; w < kGemvWaves; ++w) v += sp[w * kWave * 4];
    const int m = b * 16 + 4 * (lane >> 4) + i;
    epilogue_mb(a, t0 + tl, m, n, v, ok && m < a.M);
  }
  if (a.epi.kind == TI_EPI_LOGITS_ARGMAX && a.epi.step_ctr && blockIdx.x == 0 && tid == 0)
    *a.epi.step_ctr += a.epi.advance;
}

// ------------------------------------------------------------- rows kernel (17..64 rows)
// Batched decode at configs[3] / [4] scale (64 / 32 streams): the weights are still read once
// per launch, but every weight fragment now meets up to 64 rows.  Register operands, no LDS in
// the stream: the 8 waves form RG row groups of 8 / RG waves; a group owns MB 16-row blocks
// and splits the k-tiles over its waves (k-tile w, w + 8 / RG, ...).  Per item a wave holds
// the packed weights of the workgroup's NTL tiles at that k-tile (a WD-slot ring, issued
// WD - 1 items ahead: HBM latency) and its rows' x fragments (two slots, one item ahead: L2
// latency).  The item count is padded to a multiple of WD with zero-scale clamped items, so
// the loop body has no branches (no vmcnt(0) at a join).  After the stream the partial blocks
// of the group's waves are summed in a fixed order through LDS and the epilogue runs.
template <int MB, int NTL, int RG, bool XP = false>
struct RowsCfg {
  static constexpr int kGroupWaves = kGemvWaves / RG;
  static constexpr int kWD = MB * NTL <= 3 ? 4 : 3;   // ring slots (VGPR budget: no spills)
};
__host__ __device__ inline int rows_slab_bytes(int mb_total, int ntl) {
  return align16(ntl * mb_total * kGemvWaves * kWave * 16);
}
// batched fold (ti_hip.h TI_FOLD_SS_ROWS): per-thread partial sums [512] | 1 / rms per row [64] |
// per-tile sums of h^2 per row [4][64], behind the slab and the scales
constexpr int kFoldLdsBytes = 4096;
__host__ __device__ inline int rows_fold_offset(int mb_total, int ntl, int K, bool g32 = false) {
  return rows_slab_bytes(mb_total, ntl) + align16(ntl * (K >> 7) * 32 * (g32 ? 4 : 1));
}
__host__ __device__ inline int rows_lds_bytes(int mb_total, int ntl, int K, bool g32 = false) {
  return rows_fold_offset(mb_total, ntl, K, g32) + kFoldLdsBytes;
}

// Batched fold, consumer side: this thread's share of row `row`'s partial sums of h^2 (rows
// of R per workgroup, 512 / R threads per row taking partials part, part + P, ...; loads issued
// 8 at a time, summed in partial order).  fold_rms_finish turns the shares into rms per row.
__device__ __forceinline__ float fold_share(const GemvArgs& a, int m, int part, int P) {
  float t = 0.0f;
  if (m >= a.M) return t;
  const float* ss = a.epi.ss_in + m;
  for (int b0 = part; b0 < a.epi.n_ss; b0 += 8 * P) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = b0 + j * P < a.epi.n_ss ? ss[(size_t)(b0 + j * P) * TI_FOLD_SS_ROWS] : 0.0f;
#pragma unroll
    for (int j = 0; j < 8; ++j) t += v[j];
  }
  return t;
}
// part[512] holds every thread's share (thread = part * R + row); rms[row] = sqrt(sum / K + eps)
// (the M == 1 fold's formula, gemv_wq_kernel XM_F16F).  Call between two workgroup barriers.
__device__ __forceinline__ void fold_rms_finish(const GemvArgs& a, const float* part, float* rms, int R, int tid) {
  if (tid < R) {
    float t = 0.0f;
    for (int p = 0; p < kGemvThreads / R; ++p) t += part[p * R + tid];
    rms[tid] = sqrtf(t / (float)a.K + a.eps);
  }
}

// Workgroups: n_cg column groups x n_rb row blocks of 16 RG MB rows (narrow outputs split the
// rows: a workgroup's activation bytes shrink with its rows, and its column group's weights are
// re-read by the other row blocks from the same XCD's L2 -- blockIdx % 8 is the column group's
// low bits, a speed placement only).
// G32: group-32 int4 tiles (GGUF Q4_0 blocks, TI_BITS_G32; row-major x only): MFMA step s4 of a
// k-tile reads k-chunk 32 s4 + 8 kq and is scaled by its own block's scale (4 per tile row and
// k-tile), as in the fused and tile kernels.
template <int MB, int NTL, int RG, bool XP, bool G32>
__device__ __forceinline__ void gemm_rows_body(const GemvArgs a, int n_cg, int n_rb);
template <int MB, int NTL, int RG, bool XP, bool G32 = false>
__global__ __launch_bounds__(kGemvThreads, 1) void gemm_rows_kernel(const GemvArgs a, int n_cg, int n_rb) {
  const unsigned long long t_entry = stamp_now();
  gemm_rows_body<MB, NTL, RG, XP, G32>(a, n_cg, n_rb);
  stamp_end(a.stamp, t_entry);
}
template <int MB, int NTL, int RG, bool XP, bool G32>
__device__ __forceinline__ void gemm_rows_body(const GemvArgs a, int n_cg, int n_rb) {
  static_assert(!(XP && G32), "group-32 rows take row-major activations");
  constexpr int SG = G32 ? 4 : 1;   // scales per tile row and k-tile
  constexpr int GW = RowsCfg<MB, NTL, RG>::kGroupWaves, WD = RowsCfg<MB, NTL, RG>::kWD;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int KT = a.K >> 7, NT = a.N >> 4;
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 15, kq = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave / GW, gw = wave % GW;
  const int rest = blockIdx.x >> 3, rb = rest % n_rb, cg = (rest / n_rb) * 8 + (blockIdx.x & 7);
  if (cg >= n_cg) return;
  const int b0 = rb * RG * MB;                       // first 16-row block of this workgroup
  const int t0 = (int)(cg * (unsigned)NT / (unsigned)n_cg);
  const int t1 = (int)((cg + 1) * (unsigned)NT / (unsigned)n_cg);
  const int ntl = t1 - t0;                           // NTL or NTL - 1
  const int NI = (KT + GW - 1) / GW, NIP = (NI + WD - 1) / WD * WD;
  ROWS_TS(0);
  f32x4* slab = (f32x4*)smem;                        // after the stream: [NTL][RG * MB][8][64]
  uint16_t* sl = (uint16_t*)(smem + rows_slab_bytes(RG * MB, NTL));   // [ntl][KT][SG][16]

  // the workgroup's group scales (ntl * KT * SG <= 512: 2 SG 16-byte pieces per thread), first
  const int n_sc = ntl * KT * 2 * SG;
  const u32x4* sg = (const u32x4*)(a.scales + (size_t)t0 * KT * 16 * SG);
  u32x4 scr[2];
  if constexpr (G32) {   // transposed to [ntl][KT][16 rows][4 blocks]: one 8-byte LDS read per tile and item
    for (int i = tid; i < n_sc; i += kGemvThreads) {
      const u32x4 v = ld_w(sg + i);
      const int rr0 = (i & 1) * 8, s4 = (i >> 1) & 3, tk = i >> 3;   // piece: 8 rows of block s4 of (tile, kt)
#pragma unroll
      for (int e = 0; e < 8; ++e) sl[(tk * 16 + rr0 + e) * 4 + s4] = (uint16_t)(v[e >> 1] >> (16 * (e & 1)));
    }
  } else {
#pragma unroll
    for (int j = 0; j < 2; ++j) scr[j] = ld_w(sg + (tid + j * kGemvThreads < n_sc ? tid + j * kGemvThreads : 0));
  }

  const f16* xg = (const f16*)a.x;
  const u32x4* tb = a.tiles + lane;
  auto kt_of = [&](int it) { return min(gw + GW * it, KT - 1); };
  auto load_w = [&](u32x4 (&w)[NTL], int it) {
#if TI_GEMV_EXP & 128   // diagnostic: no weight traffic after the first ring
    it = it < WD ? it : it % WD;
#endif
    const int kt = kt_of(it);
#pragma unroll
    for (int tl = 0; tl < NTL; ++tl) w[tl] = ld_w(tb + ((size_t)(t0 + min(tl, ntl - 1)) * KT + kt) * kWave);
  };
  auto load_x = [&](f16x8 (&x)[MB][4], int it) {
#if TI_GEMV_EXP & 256   // diagnostic: no activation traffic after the first ring
    it = it < WD ? it : it % WD;
#endif
    const int kt = kt_of(it);
#pragma unroll
    for (int b = 0; b < MB; ++b) {
      if constexpr (XP) {   // TI_X_F16_PACKED: one contiguous KiB per (block, s4)
        const int bb = min(b0 + grp * MB + b, (a.M - 1) >> 4);
        const f16* xp = xg + ((size_t)(bb * KT + kt) * 4) * 512 + lane * 8;
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) x[b][s4] = *(const f16x8*)(xp + s4 * 512);
      } else {
        const int m = min((b0 + grp * MB + b) * 16 + r, a.M - 1);
        // the tile's k order (A fragments): k = 128 kt + 32 kq + 8 s4 (+ e), group-32 32 s4 + 8 kq
        const f16* xr = xg + (size_t)m * a.ldx + kt * 128 + kq * (G32 ? 8 : 32);
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) x[b][s4] = *(const f16x8*)(xr + s4 * (G32 ? 32 : 8));
      }
    }
  };
  u32x4 W[WD][NTL];
  f16x8 X[WD][MB][4];
#pragma unroll
  for (int u = 0; u < WD - 1; ++u) {
    load_w(W[u], u);
    load_x(X[u], u);
  }
  // batched fold: the consumer's per-row rms shares (after the first ring loads: their wait
  // costs nothing the first item would not wait for), the producer's per-tile h^2 sums
  constexpr int R = 16 * RG * MB;
  float* fold_l = (float*)(smem + rows_fold_offset(RG * MB, NTL, a.K, G32));
  const bool fold_in = a.epi.ss_in != nullptr, fold_out = a.epi.kind == TI_EPI_RESID_F32 && a.epi.fold_x != nullptr;
  const float share = fold_in ? fold_share(a, b0 * 16 + tid % R, tid / R, kGemvThreads / R) : 0.0f;
  if constexpr (!G32) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
      if (tid + j * kGemvThreads < n_sc) ((u32x4*)sl)[tid + j * kGemvThreads] = scr[j];
  }
  lds_barrier();
  ROWS_TS(1);

  f32x4 acc[NTL][MB];
#pragma unroll
  for (int t = 0; t < NTL; ++t)
#pragma unroll
    for (int b = 0; b < MB; ++b) acc[t][b] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
  uint32_t magic;
  asm volatile("v_mov_b32 %0, 0x64006400" : "=v"(magic));
  auto compute = [&](const u32x4 (&w)[NTL], const f16x8 (&x)[MB][4], int it) {
    const int kt = gw + GW * it;
    const bool kvalid = kt < KT;
    const int ktc = kvalid ? kt : KT - 1;
#pragma unroll
    for (int tl = 0; tl < NTL; ++tl) {
      if constexpr (G32) {   // one scale per 32-k block: each MFMA step scaled on its own
        const uint2 s4p = *(const uint2*)(sl + ((min(tl, ntl - 1) * KT + ktc) * 16 + r) * 4);
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
          const f16x8 bf = deq_int4_signed(w[tl][s4], magic);
          f32x4 t[MB];
#pragma unroll
          for (int b = 0; b < MB; ++b)
            t[b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(x[b][s4], bf, (f32x4){0.0f, 0.0f, 0.0f, 0.0f}, 0, 0, 0);
          const uint32_t sp = s4 < 2 ? s4p.x : s4p.y;
          const float sc = kvalid ? h2f((uint16_t)(sp >> (16 * (s4 & 1)))) : 0.0f;
#pragma unroll
          for (int b = 0; b < MB; ++b) {
            acc[tl][b][0] = fmaf(sc, t[b][0], acc[tl][b][0]);
            acc[tl][b][1] = fmaf(sc, t[b][1], acc[tl][b][1]);
            acc[tl][b][2] = fmaf(sc, t[b][2], acc[tl][b][2]);
            acc[tl][b][3] = fmaf(sc, t[b][3], acc[tl][b][3]);
          }
        }
        continue;
      }
      f32x4 t[MB];
#pragma unroll
      for (int b = 0; b < MB; ++b) t[b] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        const f16x8 bf = deq_int4_signed(w[tl][s4], magic);
#pragma unroll
        for (int b = 0; b < MB; ++b) t[b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(x[b][s4], bf, t[b], 0, 0, 0);
      }
      const float sc = kvalid ? h2f(sl[(min(tl, ntl - 1) * KT + ktc) * 16 + r]) : 0.0f;
#pragma unroll
      for (int b = 0; b < MB; ++b) acc[tl][b] = fma_scale4(sc, t[b], acc[tl][b]);
    }
  };
  for (int i = 0; i < NIP; i += WD) {
#pragma unroll
    for (int u = 0; u < WD; ++u) {
      load_w(W[(u + WD - 1) % WD], i + u + WD - 1);  // WD - 1 items ahead (clamped past the end)
      load_x(X[(u + WD - 1) % WD], i + u + WD - 1);
      compute(W[u], X[u], i + u);
#if TI_GEMV_EXP & 4
      if (i + u == 0) ROWS_TS(2);
#endif
    }
  }
  ROWS_TS(3);

  // ---- sum each group's waves in a fixed order, then the epilogue
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  ROWS_TS(4);
#pragma unroll
  for (int tl = 0; tl < NTL; ++tl)
#pragma unroll
    for (int b = 0; b < MB; ++b) slab[((tl * RG * MB + grp * MB + b) * kGemvWaves + wave) * kWave + lane] = acc[tl][b];
  if (fold_in) fold_l[tid] = share;
  lds_barrier();
  if (fold_in) {
    fold_rms_finish(a, fold_l, fold_l + kGemvThreads, R, tid);
    lds_barrier();
  }
  const int n = lane & 15, nblk = ntl * RG * MB * 4;
  const int nblk_pad = (nblk + kGemvWaves - 1) / kGemvWaves * kGemvWaves;
  for (int cb = wave; cb < nblk_pad; cb += kGemvWaves) {   // wave-uniform trip count (shuffles inside)
    const bool ok = cb < nblk;
    const int cbc = ok ? cb : 0, tl = cbc / (RG * MB * 4), bb = (cbc >> 2) % (RG * MB), i = cbc & 3;
    const int g = bb / MB;
    const float* sp = (const float*)(slab + (tl * RG * MB + bb) * kGemvWaves * kWave + lane) + i;
    float v = 0.0f;
#pragma unroll
    for (int w = 0; w < GW; ++w) v += sp[(g * GW + w) * kWave * 4];
    const int rl = bb * 16 + 4 * (lane >> 4) + i, m = b0 * 16 + rl;
    if (fold_in) v = v / fold_l[kGemvThreads + rl];
    if (fold_out) {   // residual add + the next call's folded input (fp16(h * w), sum of h^2 per row)
      const ti_epilogue& e = a.epi;
      const int ng = (t0 + tl) * 16 + n;
      float hn = 0.0f;
      if (ok && m < a.M) {
        float* o = (float*)e.out + (size_t)m * e.ldo + ng;
        hn = *o + v;
        *o = hn;
        float p = hn * e.fold_w[ng];
        asm volatile("" : "+v"(p));   // fp16(fp32 product): no fused multiply-convert (one rounding less)
        e.fold_x[e.fold_packed ? TI_PACKED_INDEX(m, ng, e.ldo >> 7) : (size_t)m * e.ldo + ng] = f2h(p);
      }
      const float sq = group_sum<16>(hn * hn);
      if (ok && n == 0) fold_l[kGemvThreads + 64 + tl * 64 + rl] = sq;
      continue;
    }
    epilogue_mb(a, t0 + tl, m, n, v, ok && m < a.M);
  }
  if (fold_out) {   // this column group's sum of h^2 per row, tiles in order
    lds_barrier();
    if (tid < R && b0 * 16 + tid < a.M) {
      float t = 0.0f;
      for (int tl = 0; tl < ntl; ++tl) t += fold_l[kGemvThreads + 64 + tl * 64 + tid];
      a.epi.fold_ss[(size_t)cg * TI_FOLD_SS_ROWS + b0 * 16 + tid] = t;
    }
  }
  ROWS_TS(5);
  if (a.epi.kind == TI_EPI_LOGITS_ARGMAX && a.epi.step_ctr && blockIdx.x == 0 && tid == 0)
    *a.epi.step_ctr += a.epi.advance;
}

// ------------------------------------------------------------- tile kernel (>= 128 rows)
// Prefill (forward_pass over a prompt chunk, inference_engine.cpp:1429-1491) and very large
// batches: a classic LDS-tiled MFMA GEMM, compute-bound at these row counts.  One workgroup
// computes a 128-row x 128-column block; its 8 waves form 2 (rows) x 4 (columns) and each owns
// 64 rows x 2 weight tiles.  Per 128-k group: the activation block (128 rows x 128 k fp16,
// 32 KiB) arrives in LDS by LDS-DMA one group ahead (double buffer) -- each DMA instruction
// fetches 4 contiguous 256-byte row segments, its lanes' 16-byte chunks XOR-swizzled by row so
// the A-fragment reads are bank-conflict free -- and the waves' packed weights come straight
// into VGPRs from a ring three groups ahead.  Group scales of the workgroup's tiles sit in LDS.
// Per group and wave: 2 tiles dequantized (offset-free int4 -> fp16), 16 A fragments read,
// 32 v_mfma_f32_16x16x32_f16, then the fp32 group-scale FMA.  The workgroup grid is ordered so
// that the row blocks sharing a column block run on one XCD (blockIdx % 8), where its L2
// serves their common weight stream.
// WMR: row-waves per workgroup (2: 128 rows x 4 column-waves; 1: 64 rows x 8 column-waves, half
// the activation block and no weight tile loaded twice)
// XB: activation-block buffers (2: double buffer; 4: issued three groups ahead, when the LDS holds them)
// RB: 16-row blocks per row-wave (4: 64-row waves; 2: 32-row waves for calls of at most 32 rows,
// half the activation block per group)
__host__ __device__ inline int tile_lds_bytes(int K, int tpw, bool g32 = false, int wmr = 2, int xb = 2, int rb = 4) {
  const int n = xb * 16 * rb * wmr * 256 + align16((8 / wmr) * tpw * (K >> 7) * 32 * (g32 ? 4 : 1));
  // >= the epilogue's staging blocks (tile_epi_lds_bytes) + the batched fold's rms per row
  return n > 8 * 64 * 20 * 4 + 512 ? n : 8 * 64 * 20 * 4 + 512;
}

// TPW: weight tiles per wave (2: 128 columns per workgroup; 1: 64 columns, twice the workgroups
// for the narrow N = 4096 projections, which otherwise fill only 64 of 256 CUs at 256 rows;
// 4: 256 columns, half the activation bytes per MFMA, when the rows give enough workgroups;
// 3: 192 columns, e.g. the 7B QKV's 768 tiles at 64 rows as exactly 256 workgroups).
// G32: group-32 int4 tiles (TI_BITS_G32): MFMA step s4 of a group reads k-chunk 4 s4 + kq and
// carries its own scale (one per 32-k block), so each step's product is scaled separately.
#ifndef TI_TILE_ASM
// 1: both operand streams of the k-loop issued from inline asm (the activation block's LDS-DMA,
// the weight tiles' VGPR loads) with hand-counted waits.  Beside a builtin LDS-DMA hipcc's waitcnt
// pass cannot count the VGPR weight loads and drains vmcnt(0) before every group
// (cdna_hip_programming.md section 5, "Three .s-level traps" (b)); with only the DMA hidden its
// weight waits count the DMAs as older loads and cut the lookahead; with both hidden every group's
// loads stay in flight across the barrier as deep as the rings allow.
#define TI_TILE_ASM 1
#endif
#ifndef TI_TILE_WNT
#define TI_TILE_WNT 0   // weight tiles are re-read by the row blocks of a column block (L2): default policy
#endif
// A 16-byte VGPR load hipcc does not count (beside the asm DMA it could not count its own loads
// exactly either): the caller waits with a counted s_waitcnt and ties the destination ("+v")
// before any use (cdna_hip_programming.md 5.7, item 1, form ii).
__device__ __forceinline__ u32x4 ld_w_asm(const u32x4* p) {
  u32x4 v;
#if TI_TILE_WNT
  asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(v) : "v"(p) : "memory");
#else
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
#endif
  return v;
}

#if TI_GEMV_EXP & 16384   // diagnostic (tools/probe_tile.hip): per-wave cycles by loop phase
__device__ unsigned long long g_tile_cy[4096 * 8 * 8];   // [workgroup][wave][phase]
#define TILE_CY_DECL()                                \
  unsigned long long cy_acc[6] = {0, 0, 0, 0, 0, 0}; \
  unsigned long long cy_t = __builtin_readcyclecounter()
#define TILE_CY(i)                                           \
  do {                                                       \
    const unsigned long long t_ = __builtin_readcyclecounter(); \
    cy_acc[i] += t_ - cy_t;                                  \
    cy_t = t_;                                               \
  } while (0)
#define TILE_CY_STORE()                                                                          \
  do {                                                                                           \
    if (lane == 0)                                                                               \
      for (int i_ = 0; i_ < 6; ++i_) g_tile_cy[((size_t)blockIdx.x * 8 + wave) * 8 + i_] = cy_acc[i_]; \
  } while (0)
#else
#define TILE_CY_DECL() do { } while (0)
#define TILE_CY(i) do { } while (0)
#define TILE_CY_STORE() do { } while (0)
#endif

// Split-K merge of one wave's block (n_ks > 1): every k-slice's wave stores its fp32 partial
// block write-through into the workspace and adds to the block's ticket after its stores have
// drained; the last arriver reads the other slices back (sc1 loads, CH slices per round trip),
// sums the n_ks slices in slice order (deterministic whatever the arrival order), re-arms the
// ticket and runs the epilogue.  Workspace: ti_epilogue.splitk_ws (include/ti_hip.h).
template <int TPW>
__device__ __forceinline__ bool splitk_merge(const GemvArgs& a, f32x4 (&acc)[TPW][4], int wave_id, int n_waves, int ks,
                                             int n_ks, int lane) {
  char* ws = (char*)a.epi.splitk_ws;
  int32_t* ticket = (int32_t*)ws + wave_id;
  const __amdgpu_buffer_rsrc_t rs = sc1_rsrc(ws + TI_SPLITK_TICKET_BYTES);
  constexpr int kSlab = TPW * 4 * kWave * 16;   // bytes per wave and slice
  auto off = [&](int sl, int t, int b) {
    return (uint32_t)(((size_t)sl * n_waves + wave_id) * kSlab + (size_t)((t * 4 + b) * kWave + lane) * 16);
  };
#pragma unroll
  for (int t = 0; t < TPW; ++t)
#pragma unroll
    for (int b = 0; b < 4; ++b) __builtin_amdgcn_raw_buffer_store_b128(acc[t][b], rs, off(ks, t, b), 0, kAuxSc1Load);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  int arrived = 0;
  if (lane == 0) arrived = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  arrived = __builtin_amdgcn_readfirstlane(arrived);
  if (arrived != n_ks - 1) return false;
#if TI_GEMV_EXP & 1024   // diagnostic: no read-back (the last arriver keeps its own slice)
  if (lane == 0) __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return true;
#endif
  constexpr int CH = TPW >= 4 ? 1 : 4 / TPW;   // slices per round trip (VGPR budget)
  f32x4 sum[TPW][4];
#pragma unroll
  for (int t = 0; t < TPW; ++t)
#pragma unroll
    for (int b = 0; b < 4; ++b) sum[t][b] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
  for (int s0 = 0; s0 < n_ks; s0 += CH) {
    f32x4 ld[CH][TPW][4];
#pragma unroll
    for (int c = 0; c < CH; ++c)
#pragma unroll
      for (int t = 0; t < TPW; ++t)
#pragma unroll
        for (int b = 0; b < 4; ++b)
          ld[c][t][b] = __builtin_bit_cast(
              f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off(min(s0 + c, n_ks - 1), t, b), 0, kAuxSc1Load));
#pragma unroll
    for (int c = 0; c < CH; ++c)
      if (s0 + c < n_ks)
#pragma unroll
        for (int t = 0; t < TPW; ++t)
#pragma unroll
          for (int b = 0; b < 4; ++b) sum[t][b] += s0 + c == ks ? acc[t][b] : ld[c][t][b];
  }
#pragma unroll
  for (int t = 0; t < TPW; ++t)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[t][b] = sum[t][b];
  if (lane == 0) __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // re-arm
  return true;
}

#ifndef TI_TILE_PAIR
// asm pipeline with 4 activation buffers and one weight tile per wave: one barrier per pair of
// groups (0: per group).  tools/probe_tile: TPW 1 (O, down at 512 rows) 6-9 % fewer cycles,
// TPW 2-3 5 % more (the barrier's share stays, its per-pair wait doubles), so wider shapes keep
// one barrier per group.
#define TI_TILE_PAIR 1
#endif
#ifndef TI_TILE_EPI_LDS
#define TI_TILE_EPI_LDS 1   // 0: every epilogue per element from the MFMA layout (A/B knob)
#endif
#ifndef TI_TILE_HALVES
// 1: the asm loops compute each group as two halves (compute_half: k-steps 0-1, then 2-3, half the A
// fragments live at a time); 3-5 % less time than the whole group at once (compute) on TPW 2-4 at
// 256-1024 rows (profiles/r5_tile_halves_ab.txt).  0: compute (A/B knob)
#define TI_TILE_HALVES 1
#endif
constexpr int kTileEpiStride = 20;   // floats per row of a wave's 64 x 16 staging block (padded: no bank conflicts)
__host__ __device__ constexpr int tile_epi_lds_bytes() { return kGemvWaves * 64 * kTileEpiStride * 4; }

// Epilogue of weight tile tn (16 outputs) for rows mb .. mb + 63 of one wave, from its LDS block
// stg[row][col] (row stride kTileEpiStride).  Same arithmetic as epilogue_mb, element for element.
//   STORE_F32 / RESID_F32 / QKV_ROPE_KV: lane l owns columns 4 (l & 3) .. + 3 of rows 16 it + l / 4
//   SILU_MUL_F16: lane l owns outputs 4 (l & 1) .. + 3 (gate columns, up = column + 8) of rows 32 it + l / 2
template <int RB = 4>   // the wave's rows: 16 RB
__device__ __forceinline__ void tile_epilogue_lds(const GemvArgs& a, int tn, int mb, const float* stg, int lane) {
  const ti_epilogue& e = a.epi;
  if (e.kind == TI_EPI_SILU_MUL_F16) {
    const int h = 4 * (lane & 1);
#pragma unroll
    for (int it = 0; it < RB / 2; ++it) {
      const int row = 32 * it + (lane >> 1), m = mb + row;
      const float4 g = *(const float4*)(stg + row * kTileEpiStride + h);
      const float4 u = *(const float4*)(stg + row * kTileEpiStride + 8 + h);
      if (m >= a.M) continue;
      auto sm = [](float v, float up) { return f2h(up * (v / (1.0f + expf(-v)))); };
      const uint32_t lo = sm(g.x, u.x) | ((uint32_t)sm(g.y, u.y) << 16), hi = sm(g.z, u.z) | ((uint32_t)sm(g.w, u.w) << 16);
      *(uint2*)((uint16_t*)e.out + (size_t)m * e.ldo + tn * 8 + h) = make_uint2(lo, hi);
    }
    return;
  }
  const int c4 = 4 * (lane & 3), ng = tn * 16 + c4;
  // QKV: the tile lies in one of q / k / v and one head (head_dim % 16 == 0)
  const int hd = e.head_dim;
  const bool in_q = ng < e.q_dim, in_k = !in_q && ng < e.q_dim + e.kv_dim;
  const int c = in_q ? ng : in_k ? ng - e.q_dim : ng - e.q_dim - e.kv_dim;
  const int kvh = e.kind == TI_EPI_QKV_ROPE_KV ? c / hd : 0, d = c - kvh * hd;
#pragma unroll
  for (int it = 0; it < RB; ++it) {
    const int row = 16 * it + (lane >> 2), m = mb + row;
    const float4 v = *(const float4*)(stg + row * kTileEpiStride + c4);
    if (m >= a.M) continue;
    if (e.kind == TI_EPI_STORE_F32) {
      *(float4*)((float*)e.out + (size_t)m * e.ldo + ng) = v;
    } else if (e.kind == TI_EPI_RESID_F32) {
      float4* o = (float4*)((float*)e.out + (size_t)m * e.ldo + ng);
      const float4 h = *o;
      *o = make_float4(h.x + v.x, h.y + v.y, h.z + v.z, h.w + v.w);
    } else {   // TI_EPI_QKV_ROPE_KV
      const int p = e.pos[m];
      if (in_q || in_k) {
        // (cos, sin) of pairs d / 2 and d / 2 + 1: even output fmaf(-odd, sin, even * cos), odd
        // output fmaf(odd, cos, even * sin) (epilogue_mb with partner = the other of the pair)
        const float4 cs = *(const float4*)(e.rope_cs + (size_t)p * hd + d);
        const float r0 = fmaf(-v.y, cs.y, v.x * cs.x), r1 = fmaf(v.y, cs.x, v.x * cs.y);
        const float r2 = fmaf(-v.w, cs.w, v.z * cs.z), r3 = fmaf(v.w, cs.z, v.z * cs.w);
        if (in_q) {
          *(float4*)((float*)e.out + (size_t)m * e.ldo + ng) = make_float4(r0, r1, r2, r3);
        } else {
          *(uint2*)(e.k_cache + (size_t)m * e.kv_stream_stride + ((size_t)kvh * e.max_seq + p) * hd + d) =
              make_uint2(f2h(r0) | ((uint32_t)f2h(r1) << 16), f2h(r2) | ((uint32_t)f2h(r3) << 16));
        }
      } else {
        *(uint2*)(e.v_cache + (size_t)m * e.kv_stream_stride + ((size_t)kvh * e.max_seq + p) * hd + d) =
            make_uint2(f2h(v.x) | ((uint32_t)f2h(v.y) << 16), f2h(v.z) | ((uint32_t)f2h(v.w) << 16));
      }
    }
  }
}

// Physical 16-byte chunk of logical chunk c in activation row `row` of the tile kernel's LDS image:
// c ^ tile_swz(row).  An A-fragment read (ds_read_b128, lane l: row l & 15, chunk 4 (l >> 4) + s, or
// 4 s + (l >> 4) with group-32 weights) is serviced in the lane groups {0-3,12-15,20-27},
// {4-11,16-19,28-31}, {32-35,44-47,52-59}, {36-43,48-51,60-63} (MI355X_MICROARCH.md, LDS); each
// holds the 16 rows once, rows {0-3,12-15} at one chunk column and rows {4-11} at the next.  With
// (row + 4) & 15 the first set lands in chunks 0-7 and the second in 8-15 of a row, so the 16 lanes
// of a group hit 16 different chunks (64 banks): conflict-free.  (row & 15 put both sets on the
// same 8 chunks: 2-way conflicts in every group, SQ_LDS_BANK_CONFLICT 3.3 cycles per read.)
#ifndef TI_TILE_SWZ4
#define TI_TILE_SWZ4 1
#endif
__device__ __forceinline__ int tile_swz(int row) { return TI_TILE_SWZ4 ? (row + 4) & 15 : row & 15; }

template <int TPW, bool G32, int WMR, int XB, int RB>
__device__ __forceinline__ void gemm_tile_body(const GemvArgs a, int n_cb, int n_rb, int n_ks);
template <int TPW, bool G32 = false, int WMR = 2, int XB = 2, int RB = 4>
__global__ __launch_bounds__(kGemvThreads, 1) void gemm_tile_kernel(const GemvArgs a, int n_cb, int n_rb, int n_ks) {
  const unsigned long long t_entry = stamp_now();
  gemm_tile_body<TPW, G32, WMR, XB, RB>(a, n_cb, n_rb, n_ks);
  stamp_end(a.stamp, t_entry);
}
template <int TPW, bool G32, int WMR, int XB, int RB>
__device__ __forceinline__ void gemm_tile_body(const GemvArgs a, int n_cb, int n_rb, int n_ks) {
  constexpr int WCOL = kGemvWaves / WMR, BM = 16 * RB * WMR;   // column-waves, rows per workgroup
  constexpr int ND = BM / 32;                                  // activation DMA instructions per wave and group
  static_assert(RB == 4 || (RB == 2 && WMR == 1), "32-row waves: one row-wave per workgroup");
  static_assert(XB == 2 || (XB == 4 && TI_TILE_ASM), "deep activation ring: asm-issued DMA only");
  constexpr int XL = XB - 1;                               // groups of activations issued ahead
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int KT = a.K >> 7, NT = a.N >> 4;
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 15, kq = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), wm = wave / WCOL, wn = wave % WCOL;
  // blockIdx -> (row block, k-slice, column block): the n_rb row blocks and n_ks k-slices of a
  // column block share an XCD; k-slice ks covers groups [kb, kb + nk)
  const int b8 = blockIdx.x & 7, rest = blockIdx.x >> 3;
  const int rb = rest % n_rb, r2 = rest / n_rb, ks = r2 % n_ks, cb = (r2 / n_ks) * 8 + b8;
  if (cb >= n_cb) return;
  const int kb = ks * KT / n_ks, nk = (ks + 1) * KT / n_ks - kb;
  const int m0 = rb * BM, t0 = cb * WCOL * TPW;
  f16* xb = (f16*)smem;                                       // [2][BM rows][128 k] swizzled
  constexpr int SG = G32 ? 4 : 1;                             // scales per tile row and group
  uint16_t* sl = (uint16_t*)(smem + XB * BM * 256);           // [WCOL TPW tiles][KT][SG][16]
  const int n_sc = WCOL * TPW * nk * 2 * SG;                  // 16-byte pieces of this k-slice
  const u32x4* sg = (const u32x4*)(a.scales + (size_t)t0 * KT * 16 * SG);
  const int ntile_ok = min(WCOL * TPW, NT - t0);
  // batched fold (decode rows, ti_hip.h TI_FOLD_SS_ROWS): this thread's share of its row's rms
  // (TPW 4, already short of registers: after the stream)
  const bool fold_in = a.epi.ss_in != nullptr;
  float share = fold_in && TPW < 4 ? fold_share(a, m0 + tid % BM, tid / BM, kGemvThreads / BM) : 0.0f;
  for (int i = tid; i < n_sc; i += kGemvThreads) {
    const int j = i / (nk * 2 * SG), p = (j * KT + kb) * 2 * SG + (i - j * nk * 2 * SG);   // tile j, piece in slice
    ((u32x4*)sl)[p] = j < ntile_ok ? ld_w(sg + p) : (u32x4){0u, 0u, 0u, 0u};
  }

  const f16* xg = (const f16*)a.x;
  const uint32_t xb_lds = (uint32_t)(uintptr_t)xb;   // LDS byte address of the staging buffers
  auto issue_x = [&](int kg) __attribute__((always_inline)) {   // BM / 4 DMA instructions per group
    f16* dst = xb + (kg & (XB - 1)) * BM * 128;
#pragma unroll
    for (int q = 0; q < ND; ++q) {
      const int j = wave * ND + q, row = 4 * j + (lane >> 4), p = lane & 15, c = p ^ tile_swz(row);
      const int m = min(m0 + row, a.M - 1);
      if constexpr (TI_TILE_ASM)
        dma_1k_asm(xg + (size_t)m * a.ldx + kg * 128 + c * 8,
                   __builtin_amdgcn_readfirstlane(xb_lds + (uint32_t)(((kg & (XB - 1)) * BM * 128 + j * 512) * 2)));
      else
        dma_1k(xg + (size_t)m * a.ldx + kg * 128 + c * 8, dst + j * 512);
    }
  };
#ifndef TI_TILE_XREG
#define TI_TILE_XREG 0   // 1: the activation block through VGPRs + ds_write instead of LDS-DMA
#endif
  u32x4 xreg[ND];
  auto load_xr = [&](int kg) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < ND; ++q) {
      const int j = wave * ND + q, row = 4 * j + (lane >> 4), c = (lane & 15) ^ tile_swz(row);
      xreg[q] = *(const u32x4*)(xg + (size_t)min(m0 + row, a.M - 1) * a.ldx + kg * 128 + c * 8);
    }
  };
  auto store_xr = [&](int kg) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < ND; ++q)
      *(u32x4*)(xb + (kg & 1) * BM * 128 + (wave * ND + q) * 512 + lane * 8) = xreg[q];
  };
  const u32x4* tb = a.tiles + lane;
  auto load_w = [&](u32x4 (&w)[TPW], int kg) __attribute__((always_inline)) {
    kg = min(kg, KT - 1);
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
      const u32x4* src = tb + ((size_t)min(t0 + wn * TPW + t, NT - 1) * KT + kg) * kWave;
      if constexpr (TI_TILE_ASM) w[t] = ld_w_asm(src);
      else w[t] = ld_w(src);
    }
  };
  // weight ring: 4 groups deep (2 at TPW 4, whose 4-deep ring hipcc keeps in scratch); the asm
  // pipeline keeps 3 (the covering wait then retires W(kg) together with x(kg), see below)
  constexpr int kTileWR = TI_TILE_ASM ? 3 : (TPW == 4 ? 2 : 4);
  u32x4 W[kTileWR][TPW];
  if constexpr (!TI_TILE_ASM) {   // (the asm pipeline issues its first loads inside its loop)
    if constexpr (TI_TILE_XREG) load_xr(kb);
    else issue_x(kb);
#pragma unroll
    for (int u = 0; u < kTileWR - 1; ++u) load_w(W[u], kb + min(u, nk - 1));
  }
  f32x4 acc[TPW][RB];
#pragma unroll
  for (int t = 0; t < TPW; ++t)
#pragma unroll
    for (int b = 0; b < RB; ++b) acc[t][b] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
  uint32_t magic;
  asm volatile("v_mov_b32 %0, 0x64006400" : "=v"(magic));
  auto compute = [&](const u32x4 (&w)[TPW], int kg) __attribute__((always_inline)) {
    const f16* xr = xb + (kg & (XB - 1)) * BM * 128 + (wm * 16 * RB + r) * 128;
    f16x8 xf[RB][4];
#pragma unroll
    for (int b = 0; b < RB; ++b)
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4)
        xf[b][s4] = *(const f16x8*)(xr + b * 16 * 128 + (((G32 ? s4 * 4 + kq : kq * 4 + s4) ^ tile_swz(r)) * 8));
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
      if constexpr (G32) {
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
          const f16x8 bf = deq_int4_signed(w[t][s4], magic);
          f32x4 tmp[RB];
#pragma unroll
          for (int b = 0; b < RB; ++b)
            tmp[b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xf[b][s4], bf, (f32x4){0.0f, 0.0f, 0.0f, 0.0f}, 0, 0, 0);
          const float sc = h2f(sl[(((wn * TPW + t) * KT + kg) * 4 + s4) * 16 + r]);
#pragma unroll
          for (int b = 0; b < RB; ++b) {
            acc[t][b][0] = fmaf(sc, tmp[b][0], acc[t][b][0]);
            acc[t][b][1] = fmaf(sc, tmp[b][1], acc[t][b][1]);
            acc[t][b][2] = fmaf(sc, tmp[b][2], acc[t][b][2]);
            acc[t][b][3] = fmaf(sc, tmp[b][3], acc[t][b][3]);
          }
        }
        continue;
      }
      f32x4 tmp[RB];
#pragma unroll
      for (int b = 0; b < RB; ++b) tmp[b] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        const f16x8 bf = deq_int4_signed(w[t][s4], magic);
#pragma unroll
        for (int b = 0; b < RB; ++b) tmp[b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xf[b][s4], bf, tmp[b], 0, 0, 0);
      }
      const float sc = h2f(sl[((wn * TPW + t) * KT + kg) * 16 + r]);
#pragma unroll
      for (int b = 0; b < RB; ++b) acc[t][b] = fma_scale4(sc, tmp[b], acc[t][b]);
    }
  };
  // The same group in two halves (k-steps 0-1 / 2-3; the MFMA partials tmpS carried between them):
  // the same products and sums in the same order as compute.
  f32x4 tmpS[TPW][RB];
  auto compute_half = [&](const u32x4 (&w)[TPW], int kg, auto hc) __attribute__((always_inline)) {
    constexpr int H = decltype(hc)::value;
    const f16* xr = xb + (kg & (XB - 1)) * BM * 128 + (wm * 16 * RB + r) * 128;
    f16x8 xf[RB][2];
#pragma unroll
    for (int b = 0; b < RB; ++b)
#pragma unroll
      for (int j = 0; j < 2; ++j) xf[b][j] = *(const f16x8*)(xr + b * 16 * 128 + (((kq * 4 + 2 * H + j) ^ tile_swz(r)) * 8));
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
      if constexpr (H == 0)
#pragma unroll
        for (int b = 0; b < RB; ++b) tmpS[t][b] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const f16x8 bf = deq_int4_signed(w[t][2 * H + j], magic);
#pragma unroll
        for (int b = 0; b < RB; ++b) tmpS[t][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xf[b][j], bf, tmpS[t][b], 0, 0, 0);
      }
      if constexpr (H == 1) {
        const float sc = h2f(sl[((wn * TPW + t) * KT + kg) * 16 + r]);
#pragma unroll
        for (int b = 0; b < RB; ++b) acc[t][b] = fma_scale4(sc, tmpS[t][b], acc[t][b]);
      }
    }
  };
  // Per group kg: x(kg) and W(kg) were issued earlier; issue x(kg + 1) and W(kg + WR - 1),
  // wait until only those weight loads are younger than x(kg + 1)... (see below), compute kg.
  const int KTP = (nk + kTileWR - 1) / kTileWR * kTileWR;
  TILE_CY_DECL();
  if constexpr (TI_TILE_ASM) {
    // Every group issues, in order, x(kg + XL) (2 WMR DMA instructions into buffer
    // (kg + XL) % XB, read last in group kg - 1) and W(kg + 2) (TPW loads into ring slot
    // (kg + 2) % 3), both clamped into [0, KT): the same count in every group, so the waits are
    // constants.  The loop starts at group -3 with the compute off, which also makes the first
    // loads the loop's own code (no prologue whose registers hipcc could shuffle in flight).
    //   x(kg): younger loads at the top of group kg are W(kg + 3 - XL) and XL - 1 whole groups
    //          -> vmcnt(NX), then the barrier makes every wave's part visible;
    //   W(kg): after group kg's own issue, two whole groups are younger -> vmcnt(NWT), then the
    //          slot's registers are tied ("+v") so nothing reads them earlier.
    constexpr int NX = (XL - 1) * (ND + TPW) + TPW, NWT = 2 * (ND + TPW);
    if constexpr (TI_TILE_PAIR && XB == 4 && TPW == 1) {
      // Pairs of groups per barrier (half the barriers): at the top of pair (kg, kg + 1), kg even,
      // x(kg) and x(kg + 1) have landed in every wave and every wave is done with pair kg - 2, whose
      // two buffers then take x(kg + 2) and x(kg + 3); W(kg + 2) goes out every group as before.
      // Issue order: [pair top: 2 x 2 WMR DMAs, TPW weight loads] [odd group: TPW weight loads], so
      //   x(kg + 1) at the pair top: the two groups' weight loads are younger -> vmcnt(2 TPW);
      //   W(kg) after the group's own issue: one pair's worth -> vmcnt(4 WMR + 2 TPW).
      // Slots: the loop runs in steps of 6 from -6 (k0 = 0 mod 2 and mod 3: static pair and slot
      // positions); groups before -2 issue nothing (their waits pass at once).
      constexpr int NX2 = 2 * TPW, NWT2 = 2 * ND + 2 * TPW;
      for (int k0 = -6; k0 < nk; k0 += 6) {
#pragma unroll
        for (int u = 0; u < 6; ++u) {
          const int kg = k0 + u, su = u % 3;
          __builtin_amdgcn_sched_barrier(0);   // no interleaving across groups (register pressure)
          if ((u & 1) == 0) {
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NX2) : "memory");   // x(kg), x(kg + 1)
            TILE_CY(0);
            lds_barrier();
            TILE_CY(1);
            if (kg >= -2) {
              issue_x(kb + max(0, min(kg + 2, nk - 1)));
              issue_x(kb + max(0, min(kg + 3, nk - 1)));
            }
          }
          if (kg >= -2) load_w(W[(su + 2) % 3], kb + max(0, min(kg + 2, nk - 1)));
          TILE_CY(2);
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NWT2) : "memory");   // W(kg)
#pragma unroll
          for (int t = 0; t < TPW; ++t) asm volatile("" : "+v"(W[su][t]));
          TILE_CY(3);
          if (kg >= 0 && kg < nk) {
            if constexpr (TI_TILE_HALVES && !G32) {
              compute_half(W[su], kb + kg, std::integral_constant<int, 0>());
              compute_half(W[su], kb + kg, std::integral_constant<int, 1>());
            } else {
              compute(W[su], kb + kg);
            }
          }
          TILE_CY(4);
        }
      }
    } else
    for (int k0 = -kTileWR; k0 < nk; k0 += kTileWR) {   // kg: group of this k-slice
#pragma unroll
      for (int u = 0; u < kTileWR; ++u) {
        const int kg = k0 + u;
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NX) : "memory");   // x(kg): this wave's DMA
        TILE_CY(0);
        lds_barrier();
        TILE_CY(1);
#if TI_GEMV_EXP & 4096   // diagnostic: the weight stream replaced by re-reads of the first group (L2)
        issue_x(kb + max(0, min(kg + XL, nk - 1)));
        load_w(W[(u + 2) % kTileWR], kb);
#elif TI_GEMV_EXP & 8192   // diagnostic: the activation stream replaced by re-reads of the first group
        issue_x(kb);
        load_w(W[(u + 2) % kTileWR], kb + max(0, min(kg + 2, nk - 1)));
#else
        issue_x(kb + max(0, min(kg + XL, nk - 1)));
        load_w(W[(u + 2) % kTileWR], kb + max(0, min(kg + 2, nk - 1)));
#endif
        // (also in the groups without compute: a slot's load is always consumed by its tie, so
        // hipcc never hands its registers to anything else while the load is in flight)
        TILE_CY(2);
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NWT) : "memory");   // W(kg)
#pragma unroll
        for (int t = 0; t < TPW; ++t) asm volatile("" : "+v"(W[u][t]));
        TILE_CY(3);
#if TI_GEMV_EXP & 2048   // diagnostic (tools/tile_diag.sh): operand streams only, no dequant / MFMA
        if (kg >= 0 && kg < nk && lane == 64) compute(W[u], kb + kg);
#else
        if (kg >= 0 && kg < nk) {
          if constexpr (TI_TILE_HALVES && !G32) {
            compute_half(W[u], kb + kg, std::integral_constant<int, 0>());
            compute_half(W[u], kb + kg, std::integral_constant<int, 1>());
          } else {
            compute(W[u], kb + kg);
          }
        }
#endif
        TILE_CY(4);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the clamped loads past the end
#pragma unroll
    for (int u = 0; u < kTileWR; ++u)
#pragma unroll
      for (int t = 0; t < TPW; ++t) asm volatile("" : "+v"(W[u][t]));
  } else {
  for (int k0 = 0; k0 < KTP; k0 += kTileWR) {
#pragma unroll
    for (int u = 0; u < kTileWR; ++u) {
      const int kg = k0 + u;
      // x(kg) landed (the loads younger than it: W(kg + WR - 2), TPW instructions) and every
      // wave is past compute(kg - 1), so buffer (kg + 1) & 1 is free
      if constexpr (TI_TILE_XREG) {
        if (kg < nk) store_xr(kb + kg);
      }
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(TPW) : "memory");
      lds_barrier();
      if (kg < nk) {
        if (kg + 1 < nk) {
          if constexpr (TI_TILE_XREG) load_xr(kb + kg + 1);
          else issue_x(kb + kg + 1);
        }
        load_w(W[(u + kTileWR - 1) % kTileWR], kb + min(kg + kTileWR - 1, nk - 1));
        compute(W[u], kb + kg);
      }
    }
  }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // every wave is past its last read of the x / scale images (and every DMA into them has
  // landed): the epilogue may stage through that LDS
  lds_barrier();
  const float* rmsv = (const float*)(smem + tile_epi_lds_bytes());   // batched fold: rms per row
  if (fold_in) {
    if constexpr (TPW == 4) share = fold_share(a, m0 + tid % BM, tid / BM, kGemvThreads / BM);
    ((float*)smem)[tid] = share;
    lds_barrier();
    fold_rms_finish(a, (const float*)smem, (float*)rmsv, BM, tid);
    lds_barrier();
  }
#if TI_GEMV_EXP & 512   // diagnostic: no split-K merge at all (every slice runs the epilogue)
  const bool merged = true;
#else
  bool merged = n_ks == 1;   // (32-row waves never split: tile_plan)
  if constexpr (RB == 4)
    merged = merged || splitk_merge<TPW>(a, acc, (cb * n_rb + rb) * kGemvWaves + wave, n_cb * n_rb * kGemvWaves, ks,
                                         n_ks, lane);
#endif
  // Epilogue, one weight tile at a time (the loop stays rolled: 64 inlined epilogues are too large
  // to unroll, so the tile's accumulators are picked by static selects and acc stays in
  // registers).  Kinds with row-contiguous outputs go through the wave's own LDS block
  // (tile_epilogue_lds: a lane then owns 4 consecutive outputs of a row, 8- / 16-byte accesses
  // instead of 16 scattered 2- / 4-byte ones per tile); the rest per element from the MFMA layout.
  const int ek = a.epi.kind;
  const bool via_lds = TI_TILE_EPI_LDS && (ek == TI_EPI_STORE_F32 || ek == TI_EPI_RESID_F32 || ek == TI_EPI_QKV_ROPE_KV ||
                                           (ek == TI_EPI_SILU_MUL_F16 && !a.epi.out_packed));
  float* stg = (float*)smem + wave * (64 * kTileEpiStride);
#pragma unroll 1
  for (int t = 0; t < (merged ? TPW : 0); ++t) {
    const int tn = t0 + wn * TPW + t;
    f32x4 av[RB];
#pragma unroll
    for (int tt = 0; tt < TPW; ++tt)
      if (tt == t)
#pragma unroll
        for (int b = 0; b < RB; ++b) av[b] = acc[tt][b];
    if (fold_in)
#pragma unroll
      for (int b = 0; b < RB; ++b)
#pragma unroll
        for (int i = 0; i < 4; ++i) av[b][i] = av[b][i] / rmsv[wm * 16 * RB + b * 16 + 4 * (lane >> 4) + i];
    if (via_lds) {
      // lane (r, kq) holds rows b*16 + 4 kq + i of column r; LDS program order within the wave
      // makes the reads below see these writes, and the next tile's writes follow the reads
#pragma unroll
      for (int b = 0; b < RB; ++b)
#pragma unroll
        for (int i = 0; i < 4; ++i) stg[(b * 16 + 4 * (lane >> 4) + i) * kTileEpiStride + r] = av[b][i];
      if (tn < NT) tile_epilogue_lds<RB>(a, tn, m0 + wm * 16 * RB, stg, lane);
      continue;
    }
#pragma unroll
    for (int b = 0; b < RB; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = m0 + wm * 16 * RB + b * 16 + 4 * (lane >> 4) + i;
        epilogue_mb(a, tn < NT ? tn : NT - 1, m, r, av[b][i], tn < NT && m < a.M);
      }
  }
  if (a.epi.kind == TI_EPI_LOGITS_ARGMAX && a.epi.step_ctr && blockIdx.x == 0 && tid == 0)
    *a.epi.step_ctr += a.epi.advance;
#if TI_GEMV_EXP & 16384
  if constexpr (TI_TILE_ASM) {
    TILE_CY(5);
    TILE_CY_STORE();
  }
#endif
}

static std::atomic<int> g_num_cus{0};   // (a racing first query stores the same value)

// Tile kernel shape by a per-CU byte model: a CU streams a bounded number of bytes per
// microsecond, a workgroup moves its activation block plus its weight tiles per
// 128-k group, and the launch takes ceil(workgroups / CUs) rounds; the cheapest shape wins
// (TI_TILE_NARROW / TI_TILE_WIDE / TI_TILE_WMR1 drop TPW 1 / TPW 4 / 64-row shapes, A/B knobs).
#if TI_TILE_ASM
#define TI_TILE_XB4 4
#else
#define TI_TILE_XB4 2
#endif
#define TI_TILE_FNS_XB(XB)                                                                                     \
  (const void*)gemm_tile_kernel<1, false, 2, XB>, (const void*)gemm_tile_kernel<2, false, 2, XB>,              \
      (const void*)gemm_tile_kernel<4, false, 2, XB>, (const void*)gemm_tile_kernel<1, true, 2, XB>,           \
      (const void*)gemm_tile_kernel<2, true, 2, XB>, (const void*)gemm_tile_kernel<4, true, 2, XB>,            \
      (const void*)gemm_tile_kernel<1, false, 1, XB>, (const void*)gemm_tile_kernel<2, false, 1, XB>,          \
      (const void*)gemm_tile_kernel<4, false, 1, XB>, (const void*)gemm_tile_kernel<1, true, 1, XB>,           \
      (const void*)gemm_tile_kernel<2, true, 1, XB>, (const void*)gemm_tile_kernel<4, true, 1, XB>,             \
      (const void*)gemm_tile_kernel<3, false, 2, XB>, (const void*)gemm_tile_kernel<3, true, 2, XB>,           \
      (const void*)gemm_tile_kernel<3, false, 1, XB>, (const void*)gemm_tile_kernel<3, true, 1, XB>
// 32-row waves (RB 2): one row-wave, the deep activation ring only
#define TI_TILE_FNS_RB2                                                                                          \
  (const void*)gemm_tile_kernel<1, false, 1, TI_TILE_XB4, 2>, (const void*)gemm_tile_kernel<2, false, 1, TI_TILE_XB4, 2>, \
      (const void*)gemm_tile_kernel<3, false, 1, TI_TILE_XB4, 2>, (const void*)gemm_tile_kernel<4, false, 1, TI_TILE_XB4, 2>, \
      (const void*)gemm_tile_kernel<1, true, 1, TI_TILE_XB4, 2>, (const void*)gemm_tile_kernel<2, true, 1, TI_TILE_XB4, 2>,  \
      (const void*)gemm_tile_kernel<3, true, 1, TI_TILE_XB4, 2>
#define TI_TILE_FNS TI_TILE_FNS_XB(2), TI_TILE_FNS_XB(TI_TILE_XB4), TI_TILE_FNS_RB2
__host__ inline const void* tile_fn(int tpw, bool g32, int wmr, int xb, int rb = 4) {
  static const void* const fns[] = {TI_TILE_FNS};
  if (rb == 2) return fns[32 + (g32 ? 4 : 0) + tpw - 1];   // (group-32 at TPW 4: never planned)
  const int base = xb == 4 ? 16 : 0;
  if (tpw == 3) return fns[base + 12 + (wmr == 1 ? 2 : 0) + (g32 ? 1 : 0)];
  return fns[base + (wmr == 1 ? 6 : 0) + (g32 ? 3 : 0) + (tpw == 1 ? 0 : tpw == 2 ? 1 : 2)];
}
// the deep activation ring when it fits the LDS
__host__ inline int tile_xb(int K, int tpw, bool g32, int wmr, int rb = 4) {
  if (TI_TILE_XB4 != 4) return 2;
  return tile_lds_bytes(K, tpw, g32, wmr, 4, rb) <= 160 * 1024 ? 4 : 2;
}

// 32-row waves (they need the deep activation ring)
__host__ inline bool tile_rb2_on() { return TI_TILE_XB4 == 4; }

// Shapes considered: (row-waves WMR, 16-row blocks per row-wave RB, tiles per wave TPW); a
// workgroup moves 4 RB WMR KiB of activations and WMR x (8 / WMR) TPW KiB of weights per group.
// 32-row waves (WMR 1, RB 2) only for calls of at most 32 rows: the 64-row block's activation DMA
// would move half padding (TI_TILE_RB2=0: A/B knob).  TI_TILE_WMR1=0 keeps 128-row workgroups
// (A/B knob).  Returns 32 * (RB == 2) + 8 * WMR + TPW.
__host__ inline int tile_shape(int M, int N, int K, bool g32, int cus) {
  // 32-row waves only up to 32 rows: at 33-64 rows their second row block re-reads every weight
  // tile (7-8 % slower on the wide outputs, profiles/r3c_tile_rb2_64rows.txt)
  constexpr int rb2_rows = 32;
  const int NT = N >> 4;
  int best = 8 * 2 + 2;
  long best_cost = -1;
  for (int wr : {8, 4, 2}) {   // row-wave shape: 4 RB WMR (2 x 4, 1 x 4, 1 x 2)
    const int wmr = wr == 8 ? 2 : 1, rb = wr == 2 ? 2 : 4;
    if (rb == 2 && (!tile_rb2_on() || M > rb2_rows)) continue;
    for (int tpw : {2, 1, 4, 3}) {
      // (group-32 at TPW 4 spills to scratch: kept out, its asm-loaded weight ring must stay in VGPRs)
      if ((tpw == 4 && g32 && TI_TILE_ASM) ||
          tile_lds_bytes(K, tpw, g32, wmr, 2, rb) > 160 * 1024 || (rb == 2 && tile_xb(K, tpw, g32, wmr, rb) != 4))
        continue;
      const int cols = (8 / wmr) * tpw, bm = 16 * rb * wmr;
      // rounds as launched: ceil(column blocks / 8) x row blocks workgroups on each XCD's CUs
      const long per_xcd = (long)((NT + cols - 1) / cols + 7) / 8 * ((M + bm - 1) / bm);
      const long cost = (per_xcd + cus / 8 - 1) / (cus / 8) * (4 * rb * wmr + 8 * tpw);
      if (best_cost < 0 || cost < best_cost) {
        best = (rb == 2 ? 32 : 0) + 8 * wmr + tpw;
        best_cost = cost;
      }
    }
  }
  return best;
}

// Tile GEMM plan with split-K (ti_epilogue.splitk_ws).  A split costs ≈ 5–14 µs of seam
// (write-through partial stores, the ticket, the last arriver's read-back: tools/splitk_diag.sh)
// and a tile workgroup carries ≈ 7 µs of fixed pipeline cost, so K is split only where the
// one-slice grid would leave most of the chip idle: at most a quarter of the CUs busy, each
// slice still at least 8 groups deep, the slices filling at most one round of workgroups.
// (17..64 decode rows stay on the batched-rows kernel: split there measured slower, 5–14 µs of
// seam against 12–50 µs launches.)  TI_GEMM_SPLITK=0 turns splitting off (A/B knob).
__host__ inline bool splitk_on() { return gemm_knobs().splitk; }
__host__ inline size_t splitk_slab_bytes(int n_ks, int n_cb, int n_rb, int tpw) {
  return (size_t)n_ks * n_cb * n_rb * kGemvWaves * tpw * 4 * kWave * 16;
}
__host__ inline void tile_plan(int M, int N, int K, bool g32, int cus, int64_t ws_bytes, int* wmr_o, int* tpw_o,
                               int* ks_o, int* rb_o = nullptr) {
  const int shape = tile_shape(M, N, K, g32, cus);   // the one-slice choice (knobs applied there)
  const int wmr = (shape >> 3) & 3, tpw = shape & 7, rb = shape & 32 ? 2 : 4;
  *wmr_o = wmr;
  *tpw_o = tpw;
  *ks_o = 1;
  if (rb_o) *rb_o = rb;
  if (rb == 2 || !splitk_on() || ws_bytes <= TI_SPLITK_TICKET_BYTES) return;   // (32-row waves never split)
  const int NT = N >> 4, KT = K >> 7, cols = (8 / wmr) * tpw;
  const int n_cb = (NT + cols - 1) / cols, n_rb = (M + 64 * wmr - 1) / (64 * wmr);
  const long wgs = (long)n_cb * n_rb, grid1 = (long)(n_cb + 7) / 8 * 8 * n_rb;   // (launched: whole XCD rows)
  if (wgs * 4 > cus || (size_t)wgs * kGemvWaves * 4 > TI_SPLITK_TICKET_BYTES) return;
  int S = (int)(cus / grid1);
  while (S > 1 && ((KT + S - 1) / S < 8 || splitk_slab_bytes(S, n_cb, n_rb, tpw) + TI_SPLITK_TICKET_BYTES > (size_t)ws_bytes))
    --S;
  *ks_o = S;
}

__host__ inline int gemv_xmode(int x_kind, int M, int K) {
  if (x_kind == TI_X_F16) return XM_F16;
  if (x_kind == TI_X_F16_FOLDED) return XM_F16F;
  if (x_kind == TI_X_ATTN_SPLITS) return XM_ATTN;
  if (x_kind == TI_X_F32) return XM_F32;
  return M == 1 && (K >> 3) <= kGemvThreads ? XM_NORM1 : XM_NORM;
}

template <int BITS, bool G32 = false, bool AFF = false>
static int launch_gemv(const GemvArgs& a, int lds, hipStream_t s, int grid) {
  const float* pre = a.epi.kind == TI_EPI_RESID_F32 ? (const float*)a.epi.out
                     : a.epi.kind == TI_EPI_QKV_ROPE_KV ? (const float*)a.epi.pos : (const float*)a.x;
  const int xm = gemv_xmode(a.x_kind, a.M, a.K);
  // packed preloaded arguments (see gemv_wq_kernel)
  const float* aux = xm == XM_F16F || xm == XM_ATTN ? a.epi.ss_in : xm == XM_F16 ? nullptr : a.norm_w;
  const int mgk = a.M | (grid << 6) | (a.epi.kind << 18) | (xm == XM_ATTN ? (a.epi.head_dim / 64) << 21 : 0);
  const int kx = a.K | ((xm == XM_F16F || xm == XM_ATTN ? a.epi.n_ss : a.ldx) << 16);
  const int ldo = a.epi.ldo;
  const int NT = a.N >> 4, nt_q = NT / grid, nt_r = NT % grid;   // the kernel's tile split (gemv_wq_kernel)
  if (nt_q > 255 || nt_r >= (1 << 23))
    return ti_set_error(TI_ERR_UNSUPPORTED, "gemv_wq_kernel: %d tiles over %d workgroups", NT, grid);
  const int pn = nt_q | (nt_r << 8);
  switch (xm) {
    case XM_F16: hipLaunchKernelGGL((gemv_wq_kernel<BITS, XM_F16, G32, AFF>), dim3(grid), dim3(kGemvThreads), lds, s, a.tiles, a.scales, a.x, aux, mgk, pn, kx, ldo, pre, a); break;
    case XM_F32: hipLaunchKernelGGL((gemv_wq_kernel<BITS, XM_F32, G32, AFF>), dim3(grid), dim3(kGemvThreads), lds, s, a.tiles, a.scales, a.x, aux, mgk, pn, kx, ldo, pre, a); break;
    case XM_ATTN: hipLaunchKernelGGL((gemv_wq_kernel<BITS, XM_ATTN, G32, AFF>), dim3(grid), dim3(kGemvThreads), lds, s, a.tiles, a.scales, a.x, aux, mgk, pn, kx, ldo, pre, a); break;
    case XM_F16F: hipLaunchKernelGGL((gemv_wq_kernel<BITS, XM_F16F, G32, AFF>), dim3(grid), dim3(kGemvThreads), lds, s, a.tiles, a.scales, a.x, aux, mgk, pn, kx, ldo, pre, a); break;
    case XM_NORM1: hipLaunchKernelGGL((gemv_wq_kernel<BITS, XM_NORM1, G32, AFF>), dim3(grid), dim3(kGemvThreads), lds, s, a.tiles, a.scales, a.x, aux, mgk, pn, kx, ldo, pre, a); break;
    default: hipLaunchKernelGGL((gemv_wq_kernel<BITS, XM_NORM, G32, AFF>), dim3(grid), dim3(kGemvThreads), lds, s, a.tiles, a.scales, a.x, aux, mgk, pn, kx, ldo, pre, a); break;
  }
  TI_LAUNCH_CHECK("gemv_wq_kernel");
  return TI_OK;
}

// rms_norm rows into fp16 (the batched path's activation prep): the same arithmetic as the
// fused XM_NORM staging above (per-thread k8 pieces, wave sums, 8 waves in order).
__global__ __launch_bounds__(kGemvThreads) void rmsnorm_f16_kernel(const float* x, int ldx, const float* w, float eps,
                                                                    uint16_t* y, int ldy, int K, int pk_kt) {
  __shared__ float red[kGemvWaves];
  const int m = blockIdx.x, tid = threadIdx.x, K8 = K >> 3;
  const float* xr = x + (size_t)m * ldx;
  float ss = 0.0f;
  for (int k8 = tid; k8 < K8; k8 += kGemvThreads) {
    const float4 v0 = *(const float4*)(xr + 8 * k8), v1 = *(const float4*)(xr + 8 * k8 + 4);
    ss = fmaf(v0.x, v0.x, ss); ss = fmaf(v0.y, v0.y, ss); ss = fmaf(v0.z, v0.z, ss); ss = fmaf(v0.w, v0.w, ss);
    ss = fmaf(v1.x, v1.x, ss); ss = fmaf(v1.y, v1.y, ss); ss = fmaf(v1.z, v1.z, ss); ss = fmaf(v1.w, v1.w, ss);
  }
  ss = group_sum<kWave>(ss);
  if ((tid & 63) == 0) red[tid >> 6] = ss;
  __syncthreads();
  float tot = 0.0f;
#pragma unroll
  for (int i = 0; i < kGemvWaves; ++i) tot += red[i];
  const float rms = sqrtf(tot / (float)K + eps);
  for (int k8 = tid; k8 < K8; k8 += kGemvThreads) {
    const float4 v0 = *(const float4*)(xr + 8 * k8), v1 = *(const float4*)(xr + 8 * k8 + 4);
    const float4 w0 = *(const float4*)(w + 8 * k8), w1 = *(const float4*)(w + 8 * k8 + 4);
    f16x8 h;
    h[0] = (f16)((v0.x / rms) * w0.x); h[1] = (f16)((v0.y / rms) * w0.y);
    h[2] = (f16)((v0.z / rms) * w0.z); h[3] = (f16)((v0.w / rms) * w0.w);
    h[4] = (f16)((v1.x / rms) * w1.x); h[5] = (f16)((v1.y / rms) * w1.y);
    h[6] = (f16)((v1.z / rms) * w1.z); h[7] = (f16)((v1.w / rms) * w1.w);
    *(f16x8*)(y + (pk_kt > 0 ? TI_PACKED_INDEX(m, 8 * k8, pk_kt) : (size_t)m * ldy + 8 * k8)) = h;
  }
}

// Batched-rows geometry: at most 8 tiles per workgroup (register accumulators), and the
// workgroup's scales in two 16-byte pieces per thread.
__host__ inline int mb_tiles_cap(int MB, int K) {
  const int lim = MB == 2 ? 6 : 8, cap = 512 / (K >> 7);   // (register budget: no spills)
  return cap < 1 ? 1 : (cap > lim ? lim : cap);
}
__host__ inline int mb_grid(int MB, int N, int K, int num_cus, int* ntl_out) {
  const int NT = N >> 4, cap = mb_tiles_cap(MB, K);
  int grid = NT < num_cus ? NT : num_cus;
  if ((NT + grid - 1) / grid > cap) grid = (NT + cap - 1) / cap;
  *ntl_out = (NT + grid - 1) / grid;
  return grid;
}

// One 16-row block: the register-fragment kernel; two: the LDS-DMA one.
static bool mb_use_lds(int MB) { return MB == 2; }
template <int MB, int NTL>
static int launch_mb_t(const GemvArgs& a, int grid, int lds, hipStream_t s) {
  if constexpr (MB == 1) {
    if (!mb_use_lds(MB)) {
      hipLaunchKernelGGL((gemv_mbr_kernel<MB, NTL>), dim3(grid), dim3(kGemvThreads), lds, s, a, grid);
      TI_LAUNCH_CHECK("gemv_mbr_kernel");
      return TI_OK;
    }
  }
  hipLaunchKernelGGL((gemv_mb_kernel<MB, NTL>), dim3(grid), dim3(kGemvThreads), lds, s, a, grid);
  TI_LAUNCH_CHECK("gemv_mb_kernel");
  return TI_OK;
}
static int launch_mb(const GemvArgs& a, int MB, int grid, int ntl, int lds, hipStream_t s) {
  if (MB == 2) {
    switch (ntl) {
      case 1: return launch_mb_t<2, 1>(a, grid, lds, s);
      case 2: return launch_mb_t<2, 2>(a, grid, lds, s);
      case 3: return launch_mb_t<2, 3>(a, grid, lds, s);
      case 4: return launch_mb_t<2, 4>(a, grid, lds, s);
      case 5: return launch_mb_t<2, 5>(a, grid, lds, s);
      default: return launch_mb_t<2, 6>(a, grid, lds, s);
    }
  }
  switch (ntl) {
    case 1: return launch_mb_t<1, 1>(a, grid, lds, s);
    case 2: return launch_mb_t<1, 2>(a, grid, lds, s);
    case 3: return launch_mb_t<1, 3>(a, grid, lds, s);
    case 4: return launch_mb_t<1, 4>(a, grid, lds, s);
    case 5: return launch_mb_t<1, 5>(a, grid, lds, s);
    case 6: return launch_mb_t<1, 6>(a, grid, lds, s);
    case 7: return launch_mb_t<1, 7>(a, grid, lds, s);
    default: return launch_mb_t<1, 8>(a, grid, lds, s);
  }
}
// Rows kernel (M > 16): RG row groups x MB blocks per group, NTL tiles per workgroup.
static bool rows_on() { return true; }
__host__ inline void rows_shape(int M, int* MB, int* RG) {
  const int rg = M > 32 ? 2 : 1;   // 64 rows: two groups of 32
  const int mb = (M + 16 * rg - 1) / (16 * rg);
  *MB = mb;
  *RG = rg;
}
__host__ inline bool g32_rows_on() { return true; }
// Tile kernel from this many rows on (the rows kernel takes at most 64 rows).
static int tile_rows() { return 65; }
__host__ inline int rows_tiles_cap(int MB, int K, bool g32 = false) {
  const int lim = MB >= 2 ? 3 : 4, cap = 512 / ((K >> 7) * (g32 ? 4 : 1));   // VGPR budget / scale pieces
  return cap < 1 ? 1 : (cap > lim ? lim : cap);
}
// Column groups for row blocks of MB blocks per group (one round of workgroups where the VGPR
// cap on tiles per workgroup allows).
// The launch is ceil(n_cg / 8) * 8 * n_rb workgroups spread round-robin over the 8 XCDs, so with
// row blocks the column groups per block are a multiple of 8 (3 row blocks x 85 groups = 264
// workgroups put 33 on an XCD of 32 CUs: a second round, 1.7x the time, tools/rows_m_sweep.py).
__host__ inline int rows_grid(int MB, int N, int K, int num_cus, int* ntl_out, int n_rb = 1, bool g32 = false) {
  const int NT = N >> 4, cap = rows_tiles_cap(MB, K, g32);
  const int per = n_rb > 1 ? (num_cus / n_rb / 8 * 8 > 0 ? num_cus / n_rb / 8 * 8 : 8) : num_cus;
  int n_cg = NT < per ? NT : per;
  if ((NT + n_cg - 1) / n_cg > cap) n_cg = (NT + cap - 1) / cap;
  *ntl_out = (NT + n_cg - 1) / n_cg;
  return n_cg;
}
// Rows per workgroup (16 RG MB): the fewest activation + weight bytes per workgroup over the
// launch's rounds -- a workgroup streams its rows' activations (R K 2 bytes, L2) and its tiles'
// weights (ntl 8 K bytes); narrow outputs (O, down) take 16-row blocks, wide ones all the rows.
// TI_GEMM_ROWS_SPLIT=0 keeps all rows in one workgroup (A/B knob).
__host__ inline void rows_plan(int M, int N, int K, int cus, int* MB, int* RG, int* n_rb, int* n_cg, int* ntl,
                               bool g32 = false) {
  rows_shape(M, MB, RG);   // all rows in one workgroup
  *n_rb = 1;
  *n_cg = rows_grid(*MB, N, K, cus, ntl, 1, g32);
  if (!gemm_knobs().rows_split) return;
  const int NT = N >> 4;
  auto cost = [&](int mb, int rg, int nrb, int ncg, int nt) {
    const long rounds = ((long)(ncg + 7) / 8 * 8 * nrb + cus - 1) / cus;
    return rounds * ((long)16 * rg * mb * K * 2 + (long)nt * 8 * K);
  };
  long best = cost(*MB, *RG, 1, *n_cg, *ntl);
  const int shapes[2][2] = {{1, 1}, {2, 1}};   // 16 and 32 rows per workgroup
  for (const auto& sh : shapes) {
    const int mb = sh[0], rg = sh[1], rows = 16 * mb * rg;
    if (rows >= M) continue;
    const int nrb = (M + rows - 1) / rows;
    int nt = 0;
    const int ncg = rows_grid(mb, N, K, cus, &nt, nrb, g32);
    const long c = cost(mb, rg, nrb, ncg, nt);
    if (c * 20 < best * 17 && nt <= NT) {   // a clear (15 %) win only: the model ignores round overlap
      best = c;
      *MB = mb;
      *RG = rg;
      *n_rb = nrb;
      *n_cg = ncg;
      *ntl = nt;
    }
  }
}
template <int MB, int RG, bool XP, bool G32>
static int launch_rows_t(const GemvArgs& a, int ntl, int n_cg, int n_rb, int lds, hipStream_t s) {
  const dim3 grid((unsigned)((n_cg + 7) / 8 * 8 * n_rb));
  if (ntl == 1) hipLaunchKernelGGL((gemm_rows_kernel<MB, 1, RG, XP, G32>), grid, dim3(kGemvThreads), lds, s, a, n_cg, n_rb);
  else if (ntl == 2) hipLaunchKernelGGL((gemm_rows_kernel<MB, 2, RG, XP, G32>), grid, dim3(kGemvThreads), lds, s, a, n_cg, n_rb);
  else if (ntl == 3) hipLaunchKernelGGL((gemm_rows_kernel<MB, 3, RG, XP, G32>), grid, dim3(kGemvThreads), lds, s, a, n_cg, n_rb);
  else if constexpr (MB < 2) hipLaunchKernelGGL((gemm_rows_kernel<MB, 4, RG, XP, G32>), grid, dim3(kGemvThreads), lds, s, a, n_cg, n_rb);
  else return ti_set_error(TI_ERR_ARG, "gemm_rows_kernel: %d tiles per workgroup at MB %d", ntl, MB);
  TI_LAUNCH_CHECK("gemm_rows_kernel");
  return TI_OK;
}
template <bool XP, bool G32 = false>
static int launch_rows_x(const GemvArgs& a, int MB, int RG, int ntl, int n_cg, int n_rb, int lds, hipStream_t s) {
  if (RG == 2)
    return MB == 1 ? launch_rows_t<1, 2, XP, G32>(a, ntl, n_cg, n_rb, lds, s) : launch_rows_t<2, 2, XP, G32>(a, ntl, n_cg, n_rb, lds, s);
  return MB == 1 ? launch_rows_t<1, 1, XP, G32>(a, ntl, n_cg, n_rb, lds, s) : launch_rows_t<2, 1, XP, G32>(a, ntl, n_cg, n_rb, lds, s);
}
static int launch_rows(const GemvArgs& a, int MB, int RG, int ntl, int n_cg, int n_rb, int lds, hipStream_t s,
                       bool g32 = false) {
  if (g32) return launch_rows_x<false, true>(a, MB, RG, ntl, n_cg, n_rb, lds, s);
  return a.x_kind == TI_X_F16_PACKED ? launch_rows_x<true>(a, MB, RG, ntl, n_cg, n_rb, lds, s)
                                     : launch_rows_x<false>(a, MB, RG, ntl, n_cg, n_rb, lds, s);
}
#define TI_ROWS_FNS1(MB, RG, XP, G)                                                                       \
  (const void*)gemm_rows_kernel<MB, 1, RG, XP, G>, (const void*)gemm_rows_kernel<MB, 2, RG, XP, G>,          \
      (const void*)gemm_rows_kernel<MB, 3, RG, XP, G>
#define TI_ROWS_FNS2(XP, G)                                                                              \
  TI_ROWS_FNS1(1, 1, XP, G), TI_ROWS_FNS1(2, 1, XP, G), TI_ROWS_FNS1(1, 2, XP, G), TI_ROWS_FNS1(2, 2, XP, G), \
      (const void*)gemm_rows_kernel<1, 4, 1, XP, G>, (const void*)gemm_rows_kernel<1, 4, 2, XP, G>
#define TI_ROWS_FNS TI_ROWS_FNS2(false, false), TI_ROWS_FNS2(true, false), TI_ROWS_FNS2(false, true)

#define TI_MB_FNS1(K)                                                                                \
  (const void*)K<1, 1>, (const void*)K<1, 2>, (const void*)K<1, 3>, (const void*)K<1, 4>, (const void*)K<1, 5>, \
      (const void*)K<1, 6>, (const void*)K<1, 7>, (const void*)K<1, 8>
#define TI_MB_FNS                                                                                      \
  TI_MB_FNS1(gemv_mb_kernel), TI_MB_FNS1(gemv_mbr_kernel), (const void*)gemv_mb_kernel<2, 1>,           \
      (const void*)gemv_mb_kernel<2, 2>, (const void*)gemv_mb_kernel<2, 3>, (const void*)gemv_mb_kernel<2, 4>, \
      (const void*)gemv_mb_kernel<2, 5>, (const void*)gemv_mb_kernel<2, 6>

// devices (bit per ordinal) whose attributes are set; engines may be driven from several threads
// (test_gpu_threads.py): fetch_or, and a repeated setup by a racing first call is harmless
static std::atomic<unsigned long long> g_prepared{0};

}  // namespace ti

// Raise the dynamic-LDS cap of the GEMM instantiations (call before any stream capture).
static int query_cus() {
  int n = ti::g_num_cus.load(std::memory_order_relaxed);
  if (n <= 0) {
    int dev = 0;
    if (!(hipGetDevice(&dev) == hipSuccess &&
          hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0))
      n = 256;
    ti::g_num_cus.store(n, std::memory_order_relaxed);
  }
  return n;
}

extern "C" int ti_gemm_prepare(void) {
  using namespace ti;
  query_cus();
  int dev = 0;
  TI_HIP_CHECK(hipGetDevice(&dev), "hipGetDevice");
  const unsigned long long bit = 1ull << (dev & 63);
  if (g_prepared.load(std::memory_order_acquire) & bit) return TI_OK;
  const void* fns[] = {
      (const void*)gemv_wq_kernel<4, XM_F16>,  (const void*)gemv_wq_kernel<4, XM_F32>,
      (const void*)gemv_wq_kernel<4, XM_NORM1>, (const void*)gemv_wq_kernel<4, XM_NORM>,
      (const void*)gemv_wq_kernel<8, XM_F16>,  (const void*)gemv_wq_kernel<8, XM_F32>,
      (const void*)gemv_wq_kernel<8, XM_NORM1>, (const void*)gemv_wq_kernel<8, XM_NORM>,
      (const void*)gemv_wq_kernel<16, XM_F16>, (const void*)gemv_wq_kernel<16, XM_F32>,
      (const void*)gemv_wq_kernel<16, XM_NORM1>, (const void*)gemv_wq_kernel<16, XM_NORM>,
      (const void*)gemv_wq_kernel<4, XM_F16F>, (const void*)gemv_wq_kernel<8, XM_F16F>,
      (const void*)gemv_wq_kernel<16, XM_F16F>, (const void*)gemv_wq_kernel<4, XM_ATTN>,
      (const void*)gemv_wq_kernel<8, XM_ATTN>, (const void*)gemv_wq_kernel<16, XM_ATTN>, TI_MB_FNS, TI_ROWS_FNS,
      TI_TILE_FNS};
  for (const void* f : fns)
    TI_HIP_CHECK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024),
                 "hipFuncSetAttribute(gemv_wq_kernel)");
  g_prepared.fetch_or(bit, std::memory_order_acq_rel);
  return TI_OK;
}

extern "C" int ti_gemm_lds_bytes(int M, int N, int K) {
  if (M < 1 || N < 16 || K < 128) return 0;
  const int NT = N >> 4, grid = ti::gemv_grid(M, N, K, query_cus());
  return ti::gemv_lds_bytes_tiles(M, K, (NT + grid - 1) / grid);
}

// The fused kernel takes the rows while its LDS image fits; int4 with fp16 activations
// also has the batched-rows kernel (up to TI_GEMM_MAX_ROWS rows, any K).
// int4 with more than 2 rows goes to the batched-rows kernel: from 4 rows on it is faster at
// every 7B projection (bench.py --batch 2..16, rocprof), at 2 rows the two tie.
static int fused_rows_pref(int bits) { return bits == 4 ? 2 : 16; }
static bool fused_fits(int M, int N, int K, bool g32 = false, bool aff = false) {
  if (M > 16) return false;
  const int NT = N >> 4, grid = ti::gemv_grid(M, N, K, query_cus(), g32, aff);
  return ti::gemv_lds_bytes_tiles(M, K, (NT + grid - 1) / grid, g32, aff) <= 160 * 1024;
}
static bool use_batched(int bits, int x_kind, int M, int N, int K) {
  const bool mb_ok = bits == 4 && x_kind == TI_X_F16;
  return !fused_fits(M, N, K) || (mb_ok && M > fused_rows_pref(bits));
}

// 17..64 int4 rows of a WIDE output take the tile GEMM, whose time is nearly flat there (≈ 27–31 µs
// at 64 rows for N = 22016 .. 32000, K = 4096), instead of the batched-rows kernel, which moves
// every row's activations per workgroup: rows x N >= TI_GEMM_TILE_WIDE_MN (env, default 850000;
// 0 = off) -- the measured crossover (tools/rows_ab.sh: 64 x 12288 rows kernel 19.0 vs tile 26.5 us,
// 32 x 28672 rows 36.5 vs tile 28.4, 64 x 22016 35.5 vs 28.3, 32 x 22016 25.7 vs 27.2).
// At 17..32 rows the tile kernel's 32-row waves (RB 2) move a quarter of the activation bytes the
// batched-rows kernel does and win from N >= 16384 whatever the
// rows (`profiles/r3c_tile_wide32.txt`: N = 22016 at 17-32 rows 25.1-25.5 -> 18.2-18.8 us, N = 32000
// 36.1-36.4 -> 21.2-21.8; N = 12288 stays on the rows kernel, 13.8 vs 17.2).
static bool wide_tile(int bits, int M, int N) {
  constexpr long kWideMN = 850000, kWideN32 = 16384;
  if (bits != 4 || M <= 16 || M >= ti::tile_rows()) return false;
  if (M <= 32 && ti::tile_rb2_on() && N >= kWideN32) return true;
  return (long)M * N >= kWideMN;
}
extern "C" int ti_gemm_packed_rows(int bits, int M) { return bits == 4 && M > 16 && M < ti::tile_rows() ? 1 : 0; }
extern "C" int ti_gemm_packed_rows_for(int bits, int M, int N, int K) {
  (void)K;
  return ti_gemm_packed_rows(bits, M) && !wide_tile(bits, M, N) ? 1 : 0;
}

extern "C" int ti_gemm_fold_partials(int bits, int M, int N, int K) {
  if (bits != 4 || M <= 16 || M >= ti::tile_rows() || M > TI_FOLD_SS_ROWS || N < 16 || (N & 15) || K < 128 || (K & 127))
    return 0;
  int MB = 0, RG = 0, n_rb = 0, n_cg = 0, ntl = 0;
  ti::rows_plan(M, N, K, query_cus(), &MB, &RG, &n_rb, &n_cg, &ntl);
  return n_cg;
}

extern "C" int ti_gemm_tile_plan(int bits, int M, int N, int K, int64_t ws_bytes, int* wmr, int* tpw, int* n_ks) {
  const bool g32 = (bits & TI_BITS_G32) != 0;
  if (!wmr || !tpw || !n_ks) return ti_set_error(TI_ERR_ARG, "ti_gemm_tile_plan: null pointer");
  if ((bits & ~TI_BITS_G32) != 4 || M < ti::tile_rows() || M > TI_GEMM_MAX_ROWS || N < 16 || (N & 15) || K < 128 ||
      (K & 127))
    return ti_set_error(TI_ERR_UNSUPPORTED, "ti_gemm_tile_plan: M=%d N=%d K=%d bits %d is not a tile-kernel call", M, N,
                        K, bits);
  ti::tile_plan(M, N, K, g32, query_cus(), ti::splitk_on() ? ws_bytes : 0, wmr, tpw, n_ks);
  return TI_OK;
}

extern "C" int ti_gemm_max_rows(int bits, int x_kind, int N, int K) {
  if (N < 16 || K < 128) return 0;
  if (bits & TI_BITS_G32) {   // group-32 weights: the fused kernel; int4 fp16 rows also the tile kernel
    const bool aff = (bits & TI_BITS_AFF) != 0;   // (affine blocks: fused pieces only)
    if (x_kind == TI_X_F16_PACKED) return 0;
    if ((bits & ~(TI_BITS_G32 | TI_BITS_AFF)) == 4 && x_kind == TI_X_F16) return TI_GEMM_MAX_ROWS;   // 16-row pieces
    int m = 16;
    while (m > 1 && !fused_fits(m, N, K, true, aff)) --m;
    return fused_fits(m, N, K, true, aff) ? m : 0;
  }
  if (bits == 4 && (x_kind == TI_X_F16 || x_kind == TI_X_F16_PACKED)) return TI_GEMM_MAX_ROWS;
  if (x_kind == TI_X_F16_PACKED) return 0;
  int m = fused_rows_pref(bits);
  while (m > 1 && !fused_fits(m, N, K)) --m;
  return fused_fits(m, N, K) ? m : 0;
}

extern "C" int ti_rmsnorm_f16(const float* x, int ldx, const float* w, float eps, uint16_t* y, int ldy, int M, int K,
                              ti_stream_t stream) {
  if (!x || !w || !y) return ti_set_error(TI_ERR_ARG, "ti_rmsnorm_f16: null pointer");
  if (M < 1 || K < 8 || (K & 7) || ldx < K || ldy < K)
    return ti_set_error(TI_ERR_ARG, "ti_rmsnorm_f16: bad shape (M=%d K=%d ldx=%d ldy=%d)", M, K, ldx, ldy);
  ti_stamp_next(ti::STAMP_RMSNORM, 0);   // (unstamped; keeps the stamped step's launch list whole)
  hipLaunchKernelGGL(ti::rmsnorm_f16_kernel, dim3(M), dim3(ti::kGemvThreads), 0, (hipStream_t)stream, x, ldx, w, eps,
                     y, ldy, K, 0);
  TI_LAUNCH_CHECK("rmsnorm_f16_kernel");
  return TI_OK;
}

extern "C" int ti_rmsnorm_f16_packed(const float* x, int ldx, const float* w, float eps, uint16_t* y, int M, int K,
                                     ti_stream_t stream) {
  if (!x || !w || !y) return ti_set_error(TI_ERR_ARG, "ti_rmsnorm_f16_packed: null pointer");
  if (M < 1 || K < 128 || (K & 127) || ldx < K)
    return ti_set_error(TI_ERR_ARG, "ti_rmsnorm_f16_packed: bad shape (M=%d K=%d ldx=%d)", M, K, ldx);
  ti_stamp_next(ti::STAMP_RMSNORM, 0);   // (unstamped; keeps the stamped step's launch list whole)
  hipLaunchKernelGGL(ti::rmsnorm_f16_kernel, dim3(M), dim3(ti::kGemvThreads), 0, (hipStream_t)stream, x, ldx, w, eps,
                     y, K, K, K >> 7);
  TI_LAUNCH_CHECK("rmsnorm_f16_kernel");
  return TI_OK;
}

static int gemm_impl(const void* tiles, const uint16_t* scales, int bits, const void* x, int x_kind, int ldx,
                     const float* norm_w, float eps, int M, int N, int K, const ti_epilogue* epi,
                     ti_stream_t stream) {
  using namespace ti;
  if (!tiles || !x || !epi || !epi->out) return ti_set_error(TI_ERR_ARG, "ti_gemm_wq_a16: null pointer");
  const bool g32 = (bits & TI_BITS_G32) != 0, aff = (bits & TI_BITS_AFF) != 0;
  bits &= ~(TI_BITS_G32 | TI_BITS_AFF);
  if ((bits != 4 && bits != 8 && bits != 16) || (g32 && bits == 16) || (aff && (!g32 || bits != 4)))
    return ti_set_error(TI_ERR_ARG, "ti_gemm_wq_a16: bits must be 4, 8 or 16 (+ TI_BITS_G32 for 4 / 8, + TI_BITS_AFF "
                        "for 4 | G32; got %d)", bits);
  // group-32: int4 fp16 rows from tile_rows() on run on the tile kernel, everything else on the
  // fused kernel (more than 16 rows: in 16-row pieces, below); affine blocks on the fused kernel only
  const bool g32_tile = g32 && !aff && bits == 4 && x_kind == TI_X_F16 && M >= tile_rows() && !epi->out_packed;
  // group-32 int4 fp16 rows 17..64: the batched-rows kernel (TI_GEMM_G32_ROWS=0: fused pieces, A/B knob)
  const bool g32_rowsk = g32 && !aff && bits == 4 && x_kind == TI_X_F16 && M > 16 && M < tile_rows() &&
                         !epi->out_packed && g32_rows_on();
  int g32_rows = 16;   // rows per fused launch (its LDS image holds the x rows)
  while (g32 && g32_rows > 1 && !fused_fits(g32_rows, N, K, true, aff)) --g32_rows;
  if (g32 && (x_kind == TI_X_F16_PACKED ||
              (!g32_tile && !g32_rowsk && !fused_fits(std::min(M, g32_rows), N, K, true, aff))))
    return ti_set_error(TI_ERR_UNSUPPORTED, "ti_gemm_wq_a16: group-32 weights: fused kernel rows (M=%d N=%d K=%d) "
                        "or int4 fp16 rows >= %d; no packed rows", M, N, K, tile_rows());
  if (bits != 16 && !scales) return ti_set_error(TI_ERR_ARG, "ti_gemm_wq_a16: scales required for bits %d", bits);
  if (M < 1 || M > TI_GEMM_MAX_ROWS)
    return ti_set_error(TI_ERR_ARG, "ti_gemm_wq_a16: M must be in [1,%d] (got %d)", TI_GEMM_MAX_ROWS, M);
  if (K <= 0 || (K & 127) || N <= 0 || (N & 15))
    return ti_set_error(TI_ERR_ARG, "ti_gemm_wq_a16: K %% 128 and N %% 16 must be 0 (K=%d N=%d)", K, N);
  if (x_kind < TI_X_F16 || x_kind > TI_X_F16_PACKED)
    return ti_set_error(TI_ERR_ARG, "ti_gemm_wq_a16: bad x_kind %d", x_kind);
  if (x_kind == TI_X_F16_PACKED && bits != 4)
    return ti_set_error(TI_ERR_UNSUPPORTED, "ti_gemm_wq_a16: TI_X_F16_PACKED needs bits 4 (batched-rows kernel)");
  if (x_kind == TI_X_ATTN_SPLITS &&
      (M != 1 || !epi->ss_in || epi->n_ss < 1 || epi->n_ss > TI_ATTN_MAX_PART_SPLITS ||
       (epi->head_dim != 64 && epi->head_dim != 128) || K % epi->head_dim || K > 4096))
    return ti_set_error(TI_ERR_ARG, "ti_gemm_wq_a16: TI_X_ATTN_SPLITS needs M == 1, ss_in, 1 <= n_ss <= %d, head_dim "
                        "64/128 and K <= 4096", TI_ATTN_MAX_PART_SPLITS);
  if (x_kind == TI_X_F16_FOLDED && (M != 1 || !epi->ss_in || epi->n_ss < 1 || epi->n_ss > 256))
    return ti_set_error(TI_ERR_ARG, "ti_gemm_wq_a16: TI_X_F16_FOLDED needs M == 1, ss_in and 1 <= n_ss <= 256");
  const bool fold_out = epi->kind == TI_EPI_RESID_F32 && epi->fold_x;
  if (fold_out && M == 1 && (!epi->fold_w || !epi->fold_ss || (x_kind != TI_X_F16 && x_kind != TI_X_ATTN_SPLITS)))
    return ti_set_error(TI_ERR_ARG, "ti_gemm_wq_a16: fold_x needs M == 1, fp16 x, fold_w and fold_ss");
  if (fold_out && M > 1 && (!epi->fold_w || !epi->fold_ss || x_kind != TI_X_F16_PACKED || M > TI_FOLD_SS_ROWS ||
                            (N & 127)))
    return ti_set_error(TI_ERR_ARG, "ti_gemm_wq_a16: a batched fold_x needs TI_X_F16_PACKED x, M <= %d, fold_w, "
                        "fold_ss and N %% 128 == 0", TI_FOLD_SS_ROWS);
  // batched fold consumer: fp16(h * nw) rows normalised behind the GEMM (rows / tile kernels)
  const bool fold_in = M > 1 && epi->ss_in && (x_kind == TI_X_F16 || x_kind == TI_X_F16_PACKED);
  if (fold_in && (M > TI_FOLD_SS_ROWS || epi->n_ss < 1 || epi->n_ss > 4096))
    return ti_set_error(TI_ERR_ARG, "ti_gemm_wq_a16: a batched folded input needs M <= %d and 1 <= n_ss <= 4096",
                        TI_FOLD_SS_ROWS);
  if (K > 0xffff || ldx > 0xffff)
    return ti_set_error(TI_ERR_UNSUPPORTED, "ti_gemm_wq_a16: K %d / ldx %d above 65535", K, ldx);
  if (x_kind == TI_X_F32_RMSNORM && !norm_w) return ti_set_error(TI_ERR_ARG, "ti_gemm_wq_a16: norm_w required");
  if (ldx < K) return ti_set_error(TI_ERR_ARG, "ti_gemm_wq_a16: ldx %d < K %d", ldx, K);
  switch (epi->kind) {
    case TI_EPI_STORE_F32: case TI_EPI_STORE_F16: case TI_EPI_RESID_F32:
      if (epi->ldo < N) return ti_set_error(TI_ERR_ARG, "ti_gemm_wq_a16: ldo %d < N %d", epi->ldo, N);
      break;
    case TI_EPI_SILU_MUL_F16:
      if (epi->ldo < N / 2) return ti_set_error(TI_ERR_ARG, "ti_gemm_wq_a16: ldo < N/2");
      break;
    case TI_EPI_QKV_ROPE_KV:
      if (!epi->pos || !epi->rope_cs || !epi->k_cache || !epi->v_cache || epi->head_dim <= 0 || epi->head_dim > 128 ||
          (epi->head_dim & 1) || epi->q_dim + 2 * epi->kv_dim != N || epi->q_dim % epi->head_dim ||
          epi->kv_dim % epi->head_dim || epi->ldo < epi->q_dim)
        return ti_set_error(TI_ERR_ARG, "ti_gemm_wq_a16: inconsistent QKV epilogue");
      break;
    case TI_EPI_LOGITS_ARGMAX:
      if (!epi->argmax || epi->ldo < N) return ti_set_error(TI_ERR_ARG, "ti_gemm_wq_a16: argmax/ldo");
      break;
    default:
      return ti_set_error(TI_ERR_ARG, "ti_gemm_wq_a16: unknown epilogue %d", epi->kind);
  }
  if (g32 && !g32_tile && !g32_rowsk && M > g32_rows) {   // pieces of g32_rows rows through the fused kernel
    if (x_kind == TI_X_ATTN_SPLITS || x_kind == TI_X_F16_FOLDED || epi->out_packed)
      return ti_set_error(TI_ERR_UNSUPPORTED, "ti_gemm_wq_a16: group-32 rows > 16 need plain x rows");
    const size_t x_elem = x_kind == TI_X_F16 ? 2 : 4;
    const size_t out_elem = epi->kind == TI_EPI_STORE_F16 || epi->kind == TI_EPI_SILU_MUL_F16 ? 2 : 4;
    for (int m0 = 0; m0 < M; m0 += g32_rows) {
      const int mm = std::min(g32_rows, M - m0);
      ti_epilogue ep = *epi;
      ep.out = static_cast<char*>(epi->out) + (size_t)m0 * epi->ldo * out_elem;
      if (ep.pos) ep.pos += m0;
      if (ep.k_cache) ep.k_cache += (size_t)m0 * ep.kv_stream_stride;
      if (ep.v_cache) ep.v_cache += (size_t)m0 * ep.kv_stream_stride;
      if (ep.argmax) ep.argmax += (size_t)m0 * TI_ARGMAX_SLOTS;
      if (m0 + mm < M) ep.step_ctr = nullptr;
      const int rc = gemm_impl(tiles, scales, bits | TI_BITS_G32 | (aff ? TI_BITS_AFF : 0),
                               static_cast<const char*>(x) + (size_t)m0 * ldx * x_elem,
                               x_kind, ldx, norm_w, eps, mm, N, K, &ep, stream);
      if (rc != TI_OK) return rc;
    }
    return TI_OK;
  }
  const bool packed_x = x_kind == TI_X_F16_PACKED;
  const bool batched = g32 ? (g32_tile || g32_rowsk) : (packed_x || use_batched(bits, x_kind, M, N, K));
  if (epi->out_packed && (!batched || (epi->kind != TI_EPI_STORE_F16 && epi->kind != TI_EPI_SILU_MUL_F16) ||
                          (epi->ldo & 127)))
    return ti_set_error(TI_ERR_ARG, "ti_gemm_wq_a16: out_packed needs the batched-rows kernel, a fp16 store / SiLU "
                        "epilogue and ldo %% 128 == 0");
  if (batched && fold_out && M == 1)
    return ti_set_error(TI_ERR_UNSUPPORTED, "ti_gemm_wq_a16: fold_x needs the fused kernel");
  if (batched && !(bits == 4 && (x_kind == TI_X_F16 || packed_x)))
    return ti_set_error(TI_ERR_UNSUPPORTED,
                        "ti_gemm_wq_a16: M=%d K=%d exceeds the fused kernel (ti_gemm_max_rows); the batched-rows "
                        "kernel needs bits 4 and fp16 rows (normalise with ti_rmsnorm_f16)", M, K);
  int grid = 0, lds = 0, ntl = 0, rMB = 0, rRG = 0, r_rb = 1;
  const bool has_ws = epi->splitk_ws && epi->splitk_bytes > TI_SPLITK_TICKET_BYTES && splitk_on();
  const bool tile = batched && x_kind == TI_X_F16 && (M >= tile_rows() || (!g32 && wide_tile(bits, M, N)));
  const bool rows = !tile && batched && (g32_rowsk || packed_x || M > 32 || (M > 16 && rows_on()));
  int n_cb = 0, n_rb = 0, n_ks = 1, tpw = 2, wmr = 2, xbuf = 2, trb = 4;
  if (tile) {
    tile_plan(M, N, K, g32, query_cus(), has_ws ? epi->splitk_bytes : 0, &wmr, &tpw, &n_ks, &trb);   // (tile_plan)
    n_rb = (M + 16 * trb * wmr - 1) / (16 * trb * wmr);
    n_cb = ((N >> 4) + (8 / wmr) * tpw - 1) / ((8 / wmr) * tpw);
    grid = (n_cb + 7) / 8 * 8 * n_rb * n_ks;
    xbuf = tile_xb(K, tpw, g32, wmr, trb);
    lds = tile_lds_bytes(K, tpw, g32, wmr, xbuf, trb);
  } else if (rows) {
    rows_on();
    rows_plan(M, N, K, query_cus(), &rMB, &rRG, &r_rb, &grid, &ntl, g32);   // grid: column groups
    lds = rows_lds_bytes(rRG * rMB, ntl, K, g32);
  } else if (batched) {
    const int MB = M > 16 ? 2 : 1;
    grid = mb_grid(MB, N, K, query_cus(), &ntl);
    lds = mb_use_lds(MB) ? mb_lds_bytes(MB, ntl, K) : mbr_lds_bytes(MB, ntl, K);
  } else {
    grid = gemv_grid(M, N, K, query_cus(), g32, aff);
    lds = gemv_lds_bytes_tiles(M, K, ((N >> 4) + grid - 1) / grid, g32, aff);
  }
  if ((fold_out && M > 1 && !rows) || (fold_in && !rows && !tile))
    return ti_set_error(TI_ERR_UNSUPPORTED, "ti_gemm_wq_a16: the batched fold runs on the batched-rows (fold_x) / "
                        "rows or tile (folded input) kernels (M=%d N=%d K=%d)", M, N, K);
  if (lds > 160 * 1024)
    return ti_set_error(TI_ERR_UNSUPPORTED, "ti_gemm_wq_a16: LDS image %d B too large (M=%d N=%d K=%d)", lds, M, N, K);
  if (!batched && grid > 0xfff)
    return ti_set_error(TI_ERR_UNSUPPORTED, "ti_gemm_wq_a16: %d workgroups (N=%d) above 4095", grid, N);
  if (lds > 64 * 1024) {   // no-op once this device is prepared
    const int rc = ti_gemm_prepare();
    if (rc != TI_OK) return rc;
  }
  GemvArgs a;
  a.tiles = (const u32x4*)tiles;
  a.scales = scales;
  a.x = x;
  a.norm_w = norm_w;
  a.eps = eps;
  a.x_kind = x_kind;
  a.ldx = ldx;
  a.M = M;
  a.N = N;
  a.K = K;
  a.epi = *epi;
  {   // workgroups of the launch below (stamp buffer sizing)
    const long wgs = tile ? grid : rows ? (long)((grid + 7) / 8 * 8) * r_rb : grid;
    a.stamp = ti_stamp_next(tile ? STAMP_TILE : rows ? STAMP_ROWS : batched ? STAMP_MB : STAMP_GEMV, wgs);
  }
  hipStream_t s = (hipStream_t)stream;
  if (tile) {
    const void* f = tile_fn(tpw, g32, wmr, xbuf, trb);
    void* args[] = {&a, &n_cb, &n_rb, &n_ks};
    TI_HIP_CHECK(hipLaunchKernel(f, dim3(grid), dim3(kGemvThreads), args, lds, s), "hipLaunchKernel(gemm_tile_kernel)");
    TI_LAUNCH_CHECK("gemm_tile_kernel");
    return TI_OK;
  }
  if (rows) return launch_rows(a, rMB, rRG, ntl, grid, r_rb, lds, s, g32);
  if (batched) return launch_mb(a, M > 16 ? 2 : 1, grid, ntl, lds, s);
  if (aff) return launch_gemv<4, true, true>(a, lds, s, grid);
  if (g32) return bits == 4 ? launch_gemv<4, true>(a, lds, s, grid) : launch_gemv<8, true>(a, lds, s, grid);
  if (bits == 4) return launch_gemv<4>(a, lds, s, grid);
  if (bits == 8) return launch_gemv<8>(a, lds, s, grid);
  return launch_gemv<16>(a, lds, s, grid);
}

extern "C" int ti_epilogue_bytes(void) { return (int)sizeof(ti_epilogue); }

// The kernel ti_gemm_wq_a16 launches for plain (not group-32) weights: the same predicates as
// gemm_impl (use_batched, wide_tile, tile_rows, rows_on).  For bench / profile labels.
extern "C" int ti_gemm_kernel_name(int bits, int x_kind, int M, int N, int K, char* buf, int len) {
  using namespace ti;
  if (!buf || len < 1) return ti_set_error(TI_ERR_ARG, "ti_gemm_kernel_name: null buffer");
  if ((bits != 4 && bits != 8 && bits != 16) || M < 1 || M > TI_GEMM_MAX_ROWS || N < 16 || K < 128)
    return ti_set_error(TI_ERR_ARG, "ti_gemm_kernel_name: bits %d M %d N %d K %d", bits, M, N, K);
  const bool packed_x = x_kind == TI_X_F16_PACKED;
  const bool batched = packed_x || use_batched(bits, x_kind, M, N, K);
  const bool tile = batched && x_kind == TI_X_F16 && (M >= tile_rows() || wide_tile(bits, M, N));
  const bool rows = !tile && batched && (packed_x || M > 32 || (M > 16 && rows_on()));
  const char* name = tile ? "gemm_tile_kernel" : rows ? "gemm_rows_kernel" : batched ? (mb_use_lds(M > 16 ? 2 : 1) ? "gemv_mb_kernel" : "gemv_mbr_kernel") : nullptr;
  if (name) snprintf(buf, (size_t)len, "%s", name);
  else snprintf(buf, (size_t)len, "gemv_wq_kernel<%d,%d>", bits, gemv_xmode(x_kind, M, K));
  return TI_OK;
}

extern "C" int ti_gemm_grid(int M, int N, int K) {
  if (M < 1 || M > 16 || N < 16 || K < 128 || (N & 15) || (K & 127) || !fused_fits(M, N, K)) return 0;
  return ti::gemv_grid(M, N, K, query_cus());
}

extern "C" int ti_gemm_wq_a16(const void* tiles, const uint16_t* scales, int bits, const void* x,
                              int x_kind, int ldx, const float* norm_w, float eps, int M, int N, int K,
                              const ti_epilogue* epi, ti_stream_t stream) {
  return gemm_impl(tiles, scales, bits, x, x_kind, ldx, norm_w, eps, M, N, K, epi, stream);
}

