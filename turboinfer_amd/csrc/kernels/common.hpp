// common.hpp -- shared device helpers for the gfx950 kernels (wave64, CDNA4).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ti_hip.h"

namespace ti {

typedef _Float16 f16;
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// acc + sc * t as two packed fp32 FMAs (v_pk_fma_f32): the same fused roundings as four fmaf
__device__ __forceinline__ f32x4 fma_scale4(float sc, f32x4 t, f32x4 acc) {
  const f32x2 s2 = {sc, sc};
  const f32x2 lo = __builtin_elementwise_fma(s2, (f32x2){t[0], t[1]}, (f32x2){acc[0], acc[1]});
  const f32x2 hi = __builtin_elementwise_fma(s2, (f32x2){t[2], t[3]}, (f32x2){acc[2], acc[3]});
  return (f32x4){lo[0], lo[1], hi[0], hi[1]};
}

constexpr int kWave = 64;

// ---------------------------------------------------------------- fp16 helpers
__device__ __forceinline__ float h2f(uint16_t h) { return (float)__builtin_bit_cast(f16, h); }
__device__ __forceinline__ uint16_t f2h(float f) { return __builtin_bit_cast(uint16_t, (f16)f); }

// fp32 -> fp16 bits, round to nearest even with subnormals, in integer arithmetic: used where
// device output must be bit-identical to the host / oracle (or_float_to_half); the hardware
// conversion rounds some fp16-subnormal results differently.
__device__ inline uint16_t f2h_soft(float f) {
  const uint32_t x = __builtin_bit_cast(uint32_t, f);
  const uint16_t s = (uint16_t)((x >> 16) & 0x8000u);
  const uint32_t ax = x & 0x7fffffffu;
  if (ax >= 0x7f800000u) return s | 0x7c00u | (ax > 0x7f800000u ? 0x200u : 0u);
  if (ax >= 0x477ff000u) return s | 0x7c00u;
  if (ax < 0x38800000u) {
    if (ax < 0x33000000u) return s;
    const uint32_t e = ax >> 23, m = (ax & 0x7fffffu) | 0x800000u, sh = 126u - e;
    const uint32_t hm = m >> sh, rem = m & ((1u << sh) - 1u), half = 1u << (sh - 1u);
    return s | (uint16_t)(hm + ((rem > half || (rem == half && (hm & 1u))) ? 1u : 0u));
  }
  uint32_t hb = (ax >> 13) - (112u << 10);
  const uint32_t rem = ax & 0x1fffu;
  if (rem > 0x1000u || (rem == 0x1000u && (hb & 1u))) ++hb;
  return s | (uint16_t)hb;
}

// ------------------------------------------------------------ wave reductions
template <int WIDTH>
__device__ __forceinline__ float wave_sum_xor(float v) {
#pragma unroll
  for (int o = WIDTH / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
template <int WIDTH>
__device__ __forceinline__ float wave_max_xor(float v) {
#pragma unroll
  for (int o = WIDTH / 2; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}

// Cross-lane exchanges on the VALU (DPP, gfx950 v_permlane16/32_swap) instead of the LDS
// crossbar (__shfl_xor -> ds_bpermute_b32, a round trip through the LDS pipe per step).
__device__ __forceinline__ unsigned lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0u, __builtin_bit_cast(unsigned, v), CTRL, 0xf, 0xf, false));
}
// v of lane l ^ O, exactly (O in {1, 2, 8, 16, 32}).
template <int O>
__device__ __forceinline__ float lane_xor(float v) {
  if constexpr (O == 1) {
    return dpp_f<0xB1>(v);            // quad_perm [1,0,3,2]
  } else if constexpr (O == 2) {
    return dpp_f<0x4E>(v);            // quad_perm [2,3,0,1]
  } else if constexpr (O == 8) {
    return dpp_f<0x128>(v);           // row_ror:8 within 16-lane rows == xor 8
  } else if constexpr (O == 16) {
    const unsigned u = __builtin_bit_cast(unsigned, v);
    const auto r = __builtin_amdgcn_permlane16_swap(u, u, false, false);
    return __builtin_bit_cast(float, (lane_id() & 16) ? r[0] : r[1]);
  } else {
    static_assert(O == 32, "lane_xor: O in {1, 2, 8, 16, 32}");
    const unsigned u = __builtin_bit_cast(unsigned, v);
    const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
    return __builtin_bit_cast(float, lane_id() < 32 ? r[1] : r[0]);
  }
}
template <int O>
__device__ __forceinline__ uint32_t lane_xor_u32(uint32_t v) {
  return __builtin_bit_cast(uint32_t, lane_xor<O>(__builtin_bit_cast(float, v)));
}
// All-reduce sum over aligned groups of WIDTH lanes (butterfly; the width-4 and width-8
// stages pair quads / half-rows by mirroring, which is valid once the smaller stages have
// made each quad / half-row uniform).
template <int WIDTH>
__device__ __forceinline__ float group_sum(float v) {
  if constexpr (WIDTH >= 2) v += lane_xor<1>(v);
  if constexpr (WIDTH >= 4) v += lane_xor<2>(v);
  if constexpr (WIDTH >= 8) v += dpp_f<0x141>(v);   // row_half_mirror: quad <-> other quad of the 8
  if constexpr (WIDTH >= 16) v += dpp_f<0x140>(v);  // row_mirror: half-row <-> other half of the 16
  if constexpr (WIDTH >= 32) v += lane_xor<16>(v);
  if constexpr (WIDTH >= 64) v += lane_xor<32>(v);
  return v;
}

// ------------------------------------------------------- write-through (sc1) accesses
// (persistent decode hand-offs, split merges: MI355X_MICROARCH.md "Hand-offs measured with sc1 loads")
constexpr int kAuxSc1Load = 16;   // buffer aux bit 4 = sc1 on gfx950

// 64 lanes x 16 B -> LDS at the wave-uniform byte address lds (M0 set and restored in the
// statement).  Issued from asm, so hipcc does not count it: the caller waits with a counted
// s_waitcnt vmcnt and a barrier before the LDS is read.
__device__ __forceinline__ void dma_1k_asm(const void* src_lane, uint32_t lds) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src_lane), "s"(lds)
               : "memory");
}

// max / sum with the lane 16 or 32 apart (l ^ 16, l ^ 32) through gfx950's v_permlane16/32_swap,
// VALU only (a __shfl_xor across rows is an LDS round trip): after a swap of x with itself, lane l
// holds x[l] in one result and x[l ^ 16] (x[l ^ 32]) in the other, in some order -- max and + of
// the two are exact and order-free.
__device__ __forceinline__ float xor16_max(float x) {
  const auto t = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(t[0]), __uint_as_float(t[1]));
}
__device__ __forceinline__ float xor32_max(float x) {
  const auto t = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(t[0]), __uint_as_float(t[1]));
}

// a raw buffer resource over [base, base + 2 GiB): the cache policy is the access's aux bits
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buffer_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t sc1_rsrc(const void* base) { return buffer_rsrc(base); }
__device__ __forceinline__ uint32_t ld_sc1_u32(const void* p) {
  return __hip_atomic_load((const uint32_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_sc1_f32(const float* p) { return __builtin_bit_cast(float, ld_sc1_u32(p)); }
__device__ __forceinline__ unsigned long long ld_sc1_u64(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1_u32(void* p, uint32_t v) {
  __hip_atomic_store((uint32_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1_f32(float* p, float v) { st_sc1_u32(p, __builtin_bit_cast(uint32_t, v)); }
__device__ __forceinline__ void st_sc1_u64(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ----------------------------------------------------- synthetic model stream
// Bit-identical to or_splitmix64 / or_synth_unit in oracle/ti_oracle.c.
__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}
__host__ __device__ __forceinline__ uint64_t synth_stream(uint64_t seed, uint32_t tid) {
  return splitmix64(seed ^ ((uint64_t)tid * 0xD1B54A32D192ED03ULL));
}
__host__ __device__ __forceinline__ float synth_unit(uint64_t stream, uint64_t idx) {
  const uint64_t h = splitmix64(stream + idx);
  const int32_t m = (int32_t)(h >> 40);
  return (float)(2 * m - (1 << 24)) * (1.0f / 16777216.0f);
}

// ---------------------------------------------------------------- tile layout
// See ti_hip.h: a tile is 16 output rows x 128 k; chunk c (1 KiB) holds, for lane l,
// 16 bytes of row (l & 15) starting at k = 32*(l>>4) + c*(32/chunks).
template <int BITS>
struct TileFmt {
  static constexpr int kChunks = BITS / 4;           // 1, 2, 4 dwordx4 per lane
  static constexpr int kBytes = 1024 * kChunks;
  static constexpr int kKPerChunk = 32 / kChunks;    // k values per lane per chunk
};

__host__ __device__ __forceinline__ size_t tile_index(int nt, int kt, int KT) {
  return (size_t)nt * KT + kt;
}

// ---------------------------------------------------------------- in-step launch stamps
// ti_engine_stamp_steps (ti_engine.h): the step graph captured with every decode kernel writing,
// per workgroup, wave 0's entry time and each wave's end time (s_memrealtime, 100 MHz) with plain
// vector stores into a host-owned device buffer.  `st` is NULL in every product launch (one scalar
// branch at the kernel end).
// per workgroup: [0] entry of wave 0, [1 + w] end of wave w (w < 8), [9..14] phase marks of
// diagnostic builds, [15] where wave 0 ran: XCC_ID << 32 | HW_ID (SE / SH / CU fields: which CU; two
// workgroups of a launch on one CU show here), [16 + w] diagnostic builds: wave w's end of stream
constexpr int kStampWords = 24;
__device__ __forceinline__ unsigned long long stamp_now() { return __builtin_amdgcn_s_memrealtime(); }
// Diagnostic builds (TI_STAMP_PHASES=1, never the product) also keep up to 6 phase marks of wave 0 in
// words 9..14 (kernel-specific; gemv_wq_kernel: DESIGN 4.18).
#ifndef TI_STAMP_PHASES
#define TI_STAMP_PHASES 0
#endif
#if TI_STAMP_PHASES
#define STAMP_MARK(var) const unsigned long long var = stamp_now()
#else
#define STAMP_MARK(var) const unsigned long long var = 0
#endif
__device__ __forceinline__ void stamp_end(unsigned long long* st, unsigned long long t_entry,
                                          unsigned long long ph0 = 0, unsigned long long ph1 = 0,
                                          unsigned long long ph2 = 0, unsigned long long ph3 = 0,
                                          unsigned long long ph4 = 0, unsigned long long ph5 = 0,
                                          unsigned long long wave_mark = 0) {
  if (st == nullptr) return;
  if ((threadIdx.x & 63) == 0) {
    const unsigned wave = threadIdx.x >> 6;
    const size_t wg = blockIdx.x + (size_t)gridDim.x * (blockIdx.y + (size_t)gridDim.y * blockIdx.z);
    unsigned long long* p = st + wg * kStampWords;
    if (wave < 8) p[1 + wave] = stamp_now();
    if (TI_STAMP_PHASES && wave < 8) p[16 + wave] = wave_mark;
    if (wave == 0) {
      p[0] = t_entry;
      // s_getreg_b32 HW_REG_HW_ID (4) and HW_REG_XCC_ID (20), all 32 bits
      const unsigned hw = __builtin_amdgcn_s_getreg(4 | (31 << 11)), xcc = __builtin_amdgcn_s_getreg(20 | (31 << 11));
      p[15] = ((unsigned long long)xcc << 32) | hw | (1ull << 63);
      if (TI_STAMP_PHASES) {
        p[9] = ph0; p[10] = ph1; p[11] = ph2; p[12] = ph3; p[13] = ph4; p[14] = ph5;
      }
    }
  }
}
// kinds reported with each stamped launch
enum { STAMP_OTHER = 0, STAMP_GEMV = 1, STAMP_ATTN = 2, STAMP_BEGIN = 3, STAMP_ROWS = 4, STAMP_TILE = 5,
       STAMP_RMSNORM = 6, STAMP_MB = 7 };

}  // namespace ti

// The stamp buffer slot of the next launch (host side, engine.cpp): NULL unless this thread is
// capturing a stamped step graph (ti_engine_stamp_steps) and the grid fits the buffer.
extern "C++" unsigned long long* ti_stamp_next(int kind, long grid);

// error helper shared by the launchers (defined in host/capi.cpp)
extern "C++" int ti_set_error(int code, const char* fmt, ...);
extern "C++" int ti_check_hip(hipError_t e, const char* what);
#define TI_HIP_CHECK(expr, what)                         \
  do {                                                   \
    hipError_t _e = (expr);                              \
    if (_e != hipSuccess) return ti_check_hip(_e, what); \
  } while (0)
#define TI_LAUNCH_CHECK(what) TI_HIP_CHECK(hipGetLastError(), what)

