// dequant.hpp -- packed INT4 / INT8 weight words -> fp16 MFMA B fragments (gfx950), shared by
// the decode GEMV (gemv.hip) and the persistent decode-layers kernel (pds.hip).
#pragma once
#include "common.hpp"

namespace ti {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------- dequant
// int4: word of 8 nibbles, nibble p holds element 2p, nibble p+4 element 2p+1, value q+8.
// int8: 4 signed bytes in k order; (b ^ 0x80) = b + 128 -> fp16 1024 + b + 128 - 1152.
__device__ __forceinline__ f16x2 deq_int8_pair(uint32_t t, uint32_t sel) {
  const uint32_t v = __builtin_amdgcn_perm(0x64646464u, t, sel);
  return __builtin_bit_cast(f16x2, v) - (f16x2){(f16)1152.0f, (f16)1152.0f};
}
__device__ __forceinline__ void deq_int8_word(uint32_t w, f16x8& r, int o) {
  const uint32_t t = w ^ 0x80808080u;
  const f16x2 lo = deq_int8_pair(t, 0x04010400u), hi = deq_int8_pair(t, 0x04030402u);
  r[o + 0] = lo[0];
  r[o + 1] = lo[1];
  r[o + 2] = hi[0];
  r[o + 3] = hi[1];
}

// int4, offset folded (5 VALU ops per 8 weights): fp16 lanes hold 1024 + n for the low
// nibble of each byte and 1024 + 16 n for the high one -- the raw bit patterns after one
// v_and_or_b32 each.  The activations are staged so that this is exact arithmetic: x at
// k % 8 in {2,3,6,7} (high-nibble slots) is pre-scaled by 1/16, making a_k * (1024 + 16 n)
// = 64 x_k + x_k n, and the MFMA sum t of one 128-k group then equals
//   sum_k x_k (n_k - 8) + D,   D = 1032 * sum_lo a_k + 1152 * sum_hi a_k,
// with D depending only on the activation row and the group: it is precomputed once per
// workgroup (corr table) and subtracted before the group scale is applied.
__device__ __forceinline__ f16x8 deq_int4_raw(uint32_t w, uint32_t magic) {
  const uint32_t w8 = w >> 8;
  u32x4 r;
  r[0] = (w & 0x000F000Fu) | magic;
  r[1] = (w & 0x00F000F0u) | magic;
  r[2] = (w8 & 0x000F000Fu) | magic;
  r[3] = (w8 & 0x00F000F0u) | magic;
  return __builtin_bit_cast(f16x8, r);
}

template <int BITS>
__device__ __forceinline__ f16x8 dequant_step(const u32x4 (&w)[BITS / 4], int s4, uint32_t magic) {
  if constexpr (BITS == 4) {
    return deq_int4_raw(w[0][s4], magic);
  } else if constexpr (BITS == 8) {
    f16x8 r;
    const u32x4 c = w[s4 >> 1];
    deq_int8_word(c[(s4 & 1) * 2 + 0], r, 0);
    deq_int8_word(c[(s4 & 1) * 2 + 1], r, 4);
    return r;
  } else {
    return __builtin_bit_cast(f16x8, w[s4]);
  }
}

}  // namespace ti
