// wpack.cpp -- host-side quantize + pack of linear weights into the gfx950 tile format.
//
// The reference Quantizer (src/optimize/quantization.cpp) quantizes a whole tensor with one
// symmetric scale (calculate_quantization_info :355-360, 375-378), stores INT4 unpacked in
// int32 (:45-46) and drops the scale (quantize_model :89-118).  Here the same symmetric
// formula -- scale = absmax / 7 (int4) or / 127 (int8), q = clamp(round(x / scale)) with
// std::round (half away from zero) -- is applied per group of 128 k of one output column,
// and the result is packed two nibbles per byte with an fp16 scale per group.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include <hip/hip_runtime.h>

#include "ti_hip.h"

int ti_set_error(int code, const char* fmt, ...);

namespace {

inline int map_row(int c, int row_map, int row_offset) {
  return row_map == TI_ROWS_INTERLEAVE8 ? 16 * (c >> 3) + (c & 7) + row_offset : row_offset + c;
}

inline float clamp_ref(float v, float lo, float hi) {   // std::max(lo, std::min(hi, v))
  const float t = (v < hi) ? v : hi;
  return (lo < t) ? t : lo;
}

inline uint16_t to_half(float f) {
  const _Float16 h = (_Float16)f;                         // round to nearest even
  uint16_t u;
  std::memcpy(&u, &h, 2);
  return u;
}

}  // namespace

extern "C" size_t ti_wpack_tile_bytes(int bits, int K, int N) {
  if (K <= 0 || N <= 0) return 0;
  return (size_t)(N / 16) * (size_t)(K / 128) * 256u * (size_t)(bits & ~(TI_BITS_G32 | TI_BITS_AFF));
}

extern "C" size_t ti_wpack_scale_bytes(int bits, int K, int N) {
  if (bits == 16 || K <= 0 || N <= 0) return 0;
  return (size_t)(N / 16) * (size_t)(K / 128) * 16u * sizeof(uint16_t) * ((bits & TI_BITS_G32) ? 4u : 1u) *
         ((bits & TI_BITS_AFF) ? 2u : 1u);   // affine group-32: the block minimums follow the scales
}

namespace {

// One row r of tile (nt, g): the 128 integer weights q of k-group g into the tile's lanes.
// g32: step s4 of lane kq holds k = 32 s4 + 8 kq + e (each MFMA one 32-block); else k = 32 kq +
// 8 s4 + e.  int4 nibble p of a word: element 2p at bits 4p, element 2p+1 at bits 16 + 4p, q + 8.
void pack_row(uint8_t* tile, int bits, bool g32, int r, const int8_t* q) {
  auto kidx = [&](int kq, int s4, int e) { return g32 ? 32 * s4 + 8 * kq + e : 32 * kq + 8 * s4 + e; };
  for (int kq = 0; kq < 4; ++kq) {
    const int lane = kq * 16 + r;
    if (bits == 4) {
      uint32_t words[4];
      for (int s4 = 0; s4 < 4; ++s4) {
        uint32_t wd = 0;
        for (int e = 0; e < 8; ++e) {
          const uint32_t nib = (uint32_t)(q[kidx(kq, s4, e)] + 8) & 0xF;
          wd |= nib << ((e & 1) ? (16 + 4 * (e >> 1)) : (4 * (e >> 1)));
        }
        words[s4] = wd;
      }
      std::memcpy(tile + lane * 16, words, 16);
    } else {   // int8: chunk ch holds steps 2 ch, 2 ch + 1 (8 bytes each)
      for (int ch = 0; ch < 2; ++ch) {
        int8_t b[16];
        for (int h = 0; h < 2; ++h)
          for (int e = 0; e < 8; ++e) b[8 * h + e] = q[kidx(kq, 2 * ch + h, e)];
        std::memcpy(tile + ch * 1024 + lane * 16, b, 16);
      }
    }
  }
}

}  // namespace

extern "C" int ti_wpack_q_host(const int8_t* q, const uint16_t* d, int K, int N_src, int N_total, int bits, int row_map,
                               int row_offset, void* tiles, uint16_t* scales) {
  bits &= ~TI_BITS_G32;
  if (!q || !d || !tiles || !scales) return ti_set_error(TI_ERR_ARG, "ti_wpack_q_host: null pointer");
  if (bits != 4 && bits != 8) return ti_set_error(TI_ERR_ARG, "ti_wpack_q_host: bits %d (4 or 8)", bits);
  if (K <= 0 || (K & 127) || N_total <= 0 || (N_total & 15) || N_src <= 0)
    return ti_set_error(TI_ERR_ARG, "ti_wpack_q_host: K %% 128 / N %% 16 (K=%d N_total=%d)", K, N_total);
  if (row_map == TI_ROWS_INTERLEAVE8 && (N_src & 7)) return ti_set_error(TI_ERR_ARG, "ti_wpack_q_host: interleave needs N %% 8 == 0");
  if (map_row(N_src - 1, row_map, row_offset) >= N_total || row_offset < 0)
    return ti_set_error(TI_ERR_ARG, "ti_wpack_q_host: rows do not fit N_total");
  const int lo = bits == 4 ? -8 : -127, hi = bits == 4 ? 7 : 127;
  const int KT = K / 128;
  const size_t tile_bytes = (size_t)256 * bits;
  uint8_t* tb = static_cast<uint8_t*>(tiles);
  int8_t col[128];
  for (int c = 0; c < N_src; ++c) {
    const int n = map_row(c, row_map, row_offset), nt = n >> 4, r = n & 15;
    for (int g = 0; g < KT; ++g) {
      for (int i = 0; i < 128; ++i) {
        const int v = q[(size_t)(g * 128 + i) * N_src + c];
        if (v < lo || v > hi) return ti_set_error(TI_ERR_ARG, "ti_wpack_q_host: weight %d outside [%d, %d]", v, lo, hi);
        col[i] = (int8_t)v;
      }
      for (int s4 = 0; s4 < 4; ++s4) scales[(((size_t)nt * KT + g) * 4 + s4) * 16 + r] = d[(size_t)(g * 4 + s4) * N_src + c];
      pack_row(tb + ((size_t)nt * KT + g) * tile_bytes, bits, true, r, col);
    }
  }
  return TI_OK;
}

extern "C" int ti_wpack_host(const float* w, int K, int N_src, int N_total, int bits, int scale_mode, int row_map,
                             int row_offset, void* tiles, uint16_t* scales) {
  if (!w || !tiles) return ti_set_error(TI_ERR_ARG, "ti_wpack_host: null pointer");
  if (bits == (4 | TI_BITS_G32 | TI_BITS_AFF)) {
    // fp32 weights onto an affine group-32 engine: ggml's Q4_1 rounding per 32-block
    // (d = (max - min) / 15, m = min, q = round-half-up((w - min) / d) clamped to 15), then packed exactly
    if (K <= 0 || (K & 127) || N_src <= 0) return ti_set_error(TI_ERR_ARG, "ti_wpack_host: K %% 128 (K=%d)", K);
    std::vector<uint8_t> q((size_t)K * N_src);
    std::vector<uint16_t> d((size_t)(K / 32) * N_src), m(d.size());
    for (int c = 0; c < N_src; ++c)
      for (int b = 0; b < K / 32; ++b) {
        float lo = INFINITY, hi = -INFINITY;
        for (int i = 0; i < 32; ++i) {
          const float v = w[(size_t)(b * 32 + i) * N_src + c];
          lo = std::min(lo, v);
          hi = std::max(hi, v);
        }
        const float dd = (hi - lo) / 15.0f, id = dd != 0.0f ? 1.0f / dd : 0.0f;
        d[(size_t)b * N_src + c] = to_half(dd);
        m[(size_t)b * N_src + c] = to_half(lo);
        for (int i = 0; i < 32; ++i) {
          const size_t at = (size_t)(b * 32 + i) * N_src + c;
          q[at] = (uint8_t)std::min(15, (int)((w[at] - lo) * id + 0.5f));
        }
      }
    return ti_wpack_q1_host(q.data(), d.data(), m.data(), K, N_src, N_total, row_map, row_offset, tiles, scales);
  }
  const bool g32 = (bits & TI_BITS_G32) != 0;
  bits &= ~TI_BITS_G32;
  if ((bits != 4 && bits != 8 && bits != 16) || (g32 && bits == 16)) return ti_set_error(TI_ERR_ARG, "ti_wpack_host: bits %d", bits);
  if (K <= 0 || (K & 127) || N_total <= 0 || (N_total & 15) || N_src <= 0)
    return ti_set_error(TI_ERR_ARG, "ti_wpack_host: K %% 128 / N %% 16 (K=%d N_total=%d)", K, N_total);
  if (row_map == TI_ROWS_INTERLEAVE8 && (N_src & 7)) return ti_set_error(TI_ERR_ARG, "ti_wpack_host: interleave needs N %% 8 == 0");
  if (map_row(N_src - 1, row_map, row_offset) >= N_total || row_offset < 0)
    return ti_set_error(TI_ERR_ARG, "ti_wpack_host: rows do not fit N_total");
  if (bits != 16 && !scales) return ti_set_error(TI_ERR_ARG, "ti_wpack_host: scales required");
  if (scale_mode < TI_SCALE_GROUP || scale_mode > TI_SCALE_UNIT) return ti_set_error(TI_ERR_ARG, "ti_wpack_host: scale_mode");
  const int KT = K / 128;
  uint8_t* tb = static_cast<uint8_t*>(tiles);

  if (bits == 16) {
    for (int c = 0; c < N_src; ++c) {
      const int n = map_row(c, row_map, row_offset), nt = n >> 4, r = n & 15;
      for (int k = 0; k < K; ++k) {
        const int kt = k >> 7, kk = k & 127, kq = kk >> 5, ch = (kk & 31) >> 3, e = kk & 7;
        const size_t off = ((size_t)nt * KT + kt) * 2048 + (size_t)ch * 512 + (size_t)(kq * 16 + r) * 8 + e;
        reinterpret_cast<uint16_t*>(tb)[off] = to_half(w[(size_t)k * N_src + c]);
      }
    }
    return TI_OK;
  }

  const float qmax = bits == 4 ? 7.0f : 127.0f, qlo = bits == 4 ? -7.0f : -128.0f;
  float tensor_scale = 1.0f;
  if (scale_mode == TI_SCALE_TENSOR) {
    float amax = 0.0f;
    for (size_t i = 0; i < (size_t)K * N_src; ++i) amax = std::max(amax, std::fabs(w[i]));
    tensor_scale = amax / qmax;
  }
  const size_t tile_bytes = (size_t)256 * bits;
  float col[128];
  for (int c = 0; c < N_src; ++c) {
    const int n = map_row(c, row_map, row_offset), nt = n >> 4, r = n & 15;
    for (int g = 0; g < KT; ++g) {
      for (int i = 0; i < 128; ++i) col[i] = w[(size_t)(g * 128 + i) * N_src + c];
      int8_t q[128];
      const int gsz = g32 ? 32 : 128;   // weights per scale
      for (int b0 = 0; b0 < 128; b0 += gsz) {
        float amax = 0.0f;
        for (int i = b0; i < b0 + gsz; ++i) amax = std::max(amax, std::fabs(col[i]));
        const float sc = scale_mode == TI_SCALE_GROUP ? amax / qmax : tensor_scale;
        const uint16_t sh = to_half(scale_mode == TI_SCALE_UNIT ? 1.0f : sc);
        if (g32) scales[(((size_t)nt * KT + g) * 4 + b0 / 32) * 16 + r] = sh;
        else scales[((size_t)nt * KT + g) * 16 + r] = sh;
        for (int i = b0; i < b0 + gsz; ++i) {
          const float v = scale_mode == TI_SCALE_UNIT ? std::round(col[i]) : std::round(col[i] / sc);
          q[i] = (int8_t)clamp_ref(v, qlo, qmax);
        }
      }
      pack_row(tb + ((size_t)nt * KT + g) * tile_bytes, bits, g32, r, q);
    }
  }
  return TI_OK;
}

// GGUF Q4_1 blocks (ggml: weight = d * q + m, q in 0..15): the tiles and scales of the Q4_0 form
// with q - 8 (the kernels' offset-8 nibbles hold q itself), then the block minimums m packed in
// the scales' layout right after them.
extern "C" int ti_wpack_q1_host(const uint8_t* q, const uint16_t* d, const uint16_t* m, int K, int N_src, int N_total,
                                int row_map, int row_offset, void* tiles, uint16_t* scales) {
  if (!q || !d || !m || !tiles || !scales) return ti_set_error(TI_ERR_ARG, "ti_wpack_q1_host: null pointer");
  if (K <= 0 || (K & 127) || N_total <= 0 || (N_total & 15) || N_src <= 0)
    return ti_set_error(TI_ERR_ARG, "ti_wpack_q1_host: K %% 128 / N %% 16 (K=%d N_total=%d)", K, N_total);
  std::vector<int8_t> v((size_t)K * N_src);
  for (size_t i = 0; i < v.size(); ++i) {
    if (q[i] > 15) return ti_set_error(TI_ERR_ARG, "ti_wpack_q1_host: weight %d outside [0, 15]", (int)q[i]);
    v[i] = (int8_t)((int)q[i] - 8);
  }
  int rc = ti_wpack_q_host(v.data(), d, K, N_src, N_total, 4, row_map, row_offset, tiles, scales);
  if (rc != TI_OK) return rc;
  // the minimums through the same scale packing (into a scratch tile image)
  std::vector<uint8_t> scratch(ti_wpack_tile_bytes(4, K, N_total));
  uint16_t* mins = scales + ti_wpack_scale_bytes(4 | TI_BITS_G32, K, N_total) / sizeof(uint16_t);
  return ti_wpack_q_host(v.data(), m, K, N_src, N_total, 4, row_map, row_offset, scratch.data(), mins);
}
