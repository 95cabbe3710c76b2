/*
 * ti_oracle.c -- TEST INFRASTRUCTURE ONLY.  See ti_oracle.h.
 *
 * CPU restatement of the reference's decode-path arithmetic.  Compiled with
 * -ffp-contract=off: every place where the reference build fuses a multiply-add
 * (g++ -O3 -mfma contracts `s += a*b` into vfmadd231ss, verified with objdump on
 * the compiled reference) is written here as an explicit fmaf(), and every place it
 * does not is written as separate operations, so results are bit-identical to the
 * compiled reference (checked by tests/test_oracle_golden.py).
 */
#include "ti_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* In-order dot-product accumulation as g++ -O3 -mavx2 -mfma emits it for a loop
 * `s += a[i]*b[i]` over contiguous operands: the products of the 8-wide main loop
 * and of one 4-wide epilogue step are computed by vmulps (rounded) and added in
 * order by vaddss; the last n%4 terms fall to the scalar loop, which is contracted
 * (vfmadd231ss).  Read off the disassembly of rms_norm (tensor_engine.cpp:1493). */
static float dot_ordered(float s, const float* a, const float* b, size_t n) {
  size_t i = 0;
  for (; i + 8 <= n; i += 8)
    for (int l = 0; l < 8; ++l) s = s + a[i + l] * b[i + l];
  if (i + 4 <= n) {
    for (int l = 0; l < 4; ++l) s = s + a[i + l] * b[i + l];
    i += 4;
  }
  for (; i < n; ++i) s = fmaf(a[i], b[i], s);
  return s;
}

/* ------------------------------------------------------------------ matmul */

/* tensor_engine.cpp:620-633 -- `sum += a_batch[i*K+k] * b_data[k*N+j]` for k = 0..K-1
 * starting from sum = 0.0f, contracted to one fma per k.  The loop below keeps the
 * same per-output chain but walks B row-wise (N independent chains) so it streams. */
void or_matmul(const float* a, const float* b, float* c, size_t rows, size_t K, size_t N) {
  for (size_t r = 0; r < rows; ++r) {
    float* acc = c + r * N;
    for (size_t j = 0; j < N; ++j) acc[j] = 0.0f;
    const float* ar = a + r * K;
    for (size_t k = 0; k < K; ++k) {
      const float av = ar[k];
      const float* br = b + k * N;
      for (size_t j = 0; j < N; ++j) acc[j] = fmaf(av, br[j], acc[j]);
    }
  }
}

/* ---------------------------------------------------------------- rms_norm */

/* tensor_engine.cpp:1488-1505 */
void or_rms_norm(const float* x, const float* w, float* y, size_t rows, size_t n, float eps) {
  for (size_t r = 0; r < rows; ++r) {
    const float* xr = x + r * n;
    const float ss = dot_ordered(0.0f, xr, xr, n);                 /* :1492-1495 */
    const float rms = sqrtf(ss / (float)n + eps);                  /* :1496 */
    for (size_t i = 0; i < n; ++i) y[r * n + i] = (xr[i] / rms) * w[i]; /* :1499-1501 */
  }
}

/* -------------------------------------------------------------------- RoPE */

/* tensor_engine.cpp:1561-1566 frequencies, :1592-1616 rotation of interleaved pairs
 * (2i, 2i+1).  The compiled reference evaluates (sincosf + vmulps + vfmadd132ps /
 * vfnmadd132ps on the packed pair, read off the disassembly):
 *   even = x*cos - y*sin  as fmaf(-y, sin, x*cos)
 *   odd  = x*sin + y*cos  as fmaf( y, cos, x*sin)
 * (pinned by the rope golden vectors). */
void or_apply_rope(const float* x, float* y, size_t B, size_t heads, size_t S, size_t D,
                   const float* pos, int pos_2d, float theta) {
  const size_t half = D / 2;
  float* freqs = (float*)malloc(sizeof(float) * (half ? half : 1));
  for (size_t i = 0; i < half; ++i)
    freqs[i] = 1.0f / powf(theta, (float)(2 * i) / (float)D);
  for (size_t b = 0; b < B; ++b)
    for (size_t h = 0; h < heads; ++h)
      for (size_t s = 0; s < S; ++s) {
        const float p = pos_2d ? pos[b * S + s] : pos[s];
        const size_t base = ((b * heads + h) * S + s) * D;
        for (size_t i = 0; i < half; ++i) {
          const float xe = x[base + 2 * i], xo = x[base + 2 * i + 1];
          const float ang = p * freqs[i];
          const float cv = cosf(ang), sv = sinf(ang);
          y[base + 2 * i] = fmaf(-xo, sv, xe * cv);
          y[base + 2 * i + 1] = fmaf(xo, cv, xe * sv);
        }
      }
  free(freqs);
}

/* -------------------------------------------------------------- elementwise */

void or_silu(const float* x, float* y, size_t n) {           /* :913-917 */
  for (size_t i = 0; i < n; ++i) y[i] = x[i] / (1.0f + expf(-x[i]));
}
void or_relu(const float* x, float* y, size_t n) {           /* :846-866, std::max(0.0f, x) */
  for (size_t i = 0; i < n; ++i) y[i] = (0.0f < x[i]) ? x[i] : 0.0f;
}
void or_add(const float* a, const float* b, float* y, size_t n) {  /* :1648-1675 */
  for (size_t i = 0; i < n; ++i) y[i] = a[i] + b[i];
}
void or_multiply(const float* a, const float* b, float* y, size_t n) { /* :1702-1740 */
  for (size_t i = 0; i < n; ++i) y[i] = a[i] * b[i];
}

/* ----------------------------------------------------------------- softmax */

static inline float max_ps_lane(float a, float b) { return (a > b) ? a : b; } /* _mm256_max_ps(a,b) */
static inline float min_ps_lane(float a, float b) { return (a < b) ? a : b; } /* _mm256_min_ps(a,b) */
static inline float std_max(float a, float b) { return (a < b) ? b : a; }     /* std::max(a,b) */

/* fast_exp_avx2, tensor_engine.cpp:262-302, one lane. */
float or_fast_exp(float x) {
  x = max_ps_lane(min_ps_lane(x, 88.0f), -88.0f);
  const float xl = x * 1.44269504f;
  const float fx = floorf(xl);
  const float frac = xl - fx;
  const int32_t fi = (int32_t)fx;                      /* cvtps_epi32 of an integral value */
  const uint32_t bits = (uint32_t)(fi + 127) << 23;
  float e;
  memcpy(&e, &bits, 4);
  const float xf = frac * 0.69314718f;
  float poly = 1.0f;
  poly = fmaf(xf, 0.69314718f, poly);
  const float x2 = xf * xf;
  poly = fmaf(x2, 0.24022651f, poly);
  const float x3 = x2 * xf;
  poly = fmaf(x3, 0.05550410f, poly);
  const float x4 = x3 * xf;
  poly = fmaf(x4, 0.00961812f, poly);
  return e * poly;
}

/* softmax, tensor_engine.cpp:943-1037: AVX2 path for n >= 16 (8 lane max, fast exp,
 * 8 lane sums, sequential horizontal reductions, std::exp remainder), scalar else. */
void or_softmax(const float* x, float* y, size_t rows, size_t n, float temperature) {
  for (size_t r = 0; r < rows; ++r) {
    const float* in = x + r * n;
    float* out = y + r * n;
    if (n >= 16) {
      const size_t se = (n / 8) * 8;
      float mx[8], sm[8];
      for (int l = 0; l < 8; ++l) { mx[l] = -INFINITY; sm[l] = 0.0f; }
      for (size_t i = 0; i < se; i += 8)
        for (int l = 0; l < 8; ++l) mx[l] = max_ps_lane(mx[l], in[i + l]);
      float m = -INFINITY;
      for (int l = 0; l < 8; ++l) m = std_max(m, mx[l]);
      for (size_t i = se; i < n; ++i) m = std_max(m, in[i]);
      for (size_t i = 0; i < se; i += 8)
        for (int l = 0; l < 8; ++l) {
          const float e = or_fast_exp((in[i + l] - m) / temperature);
          out[i + l] = e;
          sm[l] = sm[l] + e;
        }
      float s = 0.0f;
      for (int l = 0; l < 8; ++l) s += sm[l];
      for (size_t i = se; i < n; ++i) {
        const float e = expf((in[i] - m) / temperature);
        out[i] = e;
        s += e;
      }
      for (size_t i = 0; i < n; ++i) out[i] = out[i] / s;
    } else {
      float m = in[0];
      for (size_t i = 1; i < n; ++i) m = std_max(m, in[i]);
      float s = 0.0f;
      for (size_t i = 0; i < n; ++i) {
        const float e = expf((in[i] - m) / temperature);
        out[i] = e;
        s += e;
      }
      for (size_t i = 0; i < n; ++i) out[i] /= s;
    }
  }
}

/* ---------------------------------------------------------------- attention */

/* attention_fast_incremental, tensor_engine.cpp:1288-1385 (AVX2 build). */
void or_attention_incremental(const float* q, const float* k, const float* v, float* out,
                              size_t B, size_t S, size_t D) {
  const float scale = 1.0f / sqrtf((float)D);                           /* :1288 */
  float* sc = (float*)malloc(sizeof(float) * (S ? S : 1));
  for (size_t b = 0; b < B; ++b) {
    const float* qb = q + b * D;
    const float* kb = k + b * S * D;
    const float* vb = v + b * S * D;
    const size_t de = (D / 8) * 8;
    for (size_t j = 0; j < S; ++j) {                                    /* :1295-1327 */
      float lane[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (size_t h = 0; h < de; h += 8)
        for (int l = 0; l < 8; ++l) lane[l] = fmaf(qb[h + l], kb[j * D + h + l], lane[l]);
      float s = 0.0f;
      for (int l = 0; l < 8; ++l) s += lane[l];
      s = dot_ordered(s, qb + de, kb + j * D + de, D - de);
      sc[j] = s * scale;
    }
    float mx = sc[0];                                                   /* max_element */
    for (size_t j = 1; j < S; ++j) if (mx < sc[j]) mx = sc[j];
    float se = 0.0f;
    for (size_t j = 0; j < S; ++j) { sc[j] = expf(sc[j] - mx); se += sc[j]; } /* :1333-1336 */
    for (size_t j = 0; j < S; ++j) sc[j] /= se;
    const size_t ke = (S / 8) * 8;
    for (size_t h = 0; h < D; ++h) {                                    /* :1343-1384 */
      float lane[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (size_t j = 0; j < ke; j += 8)
        for (int l = 0; l < 8; ++l) lane[l] = fmaf(sc[j + l], vb[(j + l) * D + h], lane[l]);
      float o = 0.0f;
      for (int l = 0; l < 8; ++l) o += lane[l];
      for (size_t j = ke; j < S; ++j) o = fmaf(sc[j], vb[j * D + h], o);
      out[b * D + h] = o;
    }
  }
  free(sc);
}

/* multi_head_attention, tensor_engine.cpp:1149-1252: slice heads out of the hidden
 * dim, run attention() (-> attention_fast_incremental since q is [B,1,hd]) per head,
 * concatenate. */
void or_multi_head_attention(const float* q, const float* k, const float* v, float* out,
                             size_t B, size_t S, size_t H, size_t num_heads) {
  const size_t hd = H / num_heads;
  float* qh = (float*)malloc(sizeof(float) * B * hd);
  float* kh = (float*)malloc(sizeof(float) * B * S * hd + 4);
  float* vh = (float*)malloc(sizeof(float) * B * S * hd + 4);
  float* oh = (float*)malloc(sizeof(float) * B * hd);
  for (size_t h = 0; h < num_heads; ++h) {
    for (size_t b = 0; b < B; ++b) {
      memcpy(qh + b * hd, q + b * H + h * hd, sizeof(float) * hd);
      for (size_t s = 0; s < S; ++s) {
        memcpy(kh + (b * S + s) * hd, k + (b * S + s) * H + h * hd, sizeof(float) * hd);
        memcpy(vh + (b * S + s) * hd, v + (b * S + s) * H + h * hd, sizeof(float) * hd);
      }
    }
    or_attention_incremental(qh, kh, vh, oh, B, S, hd);
    for (size_t b = 0; b < B; ++b) memcpy(out + b * H + h * hd, oh + b * hd, sizeof(float) * hd);
  }
  free(qh); free(kh); free(vh); free(oh);
}

/* ------------------------------------------------------------ quantization */

/* calculate_quantization_info, quantization.cpp:343-392 */
void or_quant_info(const float* x, size_t n, int bits, int symmetric, float* scale, float* zero_point) {
  float mn = x[0], mx = x[0];
  for (size_t i = 1; i < n; ++i) {
    mn = (x[i] < mn) ? x[i] : mn;   /* std::min(min_val, data[i]) */
    mx = (mx < x[i]) ? x[i] : mx;   /* std::max(max_val, data[i]) */
  }
  const float amn = fabsf(mn), amx = fabsf(mx);
  const float absmax = (amn < amx) ? amx : amn;
  if (bits == 8) {
    if (symmetric) { *scale = absmax / 127.0f; *zero_point = 0.0f; }
    else { *scale = (mx - mn) / 255.0f; *zero_point = -mn / *scale; }
  } else {
    if (symmetric) { *scale = absmax / 7.0f; *zero_point = 0.0f; }
    else { *scale = (mx - mn) / 15.0f; *zero_point = -mn / *scale; }
  }
}

static inline float clampf_ref(float v, float lo, float hi) {
  /* std::max(lo, std::min(hi, v)) with std semantics (NaN -> hi, as in the reference) */
  const float t = (v < hi) ? v : hi;
  return (lo < t) ? t : lo;
}

void or_quantize_int8(const float* x, int8_t* q, size_t n, float scale, float zp) { /* :662-674 */
  for (size_t i = 0; i < n; ++i) {
    const float v = clampf_ref(roundf(x[i] / scale + zp), -128.0f, 127.0f);
    q[i] = (int8_t)v;
  }
}
void or_quantize_int4(const float* x, int32_t* q, size_t n, float scale, float zp) { /* :676-693 */
  for (size_t i = 0; i < n; ++i) {
    float v = roundf(x[i] / scale - zp);
    v = (zp == 0.0f) ? clampf_ref(v, -7.0f, 7.0f) : clampf_ref(v, 0.0f, 15.0f);
    q[i] = (int32_t)v;
  }
}
void or_dequantize_int8(const int8_t* q, float* y, size_t n, float scale, float zp) { /* :695-702 */
  for (size_t i = 0; i < n; ++i) y[i] = scale * ((float)q[i] - zp);
}
void or_dequantize_int4(const int32_t* q, float* y, size_t n, float scale, float zp) { /* :704-712 */
  for (size_t i = 0; i < n; ++i) y[i] = scale * ((float)q[i] + zp);
}

/* --------------------------------------------------------------- fp16 bits */

float or_half_to_float(uint16_t h) {
  const uint32_t s = (uint32_t)(h >> 15) << 31;
  uint32_t e = (h >> 10) & 0x1f, m = h & 0x3ff, bits;
  if (e == 0) {
    if (m == 0) bits = s;
    else {                                   /* subnormal */
      int sh = 0;
      while (!(m & 0x400)) { m <<= 1; ++sh; }
      m &= 0x3ff;
      bits = s | ((uint32_t)(113 - sh) << 23) | (m << 13);
    }
  } else if (e == 31) bits = s | 0x7f800000u | (m << 13);
  else bits = s | ((e + 112) << 23) | (m << 13);
  float f;
  memcpy(&f, &bits, 4);
  return f;
}

uint16_t or_float_to_half(float f) {
  uint32_t x;
  memcpy(&x, &f, 4);
  const uint16_t s = (uint16_t)((x >> 16) & 0x8000);
  const uint32_t ax = x & 0x7fffffffu;
  if (ax >= 0x7f800000u) return s | 0x7c00 | (ax > 0x7f800000u ? 0x200 : 0);
  if (ax >= 0x477ff000u) return s | 0x7c00;                 /* rounds to inf */
  if (ax < 0x38800000u) {                                    /* subnormal half or zero */
    if (ax < 0x33000000u) return s;                          /* < 2^-25 -> 0 (tie at 2^-25 -> even 0) */
    const uint32_t e = ax >> 23, m = (ax & 0x7fffff) | 0x800000;
    const uint32_t shift = 126 - e;                          /* half mantissa = M >> (126 - e) */
    const uint32_t hm = m >> (shift);
    const uint32_t rem = m & ((1u << shift) - 1), halfway = 1u << (shift - 1);
    uint32_t r = hm;
    if (rem > halfway || (rem == halfway && (hm & 1))) ++r;
    return s | (uint16_t)r;
  }
  uint32_t hbits = ((ax >> 13) - (112u << 10));
  const uint32_t rem = ax & 0x1fff;
  if (rem > 0x1000 || (rem == 0x1000 && (hbits & 1))) ++hbits;
  return s | (uint16_t)hbits;
}

/* Group quantizer of the build's format (restates quantize_to_int4/int8 symmetric
 * branch per group; the reference has only the per-tensor form). */
void or_quantize_groups(const float* w, size_t K, size_t N, int bits, int group, int scale_mode,
                        int8_t* q, uint16_t* scale_f16) {
  const float qmax = (bits == 4) ? 7.0f : 127.0f;
  const float qlo = (bits == 4) ? -7.0f : -128.0f;
  const size_t G = K / (size_t)group;
  float tensor_scale = 1.0f;
  if (scale_mode == 1) {
    float absmax = 0.0f;
    for (size_t i = 0; i < K * N; ++i) { const float a = fabsf(w[i]); absmax = (absmax < a) ? a : absmax; }
    tensor_scale = absmax / qmax;
  }
  for (size_t n = 0; n < N; ++n)
    for (size_t g = 0; g < G; ++g) {
      float s;
      if (scale_mode == 0) {
        float absmax = 0.0f;
        for (size_t i = 0; i < (size_t)group; ++i) {
          const float a = fabsf(w[(g * group + i) * N + n]);
          absmax = (absmax < a) ? a : absmax;
        }
        s = absmax / qmax;
      } else if (scale_mode == 1) s = tensor_scale;
      else s = 1.0f;
      scale_f16[n * G + g] = or_float_to_half(s);
      for (size_t i = 0; i < (size_t)group; ++i) {
        const size_t k = g * group + i;
        float v = (scale_mode == 2) ? roundf(w[k * N + n]) : roundf(w[k * N + n] / s);
        v = clampf_ref(v, qlo, qmax);
        q[n * K + k] = (int8_t)v;
      }
    }
}

void or_dequantize_groups(const int8_t* q, const uint16_t* scale_f16, size_t K, size_t N, int group,
                          float* w) {
  const size_t G = K / (size_t)group;
  for (size_t n = 0; n < N; ++n)
    for (size_t k = 0; k < K; ++k)
      w[k * N + n] = (float)q[n * K + k] * or_half_to_float(scale_f16[n * G + k / group]);
}

/* --------------------------------------------------------- synthetic model */

uint64_t or_splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

/* u in [-1, 1) with 24 random bits, exactly representable. */
float or_synth_unit(uint64_t seed, uint32_t tensor_id, uint64_t idx) {
  const uint64_t stream = or_splitmix64(seed ^ ((uint64_t)tensor_id * 0xD1B54A32D192ED03ULL));
  const uint64_t h = or_splitmix64(stream + idx);
  const int32_t m = (int32_t)(h >> 40);                /* 0 .. 2^24-1 */
  return (float)(2 * m - (1 << 24)) * (1.0f / 16777216.0f);
}

void or_synth_linear(uint64_t seed, uint32_t tensor_id, size_t K, size_t N, float* w) {
  const float amp = sqrtf(3.0f) / sqrtf((float)K);
  for (size_t i = 0; i < K * N; ++i) w[i] = or_synth_unit(seed, tensor_id, i) * amp;
}

enum { TID_EMB = 1, TID_OUT_NORM = 2, TID_LM_HEAD = 3, TID_LAYER0 = 16 };
enum { TL_ATTN_NORM = 0, TL_FFN_NORM, TL_Q, TL_K, TL_V, TL_O, TL_G, TL_U, TL_D };
#define TID_LAYER(l, t) ((uint32_t)(TID_LAYER0 + 16 * (l) + (t)))
#define TID_KV(l, isv) ((uint32_t)(0x100000 + 2 * (l) + (isv)))

static float* synth_quant_linear(const or_model_config* c, uint64_t seed, uint32_t tid, size_t K, size_t N) {
  float* w = (float*)malloc(sizeof(float) * K * N);
  or_synth_linear(seed, tid, K, N, w);
  if (c->bits == 16) {                                   /* fp16 weights */
    for (size_t i = 0; i < K * N; ++i) w[i] = or_half_to_float(or_float_to_half(w[i]));
    return w;
  }
  int8_t* q = (int8_t*)malloc(K * N);
  uint16_t* s = (uint16_t*)malloc(sizeof(uint16_t) * N * (K / c->group));
  or_quantize_groups(w, K, N, c->bits, c->group, 0, q, s);
  or_dequantize_groups(q, s, K, N, c->group, w);
  free(q); free(s);
  return w;
}

static float* synth_norm(uint64_t seed, uint32_t tid, size_t n, float jitter) {
  float* w = (float*)malloc(sizeof(float) * n);
  for (size_t i = 0; i < n; ++i) w[i] = 1.0f + jitter * or_synth_unit(seed, tid, i);
  return w;
}

or_model* or_model_synth(const or_model_config* cfg, uint64_t seed, float norm_jitter) {
  or_model* m = (or_model*)calloc(1, sizeof(or_model));
  m->cfg = *cfg;
  const int L = cfg->layers, H = cfg->hidden, hd = cfg->head_dim;
  const size_t qd = (size_t)cfg->heads * hd, kvd = (size_t)cfg->kv_heads * hd;
  m->emb = (float*)malloc(sizeof(float) * (size_t)cfg->vocab * H);
  for (size_t i = 0; i < (size_t)cfg->vocab * H; ++i)
    m->emb[i] = or_half_to_float(or_float_to_half(or_synth_unit(seed, TID_EMB, i) * 0.02f));
#define ALLOC_LAYERS(f) m->f = (float**)calloc((size_t)L, sizeof(float*))
  ALLOC_LAYERS(attn_norm); ALLOC_LAYERS(ffn_norm); ALLOC_LAYERS(wq); ALLOC_LAYERS(wk);
  ALLOC_LAYERS(wv); ALLOC_LAYERS(wo); ALLOC_LAYERS(wg); ALLOC_LAYERS(wu); ALLOC_LAYERS(wd);
  ALLOC_LAYERS(kc); ALLOC_LAYERS(vc);
#undef ALLOC_LAYERS
  for (int l = 0; l < L; ++l) {
    m->attn_norm[l] = synth_norm(seed, TID_LAYER(l, TL_ATTN_NORM), H, norm_jitter);
    m->ffn_norm[l] = synth_norm(seed, TID_LAYER(l, TL_FFN_NORM), H, norm_jitter);
    m->wq[l] = synth_quant_linear(cfg, seed, TID_LAYER(l, TL_Q), H, qd);
    m->wk[l] = synth_quant_linear(cfg, seed, TID_LAYER(l, TL_K), H, kvd);
    m->wv[l] = synth_quant_linear(cfg, seed, TID_LAYER(l, TL_V), H, kvd);
    m->wo[l] = synth_quant_linear(cfg, seed, TID_LAYER(l, TL_O), qd, H);
    m->wg[l] = synth_quant_linear(cfg, seed, TID_LAYER(l, TL_G), H, cfg->inter);
    m->wu[l] = synth_quant_linear(cfg, seed, TID_LAYER(l, TL_U), H, cfg->inter);
    m->wd[l] = synth_quant_linear(cfg, seed, TID_LAYER(l, TL_D), cfg->inter, H);
    m->kc[l] = (float*)calloc((size_t)cfg->max_seq * kvd, sizeof(float));
    m->vc[l] = (float*)calloc((size_t)cfg->max_seq * kvd, sizeof(float));
  }
  m->out_norm = synth_norm(seed, TID_OUT_NORM, H, norm_jitter);
  m->lm_head = synth_quant_linear(cfg, seed, TID_LM_HEAD, H, cfg->vocab);
  m->len = 0;
  return m;
}

void or_model_free(or_model* m) {
  if (!m) return;
  for (int l = 0; l < m->cfg.layers; ++l) {
    free(m->attn_norm[l]); free(m->ffn_norm[l]); free(m->wq[l]); free(m->wk[l]); free(m->wv[l]);
    free(m->wo[l]); free(m->wg[l]); free(m->wu[l]); free(m->wd[l]); free(m->kc[l]); free(m->vc[l]);
  }
  free(m->attn_norm); free(m->ffn_norm); free(m->wq); free(m->wk); free(m->wv); free(m->wo);
  free(m->wg); free(m->wu); free(m->wd); free(m->kc); free(m->vc);
  free(m->emb); free(m->out_norm); free(m->lm_head);
  free(m);
}

void or_model_fill_kv(or_model* m, int n, uint64_t seed) {
  const size_t kvd = (size_t)m->cfg.kv_heads * m->cfg.head_dim;
  for (int l = 0; l < m->cfg.layers; ++l)
    for (size_t i = 0; i < (size_t)n * kvd; ++i) {
      m->kc[l][i] = or_half_to_float(or_float_to_half(or_synth_unit(seed, TID_KV(l, 0), i)));
      m->vc[l][i] = or_half_to_float(or_float_to_half(or_synth_unit(seed, TID_KV(l, 1), i)));
    }
  m->len = n;
}

static int argmax_lowest(const float* v, size_t n) {
  size_t best = 0;
  for (size_t i = 1; i < n; ++i) if (v[i] > v[best]) best = i;
  return (int)best;
}

int or_decode_step(or_model* m, int token, float* logits, int kv_round_f16) {
  const or_model_config* c = &m->cfg;
  const size_t H = (size_t)c->hidden, hd = (size_t)c->head_dim, nh = (size_t)c->heads;
  const size_t nkv = (size_t)c->kv_heads, qd = nh * hd, kvd = nkv * hd, I = (size_t)c->inter;
  const size_t L = (size_t)m->len + 1, grp = nh / nkv;
  float* x = (float*)malloc(sizeof(float) * H);
  float* xn = (float*)malloc(sizeof(float) * H);
  float* q = (float*)malloc(sizeof(float) * qd);
  float* qr = (float*)malloc(sizeof(float) * qd);
  float* kk = (float*)malloc(sizeof(float) * kvd);
  float* kr = (float*)malloc(sizeof(float) * kvd);
  float* vv = (float*)malloc(sizeof(float) * kvd);
  float* att = (float*)malloc(sizeof(float) * qd);
  float* o = (float*)malloc(sizeof(float) * H);
  float* g = (float*)malloc(sizeof(float) * I);
  float* u = (float*)malloc(sizeof(float) * I);
  float* a = (float*)malloc(sizeof(float) * I);
  float* kx = (float*)malloc(sizeof(float) * L * qd);   /* GQA-expanded K/V [L][qd] */
  float* vx = (float*)malloc(sizeof(float) * L * qd);
  const float pos = (float)m->len;

  memcpy(x, m->emb + (size_t)token * H, sizeof(float) * H);
  for (int l = 0; l < c->layers; ++l) {
    or_rms_norm(x, m->attn_norm[l], xn, 1, H, c->eps);
    or_matmul(xn, m->wq[l], q, 1, H, qd);
    or_matmul(xn, m->wk[l], kk, 1, H, kvd);
    or_matmul(xn, m->wv[l], vv, 1, H, kvd);
    or_apply_rope(q, qr, 1, nh, 1, hd, &pos, 0, c->rope_theta);   /* [1,nh,1,hd] */
    or_apply_rope(kk, kr, 1, nkv, 1, hd, &pos, 0, c->rope_theta);
    for (size_t i = 0; i < kvd; ++i) {
      float kv_k = kr[i], kv_v = vv[i];
      if (kv_round_f16) { kv_k = or_half_to_float(or_float_to_half(kv_k)); kv_v = or_half_to_float(or_float_to_half(kv_v)); }
      m->kc[l][(size_t)m->len * kvd + i] = kv_k;
      m->vc[l][(size_t)m->len * kvd + i] = kv_v;
    }
    for (size_t s = 0; s < L; ++s)
      for (size_t h = 0; h < nh; ++h) {
        memcpy(kx + s * qd + h * hd, m->kc[l] + s * kvd + (h / grp) * hd, sizeof(float) * hd);
        memcpy(vx + s * qd + h * hd, m->vc[l] + s * kvd + (h / grp) * hd, sizeof(float) * hd);
      }
    or_multi_head_attention(qr, kx, vx, att, 1, L, qd, nh);
    or_matmul(att, m->wo[l], o, 1, qd, H);
    or_add(x, o, x, H);
    or_rms_norm(x, m->ffn_norm[l], xn, 1, H, c->eps);
    or_matmul(xn, m->wu[l], u, 1, H, I);
    or_matmul(xn, m->wg[l], g, 1, H, I);
    or_silu(g, g, I);
    or_multiply(u, g, a, I);
    or_matmul(a, m->wd[l], o, 1, I, H);
    or_add(x, o, x, H);
  }
  or_rms_norm(x, m->out_norm, xn, 1, H, c->eps);
  or_matmul(xn, m->lm_head, logits, 1, H, (size_t)c->vocab);
  m->len += 1;
  free(x); free(xn); free(q); free(qr); free(kk); free(kr); free(vv); free(att); free(o);
  free(g); free(u); free(a); free(kx); free(vx);
  return argmax_lowest(logits, (size_t)c->vocab);
}

/* ------------------------------------------------ plumbing (config 1) compat */

/* benchmark_inference.cpp:145-225 fill patterns (data, not algorithm). */
static void plumb_fill(size_t V, size_t H, size_t layers, float** up, float** down, float* lm) {
  const size_t I = 4 * H;
  for (size_t l = 0; l < layers; ++l) {
    for (size_t i = 0; i < H * I; ++i) up[l][i] = ((float)(i % 200) / 200.0f - 0.5f) * 0.02f;
    for (size_t i = 0; i < I * H; ++i) down[l][i] = ((float)(i % 200) / 200.0f - 0.5f) * 0.02f;
  }
  for (size_t i = 0; i < H * V; ++i) lm[i] = ((float)(i % 500) / 500.0f - 0.5f) * 0.01f;
}

/* One row through the compat stack: placeholder row, TransformerLayer::forward with
 * no attention weights (compute_attention returns its input, :293-296), no norms,
 * ReLU FFN (:392-395), final matmul with lm_head (:1477). */
static void plumb_row(size_t V, size_t H, size_t layers, float** up, float** down, const float* lm,
                      const float* x0, float* logits) {
  const size_t I = 4 * H;
  float* x = (float*)malloc(sizeof(float) * H);
  float* t = (float*)malloc(sizeof(float) * I);
  float* d = (float*)malloc(sizeof(float) * H);
  memcpy(x, x0, sizeof(float) * H);
  for (size_t l = 0; l < layers; ++l) {
    or_add(x, x, x, H);                 /* residual + attention(identity) */
    or_matmul(x, up[l], t, 1, H, I);
    or_relu(t, t, I);
    or_matmul(t, down[l], d, 1, I, H);
    or_add(x, d, x, H);
  }
  or_matmul(x, lm, logits, 1, H, V);
  free(x); free(t); free(d);
}

size_t or_plumbing_generate(size_t V, size_t H, size_t layers, const int* prompt, size_t n_prompt,
                            size_t max_new, size_t max_seq, int* out, float* last_logits) {
  const size_t I = 4 * H;
  float** up = (float**)malloc(sizeof(float*) * layers);
  float** down = (float**)malloc(sizeof(float*) * layers);
  for (size_t l = 0; l < layers; ++l) { up[l] = (float*)malloc(sizeof(float) * H * I); down[l] = (float*)malloc(sizeof(float) * I * H); }
  float* lm = (float*)malloc(sizeof(float) * H * V);
  plumb_fill(V, H, layers, up, down, lm);
  float* row = (float*)malloc(sizeof(float) * H);
  float* logits = (float*)malloc(sizeof(float) * V);
  size_t n = 0;
  for (size_t i = 0; i < n_prompt; ++i) out[n++] = prompt[i];
  /* forward_pass: placeholder 0.1f*(i%100) over the flat [1,n,H] buffer (:1444-1448);
   * only the last row feeds sample_next_token (:1582-1588). */
  for (size_t h = 0; h < H; ++h) row[h] = 0.1f * (float)(((n_prompt - 1) * H + h) % 100);
  plumb_row(V, H, layers, up, down, lm, row, logits);
  for (size_t step = 0; step < max_new; ++step) {
    /* sample_next_token with top_k = 1, default top_p 0.9 (the draw is irrelevant
     * once only one candidate is finite). */
    const int tok = or_sample_token(logits, V, 1.0f, 1, 0.9f, 0.5f, NULL);
    out[n++] = tok;
    if (last_logits) memcpy(last_logits, logits, sizeof(float) * V);
    if (tok == 2) break;                        /* :760 */
    if (n >= max_seq) break;                     /* :767 */
    for (size_t h = 0; h < H; ++h) row[h] = 0.1f * (float)(h % 100);  /* :1509-1512 */
    plumb_row(V, H, layers, up, down, lm, row, logits);
  }
  for (size_t l = 0; l < layers; ++l) { free(up[l]); free(down[l]); }
  free(up); free(down); free(lm); free(row); free(logits);
  return n;
}

/* forward_pass on the plumbing model (:1429-1491): row r starts from the placeholder
 * 0.1f*(i%100) at flat index i = r*H + h (:1444-1448); all rows' logits are returned, as the
 * reference returns the full [1, n, V] tensor (:1486-1489). */
void or_plumbing_forward_rows(size_t V, size_t H, size_t layers, size_t n, float* logits) {
  const size_t I = 4 * H;
  float** up = (float**)malloc(sizeof(float*) * layers);
  float** down = (float**)malloc(sizeof(float*) * layers);
  for (size_t l = 0; l < layers; ++l) { up[l] = (float*)malloc(sizeof(float) * H * I); down[l] = (float*)malloc(sizeof(float) * I * H); }
  float* lm = (float*)malloc(sizeof(float) * H * V);
  plumb_fill(V, H, layers, up, down, lm);
  float* row = (float*)malloc(sizeof(float) * H);
  for (size_t r = 0; r < n; ++r) {
    for (size_t h = 0; h < H; ++h) row[h] = 0.1f * (float)((r * H + h) % 100);
    plumb_row(V, H, layers, up, down, lm, row, logits + r * V);
  }
  for (size_t l = 0; l < layers; ++l) { free(up[l]); free(down[l]); }
  free(up); free(down); free(lm); free(row);
}
