/*
 * ti_oracle_deep.c -- TEST INFRASTRUCTURE ONLY (never linked into the product).
 *
 * The oracle's decode step (or_decode_step, ti_oracle.c) at full model depth and width:
 * 32-layer Llama-2-7B / Llama-3-8B and 22-layer TinyLlama with their KV caches filled to
 * max_seq - n.  or_model materialises every weight as dequantized fp32 (27 GB for 7B);
 * or_qmodel keeps the same group-quantized weights as int8 values + their fp16 group scales
 * (held as fp32) and forms each weight value exactly as or_dequantize_groups does,
 * (float)q * (float)half(scale), at the point of use.  Every other operation is the
 * ti_oracle.c function itself, called in the same order with the same arguments, so a step
 * is bit-identical to or_decode_step(kv_round_f16 = 1) on the same model (checked by
 * tests/test_oracle_deep.py on small shapes).  Work is split over OpenMP threads only along
 * independent outputs (matmul columns, attention heads, weight columns): every output's
 * arithmetic chain is the serial one.
 *
 * Reference lines followed are those of ti_oracle.c: TransformerLayer::forward
 * (inference_engine.cpp:203-233), compute_ffn (:376-401), forward_pass_incremental
 * (:1493-1552); matmul_3d_2d (tensor_engine.cpp:594-640).
 */
#include "ti_oracle.h"
#include "ti_oracle_deep.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

enum { TID_EMB = 1, TID_OUT_NORM = 2, TID_LM_HEAD = 3, TID_LAYER0 = 16 };
enum { TL_ATTN_NORM = 0, TL_FFN_NORM, TL_Q, TL_K, TL_V, TL_O, TL_G, TL_U, TL_D };
#define TID_LAYER(l, t) ((uint32_t)(TID_LAYER0 + 16 * (l) + (t)))
#define TID_KV(l, isv) ((uint32_t)(0x100000 + 2 * (l) + (isv)))

typedef struct or_qlinear {
  size_t K, N;
  int group;
  int8_t* qT;   /* [K][N]: q of column n at k (or_quantize_groups' q[n][k], transposed) */
  float* sT;    /* [K/group][N]: half_to_float(scale_f16[n][g]) */
} or_qlinear;

struct or_qmodel {
  or_model_config cfg;
  uint16_t* emb;         /* [vocab][hidden] fp16 bits */
  float** attn_norm;
  float** ffn_norm;
  or_qlinear* wq; or_qlinear* wk; or_qlinear* wv; or_qlinear* wo;
  or_qlinear* wg; or_qlinear* wu; or_qlinear* wd;
  float* out_norm;
  or_qlinear lm_head;
  uint16_t** kc;         /* [layers] -> [max_seq][kv*hd] fp16 bits (the device cache's values) */
  uint16_t** vc;
  int len;
};

/* or_synth_linear + or_quantize_groups(scale_mode 0), one output column at a time:
 * w = u * (sqrtf(3)/sqrtf(K)); per group s = absmax / qmax (fp32), stored half(s);
 * q = clamp(roundf(w / s)) with the fp32 s, exactly as ti_oracle.c computes them. */
static void qlinear_synth(or_qlinear* L, const or_model_config* c, uint64_t seed, uint32_t tid, size_t K,
                          size_t N) {
  L->K = K; L->N = N; L->group = c->group;
  const size_t G = K / (size_t)c->group;
  L->qT = (int8_t*)malloc(K * N);
  L->sT = (float*)malloc(sizeof(float) * G * N);
  const float amp = sqrtf(3.0f) / sqrtf((float)K);
  const float qmax = (c->bits == 4) ? 7.0f : 127.0f;
  const float qlo = (c->bits == 4) ? -7.0f : -128.0f;
  const int group = c->group;
#pragma omp parallel
  {
    float* col = (float*)malloc(sizeof(float) * (size_t)group);
#pragma omp for schedule(static)
    for (size_t n = 0; n < N; ++n)
      for (size_t g = 0; g < G; ++g) {
        float absmax = 0.0f;
        for (int i = 0; i < group; ++i) {
          const size_t k = g * (size_t)group + (size_t)i;
          col[i] = or_synth_unit(seed, tid, k * N + n) * amp;
          const float a = fabsf(col[i]);
          absmax = (absmax < a) ? a : absmax;
        }
        const float s = absmax / qmax;
        L->sT[g * N + n] = or_half_to_float(or_float_to_half(s));
        for (int i = 0; i < group; ++i) {
          float v = roundf(col[i] / s);
          const float t = (v < qmax) ? v : qmax;          /* clampf_ref: std::max(lo, std::min(hi, v)) */
          v = (qlo < t) ? t : qlo;
          L->qT[(g * (size_t)group + (size_t)i) * N + n] = (int8_t)v;
        }
      }
    free(col);
  }
}

static void qlinear_free(or_qlinear* L) {
  free(L->qT); free(L->sT);
}

/* or_matmul(x, W, y, 1, K, N) with W[k][n] = (float)q * scale: acc[n] = fmaf(x[k], W[k][n], acc[n])
 * for k ascending from 0.0f, each column's chain on one thread. */
static void qmatvec(const float* x, const or_qlinear* L, float* y) {
  const size_t K = L->K, N = L->N;
  const size_t CH = 256;
#pragma omp parallel for schedule(static)
  for (size_t n0 = 0; n0 < N; n0 += CH) {
    const size_t n1 = (n0 + CH < N) ? n0 + CH : N;
    float acc[256];
    for (size_t j = n0; j < n1; ++j) acc[j - n0] = 0.0f;
    for (size_t k = 0; k < K; ++k) {
      const float av = x[k];
      const int8_t* q = L->qT + k * N;
      const float* s = L->sT + (k / (size_t)L->group) * N;
      for (size_t j = n0; j < n1; ++j) acc[j - n0] = fmaf(av, (float)q[j] * s[j], acc[j - n0]);
    }
    for (size_t j = n0; j < n1; ++j) y[j] = acc[j - n0];
  }
}

static float* norm_synth(uint64_t seed, uint32_t tid, size_t n, float jitter) {
  float* w = (float*)malloc(sizeof(float) * n);
  for (size_t i = 0; i < n; ++i) w[i] = 1.0f + jitter * or_synth_unit(seed, tid, i);
  return w;
}

or_qmodel* or_qmodel_synth(const or_model_config* cfg, uint64_t seed, float norm_jitter) {
  if (cfg->bits != 4 && cfg->bits != 8) return NULL;
  or_qmodel* m = (or_qmodel*)calloc(1, sizeof(or_qmodel));
  m->cfg = *cfg;
  const int L = cfg->layers;
  const size_t H = (size_t)cfg->hidden, V = (size_t)cfg->vocab, hd = (size_t)cfg->head_dim;
  const size_t qd = (size_t)cfg->heads * hd, kvd = (size_t)cfg->kv_heads * hd, I = (size_t)cfg->inter;
  m->emb = (uint16_t*)malloc(sizeof(uint16_t) * V * H);
#pragma omp parallel for schedule(static)
  for (size_t i = 0; i < V * H; ++i) m->emb[i] = or_float_to_half(or_synth_unit(seed, TID_EMB, i) * 0.02f);
  m->attn_norm = (float**)calloc((size_t)L, sizeof(float*));
  m->ffn_norm = (float**)calloc((size_t)L, sizeof(float*));
  m->wq = (or_qlinear*)calloc((size_t)L, sizeof(or_qlinear));
  m->wk = (or_qlinear*)calloc((size_t)L, sizeof(or_qlinear));
  m->wv = (or_qlinear*)calloc((size_t)L, sizeof(or_qlinear));
  m->wo = (or_qlinear*)calloc((size_t)L, sizeof(or_qlinear));
  m->wg = (or_qlinear*)calloc((size_t)L, sizeof(or_qlinear));
  m->wu = (or_qlinear*)calloc((size_t)L, sizeof(or_qlinear));
  m->wd = (or_qlinear*)calloc((size_t)L, sizeof(or_qlinear));
  m->kc = (uint16_t**)calloc((size_t)L, sizeof(uint16_t*));
  m->vc = (uint16_t**)calloc((size_t)L, sizeof(uint16_t*));
  for (int l = 0; l < L; ++l) {
    m->attn_norm[l] = norm_synth(seed, TID_LAYER(l, TL_ATTN_NORM), H, norm_jitter);
    m->ffn_norm[l] = norm_synth(seed, TID_LAYER(l, TL_FFN_NORM), H, norm_jitter);
    qlinear_synth(&m->wq[l], cfg, seed, TID_LAYER(l, TL_Q), H, qd);
    qlinear_synth(&m->wk[l], cfg, seed, TID_LAYER(l, TL_K), H, kvd);
    qlinear_synth(&m->wv[l], cfg, seed, TID_LAYER(l, TL_V), H, kvd);
    qlinear_synth(&m->wo[l], cfg, seed, TID_LAYER(l, TL_O), qd, H);
    qlinear_synth(&m->wg[l], cfg, seed, TID_LAYER(l, TL_G), H, I);
    qlinear_synth(&m->wu[l], cfg, seed, TID_LAYER(l, TL_U), H, I);
    qlinear_synth(&m->wd[l], cfg, seed, TID_LAYER(l, TL_D), I, H);
    m->kc[l] = (uint16_t*)calloc((size_t)cfg->max_seq * kvd, sizeof(uint16_t));
    m->vc[l] = (uint16_t*)calloc((size_t)cfg->max_seq * kvd, sizeof(uint16_t));
  }
  m->out_norm = norm_synth(seed, TID_OUT_NORM, H, norm_jitter);
  qlinear_synth(&m->lm_head, cfg, seed, TID_LM_HEAD, H, V);
  m->len = 0;
  return m;
}

void or_qmodel_free(or_qmodel* m) {
  if (!m) return;
  for (int l = 0; l < m->cfg.layers; ++l) {
    free(m->attn_norm[l]); free(m->ffn_norm[l]);
    qlinear_free(&m->wq[l]); qlinear_free(&m->wk[l]); qlinear_free(&m->wv[l]); qlinear_free(&m->wo[l]);
    qlinear_free(&m->wg[l]); qlinear_free(&m->wu[l]); qlinear_free(&m->wd[l]);
    free(m->kc[l]); free(m->vc[l]);
  }
  free(m->attn_norm); free(m->ffn_norm); free(m->wq); free(m->wk); free(m->wv); free(m->wo);
  free(m->wg); free(m->wu); free(m->wd); free(m->kc); free(m->vc);
  free(m->emb); free(m->out_norm); qlinear_free(&m->lm_head);
  free(m);
}

/* or_model_fill_kv: positions [0, n) of every layer = fp16(u), u seeded per (layer, K|V, index) */
void or_qmodel_fill_kv(or_qmodel* m, int n, uint64_t seed) {
  const size_t kvd = (size_t)m->cfg.kv_heads * m->cfg.head_dim;
  for (int l = 0; l < m->cfg.layers; ++l) {
    uint16_t* kc = m->kc[l];
    uint16_t* vc = m->vc[l];
#pragma omp parallel for schedule(static)
    for (size_t i = 0; i < (size_t)n * kvd; ++i) {
      kc[i] = or_float_to_half(or_synth_unit(seed, TID_KV(l, 0), i));
      vc[i] = or_float_to_half(or_synth_unit(seed, TID_KV(l, 1), i));
    }
  }
  m->len = n;
}

int or_qmodel_len(const or_qmodel* m) { return m->len; }

/* Rewind the cache to n positions (0 <= n <= len): the next step writes position n.  Lets a fixture
 * generator reuse a long prompt prefix for several candidate continuations. */
int or_qmodel_set_len(or_qmodel* m, int n) {
  if (n < 0 || n > m->len) return -1;
  m->len = n;
  return n;
}

static int argmax_lowest(const float* v, size_t n) {
  size_t best = 0;
  for (size_t i = 1; i < n; ++i) if (v[i] > v[best]) best = i;
  return (int)best;
}

/* or_decode_step(m, token, logits, kv_round_f16 = 1), statement for statement. */
int or_qmodel_step(or_qmodel* m, int token, float* logits) {
  const or_model_config* c = &m->cfg;
  const size_t H = (size_t)c->hidden, hd = (size_t)c->head_dim, nh = (size_t)c->heads;
  const size_t nkv = (size_t)c->kv_heads, qd = nh * hd, kvd = nkv * hd, I = (size_t)c->inter;
  const size_t L = (size_t)m->len + 1, grp = nh / nkv;
  if ((int)L > c->max_seq) return -1;
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
  float* kh = (float*)malloc(sizeof(float) * L * kvd);   /* per kv-head contiguous [nkv][L][hd] */
  float* vh = (float*)malloc(sizeof(float) * L * kvd);
  const float pos = (float)m->len;

  for (size_t i = 0; i < H; ++i) x[i] = or_half_to_float(m->emb[(size_t)token * H + i]);
  for (int l = 0; l < c->layers; ++l) {
    or_rms_norm(x, m->attn_norm[l], xn, 1, H, c->eps);
    qmatvec(xn, &m->wq[l], q);
    qmatvec(xn, &m->wk[l], kk);
    qmatvec(xn, &m->wv[l], vv);
    or_apply_rope(q, qr, 1, nh, 1, hd, &pos, 0, c->rope_theta);
    or_apply_rope(kk, kr, 1, nkv, 1, hd, &pos, 0, c->rope_theta);
    for (size_t i = 0; i < kvd; ++i) {
      m->kc[l][(size_t)m->len * kvd + i] = or_float_to_half(kr[i]);
      m->vc[l][(size_t)m->len * kvd + i] = or_float_to_half(vv[i]);
    }
    /* or_multi_head_attention over the GQA-expanded cache: per q-head h, the rows of kv-head
     * h / grp go to or_attention_incremental(q_h, K_h, V_h, out_h, 1, L, hd). */
    const uint16_t* kc = m->kc[l];
    const uint16_t* vc = m->vc[l];
#pragma omp parallel for schedule(static)
    for (size_t j = 0; j < nkv; ++j)
      for (size_t s = 0; s < L; ++s)
        for (size_t d = 0; d < hd; ++d) {
          kh[(j * L + s) * hd + d] = or_half_to_float(kc[s * kvd + j * hd + d]);
          vh[(j * L + s) * hd + d] = or_half_to_float(vc[s * kvd + j * hd + d]);
        }
#pragma omp parallel for schedule(dynamic, 1)
    for (size_t h = 0; h < nh; ++h)
      or_attention_incremental(qr + h * hd, kh + (h / grp) * L * hd, vh + (h / grp) * L * hd, att + h * hd, 1, L,
                               hd);
    qmatvec(att, &m->wo[l], o);
    or_add(x, o, x, H);
    or_rms_norm(x, m->ffn_norm[l], xn, 1, H, c->eps);
    qmatvec(xn, &m->wu[l], u);
    qmatvec(xn, &m->wg[l], g);
    or_silu(g, g, I);
    or_multiply(u, g, a, I);
    qmatvec(a, &m->wd[l], o);
    or_add(x, o, x, H);
  }
  or_rms_norm(x, m->out_norm, xn, 1, H, c->eps);
  qmatvec(xn, &m->lm_head, logits);
  m->len += 1;
  free(x); free(xn); free(q); free(qr); free(kk); free(kr); free(vv); free(att); free(o);
  free(g); free(u); free(a); free(kh); free(vh);
  return argmax_lowest(logits, (size_t)c->vocab);
}
