/*
 * ti_oracle.h -- TEST INFRASTRUCTURE ONLY (never linked into the product).
 *
 * A plain-C restatement of the arithmetic TurboInfer's CPU path performs on the
 * quantized decode hot path.  Every function cites the reference file:line it
 * follows (paths relative to the upstream repository root).  It is used by
 *   - tests/            as the checker for the HIP path,
 *   - __graft_entry__.smoke() as the checker for one small decode step,
 *   - bench.py          only for the "cpu_baseline" leg when oracle/_ref is absent.
 *
 * Pinning: tests/test_oracle_golden.py checks every function here bit-exactly
 * against golden vectors produced by the compiled reference itself
 * (oracle/_ref/libti_ref.so, built from /root/reference sources by oracle/Makefile;
 * fixtures + generator in tests/golden/).
 */
#ifndef TI_ORACLE_H
#define TI_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------- op level (TensorEngine, src/core/tensor_engine.cpp) ---------------- */

/* matmul_3d_2d (:594-640): C[r][j] = sum_k A[r][k]*B[k][j], k ascending, fused (vfmadd231ss). */
void or_matmul(const float* a, const float* b, float* c, size_t rows, size_t K, size_t N);

/* rms_norm (:1452-1508): y = (x / sqrt(mean(x^2)+eps)) * w, per row of n. */
void or_rms_norm(const float* x, const float* w, float* y, size_t rows, size_t n, float eps);

/* apply_rope (:1510-1624), 4-D [B,heads,S,D] (heads=1 gives the 3-D case).
 * pos has S entries (pos_2d=0) or B*S entries (pos_2d=1). */
void or_apply_rope(const float* x, float* y, size_t B, size_t heads, size_t S, size_t D,
                   const float* pos, int pos_2d, float theta);

/* silu (:900-923), relu (:828-869), add (:1626-1678), multiply (:1680-1743). */
void or_silu(const float* x, float* y, size_t n);
void or_relu(const float* x, float* y, size_t n);
void or_add(const float* a, const float* b, float* y, size_t n);
void or_multiply(const float* a, const float* b, float* y, size_t n);

/* softmax (:925-1043) including the AVX2 path with fast_exp_avx2 (:262-302) for n >= 16. */
void or_softmax(const float* x, float* y, size_t rows, size_t n, float temperature);
float or_fast_exp(float x);

/* attention_fast_incremental (:1254-1388): q [B,1,D], k/v [B,S,D] -> out [B,1,D]. */
void or_attention_incremental(const float* q, const float* k, const float* v, float* out,
                              size_t B, size_t S, size_t D);

/* multi_head_attention (:1149-1252) on the decode shape: q [B,1,H], k/v [B,S,H]. */
void or_multi_head_attention(const float* q, const float* k, const float* v, float* out,
                             size_t B, size_t S, size_t H, size_t num_heads);

/* ---------------- quantization (src/optimize/quantization.cpp) ---------------- */

/* calculate_quantization_info (:335-394): per-tensor scale / zero point.
 * bits = 8 or 4; symmetric = 0/1. */
void or_quant_info(const float* x, size_t n, int bits, int symmetric, float* scale, float* zero_point);
/* quantize_to_int8 (:662-674), quantize_to_int4 (:676-693), dequantize_from_* (:695-713).
 * int4 values are held unpacked in int32 like the reference. */
void or_quantize_int8(const float* x, int8_t* q, size_t n, float scale, float zero_point);
void or_quantize_int4(const float* x, int32_t* q, size_t n, float scale, float zero_point);
void or_dequantize_int8(const int8_t* q, float* y, size_t n, float scale, float zero_point);
void or_dequantize_int4(const int32_t* q, float* y, size_t n, float scale, float zero_point);

/* Group-wise symmetric quantizer of the build's packed format: the reference's
 * symmetric formula (scale = absmax/7 or /127, q = clamp(round(x/scale))) applied
 * per group of `group` consecutive k of one output column.  w is the reference's
 * [K][N] row-major linear weight.  Outputs q[N][K] (int8 storage) and the group
 * scales rounded to fp16 (bits of IEEE half) [N][K/group].
 * scale_mode: 0 = per group, 1 = one per-tensor scale for all groups (reference
 * Quantizer semantics), 2 = unit scale (reference convert_dtype raw cast). */
void or_quantize_groups(const float* w, size_t K, size_t N, int bits, int group, int scale_mode,
                        int8_t* q, uint16_t* scale_f16);
/* Dequantize the above back into a [K][N] fp32 matrix: w = float(q) * float(scale_f16). */
void or_dequantize_groups(const int8_t* q, const uint16_t* scale_f16, size_t K, size_t N, int group,
                          float* w);

float or_half_to_float(uint16_t h);
uint16_t or_float_to_half(float f); /* round to nearest even */

/* ---------------- synthetic model ---------------- */

uint64_t or_splitmix64(uint64_t x);
/* U(-sqrt3, sqrt3)/sqrt(K) weights of tensor `tensor_id`, [K][N] row-major. */
void or_synth_linear(uint64_t seed, uint32_t tensor_id, size_t K, size_t N, float* w);
/* Seeded uniform in [-1, 1) with 24 random bits (exact in fp32):
 * h = splitmix64(splitmix64(seed ^ tid*0xD1B54A32D192ED03) + idx), u = (2*(h>>40) - 2^24) / 2^24.
 * Linear weights are u * (sqrtf(3)/sqrtf(K)); embeddings fp16(u*0.02); KV fill fp16(u). */
float or_synth_unit(uint64_t seed, uint32_t tensor_id, uint64_t idx);

/* ---------------- sampling (inference_engine.cpp:1554-1673) ---------------- */

/* sample_next_token with the uniform draw u supplied (the reference draws it from a
 * clock-seeded mt19937).  Greedy = top_k 1.  ti_oracle_sample.cpp. */
/* beam_search_decode (inference_engine.cpp:1912-2069) over a caller-supplied forward pass:
 * fwd(ctx, tokens, n, &logits) returns the distribution's length and points at its logits. */
typedef size_t (*or_forward_fn)(void* ctx, const int32_t* tokens, size_t n, const float** logits);
int or_beam_search(or_forward_fn fwd, void* ctx, const int32_t* prompt, size_t len, size_t max_new, size_t beam_size,
                   float temperature, size_t top_k, float top_p, float length_penalty, int eos, int32_t* out_tokens,
                   int32_t* out_ntok, float* out_log_prob, float* out_score, int32_t* out_finished, float* min_gap);
/* forward_pass (:1429-1491) of the plumbing model: all n rows' logits [n][V] */
void or_plumbing_forward_rows(size_t V, size_t H, size_t layers, size_t n, float* logits);
/* sample_next_token's distribution (temperature, top-k, softmax, top-p renormalised), probs[V] */
void or_sample_probs(const float* logits, size_t V, float temperature, size_t top_k, float top_p, float* probs);
int or_sample_token(const float* logits, size_t V, float temperature, size_t top_k, float top_p,
                    float u, float* logprob_out);

/* ---------------- decode step (reference-composed oracle O2) ---------------- */

typedef struct or_model_config {
  int vocab, hidden, layers, heads, kv_heads, head_dim, inter;
  float rope_theta, eps;
  int bits;        /* 4, 8 or 16 (fp16 weights) */
  int group;       /* 128 */
  int max_seq;
} or_model_config;

/* Fully materialised fp32 model (dequantized weights, [K][N] like the reference). */
typedef struct or_model {
  or_model_config cfg;
  float* emb;            /* [vocab][hidden] (fp16-rounded values) */
  float** attn_norm;     /* [layers][hidden] */
  float** ffn_norm;
  float** wq;            /* [layers] -> [hidden][heads*hd] */
  float** wk;            /* [hidden][kv*hd] */
  float** wv;
  float** wo;            /* [heads*hd][hidden] */
  float** wg;            /* [hidden][inter] */
  float** wu;
  float** wd;            /* [inter][hidden] */
  float* out_norm;
  float* lm_head;        /* [hidden][vocab] */
  /* caller-held K/V history per layer: [max_seq][kv*hd] */
  float** kc;
  float** vc;
  int len;               /* tokens currently in the cache */
} or_model;

/* Build the synthetic model of SURVEY 8(d) (seeded, quantized per group, dequantized
 * back to fp32 so the oracle sees exactly the weights the GPU holds). norm_jitter
 * = 0 gives the unit norm weights of the benchmark model. */
or_model* or_model_synth(const or_model_config* cfg, uint64_t seed, float norm_jitter);
void or_model_free(or_model* m);
/* fill cache positions [0, n) with seeded U(-1,1) rounded to fp16 (synthetic KV) */
void or_model_fill_kv(or_model* m, int n, uint64_t seed);

/* One decode step for one stream at position m->len.  Follows TransformerLayer::forward
 * (inference_engine.cpp:203-233, compute_ffn :376-401) with the per-head KV / RoPE
 * corrections of SURVEY 8(c): rms_norm -> q,k,v matmul -> apply_rope(pos) -> append
 * -> multi_head_attention (GQA by head expansion) -> o matmul -> add -> rms_norm ->
 * silu(gate)*up -> down -> add; final rms_norm + lm_head.  logits [vocab] out.
 * Returns argmax (lowest index on ties). If kv_round_f16, appended K/V are rounded
 * to fp16 (models the device cache; 0 = reference fp32 cache). */
int or_decode_step(or_model* m, int token, float* logits, int kv_round_f16);

/* reference_compat plumbing generate() (inference_engine.cpp:734-802) for the
 * benchmark's synthetic model (benchmark_inference.cpp:145-225): placeholder
 * embeddings, attention bypass (no o_proj), ReLU FFN, greedy (top_k = 1), EOS 2.
 * Returns the number of tokens written (prompt + generated). */
size_t or_plumbing_generate(size_t vocab, size_t hidden, size_t layers, const int* prompt,
                            size_t n_prompt, size_t max_new, size_t max_seq, int* out_tokens,
                            float* last_logits);

#ifdef __cplusplus
}
#endif
#endif
