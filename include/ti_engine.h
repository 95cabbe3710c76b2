/*
 * ti_engine.h -- extern "C" decode engine: the device-resident state behind
 * turboinfer::model::InferenceEngine (its pimpl InferenceEngineImpl,
 * include/turboinfer/model/inference_engine.hpp:214 in the reference) exported as a flat
 * C-ABI so the benchmark, the tests and other-language hosts can drive it.
 *
 * Replaces, per decode step, InferenceEngine::forward_pass_incremental
 * (src/model/inference_engine.cpp:1493-1552) -> TransformerLayer::forward_incremental
 * (:244-279) -> KVCache::update_incremental (:78-160), plus greedy sample_next_token
 * (:1554-1673, top_k = 1) and the generate() loop (:734-802).
 *
 * One engine = one device + one HIP stream + B decode streams (requests) whose fp16 KV
 * caches live in that device's HBM.  Independent engines on different devices are
 * independent replicas (no collectives).
 */
#ifndef TI_ENGINE_H
#define TI_ENGINE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ti_engine ti_engine;

typedef struct ti_engine_config {
  int32_t vocab, hidden, layers, heads, kv_heads, head_dim, inter;
  float rope_theta;        /* ModelMetadata::rope_theta (reference default 10000) */
  float eps;               /* rms_norm eps, reference default 1e-5 (tensor_engine.hpp:185) */
  int32_t bits;            /* weight format: 4 (INT4 g128), 8 (INT8 g128), 16 (fp16) */
  int32_t max_seq;         /* KV slots per stream */
  int32_t max_batch;       /* decode streams held by the engine */
  int32_t compat;          /* 1 = reference_compat: placeholder embeddings, attention
                              bypass, ReLU FFN, fp32 weights (benchmark plumbing model) */
  int32_t device;
  int32_t attn_splits;     /* 0 = auto */
} ti_engine_config;

enum ti_slot {
  TI_W_Q = 0, TI_W_K, TI_W_V, TI_W_O, TI_W_GATE, TI_W_UP, TI_W_DOWN, /* per layer, [K][N] */
  TI_W_LM_HEAD,                                                    /* [hidden][vocab]   */
  TI_V_ATTN_NORM, TI_V_FFN_NORM,                                   /* per layer, [hidden] */
  TI_V_OUT_NORM,                                                   /* [hidden] */
  TI_E_EMBED                                                       /* [vocab][hidden]   */
};

int ti_engine_create(const ti_engine_config* cfg, ti_engine** out);
int ti_engine_destroy(ti_engine* e);
int ti_engine_get_stream(ti_engine* e, void** stream);
int ti_engine_memory(ti_engine* e, size_t* weight_bytes, size_t* kv_bytes);

/* Upload one tensor given in the reference layout (fp32 host memory); linear weights are
 * quantized + packed per the engine's bits (scale_mode: ti_hip.h TI_SCALE_*). */
int ti_engine_set_tensor(ti_engine* e, int slot, int layer, const float* data, int scale_mode);
/* Engines created with bits = 4 or 8 | TI_BITS_G32 (ti_hip.h: group-32 weights, GGUF Q4_0 /
 * Q8_0 blocks): a linear weight given exactly, q int8 [K][N] (reference layout) and fp16 block
 * scales d [K/32][N], weight = d * q -- no re-quantization.  ti_engine_set_tensor on such an
 * engine quantizes fp32 weights per 32-block (absmax / 7 or / 127). */
int ti_engine_set_tensor_q(ti_engine* e, int slot, int layer, const int8_t* q, const uint16_t* d);
/* GGUF Q4_1 blocks (model_loader.cpp:165-182, ggml's format) kept exact on an engine with bits
 * 4 | TI_BITS_G32 | TI_BITS_AFF: q uint8 [K][N_src] (0..15), d and m fp16 [K/32][N_src],
 * weight = d * q + m (ti_wpack_q1_host). */
int ti_engine_set_tensor_q1(ti_engine* e, int slot, int layer, const uint8_t* q, const uint16_t* d, const uint16_t* m);
/* Synthetic model of SURVEY 8(d) generated on the device (bit-identical to the oracle's
 * or_model_synth for the same seed / jitter). */
int ti_engine_synth(ti_engine* e, uint64_t seed, float norm_jitter);
/* Fill KV slots [0, n) of `stream` (all layers) with seeded fp16 U(-1,1) (or_model_fill_kv). */
int ti_engine_fill_kv(ti_engine* e, int stream, int n, uint64_t seed);

/* Greedy generation for n_streams independent requests, entirely on the device: every
 * stream starts at position start_pos[s] (NULL = 0), consumes its prompt one token per
 * step, then feeds back its argmax.  out_tokens [n_streams][max_new] receives the first
 * max_new generated tokens; last_logits (nullable) [n_streams][vocab] the logits of the
 * final step. */
int ti_engine_generate(ti_engine* e, int n_streams, const int32_t* prompts, const int32_t* prompt_lens,
                       int prompt_stride, const int32_t* start_pos, int max_new, int32_t* out_tokens,
                       float* last_logits);

/* Stop token of ti_engine_generate / ti_engine_generate_sampled (-1 = none, the default).  When
 * set, the device loop runs in chunks of 4, 8, 16, 32, then 64 steps, and after each chunk the new
 * tokens are read back; the loop ends once every stream has emitted the token, as the reference's
 * generate() breaks at EOS (inference_engine.cpp:760-764, token id 2).  A stream's tokens end at its
 * first stop token (included); the rest of its max_new entries are -1. */
int ti_engine_set_stop(ti_engine* e, int32_t token);
/* Step-graph replays (decode steps, each covering every stream of its call) and prompt chunks
 * (prefill) this engine has run since it was created. */
int ti_engine_counters(ti_engine* e, uint64_t* decode_steps, uint64_t* prefill_chunks);

/* ti_engine_generate with the reference sampler on the device: after each
 * step's lm_head, ti_sample_step applies sample_next_token (inference_engine.cpp:1554-1673:
 * temperature, top-k, softmax, top-p, the draw) and feeds the token back, so the loop never
 * returns to the host.  draws [n][max_new]: the uniform draw of each stream's t-th new token
 * (the reference takes them from its engine's mt19937, uniform_real_distribution<float>);
 * 1 <= top_k <= vocab (above TI_SAMPLE_MAX_K the engine keeps a sampler workspace).  out_logprobs (nullable) [n][max_new] = log p of
 * each sampled token. */
int ti_engine_generate_sampled(ti_engine* e, int n_streams, const int32_t* prompts, const int32_t* prompt_lens,
                               int prompt_stride, const int32_t* start_pos, int max_new, float temperature,
                               int top_k, float top_p, const float* draws, int32_t* out_tokens, float* out_logprobs);

/* InferenceEngine::generate_beam_search (inference_engine.cpp:830-871, 1912-2069): the
 * reference's beam loop (max-heap on log-probability, expansion by the beam_size most probable
 * tokens after temperature / softmax / top-k / top-p renormalisation (:1798-1910), length-
 * normalised ranking log_prob / len^length_penalty, early stop at beam_size finished beams),
 * with each candidate's next-token distribution from its last position's logits.  Every live
 * beam owns a stream slot holding its KV cache: one batched decode step per expansion round, a
 * fork copies the parent's cache prefix (the reference recomputes each candidate, :1961), so
 * beam_size <= max_batch.  max_new = 0 returns the prompt as one finished beam (no tokens).
 * Results best first: out_tokens [beam_size][max_new] (new tokens, -1 padded), out_log_prob,
 * out_score (normalised), out_finished [beam_size] (nullable), *out_count beams returned. */
int ti_engine_beam_search(ti_engine* e, const int32_t* prompt, int prompt_len, int max_new, int beam_size,
                          float temperature, int top_k, float top_p, float length_penalty, int eos_token,
                          int32_t* out_tokens, float* out_log_prob, float* out_score, int32_t* out_finished,
                          int* out_count);

/* Continuous batching (generate_batch, inference_engine.cpp:804-828, at
 * serving scale): n_req greedy requests through the engine's max_batch stream slots.  The
 * device loop runs in chunks of up to `chunk` steps; between chunks, requests that ended
 * (eos_token, max_new) leave their slot and queued requests take it: the prompt is prefilled
 * into that slot's KV and the request joins the next chunk at its last prompt token, while the
 * other slots continue at their own positions.  prompts: concatenated token ids, request r
 * = prompts[offsets[r] .. offsets[r+1]); out_tokens [n_req][max_new] (-1 padded), out_len
 * [n_req] = tokens produced (the eos token included). */
int ti_engine_serve(ti_engine* e, int n_req, const int32_t* prompts, const int32_t* offsets, int max_new, int eos_token,
                    int chunk, int32_t* out_tokens, int32_t* out_len);

/* Prefill of ti_engine_generate's prompts (reference forward_pass, inference_engine.cpp:
 * 1429-1491): all but the last token of the shortest prompt are processed `rows` tokens at a
 * time as rows of the batched GEMMs and causal attention over the stream's own KV cache,
 * instead of one token per decode step.  Greedy streams whose prompts have one length (at least
 * 2 tokens) run the last token as a prefill row too, and their first token comes from the final
 * rms_norm + lm_head on that row (env TI_PREFILL_LOGITS=0: a decode step instead).
 * Default: TI_GEMM_MAX_ROWS (int4) or 16; 0 = off. */
int ti_engine_set_prefill(ti_engine* e, int rows);

/* Fused hand-offs of single-stream steps: (1) the folded rms_norm (ti_hip.h TI_X_F16_FOLDED):
 * the epilogue that updates the residual also writes fp16(h * next norm weight) and
 * per-workgroup sums of h^2, and the next projection divides its outputs by the rms instead of
 * normalising its input first; (2) the attention's split partials (ti_attn_decode_partials)
 * merged by the O projection (TI_X_ATTN_SPLITS) when the step uses 2..8 splits.  Default on
 * (env TI_FOLD=0 / TI_ATTN_PART=0 turn them off one by one).
 * on = 0/1 sets both, -1 leaves them; *active (nullable) receives whether 1-stream steps fold. */
int ti_engine_set_fold(ti_engine* e, int on, int* active);

/* QKV and attention of single-stream steps in one launch (ti_hip.h ti_qkv_attn_partials; int4 / int8
 * weights, hidden <= 4096, with the fold and split partials on, at head_dim 64 GQA (TinyLlama-1.1B)
 * and head_dim 128 MHA (Llama-2-7B); ti_qkv_attn_supported decides).  Default on (env TI_QKV_ATTN=0
 * turns it off).  Replaces round 4's function of the same name (removed then), with new semantics.
 * on = 0/1 sets it, -1 leaves it; *active (nullable) receives whether 1-stream steps of this engine
 * use it.  Changing it drops the engine's captured step graphs. */
int ti_engine_set_qkv_attn(ti_engine* e, int on, int* active);

/* One decode step: token[s] at position pos[s] for each stream; logits [n][vocab] to host
 * (used for non-greedy sampling and per-step parity). */
int ti_engine_step(ti_engine* e, int n_streams, const int32_t* tokens, const int32_t* pos, float* logits);

/* reference_compat step (compat engines): placeholder row offset, logits [vocab] to host. */
int ti_engine_compat_step(ti_engine* e, int placeholder_offset, float* logits);

/* Benchmark replay: every stream decodes at fixed position kv_len - 1 (reads
 * exactly kv_len cache slots), greedy feedback from start_token.  prepare captures the
 * step graph; run enqueues `steps` replays without synchronising. */
int ti_engine_replay_prepare(ti_engine* e, int n_streams, int kv_len, int start_token);
int ti_engine_replay_run(ti_engine* e, int steps);
int ti_engine_sync(ti_engine* e);
/* tokens decided by the last replay step, [n_streams] */
int ti_engine_last_tokens(ti_engine* e, int n_streams, int32_t* tokens);

/* In-step launch timing (bench.py's roofline; not a reference interface -- the reference
 * times wall clock only, benchmarks/benchmark_inference.cpp:309-384).  The replay step graph
 * (ti_engine_replay_prepare) is captured again with every decode kernel writing, per workgroup,
 * s_memrealtime stamps (100 MHz) of wave 0's entry and of each wave's end into an engine-owned
 * device buffer; `steps` (<= 256) steps are captured back to back into one graph, which is launched
 * once untimed and once read.  Per launch i < min(*n_launch, cap): info[3 i ..] = {kind, tag, workgroups} (workgroups 0:
 * the launch writes no stamps) and t[TI_STAMP_FIELDS i ..] the means over the steps, in us, of
 *   [0] span    first workgroup entry -> last wave end
 *   [1] period  first entry -> the next launch's first entry (the next step's first launch after a
 *               step's last): the launch's share of the step, its boundary included (the very last
 *               launch: its span + the mean boundary)
 *   [2] entry skew  first -> last workgroup entry
 *   [3] wave skew   per workgroup, first -> last wave end, averaged over the workgroups
 *   [4] tail        median workgroup end -> last wave end
 *   [5] gap         last wave end -> the next launch's first entry (the boundary; the last launch: the mean)
 *   [6] workgroups that ran on a CU another workgroup of the launch also ran on (a count)
 *   [7..12] diagnostic builds (TI_STAMP_PHASES): wave 0's phase marks, entry -> mark, workgroup mean
 *   [13]    diagnostic builds: per workgroup, first -> last wave's end of stream, workgroup mean
 * *n_launch receives the launches per step. */
#define TI_STAMP_FIELDS 14
enum { TI_STAMP_KIND_OTHER = 0, TI_STAMP_KIND_GEMV = 1, TI_STAMP_KIND_ATTN = 2, TI_STAMP_KIND_BEGIN = 3,
       TI_STAMP_KIND_ROWS = 4, TI_STAMP_KIND_TILE = 5, TI_STAMP_KIND_RMSNORM = 6, TI_STAMP_KIND_MB = 7 };
enum { TI_STAMP_TAG_BEGIN = 0, TI_STAMP_TAG_QKV = 1, TI_STAMP_TAG_ATTN = 2, TI_STAMP_TAG_O = 3,
       TI_STAMP_TAG_GATE_UP = 4, TI_STAMP_TAG_DOWN = 5, TI_STAMP_TAG_LM_HEAD = 6, TI_STAMP_TAG_OTHER = 7 };
int ti_engine_stamp_steps(ti_engine* e, int steps, int cap, int32_t* info, double* t, int* n_launch);

/* Live per-kernel timing: the step's launches of class `which` (0 qkv, 1 o, 2 gate/up,
 * 3 down, 4 lm_head, 5 attention), `reps` of them cycling through the layers,
 * captured into a graph that is replayed back to back (several ms) between two HIP events on
 * the engine stream.  avg_us = average per launch; bytes = algorithmic HBM bytes per launch. */
int ti_engine_time_kernel(ti_engine* e, int which, int n_streams, int kv_len, int reps, double* avg_us,
                          double* bytes);

/* ------------------------------------------------------------- host helpers */
/* RoPE (cos, sin) pairs for each of npos positions: out [npos][head_dim/2][2], computed on the
 * host with the reference formula (tensor_engine.cpp:1561-1566, 1595-1597) in fp32 libm. */
int ti_rope_table(const float* pos, int npos, int head_dim, float theta, float* out);
/* InferenceEngine::sample_next_token (inference_engine.cpp:1554-1673) with the uniform draw u
 * supplied: temperature, top-k (std::sort ranking, reference tie order), softmax, top-p. */
int ti_sample_token(const float* logits, int vocab, float temperature, int top_k, float top_p, float u,
                    int* token, float* logprob);

#ifdef __cplusplus
}
#endif
#endif /* TI_ENGINE_H */
