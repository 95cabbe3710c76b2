/*
 * ti_hip.h -- the flat extern "C" boundary between the turboinfer C++20 host library
 * and the hand-written gfx950 (MI355X / CDNA4) HIP kernels of the decode hot path.
 *
 * Plain pointers and sizes only (no C++ or torch types).  Every function returns
 * TI_OK (0) or a TI_ERR_* code; ti_last_error() returns the thread's last message.
 * Pointers documented "device" must be device memory (ti_malloc or hipMalloc).
 * Streams are hipStream_t values passed as void* (NULL = default stream).
 *
 * Which reference interface each entry replaces (paths relative to the reference
 * repository, juliuspleunes4/TurboInfer @ 2025-09-05):
 *   ti_gemm_wq_a16        TensorEngine::matmul -> matmul_3d_2d      src/core/tensor_engine.cpp:490-528, 594-640
 *                         (+ the convert_dtype "dequant" of int weights :2218-2284, scale restored)
 *                         + fused rms_norm :1452-1508 prologue, add :1626-1678 / silu :900-923 /
 *                         multiply :1680-1743 / apply_rope :1510-1624 epilogues, KV append
 *                         (KVCache::update_incremental, src/model/inference_engine.cpp:78-160)
 *   ti_attn_decode        TensorEngine::multi_head_attention :1149-1252 -> attention_fast_incremental :1254-1388
 *   ti_wpack_host         Quantizer::quantize_tensor / quantize_to_int{4,8}
 *                         src/optimize/quantization.cpp:36-64, 662-693 (per group of 128, packed)
 *   ti_matmul_f32         TensorEngine::matmul (fp32, bit-exact k-ascending fma chain)
 *   ti_rms_norm_f32       TensorEngine::rms_norm  :1452-1508 (bit-exact reduction order)
 *   ti_rope_f32           TensorEngine::apply_rope :1510-1624 (host cos/sin table, same fma pattern)
 *   ti_silu_f32 / ti_add_f32 / ti_mul_f32 / ti_relu_f32   :900-923, :1626-1743, :828-869
 *   ti_softmax_f32        TensorEngine::softmax :925-1043 (same fast_exp_avx2 polynomial :262-302)
 *   ti_attention_f32      TensorEngine::multi_head_attention / attention_fast_incremental (fp32 op level)
 *   ti_argmax_f32         greedy InferenceEngine::sample_next_token (top_k = 1) :1554-1673
 */
#ifndef TI_HIP_H
#define TI_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* ti_stream_t;

enum ti_status {
  TI_OK = 0,
  TI_ERR_ARG = 1,          /* bad shape / argument (host-side check, nothing launched) */
  TI_ERR_HIP = 2,          /* HIP runtime error */
  TI_ERR_UNSUPPORTED = 3,  /* configuration not supported by the kernels */
  TI_ERR_NOMEM = 4,
  TI_ERR_NODEV = 5         /* no gfx950 device visible */
};

const char* ti_last_error(void);

/* ------------------------------------------------------------ device plumbing */
int ti_device_count(int* count);
int ti_init(int device);                          /* select device, check it is gfx950 */
int ti_device_name(int device, char* buf, int len);
int ti_malloc(void** ptr, size_t bytes);
int ti_free(void* ptr);
int ti_memcpy_h2d(void* dst, const void* src, size_t bytes, ti_stream_t s);
int ti_memcpy_d2h(void* dst, const void* src, size_t bytes, ti_stream_t s);
int ti_memcpy_d2d(void* dst, const void* src, size_t bytes, ti_stream_t s);
int ti_memset(void* ptr, int value, size_t bytes, ti_stream_t s);
int ti_stream_create(ti_stream_t* s);
int ti_stream_destroy(ti_stream_t s);
int ti_stream_sync(ti_stream_t s);
int ti_device_sync(void);
int ti_event_create(void** ev);
int ti_event_destroy(void* ev);
int ti_event_record(void* ev, ti_stream_t s);
int ti_event_elapsed_ms(void* start, void* stop, float* ms); /* synchronises on stop */

/* -------------------------------------------- packed quantized linear weights
 * A linear layer y = x @ W with the reference's W[K][N] row-major layout
 * (inference_engine.cpp:299-301) is stored as tiles of 16 output rows x 128 k:
 *   bits 4 : 1 KiB per tile,  nibble q+8 (q in [-7,7], reference symmetric int4 range)
 *   bits 8 : 2 KiB per tile,  int8 q in [-128,127]
 *   bits 16: 4 KiB per tile,  fp16 weights (no scale)
 * tiles ordered [N/16][K/128]; inside a tile, 1 KiB chunk c holds for lane l (0..63)
 * at byte 1024*c + 16*l the k-run of output row (l & 15) starting at
 * k = 32*(l >> 4) + c*(32/chunks) -- one coalesced dwordx4 per lane per chunk.
 * Group scales (bits 4/8): fp16, [N/16][K/128][16].  bits may carry TI_BITS_G32 (below).
 * K must be a multiple of 128 and N a multiple of 16. */
enum ti_scale_mode { TI_SCALE_GROUP = 0, TI_SCALE_TENSOR = 1, TI_SCALE_UNIT = 2 };
enum ti_row_map { TI_ROWS_CONCAT = 0, TI_ROWS_INTERLEAVE8 = 1 };

size_t ti_wpack_tile_bytes(int bits, int K, int N);
size_t ti_wpack_scale_bytes(int bits, int K, int N);

/* Quantize + pack the fp32 [K][N_src] matrix w (host memory) into the host buffers of
 * a fused weight with N_total output rows.  Source column c lands on output row
 *   TI_ROWS_CONCAT      : row_offset + c
 *   TI_ROWS_INTERLEAVE8 : 16*(c/8) + (c%8) + row_offset   (row_offset 0 = gate, 8 = up)
 * scale_mode: per group of 128 (absmax/7 or /127, reference quantize_to_int* formula per
 * group), one per-tensor scale (reference Quantizer), or unit (reference raw cast).
 * bits | TI_BITS_G32: per 32-block absmax scales.  bits 4 | TI_BITS_G32 | TI_BITS_AFF: ggml's
 * Q4_1 rounding per 32-block (d = (max - min) / 15, m = min; scale_mode ignored). */
int ti_wpack_host(const float* w, int K, int N_src, int N_total, int bits, int scale_mode,
                  int row_map, int row_offset, void* tiles, uint16_t* scales);

/* Group-32 weights (GGUF Q4_0 / Q8_0 blocks, model_loader.cpp:165-182 / ggml's formats): bits
 * 4 or 8 with TI_BITS_G32 set.  Tiles as above except the k order inside a tile: lane l's
 * 16 bytes (int4; int8: 8 bytes per MFMA step in chunk s4 / 2) hold, for MFMA step s4, the
 * 8 weights k = 32*s4 + 8*(l >> 4) + e, so every 32-weight block is one MFMA's reduction.
 * Scales fp16 [N/16][K/128][4][16] (one per output row and 32-k block).  Runs on the fused
 * kernel (more rows than its LDS image holds: in pieces) and, int4 with fp16 rows from 65 rows
 * on, on the tile GEMM; no packed rows (ti_gemm_max_rows). */
#define TI_BITS_G32 32
/* Pack exact integer weights: q int8 [K][N_src] (int4: -8..7, int8: -127..127) with fp16 block
 * scales d [K/32][N_src]: weight(k, c) = d[k/32][c] * q[k][c] exactly, as ggml dequantizes a
 * Q4_0 / Q8_0 block (bits = 4 or 8, TI_BITS_G32 implied; rows mapped as in ti_wpack_host). */
int ti_wpack_q_host(const int8_t* q, const uint16_t* d, int K, int N_src, int N_total, int bits, int row_map,
                    int row_offset, void* tiles, uint16_t* scales);
/* Affine group-32 int4 (GGUF Q4_1 blocks, ggml's format: weight = d * q + m, q in 0..15, d and m
 * fp16 per 32-weight block): bits = 4 | TI_BITS_G32 | TI_BITS_AFF.  Tiles hold q - 8 like Q4_0
 * blocks; the scale buffer holds d [N/16][K/128][4][16] followed by m in the same layout
 * (ti_wpack_scale_bytes counts both).  The kernels add (8 d + m) * (the block's sum of x) per
 * block.  Fused kernel only (more rows run in pieces); no tile GEMM, no packed rows. */
#define TI_BITS_AFF 64
/* q uint8 [K][N_src] (0..15), d and m fp16 [K/32][N_src]: weight(k, c) = d * q + m. */
int ti_wpack_q1_host(const uint8_t* q, const uint16_t* d, const uint16_t* m, int K, int N_src, int N_total, int row_map,
                     int row_offset, void* tiles, uint16_t* scales);

/* The synthetic model of SURVEY 8(d) generated straight into device tiles:
 * element (k, c) of tensor `tensor_id` = u(seed, tensor_id, k*N_src + c) * amp,
 * amp = sqrtf(3)/sqrtf(K) (u: or_synth_unit), quantized per group like ti_wpack_host. */
int ti_wsynth_device(uint64_t seed, uint32_t tensor_id, int K, int N_src, int N_total, int bits,
                     int row_map, int row_offset, void* tiles, uint16_t* scales, ti_stream_t s);
/* dst[i] = fp16(u(seed, tensor_id, i) * mul) (+ add, fp32 variant) for i < n. */
int ti_fill_uniform_f16(uint64_t seed, uint32_t tensor_id, uint64_t n, float mul, uint16_t* dst,
                        ti_stream_t s);
int ti_fill_uniform_f32(uint64_t seed, uint32_t tensor_id, uint64_t n, float mul, float add,
                        float* dst, ti_stream_t s);
/* Synthetic KV for one stream of one layer: slots [0, n) of dst ([kv_heads][max_seq][head_dim]
 * fp16) from the oracle's [pos][kv_heads*head_dim] uniform stream (or_model_fill_kv). */
/* Beam search's fork (no reference counterpart: the reference recomputes every candidate,
 * inference_engine.cpp:1961): copy a cache prefix between stream slots.  tab: device array of
 * n_tab fp16 cache base pointers (layer K / V); per cache, `rows` rows of row_elems elements
 * (pitch row_pitch) from element offset src_off to dst_off.  row_elems, row_pitch and the
 * offsets are multiples of 8. */
int ti_kv_copy_slots(uint16_t* const* tab, int n_tab, int64_t src_off, int64_t dst_off, int rows, int64_t row_pitch,
                     int64_t row_elems, ti_stream_t s);
int ti_fill_kv_uniform(uint64_t seed, uint32_t tensor_id, int n, int kv_heads, int head_dim, int max_seq,
                       uint16_t* dst, ti_stream_t s);

/* ---------------------------------------------------- fused decode GEMM/GEMV
 * y[m][n] = sum_k xa[m][k] * W[k][n], m < M <= TI_GEMM_MAX_ROWS (see ti_gemm_max_rows), with
 *   xa = fp16(x)                               (x_kind TI_X_F16 / TI_X_F32), or
 *   xa = fp16((x / sqrt(mean(x^2)+eps)) * nw)  (x_kind TI_X_F32_RMSNORM; fused rms_norm)
 * fp16 x fp16 products on MFMA v_mfma_f32_16x16x32_f16, fp32 accumulation, group scale
 * applied in fp32 per 128-k group.
 * TI_X_F16_FOLDED (M == 1, norm_w NULL) is the same rms_norm with the normalisation moved
 * behind the GEMM, y = (W . x) / sqrt(sum(epi->ss_in[0 .. n_ss)) / K + eps): x holds
 * fp16(h * nw), written together with the partial sums of h^2 by the epilogue that produced h
 * (TI_EPI_RESID_F32 with fold_x, or ti_step_begin with fold_x), so the launch stages 2-byte
 * rows with no block-wide reduction in front of its first MFMA.
 * TI_X_ATTN_SPLITS (M == 1, K = heads * head_dim <= 4096, norm_w NULL): x is the attention
 * output still split, x = part_o of ti_attn_decode_partials with epi->ss_in = part_ml,
 * epi->n_ss = splits (<= TI_ATTN_MAX_PART_SPLITS) and epi->head_dim; the launch merges the
 * splits (max-rescaled, sum-weighted, as the attention's own merge) while staging x (also the
 * output of ti_qkv_attn_partials).
 * Epilogue (all outputs of one call): */
enum ti_x_kind { TI_X_F16 = 0, TI_X_F32 = 1, TI_X_F32_RMSNORM = 2, TI_X_F16_FOLDED = 3, TI_X_ATTN_SPLITS = 4,
                 TI_X_F16_PACKED = 5 };
/* TI_X_F16_PACKED: fp16 rows in the batched-rows kernel's fragment order, so every load of its
 * MFMA operands is one contiguous KiB per wave (bits 4).  Element (m, k) of an M x K operand
 * (K % 128 == 0) sits at TI_PACKED_INDEX(m, k, K / 128); the buffer holds ceil(M / 16) * 16
 * rows (16-row blocks of 16 * K elements, block b at b * 16 * K).  Producers: ti_rmsnorm_f16_packed,
 * ti_attn_decode_packed, and the batched epilogues TI_EPI_STORE_F16 / TI_EPI_SILU_MUL_F16 with
 * out_packed set. */
#define TI_PACKED_INDEX(m, k, kt)                                                                        \
  ((((((size_t)((m) >> 4) * (size_t)(kt) + (size_t)((k) >> 7)) * 4 + (size_t)(((k) >> 3) & 3)) * 64 +    \
     (size_t)((((k) >> 5) & 3) * 16 + ((m) & 15))) * 8 + (size_t)((k) & 7)))
enum ti_epilogue_kind {
  TI_EPI_STORE_F32 = 0,      /* out_f32[m*ldo + n] = y                                  */
  TI_EPI_STORE_F16 = 1,      /* out_f16[m*ldo + n] = fp16(y)                             */
  TI_EPI_RESID_F32 = 2,      /* out_f32[m*ldo + n] += y          (residual add, in place) */
  TI_EPI_SILU_MUL_F16 = 3,   /* rows interleaved by 8 (gate,up): out_f16[m*ldo + j] =
                                fp16(up_j * silu(gate_j)), N/2 outputs                   */
  TI_EPI_QKV_ROPE_KV = 4,    /* rows [q | k | v]: RoPE(pos[m]) on q and k, q -> out_f32,
                                k, v -> fp16 KV cache slot pos[m]                        */
  TI_EPI_LOGITS_ARGMAX = 5   /* out_f32 logits + greedy argmax keys (see below)            */
};

/* Greedy argmax keys: key = (order-preserving bits of the logit) << 32 | (0xFFFFFFFF - n), so
 * the max key is the largest logit at the lowest index.  Each workgroup folds its tiles into
 * one key per row and atomicMax-es it into one of TI_ARGMAX_SLOTS slots (no single hot word);
 * row m's key is the max over argmax[m*TI_ARGMAX_SLOTS + 0 .. SLOTS-1], its token
 * 0xFFFFFFFF - (key & 0xFFFFFFFF). */
#define TI_ARGMAX_SLOTS 32

typedef struct ti_epilogue {
  int32_t kind;
  int32_t ldo;                       /* output leading dimension (elements) */
  void* out;                         /* device output base */
  /* TI_EPI_QKV_ROPE_KV */
  int32_t q_dim, kv_dim, head_dim, max_seq;
  const int32_t* pos;                /* device [M] token positions */
  const float* rope_cs;              /* device [max_seq][head_dim/2] (cos, sin) pairs */
  uint16_t* k_cache;                 /* device fp16, this layer: [stream][kv_head][max_seq][head_dim] */
  uint16_t* v_cache;
  int64_t kv_stream_stride;          /* elements between streams; 0 = rows of one stream (prefill) */
  /* TI_EPI_LOGITS_ARGMAX */
  unsigned long long* argmax;        /* device [M][TI_ARGMAX_SLOTS] keys, zeroed before the call */
  int32_t* step_ctr;                 /* device counter += advance by one thread (nullable) */
  int32_t advance;
  /* TI_X_F16_FOLDED input: n_ss partial sums of squares of the row at ss_in.
   * Batched fold (17..64 int4 rows, TI_X_F16 / TI_X_F16_PACKED x holding fp16(h * nw), ss_in
   * non-NULL): row m is normalised behind the GEMM, y[m] = (W . x[m]) / sqrt(sum over
   * b < n_ss of ss_in[b * TI_FOLD_SS_ROWS + m] / K + eps) -- the batched-rows / tile kernels */
  int32_t n_ss;
  const float* ss_in;
  /* TI_EPI_RESID_F32, M == 1, fold_x non-NULL: besides h, write fold_x[n] = fp16(h[n] * fold_w[n])
   * and fold_ss[b] = sum of h[n]^2 over the outputs of workgroup b (b < ti_gemm_grid(...)): the
   * next launch's TI_X_F16_FOLDED input.
   * M = 17..64 on the batched-rows kernel (TI_X_F16_PACKED x): fold_x[m][n] = fp16(h[m][n] *
   * fold_w[n]) (TI_X_F16_PACKED order when fold_packed, else rows of ldo) and
   * fold_ss[b * TI_FOLD_SS_ROWS + m] = sum of h[m][n]^2 over the columns of column group b
   * (b < ti_gemm_fold_partials(...)): the next batched call's folded input */
  const float* fold_w;
  uint16_t* fold_x;
  float* fold_ss;
  /* TI_EPI_STORE_F16 / TI_EPI_SILU_MUL_F16 of the batched-rows kernels (M > 16 or packed x):
   * write the fp16 output in TI_X_F16_PACKED order (K = ldo, ldo % 128 == 0) */
  int32_t out_packed;
  /* Split-K workspace of the tile GEMM (int4 fp16 rows from TI_GEMM_TILE_ROWS on): device memory
   * of splitk_bytes bytes whose first TI_SPLITK_TICKET_BYTES the owner zeroes once (every launch
   * leaves them zeroed); the fp32 partial blocks follow.  With it, narrow outputs split K over
   * workgroups to fill the chip (ti_gemm_tile_plan); NULL = no split.  One launch at a time per
   * workspace (stream order). */
  void* splitk_ws;
  int64_t splitk_bytes;
  int32_t fold_packed;
} ti_epilogue;
#define TI_FOLD_SS_ROWS 64
#define TI_SPLITK_TICKET_BYTES (256 * 1024)
/* sizeof(ti_epilogue): a binding checks its mirror of the struct against it. */
int ti_epilogue_bytes(void);

int ti_gemm_wq_a16(const void* tiles, const uint16_t* scales, int bits, const void* x, int x_kind,
                   int ldx, const float* norm_w, float eps, int M, int N, int K,
                   const ti_epilogue* epi, ti_stream_t s);
/* LDS bytes one workgroup of the fused kernel needs for an M x N x K call (<= 160 KiB). */
int ti_gemm_lds_bytes(int M, int N, int K);
/* Rows (M) per ti_gemm_wq_a16 call the library prefers for this shape and activation kind.
 * Two kernels: the fused one (rms_norm prologue, any bits) takes up to 16 rows while its LDS
 * image fits; for bits 4 with TI_X_F16 rows the batched-rows kernel takes up to
 * TI_GEMM_MAX_ROWS rows at any K (batched decode, generate_batch inference_engine.cpp:804-828)
 * and is used above 2 rows (a fixed crossover).  An int4 caller with more rows
 * than this returns for TI_X_F32_RMSNORM should normalise them with ti_rmsnorm_f16 and pass
 * TI_X_F16 rows.  0 = shape unsupported. */
#define TI_GEMM_MAX_ROWS 1024
int ti_gemm_max_rows(int bits, int x_kind, int N, int K);
/* 1 when M rows of an int4 GEMM go to the batched-rows kernel (17 .. 64 rows): its fp16
 * operands are best given as TI_X_F16_PACKED.  From 65 rows (TI_GEMM_TILE_ROWS, env, <= 65) on
 * the LDS-tiled kernel takes TI_X_F16 rows. */
int ti_gemm_packed_rows(int bits, int M);
/* The same for one M x N x K call: 0 also where 17..64 int4 rows of a wide output take the tile
 * GEMM (rows x N >= TI_GEMM_TILE_WIDE_MN, env, default 850000), which needs TI_X_F16 rows. */
int ti_gemm_packed_rows_for(int bits, int M, int N, int K);
/* The tile GEMM's plan for an int4 (bits 4 or 4 | TI_BITS_G32) M x N x K call with a split-K
 * workspace of ws_bytes (0 = none): row-waves, weight tiles per wave and k-slices (1 = no split;
 * K is split only where one slice per column block would leave most CUs idle, TI_GEMM_SPLITK=0
 * never).  TI_ERR_UNSUPPORTED when the call would not take the tile kernel. */
int ti_gemm_tile_plan(int bits, int M, int N, int K, int64_t ws_bytes, int* wmr, int* tpw, int* n_ks);
/* y[m][0:K] = fp16(rms_norm(x[m][0:K]) * w), tensor_engine.cpp:1452-1508 (the batched path's
 * activation prep; the same arithmetic as the fused TI_X_F32_RMSNORM prologue). */
int ti_rmsnorm_f16(const float* x, int ldx, const float* w, float eps, uint16_t* y, int ldy, int M, int K,
                   ti_stream_t s);
/* ti_rmsnorm_f16 writing y in TI_X_F16_PACKED order (K % 128 == 0). */
int ti_rmsnorm_f16_packed(const float* x, int ldx, const float* w, float eps, uint16_t* y, int M, int K,
                          ti_stream_t s);
/* Workgroups of the fused kernel for an M x N x K call: the fold_ss partials a
 * TI_EPI_RESID_F32 fold epilogue writes (0 = shape not taken by the fused kernel). */
int ti_gemm_grid(int M, int N, int K);
/* Column groups of the batched-rows kernel for an int4 TI_X_F16_PACKED M x N x K call (17..64
 * rows): the fold_ss partials per row its TI_EPI_RESID_F32 fold epilogue writes (0 = the call
 * does not take the batched-rows kernel). */
int ti_gemm_fold_partials(int bits, int M, int N, int K);
/* One-time kernel attribute setup; call before capturing ti_gemm_wq_a16 into a graph. */
int ti_gemm_prepare(void);

/* ------------------------------------------------------------- decode attention
 * Single-query attention of M streams against their fp16 KV caches, GQA aware:
 * q fp32 [M][heads*head_dim]; stream m attends to cache slots [0, pos[m]] of layer cache
 * k_cache/v_cache ([stream][kv_head][max_seq][head_dim], stream stride kv_stream_stride; 0 = the
 * M rows are tokens of one stream at their own positions: causal prefill attention).
 * Split-K over the sequence (flash-decoding): `splits` partial (max, sum, o) per
 * (stream, head) in workspace, merged in the same launch by the last-arriving split, which
 * writes fp16 out [M][heads*head_dim].
 * head_dim 64 or 128; heads/kv_heads in {1, 2, 4, 8}; M <= TI_ATTN_MAX_M.
 * The workspace (ti_attn_workspace_bytes, for the largest M and splits the caller will use)
 * must be zeroed once before the first call; calls keep its ticket region re-armed.  splits
 * only shapes the work (results agree to rounding) and is capped by what one workgroup can
 * merge in LDS. */
#define TI_ATTN_MAX_M 1024
size_t ti_attn_workspace_bytes(int M, int heads, int head_dim, int splits);
int ti_attn_decode(const float* q, const uint16_t* k_cache, const uint16_t* v_cache,
                   int64_t kv_stream_stride, int max_seq, const int32_t* pos, int M, int heads,
                   int kv_heads, int head_dim, int splits, float* workspace, uint16_t* out,
                   ti_stream_t s);
/* ti_attn_decode writing out in TI_X_F16_PACKED order (K = heads * head_dim, a multiple of 128):
 * the batched O projection's operand. */
int ti_attn_decode_packed(const float* q, const uint16_t* k_cache, const uint16_t* v_cache,
                          int64_t kv_stream_stride, int max_seq, const int32_t* pos, int M, int heads,
                          int kv_heads, int head_dim, int splits, float* workspace, uint16_t* out,
                          ti_stream_t s);
/* The same attention with the split merge left to the consumer: split s of (stream m, head h)
 * writes its normalised row part_o[((m*heads + h)*splits + s)*head_dim + d] (fp16) and
 * (max, sum) at part_ml[2*((m*heads + h)*splits + s)]; an empty split writes (-inf, 0) and a
 * zero row.  The O projection merges them while staging its input (TI_X_ATTN_SPLITS), so the
 * attention launch ends without the arrival-ticket hand-off.  2 <= splits <=
 * TI_ATTN_MAX_PART_SPLITS; no workspace. */
#ifndef TI_ATTN_MAX_PART_SPLITS
#define TI_ATTN_MAX_PART_SPLITS 8
#endif
int ti_attn_decode_partials(const float* q, const uint16_t* k_cache, const uint16_t* v_cache,
                            int64_t kv_stream_stride, int max_seq, const int32_t* pos, int M, int heads,
                            int kv_heads, int head_dim, int splits, uint16_t* part_o, float* part_ml,
                            ti_stream_t s);
/* One decode stream (bits 4 or 8; head_dim 64 GQA, or head_dim 128 with heads == kv_heads; 1024 <= K <=
 * 4096; ti_qkv_attn_supported): the QKV projection of the folded input (TI_X_F16_FOLDED: fx,
 * ss_in[0 .. n_ss)) with the TI_EPI_QKV_ROPE_KV epilogue's arithmetic -- the new K / V row into
 * k_cache / v_cache ([kv_heads][max_seq][head_dim], slot pos[0]) -- and ti_attn_decode_partials over
 * the keys up to pos[0], in one launch of heads x splits workgroups (inference_engine.cpp:203-279 and
 * 291-368 -> tensor_engine.cpp:490-640, 1510-1624, 1254-1388); the last split also attends the step's own
 * key (from the k / v rows the launch computes).  The O projection merges the splits with x kind
 * TI_X_ATTN_SPLITS (x = part_o, ss_in = part_ml, n_ss = splits): part_o holds
 * ti_qkv_attn_part_o_elems and part_ml ti_qkv_attn_part_ml_elems elements.  tiles / scales: the fused
 * q | k | v weight as ti_gemm_wq_a16 takes it (N = (heads + 2 kv_heads) * head_dim).  The S workgroups
 * of a head split its q rows (tile s % (head_dim / 16), k-part s / (head_dim / 16)) and exchange them
 * through xchg (ti_qkv_attn_xchg_bytes, zeroed once by the owner, then kept: it holds a generation per
 * workgroup; one launch at a time per buffer).  splits: a multiple of head_dim / 16 whose k-parts are
 * whole multiples of 8 k-tiles. */
int ti_qkv_attn_partials(const void* tiles, const uint16_t* scales, int bits, const uint16_t* fx,
                         const float* ss_in, int n_ss, float eps, const float* rope_cs, const int32_t* pos,
                         uint16_t* k_cache, uint16_t* v_cache, int max_seq, int K, int heads, int kv_heads,
                         int head_dim, int splits, uint16_t* part_o, float* part_ml, void* xchg, ti_stream_t s);
size_t ti_qkv_attn_part_o_elems(int heads, int head_dim, int splits);
size_t ti_qkv_attn_part_ml_elems(int heads, int head_dim, int splits);
size_t ti_qkv_attn_xchg_bytes(int heads, int splits);
/* Byte offset in xchg of the launch's error word (uint32): nonzero once a wait on a sibling's granule
 * expired (bounded waits: the launch always completes, that head's q or new key is then wrong).  The
 * owner reads it after the stream's work and, when set, zeroes the whole buffer to resynchronise the
 * workgroups' generations (the engine does: ti_engine_generate / ti_engine_step return TI_ERR_HIP). */
size_t ti_qkv_attn_error_offset(int heads, int splits);
/* 1 when ti_qkv_attn_partials has a kernel for this shape (0: it would return TI_ERR_UNSUPPORTED / ARG). */
int ti_qkv_attn_supported(int bits, int K, int heads, int kv_heads, int head_dim, int splits);
/* Prefill attention (forward_pass over a prompt chunk, inference_engine.cpp:1429-1491 ->
 * multi_head_attention, tensor_engine.cpp:1149-1252): the M rows are tokens of ONE stream whose
 * cache k_cache / v_cache [kv_heads][max_seq][head_dim] fp16 already holds their K / V; row m
 * attends to keys [0, pos[m]] (0 <= pos[m] < max_seq), q [M][heads*head_dim] fp32 ->
 * out [M][heads*head_dim] fp16.  One wave per 16 (row, q-head) columns streams each key once for
 * them on fp16 MFMA with the fp32 operands split into fp16 hi + lo parts (fp32-accurate products;
 * ti_attn_decode reads the prefix once per row).  head_dim 64 or 128;
 * heads % kv_heads == 0.  Replaces ti_attn_decode(kv_stream_stride = 0) for row-major chunks.
 * At head_dim 128, chunks whose grid fills the chip run the shared-K/V kernel: a workgroup per
 * (kv-head, 4 query blocks) copies each K / V block once into LDS for all its waves. */
int ti_attn_prefill(const float* q, const uint16_t* k_cache, const uint16_t* v_cache, int max_seq,
                    const int32_t* pos, int M, int heads, int kv_heads, int head_dim, uint16_t* out,
                    ti_stream_t s);
/* Kernel choice of later ti_attn_prefill calls in this process (parity tests and A/Bs; not a
 * reference interface): 0 automatic (the default, TI_PF_WG applies), 1 the per-wave kernel,
 * 2 the shared-K/V kernel with 4-wave workgroups, 3 with 8-wave workgroups (key-split halves).
 * Modes 2 and 3 apply at head_dim 128 at any grid size; other head_dims take the per-wave kernel.
 * Returns the previous mode, or -1 for a mode outside 0..3 (nothing changed). */
int ti_attn_prefill_set_kernel(int mode);

/* The kernel ti_gemm_wq_a16 launches for plain (not group-32) weights of this shape, e.g.
 * "gemv_wq_kernel<4,4>", "gemm_rows_kernel", "gemm_tile_kernel" (bench / profile labels). */
int ti_gemm_kernel_name(int bits, int x_kind, int M, int N, int K, char* buf, int len);

/* Same-run HBM calibration (bench lines): best-of-`reps` read GB/s of a `bytes` buffer streamed
 * once by 2 workgroups per CU, and hipMemcpyAsync device-to-device GB/s (read + write bytes).
 * Not a reference interface: the reference's benchmark times wall clock only
 * (benchmarks/benchmark_inference.cpp:309-384); this lets each measured rate be read against
 * the box it ran on. */
int ti_hbm_calibrate(size_t bytes, int reps, double* read_gbps, double* copy_gbps, ti_stream_t s);

/* (Round 5: the persistent decode launch ti_pds_decode, its ti_pds_args / ti_pds_layer structs,
 * ti_pds_supported and ti_pds_granule_words were removed -- the per-layer launches beat it at every
 * shape; the ti_engine_set_pds / _pds_error / _pds_timestamps stubs left in round 6,
 * INTEGRATION.md 3.) */

/* ------------------------------------------------------- step begin (device loop)
 * One block per stream: picks the token of this step (prompt token while step < n_in[m],
 * else the previous step's argmax), records fed-back tokens, gathers the fp16 embedding row
 * into h (fp32), sets pos[m] = base_pos[m] + *step_ctr, clears argmax row m (all slots).
 * placeholder_first >= 0 selects the reference_compat placeholder embedding
 * 0.1f*((offset + i) % 100) (inference_engine.cpp:1444-1448, 1509-1512) with offset
 * placeholder_first on step 0 and 0 afterwards.
 * fold_x non-NULL: also fold_x[m][i] = fp16(h[m][i] * fold_w[i]) and fold_ss[m] = sum_i
 * h[m][i]^2, the TI_X_F16_FOLDED input (n_ss = 1) of the first layer's projection. */
typedef struct ti_step_args {
  const uint16_t* emb;               /* [vocab][hidden] fp16 */
  float* h;                          /* [M][hidden] */
  int32_t hidden, M, vocab, in_stride, out_stride, placeholder_first;
  const int32_t* in_tokens;          /* [M][in_stride] */
  const int32_t* n_in;               /* [M] */
  unsigned long long* argmax;        /* [M][TI_ARGMAX_SLOTS] */
  int32_t* out_tokens;               /* [M][out_stride] generated tokens */
  int32_t* pos;                      /* [M] */
  const int32_t* base_pos;           /* [M] */
  const int32_t* step_ctr;
  const float* fold_w;               /* [hidden] (with fold_x) */
  uint16_t* fold_x;                  /* [M][hidden] fp16, nullable */
  float* fold_ss;                    /* [M] */
} ti_step_args;
int ti_step_begin(const ti_step_args* a, ti_stream_t s);

/* ------------------------------------------------------- on-device sampling
 * InferenceEngine::sample_next_token (inference_engine.cpp:1554-1673) per stream, the uniform
 * draw supplied (the reference draws it from the engine's mt19937): temperature, top-k
 * (1 <= top_k <= V; above TI_SAMPLE_MAX_K with a workspace, below), softmax, top-p, the draw.  Sums run over the
 * survivors in index order (the reference's loops over V add exact zeros elsewhere); exp/log
 * are the device's, equal logits at the k-th place and equal probabilities at the top-p cut
 * go lowest index first.  One 1024-thread workgroup per stream. */
#define TI_SAMPLE_MAX_K 4096
/* logits [M][ldl] fp32, draws [M] -> tokens [M], logprobs [M] (nullable) = log p(token). */
int ti_sample_device(const float* logits, int ldl, int M, int V, float temperature, int top_k, float top_p,
                     const float* draws, int32_t* tokens, float* logprobs, ti_stream_t s);
/* The decode loop's form (graph-capturable, after the lm_head): stream m's token of step
 * s = *step_ctr - advance is its t-th new token, t = s - (n_in[m] - 1); prompt steps (t < 0)
 * and t >= draw_stride do nothing.  The draw is draws[m*draw_stride + t], log p goes to
 * logprobs[m*draw_stride + t] (nullable), and argmax[m*TI_ARGMAX_SLOTS] receives a key above
 * every logit key, so ti_step_begin feeds the sampled token back. */
int ti_sample_step(const float* logits, int ldl, int M, int V, float temperature, int top_k, float top_p,
                   const float* draws, int draw_stride, const int32_t* step_ctr, int advance, const int32_t* n_in,
                   unsigned long long* argmax, float* logprobs, ti_stream_t s);
/* Any top_k up to V (the reference accepts any k, inference_engine.cpp:1585-1598): above
 * TI_SAMPLE_MAX_K the survivors' arrays live in a caller-provided device workspace of
 * M * ti_sample_workspace_bytes(V, top_k) bytes (0 for top_k <= TI_SAMPLE_MAX_K, where ws may be
 * null); the _ws forms take it, the plain forms are the _ws forms with ws = null. */
size_t ti_sample_workspace_bytes(int V, int top_k);
int ti_sample_device_ws(const float* logits, int ldl, int M, int V, float temperature, int top_k, float top_p,
                        const float* draws, int32_t* tokens, float* logprobs, void* ws, ti_stream_t s);
int ti_sample_step_ws(const float* logits, int ldl, int M, int V, float temperature, int top_k, float top_p,
                      const float* draws, int draw_stride, const int32_t* step_ctr, int advance, const int32_t* n_in,
                      unsigned long long* argmax, float* logprobs, void* ws, ti_stream_t s);

/* -------------------------------------------------------------- fp32 op level */
/* y[r][n] (+)= sum_k a[r][k]*b[k][n], b the reference [K][N] fp32 layout, one fmaf per k
 * in ascending order (bit-identical to matmul_3d_2d).  mode: 0 store, 1 relu(store),
 * 2 y = resid + sum (resid may alias y). */
int ti_matmul_f32(const float* a, const float* b, float* y, const float* resid, int rows, int K,
                  int N, int mode, ti_stream_t s);
int ti_rms_norm_f32(const float* x, const float* w, float* y, int rows, int n, float eps,
                    ti_stream_t s);
/* x [B][heads][S][D] fp32; cs [S*B or S][D/2][2] (cos, sin) computed by the caller with the
 * reference formula; pos_2d selects per-(b,s) rows of cs. */
int ti_rope_f32(const float* x, float* y, const float* cs, int B, int heads, int S, int D, int pos_2d,
                ti_stream_t s);
int ti_silu_f32(const float* x, float* y, int64_t n, ti_stream_t s);
int ti_relu_f32(const float* x, float* y, int64_t n, ti_stream_t s);
int ti_add_f32(const float* a, const float* b, float* y, int64_t n, ti_stream_t s);
int ti_mul_f32(const float* a, const float* b, float* y, int64_t n, ti_stream_t s);
int ti_softmax_f32(const float* x, float* y, int rows, int n, float temperature, ti_stream_t s);
/* multi_head_attention / attention_fast_incremental at op level: q [B][H], k, v [B][S][H]
 * with `heads` heads of H/heads dims interleaved in H (heads = 1: a single head of H dims);
 * out [B][H]; scratch B*heads*S floats (device). */
int ti_attention_f32(const float* q, const float* k, const float* v, float* out, float* scratch, int B, int S,
                     int H, int heads, ti_stream_t s);
/* out[r] = argmax_n x[r][n], lowest index on ties. */
int ti_argmax_f32(const float* x, int32_t* out, int rows, int n, ti_stream_t s);

#ifdef __cplusplus
}
#endif
#endif /* TI_HIP_H */
