// engine.cpp -- the device-resident decode engine (ti_engine.h).
//
// State per engine (one device, one HIP stream):
//   * packed weights: per layer one fused [q|k|v] linear, o, one gate/up linear with rows
//     interleaved by 8 (so the SiLU*up epilogue sees both halves in one 16-row tile), down;
//     lm_head; fp16 embedding table; fp32 norm weights; RoPE (cos, sin) table computed on
//     the host with the reference formula (tensor_engine.cpp:1561-1566, 1595-1597).
//   * per stream fp16 K/V caches [layer][stream][kv_head][max_seq][head_dim].
//   * a device-side decode loop: step counter, positions, argmax feedback -- one decode
//     step is a fixed launch sequence captured once into a hipGraph and replayed, so the
//     host never waits inside generate().
// Reference counterparts: InferenceEngineImpl (src/model/inference_engine.cpp:446-693),
// KVCache (:25-172), forward_pass_incremental (:1493-1552), generate (:734-802).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <queue>
#include <cstdlib>
#include <cstring>
#include <map>
#include <utility>
#include <vector>

#include "ti_engine.h"
#include "ti_hip.h"

int ti_set_error(int code, const char* fmt, ...);
int ti_check_hip(hipError_t e, const char* what);

#define E_CHECK(expr, what)                                \
  do {                                                     \
    hipError_t _e = (expr);                                \
    if (_e != hipSuccess) return ti_check_hip(_e, what);   \
  } while (0)
#define TI_TRY(expr)                 \
  do {                               \
    const int _rc = (expr);          \
    if (_rc != TI_OK) return _rc;    \
  } while (0)

namespace {

// tensor ids of the synthetic model: identical to oracle/ti_oracle.c
constexpr uint32_t kTidEmb = 1, kTidOutNorm = 2, kTidLmHead = 3, kTidLayer0 = 16;
enum { TL_ATTN_NORM = 0, TL_FFN_NORM, TL_Q, TL_K, TL_V, TL_O, TL_G, TL_U, TL_D };
inline uint32_t tid_layer(int l, int t) { return kTidLayer0 + 16u * (uint32_t)l + (uint32_t)t; }
inline uint32_t tid_kv(int l, int v) { return 0x100000u + 2u * (uint32_t)l + (uint32_t)v; }

struct DevLinear {
  void* tiles = nullptr;
  uint16_t* scales = nullptr;
  float* f32 = nullptr;     // compat: reference-layout fp32 [K][N]
  int K = 0, N = 0;
};

struct DevLayer {
  DevLinear qkv, o, gu, down;
  float* attn_norm = nullptr;
  float* ffn_norm = nullptr;
  uint16_t* kc = nullptr;
  uint16_t* vc = nullptr;
};

uint16_t host_half(float f) {
  const _Float16 h = (_Float16)f;
  uint16_t u;
  std::memcpy(&u, &h, 2);
  return u;
}

}  // namespace

struct ti_engine {
  ti_engine_config c{};
  hipStream_t s = nullptr;
  std::vector<void*> allocs;
  std::vector<DevLayer> layer;
  DevLinear lm;
  uint16_t* emb = nullptr;
  float* out_norm = nullptr;
  float* rope_cs = nullptr;
  // step buffers
  float* h = nullptr;
  float* h_last = nullptr;   // [max_batch][hidden]: each stream's last prompt row (ti_engine_generate)
  float* q = nullptr;
  float* tmp = nullptr;        // compat FFN activations (fp32)
  float* logits = nullptr;
  float* ws = nullptr;
  uint16_t* attn = nullptr;
  uint16_t* act = nullptr;
  uint16_t* xn = nullptr;      // fp16 rms_norm rows for the batched-rows GEMM [R][hidden]
  // single-stream steps with the rms_norm folded behind the GEMM (ti_hip.h TI_X_F16_FOLDED):
  // the epilogue that writes h also writes fx = fp16(h * next norm weight) and its workgroups'
  // sums of h^2 (ss); the next projection stages fx and divides its outputs by the rms
  bool fold_on = true;         // TI_FOLD=0 / ti_engine_set_fold
  uint16_t* fx = nullptr;      // [hidden]
  float* ss = nullptr;         // [256]
  // batched fold (17..64 int4 rows): the producers' (O, down) epilogues write xn = fp16(h * next
  // norm weight) and per-column-group sums of h^2 per row [n_cg][TI_FOLD_SS_ROWS]
  float* ss_rows = nullptr;
  // single-stream attention leaves its split merge to the O projection (ti_attn_decode_partials
  // + TI_X_ATTN_SPLITS): no arrival-ticket hand-off at the end of the attention launch
  bool part_on = true;         // TI_ATTN_PART=0 turns it off
  uint16_t* part_o = nullptr;  // [heads][TI_ATTN_MAX_PART_SPLITS][head_dim]
  float* part_ml = nullptr;    // [heads][TI_ATTN_MAX_PART_SPLITS][2]
  // one stream (head_dim 64 GQA or head_dim 128 MHA): QKV and the attention in one launch (ti_qkv_attn_partials,
  // DESIGN 4.19), O merging its splits (TI_X_ATTN_SPLITS); TI_QKV_ATTN=0 turns it off
  bool qa_on = true;
  void* qa_xchg = nullptr;     // the q exchange of ti_qkv_attn_partials (zeroed once, generations kept)
  // on-device sampling (ti_engine_generate_sampled): the step graph ends with ti_sample_step
  bool samp_on = false;
  float samp_t = 1.0f, samp_p = 1.0f;
  int samp_k = 1;
  float* draws = nullptr;      // [max_batch][draw_cap] uniform draws, per new token
  float* lps = nullptr;        // [max_batch][draw_cap] log p of the sampled tokens
  int draw_cap = 0;
  void* splitk_ws = nullptr;   // tile GEMM split-K workspace (ti_epilogue.splitk_ws), int4 engines
  size_t splitk_bytes = 0;
  void* samp_ws = nullptr;     // ti_sample_step_ws workspace (top_k > TI_SAMPLE_MAX_K)
  size_t samp_ws_bytes = 0;
  // prefill (forward_pass over prompt tokens): up to pf_rows prompt tokens of one stream run
  // as rows of the batched path, sharing that stream's KV cache (stride 0)
  int pf_rows = 0;             // 0 = off (prompts consumed one token per decode step)
  int rows_cap = 0;            // R = max(max_batch, pf_rows): rows the step buffers hold
  int32_t* pf_ones = nullptr;  // [pf_rows] 1
  int32_t* pf_zero = nullptr;  // [1] 0
  int32_t* pf_base = nullptr;  // [pf_rows] positions of the chunk's rows
  unsigned long long* argmax = nullptr;
  int32_t* pos = nullptr;
  int32_t* base_pos = nullptr;
  int32_t* step_ctr = nullptr;
  int32_t* n_in = nullptr;
  int32_t* in_tokens = nullptr;
  int32_t* out_tokens = nullptr;
  int in_cap = 0, out_cap = 0;
  // generate() stop token (ti_engine_set_stop): the device loop runs in chunks and ends once every
  // stream has emitted it (the reference's `break` at EOS, inference_engine.cpp:760-764); -1 = none
  int32_t stop_token = -1;
  uint64_t n_decode_steps = 0;   // step-graph replays (ti_engine_counters)
  uint64_t n_prefill_chunks = 0; // prompt chunks through enqueue_prefill
  int splits_max = 1;
  int64_t kv_stride = 0;
  uint16_t** kv_tab = nullptr;   // device [2 * layers]: every layer's K then V cache base (ti_kv_copy_slots)
  size_t weight_bytes = 0, kv_bytes = 0;
  std::map<std::pair<int, int>, hipGraphExec_t> graphs;  // (M, advance | sampled << 1)
  int replay_M = 0;

  int qd() const { return c.heads * c.head_dim; }
  int kvd() const { return c.kv_heads * c.head_dim; }

  int alloc(void** p, size_t bytes) {
    TI_TRY(ti_malloc(p, bytes));
    allocs.push_back(*p);
    E_CHECK(hipMemsetAsync(*p, 0, bytes, s), "hipMemsetAsync(alloc)");
    return TI_OK;
  }
  template <class T>
  int alloc_t(T** p, size_t count) {
    void* v = nullptr;
    TI_TRY(alloc(&v, count * sizeof(T)));
    *p = static_cast<T*>(v);
    return TI_OK;
  }
  int alloc_linear(DevLinear& L, int K, int N) {
    L.K = K;
    L.N = N;
    if (c.compat) {
      TI_TRY(alloc_t(&L.f32, (size_t)K * N));
      weight_bytes += (size_t)K * N * 4;
      return TI_OK;
    }
    const size_t tb = ti_wpack_tile_bytes(c.bits, K, N), sb = ti_wpack_scale_bytes(c.bits, K, N);
    TI_TRY(alloc(&L.tiles, tb));
    if (sb) {
      void* p = nullptr;
      TI_TRY(alloc(&p, sb));
      L.scales = static_cast<uint16_t*>(p);
    }
    weight_bytes += tb + sb;
    return TI_OK;
  }
  // attention workgroups aimed at: one 8-wave workgroup per CU (128 / 256 / 512 measured 717 / 751 /
  // 681 tok/s); GQA partials with 8 splits
  static constexpr int attn_target = 256;
  static constexpr int gqa_part_splits = 8;
  int splits_for(int M) const {
    if (c.attn_splits > 0) return c.attn_splits;
    // one stream of a GQA model (>= 4 q-heads per kv-head) with a small cache per kv-head
    // (<= 1 MiB of K + V: TinyLlama at 2048): few long splits whose partials the O projection
    // merges (part_usable), instead of 64+ short splits merged by a last arriver
    // (attention run head by head: ti_attn_decode_partials' GQA expansion, heads x splits workgroups)
    if (M == 1 && gqa_part_splits >= 2 && part_on && c.heads >= 4 * c.kv_heads &&
        (size_t)c.max_seq * c.head_dim * 4 <= ((size_t)1 << 20))
      return std::min(gqa_part_splits, std::max(2, std::min(c.max_seq / 64, (attn_target + c.heads - 1) / c.heads)));
    // one 8-wave attention workgroup per CU: a second round of workgroups costs a whole
    // workgroup latency (load, merge hand-off) for little bandwidth (tools/probe_attn.hip)
    const int target = attn_target;
    int sp = (target + c.kv_heads * M - 1) / (c.kv_heads * M);
    const int cap = std::max(1, c.max_seq / 64);
    return std::max(1, std::min(sp, std::min(cap, 64)));
  }

  ~ti_engine() {
    for (auto& g : graphs) hipGraphExecDestroy(g.second);
    for (void* p : allocs) hipFree(p);
    if (s) hipStreamDestroy(s);
  }
};

namespace {

// Every ti_engine_* entry binds the engine's device for its duration and restores the caller's
// current device on return (lazy allocations, graph (re)instantiation and launches all run on
// e->c.device whatever device the calling thread has current): several engines on several
// devices can be driven from one process, from any host thread (the reference
// binds its device in TensorEngine::initialize, tensor_engine.cpp:425-487).
struct DeviceScope {
  int prev = -1;
  bool changed = false;
  explicit DeviceScope(int device) {
    if (device >= 0 && hipGetDevice(&prev) == hipSuccess && prev != device) changed = hipSetDevice(device) == hipSuccess;
  }
  explicit DeviceScope(const ti_engine* e) : DeviceScope(e ? e->c.device : -1) {}
  ~DeviceScope() {
    if (changed) hipSetDevice(prev);
  }
  DeviceScope(const DeviceScope&) = delete;
  DeviceScope& operator=(const DeviceScope&) = delete;
};

// In-step launch stamps (ti_engine_stamp_steps): while a stamped step graph is being captured on this
// thread, every decode launcher asks ti_stamp_next for its workgroups' slot (kernels/common.hpp
// stamp_end: kStampWords = 16 words per workgroup) and the launch's kind / tag / grid are recorded.
constexpr int kStampWords = 24;   // = ti::kStampWords (kernels/common.hpp)
struct StampCtx {
  bool on = false;
  unsigned long long* base = nullptr;   // NULL: the sizing pass (record only)
  int tag = TI_STAMP_TAG_OTHER;
  std::vector<int32_t> info;            // [launch][3] kind, tag, workgroups (0 = unstamped)
  std::vector<size_t> offs;             // word offset of each launch's slot (second pass)
};
thread_local StampCtx g_stamp;
inline void stamp_tag(int t) { g_stamp.tag = t; }

int validate(const ti_engine_config& c) {
  if (c.vocab < 1 || c.hidden < 1 || c.layers < 0 || c.inter < 1 || c.max_seq < 1 || c.max_batch < 1)
    return ti_set_error(TI_ERR_ARG, "ti_engine_create: non-positive size in config");
  if (c.compat) return TI_OK;
  if (c.heads < 1 || c.kv_heads < 1 || c.heads % c.kv_heads)
    return ti_set_error(TI_ERR_ARG, "ti_engine_create: heads %d / kv_heads %d", c.heads, c.kv_heads);
  const int G = c.heads / c.kv_heads;
  if (G != 1 && G != 2 && G != 4 && G != 8) return ti_set_error(TI_ERR_UNSUPPORTED, "ti_engine_create: GQA group %d", G);
  if (c.head_dim != 64 && c.head_dim != 128) return ti_set_error(TI_ERR_UNSUPPORTED, "ti_engine_create: head_dim %d", c.head_dim);
  if (c.bits != 4 && c.bits != 8 && c.bits != 16 && c.bits != (4 | TI_BITS_G32) && c.bits != (8 | TI_BITS_G32) &&
      c.bits != (4 | TI_BITS_G32 | TI_BITS_AFF))
    return ti_set_error(TI_ERR_ARG, "ti_engine_create: bits %d (4, 8, 16; 4 or 8 | TI_BITS_G32; 4 | TI_BITS_G32 | "
                        "TI_BITS_AFF)", c.bits);
  const int qd = c.heads * c.head_dim, kvd = c.kv_heads * c.head_dim;
  if (c.hidden % 128 || qd % 128 || c.inter % 128)
    return ti_set_error(TI_ERR_UNSUPPORTED, "ti_engine_create: hidden, heads*head_dim and inter must be multiples of 128");
  if (kvd % 16 || c.vocab % 16)
    return ti_set_error(TI_ERR_UNSUPPORTED, "ti_engine_create: kv_heads*head_dim and vocab must be multiples of 16");
  return TI_OK;
}

// Rows of the batched-rows kernel (int4, M > 16) take their fp16 operands in fragment order
// (TI_X_F16_PACKED): the rms_norm prep, the attention output and the SiLU*up output are written
// that way, so every operand load of the kernel is one contiguous KiB per wave.
bool packed_rows(const ti_engine* e, int M) { return ti_gemm_packed_rows(e->c.bits, M) != 0; }

// One projection for rows [0, M): the fused kernel in chunks of the rows its LDS image
// holds, or -- int4, when the rows do not fit -- rms_norm into fp16 rows once (e->xn) and
// the batched-rows kernel in chunks of TI_GEMM_MAX_ROWS.  Graph-capturable.
int gemm_rows(ti_engine* e, const DevLinear& W, int M, const void* x, int x_kind, int ldx, const float* nw,
              const ti_epilogue& epi, size_t out_elem, bool last_gets_ctr) {
  const ti_engine_config& c = e->c;
  int rows = ti_gemm_max_rows(c.bits, x_kind, W.N, W.K);
  if (x_kind == TI_X_F32_RMSNORM && ti_gemm_packed_rows_for(c.bits, M, W.N, W.K) && e->xn) {
    TI_TRY(ti_rmsnorm_f16_packed(static_cast<const float*>(x), ldx, nw, c.eps, e->xn, M, W.K, e->s));
    x = e->xn;
    x_kind = TI_X_F16_PACKED;
    ldx = W.K;
    rows = ti_gemm_max_rows(c.bits, x_kind, W.N, W.K);
  } else if (x_kind == TI_X_F32_RMSNORM && rows < M && (c.bits & ~TI_BITS_G32) == 4 && e->xn) {
    TI_TRY(ti_rmsnorm_f16(static_cast<const float*>(x), ldx, nw, c.eps, e->xn, W.K, M, W.K, e->s));
    x = e->xn;
    x_kind = TI_X_F16;
    ldx = W.K;
    rows = ti_gemm_max_rows(c.bits, x_kind, W.N, W.K);
  }
  if (rows < 1) return ti_set_error(TI_ERR_UNSUPPORTED, "engine: no GEMM kernel for N=%d K=%d", W.N, W.K);
  const size_t x_elem = x_kind == TI_X_F16 || x_kind == TI_X_F16_FOLDED || x_kind == TI_X_F16_PACKED ? 2 : 4;
  for (int m0 = 0; m0 < M; m0 += rows) {
    const int mm = std::min(rows, M - m0);
    ti_epilogue ep = epi;
    ep.out = static_cast<char*>(epi.out) + (size_t)m0 * epi.ldo * out_elem;
    if (ep.pos) ep.pos += m0;
    if (ep.k_cache) ep.k_cache += (size_t)m0 * ep.kv_stream_stride;
    if (ep.v_cache) ep.v_cache += (size_t)m0 * ep.kv_stream_stride;
    if (ep.argmax) ep.argmax += (size_t)m0 * TI_ARGMAX_SLOTS;
    if (!(last_gets_ctr && m0 + mm >= M)) ep.step_ctr = nullptr;
    ep.splitk_ws = e->splitk_ws;
    ep.splitk_bytes = (int64_t)e->splitk_bytes;
    const void* xm = static_cast<const char*>(x) + (size_t)m0 * ldx * x_elem;
    TI_TRY(ti_gemm_wq_a16(W.tiles, W.scales, c.bits, xm, x_kind, ldx, nw, c.eps, mm, W.N, W.K, &ep, e->s));
  }
  return TI_OK;
}


int get_graph(ti_engine* e, int M, int advance, hipGraphExec_t* out);

// n steps of M streams from the current device state: the replayed step graph.
int run_steps(ti_engine* e, int M, int advance, int n) {
  if (n <= 0) return TI_OK;
  hipGraphExec_t g = nullptr;
  TI_TRY(get_graph(e, M, advance, &g));
  for (int s = 0; s < n; ++s) E_CHECK(hipGraphLaunch(g, e->s), "hipGraphLaunch");
  e->n_decode_steps += (uint64_t)n;
  return TI_OK;
}

// The folded rms_norm hand-off applies to single-stream steps whose producers (O, down) run on
// the fused kernel with at most 256 workgroups.
bool fold_usable(ti_engine* e, int M) {
  const ti_engine_config& c = e->c;
  // (group-32 weights: their launch grid is not ti_gemm_grid's, so no fold hand-off)
  if (!e->fold_on || M != 1 || c.compat || !e->fx || (c.bits & TI_BITS_G32)) return false;
  const int H = c.hidden, I = c.inter, qd = e->qd();
  const int g_o = ti_gemm_grid(1, H, qd), g_d = ti_gemm_grid(1, H, I);
  return g_o > 0 && g_o <= 256 && g_d > 0 && g_d <= 256 && ti_gemm_max_rows(c.bits, TI_X_F16, H, qd) >= 1;
}

// The batched fold: 17..64 int4 rows on the batched-rows kernels (packed operands), the O / down
// producers' column groups within the partial buffer.
bool bfold_usable(ti_engine* e, int M) {
  const ti_engine_config& c = e->c;
  if (!e->fold_on || c.compat || c.bits != 4 || M <= 16 || M > TI_FOLD_SS_ROWS || !packed_rows(e, M) || !e->ss_rows)
    return false;
  const int po = ti_gemm_fold_partials(c.bits, M, c.hidden, e->qd()), pd = ti_gemm_fold_partials(c.bits, M, c.hidden, c.inter);
  return po >= 1 && po <= 4096 && pd >= 1 && pd <= 4096;
}

// Split partials merged by the O projection: one stream, 2..8 splits, heads*head_dim <= 4096.
bool part_usable(ti_engine* e, int M) {
  const ti_engine_config& c = e->c;
  const int sp = e->splits_for(M);
  return e->part_on && e->part_o && M == 1 && !c.compat && sp >= 2 && sp <= TI_ATTN_MAX_PART_SPLITS &&
         e->qd() <= 4096;
}


// The fused launch's bounded waits: after the stream's work, a set error word means a workgroup's q part or
// new key never came (wrong results for that step) -- reported, and the exchange zeroed so the generations
// agree again.  One 4-byte read on the engine's stream (synchronous).
bool qa_usable(ti_engine* e, int M);
int qa_fault_check(ti_engine* e) {
  if (!e->qa_xchg || !qa_usable(e, 1)) return TI_OK;   // (only engines whose 1-stream steps take the launch)
  const ti_engine_config& c = e->c;
  const size_t off = ti_qkv_attn_error_offset(c.heads, e->splits_for(1));
  if (off + 8 > ti_qkv_attn_xchg_bytes(c.heads, TI_ATTN_MAX_PART_SPLITS))
    return ti_set_error(TI_ERR_ARG, "engine: exchange error word outside the buffer");
  uint32_t err[2] = {0u, 0u};
  TI_TRY(ti_memcpy_d2h(err, static_cast<char*>(e->qa_xchg) + off, sizeof(err), e->s));
  if (!err[0] && !err[1]) return TI_OK;
  TI_TRY(ti_memset(e->qa_xchg, 0, ti_qkv_attn_xchg_bytes(c.heads, TI_ATTN_MAX_PART_SPLITS), e->s));
  TI_TRY(ti_stream_sync(e->s));
  return ti_set_error(TI_ERR_HIP, "engine: the fused QKV + attention launch's exchange timed out (a workgroup's q "
                      "part or the new key never arrived); results of the last call are wrong, exchange reset");
}

// QKV + attention in one launch (ti_qkv_attn_partials): one stream with the fold and split partials,
// int8 / int4 group-128 weights, head_dim 64 GQA (TinyLlama-1.1B) or head_dim 128 MHA (Llama-2-7B).
bool qa_usable(ti_engine* e, int M) {
  const ti_engine_config& c = e->c;
  if (!e->qa_on || M != 1 || !fold_usable(e, M) || !part_usable(e, M)) return false;
  // all heads x splits workgroups resident at once for the in-launch q exchange
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return false;
  const int sp = e->splits_for(M);
  return c.heads * sp <= cus && ti_gemm_grid(1, c.hidden, c.inter) <= 256 &&
         ti_qkv_attn_supported(c.bits, c.hidden, c.heads, c.kv_heads, c.head_dim, sp);
}

// One decode step for streams [0, M) on e->s.  Graph-capturable (no host sync / alloc).
int enqueue_step(ti_engine* e, int M, int advance) {
  const ti_engine_config& c = e->c;
  ti_step_args sa{};
  sa.emb = e->emb;
  sa.h = e->h;
  sa.hidden = c.hidden;
  sa.M = M;
  sa.vocab = c.vocab;
  sa.in_stride = e->in_cap;
  sa.out_stride = e->out_cap;
  sa.placeholder_first = -1;
  sa.in_tokens = e->in_tokens;
  sa.n_in = e->n_in;
  sa.argmax = e->argmax;
  sa.out_tokens = e->out_tokens;
  sa.pos = e->pos;
  sa.base_pos = e->base_pos;
  sa.step_ctr = e->step_ctr;
  const int H = c.hidden, qd = e->qd(), kvd = e->kvd(), I = c.inter, V = c.vocab;
  // fold (M == 1): every rms_norm input is handed over as fx + ss partials by its producer
  const bool fold = fold_usable(e, M), part = part_usable(e, M), pk = packed_rows(e, M), qa = qa_usable(e, M);
  // batched fold (17..64 rows): O / down write xn = fp16(h * next norm weight) and per-row sums of
  // h^2; QKV (after layer 0), gate/up and the lm_head normalise behind their GEMM (ti_hip.h)
  const bool bfold = !fold && bfold_usable(e, M);
  int bn_ss = 0;   // partials per row the last batched producer wrote (0: none yet, rms_norm prep)
  auto next_norm = [&](int l) -> const float* { return l < c.layers ? e->layer[l].attn_norm : e->out_norm; };
  auto next_n = [&](int l) -> int { return l < c.layers ? e->layer[l].qkv.N : e->lm.N; };
  if (fold) {
    sa.fold_w = next_norm(0);
    sa.fold_x = e->fx;
    sa.fold_ss = e->ss;
  }
  stamp_tag(TI_STAMP_TAG_BEGIN);
  TI_TRY(ti_step_begin(&sa, e->s));
  int n_ss = 1;   // partials the last producer wrote (step_begin: one)
  // producer side (RESID epilogue); n_next: output width of the call that consumes the fold
  auto fold_into = [&](ti_epilogue& ep, const float* w, int n_next) {
    if (fold) {
      ep.fold_w = w;
      ep.fold_x = e->fx;
      ep.fold_ss = e->ss;
    } else if (bfold) {
      ep.fold_w = w;
      ep.fold_x = e->xn;
      ep.fold_ss = e->ss_rows;
      ep.fold_packed = ti_gemm_packed_rows_for(c.bits, M, n_next, H);
    }
  };
  auto norm_in = [&](const void*& x, int& xk, int& ldx, const float*& nw, ti_epilogue& ep, int n) {   // consumer side
    if (fold) {
      x = e->fx;
      xk = TI_X_F16_FOLDED;
      ldx = H;
      nw = nullptr;
      ep.ss_in = e->ss;
      ep.n_ss = n_ss;
    } else if (bfold && bn_ss > 0) {
      x = e->xn;
      xk = ti_gemm_packed_rows_for(c.bits, M, n, H) ? TI_X_F16_PACKED : TI_X_F16;
      ldx = H;
      nw = nullptr;
      ep.ss_in = e->ss_rows;
      ep.n_ss = bn_ss;
    }
  };

  auto gemm = [&](const DevLinear& W, const void* x, int x_kind, int ldx, size_t /*x_elem*/, const float* nw,
                  ti_epilogue epi, size_t out_elem, bool last_gets_ctr) -> int {
    if (x_kind == TI_X_F32_RMSNORM) norm_in(x, x_kind, ldx, nw, epi, W.N);
    TI_TRY(gemm_rows(e, W, M, x, x_kind, ldx, nw, epi, out_elem, last_gets_ctr));
    if (epi.fold_x && fold) n_ss = ti_gemm_grid(M, W.N, W.K);
    if (epi.fold_x && bfold) bn_ss = ti_gemm_fold_partials(c.bits, M, W.N, W.K);
    return TI_OK;
  };

  for (int l = 0; l < c.layers; ++l) {
    DevLayer& L = e->layer[l];
    ti_epilogue ep{};
    ep.kind = TI_EPI_QKV_ROPE_KV;
    ep.ldo = qd;
    ep.out = e->q;
    ep.q_dim = qd;
    ep.kv_dim = kvd;
    ep.head_dim = c.head_dim;
    ep.max_seq = c.max_seq;
    ep.pos = e->pos;
    ep.rope_cs = e->rope_cs;
    ep.k_cache = L.kc;
    ep.v_cache = L.vc;
    ep.kv_stream_stride = e->kv_stride;
    ti_epilogue eo{};
    eo.kind = TI_EPI_RESID_F32;
    eo.ldo = H;
    eo.out = e->h;
    fold_into(eo, L.ffn_norm, L.gu.N);
    if (qa) {   // QKV + attention in one launch; O merges the splits
      stamp_tag(TI_STAMP_TAG_QKV);
      const int S = e->splits_for(M);
      TI_TRY(ti_qkv_attn_partials(L.qkv.tiles, L.qkv.scales, c.bits, e->fx, e->ss, n_ss, c.eps, e->rope_cs, e->pos,
                                  L.kc, L.vc, c.max_seq, H, c.heads, c.kv_heads, c.head_dim, S, e->part_o, e->part_ml,
                                  e->qa_xchg, e->s));
      eo.ss_in = e->part_ml;
      eo.n_ss = S;
      eo.head_dim = c.head_dim;
      stamp_tag(TI_STAMP_TAG_O);
      TI_TRY(gemm(L.o, e->part_o, TI_X_ATTN_SPLITS, qd, 2, nullptr, eo, 4, false));
    } else if (part) {   // the O projection merges the attention's splits while staging its input
      stamp_tag(TI_STAMP_TAG_QKV);
      TI_TRY(gemm(L.qkv, e->h, TI_X_F32_RMSNORM, H, 4, L.attn_norm, ep, 4, false));
      stamp_tag(TI_STAMP_TAG_ATTN);
      TI_TRY(ti_attn_decode_partials(e->q, L.kc, L.vc, e->kv_stride, c.max_seq, e->pos, M, c.heads, c.kv_heads,
                                     c.head_dim, e->splits_for(M), e->part_o, e->part_ml, e->s));
      eo.ss_in = e->part_ml;
      eo.n_ss = e->splits_for(M);
      eo.head_dim = c.head_dim;
      stamp_tag(TI_STAMP_TAG_O);
      TI_TRY(gemm(L.o, e->part_o, TI_X_ATTN_SPLITS, qd, 2, nullptr, eo, 4, false));
    } else {
      stamp_tag(TI_STAMP_TAG_QKV);
      TI_TRY(gemm(L.qkv, e->h, TI_X_F32_RMSNORM, H, 4, L.attn_norm, ep, 4, false));
      stamp_tag(TI_STAMP_TAG_ATTN);
      TI_TRY((pk ? ti_attn_decode_packed : ti_attn_decode)(e->q, L.kc, L.vc, e->kv_stride, c.max_seq, e->pos, M,
                                                           c.heads, c.kv_heads, c.head_dim, e->splits_for(M), e->ws,
                                                           e->attn, e->s));
      stamp_tag(TI_STAMP_TAG_O);
      TI_TRY(gemm(L.o, e->attn, pk ? TI_X_F16_PACKED : TI_X_F16, qd, 2, nullptr, eo, 4, false));
    }

    ti_epilogue eg{};
    eg.kind = TI_EPI_SILU_MUL_F16;
    eg.ldo = I;
    eg.out = e->act;
    eg.out_packed = pk;
    stamp_tag(TI_STAMP_TAG_GATE_UP);
    TI_TRY(gemm(L.gu, e->h, TI_X_F32_RMSNORM, H, 4, L.ffn_norm, eg, 2, false));

    ti_epilogue ed{};
    ed.kind = TI_EPI_RESID_F32;
    ed.ldo = H;
    ed.out = e->h;
    fold_into(ed, next_norm(l + 1), next_n(l + 1));
    stamp_tag(TI_STAMP_TAG_DOWN);
    TI_TRY(gemm(L.down, e->act, pk ? TI_X_F16_PACKED : TI_X_F16, I, 2, nullptr, ed, 4, false));
  }
  ti_epilogue el{};
  el.kind = TI_EPI_LOGITS_ARGMAX;
  el.ldo = V;
  el.out = e->logits;
  el.argmax = e->argmax;
  el.step_ctr = e->step_ctr;
  el.advance = advance;
  stamp_tag(TI_STAMP_TAG_LM_HEAD);
  TI_TRY(gemm(e->lm, e->h, TI_X_F32_RMSNORM, H, 4, e->out_norm, el, 4, true));
  stamp_tag(TI_STAMP_TAG_OTHER);
  if (e->samp_on)   // sample_next_token on the device; its key feeds the token back (ti_hip.h)
    TI_TRY(ti_sample_step_ws(e->logits, V, M, V, e->samp_t, e->samp_k, e->samp_p, e->draws, e->draw_cap, e->step_ctr,
                             advance, e->n_in, e->argmax, e->lps, e->samp_ws, e->s));
  return TI_OK;
}

// Prefill (reference forward_pass, inference_engine.cpp:1429-1491, with the KV kept): prompt
// tokens [t0, t0 + rows) of stream m at positions base + t0 + j, as `rows` rows of the
// batched path that share stream m's KV cache (epilogue / attention stream stride 0: row j
// appends at its own position and attends to [0, base + t0 + j], causal).  No lm_head here: the
// decode loop takes over at the last prompt token, or ti_engine_generate runs the lm_head on the
// chunk's last row.  Not graph-captured (host position upload).
// TI_ATTN_PREFILL=0: prefill chunks through the decode attention kernel (A/B knob)
static bool prefill_attn_on();

// Decode-attention workspace: the largest need over the row counts that run the split kernel --
// decode batches up to max_batch and prompt chunks of up to 64 rows (ti_gemm_packed_rows; longer
// chunks run ti_attn_prefill, no workspace), all chunk sizes when TI_ATTN_PREFILL=0.
size_t ws_bytes(const ti_engine* e) {
  const ti_engine_config& c = e->c;
  const int R = prefill_attn_on() ? std::min(e->rows_cap, std::max(c.max_batch, 64)) : e->rows_cap;
  size_t b = 0;
  for (int M = 1; M <= R; ++M) b = std::max(b, ti_attn_workspace_bytes(M, c.heads, c.head_dim, e->splits_for(M)));
  return b;
}

// TI_PREFILL_LOGITS=0: the last prompt token through a decode step instead (A/B knob, ti_engine_generate)
static bool prefill_logits_on() {
  static const int on = [] {
    const char* v = getenv("TI_PREFILL_LOGITS");
    return v ? atoi(v) != 0 : 1;
  }();
  return on != 0;
}

static bool prefill_attn_on() {
  static const int on = [] {
    const char* v = getenv("TI_ATTN_PREFILL");
    return v ? atoi(v) != 0 : 1;
  }();
  return on != 0;
}

int enqueue_prefill(ti_engine* e, int m, int t0, int rows, int base) {
  const ti_engine_config& c = e->c;
  ++e->n_prefill_chunks;
  std::vector<int32_t> bp(rows);
  for (int j = 0; j < rows; ++j) bp[j] = base + t0 + j;
  TI_TRY(ti_memcpy_h2d(e->pf_base, bp.data(), (size_t)rows * 4, e->s));
  ti_step_args sa{};
  sa.emb = e->emb;
  sa.h = e->h;
  sa.hidden = c.hidden;
  sa.M = rows;
  sa.vocab = c.vocab;
  sa.in_stride = 1;                       // row j reads in_tokens[j + step_ctr] = token t0 + j
  sa.out_stride = 0;
  sa.placeholder_first = -1;
  sa.in_tokens = e->in_tokens + (size_t)m * e->in_cap + t0;
  sa.n_in = e->pf_ones;
  sa.argmax = e->argmax;
  sa.out_tokens = nullptr;
  sa.pos = e->pos;
  sa.base_pos = e->pf_base;
  sa.step_ctr = e->pf_zero;
  TI_TRY(ti_step_begin(&sa, e->s));
  const int H = c.hidden, qd = e->qd(), kvd = e->kvd(), I = c.inter;
  for (int l = 0; l < c.layers; ++l) {
    DevLayer& L = e->layer[l];
    uint16_t* kc = L.kc + (size_t)m * e->kv_stride;
    uint16_t* vc = L.vc + (size_t)m * e->kv_stride;
    ti_epilogue ep{};
    ep.kind = TI_EPI_QKV_ROPE_KV;
    ep.ldo = qd;
    ep.out = e->q;
    ep.q_dim = qd;
    ep.kv_dim = kvd;
    ep.head_dim = c.head_dim;
    ep.max_seq = c.max_seq;
    ep.pos = e->pos;
    ep.rope_cs = e->rope_cs;
    ep.k_cache = kc;
    ep.v_cache = vc;
    ep.kv_stream_stride = 0;
    TI_TRY(gemm_rows(e, L.qkv, rows, e->h, TI_X_F32_RMSNORM, H, L.attn_norm, ep, 4, false));
    const bool pk = packed_rows(e, rows);
    if (!pk && prefill_attn_on())   // row-major chunk: one pass over the prefix per 16 rows (MFMA)
      TI_TRY(ti_attn_prefill(e->q, kc, vc, c.max_seq, e->pos, rows, c.heads, c.kv_heads, c.head_dim, e->attn, e->s));
    else
      TI_TRY((pk ? ti_attn_decode_packed : ti_attn_decode)(e->q, kc, vc, 0, c.max_seq, e->pos, rows, c.heads,
                                                           c.kv_heads, c.head_dim, e->splits_for(rows), e->ws,
                                                           e->attn, e->s));
    ti_epilogue eo{};
    eo.kind = TI_EPI_RESID_F32;
    eo.ldo = H;
    eo.out = e->h;
    TI_TRY(gemm_rows(e, L.o, rows, e->attn, pk ? TI_X_F16_PACKED : TI_X_F16, qd, nullptr, eo, 4, false));
    ti_epilogue eg{};
    eg.kind = TI_EPI_SILU_MUL_F16;
    eg.ldo = I;
    eg.out = e->act;
    eg.out_packed = pk;
    TI_TRY(gemm_rows(e, L.gu, rows, e->h, TI_X_F32_RMSNORM, H, L.ffn_norm, eg, 2, false));
    ti_epilogue ed{};
    ed.kind = TI_EPI_RESID_F32;
    ed.ldo = H;
    ed.out = e->h;
    TI_TRY(gemm_rows(e, L.down, rows, e->act, pk ? TI_X_F16_PACKED : TI_X_F16, I, nullptr, ed, 4, false));
  }
  return TI_OK;
}

int get_graph(ti_engine* e, int M, int advance, hipGraphExec_t* out) {
  auto key = std::make_pair(M, advance | (e->samp_on ? 2 : 0));
  auto it = e->graphs.find(key);
  if (it != e->graphs.end()) {
    *out = it->second;
    return TI_OK;
  }
  TI_TRY(ti_gemm_prepare());
  E_CHECK(hipStreamBeginCapture(e->s, hipStreamCaptureModeThreadLocal), "hipStreamBeginCapture");
  const int rc = enqueue_step(e, M, advance);
  hipGraph_t g = nullptr;
  const hipError_t ec = hipStreamEndCapture(e->s, &g);
  if (rc != TI_OK) {
    if (g) hipGraphDestroy(g);
    return rc;
  }
  E_CHECK(ec, "hipStreamEndCapture");
  hipGraphExec_t ex = nullptr;
  const hipError_t ei = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
  hipGraphDestroy(g);
  E_CHECK(ei, "hipGraphInstantiate");
  e->graphs[key] = ex;
  *out = ex;
  return TI_OK;
}

int ensure_io(ti_engine* e, int in_cap, int out_cap) {
  const int B = e->c.max_batch;
  if (in_cap > e->in_cap) {
    // graphs bake the buffers in: drop them
    for (auto& g : e->graphs) hipGraphExecDestroy(g.second);
    e->graphs.clear();
    void* p = nullptr;
    TI_TRY(e->alloc(&p, (size_t)B * in_cap * sizeof(int32_t)));
    e->in_tokens = static_cast<int32_t*>(p);
    e->in_cap = in_cap;
  }
  if (out_cap > e->out_cap) {
    for (auto& g : e->graphs) hipGraphExecDestroy(g.second);
    e->graphs.clear();
    void* p = nullptr;
    TI_TRY(e->alloc(&p, (size_t)B * out_cap * sizeof(int32_t)));
    e->out_tokens = static_cast<int32_t*>(p);
    e->out_cap = out_cap;
  }
  return TI_OK;
}

// Row keys of the greedy argmax: max over each row's TI_ARGMAX_SLOTS slots.
int read_argmax(ti_engine* e, int n, std::vector<unsigned long long>& keys) {
  std::vector<unsigned long long> slots((size_t)n * TI_ARGMAX_SLOTS);
  TI_TRY(ti_memcpy_d2h(slots.data(), e->argmax, slots.size() * 8, e->s));
  keys.assign((size_t)n, 0ull);
  for (int m = 0; m < n; ++m)
    for (int j = 0; j < TI_ARGMAX_SLOTS; ++j) keys[m] = std::max(keys[m], slots[(size_t)m * TI_ARGMAX_SLOTS + j]);
  return TI_OK;
}

}  // namespace

extern "C" {

int ti_engine_create(const ti_engine_config* cfg, ti_engine** out) {
  if (!cfg || !out) return ti_set_error(TI_ERR_ARG, "ti_engine_create: null");
  *out = nullptr;
  TI_TRY(validate(*cfg));
  DeviceScope bind_(cfg->device);   // restores the caller's device after ti_init's hipSetDevice
  TI_TRY(ti_init(cfg->device));
  ti_engine* e = new ti_engine();
  e->c = *cfg;
  const ti_engine_config& c = e->c;
  auto fail = [&](int rc) { delete e; return rc; };
  if (hipStreamCreateWithFlags(&e->s, hipStreamNonBlocking) != hipSuccess)
    return fail(ti_check_hip(hipErrorUnknown, "hipStreamCreate"));
  const int B = c.max_batch, H = c.hidden, I = c.inter, V = c.vocab;
  int rc = TI_OK;
  e->layer.resize((size_t)c.layers);
  if (c.compat) {
    for (auto& L : e->layer) {
      if ((rc = e->alloc_linear(L.gu, H, I)) || (rc = e->alloc_linear(L.down, I, H))) return fail(rc);
    }
    if ((rc = e->alloc_linear(e->lm, H, V))) return fail(rc);
    if ((rc = e->alloc_t(&e->tmp, (size_t)B * I))) return fail(rc);
  } else {
    const int qd = e->qd(), kvd = e->kvd(), hd = c.head_dim;
    e->kv_stride = (int64_t)c.kv_heads * c.max_seq * hd;
    for (auto& L : e->layer) {
      if ((rc = e->alloc_linear(L.qkv, H, qd + 2 * kvd)) || (rc = e->alloc_linear(L.o, qd, H)) ||
          (rc = e->alloc_linear(L.gu, H, 2 * I)) || (rc = e->alloc_linear(L.down, I, H)) ||
          (rc = e->alloc_t(&L.attn_norm, (size_t)H)) || (rc = e->alloc_t(&L.ffn_norm, (size_t)H)) ||
          (rc = e->alloc_t(&L.kc, (size_t)B * e->kv_stride)) || (rc = e->alloc_t(&L.vc, (size_t)B * e->kv_stride)))
        return fail(rc);
      e->kv_bytes += (size_t)2 * B * e->kv_stride * 2;
    }
    if ((rc = e->alloc_linear(e->lm, H, V)) || (rc = e->alloc_t(&e->emb, (size_t)V * H)) ||
        (rc = e->alloc_t(&e->out_norm, (size_t)H)) || (rc = e->alloc_t(&e->rope_cs, (size_t)c.max_seq * hd)))
      return fail(rc);
    e->weight_bytes += (size_t)V * H * 2 + (size_t)H * 4 * (2 * c.layers + 1);
    // RoPE table with the reference formula: freq_i = 1 / theta^(2i/d), angle = pos * freq_i.
    std::vector<float> cs((size_t)c.max_seq * hd), pv((size_t)c.max_seq);
    for (int p = 0; p < c.max_seq; ++p) pv[p] = (float)p;
    if ((rc = ti_rope_table(pv.data(), c.max_seq, hd, c.rope_theta, cs.data()))) return fail(rc);
    if ((rc = ti_memcpy_h2d(e->rope_cs, cs.data(), cs.size() * 4, e->s))) return fail(rc);
    if (const char* env = getenv("TI_ATTN_PART")) e->part_on = atoi(env) != 0;
    e->splits_max = e->splits_for(1);
    e->pf_rows = (c.bits & ~TI_BITS_G32) == 4 ? TI_GEMM_MAX_ROWS : 16;   // int4 (also group-32): the tile GEMM
    // (affine group-32 runs the fused kernel only: prompt chunks of its 16 rows)
    e->rows_cap = std::max(B, e->pf_rows);
    const int R = e->rows_cap;
    const int Rp = (R + 15) / 16 * 16;   // packed operands hold whole 16-row blocks
    if ((rc = e->alloc_t(&e->q, (size_t)R * qd)) || (rc = e->alloc_t(&e->attn, (size_t)Rp * qd)) ||
        (rc = e->alloc_t(&e->act, (size_t)Rp * I)) || (rc = e->alloc_t(&e->xn, (size_t)Rp * std::max(H, I))) ||
        (rc = e->alloc(reinterpret_cast<void**>(&e->ws), ws_bytes(e))) ||
        (rc = e->alloc_t(&e->pf_ones, (size_t)e->pf_rows)) || (rc = e->alloc_t(&e->pf_zero, (size_t)1)) ||
        (rc = e->alloc_t(&e->pf_base, (size_t)e->pf_rows)) || (rc = e->alloc_t(&e->fx, (size_t)H)) ||
        (rc = e->alloc_t(&e->ss, (size_t)256)) || (rc = e->alloc_t(&e->ss_rows, (size_t)4096 * TI_FOLD_SS_ROWS)) ||
        (rc = e->alloc_t(&e->part_o, ti_qkv_attn_part_o_elems(c.heads, hd, TI_ATTN_MAX_PART_SPLITS))) ||
        (rc = e->alloc_t(&e->part_ml, ti_qkv_attn_part_ml_elems(c.heads, hd, TI_ATTN_MAX_PART_SPLITS))) ||
        (rc = e->alloc(&e->qa_xchg, ti_qkv_attn_xchg_bytes(c.heads, TI_ATTN_MAX_PART_SPLITS))))
      return fail(rc);
    if (const char* env = getenv("TI_FOLD")) e->fold_on = atoi(env) != 0;
    if (const char* env = getenv("TI_QKV_ATTN")) e->qa_on = atoi(env) != 0;
    if ((c.bits & ~TI_BITS_G32) == 4) {   // batched rows and prompt chunks: split-K tile GEMM (TI_SPLITK_MB, 0 = off)
      const char* env = getenv("TI_SPLITK_MB");
      const size_t mb = env ? (size_t)std::max(0, atoi(env)) : 64;
      if (mb && (rc = e->alloc(&e->splitk_ws, mb << 20))) return fail(rc);
      e->splitk_bytes = mb << 20;
    }
    std::vector<int32_t> ones(e->pf_rows, 1);
    if ((rc = ti_memcpy_h2d(e->pf_ones, ones.data(), ones.size() * 4, e->s)) || (rc = ti_memset(e->pf_zero, 0, 4, e->s)))
      return fail(rc);
    std::vector<uint16_t*> tab;
    for (auto& L : e->layer) tab.push_back(L.kc);
    for (auto& L : e->layer) tab.push_back(L.vc);
    if ((rc = e->alloc_t(&e->kv_tab, tab.size())) || (rc = ti_memcpy_h2d(e->kv_tab, tab.data(), tab.size() * sizeof(void*), e->s)))
      return fail(rc);
  }
  const int R = std::max(B, e->rows_cap);
  if ((rc = e->alloc_t(&e->h, (size_t)R * H)) || (rc = e->alloc_t(&e->h_last, (size_t)B * H)) ||
      (rc = e->alloc_t(&e->logits, (size_t)B * V)) ||
      (rc = e->alloc_t(&e->argmax, (size_t)R * TI_ARGMAX_SLOTS)) || (rc = e->alloc_t(&e->pos, (size_t)R)) ||
      (rc = e->alloc_t(&e->base_pos, (size_t)B)) || (rc = e->alloc_t(&e->step_ctr, (size_t)1)) ||
      (rc = e->alloc_t(&e->n_in, (size_t)B)) || (rc = ensure_io(e, 8, 8)))
    return fail(rc);
  if (hipStreamSynchronize(e->s) != hipSuccess) return fail(ti_check_hip(hipErrorUnknown, "hipStreamSynchronize"));
  *out = e;
  return TI_OK;
}

int ti_engine_destroy(ti_engine* e) {
  if (e) {
    DeviceScope bind_(e);
    hipStreamSynchronize(e->s);
    delete e;
  }
  return TI_OK;
}

int ti_engine_get_stream(ti_engine* e, void** stream) {
  if (!e || !stream) return ti_set_error(TI_ERR_ARG, "ti_engine_get_stream: null");
  DeviceScope bind_(e);
  *stream = (void*)e->s;
  return TI_OK;
}

int ti_engine_memory(ti_engine* e, size_t* wb, size_t* kb) {
  if (!e) return ti_set_error(TI_ERR_ARG, "ti_engine_memory: null");
  DeviceScope bind_(e);
  if (wb) *wb = e->weight_bytes;
  if (kb) *kb = e->kv_bytes;
  return TI_OK;
}

int ti_engine_set_tensor(ti_engine* e, int slot, int layer, const float* data, int scale_mode) {
  if (!e || !data) return ti_set_error(TI_ERR_ARG, "ti_engine_set_tensor: null");
  DeviceScope bind_(e);
  const ti_engine_config& c = e->c;
  const int H = c.hidden, I = c.inter, V = c.vocab;
  const bool per_layer = slot <= TI_W_DOWN || slot == TI_V_ATTN_NORM || slot == TI_V_FFN_NORM;
  if (per_layer && (layer < 0 || layer >= c.layers))
    return ti_set_error(TI_ERR_ARG, "ti_engine_set_tensor: layer %d of %d", layer, c.layers);

  if (c.compat) {
    DevLinear* L = nullptr;
    size_t n = 0;
    switch (slot) {
      case TI_W_UP: L = &e->layer[layer].gu; n = (size_t)H * I; break;
      case TI_W_DOWN: L = &e->layer[layer].down; n = (size_t)I * H; break;
      case TI_W_LM_HEAD: L = &e->lm; n = (size_t)H * V; break;
      case TI_W_Q: case TI_W_K: case TI_W_V: case TI_E_EMBED: return TI_OK;  // unused by the compat path
      default: return ti_set_error(TI_ERR_UNSUPPORTED, "ti_engine_set_tensor: slot %d not part of the compat model", slot);
    }
    return ti_memcpy_h2d(L->f32, data, n * 4, e->s);
  }

  if (slot == TI_V_ATTN_NORM || slot == TI_V_FFN_NORM || slot == TI_V_OUT_NORM) {
    float* dst = slot == TI_V_OUT_NORM ? e->out_norm
                                       : (slot == TI_V_ATTN_NORM ? e->layer[layer].attn_norm : e->layer[layer].ffn_norm);
    return ti_memcpy_h2d(dst, data, (size_t)H * 4, e->s);
  }
  if (slot == TI_E_EMBED) {
    std::vector<uint16_t> hb((size_t)V * H);
    for (size_t i = 0; i < hb.size(); ++i) hb[i] = host_half(data[i]);
    return ti_memcpy_h2d(e->emb, hb.data(), hb.size() * 2, e->s);
  }
  const int qd = e->qd(), kvd = e->kvd();
  DevLinear* L = nullptr;
  int K = 0, Nsrc = 0, map = TI_ROWS_CONCAT, off = 0;
  switch (slot) {
    case TI_W_Q: L = &e->layer[layer].qkv; K = H; Nsrc = qd; off = 0; break;
    case TI_W_K: L = &e->layer[layer].qkv; K = H; Nsrc = kvd; off = qd; break;
    case TI_W_V: L = &e->layer[layer].qkv; K = H; Nsrc = kvd; off = qd + kvd; break;
    case TI_W_O: L = &e->layer[layer].o; K = qd; Nsrc = H; break;
    case TI_W_GATE: L = &e->layer[layer].gu; K = H; Nsrc = I; map = TI_ROWS_INTERLEAVE8; off = 0; break;
    case TI_W_UP: L = &e->layer[layer].gu; K = H; Nsrc = I; map = TI_ROWS_INTERLEAVE8; off = 8; break;
    case TI_W_DOWN: L = &e->layer[layer].down; K = I; Nsrc = H; break;
    case TI_W_LM_HEAD: L = &e->lm; K = H; Nsrc = V; break;
    default: return ti_set_error(TI_ERR_ARG, "ti_engine_set_tensor: slot %d", slot);
  }
  // read-modify-write of the fused buffer: the packer only touches this part's rows
  const size_t tb = ti_wpack_tile_bytes(c.bits, L->K, L->N), sb = ti_wpack_scale_bytes(c.bits, L->K, L->N);
  std::vector<uint8_t> th(tb);
  std::vector<uint16_t> sh(sb / 2 + 1);
  TI_TRY(ti_memcpy_d2h(th.data(), L->tiles, tb, e->s));
  if (sb) TI_TRY(ti_memcpy_d2h(sh.data(), L->scales, sb, e->s));
  TI_TRY(ti_wpack_host(data, K, Nsrc, L->N, c.bits, scale_mode, map, off, th.data(), sb ? sh.data() : nullptr));
  TI_TRY(ti_memcpy_h2d(L->tiles, th.data(), tb, e->s));
  if (sb) TI_TRY(ti_memcpy_h2d(L->scales, sh.data(), sb, e->s));
  return TI_OK;
}

// Exact group-32 weights: Q4_0 / Q8_0 blocks (q int8, d) or, with m, Q4_1 blocks (q 0..15, d, m;
// TI_BITS_AFF engines), packed without re-quantization (ti_wpack_q_host / ti_wpack_q1_host).
static int set_tensor_blocks(ti_engine* e, int slot, int layer, const void* q, const uint16_t* d, const uint16_t* m) {
  const char* fn = m ? "ti_engine_set_tensor_q1" : "ti_engine_set_tensor_q";
  if (!e || !q || !d) return ti_set_error(TI_ERR_ARG, "%s: null", fn);
  DeviceScope bind_(e);
  const ti_engine_config& c = e->c;
  if (!(c.bits & TI_BITS_G32)) return ti_set_error(TI_ERR_ARG, "%s: engine bits %d lack TI_BITS_G32", fn, c.bits);
  if (((c.bits & TI_BITS_AFF) != 0) != (m != nullptr))
    return ti_set_error(TI_ERR_ARG, "%s: engine bits %d (%s blocks expected)", fn, c.bits,
                        (c.bits & TI_BITS_AFF) ? "affine Q4_1" : "Q4_0 / Q8_0");
  if (layer < 0 || (slot <= TI_W_DOWN && layer >= c.layers)) return ti_set_error(TI_ERR_ARG, "%s: layer %d", fn, layer);
  const int H = c.hidden, I = c.inter, V = c.vocab, qd = e->qd(), kvd = e->kvd();
  DevLinear* L = nullptr;
  int K = 0, Nsrc = 0, map = TI_ROWS_CONCAT, off = 0;
  switch (slot) {
    case TI_W_Q: L = &e->layer[layer].qkv; K = H; Nsrc = qd; off = 0; break;
    case TI_W_K: L = &e->layer[layer].qkv; K = H; Nsrc = kvd; off = qd; break;
    case TI_W_V: L = &e->layer[layer].qkv; K = H; Nsrc = kvd; off = qd + kvd; break;
    case TI_W_O: L = &e->layer[layer].o; K = qd; Nsrc = H; break;
    case TI_W_GATE: L = &e->layer[layer].gu; K = H; Nsrc = I; map = TI_ROWS_INTERLEAVE8; off = 0; break;
    case TI_W_UP: L = &e->layer[layer].gu; K = H; Nsrc = I; map = TI_ROWS_INTERLEAVE8; off = 8; break;
    case TI_W_DOWN: L = &e->layer[layer].down; K = I; Nsrc = H; break;
    case TI_W_LM_HEAD: L = &e->lm; K = H; Nsrc = V; break;
    default: return ti_set_error(TI_ERR_ARG, "%s: slot %d is not a linear weight", fn, slot);
  }
  const size_t tb = ti_wpack_tile_bytes(c.bits, L->K, L->N), sb = ti_wpack_scale_bytes(c.bits, L->K, L->N);
  std::vector<uint8_t> th(tb);
  std::vector<uint16_t> sh(sb / 2 + 1);
  TI_TRY(ti_memcpy_d2h(th.data(), L->tiles, tb, e->s));
  TI_TRY(ti_memcpy_d2h(sh.data(), L->scales, sb, e->s));
  if (m)
    TI_TRY(ti_wpack_q1_host(static_cast<const uint8_t*>(q), d, m, K, Nsrc, L->N, map, off, th.data(), sh.data()));
  else
    TI_TRY(ti_wpack_q_host(static_cast<const int8_t*>(q), d, K, Nsrc, L->N, c.bits, map, off, th.data(), sh.data()));
  TI_TRY(ti_memcpy_h2d(L->tiles, th.data(), tb, e->s));
  TI_TRY(ti_memcpy_h2d(L->scales, sh.data(), sb, e->s));
  return ti_stream_sync(e->s);
}

int ti_engine_set_tensor_q(ti_engine* e, int slot, int layer, const int8_t* q, const uint16_t* d) {
  return set_tensor_blocks(e, slot, layer, q, d, nullptr);
}

int ti_engine_set_tensor_q1(ti_engine* e, int slot, int layer, const uint8_t* q, const uint16_t* d, const uint16_t* m) {
  if (!m) return ti_set_error(TI_ERR_ARG, "ti_engine_set_tensor_q1: null");
  return set_tensor_blocks(e, slot, layer, q, d, m);
}

int ti_engine_synth(ti_engine* e, uint64_t seed, float norm_jitter) {
  if (!e) return ti_set_error(TI_ERR_ARG, "ti_engine_synth: null");
  DeviceScope bind_(e);
  const ti_engine_config& c = e->c;
  if (c.compat) return ti_set_error(TI_ERR_UNSUPPORTED, "ti_engine_synth: compat engines take the reference model");
  if (c.bits & TI_BITS_G32)
    return ti_set_error(TI_ERR_UNSUPPORTED, "ti_engine_synth: group-32 engines take their weights from ti_engine_set_tensor[_q]");
  const int H = c.hidden, I = c.inter, V = c.vocab, qd = e->qd(), kvd = e->kvd(), b = c.bits;
  for (int l = 0; l < c.layers; ++l) {
    DevLayer& L = e->layer[l];
    const int nq = qd + 2 * kvd;
    TI_TRY(ti_wsynth_device(seed, tid_layer(l, TL_Q), H, qd, nq, b, TI_ROWS_CONCAT, 0, L.qkv.tiles, L.qkv.scales, e->s));
    TI_TRY(ti_wsynth_device(seed, tid_layer(l, TL_K), H, kvd, nq, b, TI_ROWS_CONCAT, qd, L.qkv.tiles, L.qkv.scales, e->s));
    TI_TRY(ti_wsynth_device(seed, tid_layer(l, TL_V), H, kvd, nq, b, TI_ROWS_CONCAT, qd + kvd, L.qkv.tiles, L.qkv.scales, e->s));
    TI_TRY(ti_wsynth_device(seed, tid_layer(l, TL_O), qd, H, H, b, TI_ROWS_CONCAT, 0, L.o.tiles, L.o.scales, e->s));
    TI_TRY(ti_wsynth_device(seed, tid_layer(l, TL_G), H, I, 2 * I, b, TI_ROWS_INTERLEAVE8, 0, L.gu.tiles, L.gu.scales, e->s));
    TI_TRY(ti_wsynth_device(seed, tid_layer(l, TL_U), H, I, 2 * I, b, TI_ROWS_INTERLEAVE8, 8, L.gu.tiles, L.gu.scales, e->s));
    TI_TRY(ti_wsynth_device(seed, tid_layer(l, TL_D), I, H, H, b, TI_ROWS_CONCAT, 0, L.down.tiles, L.down.scales, e->s));
    TI_TRY(ti_fill_uniform_f32(seed, tid_layer(l, TL_ATTN_NORM), (uint64_t)H, norm_jitter, 1.0f, L.attn_norm, e->s));
    TI_TRY(ti_fill_uniform_f32(seed, tid_layer(l, TL_FFN_NORM), (uint64_t)H, norm_jitter, 1.0f, L.ffn_norm, e->s));
  }
  TI_TRY(ti_wsynth_device(seed, kTidLmHead, H, V, V, b, TI_ROWS_CONCAT, 0, e->lm.tiles, e->lm.scales, e->s));
  TI_TRY(ti_fill_uniform_f32(seed, kTidOutNorm, (uint64_t)H, norm_jitter, 1.0f, e->out_norm, e->s));
  TI_TRY(ti_fill_uniform_f16(seed, kTidEmb, (uint64_t)V * H, 0.02f, e->emb, e->s));
  return ti_stream_sync(e->s);
}

int ti_engine_fill_kv(ti_engine* e, int stream, int n, uint64_t seed) {
  if (!e || e->c.compat) return ti_set_error(TI_ERR_ARG, "ti_engine_fill_kv: no KV cache");
  DeviceScope bind_(e);
  if (stream < 0 || stream >= e->c.max_batch || n < 0 || n > e->c.max_seq)
    return ti_set_error(TI_ERR_ARG, "ti_engine_fill_kv: stream %d n %d", stream, n);
  for (int l = 0; l < e->c.layers; ++l) {
    DevLayer& L = e->layer[l];
    TI_TRY(ti_fill_kv_uniform(seed, tid_kv(l, 0), n, e->c.kv_heads, e->c.head_dim, e->c.max_seq,
                              L.kc + (size_t)stream * e->kv_stride, e->s));
    TI_TRY(ti_fill_kv_uniform(seed, tid_kv(l, 1), n, e->c.kv_heads, e->c.head_dim, e->c.max_seq,
                              L.vc + (size_t)stream * e->kv_stride, e->s));
  }
  return ti_stream_sync(e->s);
}

int ti_engine_generate(ti_engine* e, int n, const int32_t* prompts, const int32_t* lens, int stride,
                       const int32_t* start_pos, int max_new, int32_t* out_tokens, float* last_logits) {
  if (!e || !prompts || !lens || !out_tokens) return ti_set_error(TI_ERR_ARG, "ti_engine_generate: null");
  DeviceScope bind_(e);
  const ti_engine_config& c = e->c;
  if (c.compat) return ti_set_error(TI_ERR_UNSUPPORTED, "ti_engine_generate: use ti_engine_compat_step for compat engines");
  if (n < 1 || n > c.max_batch || max_new < 1) return ti_set_error(TI_ERR_ARG, "ti_engine_generate: n=%d max_new=%d", n, max_new);
  int nin_max = 0;
  std::vector<int32_t> nin(n), base(n, 0);
  for (int m = 0; m < n; ++m) {
    if (lens[m] < 1 || lens[m] > stride) return ti_set_error(TI_ERR_ARG, "ti_engine_generate: prompt length %d", lens[m]);
    nin[m] = lens[m];
    nin_max = std::max(nin_max, lens[m]);
    if (start_pos) base[m] = start_pos[m];
  }
  const int steps = nin_max + max_new - 1;
  for (int m = 0; m < n; ++m)
    if (base[m] < 0 || base[m] + steps > c.max_seq)
      return ti_set_error(TI_ERR_ARG, "ti_engine_generate: stream %d needs %d KV slots > max_seq %d", m, base[m] + steps,
                          c.max_seq);
  TI_TRY(ensure_io(e, stride, std::max(steps, 1)));
  std::vector<int32_t> in((size_t)n * e->in_cap, 0);
  for (int m = 0; m < n; ++m) std::memcpy(&in[(size_t)m * e->in_cap], prompts + (size_t)m * stride, (size_t)lens[m] * 4);
  TI_TRY(ti_memcpy_h2d(e->in_tokens, in.data(), in.size() * 4, e->s));
  TI_TRY(ti_memcpy_h2d(e->n_in, nin.data(), (size_t)n * 4, e->s));
  TI_TRY(ti_memcpy_h2d(e->base_pos, base.data(), (size_t)n * 4, e->s));
  // All but the last prompt token of the shortest prompt go through prefill; the decode loop
  // then starts at that step (same positions, same token feed, same outputs).  Greedy streams
  // whose prompts have one length: the last prompt token is a prefill row too, and the final
  // rms_norm + lm_head + argmax run on each stream's last hidden row (the reference's forward_pass
  // computes the last position's logits the same way, inference_engine.cpp:1429-1491), so the
  // first generated token costs one lm_head GEMM, not a decode step over every layer; the decode
  // loop starts at the step that feeds it.
  int s0 = 0;
  if (e->pf_rows > 0) {
    const int lmin = *std::min_element(nin.begin(), nin.end());
    const bool one_len = *std::max_element(nin.begin(), nin.end()) == lmin;
    const bool last_in_prefill = one_len && !e->samp_on && lmin >= 2 && prefill_logits_on();
    s0 = last_in_prefill ? lmin : lmin - 1;
    int last_rows = 0;
    for (int m = 0; m < n; ++m) {
      for (int t0 = 0; t0 < s0; t0 += e->pf_rows) {
        last_rows = std::min(e->pf_rows, s0 - t0);
        TI_TRY(enqueue_prefill(e, m, t0, last_rows, base[m]));
      }
      if (last_in_prefill && n > 1)   // (the next stream's chunks reuse h)
        TI_TRY(ti_memcpy_d2d(e->h_last + (size_t)m * c.hidden, e->h + (size_t)(last_rows - 1) * c.hidden,
                             (size_t)c.hidden * 4, e->s));
    }
    if (last_in_prefill) {
      // one stream: its row in place, argmax slots cleared by the chunk's step_begin
      if (n > 1) TI_TRY(ti_memset(e->argmax, 0, (size_t)n * TI_ARGMAX_SLOTS * 8, e->s));
      ti_epilogue el{};
      el.kind = TI_EPI_LOGITS_ARGMAX;
      el.ldo = c.vocab;
      el.out = e->logits;
      el.argmax = e->argmax;
      const float* x = n > 1 ? e->h_last : e->h + (size_t)(last_rows - 1) * c.hidden;
      TI_TRY(gemm_rows(e, e->lm, n, x, TI_X_F32_RMSNORM, c.hidden, e->out_norm, el, 4, false));
    }
  }
  TI_TRY(ti_memcpy_h2d(e->step_ctr, &s0, 4, e->s));
  std::vector<int32_t> outd((size_t)n * e->out_cap);
  std::vector<unsigned long long> am;
  // generated token t of stream m once `ran` steps have run: the step feed record holds every
  // token but the last, which is still in the argmax slots
  auto token_at = [&](int m, int t, int ran) -> int32_t {
    const int produced = ran - nin[m] + 1;
    if (t < produced - 1) return outd[(size_t)m * e->out_cap + t];
    if (t == produced - 1) return (int32_t)(0xFFFFFFFFu - (uint32_t)(am[m] & 0xFFFFFFFFull));
    return -1;
  };
  int ran = steps;
  if (e->stop_token < 0) {
    TI_TRY(run_steps(e, n, 1, steps - s0));
    TI_TRY(ti_stream_sync(e->s));
    TI_TRY(ti_memcpy_d2h(outd.data(), e->out_tokens, outd.size() * 4, e->s));
    TI_TRY(read_argmax(e, n, am));
  } else {
    // chunks of 4, 8, 16, 32, then 64 steps; after each, every stream's new tokens are read back
    // (one small copy) and the loop ends once each has emitted the stop token
    ran = s0;
    bool all = false;
    auto read_back = [&]() -> int {   // every stream's tokens so far; all = each stopped or complete
      TI_TRY(ti_memcpy_d2h(outd.data(), e->out_tokens, outd.size() * 4, e->s));
      TI_TRY(read_argmax(e, n, am));   // (synchronises the stream)
      all = true;
      for (int m = 0; m < n && all; ++m) {
        bool hit = false;
        const int produced = ran - nin[m] + 1;
        for (int t = 0; t < std::min(produced, max_new) && !hit; ++t) hit = token_at(m, t, ran) == e->stop_token;
        all = hit || produced >= max_new;
      }
      return TI_OK;
    };
    // the prefill's last rows gave every stream its first token: it may already be the stop
    if (ran >= nin_max) TI_TRY(read_back());
    for (int chunk = 4; ran < steps && !all; chunk = std::min(chunk * 2, 64)) {
      const int S = std::min(chunk, steps - ran);
      TI_TRY(run_steps(e, n, 1, S));
      ran += S;
      TI_TRY(read_back());
    }
  }
  for (int m = 0; m < n; ++m) {
    bool stopped = false;
    for (int t = 0; t < max_new; ++t) {
      const int32_t tok = stopped ? -1 : token_at(m, t, ran);
      stopped = stopped || (e->stop_token >= 0 && tok == e->stop_token);
      out_tokens[(size_t)m * max_new + t] = tok;
    }
  }
  if (last_logits) TI_TRY(ti_memcpy_d2h(last_logits, e->logits, (size_t)n * c.vocab * 4, e->s));
  if (n == 1) TI_TRY(qa_fault_check(e));
  return TI_OK;
}

int ti_engine_generate_sampled(ti_engine* e, int n, const int32_t* prompts, const int32_t* lens, int stride,
                               const int32_t* start_pos, int max_new, float temperature, int top_k, float top_p,
                               const float* draws, int32_t* out_tokens, float* out_logprobs) {
  if (!e || !draws) return ti_set_error(TI_ERR_ARG, "ti_engine_generate_sampled: null");
  DeviceScope bind_(e);
  const ti_engine_config& c = e->c;
  if (c.compat) return ti_set_error(TI_ERR_UNSUPPORTED, "ti_engine_generate_sampled: compat engine");
  if (n < 1 || n > c.max_batch || max_new < 1) return ti_set_error(TI_ERR_ARG, "ti_engine_generate_sampled: n=%d max_new=%d", n, max_new);
  if (top_k < 1 || top_k > c.vocab)
    return ti_set_error(TI_ERR_ARG, "ti_engine_generate_sampled: top_k %d not in [1, vocab %d]", top_k, c.vocab);
  auto drop_graphs = [&]() -> int {
    TI_TRY(ti_stream_sync(e->s));
    for (auto& g : e->graphs) hipGraphExecDestroy(g.second);
    e->graphs.clear();
    return TI_OK;
  };
  if (max_new > e->draw_cap) {   // graphs bake the buffers in
    TI_TRY(drop_graphs());
    const int cap = std::max(max_new, 64);
    TI_TRY(e->alloc_t(&e->draws, (size_t)c.max_batch * cap));
    TI_TRY(e->alloc_t(&e->lps, (size_t)c.max_batch * cap));
    e->draw_cap = cap;
  }
  // top_k above TI_SAMPLE_MAX_K: the sampler's survivors live in an HBM workspace (per stream)
  const size_t wsb = ti_sample_workspace_bytes(c.vocab, top_k) * (size_t)c.max_batch;
  if (wsb > e->samp_ws_bytes) {
    TI_TRY(drop_graphs());
    void* p = nullptr;
    TI_TRY(e->alloc(&p, wsb));
    e->samp_ws = p;
    e->samp_ws_bytes = wsb;
  }
  if (e->samp_t != temperature || e->samp_k != top_k || e->samp_p != top_p) {   // kernel arguments of the graph
    TI_TRY(drop_graphs());
    e->samp_t = temperature;
    e->samp_k = top_k;
    e->samp_p = top_p;
  }
  std::vector<float> d((size_t)n * e->draw_cap, 0.5f);
  for (int m = 0; m < n; ++m) std::memcpy(&d[(size_t)m * e->draw_cap], draws + (size_t)m * max_new, (size_t)max_new * 4);
  TI_TRY(ti_memcpy_h2d(e->draws, d.data(), d.size() * 4, e->s));
  e->samp_on = true;
  const int rc = ti_engine_generate(e, n, prompts, lens, stride, start_pos, max_new, out_tokens, nullptr);
  e->samp_on = false;
  TI_TRY(rc);
  if (out_logprobs) {
    std::vector<float> lp((size_t)n * e->draw_cap);
    TI_TRY(ti_memcpy_d2h(lp.data(), e->lps, lp.size() * 4, e->s));
    for (int m = 0; m < n; ++m)
      for (int t = 0; t < max_new; ++t)
        out_logprobs[(size_t)m * max_new + t] = out_tokens[(size_t)m * max_new + t] < 0 ? 0.0f : lp[(size_t)m * e->draw_cap + t];
  }
  return TI_OK;
}

// ------------------------------------------------------------------------- beam search
// InferenceEngine::generate_beam_search / beam_search_decode (inference_engine.cpp:830-871,
// 1912-2069) with the reference's control flow, scoring and container orders (max-heap on
// log_prob, std::sort on probabilities and normalised scores) and its helpers softmax /
// apply_top_k_filtering / apply_top_p_filtering (:1798-1910).
// Where the reference recomputes every candidate from scratch with a full forward pass (:1961),
// here every live beam owns a stream slot whose KV cache holds its sequence: one batched decode
// step per expansion round gives all beams' next-token logits at once, and a beam that forks
// copies its parent's cache prefix into a free slot (ti_kv_copy_slots) -- the first child
// keeps the parent's slot.  One deviation from the reference's numbers: the reference reads
// seq_len x vocab "logits" of its full-sequence forward pass as one distribution; here a
// candidate's next-token distribution is its last position's logits.
}  // extern "C" (the helpers below are C++)

namespace {
struct Beam {
  std::vector<int32_t> tokens;
  float log_prob = 0.0f;
  float normalized_score = 0.0f;
  bool finished = false;
  int slot = -1;      // stream slot whose cache holds tokens[0 .. size-2] (its parent's, until forked)
};

std::vector<float> beam_softmax(const std::vector<float>& lg) {
  std::vector<float> p(lg.size());
  const float mx = *std::max_element(lg.begin(), lg.end());
  float sum = 0.0f;
  for (size_t i = 0; i < lg.size(); ++i) {
    p[i] = std::exp(lg[i] - mx);
    sum += p[i];
  }
  if (sum > 0.0f)
    for (auto& x : p) x /= sum;
  return p;
}

std::vector<float> beam_top_k(const std::vector<float>& probs, size_t k) {
  std::vector<float> f = probs;
  if (k >= probs.size()) return f;
  std::vector<std::pair<float, size_t>> pi;
  for (size_t i = 0; i < probs.size(); ++i) pi.emplace_back(probs[i], i);
  std::sort(pi.begin(), pi.end(), [](const auto& a, const auto& b) { return a.first > b.first; });
  for (size_t i = k; i < pi.size(); ++i) f[pi[i].second] = 0.0f;
  float sum = 0.0f;
  for (float x : f) sum += x;
  if (sum > 0.0f)
    for (auto& x : f) x /= sum;
  return f;
}

std::vector<float> beam_top_p(const std::vector<float>& probs, float p) {
  std::vector<float> f = probs;
  if (p >= 1.0f) return f;
  std::vector<std::pair<float, size_t>> pi;
  for (size_t i = 0; i < probs.size(); ++i) pi.emplace_back(probs[i], i);
  std::sort(pi.begin(), pi.end(), [](const auto& a, const auto& b) { return a.first > b.first; });
  float cum = 0.0f;
  std::vector<bool> in(probs.size(), false);
  for (const auto& pr : pi) {
    cum += pr.first;
    in[pr.second] = true;
    if (cum >= p) break;
  }
  for (size_t i = 0; i < probs.size(); ++i)
    if (!in[i]) f[i] = 0.0f;
  float sum = 0.0f;
  for (float x : f) sum += x;
  if (sum > 0.0f)
    for (auto& x : f) x /= sum;
  return f;
}

// Copy slot `src`'s cache positions [0, n) into slot `dst`, every layer, K and V.
int fork_slot(ti_engine* e, int src, int dst, int n) {
  const ti_engine_config& c = e->c;
  return ti_kv_copy_slots(e->kv_tab, 2 * c.layers, (int64_t)src * e->kv_stride, (int64_t)dst * e->kv_stride,
                          c.kv_heads, (int64_t)c.max_seq * c.head_dim, (int64_t)n * c.head_dim, e->s);
}
}  // namespace

extern "C" {

int ti_engine_beam_search(ti_engine* e, const int32_t* prompt, int len, int max_new, int beam_size, float temperature,
                          int top_k, float top_p, float length_penalty, int eos, int32_t* out_tokens,
                          float* out_log_prob, float* out_score, int32_t* out_finished, int* out_count) {
  if (!e || !prompt || !out_count || len < 1 || max_new < 0 || (max_new > 0 && !out_tokens))
    return ti_set_error(TI_ERR_ARG, "ti_engine_beam_search: bad arguments");
  DeviceScope bind_(e);
  if (beam_size < 1) return ti_set_error(TI_ERR_ARG, "ti_engine_beam_search: Beam size must be greater than 0");
  const ti_engine_config& c = e->c;
  if (c.compat) return ti_set_error(TI_ERR_UNSUPPORTED, "ti_engine_beam_search: compat engine");
  if (len + max_new - 1 > c.max_seq)
    return ti_set_error(TI_ERR_ARG, "ti_engine_beam_search: %d + %d tokens exceed max_seq %d", len, max_new, c.max_seq);
  // More beams than stream slots: every candidate's next-token logits come from a full pass over
  // its sequence in slot 0 (prefill + one step), as the reference recomputes each candidate
  // (:1961) -- slower, same decisions.
  const bool recompute = beam_size > c.max_batch;
  const size_t V = (size_t)c.vocab;
  std::vector<float> logits((size_t)std::max(c.max_batch, beam_size) * V);
  auto cmp = [](const Beam& a, const Beam& b) { return a.log_prob < b.log_prob; };
  std::priority_queue<Beam, std::vector<Beam>, decltype(cmp)> beam(cmp);
  Beam init;
  init.tokens.assign(prompt, prompt + len);
  init.slot = 0;
  beam.push(init);
  std::vector<Beam> done;
  const size_t bs = (size_t)beam_size, target = (size_t)len + (size_t)max_new;
  std::vector<int32_t> feed(c.max_batch), pos(c.max_batch);
  for (int step = 0; step < max_new; ++step) {
    std::vector<Beam> cur;
    while (!beam.empty()) {
      cur.push_back(beam.top());
      beam.pop();
    }
    if (cur.empty()) break;
    // next-token logits of every live beam: the prompt's prefill + first step into slot 0, then
    // one batched decode step over the slots (each feeds its last token at its own position;
    // slots no beam owns decode a dummy token into their own, unused cache)
    if (recompute) {
      for (size_t i = 0; i < cur.size(); ++i) {
        cur[i].slot = (int)i;   // row of `logits`
        const int n = (int)cur[i].tokens.size();
        int32_t tok = 0;
        TI_TRY(ti_engine_generate(e, 1, cur[i].tokens.data(), &n, n, nullptr, 1, &tok, logits.data() + i * V));
      }
    } else if (step == 0) {
      int32_t tok = 0;
      TI_TRY(ti_engine_generate(e, 1, prompt, &len, len, nullptr, 1, &tok, logits.data()));
    } else {
      int M = 0;
      for (const auto& cand : cur) M = std::max(M, cand.slot + 1);
      std::fill(feed.begin(), feed.end(), 0);
      std::fill(pos.begin(), pos.end(), 0);
      for (const auto& cand : cur) {
        feed[cand.slot] = cand.tokens.back();
        pos[cand.slot] = (int32_t)cand.tokens.size() - 1;
      }
      TI_TRY(ti_engine_step(e, M, feed.data(), pos.data(), logits.data()));
    }
    std::vector<Beam> next;
    for (const auto& cand : cur) {
      if (cand.finished) {
        done.push_back(cand);
        continue;
      }
      std::vector<float> lg(logits.begin() + (size_t)cand.slot * V, logits.begin() + (size_t)(cand.slot + 1) * V);
      if (temperature != 1.0f)
        for (auto& x : lg) x /= temperature;
      std::vector<float> probs = beam_softmax(lg);
      if (top_k > 0 && (size_t)top_k < probs.size()) probs = beam_top_k(probs, (size_t)top_k);
      if (top_p < 1.0f) probs = beam_top_p(probs, top_p);
      std::vector<std::pair<float, int>> pt;
      for (size_t i = 0; i < probs.size(); ++i)
        if (probs[i] > 0.0f) pt.emplace_back(probs[i], (int)i);
      std::sort(pt.begin(), pt.end(), [](const auto& a, const auto& b) { return a.first > b.first; });
      const size_t ex = std::min(bs, pt.size());
      for (size_t i = 0; i < ex; ++i) {
        if (pt[i].first <= 0.0f) continue;
        Beam nb = cand;
        nb.tokens.push_back(pt[i].second);
        nb.log_prob += std::log(pt[i].first);
        nb.finished = pt[i].second == eos || nb.tokens.size() >= target;
        next.push_back(std::move(nb));
      }
    }
    for (auto& b : next) b.normalized_score = b.log_prob / std::pow((float)b.tokens.size(), length_penalty);
    std::sort(next.begin(), next.end(), [](const Beam& a, const Beam& b) { return a.normalized_score > b.normalized_score; });
    const size_t keep = std::min(bs, next.size());
    // slots of the surviving beams: the first survivor of each parent keeps the parent's slot,
    // the others fork the parent's cache (positions 0 .. parent length - 1) into a free slot
    std::vector<char> owned(c.max_batch, 0);
    std::vector<size_t> forks;
    for (size_t i = 0; i < (recompute ? 0 : keep); ++i) {
      if (next[i].finished) continue;
      if (!owned[next[i].slot]) owned[next[i].slot] = 1;
      else forks.push_back(i);
    }
    int free_slot = 0;
    for (size_t i : forks) {
      while (owned[free_slot]) ++free_slot;   // a free slot exists: at most beam_size <= max_batch survivors
      TI_TRY(fork_slot(e, next[i].slot, free_slot, (int)next[i].tokens.size() - 1));
      owned[free_slot] = 1;
      next[i].slot = free_slot;
    }
    for (size_t i = 0; i < keep; ++i) {
      if (next[i].finished) done.push_back(next[i]);
      else beam.push(next[i]);
    }
    if (done.size() >= bs) break;
  }
  while (!beam.empty()) {
    Beam b = beam.top();
    beam.pop();
    b.finished = true;
    done.push_back(b);
  }
  std::sort(done.begin(), done.end(), [](const Beam& a, const Beam& b) { return a.normalized_score > b.normalized_score; });
  const size_t nres = std::min(bs, done.size());
  *out_count = (int)nres;
  for (size_t r = 0; r < nres; ++r) {
    const Beam& b = done[r];
    for (int t = 0; t < max_new; ++t) {
      const size_t j = (size_t)len + (size_t)t;
      out_tokens[r * max_new + t] = j < b.tokens.size() ? b.tokens[j] : -1;
    }
    if (out_log_prob) out_log_prob[r] = b.log_prob;
    if (out_score) out_score[r] = b.normalized_score;
    if (out_finished) out_finished[r] = b.finished ? 1 : 0;
  }
  return TI_OK;
}

// ------------------------------------------------------------------ continuous batching
// Requests flow through the engine's max_batch stream slots.  Every chunk of the device loop
// starts with each slot feeding one token at its own position (step_ctr 0, n_in 1): a
// continuing request its last generated token, a newly admitted one the last token of its
// prompt, whose other tokens were prefilled into the slot's KV (enqueue_prefill) just before.
// After the chunk the slots' new tokens are read back (the step feed record + the last
// argmax); finished requests (EOS, max_new) free their slot for the next queued request.
int ti_engine_serve(ti_engine* e, int n_req, const int32_t* prompts, const int32_t* offsets, int max_new, int eos,
                    int chunk, int32_t* out_tokens, int32_t* out_len) {
  if (!e || !prompts || !offsets || !out_tokens || !out_len || n_req < 1 || max_new < 1 || chunk < 1)
    return ti_set_error(TI_ERR_ARG, "ti_engine_serve: bad arguments");
  DeviceScope bind_(e);
  const ti_engine_config& c = e->c;
  if (c.compat) return ti_set_error(TI_ERR_UNSUPPORTED, "ti_engine_serve: compat engine");
  const int B = c.max_batch;
  const int pf = e->pf_rows > 0 ? e->pf_rows : std::min(e->rows_cap, (c.bits & ~TI_BITS_G32) == 4 ? TI_GEMM_MAX_ROWS : 16);
  int max_len = 1;
  for (int r = 0; r < n_req; ++r) {
    const int L = offsets[r + 1] - offsets[r];
    if (L < 1 || L + max_new - 1 > c.max_seq)
      return ti_set_error(TI_ERR_ARG, "ti_engine_serve: request %d: %d prompt + %d new tokens exceed max_seq %d", r, L,
                          max_new, c.max_seq);
    max_len = std::max(max_len, L);
  }
  TI_TRY(ensure_io(e, max_len, chunk + 1));
  for (int i = 0; i < n_req * max_new; ++i) out_tokens[i] = -1;
  for (int r = 0; r < n_req; ++r) out_len[r] = 0;
  std::vector<int> slot_req(B, -1), slot_pos(B, 0), slot_tok(B, 0);
  std::vector<int32_t> in((size_t)B * e->in_cap, 0), nin(B, 1), base(B, 0), outd((size_t)B * e->out_cap);
  std::vector<unsigned long long> am;
  int next = 0, live = 0;
  for (;;) {
    // admit queued requests into free slots: prefill all but the prompt's last token
    std::vector<int> fresh;
    for (int m = 0; m < B && next < n_req; ++m)
      if (slot_req[m] < 0) {
        const int r = next++, L = offsets[r + 1] - offsets[r];
        slot_req[m] = r;
        slot_pos[m] = L - 1;
        slot_tok[m] = prompts[offsets[r] + L - 1];
        fresh.push_back(m);
        ++live;
      }
    if (live == 0) break;
    if (!fresh.empty()) {
      for (int m : fresh) {
        const int r = slot_req[m], L = offsets[r + 1] - offsets[r];
        std::memcpy(&in[(size_t)m * e->in_cap], prompts + offsets[r], (size_t)L * 4);
      }
      TI_TRY(ti_memcpy_h2d(e->in_tokens, in.data(), in.size() * 4, e->s));
      for (int m : fresh) {
        const int L = offsets[slot_req[m] + 1] - offsets[slot_req[m]];
        for (int t0 = 0; t0 < L - 1; t0 += pf) TI_TRY(enqueue_prefill(e, m, t0, std::min(pf, L - 1 - t0), 0));
      }
    }
    // one chunk: every slot feeds one token at its position; no slot may run past max_seq
    int S = chunk;
    for (int m = 0; m < B; ++m) {
      nin[m] = 1;
      base[m] = slot_req[m] >= 0 ? slot_pos[m] : 0;
      in[(size_t)m * e->in_cap] = slot_req[m] >= 0 ? slot_tok[m] : 0;
      if (slot_req[m] >= 0) S = std::min(S, c.max_seq - slot_pos[m]);
    }
    // (stream order: these copies land after the prefill launches have read in_tokens)
    TI_TRY(ti_memcpy_h2d(e->in_tokens, in.data(), in.size() * 4, e->s));
    TI_TRY(ti_memcpy_h2d(e->n_in, nin.data(), (size_t)B * 4, e->s));
    TI_TRY(ti_memcpy_h2d(e->base_pos, base.data(), (size_t)B * 4, e->s));
    const int32_t zero = 0;
    TI_TRY(ti_memcpy_h2d(e->step_ctr, &zero, 4, e->s));
    TI_TRY(run_steps(e, B, 1, S));
    TI_TRY(ti_memcpy_d2h(outd.data(), e->out_tokens, outd.size() * 4, e->s));
    TI_TRY(read_argmax(e, B, am));   // synchronises the stream
    for (int m = 0; m < B; ++m) {
      const int r = slot_req[m];
      if (r < 0) continue;
      // the token generated at chunk step s: fed back and recorded at step s + 1, the last
      // one still in the argmax slots
      for (int s = 0; s < S && slot_req[m] >= 0; ++s) {
        const int32_t tok = s < S - 1 ? outd[(size_t)m * e->out_cap + s]
                                      : (int32_t)(0xFFFFFFFFu - (uint32_t)(am[m] & 0xFFFFFFFFull));
        out_tokens[(size_t)r * max_new + out_len[r]++] = tok;
        slot_tok[m] = tok;
        if (out_len[r] >= max_new || tok == eos) {
          slot_req[m] = -1;
          --live;
        }
      }
      if (slot_req[m] >= 0) slot_pos[m] += S;
    }
  }
  return TI_OK;
}

int ti_engine_set_stop(ti_engine* e, int32_t token) {
  if (!e || token < -1 || token >= e->c.vocab) return ti_set_error(TI_ERR_ARG, "ti_engine_set_stop: token %d", token);
  e->stop_token = token;
  return TI_OK;
}

int ti_engine_counters(ti_engine* e, uint64_t* decode_steps, uint64_t* prefill_chunks) {
  if (!e) return ti_set_error(TI_ERR_ARG, "ti_engine_counters: null");
  if (decode_steps) *decode_steps = e->n_decode_steps;
  if (prefill_chunks) *prefill_chunks = e->n_prefill_chunks;
  return TI_OK;
}

int ti_engine_set_prefill(ti_engine* e, int rows) {
  if (!e || e->c.compat || rows < 0 || rows > e->rows_cap || (rows > 0 && rows > ((e->c.bits & ~TI_BITS_G32) == 4 ? TI_GEMM_MAX_ROWS : 16)))
    return ti_set_error(TI_ERR_ARG, "ti_engine_set_prefill: rows %d", rows);
  DeviceScope bind_(e);
  e->pf_rows = rows;
  return TI_OK;
}

int ti_engine_step(ti_engine* e, int n, const int32_t* tokens, const int32_t* pos, float* logits) {
  if (!e || !tokens || !pos) return ti_set_error(TI_ERR_ARG, "ti_engine_step: null");
  DeviceScope bind_(e);
  const ti_engine_config& c = e->c;
  if (c.compat) return ti_set_error(TI_ERR_UNSUPPORTED, "ti_engine_step: compat engine");
  if (n < 1 || n > c.max_batch) return ti_set_error(TI_ERR_ARG, "ti_engine_step: n=%d", n);
  for (int m = 0; m < n; ++m)
    if (pos[m] < 0 || pos[m] >= c.max_seq) return ti_set_error(TI_ERR_ARG, "ti_engine_step: pos %d", pos[m]);
  TI_TRY(ensure_io(e, 1, 1));
  std::vector<int32_t> in((size_t)n * e->in_cap, 0), one(n, 1);
  for (int m = 0; m < n; ++m) in[(size_t)m * e->in_cap] = tokens[m];
  TI_TRY(ti_memcpy_h2d(e->in_tokens, in.data(), in.size() * 4, e->s));
  TI_TRY(ti_memcpy_h2d(e->n_in, one.data(), (size_t)n * 4, e->s));
  TI_TRY(ti_memcpy_h2d(e->base_pos, pos, (size_t)n * 4, e->s));
  TI_TRY(ti_memset(e->step_ctr, 0, 4, e->s));
  TI_TRY(run_steps(e, n, 1, 1));
  TI_TRY(ti_stream_sync(e->s));
  if (logits) TI_TRY(ti_memcpy_d2h(logits, e->logits, (size_t)n * c.vocab * 4, e->s));
  if (n == 1) TI_TRY(qa_fault_check(e));
  return TI_OK;
}

int ti_engine_compat_step(ti_engine* e, int placeholder_offset, float* logits) {
  if (!e || !e->c.compat) return ti_set_error(TI_ERR_ARG, "ti_engine_compat_step: not a compat engine");
  DeviceScope bind_(e);
  const ti_engine_config& c = e->c;
  const int H = c.hidden, I = c.inter, V = c.vocab;
  std::vector<int32_t> zero(1, 0);
  TI_TRY(ti_memset(e->step_ctr, 0, 4, e->s));
  ti_step_args sa{};
  sa.h = e->h;
  sa.hidden = H;
  sa.M = 1;
  sa.vocab = V;
  sa.placeholder_first = placeholder_offset;
  sa.argmax = e->argmax;
  sa.pos = e->pos;
  sa.base_pos = e->base_pos;
  sa.step_ctr = e->step_ctr;
  TI_TRY(ti_step_begin(&sa, e->s));
  for (int l = 0; l < c.layers; ++l) {
    DevLayer& L = e->layer[l];
    // TransformerLayer::forward without attention weights (inference_engine.cpp:293-296):
    // post_attn = add(x, x); ffn = relu(post_attn @ up) @ down (:392-398); out = add(post_attn, ffn).
    TI_TRY(ti_add_f32(e->h, e->h, e->h, H, e->s));
    TI_TRY(ti_matmul_f32(e->h, L.gu.f32, e->tmp, nullptr, 1, H, I, 1, e->s));
    TI_TRY(ti_matmul_f32(e->tmp, L.down.f32, e->h, e->h, 1, I, H, 2, e->s));
  }
  TI_TRY(ti_matmul_f32(e->h, e->lm.f32, e->logits, nullptr, 1, H, V, 0, e->s));
  TI_TRY(ti_stream_sync(e->s));
  if (logits) TI_TRY(ti_memcpy_d2h(logits, e->logits, (size_t)V * 4, e->s));
  return TI_OK;
}

int ti_engine_replay_prepare(ti_engine* e, int n, int kv_len, int start_token) {
  if (!e || e->c.compat) return ti_set_error(TI_ERR_ARG, "ti_engine_replay_prepare: bad engine");
  DeviceScope bind_(e);
  const ti_engine_config& c = e->c;
  if (n < 1 || n > c.max_batch || kv_len < 1 || kv_len > c.max_seq || start_token < 0 || start_token >= c.vocab)
    return ti_set_error(TI_ERR_ARG, "ti_engine_replay_prepare: n=%d kv_len=%d", n, kv_len);
  TI_TRY(ensure_io(e, 1, 1));
  std::vector<int32_t> base(n, kv_len - 1), zero(n, 0);
  std::vector<unsigned long long> am((size_t)n * TI_ARGMAX_SLOTS, 0ull);
  for (int m = 0; m < n; ++m) am[(size_t)m * TI_ARGMAX_SLOTS] = 0xFFFFFFFFu - (uint32_t)start_token;
  TI_TRY(ti_memcpy_h2d(e->base_pos, base.data(), (size_t)n * 4, e->s));
  TI_TRY(ti_memcpy_h2d(e->n_in, zero.data(), (size_t)n * 4, e->s));
  TI_TRY(ti_memcpy_h2d(e->argmax, am.data(), am.size() * 8, e->s));
  TI_TRY(ti_memset(e->step_ctr, 0, 4, e->s));
  hipGraphExec_t g = nullptr;
  TI_TRY(get_graph(e, n, 0, &g));
  e->replay_M = n;
  return ti_stream_sync(e->s);
}

int ti_engine_replay_run(ti_engine* e, int steps) {
  if (!e || e->replay_M < 1) return ti_set_error(TI_ERR_ARG, "ti_engine_replay_run: call ti_engine_replay_prepare first");
  DeviceScope bind_(e);
  return run_steps(e, e->replay_M, 0, steps);
}

int ti_engine_sync(ti_engine* e) {
  if (!e) return ti_set_error(TI_ERR_ARG, "ti_engine_sync: null");
  DeviceScope bind_(e);
  TI_TRY(ti_stream_sync(e->s));
  return TI_OK;
}


int ti_engine_set_fold(ti_engine* e, int on, int* active) {
  if (!e) return ti_set_error(TI_ERR_ARG, "ti_engine_set_fold: null");
  DeviceScope bind_(e);
  if (on >= 0 && ((on != 0) != e->fold_on || (on != 0) != e->part_on)) {
    TI_TRY(ti_stream_sync(e->s));   // captured step graphs bake the setting in
    for (auto& g : e->graphs) hipGraphExecDestroy(g.second);
    e->graphs.clear();
    e->fold_on = e->part_on = on != 0;
  }
  if (active) *active = fold_usable(e, 1) ? 1 : 0;
  return TI_OK;
}

int ti_engine_set_qkv_attn(ti_engine* e, int on, int* active) {
  if (!e) return ti_set_error(TI_ERR_ARG, "ti_engine_set_qkv_attn: null");
  DeviceScope bind_(e);
  if (on >= 0 && (on != 0) != e->qa_on) {
    TI_TRY(ti_stream_sync(e->s));   // captured step graphs bake the setting in
    for (auto& g : e->graphs) hipGraphExecDestroy(g.second);
    e->graphs.clear();
    e->qa_on = on != 0;
  }
  if (active) *active = qa_usable(e, 1) ? 1 : 0;
  return TI_OK;
}

int ti_engine_last_tokens(ti_engine* e, int n, int32_t* tokens) {
  if (!e || !tokens || n < 1 || n > e->c.max_batch) return ti_set_error(TI_ERR_ARG, "ti_engine_last_tokens");
  DeviceScope bind_(e);
  std::vector<unsigned long long> am;
  TI_TRY(read_argmax(e, n, am));
  for (int m = 0; m < n; ++m) tokens[m] = (int32_t)(0xFFFFFFFFu - (uint32_t)(am[m] & 0xFFFFFFFFull));
  return TI_OK;
}

int ti_engine_time_kernel(ti_engine* e, int which, int n, int kv_len, int reps, double* avg_us, double* bytes) {
  if (!e || e->c.compat || !avg_us || !bytes || reps < 1 || n < 1 || n > e->c.max_batch || e->c.layers < 1)
    return ti_set_error(TI_ERR_ARG, "ti_engine_time_kernel: bad arguments");
  DeviceScope bind_(e);
  const ti_engine_config& c = e->c;
  const int H = c.hidden, I = c.inter, qd = e->qd(), kvd = e->kvd();
  const bool fold = fold_usable(e, n), part = part_usable(e, n), bfold = !fold && bfold_usable(e, n);
  // Launch r uses layer r % layers, so (as in a real step) its weights are not still in
  // the 256 MB Infinity Cache from the previous launch.
  int cur = 0;
  auto setup = [&](DevLayer& L, const DevLinear*& W, const void*& x, int& xk, int& ldx, const float*& nw,
                     ti_epilogue& ep) -> int {
    W = nullptr; x = nullptr; xk = TI_X_F16; ldx = 0; nw = nullptr; ep = ti_epilogue{};
    switch (which) {
      case 0: W = &L.qkv; x = e->h; xk = TI_X_F32_RMSNORM; ldx = H; nw = L.attn_norm;
        ep.kind = TI_EPI_QKV_ROPE_KV; ep.ldo = qd; ep.out = e->q; ep.q_dim = qd; ep.kv_dim = kvd; ep.head_dim = c.head_dim;
        ep.max_seq = c.max_seq; ep.pos = e->pos; ep.rope_cs = e->rope_cs; ep.k_cache = L.kc; ep.v_cache = L.vc;
        ep.kv_stream_stride = e->kv_stride; break;
      case 1: W = &L.o; x = e->attn; ldx = qd; ep.kind = TI_EPI_STORE_F32; ep.ldo = H; ep.out = e->tmp ? e->tmp : e->q; break;
      case 2: W = &L.gu; x = e->h; xk = TI_X_F32_RMSNORM; ldx = H; nw = L.ffn_norm;
        ep.kind = TI_EPI_SILU_MUL_F16; ep.ldo = I; ep.out = e->act; break;
      case 3: W = &L.down; x = e->act; ldx = I; ep.kind = TI_EPI_STORE_F32; ep.ldo = H; ep.out = e->q; break;
      case 4: W = &e->lm; x = e->h; xk = TI_X_F32_RMSNORM; ldx = H; nw = e->out_norm;
        ep.kind = TI_EPI_LOGITS_ARGMAX; ep.ldo = c.vocab; ep.out = e->logits; ep.argmax = e->argmax; break;
      case 5: break;
      default: return ti_set_error(TI_ERR_ARG, "ti_engine_time_kernel: which=%d", which);
    }
    if (which == 1 || which == 3) {
      // STORE_F32 into a scratch of n*H floats: q holds n*qd >= n*H only if qd >= H
      if ((size_t)qd < (size_t)H) return ti_set_error(TI_ERR_UNSUPPORTED, "ti_engine_time_kernel: scratch too small");
      ep.out = e->q;
      if (fold) {   // the step's producer form: residual add into the scratch + fold outputs
        ep.kind = TI_EPI_RESID_F32;
        ep.fold_w = L.ffn_norm;
        ep.fold_x = e->fx;
        ep.fold_ss = e->ss;
      } else if (bfold) {   // the batched fold's producer form (enqueue_step)
        ep.kind = TI_EPI_RESID_F32;
        ep.fold_w = L.ffn_norm;
        ep.fold_x = e->xn;
        ep.fold_ss = e->ss_rows;
        ep.fold_packed = ti_gemm_packed_rows_for(c.bits, n, which == 1 ? L.gu.N : L.qkv.N, H);
      }
      if (which == 1 && part) {   // O merges the attention's split partials
        x = e->part_o;
        xk = TI_X_ATTN_SPLITS;
        ep.ss_in = e->part_ml;
        ep.n_ss = e->splits_for(n);
        ep.head_dim = c.head_dim;
      }
    }
    if (packed_rows(e, n) && (which == 1 || which == 3)) xk = TI_X_F16_PACKED;   // enqueue_step's operands
    if (packed_rows(e, n) && which == 2) ep.out_packed = 1;
    if (fold && xk == TI_X_F32_RMSNORM) {   // the step's consumer form (enqueue_step)
      x = e->fx;
      xk = TI_X_F16_FOLDED;
      nw = nullptr;
      ep.ss_in = e->ss;
      ep.n_ss = ti_gemm_grid(1, H, which == 2 ? qd : I);
    } else if (bfold && xk == TI_X_F32_RMSNORM) {   // the batched fold's consumer form
      x = e->xn;
      xk = ti_gemm_packed_rows_for(c.bits, n, W->N, H) ? TI_X_F16_PACKED : TI_X_F16;
      nw = nullptr;
      ep.ss_in = e->ss_rows;
      ep.n_ss = ti_gemm_fold_partials(c.bits, n, H, which == 2 ? qd : I);
    }
    return TI_OK;
  };
  const DevLinear* W = nullptr;
  const void* x = nullptr;
  int xk = TI_X_F16, ldx = 0;
  const float* nw = nullptr;
  ti_epilogue ep{};
  TI_TRY(setup(e->layer[0], W, x, xk, ldx, nw, ep));
  if (ep.ss_in == e->ss_rows && ep.n_ss > 0) {   // batched fold: partials of rms 1 per row
    const float v = (float)H / (float)ep.n_ss;
    TI_TRY(ti_fill_uniform_f32(1, 0, (uint64_t)ep.n_ss * TI_FOLD_SS_ROWS, 0.0f, v, e->ss_rows, e->s));
  }
  std::vector<int32_t> base(n, kv_len - 1);
  TI_TRY(ti_memcpy_h2d(e->pos, base.data(), (size_t)n * 4, e->s));
  auto launch = [&]() -> int {
    DevLayer& L = e->layer[cur];
    cur = (cur + 1) % c.layers;
    TI_TRY(setup(L, W, x, xk, ldx, nw, ep));
    // (the one lm_head, 68 MB at 7B, fits the Infinity Cache: back-to-back it runs warm)
    if (which == 5 && part)
      return ti_attn_decode_partials(e->q, L.kc, L.vc, e->kv_stride, c.max_seq, e->pos, n, c.heads, c.kv_heads,
                                     c.head_dim, e->splits_for(n), e->part_o, e->part_ml, e->s);
    if (which == 5)
      return (packed_rows(e, n) ? ti_attn_decode_packed : ti_attn_decode)(e->q, L.kc, L.vc, e->kv_stride, c.max_seq,
                                                                           e->pos, n, c.heads, c.kv_heads, c.head_dim,
                                                                           e->splits_for(n), e->ws, e->attn, e->s);
    return gemm_rows(e, *W, n, x, xk, ldx, nw, ep, which == 2 ? 2 : 4, false);
  };
  // The `reps` launches are captured once into a graph and the graph is replayed `rounds`
  // times between two HIP events: no host launch cost inside the timed region (eager
  // launches of ~10 us kernels can go host-bound on a slow host and read 2x long), and
  // several milliseconds of back-to-back work, so the clocks are those of a running step.
  TI_TRY(ti_gemm_prepare());
  TI_TRY(ti_stream_sync(e->s));
  E_CHECK(hipStreamBeginCapture(e->s, hipStreamCaptureModeThreadLocal), "hipStreamBeginCapture");
  int rc = TI_OK;
  for (int r = 0; r < reps && rc == TI_OK; ++r) rc = launch();
  hipGraph_t graph = nullptr;
  const hipError_t ec = hipStreamEndCapture(e->s, &graph);
  if (rc != TI_OK) {
    if (graph) hipGraphDestroy(graph);
    return rc;
  }
  E_CHECK(ec, "hipStreamEndCapture");
  hipGraphExec_t gx = nullptr;
  const hipError_t ei = hipGraphInstantiate(&gx, graph, nullptr, nullptr, 0);
  hipGraphDestroy(graph);
  E_CHECK(ei, "hipGraphInstantiate");
  const int rounds = which == 6 ? std::max(4, 32 / reps) : std::max(4, 4096 / reps);
  hipEvent_t a = nullptr, b = nullptr;
  hipError_t el = hipEventCreate(&a);
  if (el == hipSuccess) el = hipEventCreate(&b);
  if (el == hipSuccess) el = hipGraphLaunch(gx, e->s);   // warm (code objects, caches, clocks)
  if (el == hipSuccess) el = hipEventRecord(a, e->s);
  for (int r = 0; r < rounds && el == hipSuccess; ++r) el = hipGraphLaunch(gx, e->s);
  if (el == hipSuccess) el = hipEventRecord(b, e->s);
  if (el == hipSuccess) el = hipEventSynchronize(b);
  float ms = 0.0f;
  if (el == hipSuccess) el = hipEventElapsedTime(&ms, a, b);
  if (a) hipEventDestroy(a);
  if (b) hipEventDestroy(b);
  hipGraphExecDestroy(gx);   // on every path after instantiation
  E_CHECK(el, "ti_engine_time_kernel: graph replay");
  // per projection (all row chunks of it, and the rms_norm prep of the batched path)
  *avg_us = (double)ms * 1000.0 / ((double)reps * rounds);
  if (which == 5) {
    *bytes = 2.0 * n * (double)kvd * kv_len * 2.0 + (double)n * qd * (4 + 2);
  } else if (which == 6) {   // every layer's weights + scales, K/V read at kv_len, K/V row written
    double wl = 0.0;
    for (const DevLinear* L : {&e->layer[0].qkv, &e->layer[0].o, &e->layer[0].gu, &e->layer[0].down})
      wl += (double)ti_wpack_tile_bytes(c.bits, L->K, L->N) + (double)ti_wpack_scale_bytes(c.bits, L->K, L->N);
    *bytes = c.layers * (wl + 2.0 * (double)kvd * kv_len * 2.0 + 2.0 * kvd * 2.0);
  } else {
    const double wbytes = (double)ti_wpack_tile_bytes(c.bits, W->K, W->N) + (double)ti_wpack_scale_bytes(c.bits, W->K, W->N);
    *bytes = wbytes + (double)n * W->K * (xk == TI_X_F16 || xk == TI_X_F16_FOLDED ? 2 : 4);
    if (xk == TI_X_ATTN_SPLITS) *bytes = wbytes + (double)n * W->K * 2;   // the merged row, as the unsplit input
  }
  return TI_OK;
}

}  // extern "C"


// ------------------------------------------------------------- in-step launch stamps
unsigned long long* ti_stamp_next(int kind, long grid) {
  StampCtx& c = g_stamp;
  if (!c.on) return nullptr;
  const size_t i = c.info.size() / 3;
  const bool stamped = grid > 0 && kind != TI_STAMP_KIND_RMSNORM && kind != TI_STAMP_KIND_OTHER;
  c.info.insert(c.info.end(), {(int32_t)kind, (int32_t)c.tag, stamped ? (int32_t)grid : 0});
  if (!c.base || i >= c.offs.size() || !stamped) return nullptr;
  return c.base + c.offs[i];
}

namespace {

// Capture `ksteps` replay steps back to back as one graph with the stamp context on (base NULL:
// record only).
int capture_stamped(ti_engine* e, int ksteps, unsigned long long* base, const std::vector<size_t>& offs,
                    std::vector<int32_t>& info, hipGraphExec_t* out) {
  StampCtx& c = g_stamp;
  c = StampCtx{};
  c.on = true;
  c.base = base;
  c.offs = offs;
  TI_TRY(ti_gemm_prepare());
  hipError_t eb = hipStreamBeginCapture(e->s, hipStreamCaptureModeThreadLocal);
  if (eb != hipSuccess) {
    c = StampCtx{};
    return ti_check_hip(eb, "hipStreamBeginCapture");
  }
  int rc = TI_OK;
  for (int k = 0; k < ksteps && rc == TI_OK; ++k) rc = enqueue_step(e, e->replay_M, 0);
  hipGraph_t g = nullptr;
  const hipError_t ec = hipStreamEndCapture(e->s, &g);
  info = c.info;
  c = StampCtx{};
  if (rc != TI_OK) {
    if (g) hipGraphDestroy(g);
    return rc;
  }
  E_CHECK(ec, "hipStreamEndCapture");
  if (!out) {
    hipGraphDestroy(g);
    return TI_OK;
  }
  const hipError_t ei = hipGraphInstantiate(out, g, nullptr, nullptr, 0);
  hipGraphDestroy(g);
  E_CHECK(ei, "hipGraphInstantiate");
  return TI_OK;
}

}  // namespace

int ti_engine_stamp_steps(ti_engine* e, int steps, int cap, int32_t* info_out, double* t_out, int* n_launch) {
  if (!e || e->replay_M < 1 || steps < 1 || steps > 256 || cap < 1 || !info_out || !t_out || !n_launch)
    return ti_set_error(TI_ERR_ARG, "ti_engine_stamp_steps: call ti_engine_replay_prepare first; 1 <= steps <= 256, "
                        "cap >= 1");
  DeviceScope bind_(e);
  TI_TRY(ti_stream_sync(e->s));
  // pass 1: one step's launch list and grids; pass 2: `steps` steps back to back in one graph, every
  // stamped launch with its own slot (so the timed steps run as replays do: no host gap between them)
  std::vector<int32_t> info, info2;
  TI_TRY(capture_stamped(e, 1, nullptr, {}, info, nullptr));
  const size_t n = info.size() / 3, nt = n * (size_t)steps;
  std::vector<size_t> offs(nt);
  size_t words = 0;
  for (size_t i = 0; i < nt; ++i) {
    offs[i] = words;
    words += (size_t)info[3 * (i % n) + 2] * kStampWords;
  }
  if (words == 0) return ti_set_error(TI_ERR_UNSUPPORTED, "ti_engine_stamp_steps: no stamped launch in the step");
  void* buf = nullptr;
  TI_TRY(ti_malloc(&buf, words * 8));
  unsigned long long* st = static_cast<unsigned long long*>(buf);
  hipGraphExec_t g = nullptr;
  int rc = capture_stamped(e, steps, st, offs, info2, &g);
  if (rc == TI_OK && (info2.size() != nt * 3 || !std::equal(info.begin(), info.end(), info2.begin())))
    rc = ti_set_error(TI_ERR_UNSUPPORTED, "ti_engine_stamp_steps: the two captures differ");
  std::vector<unsigned long long> h(words);
  for (int it = 0; rc == TI_OK && it < 2; ++it) {   // it 0: untimed (caches, clocks); it 1: the one read
    hipError_t he = hipMemsetAsync(st, 0, words * 8, e->s);
    if (he == hipSuccess) he = hipGraphLaunch(g, e->s);
    if (he == hipSuccess && it == 1) he = hipMemcpyAsync(h.data(), st, words * 8, hipMemcpyDeviceToHost, e->s);
    if (he == hipSuccess) he = hipStreamSynchronize(e->s);
    if (he != hipSuccess) rc = ti_check_hip(he, "ti_engine_stamp_steps: replay");
  }
  if (g) hipGraphExecDestroy(g);
  ti_free(buf);
  TI_TRY(rc);
  // per launch (all steps): first / last entry, last end, median workgroup end, mean wave-end skew,
  // workgroups sharing a CU, phase marks
  constexpr double kUs = 0.01;   // s_memrealtime: 100 MHz
  std::vector<double> acc(n * TI_STAMP_FIELDS, 0.0), first(nt, 0.0), last_end(nt, 0.0);
  for (size_t i = 0; i < nt; ++i) {
    const int wgs = info[3 * (i % n) + 2];
    if (wgs == 0) continue;
    unsigned long long f = ~0ull, le = 0, lent = 0;
    double wskew = 0.0;
    std::vector<unsigned long long> ends, cus;   // cus: (XCC, SE / SH / CU) of each workgroup
    ends.reserve(wgs);
    double ph[6] = {0, 0, 0, 0, 0, 0}, sskew = 0.0;
    int sskew_n = 0;
    int phn[6] = {0, 0, 0, 0, 0, 0};
    for (int w = 0; w < wgs; ++w) {
      const unsigned long long* p = h.data() + offs[i] + (size_t)w * kStampWords;
      if (p[0]) {
        f = std::min(f, p[0]);
        lent = std::max(lent, p[0]);
      }
      if (p[15]) cus.push_back((p[15] & 0x7FFFFFFF00000000ull) | (p[15] & 0xFF00ull));
      unsigned long long smn = ~0ull, smx = 0;   // diagnostic builds: the waves' ends of stream
      for (int k = 16; k < 24; ++k)
        if (p[k]) {
          smn = std::min(smn, p[k]);
          smx = std::max(smx, p[k]);
        }
      if (smx) {
        sskew += (double)(smx - smn);
        ++sskew_n;
      }
      unsigned long long mn = ~0ull, mx = 0;
      for (int k = 1; k <= 8; ++k)   // wave ends (words 1..8)
        if (p[k]) {
          mn = std::min(mn, p[k]);
          mx = std::max(mx, p[k]);
        }
      if (mx) {
        ends.push_back(mx);
        le = std::max(le, mx);
        wskew += (double)(mx - mn);
      }
      for (int k = 0; k < 6; ++k)   // phase marks of diagnostic builds (words 9..14), relative to entry
        if (p[0] && p[9 + k] >= p[0]) {
          ph[k] += (double)(p[9 + k] - p[0]);
          ++phn[k];
        }
    }
    if (f == ~0ull || ends.empty()) continue;
    std::nth_element(ends.begin(), ends.begin() + ends.size() / 2, ends.end());
    const unsigned long long med = ends[ends.size() / 2];
    first[i] = (double)f;
    last_end[i] = (double)le;
    double* a = acc.data() + (i % n) * TI_STAMP_FIELDS;
    a[0] += (double)(le - f) * kUs;
    a[2] += (double)(lent - f) * kUs;
    a[3] += wskew / (double)ends.size() * kUs;
    a[4] += (double)(le - med) * kUs;
    std::sort(cus.begin(), cus.end());
    a[6] += (double)(cus.end() - std::unique(cus.begin(), cus.end()));   // workgroups on an already-used CU
    for (int k = 0; k < 6; ++k) a[7 + k] += phn[k] ? ph[k] / phn[k] * kUs : 0.0;
    a[13] += sskew_n ? sskew / sskew_n * kUs : 0.0;
  }
  // periods: first entry -> the next stamped launch's first entry (across step boundaries: the steps
  // ran back to back); the very last launch: its span + the mean boundary
  double gap_sum = 0.0;
  int gap_n = 0;
  size_t last = nt;
  for (size_t i = 0; i < nt; ++i) {
    if (!first[i]) continue;
    size_t j = i + 1;
    while (j < nt && !first[j]) ++j;
    double* a = acc.data() + (i % n) * TI_STAMP_FIELDS;
    if (j < nt) {
      a[1] += (first[j] - first[i]) * kUs;
      a[5] += (first[j] - last_end[i]) * kUs;
      gap_sum += (first[j] - last_end[i]) * kUs;
      ++gap_n;
    } else {
      last = i;
    }
  }
  if (last < nt) {
    const double gap = gap_n ? gap_sum / gap_n : 0.0;
    acc[(last % n) * TI_STAMP_FIELDS + 1] += (last_end[last] - first[last]) * kUs + gap;
    acc[(last % n) * TI_STAMP_FIELDS + 5] += gap;
  }
  *n_launch = (int)n;
  for (size_t i = 0; i < n && (int)i < cap; ++i) {
    for (int k = 0; k < 3; ++k) info_out[3 * i + k] = info[3 * i + k];
    for (int k = 0; k < TI_STAMP_FIELDS; ++k) t_out[i * TI_STAMP_FIELDS + k] = acc[i * TI_STAMP_FIELDS + k] / steps;
  }
  return TI_OK;
}
