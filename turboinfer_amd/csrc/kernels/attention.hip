// attention.hip -- split-K single-query decode attention over the fp16 KV cache.
//
// Replaces TensorEngine::multi_head_attention (src/core/tensor_engine.cpp:1149-1252),
// whose decode call lands in attention_fast_incremental (:1254-1388): per head
// s_j = (q . k_j) / sqrt(hd), p = softmax(s), o = sum_j p_j v_j.  GQA maps q-head h to
// kv-head h / (heads / kv_heads) (the reference has no GQA; the oracle expands heads).
//
// HBM-bound (2 * L * hd * 2 bytes of K/V per kv-head per stream), no MFMA:
//   grid (splits, kv_heads, M); a workgroup = 8 waves owns keys [s0, s1) of one
//   (stream, kv-head) and ALL q-heads of its group, so each K/V byte is read once.
//   hd/8 lanes hold one key row (8 fp16 = one dwordx4); a wave-load covers 64/(hd/8)
//   keys ("slot"); wave w takes slots w, w+8, ... and keeps R of them (K and V) in flight
//   in a register ring refilled R slots ahead (the GEMV's streaming scheme).
//   Softmax is online PER LANE GROUP (one key row per group and slot): running max, sum
//   and o-accumulator live in the group's lanes, so the stream needs no cross-group
//   reduction; groups, then waves (LDS), then splits are merged at the end.
//   Splits of a (stream, kv-head) are merged in the same launch by the workgroup that
//   arrives last: partials are stored write-through (sc1) and drained, one lane adds to
//   the arrival ticket, the last arriver reads them back with sc1 loads
//   (MI355X_MICROARCH.md "Hand-offs measured with sc1 loads"; no L2 write-back fence).
#include <math.h>

#include <algorithm>

#include "common.hpp"

#include "attention_body.hpp"

namespace ti {

template <int HD, int G, int R, bool HP, int NW, bool ROT>
__global__ __launch_bounds__(NW * kWave, 1) void attn_split_kernel(const AttnArgs a) {
  const unsigned long long t_entry = stamp_now();
  attn_split_body<HD, G, R, HP, NW, ROT>(a, blockIdx.x, blockIdx.y, blockIdx.z);
  stamp_end(a.stamp, t_entry);
}

template <int HD, int G, int R, bool HP, int NW = kAttnWaves, bool ROT = false>
static int launch_one(const AttnArgs& a, hipStream_t s, size_t lds_pad = 0) {
  const dim3 grid(a.splits, a.kv_heads, a.M);
  hipLaunchKernelGGL((attn_split_kernel<HD, G, R, HP, NW, ROT>), grid, dim3(NW * kWave), lds_pad, s, a);
  TI_LAUNCH_CHECK("attn_split_kernel");
  return TI_OK;
}

template <int HD, int G>
static int launch_attn(const AttnArgs& a, hipStream_t s) {
  const bool long_range = G >= 4 && a.max_seq / a.splits >= 1024;   // keys per split (upper bound)
#ifndef TI_ATTN_HP
#define TI_ATTN_HP 1   // head-parallel lanes for GQA groups of 4-8 over short ranges
#endif
  if constexpr (TI_ATTN_HP && G >= 4 && HD / (64 / G) == 8) {
    if (!long_range) return launch_one<HD, G, TI_ATTN_RING_HP, true>(a, s);   // head-parallel lanes
  }
#ifndef TI_ATTN_LONG_WAVES
#define TI_ATTN_LONG_WAVES 8
#endif
#ifndef TI_ATTN_LONG_PAD
#define TI_ATTN_LONG_PAD 0   // dynamic LDS bytes added to the long-range launch (1 workgroup per CU)
#endif
#ifndef TI_ATTN_LONG_ROT
#define TI_ATTN_LONG_ROT 0
#endif
  if (long_range)
    return launch_one<HD, G, TI_ATTN_RING_LONG, false, TI_ATTN_LONG_WAVES, TI_ATTN_LONG_ROT != 0>(a, s, TI_ATTN_LONG_PAD);
  if constexpr (G == 1) {   // one stream, MHA (the 7B decode): 3 slots (bench A/B 745 vs 741 tok/s)
    if (a.M == 1) return launch_one<HD, G, TI_ATTN_RING_M1, false>(a, s);
  }
  return launch_one<HD, G, TI_ATTN_RING, false>(a, s);
}

template <int HD>
static int dispatch_group(const AttnArgs& a, int G, hipStream_t s) {
  switch (G) {
    case 1: return launch_attn<HD, 1>(a, s);
    case 2: return launch_attn<HD, 2>(a, s);
    case 4: return launch_attn<HD, 4>(a, s);
    case 8: return launch_attn<HD, 8>(a, s);
    default: return ti_set_error(TI_ERR_UNSUPPORTED, "ti_attn_decode: heads/kv_heads = %d not in {1,2,4,8}", G);
  }
}

}  // namespace ti

// Workspace: the arrival tickets first, at a fixed place for every call ([TI_ATTN_MAX_M][heads]
// int32, sized for heads >= kv_heads, zero before the first call and re-armed by every
// call), then the partials [M][heads][splits][head_dim + 4] fp32.  A fixed ticket region
// keeps calls with different M or splits from reading each other's partials as tickets.
static size_t ticket_bytes(int heads) { return ((size_t)TI_ATTN_MAX_M * heads * sizeof(int32_t) + 255) & ~(size_t)255; }

extern "C" size_t ti_attn_workspace_bytes(int M, int heads, int head_dim, int splits) {
  return ticket_bytes(heads) + (size_t)M * heads * splits * ti::ws_row(head_dim) * sizeof(float);
}

static int attn_impl(const float* q, const uint16_t* k_cache, const uint16_t* v_cache, int64_t kv_stream_stride,
                     int max_seq, const int32_t* pos, int M, int heads, int kv_heads, int head_dim, int splits,
                     float* workspace, uint16_t* out, ti_stream_t stream,
                     uint16_t* part_o = nullptr, float* part_ml = nullptr, bool packed = false) {
  using namespace ti;
  if (!q || !k_cache || !v_cache || !pos || ((!workspace || !out) && !part_o))
    return ti_set_error(TI_ERR_ARG, "ti_attn_decode: null pointer");
  if (M < 1 || M > TI_ATTN_MAX_M || heads < 1 || kv_heads < 1 || heads % kv_heads || splits < 1 || max_seq < 1)
    return ti_set_error(TI_ERR_ARG, "ti_attn_decode: bad sizes M=%d heads=%d kv_heads=%d splits=%d", M, heads,
                        kv_heads, splits);
  if (head_dim != 64 && head_dim != 128)
    return ti_set_error(TI_ERR_UNSUPPORTED, "ti_attn_decode: head_dim %d not in {64,128}", head_dim);
  // stride 0: the M rows are tokens of ONE stream (prefill), each attending to its own
  // prefix [0, pos[m]] of the shared cache
  if (kv_stream_stride != 0 && kv_stream_stride < (int64_t)kv_heads * max_seq * head_dim)
    return ti_set_error(TI_ERR_ARG, "ti_attn_decode: kv_stream_stride too small");
  // one stream, partials mode, GQA: run head by head (AttnArgs::kv_shift), so a short cache per
  // kv-head is streamed by G times as many workgroups (from the L2 / MALL after the first)
  const bool expand = part_o && M == 1 && heads > kv_heads;
  const int G = expand ? 1 : heads / kv_heads;
  int kv_shift = 0;
  if (expand) {
    while ((kv_heads << kv_shift) < heads) ++kv_shift;
    if ((kv_heads << kv_shift) != heads)
      return ti_set_error(TI_ERR_UNSUPPORTED, "ti_attn_decode_partials: heads/kv_heads %d not a power of two",
                          heads / kv_heads);
  }
  // splits only shape the work (results agree to rounding); the merge stages all partials
  // of a kv-head group in LDS, which bounds them.
  if (!part_o) splits = std::min(splits, std::max(1, ti::attn_max_splits(G, head_dim)));
  if (packed && (((heads * head_dim) & 127) || part_o))
    return ti_set_error(TI_ERR_ARG, "ti_attn_decode_packed: heads * head_dim %d not a multiple of 128",
                        heads * head_dim);
  AttnArgs a;
  a.out_kt = packed ? heads * head_dim / 128 : 0;
  a.part_o = part_o;
  a.part_ml = part_ml;
  a.q = q;
  a.kc = k_cache;
  a.vc = v_cache;
  a.pos = pos;
  a.counters = (int32_t*)workspace;
  a.ws = workspace ? (float*)((char*)workspace + ticket_bytes(heads)) : nullptr;
  a.out = out;
  a.stride = kv_stream_stride;
  a.max_seq = max_seq;
  a.M = M;
  a.heads = heads;
  a.kv_heads = expand ? heads : kv_heads;
  a.kv_shift = kv_shift;
  a.splits = splits;
  a.scale = 1.0f / sqrtf((float)head_dim);   // tensor_engine.cpp:1288 (hidden = head_dim per head)
  a.stamp = ti_stamp_next(STAMP_ATTN, (long)a.splits * a.kv_heads * a.M);
  hipStream_t s = (hipStream_t)stream;
  return head_dim == 128 ? dispatch_group<128>(a, G, s) : dispatch_group<64>(a, G, s);
}

extern "C" int ti_attn_decode(const float* q, const uint16_t* k_cache, const uint16_t* v_cache,
                              int64_t kv_stream_stride, int max_seq, const int32_t* pos, int M, int heads,
                              int kv_heads, int head_dim, int splits, float* workspace, uint16_t* out,
                              ti_stream_t stream) {
  return attn_impl(q, k_cache, v_cache, kv_stream_stride, max_seq, pos, M, heads, kv_heads, head_dim, splits, workspace,
                   out, stream);
}

extern "C" int ti_attn_decode_packed(const float* q, const uint16_t* k_cache, const uint16_t* v_cache,
                                     int64_t kv_stream_stride, int max_seq, const int32_t* pos, int M, int heads,
                                     int kv_heads, int head_dim, int splits, float* workspace, uint16_t* out,
                                     ti_stream_t stream) {
  return attn_impl(q, k_cache, v_cache, kv_stream_stride, max_seq, pos, M, heads, kv_heads, head_dim, splits, workspace,
                   out, stream, nullptr, nullptr, true);
}


extern "C" int ti_attn_decode_partials(const float* q, const uint16_t* k_cache, const uint16_t* v_cache,
                                       int64_t kv_stream_stride, int max_seq, const int32_t* pos, int M, int heads,
                                       int kv_heads, int head_dim, int splits, uint16_t* part_o, float* part_ml,
                                       ti_stream_t stream) {
  if (!part_o || !part_ml) return ti_set_error(TI_ERR_ARG, "ti_attn_decode_partials: null partials");
  if (splits < 2 || splits > TI_ATTN_MAX_PART_SPLITS)
    return ti_set_error(TI_ERR_ARG, "ti_attn_decode_partials: splits %d not in [2, %d]", splits, TI_ATTN_MAX_PART_SPLITS);
  return attn_impl(q, k_cache, v_cache, kv_stream_stride, max_seq, pos, M, heads, kv_heads, head_dim, splits, nullptr,
                   nullptr, stream, part_o, part_ml);
}
