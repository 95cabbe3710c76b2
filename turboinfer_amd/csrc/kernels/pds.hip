// pds.hip -- the 32 decode layers of one single-stream step in ONE persistent launch (gfx950).
//
// Replaces the per-layer launch chain of the decode step (QKV, attention, O, gate/up, down:
// TransformerLayer::forward_incremental, src/model/inference_engine.cpp:203-279, 291-368,
// 376-401, with the matmuls of tensor_engine.cpp:594-640 and attention_fast_incremental
// :1254-1388) for the configuration the bench is quoted on: one stream, INT4 group-128
// weights, multi-head attention with head_dim 128 and kv_heads * 8 == the grid (Llama-2-7B).
//
// Why: a layer as five launches pays, per launch, the kernel boundary plus the latency from
// launch to the first weight bytes landing (~4 us per launch, ~0.6 ms of the
// 1.36 ms step).  Here every workgroup streams ITS weight tiles and K/V rows for all layers as
// one continuous sequence: each consumer wave keeps a ring of RING units (2 KiB each) in flight
// and refills it past phase and layer boundaries, so while a workgroup waits for the previous
// phase's output vector its next phase's first bytes are already landing.
//
// Shape: one 8-wave workgroup per CU (grid = kv_heads * 8 = 256).
//   * waves 0-7 ("C"): the weight / K/V stream and the MFMA / softmax math, item for item
//     the arithmetic of gemv_wq_kernel (fold, partials modes) and attn_split_body (non-HP,
//     G = 1): wave w owns k-tiles w, w+8, ... of every tile, key slots w, w+8, ... of its
//     split; they issue only ring loads (plus the staging loads right after a hand-off).
//   * wave 7 is also the control wave ("X"): it polls the hand-off counters, reduces the C waves'
//     partials and runs the epilogues (RoPE + KV append, residual + folded rms_norm, SiLU*up,
//     split partials), then publishes them write-through (sc1) and signals.  The next phase's
//     ring units are issued only after that signal, so its s_waitcnt vmcnt(0) drains only its
//     own stores.  (A 9th, stream-free control wave was measured slower: DESIGN 4.15.)
// Per phase: X polls -> barrier -> C waves stage x / scales with sc1 loads (+ int4 offset
// correction) -> barrier -> C waves consume their units -> barrier -> X epilogue + signal.
// Hand-off form: MI355X_MICROARCH.md "Hand-offs measured with sc1 loads", first row (one lane
// per storing workgroup adds to a sharded agent-scope counter after the storing wave's
// vmcnt(0); the polling wave releases the workgroup through a barrier; every handed-off byte
// stored and loaded sc1; one workgroup per CU).  Counters are monotonic: launch e of a
// workgroup (its private launch count) waits for 256 * (e + 1) arrivals.
//
// Results are bit-identical to the graph path with the fold and partials hand-offs
// (tests/test_gpu_pds.py): same items in the same per-wave order, same reductions.
#include <math.h>

#include "common.hpp"
#include "attention_body.hpp"
#include "dequant.hpp"

namespace ti {

#ifndef TI_PDS_RING
#define TI_PDS_RING 8   // units (2 KiB per wave each) in flight per consumer wave
#endif
constexpr int kPdsRing = TI_PDS_RING;
#ifndef TI_PDS_PRE
#define TI_PDS_PRE 8   // ring units issued ahead of a hand-off, the rest after the input is staged (A/B: 8 best)
#endif
constexpr int kPdsPre = TI_PDS_PRE < TI_PDS_RING ? TI_PDS_PRE : TI_PDS_RING;
constexpr int kPdsC = 8;                         // consumer waves
constexpr int kPdsThreads = kPdsC * kWave;      // wave 7 is also the control wave
constexpr int kPdsCThreads = kPdsC * kWave;
constexpr int kPdsSplits = 8;
constexpr int kPdsHd = 128;
constexpr int kPdsMaxNtl = 8;
constexpr int kPdsShards = 8;
constexpr int kPdsShardWords = 32;               // one 128-byte line per shard
enum { PH_QKV = 0, PH_ATT, PH_O, PH_GU, PH_DN, PH_N };

typedef ti_pds_layer PdsLayerDev;   // ti_hip.h: tiles[4] (qkv, o, gate/up, down), scales[4], norms, K/V cache

struct PdsArgs {
  const PdsLayerDev* layers;
  int n_layers, H, I, qd, max_seq, n_ss0;
  float eps, scale;
  const int32_t* pos;
  const float* rope_cs;     // [max_seq][hd] (cos, sin) pairs
  const float* out_norm;
  float* h;                 // [H] residual (read at start, written at end)
  uint16_t* fx;             // [H] fp16 h * next norm weight (fold hand-off)
  float* ss;                // [grid] sums of h^2 (fold hand-off)
  float* q;                 // [qd]
  uint16_t* act;            // [I]
  uint16_t* part_o;         // [heads][8][128]
  float* part_ml;           // [heads][8][2]
  uint32_t* ctr;            // [layers][PH_N][8 shards][32]
  uint32_t* launches;       // [grid] private launch counts
  uint32_t* err;            // poll timeouts
  const u32x4* zero;        // >= 2 KiB readable, never written: dummy ring loads
  unsigned long long* ts;   // diagnostic phase timestamps [grid][layers][5][8] or null
  // granule hand-offs (8-byte {payload, tag}, one sc1 store / one sc1 load each)
  unsigned long long* fxg;  // [H / 2]: fp16 pairs of the fold (O -> gate/up, down -> next QKV)
  unsigned long long* ssg;  // [grid]: the fold's sums of h^2
  unsigned long long* qg;   // [qd]: RoPE'd q (QKV -> attention)
  unsigned long long* kvg;  // [heads][2][head_dim / 2]: the fresh K, V rows (fp16 pairs)
  unsigned long long* actg; // [I / 2]: SiLU * up (gate/up -> down)
};

// Granule layout of PdsArgs (ti_pds_granule_words)
__host__ __device__ inline size_t pds_gran_words(int H, int I, int qd, int heads, int grid) {
  return (size_t)H / 2 + (size_t)grid + (size_t)qd + (size_t)heads * kPdsHd + (size_t)I / 2;
}

// Static partition of a GEMV phase for workgroup bid (the same as gemv_wq_kernel's grid).
struct PdsLin {
  int K, KT, t0, ntl, KW, n_items, n_units, lin;
};
__device__ __forceinline__ PdsLin pds_lin(int lin, int K, int N, int bid, int grid, int wave) {
  PdsLin p;
  p.lin = lin;
  p.K = K;
  p.KT = K >> 7;
  const int NT = N >> 4;
  p.t0 = (int)((unsigned)bid * (unsigned)NT / (unsigned)grid);
  p.ntl = (int)((unsigned)(bid + 1) * (unsigned)NT / (unsigned)grid) - p.t0;
  p.KW = wave < p.KT ? (p.KT - wave + kPdsC - 1) / kPdsC : 0;
  p.n_items = p.ntl * p.KW;
  p.n_units = (p.n_items + 1) >> 1;
  return p;
}

// LDS layout (bytes)
constexpr int kLdsX = 0;                              // x fp16 [K + 8], K <= 16376
constexpr int kLdsXBytes = 32768;
constexpr int kLdsSc = kLdsX + kLdsXBytes;            // scales [ntl][KT][16] fp16
constexpr int kLdsScBytes = 16384;
constexpr int kLdsCorr = kLdsSc + kLdsScBytes;        // [KT] f32
constexpr int kLdsSlab = kLdsCorr + 512;              // [kPdsMaxNtl][8][16] f32
constexpr int kLdsAcc = kLdsSlab + kPdsMaxNtl * kPdsC * 16 * 4;   // attention [8][128] f32
constexpr int kLdsML = kLdsAcc + kPdsC * kPdsHd * 4;  // [8] m, [8] l
constexpr int kLdsQ = kLdsML + 64;                    // q of the head [128] f32
constexpr int kLdsKV = kLdsQ + kPdsHd * 4;            // fresh K row [128], V row [128] fp16
constexpr int kLdsH = kLdsKV + 2 * kPdsHd * 2;        // residual rows [16] f32
constexpr int kLdsCs = kLdsH + 64;                    // RoPE (cos, sin) [128] f32
constexpr int kLdsMisc = kLdsCs + kPdsHd * 4;          // launch epoch, dead flag (u32)
constexpr int kLdsBytes = kLdsMisc + 16;

__device__ __forceinline__ void pds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// X wave: wait until the counter's shards sum to target.  Bounded: after ~50 ms *err |= 1 and
// `dead` is set, after which no wait of this launch or of later launches (which read *err at
// their start) blocks again, so a broken hand-off costs one timeout, not one per wait.
__device__ __forceinline__ void pds_poll(const uint32_t* c, uint32_t target, uint32_t* err, int lane, bool& dead) {
  if (dead) return;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (true) {
    uint32_t v = lane < kPdsShards ? ld_sc1_u32(c + lane * kPdsShardWords) : 0u;
    v += __shfl_xor(v, 1, 64);
    v += __shfl_xor(v, 2, 64);
    v += __shfl_xor(v, 4, 64);
    if (__builtin_amdgcn_readfirstlane(v) >= target) break;
    if (__builtin_amdgcn_s_memrealtime() - t0 > 5000000ull) {
      if (lane == 0) atomicOr(err, 1u);
      dead = true;
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}
// X wave: drain its write-through stores, then one lane signals the workgroup's shard.
__device__ __forceinline__ void pds_signal(uint32_t* c, int bid, int lane) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane == 0)
    __hip_atomic_fetch_add(c + (bid & (kPdsShards - 1)) * kPdsShardWords, 1u, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}

// ---- data-tagged hand-offs (MI355X_MICROARCH.md price list: granule, handoff-1to1, allgather):
// a producer stores {payload, tag} as ONE 8-byte sc1 store -- no drain, no counter -- and the
// consumer polls the data itself with 8-byte sc1 loads until every tag is this launch's.  The
// tag names (launch epoch, layer, producing phase) and is never 0, the zeroed buffer's value.
// A buffer is rewritten only after a full all-to-all dependency on its readers (fx: O(l) then
// down(l); ss likewise; q, kv, act once per layer), so no reader can see a granule overwritten.
__device__ __forceinline__ uint32_t pds_tag(uint32_t epoch, int l, int ph) {
  return ((epoch * 64u + (uint32_t)l) * 8u + (uint32_t)ph) + 1u;
}
__device__ __forceinline__ void st_gran(unsigned long long* p, uint32_t payload, uint32_t tag) {
  st_sc1_u64(p, ((unsigned long long)tag << 32) | payload);
}
// NG granules at g[0], g[stride], ...: wait (bounded, like pds_poll) until all carry `tag`.
template <int NG>
__device__ __forceinline__ void gather_gran(const unsigned long long* g, int stride, uint32_t tag, uint32_t (&out)[NG],
                                            uint32_t* err, bool& dead) {
  unsigned long long v[NG];
#pragma unroll
  for (int i = 0; i < NG; ++i) v[i] = ld_sc1_u64(g + i * stride);
  auto ready = [&]() {
    bool ok = true;
#pragma unroll
    for (int i = 0; i < NG; ++i) ok = ok && (uint32_t)(v[i] >> 32) == tag;
    return ok;
  };
  if (!ready() && !dead) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (true) {
      __builtin_amdgcn_s_sleep(1);
#pragma unroll
      for (int i = 0; i < NG; ++i)
        if ((uint32_t)(v[i] >> 32) != tag) v[i] = ld_sc1_u64(g + i * stride);
      if (ready()) break;
      if (__builtin_amdgcn_s_memrealtime() - t0 > 5000000ull) {
        atomicOr(err, 2u);
        dead = true;
        break;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < NG; ++i) out[i] = (uint32_t)v[i];
}

// Pointers reach the kernel through the layer table (generic): cast them to the global address
// space, or the compiler emits flat loads, which also count in lgkmcnt -- every LDS wait would
// then wait for the whole weight ring.
template <class T>
__device__ __forceinline__ const __attribute__((address_space(1))) T* gptr(const T* p) {
  return (const __attribute__((address_space(1))) T*)p;
}
template <class T>
__device__ __forceinline__ __attribute__((address_space(1))) T* gptr_w(T* p) {
  return (__attribute__((address_space(1))) T*)p;
}
__device__ __forceinline__ u32x4 pds_ld_w(const u32x4* p) { return __builtin_nontemporal_load(gptr(p)); }
__device__ __forceinline__ u32x4 ld_sc1_b128(const void* base, uint32_t byte_off) {
  return __builtin_amdgcn_raw_buffer_load_b128(sc1_rsrc(base), byte_off, 0, kAuxSc1Load);
}

// Every phase of a consumer wave is padded to whole blocks of RING units (dummy units are not
// loaded and are consumed as nothing), so each phase starts at ring slot 0 and the slot indices
// stay static (VGPRs, not scratch).  Blocks before the last refill from the phase's own cursor;
// after the last block the wave passes the phase's closing barrier and only then issues the NEXT
// phase's first RING units (the control wave after its signal), so the issue stalls of a full
// memory queue stay off the phase's critical path and the next phase starts with RING units
// already landed.
template <class C, class R0>
__device__ __forceinline__ void pds_blocks(u32x4 (&ring)[kPdsRing][2], int nblk, C& consume, R0& refill_in) {
  for (int b = 0; b + 1 < nblk; ++b) {
#pragma unroll
    for (int k = 0; k < kPdsRing; ++k) {
      consume(ring[k]);
      refill_in(ring[k]);
    }
  }
#pragma unroll
  for (int k = 0; k < kPdsRing; ++k) consume(ring[k]);   // the next phase refills after the barrier
}
__device__ __forceinline__ int pds_nblk(int units) { return units > 0 ? (units + kPdsRing - 1) / kPdsRing : 1; }

// Refill cursors of a consumer wave.  GEMV phase: this wave's items (tile t, k-tile cw + 8 kk) of
// the workgroup's tiles, two per unit; attention: key slot cw + 8 u of the split (K and V).
struct GCur {
  const u32x4* base;   // lane's address of item (0, 0)
  int KT, KW, ntl, t, kk;
};
struct ACur {
  const uint16_t* kb;  // lane's K / V element of slot 0
  const uint16_t* vb;
  int u, key0;         // key of slot 0 for this lane
};

__global__ __launch_bounds__(kPdsThreads, 1) void pds_kernel(const PdsArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  f16* xl = (f16*)(smem + kLdsX);
  uint16_t* sl = (uint16_t*)(smem + kLdsSc);
  float* corr = (float*)(smem + kLdsCorr);
  float* slab = (float*)(smem + kLdsSlab);
  float* s_acc = (float*)(smem + kLdsAcc);
  float* s_m = (float*)(smem + kLdsML);
  float* s_l = s_m + kPdsC;
  float* q_l = (float*)(smem + kLdsQ);
  uint16_t* kf_l = (uint16_t*)(smem + kLdsKV);
  uint16_t* vf_l = kf_l + kPdsHd;
  float* h_l = (float*)(smem + kLdsH);
  float* cs_l = (float*)(smem + kLdsCs);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int bid = blockIdx.x, grid = gridDim.x;
  const bool is_x = wave == kPdsC - 1;   // control wave (also a consumer)
  const int H = a.H, I = a.I, qd = a.qd, HD = kPdsHd;
  const int pos = __builtin_amdgcn_readfirstlane(gptr(a.pos)[0]);
  const int L = pos + 1;
  // attention split of this workgroup (kv-head kvh, split sp; heads == kv_heads)
  const int kvh = bid / kPdsSplits, sp = bid - kvh * kPdsSplits;
  const int chunk = (L + kPdsSplits - 1) / kPdsSplits;
  const int s0 = sp * chunk, s1 = min(L, s0 + chunk);
  const int nslot = s1 > s0 ? (s1 - s0 + 3) / 4 : 0;
  const int cw = wave;
  const int att_units = cw < nslot ? (nslot - cw + kPdsC - 1) / kPdsC : 0;
  const int64_t kv_off = (int64_t)kvh * a.max_seq * HD;
  // GEMV partitions (the same for every layer)
  // recomputed where needed (a few scalar ops) rather than kept live across the kernel
  auto lin_params = [&](int ph) -> PdsLin {
    const int lin = ph == PH_QKV ? 0 : ph == PH_O ? 1 : ph == PH_GU ? 2 : 3;
    const int K = ph == PH_DN ? I : ph == PH_O ? qd : H;
    const int N = ph == PH_QKV ? 3 * qd : ph == PH_GU ? 2 * I : H;
    return pds_lin(lin, K, N, bid, grid, cw);
  };

  // ---------------------------------------------------------------- C waves: the stream
  const u32x4* zero_l = a.zero + lane;
  auto gcur = [&](int l, int ph) -> GCur {
    GCur c{};
    if (l >= a.n_layers) { c.ntl = 0; c.KW = 1; return c; }   // past the last layer: dummies
    const PdsLin p = lin_params(ph);
    c.KT = p.KT;
    c.KW = p.KW > 0 ? p.KW : 1;
    c.ntl = p.KW > 0 ? p.ntl : 0;
    c.base = (const u32x4*)a.layers[l].tiles[p.lin] + ((size_t)p.t0 * p.KT + cw) * kWave + lane;
    return c;
  };
  auto gnext = [&](GCur& c) -> const u32x4* {
    if (c.t >= c.ntl) return zero_l;
    const u32x4* q = c.base + ((size_t)c.t * c.KT + kPdsC * c.kk) * kWave;
    if (++c.kk == c.KW) { c.kk = 0; ++c.t; }
    return q;
  };
  auto grefill = [&](GCur& c, u32x4 (&slot)[2]) {
    if (c.t >= c.ntl) return;   // dummy unit: nothing to load (consumed as nothing)
    const u32x4* p0 = gnext(c);
    const u32x4* p1 = gnext(c);
    slot[0] = pds_ld_w(p0);
    slot[1] = pds_ld_w(p1);
  };
  auto acur = [&](int l) -> ACur {
    ACur c{};
    const int key = s0 + cw * 4 + (lane >> 4);
    c.u = 0;
    c.key0 = key;
    const size_t e = (size_t)kv_off + (size_t)key * HD + (lane & 15) * 8;
    c.kb = a.layers[l].k_cache + e;
    c.vb = a.layers[l].v_cache + e;
    return c;
  };
  auto arefill = [&](ACur& c, u32x4 (&slot)[2]) {
    const int du = kPdsC * 4 * c.u;                  // keys from slot 0
    // the row at pos is written by this launch's QKV epilogue: never stream it (its stale
    // line must not sit in a cache ahead of the sc1 load after the hand-off)
    const bool ok = c.key0 + du < s1 && c.key0 + du != pos;
    ++c.u;
    if (kPdsC * 4 * (c.u - 1) + s0 + cw * 4 >= s1) return;   // no key of the wave's slot: dummy unit
    const u32x4* pk = ok ? (const u32x4*)(c.kb + (size_t)du * HD) : zero_l;
    const u32x4* pv = ok ? (const u32x4*)(c.vb + (size_t)du * HD) : zero_l + kWave;
    slot[0] = pds_ld_w(pk);
    slot[1] = pds_ld_w(pv);
  };

  u32x4 ring[kPdsRing][2];
#pragma unroll
  for (int s = 0; s < kPdsRing; ++s) ring[s][0] = ring[s][1] = (u32x4){0u, 0u, 0u, 0u};
  GCur gc{};   // the current GEMV phase's cursor (started by the previous phase's last block)
  ACur ac{};
  gc = gcur(0, PH_QKV);
#pragma unroll
  for (int s = 0; s < kPdsPre; ++s) grefill(gc, ring[s]);

  // ---------------------------------------------------------------- X wave: setup
  uint32_t epoch = 0;
  bool dead = false;   // a hand-off wait timed out (this or an earlier launch): no wait blocks again
  uint32_t* misc_l = (uint32_t*)(smem + kLdsMisc);
  const int t0o = (int)((unsigned)bid * (unsigned)(H >> 4) / (unsigned)grid);   // O / down tile of this workgroup (N = H: the same partition)
  if (is_x) {
    if (lane == 0) {
      epoch = gptr(a.launches)[bid];
      gptr_w(a.launches)[bid] = epoch + 1;
    }
    epoch = __builtin_amdgcn_readfirstlane(epoch);
    dead = __builtin_amdgcn_readfirstlane(ld_sc1_u32(a.err)) != 0u;
    if (lane < 16) h_l[lane] = gptr(a.h)[t0o * 16 + lane];
    for (int j = lane; j < HD; j += kWave) cs_l[j] = gptr(a.rope_cs)[(size_t)pos * HD + j];
    if (lane == 0) {
      misc_l[0] = epoch;
      misc_l[1] = dead ? 1u : 0u;
    }
  }
  pds_barrier();
  epoch = __builtin_amdgcn_readfirstlane(misc_l[0]);   // every wave: the granule tags
  dead = misc_l[1] != 0u;
  const uint32_t target = (uint32_t)grid * (epoch + 1);   // X only: arrivals of this launch (ATT -> O)
  // diagnostic: s_memrealtime (100 MHz) at phase events k of (layer l, phase ph), lane 0 of the
  // X wave (k = 0 poll start, 1 poll done, 2 staged, 4 consumed, 5 signalled) or C wave 0 (3)
  auto ts = [&](int l, int ph, int k) {
    if (a.ts != nullptr && lane == 0)
      a.ts[(((size_t)bid * a.n_layers + l) * PH_N + ph) * 8 + k] = __builtin_amdgcn_s_memrealtime();
  };

  uint32_t magic;
  asm volatile("v_mov_b32 %0, 0x64006400" : "=v"(magic));
  const int r = lane & 15, kq = lane >> 4;

  // C waves: stage an fp16 x row (K halves) with sc1 loads, pre-scale the high-nibble
  // slots by 1/16 and build corr[kt] (gemv_body steps 3 + the int4 pass, M = 1).
  auto stage_f16 = [&](const uint16_t* src, int K) {
    const int K8 = K >> 3;
    for (int i0 = 0; i0 < K8; i0 += kPdsCThreads) {
      const int idx = i0 + tid;
      float part = 0.0f;
      if (idx < K8) {
        f16x8 hx = __builtin_bit_cast(f16x8, ld_sc1_b128(src, (uint32_t)idx * 16u));
        const f16 s16 = (f16)0.0625f;
        hx[2] *= s16; hx[3] *= s16; hx[6] *= s16; hx[7] *= s16;
        *(f16x8*)(xl + 8 * idx) = hx;
        const float lo = ((float)hx[0] + (float)hx[1]) + ((float)hx[4] + (float)hx[5]);
        const float hi = ((float)hx[2] + (float)hx[3]) + ((float)hx[6] + (float)hx[7]);
        part = 1032.0f * lo + 1152.0f * hi;
      }
      part = group_sum<16>(part);
      if (idx < K8 && (lane & 15) == 0) corr[idx >> 4] = part;
    }
  };
  // the same from granules: thread idx's 8 fp16 are 4 granules {fp16 pair, tag}
  auto stage_f16_g = [&](const unsigned long long* g, int K, uint32_t tag) {
    const int K8 = K >> 3;
    for (int i0 = 0; i0 < K8; i0 += kPdsCThreads) {
      const int idx = i0 + tid;
      float part = 0.0f;
      if (idx < K8) {
        uint32_t w[4];
        gather_gran<4>(g + 4 * idx, 1, tag, w, a.err, dead);
        f16x8 hx = __builtin_bit_cast(f16x8, (u32x4){w[0], w[1], w[2], w[3]});
        const f16 s16 = (f16)0.0625f;
        hx[2] *= s16; hx[3] *= s16; hx[6] *= s16; hx[7] *= s16;
        *(f16x8*)(xl + 8 * idx) = hx;
        const float lo = ((float)hx[0] + (float)hx[1]) + ((float)hx[4] + (float)hx[5]);
        const float hi = ((float)hx[2] + (float)hx[3]) + ((float)hx[6] + (float)hx[7]);
        part = 1032.0f * lo + 1152.0f * hi;
      }
      part = group_sum<16>(part);
      if (idx < K8 && (lane & 15) == 0) corr[idx >> 4] = part;
    }
  };
  auto stage_scales = [&](const PdsLin& p, const uint16_t* sc) {
    const int n = p.ntl * p.KT * 2;   // 16-byte pieces
    const u32x4* sg = (const u32x4*)(sc + (size_t)p.t0 * p.KT * 16);
    for (int i = tid; i < n; i += kPdsCThreads) ((u32x4*)sl)[i] = gptr(sg)[i];
  };

  // C waves: consume one GEMV phase of partition p (acc per tile into the slab); the last
  // block refills from the next phase (rnext)
  auto gemv_phase = [&](const PdsLin& p) {
    const f16* xrow = xl + kq * 32;
    f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
    int ct = 0, ck = 0, j = 0;
    auto item = [&](const u32x4& w) {
      if (j >= p.n_items) return;
      ++j;
      const int kt = cw + kPdsC * ck;
      f32x4 t = {0.0f, 0.0f, 0.0f, 0.0f};
      const u32x4 wv[1] = {w};
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        const f16x8 bf = dequant_step<4>(wv, s4, magic);
        const f16x8 af = *(const f16x8*)(xrow + kt * 128 + s4 * 8);
        t = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, bf, t, 0, 0, 0);
      }
      t -= corr[kt];
      const float sc = h2f(sl[(ct * p.KT + kt) * 16 + r]);
      acc[0] = fmaf(sc, t[0], acc[0]);
      acc[1] = fmaf(sc, t[1], acc[1]);
      acc[2] = fmaf(sc, t[2], acc[2]);
      acc[3] = fmaf(sc, t[3], acc[3]);
      if (++ck == p.KW) {
        if (lane < 16) slab[(ct * kPdsC + cw) * 16 + lane] = acc[0];
        acc = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
        ck = 0;
        ++ct;
      }
    };
    auto consume = [&](const u32x4 (&u)[2]) {
      item(u[0]);
      item(u[1]);
    };
    auto rin = [&](u32x4 (&slot)[2]) { grefill(gc, slot); };
    pds_blocks(ring, pds_nblk(p.n_units), consume, rin);
    if (p.KW == 0)
      for (int tl = 0; tl < p.ntl; ++tl)
        if (lane < 16) slab[(tl * kPdsC + cw) * 16 + lane] = 0.0f;
  };

  // X wave: the tile sums of the 8 waves (gemv_body's fixed order) for output (tl, n)
  auto tile_sum = [&](int tl, int n) {
    const float* sp = slab + tl * kPdsC * 16 + n;
    float v = sp[0];
#pragma unroll
    for (int w = 1; w < kPdsC; ++w) v += sp[w * 16];
    return v;
  };
  // X wave: rms of the folded input from the producer's partial sums (gemv_body XM_F16F)
  auto fold_rms = [&](int n_ss, int K) {
    float ss4[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) ss4[j] = ld_sc1_f32(a.ss + (lane + 64 * j < n_ss ? lane + 64 * j : 0));
    float t = 0.0f;
#pragma unroll
    for (int j = 0; j < 4; ++j) t += lane + 64 * j < n_ss ? ss4[j] : 0.0f;
    t = group_sum<kWave>(t);
    return sqrtf(t / (float)K + a.eps);
  };
  auto fold_rms_g = [&](int n_ss, int K, uint32_t tag) {
    float t = 0.0f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      uint32_t w[1];
      gather_gran<1>(a.ssg + (lane + 64 * j < n_ss ? lane + 64 * j : 0), 1, tag, w, a.err, dead);
      t += lane + 64 * j < n_ss ? __builtin_bit_cast(float, w[0]) : 0.0f;
    }
    t = group_sum<kWave>(t);
    return sqrtf(t / (float)K + a.eps);
  };
  // X wave: residual epilogue of the workgroup's single tile (O, down) with the fold into the
  // next projection's input (epilogue TI_EPI_RESID_F32 with fold_x, M = 1)
  auto resid_fold = [&](const float* nw, uint32_t gtag) {   // gtag 0: plain stores (the lm_head's input)
    const int n = lane & 15;
    const float v = tile_sum(0, n);
    const float fw = gptr(nw)[t0o * 16 + n];
    float ssacc = 0.0f;
    float rr = 0.0f;
    if (lane < 16) {
      rr = h_l[n] + v;
      h_l[n] = rr;
      ssacc = fmaf(rr, rr, ssacc);
    }
    const uint32_t hv = f2h(rr * fw), hp = lane_xor_u32<1>(hv);
    const float sw = group_sum<kWave>(ssacc);
    if (gtag) {
      if (lane < 16 && !(n & 1)) st_gran(a.fxg + (t0o * 16 + n) / 2, hv | (hp << 16), gtag);
      if (lane == 0) st_gran(a.ssg + bid, __builtin_bit_cast(uint32_t, sw), gtag);
    } else {
      if (lane < 16 && !(n & 1)) st_sc1_u32(a.fx + t0o * 16 + n, hv | (hp << 16));
      if (lane == 0) st_sc1_f32(a.ss + bid, sw);
    }
  };

  for (int l = 0; l < a.n_layers; ++l) {
    const PdsLayerDev& ly = a.layers[l];
    uint32_t* cl = a.ctr + (size_t)l * PH_N * kPdsShards * kPdsShardWords;
    auto ctr_of = [&](int ll, int ph) { return a.ctr + ((size_t)ll * PH_N + ph) * kPdsShards * kPdsShardWords; };

    // ---------------- QKV: x = fx (fold of the previous down / step_begin), RoPE + KV append
    {
      const PdsLin p = lin_params(PH_QKV);
      if (is_x) ts(l, PH_QKV, 0);
      if (is_x) ts(l, PH_QKV, 1);
      stage_scales(p, ly.scales[0]);   // constant: before the hand-off
      pds_barrier();
      float rms = 1.0f;
      // layer 0: the fold step_begin wrote before this launch; then the previous down's granules
      if (l == 0) stage_f16(a.fx, H);
      else stage_f16_g(a.fxg, H, pds_tag(epoch, l - 1, PH_DN));
      if (is_x) rms = l == 0 ? fold_rms(a.n_ss0, H) : fold_rms_g(grid, H, pds_tag(epoch, l - 1, PH_DN));
      pds_barrier();
#pragma unroll
      for (int s = kPdsPre; s < kPdsRing; ++s) grefill(gc, ring[s]);   // the input is staged: the rest of the ring
      if (is_x) ts(l, PH_QKV, 2);
      ac = acur(l);   // the attention's first block: issued after the closing barrier
      gemv_phase(p);
      if (wave == 0) ts(l, PH_QKV, 3);
      pds_barrier();
      if (is_x) ts(l, PH_QKV, 4);
      if (!is_x) {   // the control wave issues these after its signal
      }
      if (is_x) {
        // outputs (tl, n) = lane (ntl <= 4): gemv epilogue TI_EPI_QKV_ROPE_KV, M = 1
        const int tl = lane >> 4, n = lane & 15;
        const bool ok = tl < p.ntl;
        const float v = (ok ? tile_sum(tl, n) : 0.0f) / rms;
        const float partner = lane_xor<1>(v);
        const int ng = (p.t0 + tl) * 16 + n;
        const bool qk = ng < 2 * qd;
        float rv = v;
        if (ok && qk) {
          const int base = ng < qd ? 0 : qd;
          const int d = (ng - base) % HD;
          const float2 cs = *(const float2*)(cs_l + (d & ~1));
          rv = (d & 1) == 0 ? fmaf(-partner, cs.y, v * cs.x) : fmaf(v, cs.x, partner * cs.y);
        }
        const uint32_t hv = f2h(rv), hp = lane_xor_u32<1>(hv);
        const uint32_t tq = pds_tag(epoch, l, PH_QKV);
        if (ok) {
          if (ng < qd) {
            st_gran(a.qg + ng, __builtin_bit_cast(uint32_t, rv), tq);
          } else if (!(n & 1)) {
            const bool is_k = qk;
            const int c = ng - qd - (is_k ? 0 : qd);
            const int kh = c / HD, d = c - kh * HD;
            uint16_t* cache = is_k ? ly.k_cache : ly.v_cache;   // for later launches
            gptr_w((uint32_t*)(cache + ((size_t)kh * a.max_seq + pos) * HD + d))[0] = hv | (hp << 16);
            st_gran(a.kvg + ((size_t)kh * 2 + (is_k ? 0 : 1)) * (HD / 2) + d / 2, hv | (hp << 16), tq);
          }
        }
        ts(l, PH_QKV, 5);
      }
      // the next phase's first units: issued once the epilogue's stores have drained (they
      // would queue behind these in the CU's memory pipeline)
      pds_barrier();
#pragma unroll
      for (int s = 0; s < kPdsPre; ++s) arefill(ac, ring[s]);
    }

    // ---------------- attention split (kvh, sp): partials as ti_attn_decode_partials
    {
      if (is_x) {
        ts(l, PH_ATT, 0);
        ts(l, PH_ATT, 1);
        // q of the head and, if this split holds it, the fresh K/V row at pos: QKV's granules
        const uint32_t tq = pds_tag(epoch, l, PH_QKV);
        {
          uint32_t w[2];
          gather_gran<2>(a.qg + kvh * HD + lane, kWave, tq, w, a.err, dead);
          q_l[lane] = __builtin_bit_cast(float, w[0]);
          q_l[lane + kWave] = __builtin_bit_cast(float, w[1]);
        }
        if (pos >= s0 && pos < s1) {
          uint32_t w[2];
          gather_gran<2>(a.kvg + (size_t)kvh * 2 * (HD / 2) + lane, HD / 2, tq, w, a.err, dead);
          ((uint32_t*)kf_l)[lane] = w[0];
          ((uint32_t*)vf_l)[lane] = w[1];
        }
      }
      pds_barrier();
      pds_barrier();
#pragma unroll
      for (int s = kPdsPre; s < kPdsRing; ++s) arefill(ac, ring[s]);
      if (is_x) ts(l, PH_ATT, 2);
      {
        const int dl = lane & 15, kg = lane >> 4;
        float qv[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) qv[e] = q_l[dl * 8 + e] * a.scale;
        float mrun = -INFINITY, lrun = 0.0f, acc[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] = 0.0f;
        int ci = 0;
        auto consume = [&](const u32x4 (&u)[2]) {
          const int key = s0 + (cw + kPdsC * ci) * 4 + kg;
          ++ci;
          const bool valid = key < s1;
          u32x4 kv = u[0], vv = valid ? u[1] : (u32x4){0u, 0u, 0u, 0u};   // dummy units hold stale data
          if (valid && key == pos) {
            kv = *(const u32x4*)(kf_l + dl * 8);
            vv = *(const u32x4*)(vf_l + dl * 8);
          }
          float kf[8], vf[8];
          unpack8(kv, kf);
          unpack8(vv, vf);
          float d = 0.0f;
#pragma unroll
          for (int e = 0; e < 8; ++e) d = fmaf(qv[e], kf[e], d);
          d = group_sum<16>(d);
          const float sc = valid ? d : -INFINITY;
          const float mn = fmaxf(mrun, sc);
          const float alpha = mrun == mn ? 1.0f : __expf(mrun - mn);
          const float pr = valid ? __expf(sc - mn) : 0.0f;
          lrun = fmaf(lrun, alpha, pr);
          mrun = mn;
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[e] = fmaf(pr, vf[e], acc[e] * alpha);
        };
        gc = gcur(l, PH_O);
        auto rin = [&](u32x4 (&slot)[2]) { arefill(ac, slot); };
        pds_blocks(ring, pds_nblk(att_units), consume, rin);
        // merge the lane groups of the wave (attn_split_body, LPK = 16)
        const float mx = groups_max<16>(mrun);
        const float f = mrun == -INFINITY ? 0.0f : __expf(mrun - mx);
        const float lsum = groups_sum<16>(lrun * f);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] = groups_sum<16>(acc[e] * f);
        if (lane < 16) {
#pragma unroll
          for (int e = 0; e < 8; ++e) s_acc[cw * HD + dl * 8 + e] = acc[e];
        }
        if (lane == 0) {
          s_m[cw] = mx;
          s_l[cw] = lsum;
        }
      }
      if (wave == 0) ts(l, PH_ATT, 3);
      pds_barrier();
      if (is_x) ts(l, PH_ATT, 4);
      if (is_x) {
        // merge the waves: dims 2 lane, 2 lane + 1 of head kvh
        float mx = s_m[0];
#pragma unroll
        for (int w = 1; w < kPdsC; ++w) mx = fmaxf(mx, s_m[w]);
        float o2[2] = {0.0f, 0.0f}, lsum = 0.0f;
        if (mx != -INFINITY) {
#pragma unroll
          for (int w = 0; w < kPdsC; ++w) {
            const float f = s_m[w] == -INFINITY ? 0.0f : __expf(s_m[w] - mx);
            o2[0] = fmaf(f, s_acc[w * HD + 2 * lane], o2[0]);
            o2[1] = fmaf(f, s_acc[w * HD + 2 * lane + 1], o2[1]);
            lsum = fmaf(f, s_l[w], lsum);
          }
        }
        const size_t row = (size_t)kvh * kPdsSplits + sp;
        const uint32_t lo = f2h(lsum > 0.0f ? o2[0] / lsum : 0.0f), hi = f2h(lsum > 0.0f ? o2[1] / lsum : 0.0f);
        st_sc1_u32(a.part_o + row * HD + 2 * lane, lo | (hi << 16));
        if (lane == 0)
          st_sc1_u64((unsigned long long*)(a.part_ml + 2 * row),
                     ((unsigned long long)__builtin_bit_cast(uint32_t, lsum) << 32) | __builtin_bit_cast(uint32_t, mx));
        pds_signal(cl + PH_ATT * kPdsShards * kPdsShardWords, bid, lane);
        ts(l, PH_ATT, 5);
      }
      // the next phase's first units: issued once the epilogue's stores have drained (they
      // would queue behind these in the CU's memory pipeline)
      pds_barrier();
#pragma unroll
      for (int s = 0; s < kPdsPre; ++s) grefill(gc, ring[s]);
    }

    // ---------------- O: x = the splits merged (gemv XM_ATTN staging), residual + fold (ffn_norm)
    {
      const PdsLin p = lin_params(PH_O);
      if (is_x) ts(l, PH_O, 0);
      if (is_x) pds_poll(ctr_of(l, PH_ATT), target, a.err, lane, dead);
      if (is_x) ts(l, PH_O, 1);
      stage_scales(p, ly.scales[1]);
      pds_barrier();
      {
        const int K8 = qd >> 3;
        for (int i0 = 0; i0 < K8; i0 += kPdsCThreads) {
          const int idx = i0 + tid;
          float part = 0.0f;
          if (idx < K8) {
            const int hh = (8 * idx) >> 7, d = (8 * idx) & 127;
            float2 pml[kPdsSplits];
            u32x4 po[kPdsSplits];
#pragma unroll
            for (int s = 0; s < kPdsSplits; ++s) {
              pml[s] = __builtin_bit_cast(float2, ld_sc1_u64((const unsigned long long*)(a.part_ml + 2 * (hh * kPdsSplits + s))));
              po[s] = ld_sc1_b128(a.part_o, (uint32_t)(((size_t)(hh * kPdsSplits + s) * HD + d) * 2));
            }
            float mx = -INFINITY;
#pragma unroll
            for (int s = 0; s < kPdsSplits; ++s) mx = fmaxf(mx, pml[s].x);
            float num[8] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f}, den = 0.0f;
#pragma unroll
            for (int s = 0; s < kPdsSplits; ++s) {
              const float f = pml[s].x != -INFINITY ? pml[s].y * __expf(pml[s].x - mx) : 0.0f;
              den += f;
              const f16x8 o = __builtin_bit_cast(f16x8, po[s]);
#pragma unroll
              for (int e = 0; e < 8; ++e) num[e] = fmaf(f, (float)o[e], num[e]);
            }
            f16x8 hx;
#pragma unroll
            for (int e = 0; e < 8; ++e) hx[e] = (f16)(den > 0.0f ? num[e] / den : 0.0f);
            const f16 s16 = (f16)0.0625f;
            hx[2] *= s16; hx[3] *= s16; hx[6] *= s16; hx[7] *= s16;
            *(f16x8*)(xl + 8 * idx) = hx;
            const float lo = ((float)hx[0] + (float)hx[1]) + ((float)hx[4] + (float)hx[5]);
            const float hi = ((float)hx[2] + (float)hx[3]) + ((float)hx[6] + (float)hx[7]);
            part = 1032.0f * lo + 1152.0f * hi;
          }
          part = group_sum<16>(part);
          if (idx < K8 && (lane & 15) == 0) corr[idx >> 4] = part;
        }
      }
      pds_barrier();
#pragma unroll
      for (int s = kPdsPre; s < kPdsRing; ++s) grefill(gc, ring[s]);
      if (is_x) ts(l, PH_O, 2);
      GCur gnx = gcur(l, PH_GU);
      gemv_phase(p);
      if (wave == 0) ts(l, PH_O, 3);
      pds_barrier();
      if (is_x) ts(l, PH_O, 4);
      if (is_x) {
        resid_fold(ly.ffn_norm, pds_tag(epoch, l, PH_O));
        ts(l, PH_O, 5);
      }
      // the next phase's first units: issued once the epilogue's stores have drained (they
      // would queue behind these in the CU's memory pipeline)
      pds_barrier();
#pragma unroll
      for (int s = 0; s < kPdsPre; ++s) grefill(gnx, ring[s]);
      gc = gnx;
    }

    // ---------------- gate/up: x = fx (fold of O), SiLU * up
    {
      const PdsLin p = lin_params(PH_GU);
      if (is_x) ts(l, PH_GU, 0);
      if (is_x) ts(l, PH_GU, 1);
      stage_scales(p, ly.scales[2]);
      pds_barrier();
      float rms = 1.0f;
      stage_f16_g(a.fxg, H, pds_tag(epoch, l, PH_O));
      if (is_x) rms = fold_rms_g(grid, H, pds_tag(epoch, l, PH_O));
      pds_barrier();
#pragma unroll
      for (int s = kPdsPre; s < kPdsRing; ++s) grefill(gc, ring[s]);
      if (is_x) ts(l, PH_GU, 2);
      GCur gnx = gcur(l, PH_DN);
      gemv_phase(p);
      if (wave == 0) ts(l, PH_GU, 3);
      pds_barrier();
      if (is_x) ts(l, PH_GU, 4);
      if (is_x) {
        for (int tb = 0; tb < p.ntl * 16; tb += kWave) {
          const int t = tb + lane, tl = t >> 4, n = lane & 15;
          const bool ok = t < p.ntl * 16;
          const float v = (ok ? tile_sum(tl, n) : 0.0f) / rms;
          const float up = lane_xor<8>(v);
          const float s = v / (1.0f + expf(-v));
          const uint32_t hv = f2h(up * s), hp = lane_xor_u32<1>(hv);
          if (ok && n < 8 && !(n & 1)) st_gran(a.actg + ((p.t0 + tl) * 8 + n) / 2, hv | (hp << 16), pds_tag(epoch, l, PH_GU));
        }
        ts(l, PH_GU, 5);
      }
      // the next phase's first units: issued once the epilogue's stores have drained (they
      // would queue behind these in the CU's memory pipeline)
      pds_barrier();
#pragma unroll
      for (int s = 0; s < kPdsPre; ++s) grefill(gnx, ring[s]);
      gc = gnx;
    }

    // ---------------- down: x = act, residual + fold (next layer's attention_norm / final norm)
    {
      const PdsLin p = lin_params(PH_DN);
      if (is_x) ts(l, PH_DN, 0);
      if (is_x) ts(l, PH_DN, 1);
      stage_scales(p, ly.scales[3]);
      pds_barrier();
      stage_f16_g(a.actg, I, pds_tag(epoch, l, PH_GU));
      pds_barrier();
#pragma unroll
      for (int s = kPdsPre; s < kPdsRing; ++s) grefill(gc, ring[s]);
      if (is_x) ts(l, PH_DN, 2);
      GCur gnx = gcur(l + 1, PH_QKV);
      gemv_phase(p);
      if (wave == 0) ts(l, PH_DN, 3);
      pds_barrier();
      if (is_x) ts(l, PH_DN, 4);
      if (is_x) {
        // the last layer's fold goes to the lm_head launch: plain write-through stores
        resid_fold(l + 1 < a.n_layers ? a.layers[l + 1].attn_norm : a.out_norm,
                   l + 1 < a.n_layers ? pds_tag(epoch, l, PH_DN) : 0u);
        ts(l, PH_DN, 5);
      }
      // the next phase's first units: issued once the epilogue's stores have drained (they
      // would queue behind these in the CU's memory pipeline)
      pds_barrier();
#pragma unroll
      for (int s = 0; s < kPdsPre; ++s) grefill(gnx, ring[s]);
      gc = gnx;
    }
  }
  if (is_x && lane < 16) gptr_w(a.h)[t0o * 16 + lane] = h_l[lane];
}

}  // namespace ti

using namespace ti;

extern "C" {

size_t ti_pds_granule_words(int H, int I, int qd, int heads, int grid) { return pds_gran_words(H, I, qd, heads, grid); }

int ti_pds_decode(const ti_pds_args* h, ti_stream_t s) {
  if (!h || !h->layers || !h->pos || !h->h || !h->fx || !h->ss || !h->q || !h->act || !h->part_o || !h->part_ml ||
      !h->ctr || !h->launches || !h->err || !h->zero || !h->rope_cs || !h->out_norm || !h->gran)
    return ti_set_error(TI_ERR_ARG, "ti_pds_decode: null pointer");
  if (h->n_layers < 1 || h->n_layers > 64)
    return ti_set_error(TI_ERR_UNSUPPORTED, "ti_pds_decode: %d layers (granule tags hold 64)", h->n_layers);
  if (h->head_dim != kPdsHd || h->heads != h->kv_heads || h->heads * kPdsSplits != h->grid || h->grid > 256 ||
      h->qd != h->heads * h->head_dim || h->H % 128 || h->I % 128 || h->qd % 128 || h->H / 16 != h->grid ||
      h->qd > 4096 || h->I + 8 > kLdsXBytes / 2 || h->H + 8 > kLdsXBytes / 2)
    return ti_set_error(TI_ERR_UNSUPPORTED, "ti_pds_decode: shape not supported (heads %d kv %d hd %d grid %d H %d I %d)",
                        h->heads, h->kv_heads, h->head_dim, h->grid, h->H, h->I);
  // per-workgroup tile counts must fit the slab and scale images
  const int nts[3] = {3 * h->qd / 16, 2 * h->I / 16, h->H / 16};
  const int kts[3] = {h->H / 128, h->H / 128, h->I / 128};
  for (int i = 0; i < 3; ++i) {
    const int ntl = (nts[i] + h->grid - 1) / h->grid;
    if (ntl > kPdsMaxNtl || ntl * kts[i] * 32 > kLdsScBytes || kts[i] * 4 > 512)
      return ti_set_error(TI_ERR_UNSUPPORTED, "ti_pds_decode: %d tiles per workgroup", ntl);
  }
  if ((3 * h->qd / 16 + h->grid - 1) / h->grid > 4)
    return ti_set_error(TI_ERR_UNSUPPORTED, "ti_pds_decode: QKV tiles per workgroup > 4");
  PdsArgs a{};
  a.layers = (const PdsLayerDev*)h->layers;
  a.n_layers = h->n_layers;
  a.H = h->H;
  a.I = h->I;
  a.qd = h->qd;
  a.max_seq = h->max_seq;
  a.n_ss0 = h->n_ss0;
  a.eps = h->eps;
  a.scale = 1.0f / sqrtf((float)h->head_dim);
  a.pos = h->pos;
  a.rope_cs = h->rope_cs;
  a.out_norm = h->out_norm;
  a.h = h->h;
  a.fx = h->fx;
  a.ss = h->ss;
  a.q = h->q;
  a.act = h->act;
  a.part_o = h->part_o;
  a.part_ml = h->part_ml;
  a.ctr = h->ctr;
  a.launches = h->launches;
  a.err = h->err;
  a.zero = (const u32x4*)h->zero;
  a.ts = h->ts;
  a.fxg = h->gran;
  a.ssg = a.fxg + h->H / 2;
  a.qg = a.ssg + h->grid;
  a.kvg = a.qg + h->qd;
  a.actg = a.kvg + (size_t)h->heads * kPdsHd;
  // per device: the LDS attribute, and co-residency -- every wait in the kernel needs all `grid`
  // workgroups resident at once (one per CU): the occupancy query times the CU count must cover
  // the grid, or nothing is launched.  (Residency taken by other work at run time is caught by
  // the bounded waits: pds_err, fatal in the engine's hand-off check.)
  static unsigned long long attr = 0;
  static int resident[64] = {0};
  int dev = 0;
  TI_HIP_CHECK(hipGetDevice(&dev), "hipGetDevice");
  dev &= 63;
  if (!(attr >> dev & 1ull)) {
    TI_HIP_CHECK(hipFuncSetAttribute((const void*)pds_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes),
                 "hipFuncSetAttribute(pds_kernel)");
    int per_cu = 0, cus = 0;
    TI_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)pds_kernel, kPdsThreads, kLdsBytes),
                 "hipOccupancyMaxActiveBlocksPerMultiprocessor(pds_kernel)");
    TI_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev), "hipDeviceGetAttribute(CUs)");
    resident[dev] = per_cu * cus;
    attr |= 1ull << dev;
  }
  if (resident[dev] < h->grid)
    return ti_set_error(TI_ERR_UNSUPPORTED, "ti_pds_decode: %d workgroups cannot all be resident (%d)", h->grid,
                        resident[dev]);
  hipLaunchKernelGGL(pds_kernel, dim3(h->grid), dim3(kPdsThreads), kLdsBytes, (hipStream_t)s, a);
  TI_LAUNCH_CHECK("pds_kernel");
  return TI_OK;
}

}  // extern "C"
