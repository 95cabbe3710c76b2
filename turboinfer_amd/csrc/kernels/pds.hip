// pds.hip -- the decode layers of one single-stream step in ONE persistent launch (gfx950),
// built as a weight-streaming engine: per CU a loader wave runs ahead through an LDS ring.
//
// Replaces the per-layer launch chain of the decode step (QKV, attention, O, gate/up, down:
// TransformerLayer::forward_incremental, src/model/inference_engine.cpp:203-279, 291-368,
// 376-401, with the matmuls of tensor_engine.cpp:594-640 and attention_fast_incremental
// :1254-1388; the layer loop of forward_pass_incremental :1525-1530) for one stream with INT4 or
// INT8 group-128 weights, head_dim 64 or 128, MHA or GQA, grid = 8 * heads workgroups (one per CU:
// Llama-2-7B and TinyLlama-1.1B both 256).
//
// Why: a layer as five launches pays, per launch, the kernel boundary plus the latency from launch
// to the first weight bytes (~4.1 us per launch, 5 per layer).  Here each CU's weight /
// K/V bytes for ALL layers are one stream that never waits for a dependency: while the CU's
// consumers wait for the previous phase's output vector, its loader keeps filling the ring with the
// next phases' bytes (MI355X_MICROARCH.md price list: prefetch-credit, ldsdma-fill, engine-vs-launches).
//
// Shape: one 5-wave workgroup per CU.
//   * wave 4, the LOADER: issues the CU's stream as global_load_lds_dwordx4 ... nt (1 KiB per wave
//     instruction, "a piece") into a ring of n_slots 16 KiB slots in LDS; publishes a slot (LDS word
//     FULL) behind a counted vmcnt that leaves up to 2 more slots in flight (1 while the CU gathers:
//     gather-pass); reuses a slot once all four consumers released it (LDS words FREE[c]).
//   * waves 0-3, the CONSUMERS: dequant + v_mfma_f32_16x16x32_f16 out of the ring (GEMV phases) or
//     the online softmax over K/V pieces (attention); they emulate the per-layer kernels' 8 waves
//     (virtual wave v = k-tile % 8 or key slot % 8, consumer v % 4), so every partial sum is formed
//     in the same order as gemv_wq_kernel / attn_split_body and results are bit-identical to the
//     graph path.  Consumer 0 also runs the epilogues (tile sums in the fixed wave order, residual +
//     folded rms_norm, RoPE + KV append, SiLU*up, the split merge) and publishes.  Consumers meet at
//     LDS counter barriers (the loader never takes part in a barrier).
// Hand-offs: data-tagged 8-byte granules {payload, tag} (one sc1 store each, no flag, no fence),
// gathered by the consumers with sc1 loads until every tag is this launch's (MI355X_MICROARCH.md
// handoff-1to1 / allgather; cdna_hip_programming.md Guideline 16 R2).  Per layer:
//   down(l-1) -> QKV: h folded with attn_norm (fp16 pairs) + one sum of h^2 per tile    all-to-all
//   QKV -> attention: q of head h, the fresh K, V row of its kv-head                     few-to-one
//   attention -> merge: split partials of head h from its 8 splits                       head group
//   merge -> O: the merged attention output (fp16 pairs)                                all-to-all
//   O -> gate/up: h folded with ffn_norm + sums of h^2                                  all-to-all
//   gate/up -> down: SiLU(gate) * up (fp16 pairs)                                       all-to-all
// Workgroup b = (head h = b % heads, split s = b / heads): the 8 splits of a head share an XCD
// (round-robin placement; speed only).  QKV: for MHA with head_dim 128 and q_dim / 16 == grid, CU
// (h, s) computes q / k / v tile 8h + s of each, so the attention's inputs come from its own head
// group; otherwise tiles [b NT / grid, (b + 1) NT / grid).  O / down: tile b (b < hidden / 16);
// gate/up: tiles [b NT / grid, (b + 1) NT / grid) -- the per-layer kernels' partition.
// Every wait is bounded (~50 ms): on expiry the workgroup sets a shared LDS dead flag and *err, every
// later wait of every wave passes at once, and every other workgroup leaves its waits on seeing *err,
// so a broken hand-off costs one timeout per launch; the engine treats it as fatal.
#include <math.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <vector>

#include "common.hpp"
#include "attention_body.hpp"
#include "dequant.hpp"

namespace ti {

#ifndef TI_PDS_LOADERS
#define TI_PDS_LOADERS 4   // loader waves (1, 2 or 4): one wave's VMEM issue is ~0.1 us per 1 KiB piece here
#endif
#ifndef TI_PDS_CONSUMERS
#define TI_PDS_CONSUMERS 8   // consumer waves (4 or 8): each runs 8 / kEC of the per-layer kernels' 8 waves
#endif
constexpr int kEC = TI_PDS_CONSUMERS;           // consumer waves
constexpr int kNL = TI_PDS_LOADERS;            // loader waves kEC .. kEC + kNL - 1
constexpr int kEThreads = (kEC + kNL) * kWave;
static_assert(kNL == 1 || kNL == 2 || kNL == 4, "loader waves");
static_assert(kEC == 4 || kEC == 8, "consumer waves");
constexpr int kVPC = 8 / kEC;                  // virtual waves per consumer: c, c + kEC, ...
constexpr int kVW = 8;                         // virtual waves: the per-layer kernels' 8 waves
constexpr int kPiece = 1024;                   // bytes per LDS-DMA wave instruction
constexpr int kFill = 16;                      // pieces per ring slot
constexpr int kSlotBytes = kFill * kPiece;
constexpr int kMaxSlots = 8;
constexpr int kSplits = 8;
constexpr int kHdMax = 128;
constexpr int kMaxQkvTiles = 4, kMaxGuTiles = 8;
enum { PH_QKV = 0, PH_ATT, PH_O, PH_GU, PH_DN, PH_MRG, PH_N = 5 };
// FULL: fills loader 0 has published (loaders w > 0: C_FULLX + w - 1); FREE + c: fills consumer c released
enum { C_FULL = 0, C_FREE = 1, C_BAR = 1 + kEC, C_GATHER = 2 + kEC, C_DEAD = 3 + kEC, C_EPOCH = 4 + kEC,
       C_FULLX = 5 + kEC, C_WORDS = 16 };
static_assert(C_FULLX + kNL - 1 <= C_WORDS, "control words");
#ifndef TI_PDS_THIN
#define TI_PDS_THIN 1   // the loader keeps one slot in flight while its consumers gather (gather-pass)
#endif
#ifndef TI_PDS_AHEAD
#define TI_PDS_AHEAD 3  // slots in flight otherwise (vmcnt 16 * AHEAD <= 63)
#endif
static_assert(TI_PDS_AHEAD >= 1 && TI_PDS_AHEAD * (16 / TI_PDS_LOADERS) <= 63, "vmcnt immediate");
#ifndef TI_PDS_NT
#define TI_PDS_NT 1       // loader DMA non-temporal (0: default policy; diagnostic A/B)
#endif
#ifndef TI_PDS_PRIO
#define TI_PDS_PRIO 0     // diagnostic: the loader wave at s_setprio 3
#endif
#ifndef TI_PDS_DIAG
#define TI_PDS_DIAG 0     // diagnostic builds only: 1 consumers only acquire / release the ring (no math, no
                          // hand-offs: garbage results); 2 the loader re-reads layer 0's QKV tiles (L2);
                          // 4 the GEMV phases skip their math (garbage results, hand-offs kept);
                          // 8 granule gathers take what they find (no tag waits: garbage results)
#endif
#ifndef TI_PDS_FTRACE
#define TI_PDS_FTRACE 0   // diagnostic build (tools/pds_ftrace.py): per-fill ring events of workgroups 0..3
#endif
#if TI_PDS_FTRACE
constexpr int kFtWg = 4, kFtFills = 2048;
// [wg][fill][k]: 0 loader issue begins, 1 loader publishes it (FULL > fill), 2 consumer 0's wait
// for it ends, 3 consumer 0 releases it, 4 the loader starts waiting for a FREE slot before it,
// 5 that wait ends, 6 the loader's last piece of it issued, 7 consumer 0's math on it done (GEMV)
static __device__ unsigned long long g_pds_ft[kFtWg][kFtFills][8];
#define PDS_FT(f, k)                                                                                  \
  do {                                                                                                \
    if (blockIdx.x < kFtWg && (f) < (uint32_t)kFtFills && lane == 0)                                  \
      g_pds_ft[blockIdx.x][(f)][(k)] = __builtin_amdgcn_s_memrealtime();                              \
  } while (0)
#else
#define PDS_FT(f, k) do { } while (0)
#endif

typedef ti_pds_layer PdsLayerDev;

struct PdsArgs {
  const PdsLayerDev* layers;
  int n_layers, H, I, qd, kvd, max_seq, n_ss0, heads, kv_shift, grid, n_slots, nt_h, head_group;
  float eps, scale;
  const int32_t* pos;
  const float* rope_cs;     // [max_seq][hd] (cos, sin) pairs
  const float* out_norm;
  float* h;                 // [H] residual (read at start, written at end)
  uint16_t* fx;             // [H] fp16 h * next norm weight: layer 0's input, the lm_head's output
  float* ss;                // [nt_h] sums of h^2 (likewise)
  uint32_t* launches;       // [grid] private launch counts (granule epochs)
  uint32_t* err;            // bit 0: a hand-off wait timed out
  const char* zero;         // >= 1 KiB of zeros, never written: dummy / masked DMA source
  unsigned long long* ts;   // diagnostic phase timestamps [grid][layers][5][8] or null
  int drop_wg;              // diagnostic: this workgroup withholds its layer-0 down granules (-1: none)
  // granules (8-byte {payload, tag}, one sc1 store / sc1 load each)
  unsigned long long* fxg;    // [H / 2]: fp16 pairs of the fold (O -> gate/up, down -> next QKV)
  unsigned long long* ssg;    // [nt_h]: the fold's sums of h^2, one per O / down tile
  unsigned long long* qg;     // [qd]: RoPE'd q, fp32
  unsigned long long* kvg;    // [kv_heads][2][hd / 2]: the fresh K, V rows (fp16 pairs)
  unsigned long long* partg;  // [heads][8 splits][hd / 2 + 2]: split partials
  unsigned long long* aog;    // [qd / 2]: the merged attention output (fp16 pairs)
  unsigned long long* actg;   // [I / 2]: SiLU * up (fp16 pairs)
  // LDS layout (bytes)
  int l_x, l_sc, l_corr, l_slab, l_att, l_ctl, l_total;
};

__host__ __device__ inline size_t pds_gran_words(int H, int I, int qd, int heads, int grid) {
  // (kv rows sized for MHA at head_dim 128: an upper bound for every supported shape)
  return (size_t)H / 2 + (size_t)grid + (size_t)qd + (size_t)heads * kHdMax + (size_t)heads * kSplits * (kHdMax / 2 + 2) +
         (size_t)qd / 2 + (size_t)I / 2;
}

__device__ __forceinline__ uint32_t pds_tag(uint32_t epoch, int l, int ph) {
  return ((epoch * 64u + (uint32_t)l) * 8u + (uint32_t)ph) + 1u;
}

// Pointers reach the kernel through the layer table (generic): cast them to the global address
// space, or the compiler emits flat loads, which also count in lgkmcnt.
template <class T>
__device__ __forceinline__ const __attribute__((address_space(1))) T* gptr(const T* p) {
  return (const __attribute__((address_space(1))) T*)p;
}
template <class T>
__device__ __forceinline__ __attribute__((address_space(1))) T* gptr_w(T* p) {
  return (__attribute__((address_space(1))) T*)p;
}
// The layer table is read-only for the whole launch: read it through the constant address space, so
// its fields come by scalar loads (lgkmcnt).  As plain global loads they were VECTOR loads whose
// s_waitcnt vmcnt(0) drained every LDS-DMA in flight: once per phase, and once per attention piece
// (the K / V base pointer), where it serialised the loader (fill trace: 6.4 us per 16 KiB fill).
typedef const __attribute__((address_space(4))) PdsLayerDev* CLayer;
__device__ __forceinline__ CLayer layer_c(const PdsLayerDev* t, int l) { return (CLayer)t + l; }
__device__ __forceinline__ u32x4 ld_sc1_b128(const void* base, uint32_t byte_off) {
  return __builtin_amdgcn_raw_buffer_load_b128(sc1_rsrc(base), byte_off, 0, kAuxSc1Load);
}
__device__ __forceinline__ void st_gran(unsigned long long* p, uint32_t payload, uint32_t tag) {
  st_sc1_u64(p, ((unsigned long long)tag << 32) | payload);
}

// LDS control words: relaxed workgroup-scope atomics (ds_read / ds_write / ds_add)
__device__ __forceinline__ uint32_t cget(uint32_t* c) { return __hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
__device__ __forceinline__ void cset(uint32_t* c, uint32_t v) { __hip_atomic_store(c, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }

constexpr unsigned long long kSpinTicks = 5000000ull;   // ~50 ms of s_memrealtime (100 MHz)

// One bounded wait: tick() once per unsuccessful poll; false = give up (this workgroup is dead:
// its own expiry, an earlier one of another wave, or *err set by another workgroup).
struct Spin {
  uint32_t* ctl;
  const uint32_t* err;
  unsigned long long t0 = 0;
  uint32_t n = 0;
  __device__ bool check() {
    if (cget(ctl + C_DEAD)) return false;
    if (n == 0) t0 = __builtin_amdgcn_s_memrealtime();
    ++n;
    if ((n & 63) == 0) {
      const bool remote = ld_sc1_u32(err) != 0u;
      if (remote || __builtin_amdgcn_s_memrealtime() - t0 > kSpinTicks) {
        if (!remote) atomicOr((uint32_t*)err, 1u);
        cset(ctl + C_DEAD, 1u);
        return false;
      }
    }
    return true;
  }
  // polls of LDS words: a short sleep
  __device__ bool tick() {
    if (!check()) return false;
    __builtin_amdgcn_s_sleep(1);
    return true;
  }
  // re-polls of granules in memory (sc1 loads that reach L2): every CU of the grid may be polling
  // at once, and the re-loads compete with the weight streams for L2 / the CUs' load pipelines,
  // so they back off ~0.2 us (s_sleep 8 = 512 clocks) and poll one batch at a time (stage_x)
  __device__ bool tick_g() {
    if (!check()) return false;
    __builtin_amdgcn_s_sleep(8);
    return true;
  }
};

// Consumer barrier: monotonic LDS counter, every consumer wave arrives once per call.
__device__ __forceinline__ void cbar(uint32_t* ctl, const uint32_t* err, uint32_t& gen, int lane) {
  gen += kEC;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (lane == 0) __hip_atomic_fetch_add(ctl + C_BAR, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  Spin sp{ctl, err};
  while (cget(ctl + C_BAR) < gen)
    if (!sp.tick()) break;
  asm volatile("" ::: "memory");
}

// 64 lanes x 16 B -> LDS at the wave-uniform byte address lds, non-temporal (streamed once)
__device__ __forceinline__ void dma_nt(const void* src_lane, uint32_t lds) {
  uint32_t keep;
#if TI_PDS_NT
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
#else
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
#endif
               : "=&s"(keep)
               : "v"(src_lane), "s"(lds)
               : "memory");
}

// Per-workgroup geometry, the same for every layer.
struct PdsGeo {
  int h, s, kvh;           // q-head, split, kv-head
  int L, s0, s1, nslot;    // keys [s0, s1) of the split, in slots of KPW keys (one piece each)
  int KTh, KTq, KTi;       // k-tiles of H, qd, I
  int q0, qs, qn;          // QKV tiles q0 + t * qs, t < qn
  int gu0, gun;            // gate/up tiles
  int on;                  // O / down: tile bid (1) or none (0)
};
template <int HD>
__device__ __forceinline__ PdsGeo pds_geo(const PdsArgs& a, int bid, int pos) {
  constexpr int KPW = 64 / (HD / 8);
  PdsGeo g;
  g.h = bid % a.heads;
  g.s = bid / a.heads;
  g.kvh = g.h >> a.kv_shift;
  g.L = pos + 1;
  const int chunk = (g.L + kSplits - 1) / kSplits;
  g.s0 = g.s * chunk;
  g.s1 = min(g.L, g.s0 + chunk);
  g.nslot = g.s1 > g.s0 ? (g.s1 - g.s0 + KPW - 1) / KPW : 0;
  g.KTh = a.H >> 7;
  g.KTq = a.qd >> 7;
  g.KTi = a.I >> 7;
  if (a.head_group) {   // MHA, head_dim 128, qd / 16 == grid: q / k / v tile 8h + s
    g.q0 = g.h * (HD / 16) + g.s;
    g.qs = a.qd >> 4;
    g.qn = 3;
  } else {
    const int NT = (a.qd + 2 * a.kvd) >> 4;
    g.q0 = (int)((unsigned)bid * (unsigned)NT / (unsigned)a.grid);
    g.qn = (int)((unsigned)(bid + 1) * (unsigned)NT / (unsigned)a.grid) - g.q0;
    g.qs = 1;
  }
  const int NTg = (2 * a.I) >> 4;
  g.gu0 = (int)((unsigned)bid * (unsigned)NTg / (unsigned)a.grid);
  g.gun = (int)((unsigned)(bid + 1) * (unsigned)NTg / (unsigned)a.grid) - g.gu0;
  g.on = bid < a.nt_h ? 1 : 0;
  return g;
}
// pieces of a phase (C pieces per weight item)
template <int C>
__device__ __forceinline__ int pds_pieces(const PdsGeo& g, int ph) {
  return ph == PH_QKV ? g.qn * g.KTh * C : ph == PH_ATT ? 2 * g.nslot : ph == PH_O ? g.on * g.KTq * C
         : ph == PH_GU ? g.gun * g.KTh * C : g.on * g.KTi * C;
}
__device__ __forceinline__ int pds_fills(int np) { return (np + kFill - 1) / kFill; }

// ------------------------------------------------------------------------------------- loader
template <int BITS, int HD>
__device__ __forceinline__ void pds_loader(const PdsArgs& a, const PdsGeo& g, int bid, int pos, uint32_t ring_lds,
                                           uint32_t* ctl, int lane, int wl) {
  // loader wl issues pieces wl, wl + kNL, ... of every fill (at kNL = 2 / 4 the attention's K and V
  // pieces go to different waves) and publishes its own FULL word
  constexpr int C = BITS / 4;
  constexpr int LPK = HD / 8, KPW = 64 / LPK;
  constexpr int PPL = kFill / kNL;   // pieces per loader and fill
  const int NS = a.n_slots;
  const bool ft = wl == 0;           // the trace / timestamps: loader 0
  uint32_t* full_w = ctl + (wl == 0 ? (int)C_FULL : (int)C_FULLX + wl - 1);
  uint32_t f = 0, pub = 0;   // fills issued / published
  auto publish = [&](uint32_t upto) {
    if (upto > pub) {
#if TI_PDS_FTRACE
      if (ft)
        for (uint32_t q = pub; q < upto; ++q) PDS_FT(q, 1);
#endif
      pub = upto;
      cset(full_w, pub);
    }
  };
  auto min_free = [&]() {
    uint32_t m = cget(ctl + C_FREE);
#pragma unroll
    for (int c = 1; c < kEC; ++c) m = min(m, cget(ctl + C_FREE + c));
    return m;
  };
#if TI_PDS_PRIO
  __builtin_amdgcn_s_setprio(3);
#endif
  const char* zl = a.zero + lane * 16;
  const size_t kv_off = ((size_t)g.kvh * a.max_seq) * HD * 2;   // bytes: this split's kv-head
  for (int l = 0; l < a.n_layers; ++l) {
    const CLayer ly = layer_c(a.layers, l);
    const char* const kcache = (const char*)ly->k_cache;
    const char* const vcache = (const char*)ly->v_cache;
    for (int ph = 0; ph < PH_N; ++ph) {
      const int np = pds_pieces<C>(g, ph), nf = pds_fills(np);
      if (a.ts && ft && lane == 0) a.ts[(((size_t)bid * a.n_layers + l) * PH_N + ph) * 8 + 6] = __builtin_amdgcn_s_memrealtime();
      // GEMV phases: piece i = chunk i % C of item i / C = (tile t0 + (item / KT) * ts, k-tile item % KT)
      const char* wbase = nullptr;
      int KT = 1, t0 = 0, tstr = 1;
      if (ph == PH_QKV) { wbase = (const char*)ly->tiles[0]; KT = g.KTh; t0 = g.q0; tstr = g.qs; }
      else if (ph == PH_O) { wbase = (const char*)ly->tiles[1]; KT = g.KTq; t0 = bid; }
      else if (ph == PH_GU) { wbase = (const char*)ly->tiles[2]; KT = g.KTh; t0 = g.gu0; }
      else if (ph == PH_DN) { wbase = (const char*)ly->tiles[3]; KT = g.KTi; t0 = bid; }
      const int SEG = KT * C;   // pieces per tile
      for (int fi = 0; fi < nf; ++fi) {
        // the slot must be released by every consumer
        if (f >= (uint32_t)NS) {
          const uint32_t need = f - NS + 1;
          if (min_free() < need) {
            if (ft) PDS_FT(f, 4);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            publish(f);
            Spin sp{ctl, a.err};
            while (min_free() < need)
              if (!sp.tick()) break;
            if (ft) PDS_FT(f, 5);
          }
        }
        if (ft) PDS_FT(f, 0);
        const uint32_t base = ring_lds + (uint32_t)(f % NS) * kSlotBytes;
        // split tiles (tstr > 1): this loader's first piece of the fill as (tile seg, piece ii), one
        // division per fill, then stepped (a fill may span several short tiles)
        int seg = tstr == 1 ? 0 : (fi * kFill + wl) / SEG;
        int ii = fi * kFill + wl - seg * SEG;
#pragma unroll
        for (int jj = 0; jj < PPL; ++jj) {
          const int j = wl + jj * kNL, i = fi * kFill + j;
          const char* src = zl;
          if (i < np) {
            if (ph == PH_ATT) {
              const int slot = i >> 1, key = g.s0 + KPW * slot + lane / LPK;
              // keys of the next split, past L, and the row this launch writes (pos) are not read
              if (key < g.s1 && key != pos)
                src = ((i & 1) ? vcache : kcache) + kv_off + (size_t)key * HD * 2 + (lane % LPK) * 16;
            } else {
              src = wbase + ((size_t)(t0 + seg * tstr) * SEG + ii) * kPiece + lane * 16;
            }
          }
          ii += kNL;
          if (tstr != 1)
            while (ii >= SEG) {
              ii -= SEG;
              ++seg;
            }
#if TI_PDS_DIAG & 2   // diagnostic: every piece from this CU's own 96 KiB of layer 0's QKV tiles (L2 hits)
          src = (const char*)layer_c(a.layers, 0)->tiles[0] + ((size_t)bid * 96 + (size_t)(i % 96)) * kPiece + lane * 16;
#endif
          dma_nt(src, __builtin_amdgcn_readfirstlane(base + j * kPiece));
        }
        if (ft) PDS_FT(f, 6);
        ++f;
        if (TI_PDS_THIN && cget(ctl + C_GATHER)) {
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PPL) : "memory");
          publish(f - 1);
        } else {
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PPL * TI_PDS_AHEAD) : "memory");
          if (f >= TI_PDS_AHEAD) publish(f - TI_PDS_AHEAD);
        }
      }
      if (a.ts && ft && lane == 0) a.ts[(((size_t)bid * a.n_layers + l) * PH_N + ph) * 8 + 7] = __builtin_amdgcn_s_memrealtime();
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  publish(f);
}

// ----------------------------------------------------------------------------------- consumers
template <int BITS, int HD>
__global__ __launch_bounds__(kEThreads, 1) void pds_kernel(const PdsArgs a) {
  constexpr int C = BITS / 4;                  // pieces per weight item (16 rows x 128 k)
  constexpr int IPF = kFill / C;               // items per fill
  constexpr int LPK = HD / 8, KPW = 64 / LPK;  // attention: lanes per key row, keys per slot (one piece)
  constexpr int NPS = HD / 16;                 // fp16 pairs per split and CU in the head-group merge
  constexpr int PG = HD / 2 + 2;               // granules per split partial
  extern __shared__ __attribute__((aligned(16))) char smem[];
  f16* xl = (f16*)(smem + a.l_x);
  uint16_t* sl = (uint16_t*)(smem + a.l_sc);
  float* corr = (float*)(smem + a.l_corr);
  float* slab = (float*)(smem + a.l_slab);          // [ntl][8 virtual waves][16]
  float* s_acc = (float*)(smem + a.l_att);          // [8][HD]
  float* s_m = s_acc + kVW * kHdMax;                // [8]
  float* s_l = s_m + kVW;                           // [8]
  float* q_l = s_l + kVW;                           // [HD] q of the head
  uint16_t* kf_l = (uint16_t*)(q_l + kHdMax);       // fresh K row [HD], V row [HD] fp16
  uint16_t* vf_l = kf_l + kHdMax;
  float* cs_l = (float*)(vf_l + kHdMax);            // RoPE (cos, sin) [HD]
  float* h_l = cs_l + kHdMax;                       // residual rows [16]
  float* mg_o = h_l + 16;                           // split merge: [8 splits][HD / 8 dims]
  float* mg_ml = mg_o + kSplits * 16;               // [8][2]
  uint32_t* ctl = (uint32_t*)(smem + a.l_ctl);
  const uint32_t ring_lds = (uint32_t)(uintptr_t)smem;   // the ring starts the LDS image

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int bid = blockIdx.x;
  const int pos = __builtin_amdgcn_readfirstlane(gptr(a.pos)[0]);
  const PdsGeo g = pds_geo<HD>(a, bid, pos);
  const int H = a.H, I = a.I, qd = a.qd, kvd = a.kvd;

  // ---- setup (the one workgroup barrier of the launch)
  if (wave == 0) {
    uint32_t epoch = 0;
    if (lane == 0) {
      epoch = gptr(a.launches)[bid];
      gptr_w(a.launches)[bid] = epoch + 1;
    }
    epoch = __builtin_amdgcn_readfirstlane(epoch);
    const uint32_t dead0 = ld_sc1_u32(a.err) != 0u ? 1u : 0u;
    if (lane < C_WORDS) ctl[lane] = lane == C_EPOCH ? epoch : lane == C_DEAD ? dead0 : 0u;
    if (lane < 16 && g.on) h_l[lane] = gptr(a.h)[bid * 16 + lane];
    for (int j = lane; j < HD; j += kWave) cs_l[j] = gptr(a.rope_cs)[(size_t)pos * HD + j];
  }
  __syncthreads();
  if (wave >= kEC) {
    pds_loader<BITS, HD>(a, g, bid, pos, ring_lds, ctl, lane, wave - kEC);
    return;
  }
  const uint32_t epoch = __builtin_amdgcn_readfirstlane(cget(ctl + C_EPOCH));
  const int c = wave;                 // consumer index
  const int ctid = tid;               // 0 .. 255 over the consumers
  uint32_t bar_gen = 0;
  auto bar = [&]() { cbar(ctl, a.err, bar_gen, lane); };
  auto ts = [&](int l, int ph, int k) {
    if (a.ts != nullptr && c == 0 && lane == 0)
      a.ts[(((size_t)bid * a.n_layers + l) * PH_N + ph) * 8 + k] = __builtin_amdgcn_s_memrealtime();
  };
  uint32_t magic;
  asm volatile("v_mov_b32 %0, 0x64006400" : "=v"(magic));
  const int r = lane & 15, kq = lane >> 4;
  uint32_t fbase = 0;   // ring fill of the current phase's first piece

  // ---- gathers
  // An fp16 vector of K (K/2 granules, or K halves in plain memory) staged into xl by all four
  // consumers; int4: with the high-nibble slots pre-scaled by 1/16 and the offset correction corr[kt]
  // (gemv_body's int4 pass, M = 1).
  auto stage_x = [&](const void* src, int K, uint32_t tag, bool plain) {
    const int K8 = K >> 3;
    constexpr int B = 6;
    for (int i0 = 0; i0 < K8; i0 += B * kEC * kWave) {
      u32x4 gv[B][2];
#pragma unroll
      for (int b = 0; b < B; ++b) {
        const int idx = min(i0 + b * kEC * kWave + ctid, K8 - 1);
        gv[b][0] = gv[b][1] = (u32x4){0u, tag, 0u, tag};
        if (i0 + b * kEC * kWave >= K8) continue;   // uniform: past the vector
        if (plain) {
          gv[b][0] = ld_sc1_b128(src, (uint32_t)idx * 16u);
          gv[b][1] = gv[b][0];
        } else {
          gv[b][0] = ld_sc1_b128(src, (uint32_t)idx * 32u);
          gv[b][1] = ld_sc1_b128(src, (uint32_t)idx * 32u + 16u);
        }
      }
      if (!plain && !(TI_PDS_DIAG & 8)) {
        auto ok_b = [&](int b) {
          return gv[b][0][1] == tag && gv[b][0][3] == tag && gv[b][1][1] == tag && gv[b][1][3] == tag;
        };
        Spin sp{ctl, a.err};
        while (true) {
          // the first batch with a granule of an earlier launch in any lane (wave-uniform)
          int first = -1;
#pragma unroll
          for (int b = 0; b < B; ++b)
            if (first < 0 && __builtin_amdgcn_ballot_w64(!ok_b(b)) != 0ull) first = b;
          if (first < 0) break;
          if (!sp.tick_g()) break;
#pragma unroll
          for (int b = 0; b < B; ++b) {
            if (b == first && !ok_b(b)) {
              const int idx = min(i0 + b * kEC * kWave + ctid, K8 - 1);
              gv[b][0] = ld_sc1_b128(src, (uint32_t)idx * 32u);
              gv[b][1] = ld_sc1_b128(src, (uint32_t)idx * 32u + 16u);
            }
          }
        }
      }
#pragma unroll
      for (int b = 0; b < B; ++b) {
        const int idx = i0 + b * kEC * kWave + ctid;
        float part = 0.0f;
        if (idx < K8) {
          const u32x4 w = plain ? gv[b][0] : (u32x4){gv[b][0][0], gv[b][0][2], gv[b][1][0], gv[b][1][2]};
          f16x8 hx = __builtin_bit_cast(f16x8, w);
          if constexpr (BITS == 4) {
            const f16 s16 = (f16)0.0625f;
            hx[2] *= s16; hx[3] *= s16; hx[6] *= s16; hx[7] *= s16;
            const float lo = ((float)hx[0] + (float)hx[1]) + ((float)hx[4] + (float)hx[5]);
            const float hi = ((float)hx[2] + (float)hx[3]) + ((float)hx[6] + (float)hx[7]);
            part = 1032.0f * lo + 1152.0f * hi;
          }
          *(f16x8*)(xl + 8 * idx) = hx;
        }
        if constexpr (BITS == 4) {
          part = group_sum<16>(part);
          if (idx < K8 && (lane & 15) == 0) corr[idx >> 4] = part;
        }
      }
    }
  };
  // rms of the folded input from n_ss producer sums (gemv_body XM_F16F), consumer 0
  auto fold_rms = [&](const void* src, int n_ss, int K, uint32_t tag, bool plain) {
    float t = 0.0f;
    uint32_t w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = lane + 64 * j < n_ss ? lane + 64 * j : 0;
      w[j] = plain ? ld_sc1_u32((const float*)src + i) : 0u;
    }
    if (!plain) {
      unsigned long long v[4];
      constexpr bool kPoll = !(TI_PDS_DIAG & 8);
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = ld_sc1_u64((const unsigned long long*)src + (lane + 64 * j < n_ss ? lane + 64 * j : 0));
      Spin sp{ctl, a.err};
      while (kPoll) {
        bool ok = true;
#pragma unroll
        for (int j = 0; j < 4; ++j) ok = ok && (uint32_t)(v[j] >> 32) == tag;
        if (__builtin_amdgcn_ballot_w64(!ok) == 0ull) break;
        if (!sp.tick_g()) break;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if ((uint32_t)(v[j] >> 32) != tag)
            v[j] = ld_sc1_u64((const unsigned long long*)src + (lane + 64 * j < n_ss ? lane + 64 * j : 0));
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) w[j] = (uint32_t)v[j];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) t += lane + 64 * j < n_ss ? __builtin_bit_cast(float, w[j]) : 0.0f;
    t = group_sum<kWave>(t);
    return sqrtf(t / (float)K + a.eps);
  };
  // The fold's sums of h^2 (n_ss <= 32 kEC granules) gathered by every consumer beside its x sweep
  // (consumer c: granules [32 c, 32 c + 32), its load issued before the sweep so both share one round
  // trip) into LDS (the attention's s_acc, idle outside the attention phase); after the barrier
  // consumer 0 forms the rms from them in fold_rms's order (bit-identical).
  auto ss_issue = [&](int n_ss) -> unsigned long long {
    const int i = c * 32 + lane;
    return lane < 32 && i < n_ss ? ld_sc1_u64(a.ssg + i) : 0ull;
  };
  auto ss_finish = [&](unsigned long long v, int n_ss, uint32_t tag) {
    const int i = c * 32 + lane;
    const bool want = lane < 32 && i < n_ss;
    Spin sp{ctl, a.err};
    while (!(TI_PDS_DIAG & 8) && __builtin_amdgcn_ballot_w64(want && (uint32_t)(v >> 32) != tag) != 0ull) {
      if (!sp.tick_g()) break;
      if (want && (uint32_t)(v >> 32) != tag) v = ld_sc1_u64(a.ssg + i);
    }
    if (want) s_acc[i] = __builtin_bit_cast(float, (uint32_t)v);
  };
  auto rms_lds = [&](int n_ss, int K) {
    float t = 0.0f;
#pragma unroll
    for (int j = 0; j < 4; ++j) t += lane + 64 * j < n_ss ? s_acc[lane + 64 * j] : 0.0f;
    t = group_sum<kWave>(t);
    return sqrtf(t / (float)K + a.eps);
  };
  // single granules of one wave: base[idx] for lanes with want, bounded
  auto gather1 = [&](const unsigned long long* base, int idx, bool want, uint32_t tag) -> uint32_t {
    unsigned long long v = want ? ld_sc1_u64(base + idx) : 0ull;
    Spin sp{ctl, a.err};
    while (!(TI_PDS_DIAG & 8) && __builtin_amdgcn_ballot_w64(want && (uint32_t)(v >> 32) != tag) != 0ull) {
      if (!sp.tick_g()) break;
      if (want && (uint32_t)(v >> 32) != tag) v = ld_sc1_u64(base + idx);
    }
    return (uint32_t)v;
  };
  // group scales of a phase's tiles t0 + t * tstride, t < ntl, into sl ([ntl][KT][16] fp16)
  auto stage_scales = [&](const uint16_t* sc, int t0, int tstride, int ntl, int KT) {
    const int per = KT * 2;   // 16-byte pieces per tile
    for (int i = ctid; i < ntl * per; i += kEC * kWave) {
      const int t = i / per, p = i - t * per;
      ((u32x4*)sl)[i] = gptr((const u32x4*)(sc + (size_t)(t0 + t * tstride) * KT * 16))[p];
    }
  };

  // The phase's group scales issued BEFORE its gather and written to LDS after it, so their load
  // shares the gather's round trip (one 16-byte piece per consumer thread; larger phases stage
  // them up front as before)
  auto scales_issue = [&](const uint16_t* sc, int t0, int tstride, int ntl, int KT, u32x4& r) -> bool {
    const int per = KT * 2, n = ntl * per;
    if (n > kEC * kWave) {
      stage_scales(sc, t0, tstride, ntl, KT);
      return false;
    }
    if (ctid < n) {
      const int t = ctid / per, p = ctid - t * per;
      r = gptr((const u32x4*)(sc + (size_t)(t0 + t * tstride) * KT * 16))[p];
    }
    return true;
  };
  auto scales_commit = [&](int ntl, int KT, const u32x4& r, bool issued) {
    if (issued && ctid < ntl * KT * 2) ((u32x4*)sl)[ctid] = r;
  };

  // ---- ring consumption
  auto wait_full = [&](uint32_t fill) {
    Spin sp{ctl, a.err};
    auto full = [&]() {
      uint32_t m = cget(ctl + C_FULL);
#pragma unroll
      for (int w = 1; w < kNL; ++w) m = min(m, cget(ctl + C_FULLX + w - 1));
      return m;
    };
    while (full() <= fill)
      if (!sp.tick()) break;
    asm volatile("" ::: "memory");
    if (c == 0) PDS_FT(fill, 2);
  };
  auto release = [&](uint32_t fill) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane == 0) cset(ctl + C_FREE + c, fill + 1);
    if (c == 0) PDS_FT(fill, 3);
  };
#if TI_PDS_DIAG & 1   // diagnostic: the ring alone (acquire / release every fill, nothing else)
  {
    uint32_t nf_all = 0;
    for (int l = 0; l < a.n_layers; ++l)
      for (int ph = 0; ph < PH_N; ++ph) nf_all += pds_fills(pds_pieces<C>(g, ph));
    for (uint32_t f = 0; f < nf_all; ++f) {
      wait_full(f);
      release(f);
    }
    return;
  }
#endif
  // GEMV phase over items (tile item / KT, k-tile item % KT): this consumer's items are k-tiles == c
  // (mod kEC), virtual waves kt % 8 in {c, c + kEC, ...}: the partial of (tile, virtual wave) accumulates
  // exactly as wave kt % 8 of gemv_wq_kernel does, then lands in slab[tile][v] (lanes 0-15).
  auto gemv_phase = [&](int ntl, int KT) {
    const int ni = ntl * KT, nf = pds_fills(ni * C);
    const f16* xrow = xl + kq * 32;
    for (int t = 0; t < ntl; ++t)
      if (lane < 16)
#pragma unroll
        for (int j = 0; j < kVPC; ++j) slab[(t * kVW + c + kEC * j) * 16 + lane] = 0.0f;
    f32x4 acc[kVPC];
#pragma unroll
    for (int j = 0; j < kVPC; ++j) acc[j] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
    int cur = 0, tl = 0, kt = 0;
    auto flush = [&]() {
      if (lane < 16)
#pragma unroll
        for (int j = 0; j < kVPC; ++j) slab[(cur * kVW + c + kEC * j) * 16 + lane] = acc[j][0];
#pragma unroll
      for (int j = 0; j < kVPC; ++j) acc[j] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
    };
    // one item's 4 MFMAs on (x, dequantized W)
    auto item_mfma = [&](const u32x4 (&wv)[C], int ik) {
      f32x4 t = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        const f16x8 bf = dequant_step<BITS>(wv, s4, magic);
        const f16x8 af = *(const f16x8*)(xrow + ik * 128 + s4 * 8);
        t = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, bf, t, 0, 0, 0);
      }
      return t;
    };
    // an item's MFMA result into its virtual wave's partial: the int4 offset correction cr, the group
    // scale sc (both read from LDS before the MFMAs where the caller can)
    auto item_acc2 = [&](f32x4 t, int it, int ik, float cr, float sc) {
      if (it != cur) {
        flush();
        cur = it;
      }
      if constexpr (BITS == 4) t -= cr;
      if (kVPC == 2 && ((ik / kEC) & 1)) {   // virtual wave c + kEC (static register indices: no scratch)
        acc[kVPC - 1][0] = fmaf(sc, t[0], acc[kVPC - 1][0]);
        acc[kVPC - 1][1] = fmaf(sc, t[1], acc[kVPC - 1][1]);
        acc[kVPC - 1][2] = fmaf(sc, t[2], acc[kVPC - 1][2]);
        acc[kVPC - 1][3] = fmaf(sc, t[3], acc[kVPC - 1][3]);
      } else {
        acc[0][0] = fmaf(sc, t[0], acc[0][0]);
        acc[0][1] = fmaf(sc, t[1], acc[0][1]);
        acc[0][2] = fmaf(sc, t[2], acc[0][2]);
        acc[0][3] = fmaf(sc, t[3], acc[0][3]);
      }
    };
    auto item_acc = [&](f32x4 t, int it, int ik) {
      item_acc2(t, it, ik, BITS == 4 ? corr[ik] : 0.0f, h2f(sl[(it * KT + ik) * 16 + r]));
    };
    if (KT % kEC == 0 || ntl == 1) {
      // k-tile == item index (mod kEC): this consumer's items sit at items c, c + kEC, ... of every
      // fill.  They are all read, the slot is released, then the math runs.
      constexpr int NU = IPF / kEC;
      tl = 0;
      kt = c;
      for (int fi = 0; fi < nf; ++fi) {
        const uint32_t fill = fbase + fi;
        wait_full(fill);
        const char* slot = smem + (fill % (uint32_t)a.n_slots) * kSlotBytes + lane * 16;
        u32x4 w[NU][C];
        int itl[NU], ikt[NU];
        bool live[NU];
#pragma unroll
        for (int u = 0; u < NU; ++u) {
          itl[u] = tl;
          ikt[u] = kt;
          live[u] = fi * IPF + c + kEC * u < ni;
#pragma unroll
          for (int cc = 0; cc < C; ++cc)
            w[u][cc] = live[u] ? *(const u32x4*)(slot + ((c + kEC * u) * C + cc) * kPiece) : (u32x4){0u, 0u, 0u, 0u};
          kt += kEC;
          if (kt >= KT && ntl > 1) {
            kt -= KT;
            ++tl;
          }
        }
        // each item's correction and scale, read before the MFMAs (their LDS latency overlaps them)
        float crv[NU], scv[NU];
#pragma unroll
        for (int u = 0; u < NU; ++u) {
          crv[u] = BITS == 4 && live[u] ? corr[ikt[u]] : 0.0f;
          scv[u] = live[u] ? h2f(sl[(itl[u] * KT + ikt[u]) * 16 + r]) : 0.0f;
        }
        release(fill);
#if TI_PDS_DIAG & 4   // diagnostic: no GEMV math (garbage results; the ring and hand-offs only)
        if (c == 0) PDS_FT(fill, 7);
        continue;
#endif
        // the fill's NU MFMA chains interleaved (independent accumulators hide the MFMA latency),
        // then accumulated in item order (the same sums, in the same order, as item by item)
        f32x4 tv[NU];
#pragma unroll
        for (int u = 0; u < NU; ++u) tv[u] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
          for (int u = 0; u < NU; ++u) {
            const f16x8 bf = dequant_step<BITS>(w[u], s4, magic);
            const f16x8 af = *(const f16x8*)(xrow + (live[u] ? ikt[u] : 0) * 128 + s4 * 8);
            tv[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, bf, tv[u], 0, 0, 0);
          }
#pragma unroll
        for (int u = 0; u < NU; ++u)
          if (live[u]) item_acc2(tv[u], itl[u], ikt[u], crv[u], scv[u]);
        if (c == 0) PDS_FT(fill, 7);
      }
    } else {
      // general shapes (K % 512 != 0 with several tiles): item by item
      for (int fi = 0; fi < nf; ++fi) {
        const uint32_t fill = fbase + fi;
        wait_full(fill);
        const char* slot = smem + (fill % (uint32_t)a.n_slots) * kSlotBytes + lane * 16;
        for (int j = 0; j < IPF; ++j) {
          if (fi * IPF + j >= ni) break;
          if (kt % kEC == c) {
            u32x4 w[C];
#pragma unroll
            for (int cc = 0; cc < C; ++cc) w[cc] = *(const u32x4*)(slot + (j * C + cc) * kPiece);
            item_acc(item_mfma(w, kt), tl, kt);
          }
          if (++kt == KT) {
            kt = 0;
            ++tl;
          }
        }
        release(fill);
      }
    }
    if (ni > 0) flush();
    fbase += nf;
  };
  // tile sums (the 8 virtual waves in order), output n of tile tl
  auto tile_sum = [&](int tl, int n) {
    const float* sp = slab + tl * kVW * 16 + n;
    float v = sp[0];
#pragma unroll
    for (int w = 1; w < kVW; ++w) v += sp[w * 16];
    return v;
  };
  // residual epilogue of the workgroup's tile (O, down) with the fold into the next projection's
  // input (TI_EPI_RESID_F32 + fold_x, M = 1); gtag 0: the lm_head's input, plain sc1 stores
  auto resid_fold = [&](const float* nw, uint32_t gtag) {
    const int n = lane & 15;
    const float v = tile_sum(0, n);
    const float fw = gptr(nw)[bid * 16 + n];
    float ssacc = 0.0f, rr = 0.0f;
    if (lane < 16) {
      rr = h_l[n] + v;
      h_l[n] = rr;
      ssacc = fmaf(rr, rr, ssacc);
    }
    const uint32_t hv = f2h(rr * fw), hp = lane_xor_u32<1>(hv);
    const float sw = group_sum<kWave>(ssacc);
    if (gtag) {
      if (lane < 16 && !(n & 1)) st_gran(a.fxg + (bid * 16 + n) / 2, hv | (hp << 16), gtag);
      if (lane == 0) st_gran(a.ssg + bid, __builtin_bit_cast(uint32_t, sw), gtag);
    } else {
      if (lane < 16 && !(n & 1)) st_sc1_u32(a.fx + bid * 16 + n, hv | (hp << 16));
      if (lane == 0) st_sc1_f32(a.ss + bid, sw);
    }
  };
  auto gathering = [&](bool on) {
    if (c == 0 && lane == 0) cset(ctl + C_GATHER, on ? 1u : 0u);
  };

  for (int l = 0; l < a.n_layers; ++l) {
    const CLayer ly = layer_c(a.layers, l);
    // ============================================================== QKV (RoPE + KV append)
    float rms = 1.0f;
    {
      ts(l, PH_QKV, 0);
      u32x4 scr = {0u, 0u, 0u, 0u};
      const bool sci = scales_issue(ly->scales[0], g.q0, g.qs, g.qn, g.KTh, scr);
      gathering(true);
      const bool ssp = l > 0 && a.nt_h <= kEC * 32;   // the sums gathered by every consumer
      const unsigned long long ssv = ssp ? ss_issue(a.nt_h) : 0ull;
      if (l == 0) stage_x(a.fx, H, 0u, true);
      else stage_x(a.fxg, H, pds_tag(epoch, l - 1, PH_DN), false);
      if (ssp) ss_finish(ssv, a.nt_h, pds_tag(epoch, l - 1, PH_DN));
      else if (c == 0) rms = l == 0 ? fold_rms(a.ss, a.n_ss0, H, 0u, true) : fold_rms(a.ssg, a.nt_h, H, pds_tag(epoch, l - 1, PH_DN), false);
      scales_commit(g.qn, g.KTh, scr, sci);
      bar();
      if (ssp && c == 0) rms = rms_lds(a.nt_h, H);
      gathering(false);
      ts(l, PH_QKV, 1);
      gemv_phase(g.qn, g.KTh);
      bar();
      ts(l, PH_QKV, 2);
      if (c == 0) {
        // outputs (tile tl, n) = lane < 16 qn: TI_EPI_QKV_ROPE_KV, M = 1
        const int tl = lane >> 4, n = lane & 15;
        const bool ok = tl < g.qn;
        const float v = (ok ? tile_sum(tl, n) : 0.0f) / rms;
        const float partner = lane_xor<1>(v);
        const int ng = (g.q0 + tl * g.qs) * 16 + n;
        const bool qk = ng < qd + kvd;
        const int base = ng < qd ? 0 : ng < qd + kvd ? qd : qd + kvd;
        const int d = (ng - base) % HD, hh = (ng - base) / HD;
        float rv = v;
        if (ok && qk) {
          const float2 cs = *(const float2*)(cs_l + (d & ~1));
          rv = (d & 1) == 0 ? fmaf(-partner, cs.y, v * cs.x) : fmaf(v, cs.x, partner * cs.y);
        }
        const uint32_t hv = f2h(rv), hp = lane_xor_u32<1>(hv);
        const uint32_t tq = pds_tag(epoch, l, PH_QKV);
        if (ok && ng < qd) {
          st_gran(a.qg + ng, __builtin_bit_cast(uint32_t, rv), tq);
        } else if (ok && !(n & 1)) {
          const bool is_k = qk;
          uint16_t* cache = is_k ? ly->k_cache : ly->v_cache;   // for later launches
          gptr_w((uint32_t*)(cache + ((size_t)hh * a.max_seq + pos) * HD + d))[0] = hv | (hp << 16);
          st_gran(a.kvg + ((size_t)hh * 2 + (is_k ? 0 : 1)) * (HD / 2) + d / 2, hv | (hp << 16), tq);
        }
        ts(l, PH_QKV, 3);
      }
    }
    // ============================================================== attention split (h, s)
    {
      ts(l, PH_ATT, 0);
      const uint32_t tq = pds_tag(epoch, l, PH_QKV);
      if (c == 0) {
        q_l[lane] = __builtin_bit_cast(float, gather1(a.qg + g.h * HD, lane, lane < HD, tq));
        if (HD > kWave) q_l[lane + kWave] = __builtin_bit_cast(float, gather1(a.qg + g.h * HD, lane + kWave, true, tq));
      } else if (c == 1 && pos >= g.s0 && pos < g.s1) {
        ((uint32_t*)kf_l)[lane] = gather1(a.kvg + (size_t)g.kvh * HD, lane, lane < HD / 2, tq);
        ((uint32_t*)vf_l)[lane] = gather1(a.kvg + (size_t)g.kvh * HD + HD / 2, lane, lane < HD / 2, tq);
      }
      bar();
      ts(l, PH_ATT, 1);
      const int dl = lane % LPK, kg = lane / LPK;
      float qv[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) qv[e] = q_l[dl * 8 + e] * a.scale;
      float mrun[kVPC], lrun[kVPC], acc[kVPC][8];
#pragma unroll
      for (int u = 0; u < kVPC; ++u) {
        mrun[u] = -INFINITY;
        lrun[u] = 0.0f;
      }
#pragma unroll
      for (int u = 0; u < kVPC; ++u)
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[u][e] = 0.0f;
      const int np = 2 * g.nslot, nf = pds_fills(np);
      for (int fi = 0; fi < nf; ++fi) {
        const uint32_t fill = fbase + fi;
        wait_full(fill);
        const char* slot = smem + (fill % (uint32_t)a.n_slots) * kSlotBytes + lane * 16;
        u32x4 kr[kVPC], vr[kVPC];
#pragma unroll
        for (int u = 0; u < kVPC; ++u) {
          const int su = c + kEC * u, si = fi * 8 + su;
          kr[u] = si < g.nslot ? *(const u32x4*)(slot + (2 * su) * kPiece) : (u32x4){0u, 0u, 0u, 0u};
          vr[u] = si < g.nslot ? *(const u32x4*)(slot + (2 * su + 1) * kPiece) : (u32x4){0u, 0u, 0u, 0u};
        }
        release(fill);
#pragma unroll
        for (int u = 0; u < kVPC; ++u) {
          const int su = c + kEC * u, si = fi * 8 + su;   // slot of the split; virtual wave su
          if (si < g.nslot) {
            const int key = g.s0 + KPW * si + kg;
            const bool valid = key < g.s1;
            u32x4 kv = kr[u];
            u32x4 vv = valid ? vr[u] : (u32x4){0u, 0u, 0u, 0u};
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
            d = group_sum<LPK>(d);
            const float sc = valid ? d : -INFINITY;
            const float mn = fmaxf(mrun[u], sc);
            const float alpha = mrun[u] == mn ? 1.0f : __expf(mrun[u] - mn);
            const float pr = valid ? __expf(sc - mn) : 0.0f;
            lrun[u] = fmaf(lrun[u], alpha, pr);
            mrun[u] = mn;
#pragma unroll
            for (int e = 0; e < 8; ++e) acc[u][e] = fmaf(pr, vf[e], acc[u][e] * alpha);
          }
        }
      }
      fbase += nf;
      // merge the lane groups of each virtual wave (attn_split_body)
#pragma unroll
      for (int u = 0; u < kVPC; ++u) {
        const int v = c + kEC * u;
        const float mx = groups_max<LPK>(mrun[u]);
        const float f = mrun[u] == -INFINITY ? 0.0f : __expf(mrun[u] - mx);
        const float lsum = groups_sum<LPK>(lrun[u] * f);
        float o[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = groups_sum<LPK>(acc[u][e] * f);
        if (lane < LPK) {
#pragma unroll
          for (int e = 0; e < 8; ++e) s_acc[v * kHdMax + dl * 8 + e] = o[e];
        }
        if (lane == 0) {
          s_m[v] = mx;
          s_l[v] = lsum;
        }
      }
      bar();
      ts(l, PH_ATT, 2);
      if (c == 0) {
        // merge the 8 virtual waves: dims 2 lane, 2 lane + 1 (lane < HD / 2) -> this split's partial
        const int dd = lane < HD / 2 ? 2 * lane : 0;
        float mx = s_m[0];
#pragma unroll
        for (int w = 1; w < kVW; ++w) mx = fmaxf(mx, s_m[w]);
        float o2[2] = {0.0f, 0.0f}, lsum = 0.0f;
        if (mx != -INFINITY) {
#pragma unroll
          for (int w = 0; w < kVW; ++w) {
            const float f = s_m[w] == -INFINITY ? 0.0f : __expf(s_m[w] - mx);
            o2[0] = fmaf(f, s_acc[w * kHdMax + dd], o2[0]);
            o2[1] = fmaf(f, s_acc[w * kHdMax + dd + 1], o2[1]);
            lsum = fmaf(f, s_l[w], lsum);
          }
        }
        const uint32_t ta = pds_tag(epoch, l, PH_ATT);
        unsigned long long* pg = a.partg + ((size_t)g.h * kSplits + g.s) * PG;
        const uint32_t lo = f2h(lsum > 0.0f ? o2[0] / lsum : 0.0f), hi = f2h(lsum > 0.0f ? o2[1] / lsum : 0.0f);
        if (lane < HD / 2) st_gran(pg + lane, lo | (hi << 16), ta);
        if (lane == 0) {
          st_gran(pg + HD / 2, __builtin_bit_cast(uint32_t, mx), ta);
          st_gran(pg + HD / 2 + 1, __builtin_bit_cast(uint32_t, lsum), ta);
        }
        ts(l, PH_ATT, 3);
        // the head group's split merge for dims [s HD / 8, (s + 1) HD / 8): lane = split sp * NPS +
        // pair j (the O projection's TI_X_ATTN_SPLITS staging arithmetic: weights l_s exp(m_s - max))
        {
          const int sp = lane / NPS, j = lane % NPS;
          const bool mine = lane < kSplits * NPS;
          const uint32_t pw = gather1(a.partg + ((size_t)g.h * kSplits + (mine ? sp : 0)) * PG, g.s * NPS + j, mine, ta);
          const uint32_t mw = gather1(a.partg + ((size_t)g.h * kSplits + (lane >> 1)) * PG, HD / 2 + (lane & 1),
                                      lane < 2 * kSplits, ta);
          const f16x2 ph2 = __builtin_bit_cast(f16x2, pw);
          if (mine) {
            mg_o[sp * 16 + 2 * j] = (float)ph2[0];
            mg_o[sp * 16 + 2 * j + 1] = (float)ph2[1];
          }
          if (lane < 2 * kSplits) mg_ml[lane] = __builtin_bit_cast(float, mw);
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          const int dm = lane % (HD / 8);
          float mxs = -INFINITY;
#pragma unroll
          for (int q = 0; q < kSplits; ++q) mxs = fmaxf(mxs, mg_ml[2 * q]);
          float num = 0.0f, den = 0.0f;
#pragma unroll
          for (int q = 0; q < kSplits; ++q) {
            const float f = mg_ml[2 * q] != -INFINITY ? mg_ml[2 * q + 1] * __expf(mg_ml[2 * q] - mxs) : 0.0f;
            den += f;
            num = fmaf(f, mg_o[q * 16 + dm], num);
          }
          const uint32_t xv = f2h(den > 0.0f ? num / den : 0.0f), xp = lane_xor_u32<1>(xv);
          if (lane < HD / 8 && !(lane & 1))
            st_gran(a.aog + (g.h * HD + g.s * (HD / 8) + lane) / 2, xv | (xp << 16), pds_tag(epoch, l, PH_MRG));
        }
        ts(l, PH_ATT, 4);
      }
    }
    // ============================================================== O: residual + fold (ffn_norm)
    {
      ts(l, PH_O, 0);
      u32x4 scr = {0u, 0u, 0u, 0u};
      const bool sci = scales_issue(ly->scales[1], bid, 0, g.on, g.KTq, scr);
      gathering(true);
      stage_x(a.aog, qd, pds_tag(epoch, l, PH_MRG), false);
      scales_commit(g.on, g.KTq, scr, sci);
      bar();
      gathering(false);
      ts(l, PH_O, 1);
      gemv_phase(g.on, g.KTq);
      bar();
      ts(l, PH_O, 2);
      if (c == 0 && g.on) resid_fold(ly->ffn_norm, pds_tag(epoch, l, PH_O));
      ts(l, PH_O, 3);
    }
    // ============================================================== gate/up: SiLU * up
    {
      ts(l, PH_GU, 0);
      u32x4 scr = {0u, 0u, 0u, 0u};
      const bool sci = scales_issue(ly->scales[2], g.gu0, 1, g.gun, g.KTh, scr);
      gathering(true);
      const bool ssp = a.nt_h <= kEC * 32;
      const unsigned long long ssv = ssp ? ss_issue(a.nt_h) : 0ull;
      stage_x(a.fxg, H, pds_tag(epoch, l, PH_O), false);
      if (ssp) ss_finish(ssv, a.nt_h, pds_tag(epoch, l, PH_O));
      else if (c == 0) rms = fold_rms(a.ssg, a.nt_h, H, pds_tag(epoch, l, PH_O), false);
      scales_commit(g.gun, g.KTh, scr, sci);
      bar();
      if (ssp && c == 0) rms = rms_lds(a.nt_h, H);
      gathering(false);
      ts(l, PH_GU, 1);
      gemv_phase(g.gun, g.KTh);
      bar();
      ts(l, PH_GU, 2);
      if (c == 0) {
        for (int tb = 0; tb < g.gun * 16; tb += kWave) {
          const int t = tb + lane, tl = t >> 4, n = lane & 15;
          const bool ok = t < g.gun * 16;
          const float v = (ok ? tile_sum(tl, n) : 0.0f) / rms;
          const float up = lane_xor<8>(v);
          const float s = v / (1.0f + expf(-v));
          const uint32_t hv = f2h(up * s), hp = lane_xor_u32<1>(hv);
          if (ok && n < 8 && !(n & 1))
            st_gran(a.actg + ((g.gu0 + tl) * 8 + n) / 2, hv | (hp << 16), pds_tag(epoch, l, PH_GU));
        }
        ts(l, PH_GU, 3);
      }
    }
    // ============================================================== down: residual + fold (next norm)
    {
      ts(l, PH_DN, 0);
      u32x4 scr = {0u, 0u, 0u, 0u};
      const bool sci = scales_issue(ly->scales[3], bid, 0, g.on, g.KTi, scr);
      gathering(true);
      stage_x(a.actg, I, pds_tag(epoch, l, PH_GU), false);
      scales_commit(g.on, g.KTi, scr, sci);
      bar();
      gathering(false);
      ts(l, PH_DN, 1);
      gemv_phase(g.on, g.KTi);
      bar();
      ts(l, PH_DN, 2);
      // the last layer's fold goes to the lm_head launch: plain write-through stores
      if (c == 0 && g.on && !(l == 0 && bid == a.drop_wg && l + 1 < a.n_layers))
        resid_fold(l + 1 < a.n_layers ? layer_c(a.layers, l + 1)->attn_norm : a.out_norm,
                   l + 1 < a.n_layers ? pds_tag(epoch, l, PH_DN) : 0u);
      ts(l, PH_DN, 3);
    }
  }
  if (c == 0 && lane < 16 && g.on) gptr_w(a.h)[bid * 16 + lane] = h_l[lane];
}

}  // namespace ti

using namespace ti;

namespace {
template <int BITS, int HD>
const void* pds_fn() { return (const void*)pds_kernel<BITS, HD>; }
}  // namespace

extern "C" {

size_t ti_pds_granule_words(int H, int I, int qd, int heads, int grid) { return pds_gran_words(H, I, qd, heads, grid); }

int ti_pds_supported(int bits, int H, int I, int heads, int kv_heads, int head_dim, int grid, int layers) {
  if ((bits != 4 && bits != 8) || (head_dim != 64 && head_dim != 128) || heads < 1 || kv_heads < 1 || heads % kv_heads)
    return 0;
  int sh = 0;
  while ((kv_heads << sh) < heads) ++sh;
  if ((kv_heads << sh) != heads || grid != heads * kSplits || grid > 256 || layers < 1 || layers > 64) return 0;
  const int qd = heads * head_dim, kvd = kv_heads * head_dim;
  if (H % 128 || I % 128 || qd % 128 || H / 16 > grid) return 0;
  const int nt_qkv = (qd + 2 * kvd) / 16, nt_gu = 2 * I / 16;
  if ((nt_qkv + grid - 1) / grid > kMaxQkvTiles || (nt_gu + grid - 1) / grid > kMaxGuTiles) return 0;
  return 1;
}

#if TI_PDS_FTRACE
// diagnostic build only: copy the fill trace ([4][2048][8] u64) to host and clear it
int ti_pds_ftrace(unsigned long long* host, size_t n) {
  const size_t bytes = sizeof(unsigned long long) * (size_t)ti::kFtWg * ti::kFtFills * 8;
  if (!host || n * sizeof(unsigned long long) < bytes) return ti_set_error(TI_ERR_ARG, "ti_pds_ftrace: buffer");
  if (hipMemcpyFromSymbol(host, HIP_SYMBOL(ti::g_pds_ft), bytes, 0, hipMemcpyDeviceToHost) != hipSuccess)
    return ti_set_error(TI_ERR_HIP, "ti_pds_ftrace: copy");
  static std::vector<unsigned long long> zero;
  zero.assign(bytes / 8, 0ull);
  if (hipMemcpyToSymbol(HIP_SYMBOL(ti::g_pds_ft), zero.data(), bytes, 0, hipMemcpyHostToDevice) != hipSuccess)
    return ti_set_error(TI_ERR_HIP, "ti_pds_ftrace: clear");
  return TI_OK;
}
#endif

int ti_pds_decode(const ti_pds_args* h, ti_stream_t s) {
  if (!h || !h->layers || !h->pos || !h->h || !h->fx || !h->ss || !h->launches || !h->err || !h->zero ||
      !h->rope_cs || !h->out_norm || !h->gran)
    return ti_set_error(TI_ERR_ARG, "ti_pds_decode: null pointer");
  if (!ti_pds_supported(h->bits, h->H, h->I, h->heads, h->kv_heads, h->head_dim, h->grid, h->n_layers) ||
      h->qd != h->heads * h->head_dim)
    return ti_set_error(TI_ERR_UNSUPPORTED, "ti_pds_decode: shape not supported (bits %d heads %d kv %d hd %d grid %d H %d "
                        "I %d layers %d)", h->bits, h->heads, h->kv_heads, h->head_dim, h->grid, h->H, h->I, h->n_layers);
  const int HD = h->head_dim;
  PdsArgs a{};
  a.layers = (const PdsLayerDev*)h->layers;
  a.n_layers = h->n_layers;
  a.H = h->H;
  a.I = h->I;
  a.qd = h->qd;
  a.kvd = h->kv_heads * HD;
  a.max_seq = h->max_seq;
  a.n_ss0 = h->n_ss0;
  a.heads = h->heads;
  while ((h->kv_heads << a.kv_shift) < h->heads) ++a.kv_shift;
  a.grid = h->grid;
  a.nt_h = h->H / 16;
  a.head_group = HD == 128 && h->heads == h->kv_heads && h->qd / 16 == h->grid;
  a.eps = h->eps;
  a.scale = 1.0f / sqrtf((float)HD);
  a.pos = h->pos;
  a.rope_cs = h->rope_cs;
  a.out_norm = h->out_norm;
  a.h = h->h;
  a.fx = h->fx;
  a.ss = h->ss;
  a.launches = h->launches;
  a.err = h->err;
  a.zero = (const char*)h->zero;
  a.ts = h->ts;
  a.drop_wg = h->drop_wg;
  a.fxg = h->gran;
  a.ssg = a.fxg + h->H / 2;
  a.qg = a.ssg + h->grid;
  a.kvg = a.qg + h->qd;
  a.partg = a.kvg + (size_t)h->heads * kHdMax;
  a.aog = a.partg + (size_t)h->heads * kSplits * (kHdMax / 2 + 2);
  a.actg = a.aog + h->qd / 2;
  // LDS: ring, x [max K + 8] fp16, scales, corr, slab, attention / control scratch
  const int KTh = h->H / 128, KTi = h->I / 128, KTq = h->qd / 128;
  const int nt_qkv = (a.qd + 2 * a.kvd) / 16, NTg = 2 * h->I / 16;
  const int q_ntl = a.head_group ? 3 : (nt_qkv + h->grid - 1) / h->grid, gu_ntl = (NTg + h->grid - 1) / h->grid;
  const int kmax = std::max(h->H, std::max(h->I, h->qd));
  const int sc_bytes = std::max(std::max(q_ntl * KTh, gu_ntl * KTh), std::max(KTq, KTi)) * 32;
  const int ntl_max = std::max(q_ntl, gu_ntl);
  auto al = [](int b) { return (b + 15) & ~15; };
  const int att_bytes = (kVW * kHdMax + 2 * kVW + kHdMax) * 4 + 2 * kHdMax * 2 + kHdMax * 4 + 16 * 4 +
                        kSplits * 16 * 4 + kSplits * 2 * 4;
  const int rest = al((kmax + 8) * 2) + al(sc_bytes) + al(std::max(KTh, std::max(KTi, KTq)) * 4) +
                   al(ntl_max * kVW * 16 * 4) + al(att_bytes) + C_WORDS * 4;
  const int lds_cap = 160 * 1024;
  const int n_slots = std::min(kMaxSlots, (lds_cap - rest) / kSlotBytes);
  if (n_slots < 3) return ti_set_error(TI_ERR_UNSUPPORTED, "ti_pds_decode: LDS ring of %d slots", n_slots);
  a.n_slots = n_slots;
  a.l_x = n_slots * kSlotBytes;
  a.l_sc = a.l_x + al((kmax + 8) * 2);
  a.l_corr = a.l_sc + al(sc_bytes);
  a.l_slab = a.l_corr + al(std::max(KTh, std::max(KTi, KTq)) * 4);
  a.l_att = a.l_slab + al(ntl_max * kVW * 16 * 4);
  a.l_ctl = a.l_att + al(att_bytes);
  a.l_total = a.l_ctl + C_WORDS * 4;
  const void* fn = h->bits == 4 ? (HD == 128 ? pds_fn<4, 128>() : pds_fn<4, 64>())
                                : (HD == 128 ? pds_fn<8, 128>() : pds_fn<8, 64>());
  const int variant = (h->bits == 8 ? 2 : 0) + (HD == 64 ? 1 : 0);
  // per device and variant: the LDS attribute and co-residency -- every wait needs all `grid`
  // workgroups resident at once (one per CU): the occupancy query times the CU count must cover
  // the grid, or nothing is launched (residency taken by other work at run time is caught by the
  // bounded waits).
  static std::atomic<unsigned long long> prepared[4];
  static std::atomic<int> resident[4][64];
  static std::mutex mu;
  int dev = 0;
  TI_HIP_CHECK(hipGetDevice(&dev), "hipGetDevice");
  dev &= 63;
  if (!(prepared[variant].load() >> dev & 1ull)) {
    std::lock_guard<std::mutex> lk(mu);
    if (!(prepared[variant].load() >> dev & 1ull)) {
      TI_HIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, lds_cap),
                   "hipFuncSetAttribute(pds_kernel)");
      int per_cu = 0, cus = 0;
      TI_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kEThreads, lds_cap),
                   "hipOccupancyMaxActiveBlocksPerMultiprocessor(pds_kernel)");
      TI_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev), "hipDeviceGetAttribute(CUs)");
      resident[variant][dev].store(per_cu * cus);
      prepared[variant].fetch_or(1ull << dev);
    }
  }
  if (resident[variant][dev].load() < h->grid)
    return ti_set_error(TI_ERR_UNSUPPORTED, "ti_pds_decode: %d workgroups cannot all be resident (%d)", h->grid,
                        resident[variant][dev].load());
  void* args[] = {&a};
  TI_HIP_CHECK(hipLaunchKernel(fn, dim3(h->grid), dim3(kEThreads), args, a.l_total, (hipStream_t)s),
               "hipLaunchKernel(pds_kernel)");
  TI_LAUNCH_CHECK("pds_kernel");
  return TI_OK;
}

}  // extern "C"
