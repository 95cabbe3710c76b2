// qkv_attn.hip -- one decode stream (TinyLlama-1.1B GQA head_dim 64, configs[1]; Llama-2-7B MHA head_dim 128,
// configs[2]): the QKV projection and the attention over the cache in ONE launch (ti_qkv_attn_partials,
// DESIGN 4.19), i.e. TransformerLayer::forward_incremental's q / k / v projections, RoPE, KV append and
// compute_attention (inference_engine.cpp:203-279, 291-368; tensor_engine.cpp:1254-1388).
//
// Workgroup (head h, split s) = blockIdx (s + S h); S = splits workgroups per head.
//   1. x = fp16(h * nw) of the rms_norm fold (TI_X_F16_FOLDED) staged in LDS, the rms from the
//      producer's partial sums of squares;
//   2. its share of the head's q rows: tile s % QT of the head (QT = head_dim / 16 tiles), k-part
//      s / QT of S / QT, with the fused GEMV's item arithmetic; the 8 waves' partials summed in a
//      fixed order and published as 16 data-tagged 8-byte granules {value, generation} (agent-scope
//      stores); then its k / v tiles (qa_kv_tile: GQA, split S - 1 first; MHA, a k and a v tile each):
//      the QKV epilogue's arithmetic (RoPE of k), the new K / V row into the cache at p = pos[0], and
//      the row's fp16 values published in pairs as 8 more granules per tile;
//   3. the head's q gathered from its S workgroups' granules (each workgroup keeps a generation count
//      in its own slot: every launch advances every slot by one, so the siblings' expected tag is its
//      own), summed over the k-parts in order, / rms, RoPE;
//   4. the split's share of the OLD keys [0, p) against q_h (attn_split_body's one-query lane
//      layout, online softmax); the last wave of split S - 1 then attends the new key p itself, its
//      k_p / v_p taken from the k / v tiles' granules; wave merge; the split's normalised row and
//      (max, sum) written as ti_attn_decode_partials writes them, for the O projection to merge
//      (TI_X_ATTN_SPLITS).  Split S - 1 is shorter (last_extra keys) for its tiles / the new key.
// Every wait on a granule is bounded (a lost sibling costs a wrong result, not a hang).
#include <math.h>
#include <stdlib.h>

#include "attention_body.hpp"
#include "common.hpp"
#include "dequant.hpp"
#include "ti_hip.h"

namespace ti {

struct QkvAttnArgs {
  const u32x4* tiles;          // QKV weight tiles [N / 16][K / 128]
  const uint16_t* scales;      // [N / 16][K / 128][16]
  const uint16_t* fx;          // fp16(h * nw), [K]
  const float* ss;             // the producer's partial sums of h^2
  int n_ss;
  float eps;
  const float* rope_cs;        // [max_seq][head_dim] (cos, sin) pairs
  const int32_t* pos;          // [1]
  uint16_t* kc;                // this layer's cache, stream 0: [kv_heads][max_seq][head_dim]
  uint16_t* vc;
  int max_seq, K, heads, kv_heads, kv_shift, splits, kv_tiles;
  int last_extra;              // keys' worth of bytes the last split's k / v tile streams: that split is shorter
  float scale;
  uint16_t* part_o;            // [heads][S][HD], then k_p [heads][HD] and v_p [heads][HD]
  float* part_ml;              // [heads][S][2], then q [heads][HD]
  unsigned long long* xchg;    // [heads * S][16] granules {float value, uint32 generation}
  unsigned long long* stamp;
  uint32_t* err;               // set to 1 when a wait on a granule expired (behind the granules of xchg)
  int drop;                    // test hook (TI_QA_DROP): this workgroup withholds its q part; -1 = none
};

constexpr int kQaWaves = 8, kQaThreads = kQaWaves * kWave;
#ifndef TI_QA_KV_RING
#define TI_QA_KV_RING 3   // K / V slots of 8 keys in flight per wave (5: 1704 vs 1722 tok/s, profiles/r6_qa_ab.txt)
#endif
#ifndef TI_QA_ISSUE_BARRIER
#define TI_QA_ISSUE_BARRIER 0   // head_dim 128: a barrier between the small loads and the weights (802 vs 806 tok/s: off)
#endif
#ifndef TI_QA_KVW_LATE
#define TI_QA_KVW_LATE 0   // 1: the k / v tiles' weights issued after the q part instead of after staging (A/B)
#endif
#ifndef TI_QA_KV_LATE
// the K/V ring issued after the q part (1) or before the GEMV (0); -1: after at head_dim 128, where a
// workgroup's keys are 4x a q part's bytes (7B 790.6 vs 776.5 tok/s), before at 64 (TinyLlama 1733 vs
// 1712; profiles/r6_qa_ab.txt)
#define TI_QA_KV_LATE -1
#endif
constexpr int kQaSlot = 32;   // granules per workgroup: the q part's 16, then 8 per k / v tile (k_p / v_p pairs)
constexpr int kQaMaxK = 4096;
constexpr int kQaMaxKv = 2;      // k / v tiles per workgroup (MHA at 8 splits: a k and a v tile each)
constexpr unsigned kQaSpin = 1u << 16;   // bounded wait per granule (a poll is a ~1 us round trip: ~0.1 s)

// gemv.hip int4_x_prep: the high-nibble slots of an x piece scaled by 1/16 (exact in fp16) and the
// piece's share of the offset correction 1032 * sum_lo x + 1152 * sum_hi x (deq_int4_raw)
__device__ __forceinline__ float int4_x_prep_qa(f16x8& h) {
  const f16 s16 = (f16)0.0625f;
  h[2] *= s16; h[3] *= s16; h[6] *= s16; h[7] *= s16;
  const float lo = ((float)h[0] + (float)h[1]) + ((float)h[4] + (float)h[5]);
  const float hi = ((float)h[2] + (float)h[3]) + ((float)h[6] + (float)h[7]);
  return 1032.0f * lo + 1152.0f * hi;
}

// workgroup (h, s) -> its i-th k / v tile (index into the kv_tiles tiles after the q rows), or -1: tiles
// j = h + heads (S - 1 - s) + heads S i, so split S - 1 takes them first when there are fewer than
// workgroups (GQA), and every workgroup two when there are twice as many (MHA)
__host__ __device__ inline int qa_kv_tile(int h, int s, int i, int heads, int splits, int kv_tiles) {
  const int j = h + heads * (splits - 1 - s) + heads * splits * i;
  return j < kv_tiles ? j : -1;
}

// NQ: q items per wave (k-tiles of the part / 8), NK: items per wave of a k / v tile (k-tiles / 8): compile-time,
// so the weight loads need no branch (a branch around a load whose value feeds a phi makes the compiler
// wait for it at once)
template <int BITS, int HD, int NQ, int NK>
__global__ __launch_bounds__(kQaThreads, 1) void qkv_attn_kernel(const QkvAttnArgs a) {
  const unsigned long long t_entry = stamp_now();
  constexpr int C = TileFmt<BITS>::kChunks;
  constexpr int QT = HD / 16;                 // q tiles of a head
  __shared__ __attribute__((aligned(16))) f16 xl[kQaMaxK + 8];   // (8 * 512 threads = kQaMaxK)
  __shared__ __attribute__((aligned(16))) uint16_t sl[1 + kQaMaxKv][kQaMaxK / 128][16];   // scales: q tile, k / v tiles
  __shared__ __attribute__((aligned(16))) float corr[kQaMaxK / 128][16];
  __shared__ u32x4 sl_dummy;
  __shared__ float slab[1 + kQaMaxKv][kQaWaves][16];
  __shared__ float q_s[HD];
  __shared__ float s_m[kQaWaves], s_l[kQaWaves];
  __shared__ __attribute__((aligned(16))) float s_acc[kQaWaves][HD];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // blockIdx = s + S h: split s of every head on XCD s % 8 (blockIdx % 8), so the G q-heads of a kv-head
  // that read the same key range share that XCD's L2 (heads on the same XCD would read every kv-head's
  // keys from each of the 8 L2s)
  const int S = a.splits, h = (int)blockIdx.x / S, s = (int)blockIdx.x % S;
  const int K = a.K, KT = K >> 7, K8 = K >> 3;
  const int qd = a.heads * HD, kvd = a.kv_heads * HD;
  const int kparts = S / QT, tq = s % QT, kp = s / QT;   // this workgroup's q tile and k-part
  const int KTP = KT / kparts;                           // k-tiles of a part (a multiple of 8)
  int gk[kQaMaxKv], nkv = 0;   // global tiles of the workgroup's k / v tiles (the first nkv)
#pragma unroll
  for (int i = 0; i < kQaMaxKv; ++i) {
    const int j = qa_kv_tile(h, s, i, a.heads, S, a.kv_tiles);
    gk[i] = qd / 16 + (j >= 0 ? j : 0);
    nkv += j >= 0 ? 1 : 0;
  }
  const int gq = h * QT + tq;   // global tile of the q part
  unsigned long long* my_slot = a.xchg + ((size_t)h * S + s) * kQaSlot;

  // ---- 1. small inputs first: position, own generation, scales, x piece, the rms partials, then the
  // whole weight stream.  The position goes through a VGPR the compiler cannot prove uniform (a
  // uniform load would be waited for at once, in front of every other load).
  int zero;
  asm volatile("v_mov_b32 %0, 0" : "=v"(zero));
  const int p_v = a.pos[zero];
  // (only the tag word: a 64-bit load whose unused half the allocator hands out again waits at once)
  const uint32_t gen_prev = ld_sc1_u32((const uint32_t*)(my_slot + (zero & 15)) + 1);
  // scales: the q tile's k-part and the k / v tiles, 16-byte pieces (KT * 2 per whole tile)
  const int n_scq = KTP * 2, n_sc = n_scq + nkv * KT * 2;
  u32x4 sc_reg;
  {
    // (selects, no branch and no dynamic index into gk[]: either would put a wait in front of the loads)
    const int ic = tid < n_sc ? tid : 0, r2 = ic - n_scq, ik = r2 >= KT * 2 ? 1 : 0;
    const int g = ic < n_scq ? gq : ik ? gk[1] : gk[0];
    const int piece = ic < n_scq ? kp * KTP * 2 + ic : r2 - ik * KT * 2;
    sc_reg = *((const u32x4*)(a.scales + (size_t)g * KT * 16) + piece);
  }
  const u32x4 xr0 = *(const u32x4*)(a.fx + 8 * (tid < K8 ? tid : K8 - 1));
  float ss4[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) ss4[j] = a.ss[lane + 64 * j < a.n_ss ? lane + 64 * j : 0];
  asm volatile("" ::: "memory");   // (the small loads stay ahead of the weights: staging waits for them only)
  // head_dim 128: every wave's small loads enter the CU's queue before any wave's 12 KiB of weights (a
  // barrier orders the issue only; it waits for no load), so no wave's x waits behind the others' weights
  if constexpr (HD == 128 && TI_QA_ISSUE_BARRIER) __builtin_amdgcn_s_barrier();
  // weights: q items kt = kp * KTP + wave + 8 i (i < KTP / 8), k / v items kt = wave + 8 i (i < KT / 8)
  u32x4 wq[NQ][C];
#pragma unroll
  for (int i = 0; i < NQ; ++i) {
    const u32x4* src = a.tiles + ((size_t)gq * KT + kp * KTP + wave + kQaWaves * i) * (kWave * C) + lane;
#pragma unroll
    for (int c = 0; c < C; ++c) wq[i][c] = *(src + c * kWave);
  }
  // The k / v tiles' weights: at head_dim 128 (MHA: every workgroup exactly kQaMaxKv tiles, checked on the
  // host) right behind the q part's, with no branch, so the CU's queue stays full from the start; with a
  // runtime count (GQA) after the staging barrier (a branch around loads issued before it would make the
  // staging wait count them: they are needed only after the q part)
  constexpr bool kKvwUniform = HD == 128;
  u32x4 wk[kQaMaxKv][NK][C];
  auto load_kv_weights = [&]() {
#pragma unroll
    for (int t = 0; t < kQaMaxKv; ++t)
#pragma unroll
      for (int i = 0; i < NK; ++i)
        if (kKvwUniform || t < nkv) {   // (wave-uniform)
          const u32x4* src = a.tiles + ((size_t)gk[t] * KT + wave + kQaWaves * i) * (kWave * C) + lane;
#pragma unroll
          for (int c = 0; c < C; ++c) wk[t][i][c] = __builtin_nontemporal_load(src + c * kWave);
        }
  };
  if constexpr (kKvwUniform && !TI_QA_KVW_LATE) load_kv_weights();
  // every weight load issued before the staging's first wait: memory ops cannot cross the first asm, and
  // the small loads' values pass through the second, so no use of them is scheduled above the loads
  asm volatile("" ::: "memory");
  u32x4 xr = xr0;
  if constexpr (kKvwUniform)
    asm volatile("" : "+v"(xr), "+v"(sc_reg), "+v"(ss4[0]), "+v"(ss4[1]), "+v"(ss4[2]), "+v"(ss4[3]));
  // ---- 2. stage x (int4: the high-nibble slots scaled by 1/16 and the offset correction, as
  // gemv_wq_kernel's register prep), the scales; rms of the row
  {
    f16x8 hx = __builtin_bit_cast(f16x8, xr);
    float part = 0.0f;
    if constexpr (BITS == 4) part = int4_x_prep_qa(hx);
    *(f16x8*)(xl + 8 * tid) = hx;   // (every thread: no branch for the compiler to sink the x load into;
                                    // pieces past K land in LDS no one reads, 8 * 512 = kQaMaxK)
    if constexpr (BITS == 4) {
      part = group_sum<16>(part);
      if (tid < K8 && (lane & 15) == 0) corr[tid >> 4][0] = part;
    }
  }
  // (every thread stores, the surplus into a dummy slot: a conditional store lets the compiler sink the
  // load into the branch, behind the weight stream, and wait for all of it there)
  {
    const int r2 = tid - n_scq, ik = r2 >= KT * 2 ? 1 : 0;
    *(tid < n_scq ? (u32x4*)&sl[0][0][0] + (kp * KTP * 2 + tid)
                  : tid < n_sc ? (u32x4*)&sl[1 + ik][0][0] + (r2 - ik * KT * 2) : &sl_dummy) = sc_reg;
  }
  float rms;
  {
    float t = 0.0f;
#pragma unroll
    for (int j = 0; j < 4; ++j) t += lane + 64 * j < a.n_ss ? ss4[j] : 0.0f;
    t = group_sum<kWave>(t);
    rms = sqrtf(t / (float)K + a.eps);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  STAMP_MARK(ph_staged);
  const int p = __builtin_amdgcn_readfirstlane(p_v);
  const unsigned gen = (unsigned)__builtin_amdgcn_readfirstlane((int)gen_prev) + 1u;

  // RoPE (cos, sin) of the thread's q dim (threads < HD) or k row (wave 2 + i, lanes < 16: the i-th
  // k / v tile's row) (loaded by every thread, clamped: no branch around the load)
  float2 cs;
  {
    const int gkw = wave == 3 ? gk[1] : gk[0];
    const int d = tid < HD ? tid : ((gkw - qd / 16) * 16 + (tid & 15)) % HD;
    cs = *(const float2*)(a.rope_cs + (size_t)p * HD + (d & ~1));
  }

  if constexpr (!kKvwUniform && !TI_QA_KVW_LATE) load_kv_weights();


  // ---- 3. the K/V ring of the attention goes out now (its addresses need only p)
  constexpr int LPK = HD / 8, KPW = 64 / LPK, RA = TI_QA_KV_RING;   // (5: a whole 2048-key split in flight)
  const int dl = lane % LPK, kg = lane / LPK;
  const int L = p;   // the old keys [0, p); split S - 1 is last_extra keys short
  const int chunk = (L + a.last_extra + S - 1) / S;
  const int s0 = min(L, s * chunk), s1 = s == S - 1 ? L : min(L, s0 + chunk);
  const int nslot = s1 > s0 ? (s1 - s0 + KPW - 1) / KPW : 0;
  const int atot = wave < nslot ? (nslot - wave + kQaWaves - 1) / kQaWaves : 0;
  const size_t kv_off = (size_t)(h >> a.kv_shift) * a.max_seq * HD;
  auto slot_key = [&](int i) { return s0 + (wave + kQaWaves * i) * KPW + kg; };
  int arj = 0;
  u32x4 kr[RA], vr[RA];
  auto arefill = [&](int q) {
    const int key = min(slot_key(arj < atot ? arj : max(atot - 1, 0)), max(s1 - 1, 0));
    ++arj;
    kr[q] = ld_kv((const u32x4*)(a.kc + kv_off + (size_t)key * HD + dl * 8));
    vr[q] = ld_kv((const u32x4*)(a.vc + kv_off + (size_t)key * HD + dl * 8));
  };
  constexpr bool kKvLate = TI_QA_KV_LATE < 0 ? HD == 128 : TI_QA_KV_LATE != 0;
  if constexpr (!kKvLate) {
#pragma unroll
    for (int q = 0; q < RA; ++q) arefill(q);
  }

  // ---- 4. the GEMV items (gemv_wq_kernel's: 4 MFMA steps, the int4 correction, one fp32 FMA by the
  // group scale), the q part and the k / v tile each into its slab row
  const int r = lane & 15, kq = lane >> 4;
  const f16* xrow = xl + kq * 32;
  uint32_t magic;
  asm volatile("v_mov_b32 %0, 0x64006400" : "=v"(magic));
  auto item = [&](const u32x4 (&w)[C], int kt, const uint16_t* scl, f32x4& acc) {
    f32x4 t = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      const f16x8 bf = dequant_step<BITS>(w, s4, magic);
      const f16x8 af = *(const f16x8*)(xrow + kt * 128 + s4 * 8);
      t = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, bf, t, 0, 0, 0);
    }
    if constexpr (BITS == 4) t -= *(const f32x4*)(&corr[kt][4 * kq]);
    const float sc = h2f(scl[kt * 16 + r]);
    acc[0] = fmaf(sc, t[0], acc[0]);
    acc[1] = fmaf(sc, t[1], acc[1]);
    acc[2] = fmaf(sc, t[2], acc[2]);
    acc[3] = fmaf(sc, t[3], acc[3]);
  };
  {   // the q part first: the head's siblings wait for it
    f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int i = 0; i < NQ; ++i) item(wq[i], kp * KTP + wave + kQaWaves * i, &sl[0][0][0], acc);
    if (lane < 16) slab[0][wave][lane] = acc[0];   // row 0 of the C layout: lanes 0-15, component 0
  }
  STAMP_MARK(ph_qdata);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  STAMP_MARK(ph_qpart);
#if TI_QA_KVW_LATE   // the k / v tiles' weights only now: nothing competes with the q part's bytes
  load_kv_weights();
#endif
  if constexpr (kKvLate) {   // the K/V ring after the q part: the keys then do not compete with the q stream
#pragma unroll
    for (int q = 0; q < RA; ++q) arefill(q);
  }
  // ---- 5. wave 0: publish the q part (16 sums over the 8 waves, fixed order); then the k / v tile
  if (wave == 0 && lane < 16 && (int)blockIdx.x != a.drop) {
    float v = slab[0][0][lane];
#pragma unroll
    for (int w = 1; w < kQaWaves; ++w) v += slab[0][w][lane];
    st_sc1_u64(my_slot + lane, ((unsigned long long)gen << 32) | __builtin_bit_cast(uint32_t, v));
  }
  if (nkv > 0) {
#pragma unroll
    for (int t = 0; t < kQaMaxKv; ++t)
      if (t < nkv) {
        f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int i = 0; i < NK; ++i) item(wk[t][i], wave + kQaWaves * i, &sl[1 + t][0][0], acc);
        if (lane < 16) slab[1 + t][wave][lane] = acc[0];
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();   // (uniform: nkv is the workgroup's)
    asm volatile("" ::: "memory");
  }
  STAMP_MARK(ph_kv);
  // waves 2, 3: the k / v tiles' epilogues (/ rms, RoPE of k, the cache row and the per-q-head copies)
  if (wave >= 2 && wave - 2 < nkv) {
    const int ik = wave - 2, n = lane & 15;
    float v = slab[1 + ik][0][n];
#pragma unroll
    for (int w = 1; w < kQaWaves; ++w) v += slab[1 + ik][w][n];
    v = v / rms;
    const float partner = lane_xor<1>(v);
    if (lane < 16) {
      const int ng = (ik ? gk[1] : gk[0]) * 16 + n;
      const bool is_k = ng < qd + kvd;
      float rr = v;
      if (is_k) {
        const int d = (ng - qd) % HD;
        rr = (d & 1) == 0 ? fmaf(-partner, cs.y, v * cs.x) : fmaf(v, cs.x, partner * cs.y);
      }
      const int c = ng - qd - (is_k ? 0 : kvd), kvh = c / HD, dd = c - kvh * HD;
      const uint16_t hv = f2h(rr);
      (is_k ? a.kc : a.vc)[((size_t)kvh * a.max_seq + p) * HD + dd] = hv;
      // the row's fp16 values in pairs {lo | hi << 16, generation} for the split that attends the new key
      const uint32_t pair = (uint32_t)hv | (lane_xor_u32<1>((uint32_t)hv) << 16);
      if ((n & 1) == 0) st_sc1_u64(my_slot + 16 + ik * 8 + (n >> 1), ((unsigned long long)gen << 32) | pair);
    }
  }

  // ---- 6. threads < head_dim: gather the head's q from its S workgroups (tile d / 16 from workgroups
  // tile + QT part, parts in order), / rms, RoPE (tensor_engine.cpp:1602-1612, the fused epilogue's pattern)
  if (tid < HD) {
    const int d = tid, t = d >> 4, n = d & 15;
    float v = 0.0f;
    bool lost = false;
    for (int part = 0; part < kparts; ++part) {
      const unsigned long long* g = a.xchg + ((size_t)h * S + t + QT * part) * kQaSlot + n;
      unsigned long long x = ld_sc1_u64(g);
      unsigned spin = 0;
      while ((unsigned)(x >> 32) != gen && ++spin < kQaSpin) {
        __builtin_amdgcn_s_sleep(1);
        x = ld_sc1_u64(g);
      }
      lost |= spin >= kQaSpin;
      v += __builtin_bit_cast(float, (uint32_t)x);
    }
    if (lost) st_sc1_u32(a.err + (tid & 1), 1u);   // (a per-lane address: one vector store)
    v = v / rms;
    const float partner = lane_xor<1>(v);
    const float rr = (d & 1) == 0 ? fmaf(-partner, cs.y, v * cs.x) : fmaf(v, cs.x, partner * cs.y);
    q_s[d] = rr;
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  STAMP_MARK(ph_gathered);

  // the new key (position p) of the head's kv-head: attended by the last wave of split S - 1 after its old keys
  constexpr int kNewWave = kQaWaves - 1;
  const bool new_key = s == S - 1 && wave == kNewWave;   // (wave-uniform)
  // lane dl: dims 8 dl .. 8 dl + 7 of k_p and v_p, in the granules 16 + 8 i + (dl & 1) * 4 + 0..3 of the owners of
  // k / v tile j = kv-head * (HD / 16) + dl / 2 (the inverse of qa_kv_tile; j < 2 heads S, and r / heads with r < 512
  // exact in fp32 from the +0.5 offset)
  const unsigned long long* nk_base[2];
  {
    const int dl0 = lane % (HD / 8), jk = (h >> a.kv_shift) * (HD / 16) + (dl0 >> 1), hs = a.heads * S;
    const float inv_heads = __builtin_amdgcn_rcpf((float)a.heads);
#pragma unroll
    for (int kv = 0; kv < 2; ++kv) {
      const int j = jk + kv * (a.kv_tiles >> 1), i = j >= hs ? 1 : 0, r2 = j - i * hs;
      const int q2 = (int)(((float)r2 + 0.5f) * inv_heads);
      nk_base[kv] = a.xchg + (size_t)((r2 - q2 * a.heads) * S + (S - 1 - q2)) * kQaSlot + 16 + i * 8 + (dl0 & 1) * 4;
    }
  }

  // ---- 7. attention of q_h over the split's old keys (attn_split_body, one q-head, LPK lanes a key)
  float qf[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) qf[e] = q_s[dl * 8 + e] * a.scale;
  float mrun = -INFINITY, lrun = 0.0f, oacc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) oacc[e] = 0.0f;
  int ci = 0;
  auto consume_key = [&](const u32x4& kv, const u32x4& vv, bool valid) {
    float kf[8], vf[8];
    unpack8(kv, kf);
    unpack8(vv, vf);
    float dq = 0.0f;
#pragma unroll
    for (int e = 0; e < 8; ++e) dq = fmaf(qf[e], kf[e], dq);
    dq = group_sum<LPK>(dq);
    const float sc = valid ? dq : -INFINITY;
    const float mn = fmaxf(mrun, sc);
    const float alpha = mrun == mn ? 1.0f : __expf(mrun - mn);
    const float pr = valid ? __expf(sc - mn) : 0.0f;
    lrun = fmaf(lrun, alpha, pr);
    mrun = mn;
#pragma unroll
    for (int e = 0; e < 8; ++e) oacc[e] = fmaf(pr, vf[e], oacc[e] * alpha);
  };
  auto consume = [&](const u32x4& kv, const u32x4& vv) {
    const bool valid = slot_key(ci) < s1;
    ++ci;
    consume_key(kv, vv, valid);
  };
  int a0 = 0;
  for (; a0 + RA <= atot; a0 += RA) {
#pragma unroll
    for (int q = 0; q < RA; ++q) {
      ring_pin(kr[q], vr[q], lrun);
      consume(kr[q], vr[q]);
      arefill(q);
    }
  }
  auto ring_tail = [&]() {
#pragma unroll
    for (int q = 0; q < RA; ++q)
      if (a0 + q < atot) consume(kr[q], vr[q]);
  };
  if (new_key) {
    // k_p / v_p's granules (nk_base), loaded once every refill is out (a younger load would hold up the ring's
    // waits), checked after the ring's last slots -- the owners' epilogues published them long before (a bounded wait)
    const unsigned long long* gp[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) gp[e] = nk_base[e >> 2] + (e & 3);
    unsigned long long nkg[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) nkg[e] = ld_sc1_u64(gp[e]);
    // (the last slots' values pass through here: the tail's math stays below the granule loads)
#pragma unroll
    for (int q = 0; q < RA; ++q) asm volatile("" : "+v"(kr[q]), "+v"(vr[q])::"memory");
    ring_tail();
    bool lost = false;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      unsigned spin = 0;
      while ((unsigned)(nkg[e] >> 32) != gen && ++spin < kQaSpin) {
        __builtin_amdgcn_s_sleep(1);
        nkg[e] = ld_sc1_u64(gp[e]);
      }
      lost |= spin >= kQaSpin;
    }
    if (lost) st_sc1_u32(a.err + (lane & 1), 1u);
    const u32x4 kk = {(uint32_t)nkg[0], (uint32_t)nkg[1], (uint32_t)nkg[2], (uint32_t)nkg[3]};
    const u32x4 vv = {(uint32_t)nkg[4], (uint32_t)nkg[5], (uint32_t)nkg[6], (uint32_t)nkg[7]};
    consume_key(kk, vv, kg == 0);
  } else {
    ring_tail();
  }
  {   // merge the lane groups of the wave
    const float mx = groups_max<LPK>(mrun);
    const float f = mrun == -INFINITY ? 0.0f : __expf(mrun - mx);
    const float l = groups_sum<LPK>(lrun * f);
#pragma unroll
    for (int e = 0; e < 8; ++e) oacc[e] = groups_sum<LPK>(oacc[e] * f);
    mrun = mx;
    lrun = l;
  }
  STAMP_MARK(ph_attn);
  if (lane < LPK)
#pragma unroll
    for (int e = 0; e < 8; ++e) s_acc[wave][dl * 8 + e] = oacc[e];
  if (lane == 0) {
    s_m[wave] = mrun;
    s_l[wave] = lrun;
  }
  __syncthreads();
  if (tid < HD) {   // merge the waves; the split's normalised row and (max, sum)
    const int d = tid;
    float mx = s_m[0];
#pragma unroll
    for (int w = 1; w < kQaWaves; ++w) mx = fmaxf(mx, s_m[w]);
    float o = 0.0f, l = 0.0f;
    if (mx != -INFINITY) {
#pragma unroll
      for (int w = 0; w < kQaWaves; ++w) {
        const float f = s_m[w] == -INFINITY ? 0.0f : __expf(s_m[w] - mx);
        o = fmaf(f, s_acc[w][d], o);
        l = fmaf(f, s_l[w], l);
      }
    }
    const size_t rrow = (size_t)h * S + s;
    a.part_o[rrow * HD + d] = f2h(l > 0.0f ? o / l : 0.0f);
    if (d == 0) *(float2*)(a.part_ml + 2 * rrow) = make_float2(mx, l);
  }
  STAMP_MARK(ph_end);
  stamp_end(a.stamp, t_entry, ph_staged, ph_qdata, ph_qpart, ph_kv, ph_gathered, ph_attn, ph_end);
}

}  // namespace ti

using namespace ti;

extern "C" size_t ti_qkv_attn_part_o_elems(int heads, int head_dim, int splits) {
  return (size_t)heads * head_dim * (size_t)(splits + 2);
}
extern "C" size_t ti_qkv_attn_part_ml_elems(int heads, int head_dim, int splits) {
  return (size_t)heads * 2 * (size_t)splits + (size_t)heads * head_dim;
}
// the granules, then the error words (a wait expired: a sibling's part never came)
static size_t qa_granule_bytes(int heads, int splits) { return (size_t)heads * splits * kQaSlot * 8; }
extern "C" size_t ti_qkv_attn_xchg_bytes(int heads, int splits) { return qa_granule_bytes(heads, splits) + 64; }
extern "C" size_t ti_qkv_attn_error_offset(int heads, int splits) { return qa_granule_bytes(heads, splits); }

// the (q items, k / v items) per wave a kernel is instantiated for, by bits and head_dim (see the dispatch)
// (head_dim 128 kernels assume every workgroup has exactly kQaMaxKv k / v tiles: kv_tiles = 2 heads splits)
static bool qa_has_kernel(int bits, int head_dim, int nq, int nk, bool kv_uniform) {
  if (head_dim == 64) return (bits == 4 || bits == 8) && ((nq == 1 && (nk == 1 || nk == 2)) || (nq == 2 && nk == 2));
  return head_dim == 128 && (bits == 4 || bits == 8) && nq == 4 && nk == 4 && kv_uniform;
}

extern "C" int ti_qkv_attn_supported(int bits, int K, int heads, int kv_heads, int head_dim, int splits) {
  if ((bits != 4 && bits != 8) || (head_dim != 64 && head_dim != 128) || K < 1024 || K > kQaMaxK || K % 128 ||
      heads * head_dim > 4096 || kv_heads < 1 || heads < kv_heads || heads % kv_heads || (heads / kv_heads) & (heads / kv_heads - 1))
    return 0;
  const int QT = head_dim / 16, KT = K / 128, kv_tiles = 2 * kv_heads * head_dim / 16;
  if (splits < QT || splits > TI_ATTN_MAX_PART_SPLITS || splits % QT || KT % (splits / QT) || (KT / (splits / QT)) % 8 ||
      kv_tiles > heads * splits * kQaMaxKv)
    return 0;
  return qa_has_kernel(bits, head_dim, KT / (splits / QT) / kQaWaves, KT / kQaWaves, kv_tiles == kQaMaxKv * heads * splits)
             ? 1 : 0;
}

extern "C" int ti_qkv_attn_partials(const void* tiles, const uint16_t* scales, int bits, const uint16_t* fx,
                                    const float* ss_in, int n_ss, float eps, const float* rope_cs, const int32_t* pos,
                                    uint16_t* k_cache, uint16_t* v_cache, int max_seq, int K, int heads, int kv_heads,
                                    int head_dim, int splits, uint16_t* part_o, float* part_ml, void* xchg,
                                    ti_stream_t stream) {
  if (!tiles || !scales || !fx || !ss_in || !rope_cs || !pos || !k_cache || !v_cache || !part_o || !part_ml || !xchg)
    return ti_set_error(TI_ERR_ARG, "ti_qkv_attn_partials: null pointer");
  if (bits != 4 && bits != 8)
    return ti_set_error(TI_ERR_UNSUPPORTED, "ti_qkv_attn_partials: bits %d (4 or 8)", bits);
  if (head_dim != 64 && head_dim != 128)
    return ti_set_error(TI_ERR_UNSUPPORTED, "ti_qkv_attn_partials: head_dim %d (64 or 128)", head_dim);
  const int QT = head_dim / 16, KT = K / 128;
  if (K < 1024 || K > kQaMaxK || K % 128 || n_ss < 1 || n_ss > 256 || max_seq < 1 || heads * head_dim > 4096)
    return ti_set_error(TI_ERR_ARG, "ti_qkv_attn_partials: K %d (1024..%d, %% 128), n_ss %d (1..256)", K, kQaMaxK, n_ss);
  int kv_shift = 0;
  while (kv_heads > 0 && (kv_heads << kv_shift) < heads) ++kv_shift;
  if (kv_heads < 1 || heads < kv_heads || (kv_heads << kv_shift) != heads)
    return ti_set_error(TI_ERR_UNSUPPORTED, "ti_qkv_attn_partials: heads %d / kv_heads %d (a power of two)", heads,
                        kv_heads);
  const int kv_tiles = 2 * kv_heads * head_dim / 16;
  // splits: a multiple of the q tiles of a head, each k-part a multiple of 8 k-tiles (whole waves)
  if (splits < QT || splits > TI_ATTN_MAX_PART_SPLITS || splits % QT || KT % (splits / QT) ||
      (KT / (splits / QT)) % 8 || kv_tiles > heads * splits * kQaMaxKv)
    return ti_set_error(TI_ERR_ARG, "ti_qkv_attn_partials: splits %d (a multiple of %d up to %d that splits %d k-tiles "
                        "into multiples of 8)", splits, QT, TI_ATTN_MAX_PART_SPLITS, KT);
  QkvAttnArgs a;
  a.tiles = (const u32x4*)tiles;
  a.scales = scales;
  a.fx = fx;
  a.ss = ss_in;
  a.n_ss = n_ss;
  a.eps = eps;
  a.rope_cs = rope_cs;
  a.pos = pos;
  a.kc = k_cache;
  a.vc = v_cache;
  a.max_seq = max_seq;
  a.K = K;
  a.heads = heads;
  a.kv_heads = kv_heads;
  a.kv_shift = kv_shift;
  a.splits = splits;
  a.kv_tiles = kv_tiles;
  // the last split's workgroups also compute a k / v tile (when every head's has one): give that split
  // twice as many fewer keys as the tile has bytes (its epilogue and cache writes besides; 0 / 1x / 2x:
  // 1684 / 1704 / 1710 tok/s with the 5-slot ring, 1x / 2x 1716 / 1730 with 3 slots, profiles/r6_qa_ab.txt;
  // TI_QA_EXTRA overrides, 0 = equal splits)
  {
    const int tile_bytes = KT * 1024 * (bits / 4), key_bytes = 2 * head_dim * 2;
    static const int env = [] {
      const char* v = getenv("TI_QA_EXTRA");
      return v ? atoi(v) : -1;
    }();
    // (MHA, every split with its tiles: with the new key attended in the launch, split S - 1's last wave reads 8
    // granules before it -- one ring slot of keys per wave less there covers their latency)
    a.last_extra = env >= 0 ? env
                   : kv_tiles >= heads && kv_tiles < heads * splits ? 2 * tile_bytes / key_bytes
                   : kQaWaves * (64 / (head_dim / 8));
  }
  a.scale = 1.0f / sqrtf((float)head_dim);   // tensor_engine.cpp:1288, as ti_attn_decode
  a.part_o = part_o;
  a.part_ml = part_ml;
  a.xchg = (unsigned long long*)xchg;
  a.err = (uint32_t*)((char*)xchg + qa_granule_bytes(heads, splits));
  {   // (read per call: a test sets and clears it; captured graphs keep the value they were captured with)
    const char* v = getenv("TI_QA_DROP");
    a.drop = v ? atoi(v) : -1;
  }
  const int grid = heads * splits;
  a.stamp = ti_stamp_next(STAMP_ATTN, grid);
  hipStream_t s = (hipStream_t)stream;
  if (head_dim == 128 && kv_tiles != kQaMaxKv * heads * splits)
    return ti_set_error(TI_ERR_UNSUPPORTED, "ti_qkv_attn_partials: head_dim 128 needs %d k / v tiles per workgroup",
                        kQaMaxKv);
  const int nq = KT / (splits / QT) / kQaWaves, nk = KT / kQaWaves, key = nq * 10 + nk;
  const dim3 g(grid), blk(kQaThreads);
#define TI_QA_CASE(B, H, Q, KK)                                                          \
  if (bits == B && head_dim == H && key == Q * 10 + KK) {                                \
    hipLaunchKernelGGL((qkv_attn_kernel<B, H, Q, KK>), g, blk, 0, s, a);               \
    TI_LAUNCH_CHECK("qkv_attn_kernel");                                                  \
    return TI_OK;                                                                        \
  }
  TI_QA_CASE(8, 64, 1, 2)   // TinyLlama-1.1B (K 2048, 8 splits: two k-parts of 8 k-tiles)
  TI_QA_CASE(4, 64, 1, 2)
  TI_QA_CASE(8, 64, 1, 1)   // K 1024, 4 splits
  TI_QA_CASE(4, 64, 1, 1)
  TI_QA_CASE(8, 64, 2, 2)   // K 2048, 4 splits
  TI_QA_CASE(4, 64, 2, 2)
  TI_QA_CASE(4, 128, 4, 4)  // Llama-2-7B (K 4096, 8 splits: one q tile each)
  TI_QA_CASE(8, 128, 4, 4)
#undef TI_QA_CASE
  return ti_set_error(TI_ERR_UNSUPPORTED, "ti_qkv_attn_partials: no kernel for bits %d, head_dim %d, %d q / %d k-v items per wave",
                      bits, head_dim, nq, nk);
}
