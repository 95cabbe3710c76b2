// prefill_attn.hip -- causal attention of a prompt chunk over its own stream's cache, on MFMA.
//
// The attention of forward_pass over prompt rows (inference_engine.cpp:1429-1491, which calls
// TensorEngine::multi_head_attention, src/core/tensor_engine.cpp:1149-1252): row m (position
// pos[m]) attends to keys [0, pos[m]] of the stream's fp16 cache, s_j = (q . k_j) / sqrt(hd),
// softmax, o = sum_j p_j v_j; q-head h reads kv-head h / (heads / kv_heads).
//
// The decode kernel (attention.hip) gives every row its own workgroups, so a chunk of R rows
// reads the prefix R times.  Here one wave owns 16 (row, q-head) columns -- 16 rows of one head,
// or 16 / G rows of all G heads of a GQA group -- and streams the kv-head's keys once for them in
// blocks of 16, on fp16 MFMA with the fp32 operand (q, p) split into fp16 hi + lo: two MFMAs
// give the products and sums to ~fp32 accuracy, as in the reference (K / V are fp16 exactly),
// in an eighth of the MFMA cycles of v_mfma_f32_16x16x4_f32 (the first version):
//   S^T = K Q^T   v_mfma_f32_16x16x32_f16, A = K (lane: key l&15, dims 32c + 8(l>>4) + e),
//                 B = Q^T (column l&15, same dims), hd/32 steps x (hi, lo); D holds
//                 S^T[key 4(l>>4)+i][column l&15]
//   online softmax per column: 4 values per lane, two xor-shuffles across the lane groups;
//                 masked keys (key > pos[row]) get p = 0
//   O^T += V^T P^T v_mfma_f32_16x16x16_f16: its B fragment (column l&15, keys 4(l>>4) + e) is
//                 exactly the lane's own 4 p values (hi, lo); A for output tile t is V[key][dim
//                 (l&15) hd/16 + t], half t of the lane's four 16-byte V loads (byte permutes);
//                 D holds O^T[dim (4(l>>4) + i) hd/16 + t][column l&15]
// So every accumulator row of a lane belongs to the lane's own column: each block's alpha rescales
// it in place, and the lane writes hd/4 contiguous outputs of its column at the end.
// Queries are dealt longest-prefix first; a 4-block K / V ring per wave hides the loads.
#include <math.h>
#include <stdlib.h>

#include <atomic>

#include "common.hpp"

namespace ti {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int HD>
struct PfRaw;   // one lane's 16 (K) / hd/16 (V) fp16 values
template <>
struct PfRaw<128> {
  using K = u32x4[4];   // 32 dims
  using V = u32x4;      // 8 dims
};
template <>
struct PfRaw<64> {
  using K = u32x4[2];   // 16 dims
  using V = uint2;      // 4 dims
};

typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));

// fp32 x -> (hi, lo) fp16 with hi + lo = x to ~2^-22 relative
__device__ __forceinline__ void pf_split(float x, _Float16& hi, _Float16& lo) {
  hi = (_Float16)x;
  lo = (_Float16)(x - (float)hi);
}

#ifndef TI_PF_DIAG
#define TI_PF_DIAG 0   // diagnostics only (tools/r5_pfdiag.sh, r5_pfwgdiag.sh): 1 cache-resident K / V, 2 no math;
                       // shared-K/V kernel: 4 ring and barriers only, 8 no copies past the prologue
#endif
#ifndef TI_PF_PERMLANE
#define TI_PF_PERMLANE 1   // the softmax's cross-row max by v_permlane16/32_swap instead of ds_bpermute
#endif
#ifndef TI_PF_RING
#define TI_PF_RING 3   // K / V blocks in flight per wave (3: two waves per SIMD, held to 256 registers)
#endif
#ifndef TI_PF_RING_DEEP
#define TI_PF_RING_DEEP 4   // the ring when every wave of the launch has a SIMD to itself (4 and 6 measured equal)
#endif

// WPE: waves per SIMD the shallow-ring build must fit (2: at most 256 registers with the AGPRs)
template <int HD, int RING = TI_PF_RING, int WPE = 1>
__global__ __launch_bounds__(64, WPE) void attn_prefill_kernel(const float* __restrict__ q, const uint16_t* __restrict__ kc,
                                                          const uint16_t* __restrict__ vc, int max_seq,
                                                          const int32_t* __restrict__ pos, int M, int heads, int gsh,
                                                          float scale, uint16_t* __restrict__ out) {
  constexpr int DV = HD / 16, KW = HD / 32;   // K: one 32-dim MFMA step per u32x4
  using KRaw = typename PfRaw<HD>::K;
  using VRaw = typename PfRaw<HD>::V;
  const int lane = threadIdx.x, r = lane & 15, g = lane >> 4;
  // GQA: the 16 columns are (16 / G) rows x the G q-heads of kv-head blockIdx.y (column c: row
  // c >> gsh, head c & (G - 1)), so each K / V block serves the whole group
  const int G = 1 << gsh, qpw = 16 >> gsh;
  const int qb = gridDim.x - 1 - blockIdx.x, kvh = blockIdx.y;
  const int q0 = qb * qpw, qi = min(q0 + (r >> gsh), M - 1), h = kvh * G + (r & (G - 1));
  const int p = pos[qi];
  int kmax = p, kmin = p;
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) {
    kmax = max(kmax, __shfl_xor(kmax, o, 64));
    kmin = min(kmin, __shfl_xor(kmin, o, 64));
  }
  // B operand of step c: dims 32c + 8g + e of this lane's column, split into fp16 hi + lo
  f16x8 qh[KW], ql[KW];
  {
    const float* qr = q + ((size_t)qi * heads + h) * HD + 8 * g;
#pragma unroll
    for (int c = 0; c < KW; ++c) {
      const float4 t0 = *(const float4*)(qr + 32 * c), t1 = *(const float4*)(qr + 32 * c + 4);
      const float v[8] = {t0.x, t0.y, t0.z, t0.w, t1.x, t1.y, t1.z, t1.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        _Float16 hi, lo;
        pf_split(v[e] * scale, hi, lo);
        qh[c][e] = hi;
        ql[c][e] = lo;
      }
    }
  }
  // K / V through buffer loads (the kv-head's cache is the resource, byte offsets per lane): a
  // plain load whose value feeds the ring's loop phi is sunk below the phi by the compiler (one
  // load at the use, nothing in flight); the buffer intrinsic keeps each refill where it is issued
  const auto krs = buffer_rsrc(kc + (size_t)kvh * max_seq * HD), vrs = buffer_rsrc(vc + (size_t)kvh * max_seq * HD);
  // keys past every column's prefix (kmax) may be unwritten (NaN): they read row kmax instead,
  // finite, which their p = 0 then multiplies away exactly (no branch per load); a block past the
  // last (a refill that is never consumed) reads row kmax too, a cache hit
  const int kl = min(kmax, max_seq - 1);
  auto load = [&](int kb, KRaw& k, VRaw (&v)[4]) {
#if TI_PF_DIAG & 1   // diagnostic: every block re-reads block 0 (cache-resident K / V)
    kb = 0;
#endif
    const int kk = min(kb * 16 + r, kl);
#pragma unroll
    for (int c = 0; c < KW; ++c)
      k[c] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(krs, (kk * HD + 8 * g + 32 * c) * 2, 0, 0));
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int off = (min(kb * 16 + 4 * g + j, kl) * HD + r * DV) * 2;
      if constexpr (HD == 128) v[j] = __builtin_bit_cast(VRaw, __builtin_amdgcn_raw_buffer_load_b128(vrs, off, 0, 0));
      else v[j] = __builtin_bit_cast(VRaw, __builtin_amdgcn_raw_buffer_load_b64(vrs, off, 0, 0));
    }
  };
  f32x4 acc[DV];
#pragma unroll
  for (int t = 0; t < DV; ++t) acc[t] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
  float m_run = -INFINITY, l_run = 0.0f;
  const int nkb = kmax / 16 + 1;
  // K / V blocks in flight: a ring of kPfRing blocks, each slot refilled right after its block
  // is consumed (one or two waves per SIMD: the ring, not other waves, hides the load latency)
  constexpr int kPfRing = RING;
  KRaw kr[kPfRing];
  VRaw vr[kPfRing][4];
#pragma unroll
  for (int u = 0; u < kPfRing; ++u) load(u, kr[u], vr[u]);   // past nkb: clamped rows, zero V
  // let the first blocks land before the loop: with loads of the prologue still in flight at the
  // loop head the compiler merges their (different) issue order with the loop's own and waits for
  // every load at the top of each pass; with none, the loop's count alone sets the waits
  __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
  // NB blocks (16 NB keys) per online-softmax step: one column max across the four lanes, one
  // alpha and one rescale of O per step (2 when the ring divides into pairs); the wave's time is
  // this chain, not the K / V stream
#ifndef TI_PF_NB
#define TI_PF_NB 2   // blocks per softmax step (at most; a divisor of the ring)
#endif
  constexpr int NB = kPfRing % TI_PF_NB == 0 ? TI_PF_NB : kPfRing % 2 == 0 ? 2 : 1;
  for (int kb0 = 0; kb0 < nkb; kb0 += kPfRing) {
#pragma unroll
    for (int u = 0; u < kPfRing; u += NB) {
      // no exit inside the pass: blocks past nkb hold only keys past every column's position, so
      // they score -inf, leave m and l alone (alpha 1) and add p = 0 times finite V -- exactly
      // nothing; a straight-line pass keeps the loads in flight across the back edge countable
      const int kb = kb0 + u;
      // order the steps: this step's K enters through an empty asm issued after the previous step's
      // softmax, so its S = K Q^T cannot be hoisted into earlier steps, where it would wait for the
      // blocks loaded last and drain the ring once per pass
#pragma unroll
      for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int c = 0; c < KW; ++c) asm volatile("" : "+v"(kr[u + b][c]));
#if TI_PF_DIAG & 2   // diagnostic: the K / V stream alone (each slot waited for and refilled, no math)
      if constexpr (HD == 128) {
#pragma unroll
        for (int b = 0; b < NB; ++b) {
#pragma unroll
          for (int j = 0; j < 4; ++j) asm volatile("" : "+v"(vr[u + b][j]));
          load(kb + b + kPfRing, kr[u + b], vr[u + b]);
        }
        continue;
      }
#endif
      f32x4 s[NB];
#pragma unroll
      for (int b = 0; b < NB; ++b) s[b] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int c = 0; c < KW; ++c)
#pragma unroll
        for (int b = 0; b < NB; ++b) {
          const f16x8 kf = __builtin_bit_cast(f16x8, kr[u + b][c]);
          s[b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf, qh[c], s[b], 0, 0, 0);
          s[b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf, ql[c], s[b], 0, 0, 0);
        }
      // keys past the column's position (and a second block past nkb: its keys are past kmax) score
      // -inf; only the steps that reach past the shortest column's position (kmin) test them
      float pv[NB][4], bm = -INFINITY;
#pragma unroll
      for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int i = 0; i < 4; ++i) pv[b][i] = s[b][i];
      if ((kb + NB) * 16 - 1 > kmin) {   // wave-uniform
        const int lim = p - kb * 16 - 4 * g;
#pragma unroll
        for (int b = 0; b < NB; ++b)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (16 * b + i > lim) pv[b][i] = -INFINITY;
      }
#pragma unroll
      for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int i = 0; i < 4; ++i) bm = fmaxf(bm, pv[b][i]);
#if TI_PF_PERMLANE
      bm = xor32_max(xor16_max(bm));   // the column's max over its 4 lane groups, VALU only
#else
      bm = fmaxf(bm, __shfl_xor(bm, 16, 64));
      bm = fmaxf(bm, __shfl_xor(bm, 32, 64));
#endif
      // The running max moves only when a column's block max exceeds it by more than kPfSlack
      // (e^8: p stays below 2981, exact enough in the fp16 hi + lo split, and l, O in fp32): the
      // O rescale -- 32 accumulators read, scaled and written back per lane -- then runs in the
      // first steps and rarely after.  softmax(s) = exp(s - m) / sum exp(s - m) for any m.
      constexpr float kPfSlack = 8.0f;
      const float mn = fmaxf(m_run, bm);   // finite: key 0 is in every row's prefix
      if (__builtin_amdgcn_ballot_w64(mn > m_run + kPfSlack) != 0) {   // wave-uniform; the first step
        const float alpha = m_run == mn ? 1.0f : __expf(m_run - mn);
        l_run *= alpha;
        m_run = mn;
#pragma unroll
        for (int t = 0; t < DV; ++t)   // O^T: every row of the lane's accumulators is its own column's
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[t][i] *= alpha;
      }
      float ps = 0.0f;
#pragma unroll
      for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          pv[b][i] = __expf(pv[b][i] - m_run);   // a masked key: exp2(-inf) = 0 exactly
          ps += pv[b][i];
        }
      l_run += ps;
      asm volatile("" : "+v"(l_run));
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        f16x4 ph, pl;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          _Float16 hi, lo;
          pf_split(pv[b][e], hi, lo);
          ph[e] = hi;
          pl[e] = lo;
        }
        uint32_t vw[4][DV / 2];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if constexpr (HD == 128) {
            vw[j][0] = vr[u + b][j][0]; vw[j][1] = vr[u + b][j][1]; vw[j][2] = vr[u + b][j][2]; vw[j][3] = vr[u + b][j][3];
          } else {
            vw[j][0] = vr[u + b][j].x; vw[j][1] = vr[u + b][j].y;
          }
        }
#pragma unroll
        for (int t = 0; t < DV; ++t) {
          const uint32_t sel = (t & 1) ? 0x07060302u : 0x05040100u;
          const uint32_t b01 = __builtin_amdgcn_perm(vw[1][t >> 1], vw[0][t >> 1], sel);
          const uint32_t b23 = __builtin_amdgcn_perm(vw[3][t >> 1], vw[2][t >> 1], sel);
          const f16x4 bf = __builtin_bit_cast(f16x4, ((unsigned long long)b23 << 32) | b01);
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x16f16(bf, ph, acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x16f16(bf, pl, acc[t], 0, 0, 0);
        }
        // unconditional refill: a branch here leaves the loop's back edge with a variable count of
        // loads in flight, and the compiler then waits for all of them at the top of every pass
        load(kb + b + kPfRing, kr[u + b], vr[u + b]);
      }
    }
  }
  float lt = l_run + __shfl_xor(l_run, 16, 64);
  lt += __shfl_xor(lt, 32, 64);
  // lane (r, g) holds O^T[dim DV (4g + i) + t][column r] in acc[t][i]: dims 4g DV .. 4g DV + 4 DV - 1
  // of column r's (row, head), contiguous
  const float inv = 1.0f / lt;
  const int row = q0 + (r >> gsh), hh = kvh * G + (r & (G - 1));
  if (row < M) {
    uint16_t* dst = out + ((size_t)row * heads + hh) * HD + 4 * g * DV;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      uint32_t o[DV / 2];
#pragma unroll
      for (int t = 0; t < DV / 2; ++t) {
        const uint16_t lo = __builtin_bit_cast(uint16_t, (_Float16)(acc[2 * t][i] * inv));
        const uint16_t hi = __builtin_bit_cast(uint16_t, (_Float16)(acc[2 * t + 1][i] * inv));
        o[t] = lo | ((uint32_t)hi << 16);
      }
      if constexpr (HD == 128) *(ti::u32x4*)(dst + i * DV) = (ti::u32x4){o[0], o[1], o[2], o[3]};
      else *(uint2*)(dst + i * DV) = make_uint2(o[0], o[1]);
    }
  }
}

// ---------------------------------------------------------------- shared K / V blocks (hd 128)
// The kernel above gives every wave its own K / V stream from L2, and that stream bounds it
// (profiles/r5_prefill_attn_diag.txt: 21.5 of 24 us at 512 rows; half-line K reads, ~80 block loads
// per CU).  Here a workgroup takes 4 query blocks of one kv-head -- query wave q block j + q QG, so
// every workgroup holds long and short chains -- and copies each K / V block of their union once
// into an LDS ring (LDS-DMA, full 128-byte lines), which all its waves read.
// The per-wave math is the kernel above's: S^T = K Q^T on fp16 MFMA with the fp32 operand in hi + lo,
// online softmax per column, two blocks per step, and O^T += V^T P^T as one 32-key 16x16x32 product.
//   K block in LDS: [16 keys][16 chunks of 16 B], the logical chunk c of key row r at physical c ^ r
//   (an A-fragment read, lane (r, g) chunk 4c + g, is conflict-free in every ds_read_b128 lane group);
//   V block: [16 keys][16 chunks], unswizzled (lane (r, g) reads chunk r of rows 4g + j).
// Per iteration of BI blocks (2 per half): wait for this wave's 4 DMAs of the iteration; barrier
// (everyone's landed, and everyone is done with the previous iteration's blocks); DMA the iteration
// R / BI - 1 ahead into the slots just freed; compute.  Waves past their own chain keep copying until
// the workgroup's longest is done; the last DMAs drain before the ring's LDS is reused or released.
#ifndef TI_PF_WG_RING
#define TI_PF_WG_RING 6    // K / V blocks in the LDS ring (8 KiB each), 4-wave workgroups
#endif
#ifndef TI_PF_QK_SPLIT
#define TI_PF_QK_SPLIT 0   // shared-K/V kernel: S = K Q^T's hi and lo products in separate chains
#endif
#ifndef TI_PF_WG_LATE_DMA
#define TI_PF_WG_LATE_DMA 0   // 1: DMAs issued after the step's S = K Q^T (even, profiles/r5_prefill_wg_latedma_ab.txt)
#endif
#ifndef TI_PF_WG_RING2
#define TI_PF_WG_RING2 8   // the same, 8-wave workgroups (4 blocks per iteration; 8 beat 12 and 16, profiles/r5_prefill_wg_ring_ab.txt)
#endif
// HALVES 2: 8 waves, two per SIMD -- waves w and w + 4 share query block w & 3 and take alternate
// pairs of its key blocks (iteration = 4 blocks, half h computes blocks 2 h, 2 h + 1 of it), merging
// their (max, sum, O) through LDS at the end: two chains per SIMD hide each other's latencies.
template <int HALVES, int R>
__global__ __launch_bounds__(256 * HALVES, 1) void attn_prefill_wg_kernel(const float* __restrict__ q, const uint16_t* __restrict__ kc,
                                                                 const uint16_t* __restrict__ vc, int max_seq,
                                                                 const int32_t* __restrict__ pos, int M, int heads, int gsh,
                                                                 float scale, uint16_t* __restrict__ out) {
  constexpr int HD = 128, DV = HD / 16, KW = HD / 32, NB = 2, BI = NB * HALVES;   // BI: blocks per iteration
  static_assert(R % BI == 0 && R >= 2 * BI, "ring: whole iterations, one in flight beside the one computed");
  // K and V rings in ONE array: the halves' merge at the end reuses it as scratch (4 query blocks x
  // 64 lanes x (4 DV + 2) floats), which is larger than the K ring alone
  __shared__ __attribute__((aligned(16))) uint16_t skv[2][R][16 * HD];
  static_assert(HALVES == 1 || 4 * 64 * (4 * DV + 2) * sizeof(float) <= sizeof(skv), "halves' merge scratch");
  auto& sk = skv[0];
  auto& sv = skv[1];
  __shared__ int s_kmax[4];
  const int lane = threadIdx.x & 63, r = lane & 15, g = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), qw = wave & 3, half = wave >> 2;
  const int G = 1 << gsh, qpw = 16 >> gsh;
  const int kvh = blockIdx.y, QG = gridDim.x, nq = (M + qpw - 1) / qpw;
  const int qb = (QG - 1 - blockIdx.x) + qw * QG;   // longest chains first
  const bool live = qb < nq;                        // (a wave past the chunk only copies)
  const int q0 = qb * qpw, qi = min(q0 + (r >> gsh), M - 1), h = kvh * G + (r & (G - 1));
  const int p = pos[qi];
  int kmax = p, kmin = p;
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) {
    kmax = max(kmax, __shfl_xor(kmax, o, 64));
    kmin = min(kmin, __shfl_xor(kmin, o, 64));
  }
  if (lane == 0 && half == 0) s_kmax[qw] = live ? kmax : 0;
  f16x8 qh[KW], ql[KW];
  {
    const float* qr = q + ((size_t)qi * heads + h) * HD + 8 * g;
#pragma unroll
    for (int c = 0; c < KW; ++c) {
      const float4 t0 = *(const float4*)(qr + 32 * c), t1 = *(const float4*)(qr + 32 * c + 4);
      const float v[8] = {t0.x, t0.y, t0.z, t0.w, t1.x, t1.y, t1.z, t1.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        _Float16 hi, lo;
        pf_split(v[e] * scale, hi, lo);
        qh[c][e] = hi;
        ql[c][e] = lo;
      }
    }
  }
  __syncthreads();
  const int kmax_wg = max(max(s_kmax[0], s_kmax[1]), max(s_kmax[2], s_kmax[3]));
  const int kl = min(kmax_wg, max_seq - 1);   // rows past it may be unwritten: read row kl instead
  const int nkb = kmax_wg / 16 + 1, nkb_w = live ? kmax / 16 + 1 : 0;
  const uint16_t* kbase = kc + (size_t)kvh * max_seq * HD;
  const uint16_t* vbase = vc + (size_t)kvh * max_seq * HD;
  const uint32_t sk_lds = (uint32_t)(uintptr_t)&sk[0][0], sv_lds = (uint32_t)(uintptr_t)&sv[0][0];
  // An iteration's BI blocks are 8 BI DMA instructions of 1 KiB (a block: K rows 0-3, 4-7, 8-11, 12-15,
  // then V's); wave w issues instructions 4 w .. 4 w + 3: all of K or all of V of block w / 2.
  const int dblk = wave >> 1, dv = wave & 1, dch = lane & 15;
  auto issue = [&](int kb0) {   // the iteration starting at block kb0
#if TI_PF_DIAG & 8   // diagnostic: no copies past the prologue (the math on stale blocks)
    if (kb0 >= R - BI) return;
#endif
    const int kb = kb0 + dblk, slot = kb % R;
    const uint32_t base = (dv ? sv_lds : sk_lds) + (uint32_t)(slot * 16 * HD * 2);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = 4 * i + (lane >> 4), key = min(kb * 16 + row, kl);
      const uint16_t* src = dv ? vbase + (size_t)key * HD + dch * 8 : kbase + (size_t)key * HD + ((dch ^ row) * 8);
      dma_1k_asm(src, __builtin_amdgcn_readfirstlane(base + (uint32_t)(i * 4 * HD * 2)));
    }
  };
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // q and pos in: only the DMAs are counted below
#pragma unroll
  for (int kb = 0; kb < R - BI; kb += BI) issue(kb);
  f32x4 acc[DV];
#pragma unroll
  for (int t = 0; t < DV; ++t) acc[t] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
  float m_run = -INFINITY, l_run = 0.0f;
  constexpr float kPfSlack = 8.0f;   // as above: O rescaled only when a column max moves by > 8
  for (int kbi = 0; kbi < nkb; kbi += BI) {
    // this wave's 4 DMAs of iteration kbi are the oldest of the 4 (R / BI - 1) in flight
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * (R / BI - 2)) : "memory");
    __syncthreads();
#if !TI_PF_WG_LATE_DMA
    issue(kbi + R - BI);
#endif
    const int kb = kbi + NB * half;   // this half's pair
#if TI_PF_DIAG & 4   // diagnostic: the ring and its barriers alone, no math
    const bool act = false;
#else
    const bool act = kb < nkb_w;      // wave-uniform
#endif
    f32x4 sacc[NB];
    u32x4 vraw[NB][4];
    if (act) {
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        const uint16_t* kr = &sk[(kb + b) % R][r * HD];
#if TI_PF_QK_SPLIT   // the hi and lo products in two chains (four independent per step), summed after
        f32x4 sh = (f32x4){0.0f, 0.0f, 0.0f, 0.0f}, sl = sh;
#pragma unroll
        for (int c = 0; c < KW; ++c) {
          const f16x8 kf = __builtin_bit_cast(f16x8, *(const u32x4*)(kr + (((4 * c + g) ^ r) * 8)));
          sh = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf, qh[c], sh, 0, 0, 0);
          sl = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf, ql[c], sl, 0, 0, 0);
        }
        sacc[b] = sh + sl;
#else
        sacc[b] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int c = 0; c < KW; ++c) {
          const f16x8 kf = __builtin_bit_cast(f16x8, *(const u32x4*)(kr + (((4 * c + g) ^ r) * 8)));
          sacc[b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf, qh[c], sacc[b], 0, 0, 0);
          sacc[b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf, ql[c], sacc[b], 0, 0, 0);
        }
#endif
        const uint16_t* vb = &sv[(kb + b) % R][0];
#pragma unroll
        for (int j = 0; j < 4; ++j) vraw[b][j] = *(const u32x4*)(vb + (4 * g + j) * HD + r * DV);
      }
    }
#if TI_PF_WG_LATE_DMA   // the next DMAs issued under this step's S = K Q^T rather than before it
    issue(kbi + R - BI);
#endif
    if (act) {
      float pv[NB][4], bm = -INFINITY;
#pragma unroll
      for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int i = 0; i < 4; ++i) pv[b][i] = sacc[b][i];
      if ((kb + NB) * 16 - 1 > kmin) {   // wave-uniform: a step past the shortest column's position
        const int lim = p - kb * 16 - 4 * g;
#pragma unroll
        for (int b = 0; b < NB; ++b)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (16 * b + i > lim) pv[b][i] = -INFINITY;
      }
#pragma unroll
      for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int i = 0; i < 4; ++i) bm = fmaxf(bm, pv[b][i]);
#if TI_PF_PERMLANE
      bm = xor32_max(xor16_max(bm));   // the column's max over its 4 lane groups, VALU only
#else
      bm = fmaxf(bm, __shfl_xor(bm, 16, 64));
      bm = fmaxf(bm, __shfl_xor(bm, 32, 64));
#endif
      const float mn = fmaxf(m_run, bm);
      if (__builtin_amdgcn_ballot_w64(mn > m_run + kPfSlack) != 0) {
        const float alpha = m_run == mn ? 1.0f : __expf(m_run - mn);
        l_run *= alpha;
        m_run = mn;
#pragma unroll
        for (int t = 0; t < DV; ++t)
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[t][i] *= alpha;
      }
      float ps = 0.0f;
#pragma unroll
      for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          // (half 1 may meet a column whose keys so far are all masked: m_run -inf, p 0)
          pv[b][i] = HALVES == 2 && m_run == -INFINITY ? 0.0f : __expf(pv[b][i] - m_run);
          ps += pv[b][i];
        }
      l_run += ps;
      // O^T += V^T P^T over both blocks in one 32-key product (16x16x32, the full-rate form): k index
      // 8 g + e is key 4 g + e of the first block for e < 4 and of the second for e >= 4, in the
      // A fragment (V, lane (dim r DV + t, k)) and the B fragment (P, lane (column r, k)) alike
      f16x8 ph, pl;
#pragma unroll
      for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          _Float16 hi, lo;
          pf_split(pv[b][e], hi, lo);
          ph[4 * b + e] = hi;
          pl[4 * b + e] = lo;
        }
#pragma unroll
      for (int t = 0; t < DV; ++t) {
        const uint32_t sel = (t & 1) ? 0x07060302u : 0x05040100u;
        uint32_t w[4];
#pragma unroll
        for (int b = 0; b < NB; ++b) {
          w[2 * b] = __builtin_amdgcn_perm(vraw[b][1][t >> 1], vraw[b][0][t >> 1], sel);
          w[2 * b + 1] = __builtin_amdgcn_perm(vraw[b][3][t >> 1], vraw[b][2][t >> 1], sel);
        }
        const f16x8 bf = __builtin_bit_cast(f16x8, (u32x4){w[0], w[1], w[2], w[3]});
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf, ph, acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf, pl, acc[t], 0, 0, 0);
      }
    }
  }
  // the ring's last copies (clamped rows past the end) land before the ring is reused / released
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if constexpr (HALVES == 2) {   // half 1 hands (m, l, O) to half 0 through the ring's LDS
    float* xs = (float*)&skv[0][0][0] + (size_t)qw * 64 * (4 * DV + 2);   // (within skv: static_assert above)
    if (half == 1) {
#pragma unroll
      for (int t = 0; t < DV; ++t) *(f32x4*)(xs + (4 * t) * 64 + 4 * lane) = acc[t];
      xs[4 * DV * 64 + lane] = m_run;
      xs[4 * DV * 64 + 64 + lane] = l_run;
    }
    __syncthreads();
    if (half == 1) return;
    const float m1 = xs[4 * DV * 64 + lane], l1 = xs[4 * DV * 64 + 64 + lane];
    const float mx = fmaxf(m_run, m1);
    const float f0 = m_run == -INFINITY ? 0.0f : __expf(m_run - mx), f1 = m1 == -INFINITY ? 0.0f : __expf(m1 - mx);
    l_run = l_run * f0 + l1 * f1;
#pragma unroll
    for (int t = 0; t < DV; ++t) {
      const f32x4 o1 = *(const f32x4*)(xs + (4 * t) * 64 + 4 * lane);
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[t][i] = acc[t][i] * f0 + o1[i] * f1;
    }
  }
  if (!live) return;
  float lt = l_run + __shfl_xor(l_run, 16, 64);
  lt += __shfl_xor(lt, 32, 64);
  const float inv = 1.0f / lt;
  const int row = q0 + (r >> gsh), hh = kvh * G + (r & (G - 1));
  if (row < M) {
    uint16_t* dst = out + ((size_t)row * heads + hh) * HD + 4 * g * DV;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      uint32_t o[DV / 2];
#pragma unroll
      for (int t = 0; t < DV / 2; ++t) {
        const uint16_t lo = __builtin_bit_cast(uint16_t, (_Float16)(acc[2 * t][i] * inv));
        const uint16_t hi = __builtin_bit_cast(uint16_t, (_Float16)(acc[2 * t + 1][i] * inv));
        o[t] = lo | ((uint32_t)hi << 16);
      }
      *(ti::u32x4*)(dst + i * DV) = (ti::u32x4){o[0], o[1], o[2], o[3]};
    }
  }
}

}  // namespace ti

static std::atomic<int> g_pf_kernel{0};

extern "C" int ti_attn_prefill_set_kernel(int mode) {
  if (mode < 0 || mode > 3) return -1;
  return g_pf_kernel.exchange(mode);
}

extern "C" int ti_attn_prefill(const float* q, const uint16_t* k_cache, const uint16_t* v_cache, int max_seq,
                               const int32_t* pos, int M, int heads, int kv_heads, int head_dim, uint16_t* out,
                               ti_stream_t stream) {
  if (!q || !k_cache || !v_cache || !pos || !out) return ti_set_error(TI_ERR_ARG, "ti_attn_prefill: null pointer");
  if (M < 1 || heads < 1 || kv_heads < 1 || heads % kv_heads || max_seq < 1 || M > 65535 * 16 || heads > 65535)
    return ti_set_error(TI_ERR_ARG, "ti_attn_prefill: bad sizes M=%d heads=%d kv_heads=%d max_seq=%d", M, heads,
                        kv_heads, max_seq);
  if (head_dim != 64 && head_dim != 128)
    return ti_set_error(TI_ERR_UNSUPPORTED, "ti_attn_prefill: head_dim %d not in {64,128}", head_dim);
  const int G = heads / kv_heads;
  if (G & (G - 1) || G > 16) return ti_set_error(TI_ERR_UNSUPPORTED, "ti_attn_prefill: heads / kv_heads %d not a power of 2 <= 16", G);
  const int gsh = __builtin_ctz(G), qpw = 16 >> gsh;
  const dim3 grid((M + qpw - 1) / qpw, kv_heads);
  const float scale = 1.0f / sqrtf((float)head_dim);   // tensor_engine.cpp:1288
  hipStream_t s = (hipStream_t)stream;
  // One wave per workgroup.  While the launch has at most one wave per SIMD (a 7B chunk of up to
  // 512 rows: 1024 waves on 256 CUs x 4 SIMDs) nothing is gained by fitting two waves on a SIMD,
  // so each wave keeps the deep ring: the longest rows' waves set the time, and their key
  // stream is latency-bound (one block per ~1.1 us at 3 in flight).  Larger chunks keep the
  // 3-deep ring, two waves per SIMD.
  static std::atomic<int> simds{0};
  int ns = simds.load(std::memory_order_relaxed);
  if (ns == 0) {
    int dev = 0, n = 0;
    ns = hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess
             ? 4 * n : -1;
    simds.store(ns, std::memory_order_relaxed);   // (a racing first call stores the same value)
  }
  const bool deep = (long)grid.x * grid.y <= ns;
  static const int wgk = [] {   // 0: per-wave kernel, 1: workgroup of 4 waves, 2: of 8 (key-split halves)
    const char* e = getenv("TI_PF_WG");
    return e && e[0] >= '0' && e[0] <= '2' ? e[0] - '0' : 2;
  }();
  const int forced = g_pf_kernel.load(std::memory_order_relaxed);   // ti_attn_prefill_set_kernel
  const int k = forced == 0 ? wgk : forced - 1;
  const bool wg = k > 0, wg2 = k == 2;
  const dim3 gw((grid.x + 3) / 4, kv_heads);
  // 4 query blocks of a kv-head per workgroup, K / V shared in LDS -- when that still gives every CU
  // a workgroup (256 rows of 7B: 128 workgroups, the per-wave kernel's 512 waves are faster)
  if (head_dim == 128 && wg && (forced > 1 || (long)gw.x * gw.y * 4 >= ns)) {
    if (wg2)
      hipLaunchKernelGGL((ti::attn_prefill_wg_kernel<2, TI_PF_WG_RING2>), gw, dim3(512), 0, s, q, k_cache, v_cache, max_seq,
                         pos, M, heads, gsh, scale, out);
    else
      hipLaunchKernelGGL((ti::attn_prefill_wg_kernel<1, TI_PF_WG_RING>), gw, dim3(256), 0, s, q, k_cache, v_cache, max_seq,
                         pos, M, heads, gsh, scale, out);
  } else if (head_dim == 128) {
    if (deep)
      hipLaunchKernelGGL((ti::attn_prefill_kernel<128, TI_PF_RING_DEEP>), grid, dim3(64), 0, s, q, k_cache, v_cache,
                         max_seq, pos, M, heads, gsh, scale, out);
    else
      hipLaunchKernelGGL((ti::attn_prefill_kernel<128, TI_PF_RING, 2>), grid, dim3(64), 0, s, q, k_cache, v_cache, max_seq,
                         pos, M, heads, gsh, scale, out);
  } else {
    if (deep)
      hipLaunchKernelGGL((ti::attn_prefill_kernel<64, TI_PF_RING_DEEP>), grid, dim3(64), 0, s, q, k_cache, v_cache,
                         max_seq, pos, M, heads, gsh, scale, out);
    else
      hipLaunchKernelGGL((ti::attn_prefill_kernel<64, TI_PF_RING, 2>), grid, dim3(64), 0, s, q, k_cache, v_cache, max_seq,
                         pos, M, heads, gsh, scale, out);
  }
  TI_LAUNCH_CHECK("attn_prefill_kernel");
  return TI_OK;
}
