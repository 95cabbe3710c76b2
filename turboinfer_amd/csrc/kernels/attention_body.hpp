// attention_body.hpp -- the split-K decode attention of attention.hip as a device function,
// used by attn_split_kernel (attention.hip).
#pragma once
#include <math.h>

#include "common.hpp"

namespace ti {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct AttnArgs {
  const float* q;
  const uint16_t* kc;
  const uint16_t* vc;
  const int32_t* pos;
  float* ws;
  int32_t* counters;
  uint16_t* out;
  int64_t stride;
  int32_t max_seq, M, heads, kv_heads, splits;
  float scale;
  // partials mode (ti_attn_decode_partials): every split writes its normalised row and
  // (max, sum) and the merge is left to the consumer (the O projection's x staging)
  uint16_t* part_o;   // [M][heads][splits][HD] fp16, nullptr = merge in this launch
  float* part_ml;     // [M][heads][splits][2]
  int32_t out_kt;     // > 0: out in TI_X_F16_PACKED order with K / 128 = out_kt (ti_attn_decode_packed)
  // GQA run head by head (kv_heads here = heads, G = 1): workgroup head h reads the cache of kv-head
  // h >> kv_shift.  The G q-heads of a kv-head then stream its K/V from the L2 / MALL in parallel
  // instead of one workgroup serving all of them (one stream, partials mode: DESIGN 4.16).
  int32_t kv_shift;
  unsigned long long* stamp;   // in-step launch stamps (common.hpp stamp_end), NULL in product launches
};

#ifndef TI_ATTN_RING
// K (and V) slots in flight per wave: 2 for the short per-split ranges of single-stream
// decode (deeper stalls on issue, tools/probe_attn.hip); 4 when a workgroup streams a long
// range for a GQA group (Llama-3-8B, 32 streams x 8192 keys: 236 -> 197 us per layer).
#define TI_ATTN_RING 2
#endif
#ifndef TI_ATTN_RING_M1
#define TI_ATTN_RING_M1 3   // one stream, one q-head per kv-head (tools/ab_attn_ring.sh)
#endif
#ifndef TI_ATTN_RING_HP
#define TI_ATTN_RING_HP 8   // keys in flight per wave in the head-parallel layout
#endif
#ifndef TI_ATTN_RING_LONG
#define TI_ATTN_RING_LONG 4
#endif
#ifndef TI_ATTN_EXP
#define TI_ATTN_EXP 0   // product build; tools/probe_attn.hip: +4 = per-workgroup phase timestamps
#endif
#if TI_ATTN_EXP & 4
static __device__ unsigned long long g_attn_ts[4096 * 8];
#define ATTN_TS(k)                                                                                        \
  do {                                                                                                    \
    if (threadIdx.x == 0)                                                                                 \
      g_attn_ts[(blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x * 8 + blockIdx.x * 8 + (k)] =            \
          __builtin_amdgcn_s_memrealtime();                                                               \
  } while (0)
#else
#define ATTN_TS(k) do { } while (0)
#endif
constexpr int kAttnWaves = 8;
constexpr int kAttnThreads = kAttnWaves * kWave;

__host__ __device__ inline int ws_row(int hd) { return hd + 4; }

__device__ __forceinline__ void unpack8(const u32x4 v, float (&f)[8]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    // copy the element out first: __builtin_bit_cast applied to an ext_vector element
    // expression reads element 0 (hipcc / ROCm 7.2), silently duplicating dims.
    const uint32_t w = v[i];
    const f16x2 h = __builtin_bit_cast(f16x2, w);
    f[2 * i] = (float)h[0];
    f[2 * i + 1] = (float)h[1];
  }
}

// Write-through (sc1) 16-byte buffer store / load for the split hand-off (aux bit 4 = sc1
// on gfx950); builtins, so the compiler counts them for its waitcnts.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t ws_rsrc(const float* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), 0, 0x7fffffff, 0x00020000);
}
constexpr int kAuxSc1 = 16;

// Largest split count whose partials (splits x G rows of hd + 4 floats) the merging
// workgroup can stage in its 48 KiB LDS buffer.
__host__ __device__ constexpr int attn_max_splits(int G, int HD) { return (48 * 1024) / (G * (HD + 4) * 4); }

// K/V rows are read once per step: non-temporal where that pays (TI_ATTN_NT).
#ifndef TI_ATTN_NT
#define TI_ATTN_NT 1
#endif
__device__ __forceinline__ u32x4 ld_kv(const u32x4* p) {
#if TI_ATTN_NT
  return __builtin_nontemporal_load(p);
#else
  return *p;
#endif
}

// Merge across the lane groups of a wave (lanes l, l ^ O, ... with O = LPK, 2 LPK, ... 32:
// the same dims of the other key rows), max and sum.
template <int O>
__device__ __forceinline__ float groups_max(float v) {
  if constexpr (O < 64) return groups_max<2 * O>(fmaxf(v, lane_xor<O>(v)));
  else return v;
}
template <int O>
__device__ __forceinline__ float groups_sum(float v) {
  if constexpr (O < 64) return groups_sum<2 * O>(v + lane_xor<O>(v));
  else return v;
}

// Slot order in the K/V ring: the slot's registers pass through an empty asm issued after the
// previous slot's softmax (tied to its running sum), so the scores of later slots cannot be
// hoisted to the top of the pass -- where they would wait for the loads issued last and drain the
// ring once per pass -- and each slot waits only for its own loads.
__device__ __forceinline__ void ring_pin(u32x4& k, u32x4& v, float& prev) {
  asm volatile("" : "+v"(k), "+v"(v), "+v"(prev));
}

template <int HD, int G, int R, bool HP, int NW = kAttnWaves, bool ROT = false>   // HP: head-parallel lanes (G >= 4, HD / (64 / G) == 8; see below)
__device__ __forceinline__ void attn_split_body(const AttnArgs& a, int split, int kvh, int m) {
  static_assert(!HP || (G >= 4 && HD / (64 / G) == 8), "head-parallel layout: 8 dims per lane");
  constexpr int LPK = HD / 8;       // lanes per key row
  constexpr int KPW = 64 / LPK;     // keys per slot (wave-load)
  __shared__ float s_m[NW][G], s_l[NW][G];
  __shared__ __attribute__((aligned(16))) float s_acc[NW][G][HD];
  __shared__ __attribute__((aligned(16))) float s_part[48 * 1024 / 4];   // merged rows, then all partials
  __shared__ int s_last;

  ATTN_TS(0);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int dl = lane % LPK, kg = lane / LPK;
  const int L = a.pos[m] + 1;
  // K/V of this workgroup's (stream, kv-head): [max_seq][HD] fp16 from wg_off
  const int64_t wg_off = (int64_t)m * a.stride + (int64_t)(kvh >> a.kv_shift) * a.max_seq * HD;
  auto ld_k = [&](int64_t elem) -> u32x4 { return ld_kv((const u32x4*)(a.kc + wg_off + elem)); };
  auto ld_v = [&](int64_t elem) -> u32x4 { return ld_kv((const u32x4*)(a.vc + wg_off + elem)); };
  auto ld_q4 = [&](size_t elem) -> float4 { return *(const float4*)(a.q + elem); };
  // fp16 output element idx
  auto store_out = [&](size_t idx, float val) {
    if (a.out_kt > 0) {   // packed: row m = idx / K, column idx % K
      const int K = a.heads * HD, m = (int)(idx / (size_t)K), k = (int)(idx - (size_t)m * K);
      idx = TI_PACKED_INDEX(m, k, a.out_kt);
    }
    a.out[idx] = f2h(val);
  };
  const int chunk = (L + a.splits - 1) / a.splits;
  const int s0 = split * chunk, s1 = min(L, s0 + chunk);
  const int nslot = s1 > s0 ? (s1 - s0 + KPW - 1) / KPW : 0;               // slots of the chunk
  const int total = wave < nslot ? (nslot - wave + NW - 1) / NW : 0;   // this wave's

  if constexpr (HP) {
    // head-parallel layout (G >= 4 q-heads per kv-head): lane l serves q-head l / LPH of the
    // group, dims 8 (l % LPH) .. +8, one key per wave step; every head's (max, sum, o) stays
    // in its own LPH lanes, so no lane-group merge is needed after the stream.
    constexpr int LPH = 64 / G;
    const int hg = lane / LPH, dh = lane % LPH;
    const int nkey = s1 > s0 ? s1 - s0 : 0;
    const int total = wave < nkey ? (nkey - wave + NW - 1) / NW : 0;   // this wave's keys
    int rj = 0;
    u32x4 kr[R], vr[R];
    auto refill = [&](int s) {
      const int key = min(s0 + wave + NW * (rj < total ? rj : max(total - 1, 0)), max(s1 - 1, 0));
      ++rj;
      kr[s] = ld_k((int64_t)key * HD + dh * 8);
      vr[s] = ld_v((int64_t)key * HD + dh * 8);
    };
    // q first, then the ring, all issued before any wait: the loop head then sees the ring's loads
    // youngest and in slot order, as its own back edge does, and waits for one slot at a time
    const size_t qe = (size_t)m * a.heads * HD + (size_t)(kvh * G + hg) * HD + dh * 8;
    const float4 q0 = ld_q4(qe), q1 = ld_q4(qe + 4);
#pragma unroll
    for (int s = 0; s < R; ++s) refill(s);
    float qh[8];
    qh[0] = q0.x * a.scale; qh[1] = q0.y * a.scale; qh[2] = q0.z * a.scale; qh[3] = q0.w * a.scale;
    qh[4] = q1.x * a.scale; qh[5] = q1.y * a.scale; qh[6] = q1.z * a.scale; qh[7] = q1.w * a.scale;
    float m1 = -INFINITY, l1 = 0.0f, acc1[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc1[e] = 0.0f;
    int ci = 0;
    auto consume = [&](const u32x4& kv, const u32x4& vv) {
      const bool valid = ci < total;
      ++ci;
      float kf[8], vf[8];
      unpack8(kv, kf);
      unpack8(vv, vf);
      float d = 0.0f;
#pragma unroll
      for (int e = 0; e < 8; ++e) d = fmaf(qh[e], kf[e], d);
      d = group_sum<LPH>(d);
      const float sc = valid ? d : -INFINITY;
      const float mn = fmaxf(m1, sc);
      const float alpha = m1 == mn ? 1.0f : __expf(m1 - mn);
      const float pr = valid ? __expf(sc - mn) : 0.0f;
      l1 = fmaf(l1, alpha, pr);
      m1 = mn;
#pragma unroll
      for (int e = 0; e < 8; ++e) acc1[e] = fmaf(pr, vf[e], acc1[e] * alpha);
    };
    int j0 = 0;
    for (; j0 + R <= total; j0 += R) {
#pragma unroll
      for (int s = 0; s < R; ++s) {
        ring_pin(kr[s], vr[s], l1);
        consume(kr[s], vr[s]);
        refill(s);
      }
    }
#pragma unroll
    for (int s = 0; s < R; ++s)
      if (j0 + s < total) consume(kr[s], vr[s]);
    ATTN_TS(1);
#pragma unroll
    for (int e = 0; e < 8; ++e) s_acc[wave][hg][dh * 8 + e] = acc1[e];
    if (dh == 0) {
      s_m[wave][hg] = m1;
      s_l[wave][hg] = l1;
    }
    __syncthreads();
  } else {
    // q first, then the K/V ring, all issued before any wait: the loop head then sees the ring's
    // loads youngest and in slot order, as its own back edge does, and waits for one slot at a time
    int rj = 0;
    // ROT: each workgroup starts its sweep at its own slot (wrapping), so the workgroups of a
    // launch do not walk their equally aligned K/V ranges in lockstep
    const int rot = ROT && nslot > 0 ? (int)(((unsigned)(m * a.kv_heads + kvh) * 61u) % (unsigned)nslot) : 0;
    auto slot_key = [&](int i) {
      int j = wave + NW * i;
      if constexpr (ROT) j = j + rot >= nslot ? j + rot - nslot : j + rot;
      return s0 + j * KPW + kg;
    };
    u32x4 kr[R], vr[R];
    auto refill = [&](int s) {
      const int key = min(slot_key(rj < total ? rj : max(total - 1, 0)), max(s1 - 1, 0));
      ++rj;
      kr[s] = ld_k((int64_t)key * HD + dl * 8);
      vr[s] = ld_v((int64_t)key * HD + dl * 8);
    };
    float4 qr[G][2];
  #pragma unroll
    for (int g = 0; g < G; ++g) {
      const size_t qe = (size_t)m * a.heads * HD + (size_t)(kvh * G + g) * HD + dl * 8;
      qr[g][0] = ld_q4(qe);
      qr[g][1] = ld_q4(qe + 4);
    }
  #pragma unroll
    for (int s = 0; s < R; ++s) refill(s);

    float q[G][8];
  #pragma unroll
    for (int g = 0; g < G; ++g) {
      const float4 q0 = qr[g][0], q1 = qr[g][1];
      q[g][0] = q0.x * a.scale; q[g][1] = q0.y * a.scale; q[g][2] = q0.z * a.scale; q[g][3] = q0.w * a.scale;
      q[g][4] = q1.x * a.scale; q[g][5] = q1.y * a.scale; q[g][6] = q1.z * a.scale; q[g][7] = q1.w * a.scale;
    }
    float mrun[G], lrun[G], acc[G][8];
  #pragma unroll
    for (int g = 0; g < G; ++g) {
      mrun[g] = -INFINITY;
      lrun[g] = 0.0f;
  #pragma unroll
      for (int e = 0; e < 8; ++e) acc[g][e] = 0.0f;
    }

    int ci = 0;   // compute cursor (slot index of this wave)
    auto consume = [&](const u32x4& kv, const u32x4& vv) {
      const bool valid = slot_key(ci) < s1;
      ++ci;
      float kf[8], vf[8];
      unpack8(kv, kf);
      unpack8(vv, vf);
  #pragma unroll
      for (int g = 0; g < G; ++g) {
        float d = 0.0f;
  #pragma unroll
        for (int e = 0; e < 8; ++e) d = fmaf(q[g][e], kf[e], d);
        d = group_sum<LPK>(d);
        const float sc = valid ? d : -INFINITY;
        const float mn = fmaxf(mrun[g], sc);
        const float alpha = mrun[g] == mn ? 1.0f : __expf(mrun[g] - mn);
        const float p = valid ? __expf(sc - mn) : 0.0f;
        lrun[g] = fmaf(lrun[g], alpha, p);
        mrun[g] = mn;
  #pragma unroll
        for (int e = 0; e < 8; ++e) acc[g][e] = fmaf(p, vf[e], acc[g][e] * alpha);
      }
    };
    int j0 = 0;
    for (; j0 + R <= total; j0 += R) {
  #pragma unroll
      for (int s = 0; s < R; ++s) {
        ring_pin(kr[s], vr[s], lrun[G - 1]);
        consume(kr[s], vr[s]);
        refill(s);
      }
    }
  #pragma unroll
    for (int s = 0; s < R; ++s)
      if (j0 + s < total) consume(kr[s], vr[s]);

    ATTN_TS(1);
    // merge the lane groups of the wave (each holds its own max / sum / o)
  #pragma unroll
    for (int g = 0; g < G; ++g) {
      const float mx = groups_max<LPK>(mrun[g]);
      const float f = mrun[g] == -INFINITY ? 0.0f : __expf(mrun[g] - mx);
      const float l = groups_sum<LPK>(lrun[g] * f);
  #pragma unroll
      for (int e = 0; e < 8; ++e) acc[g][e] = groups_sum<LPK>(acc[g][e] * f);
      mrun[g] = mx;
      lrun[g] = l;
    }
    if (lane < LPK) {
  #pragma unroll
      for (int g = 0; g < G; ++g)
  #pragma unroll
        for (int e = 0; e < 8; ++e) s_acc[wave][g][dl * 8 + e] = acc[g][e];
    }
    if (lane == 0) {
  #pragma unroll
      for (int g = 0; g < G; ++g) {
        s_m[wave][g] = mrun[g];
        s_l[wave][g] = lrun[g];
      }
    }
    __syncthreads();
  }

  // merge the waves; one thread per (q-head of the group, dim)
  const int row = ws_row(HD);
  for (int idx = tid; idx < G * HD; idx += (NW * kWave)) {
    const int g = idx / HD, d = idx - g * HD;
    float mx = s_m[0][g];
#pragma unroll
    for (int w = 1; w < NW; ++w) mx = fmaxf(mx, s_m[w][g]);
    float o = 0.0f, l = 0.0f;
    if (mx != -INFINITY) {
#pragma unroll
      for (int w = 0; w < NW; ++w) {
        const float f = s_m[w][g] == -INFINITY ? 0.0f : __expf(s_m[w][g] - mx);
        o = fmaf(f, s_acc[w][g][d], o);
        l = fmaf(f, s_l[w][g], l);
      }
    }
    const int h = kvh * G + g;
    if (a.splits == 1) {     // the whole sequence is ours: normalise and write out directly
      store_out((size_t)m * a.heads * HD + (size_t)h * HD + d, l > 0.0f ? o / l : 0.0f);
      continue;
    }
    if (a.part_o) {   // partials mode: this split's normalised row and (max, sum)
      const size_t r = ((size_t)m * a.heads + h) * a.splits + split;
      a.part_o[r * HD + d] = f2h(l > 0.0f ? o / l : 0.0f);
      if (d == 0) *(float2*)(a.part_ml + 2 * r) = make_float2(mx, l);
      continue;
    }
    s_part[g * row + d] = o;   // this split's row [o | max, sum, 0, 0]
    if (d == 0) {
      s_part[g * row + HD] = mx;
      s_part[g * row + HD + 1] = l;
      s_part[g * row + HD + 2] = 0.0f;
      s_part[g * row + HD + 3] = 0.0f;
    }
  }
  if (a.splits == 1 || a.part_o) return;
  __syncthreads();

  ATTN_TS(2);
  // ---- publish: the G rows of this split, write-through 16-byte stores.  Partials of
  // (stream, head) are contiguous: [m][h][split][row].
  constexpr int V4 = (HD + 4) / 4;
  const __amdgpu_buffer_rsrc_t wsr = ws_rsrc(a.ws);
  for (int i = tid; i < G * V4; i += (NW * kWave)) {
    const int g = i / V4, c = i - g * V4, h = kvh * G + g;
    const int off = (((m * a.heads + h) * a.splits + split) * row + 4 * c) * 4;
    __builtin_amdgcn_raw_buffer_store_b128(*(const f32x4*)(s_part + g * row + 4 * c), wsr, off, 0, kAuxSc1);
  }
  // ---- split merge by the last arriver: every storing wave drains its write-through
  // stores, barrier, one lane adds to the ticket; its returned value names the last.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int32_t* ticket = a.counters + (size_t)m * a.kv_heads + kvh;
  if (tid == 0) {
    const int t = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = (t == a.splits - 1);
  }
  __syncthreads();
  ATTN_TS(3);
  if (!s_last) return;
  // all partials of the group's heads in one round trip: s_part[g][split][row]
  const int nv = G * a.splits * V4;
  for (int i = tid; i < nv; i += (NW * kWave)) {
    const int g = i / (a.splits * V4), rem = i - g * a.splits * V4;
    const int h = kvh * G + g;
    const f32x4 v = __builtin_amdgcn_raw_buffer_load_b128(wsr, ((m * a.heads + h) * a.splits * row + 4 * rem) * 4, 0,
                                                          kAuxSc1);
    *(f32x4*)(s_part + (size_t)g * a.splits * row + 4 * rem) = v;
  }
  __syncthreads();
  for (int idx = tid; idx < G * HD; idx += (NW * kWave)) {
    const int g = idx / HD, d = idx - g * HD, h = kvh * G + g;
    const float* pb = s_part + (size_t)g * a.splits * row;
    float mx = -INFINITY;
    for (int sp = 0; sp < a.splits; ++sp) mx = fmaxf(mx, pb[sp * row + HD]);
    float num = 0.0f, den = 0.0f;
    for (int sp = 0; sp < a.splits; ++sp) {
      const float ms = pb[sp * row + HD];
      const float f = ms == -INFINITY ? 0.0f : __expf(ms - mx);   // empty split: weight 0
      den = fmaf(f, pb[sp * row + HD + 1], den);
      num = fmaf(f, pb[sp * row + d], num);
    }
    store_out((size_t)m * a.heads * HD + (size_t)h * HD + d, num / den);
  }
  if (tid == 0) __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
  ATTN_TS(4);
}

}  // namespace ti
