// attention.hip -- split-K single-query decode attention over the fp16 KV cache.
//
// Replaces TensorEngine::multi_head_attention (src/core/tensor_engine.cpp:1149-1252),
// whose decode call lands in attention_fast_incremental (:1254-1388): per head
// s_j = (q . k_j) / sqrt(hd), p = softmax(s), o = sum_j p_j v_j.  GQA maps q-head h to
// kv-head h / (heads / kv_heads) (the reference has no GQA; the oracle expands heads).
//
// Bandwidth-bound (2 * L * hd * 2 bytes of K/V per kv-head per stream): no MFMA.
//   grid (splits, kv_heads, M); a workgroup = 4 waves owns keys [s0, s1) of one
//   (stream, kv-head) and ALL q-heads of its group, so each K/V byte is read once.
//   hd/8 lanes hold one key row (8 fp16 = one dwordx4 each); a wave-load covers
//   64/(hd/8) keys; every wave keeps R = 4 K loads and 4 V loads in flight.
//   Per wave: online softmax (running max / sum, rescale by exp(m_old - m_new) once per
//   block); waves combined through LDS; the splits of a (stream, kv-head) are combined
//   in the same launch by whichever workgroup arrives last (agent-scope ticket).
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
};

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

template <int HD, int G>
__global__ __launch_bounds__(256) void attn_split_kernel(const AttnArgs a) {
  constexpr int LPK = HD / 8;       // lanes per key row
  constexpr int KPW = 64 / LPK;     // keys per wave-load
  constexpr int R = 4;              // wave-loads in flight per operand
  constexpr int KPB = 4 * KPW * R;  // keys per workgroup block
  __shared__ float s_m[4][G], s_l[4][G];
  __shared__ __attribute__((aligned(16))) float s_acc[4][G][HD];

  const int split = blockIdx.x, kvh = blockIdx.y, m = blockIdx.z;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int dl = lane % LPK, kg = lane / LPK;
  const int L = a.pos[m] + 1;
  const int chunk = (L + a.splits - 1) / a.splits;
  const int s0 = split * chunk, s1 = min(L, s0 + chunk);
  const uint16_t* kb = a.kc + (int64_t)m * a.stride + (int64_t)kvh * a.max_seq * HD + dl * 8;
  const uint16_t* vb = a.vc + (int64_t)m * a.stride + (int64_t)kvh * a.max_seq * HD + dl * 8;

  float q[G][8];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const float* qp = a.q + (size_t)m * a.heads * HD + (size_t)(kvh * G + g) * HD + dl * 8;
    const float4 q0 = *(const float4*)qp, q1 = *(const float4*)(qp + 4);
    q[g][0] = q0.x; q[g][1] = q0.y; q[g][2] = q0.z; q[g][3] = q0.w;
    q[g][4] = q1.x; q[g][5] = q1.y; q[g][6] = q1.z; q[g][7] = q1.w;
  }
  float mrun[G], lrun[G], acc[G][8];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    mrun[g] = -INFINITY;
    lrun[g] = 0.0f;
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[g][e] = 0.0f;
  }

  for (int blk = s0; blk < s1; blk += KPB) {
    u32x4 kr[R], vr[R];
    int jr[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      jr[r] = blk + (r * 4 + wave) * KPW + kg;
      const int jc = min(jr[r], s1 - 1);            // always a valid slot; masked below
      kr[r] = *(const u32x4*)(kb + (int64_t)jc * HD);
      vr[r] = *(const u32x4*)(vb + (int64_t)jc * HD);
    }
    float sc[G][R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      float kf[8];
      unpack8(kr[r], kf);
#pragma unroll
      for (int g = 0; g < G; ++g) {
        float d = 0.0f;
#pragma unroll
        for (int e = 0; e < 8; ++e) d = fmaf(q[g][e], kf[e], d);
        d = wave_sum_xor<LPK>(d);
        sc[g][r] = jr[r] < s1 ? d * a.scale : -INFINITY;
      }
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      float bm = sc[g][0];
#pragma unroll
      for (int r = 1; r < R; ++r) bm = fmaxf(bm, sc[g][r]);
#pragma unroll
      for (int o = LPK; o < 64; o <<= 1) bm = fmaxf(bm, __shfl_xor(bm, o, kWave));
      const float mn = fmaxf(mrun[g], bm);
      if (mn == -INFINITY) continue;                 // wave-uniform: nothing valid yet
      const float alpha = __expf(mrun[g] - mn);
      float p[R], ps = 0.0f;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        p[r] = __expf(sc[g][r] - mn);
        ps += p[r];
      }
#pragma unroll
      for (int o = LPK; o < 64; o <<= 1) ps += __shfl_xor(ps, o, kWave);
      lrun[g] = lrun[g] * alpha + ps;
      mrun[g] = mn;
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[g][e] *= alpha;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        float vf[8];
        unpack8(vr[r], vf);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[g][e] = fmaf(p[r], vf[e], acc[g][e]);
      }
    }
  }

  // sum the per-lane partials over the key groups of the wave
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int e = 0; e < 8; ++e)
#pragma unroll
      for (int o = LPK; o < 64; o <<= 1) acc[g][e] += __shfl_xor(acc[g][e], o, kWave);
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
  const int row = ws_row(HD);
  for (int idx = tid; idx < G * HD; idx += 256) {
    const int g = idx / HD, d = idx - g * HD;
    float mx = s_m[0][g];
#pragma unroll
    for (int w = 1; w < 4; ++w) mx = fmaxf(mx, s_m[w][g]);
    float o = 0.0f, l = 0.0f;
    if (mx != -INFINITY) {
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        if (s_m[w][g] == -INFINITY) continue;
        const float f = __expf(s_m[w][g] - mx);
        o = fmaf(f, s_acc[w][g][d], o);
        l = fmaf(f, s_l[w][g], l);
      }
    }
    const int h = kvh * G + g;
    if (a.splits == 1) {     // the whole sequence is ours: normalise and write out directly
      a.out[(size_t)m * a.heads * HD + (size_t)h * HD + d] = f2h(l > 0.0f ? o / l : 0.0f);
      continue;
    }
    float* dst = a.ws + ((size_t)(m * a.heads + h) * a.splits + split) * row;
    dst[d] = o;
    if (d == 0) {
      dst[HD] = mx;
      dst[HD + 1] = l;
    }
  }
  if (a.splits == 1) return;

  // ---- split combine, inside the launch: the last of the `splits` workgroups of this
  // (stream, kv-head) to arrive merges all partials.  Hand-off per MI355X_MICROARCH.md
  // "inter-workgroup visibility": every storing wave drains its stores, workgroup barrier,
  // one lane agent-release + relaxed ticket; the last arriver agent-acquires before reading.
  __shared__ int s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int32_t* ticket = a.counters + (size_t)m * a.kv_heads + kvh;
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int t = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = (t == a.splits - 1);
    if (s_last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  if (!s_last) return;
  for (int idx = tid; idx < G * HD; idx += 256) {
    const int g = idx / HD, d = idx - g * HD, h = kvh * G + g;
    const float* base = a.ws + (size_t)(m * a.heads + h) * a.splits * row;
    float mx = -INFINITY;
#pragma unroll 8
    for (int s = 0; s < a.splits; ++s) mx = fmaxf(mx, base[s * row + HD]);
    float num = 0.0f, den = 0.0f;
#pragma unroll 8
    for (int s = 0; s < a.splits; ++s) {
      const float ms = base[s * row + HD];
      const float f = ms == -INFINITY ? 0.0f : __expf(ms - mx);   // empty split: weight 0
      den = fmaf(f, base[s * row + HD + 1], den);
      num = fmaf(f, base[s * row + d], num);
    }
    a.out[(size_t)m * a.heads * HD + (size_t)h * HD + d] = f2h(num / den);
  }
  if (tid == 0) __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
}

template <int HD, int G>
static int launch_attn(const AttnArgs& a, hipStream_t s) {
  hipLaunchKernelGGL((attn_split_kernel<HD, G>), dim3(a.splits, a.kv_heads, a.M), dim3(256), 0, s, a);
  TI_LAUNCH_CHECK("attn_split_kernel");
  return TI_OK;
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

static size_t partial_bytes(int M, int heads, int head_dim, int splits) {
  return ((size_t)M * heads * splits * ti::ws_row(head_dim) * sizeof(float) + 255) & ~(size_t)255;
}

// partials [M][heads][splits][head_dim + 4] fp32, then the arrival tickets [M][heads] int32
// (sized for heads >= kv_heads); the tickets must be zero before the first call and are
// re-armed by every call.
extern "C" size_t ti_attn_workspace_bytes(int M, int heads, int head_dim, int splits) {
  return partial_bytes(M, heads, head_dim, splits) + (size_t)M * heads * sizeof(int32_t);
}

extern "C" int ti_attn_decode(const float* q, const uint16_t* k_cache, const uint16_t* v_cache,
                              int64_t kv_stream_stride, int max_seq, const int32_t* pos, int M, int heads,
                              int kv_heads, int head_dim, int splits, float* workspace, uint16_t* out,
                              ti_stream_t stream) {
  using namespace ti;
  if (!q || !k_cache || !v_cache || !pos || !workspace || !out)
    return ti_set_error(TI_ERR_ARG, "ti_attn_decode: null pointer");
  if (M < 1 || heads < 1 || kv_heads < 1 || heads % kv_heads || splits < 1 || max_seq < 1)
    return ti_set_error(TI_ERR_ARG, "ti_attn_decode: bad sizes M=%d heads=%d kv_heads=%d splits=%d", M, heads,
                        kv_heads, splits);
  if (head_dim != 64 && head_dim != 128)
    return ti_set_error(TI_ERR_UNSUPPORTED, "ti_attn_decode: head_dim %d not in {64,128}", head_dim);
  if (kv_stream_stride < (int64_t)kv_heads * max_seq * head_dim)
    return ti_set_error(TI_ERR_ARG, "ti_attn_decode: kv_stream_stride too small");
  AttnArgs a;
  a.q = q;
  a.kc = k_cache;
  a.vc = v_cache;
  a.pos = pos;
  a.ws = workspace;
  a.counters = (int32_t*)((char*)workspace + partial_bytes(M, heads, head_dim, splits));
  a.out = out;
  a.stride = kv_stream_stride;
  a.max_seq = max_seq;
  a.M = M;
  a.heads = heads;
  a.kv_heads = kv_heads;
  a.splits = splits;
  a.scale = 1.0f / sqrtf((float)head_dim);   // tensor_engine.cpp:1288 (hidden = head_dim per head)
  const int G = heads / kv_heads;
  hipStream_t s = (hipStream_t)stream;
  return head_dim == 128 ? dispatch_group<128>(a, G, s) : dispatch_group<64>(a, G, s);
}
