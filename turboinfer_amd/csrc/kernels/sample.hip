// sample.hip -- on-device token sampler.
//
// InferenceEngine::sample_next_token (src/model/inference_engine.cpp:1554-1673) for one
// stream per workgroup, with the uniform draw supplied by the caller:
//   * temperature: logit /= T unless T == 1 or T <= 0                        (:1577-1582)
//   * top-k: the k largest logits survive, the rest become -inf           (:1584-1599)
//   * softmax with exp(l - max), summed in index order, divided by the sum (:1601-1614)
//   * top-p: probabilities in descending order, cut where the running sum first reaches p,
//     the rest zeroed, renormalised in index order                        (:1616-1649)
//   * the draw: first index (ascending) whose running sum reaches u; else the last index
//                                                                           (:1651-1672)
// Only the k <= TI_SAMPLE_MAX_K survivors carry probability, so after the selection every
// step runs on a list of them kept in index order: the sums see the same fp32 values in the
// same order as the reference's loops over all V entries (the others add exact zeros).
// Selection: the k-th largest of the 1024 threads' run maxima bounds the k-th largest logit
// from below; the few keys above that bound are ranked exactly in LDS (a 4-pass 8-bit radix
// select over the whole row, LDS histograms, when there are more than 2048 of them); the
// survivors (ties lowest index first) are compacted in index order with block scans.  (A
// radix pass over the row costs ~14 us: one bin takes most keys, so the LDS atomics
// serialise.)  k above 1024 goes to the radix select directly, and the per-survivor steps
// stride over the survivors; above TI_SAMPLE_MAX_K (any k up to V) the survivor arrays live in a
// per-row HBM workspace instead of LDS (sample_kernel<true>).  Differences to the reference: exp / log are the device's (<= 1 ulp from
// glibc), and equal logits at the k-th place / equal probabilities at the top-p cut are taken
// lowest index first (libstdc++'s std::sort leaves their order unspecified).
#include <math.h>

#include "common.hpp"

namespace ti {

constexpr int kSampThreads = 1024;
constexpr int kSampWaves = kSampThreads / kWave;

struct SampArgs {
  const float* logits;
  int32_t ldl, V, top_k;
  float temperature, top_p;
  const float* draws;          // [M][draw_stride]
  int32_t draw_stride;
  int32_t advance;             // with step_ctr / n_in: draw index t = (*step_ctr - advance) - (n_in[m] - 1)
  const int32_t* step_ctr;     // nullable: t = 0
  const int32_t* n_in;
  unsigned long long* argmax;  // [M][TI_ARGMAX_SLOTS], nullable: slot 0 gets the token's feedback key
  int32_t* tokens;             // [M], nullable
  float* logprobs;             // [M][lp_stride], nullable
  int32_t lp_stride;
  char* ws;                    // top_k > TI_SAMPLE_MAX_K: per-row survivor arrays in HBM (ws_bytes each)
  size_t ws_bytes;
};

// Survivor arrays of one row when they do not fit in LDS (top_k > TI_SAMPLE_MAX_K, up to V):
// val f32[V], idx i32[V], p f32[V], sorted f32[V], rank i32[V] (each 16-byte aligned: the
// sequential sums read float4s), then the top-p sort keys u64[P]
// (P = the power of two >= V, at least 64).  Read and written by the row's one workgroup only
// (its barriers order them).
__host__ __device__ inline int samp_pow2(int n) {
  int P = 64;
  while (P < n) P <<= 1;
  return P;
}
__host__ __device__ inline size_t samp_ws_array(int V) { return ((size_t)V * 4 + 15) & ~(size_t)15; }   // 16-B aligned
__host__ __device__ inline size_t samp_ws_row_bytes(int V) { return 5 * samp_ws_array(V) + (size_t)samp_pow2(V) * 8; }

__device__ __forceinline__ uint32_t samp_key(float v) {
  const uint32_t u = __builtin_bit_cast(uint32_t, v);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// exclusive prefix sum over the block (1024 threads); also returns the total
__device__ int block_excl_scan(int v, int* total, int* s_w) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) s_w[w] = x;
  __syncthreads();
  if (threadIdx.x < 64) {   // the wave totals, scanned by wave 0
    const int t = lane < kSampWaves ? s_w[lane] : 0;
    int y = t;
#pragma unroll
    for (int o = 1; o < kSampWaves; o <<= 1) {
      const int z = __shfl_up(y, o, 64);
      if (lane >= o) y += z;
    }
    if (lane < kSampWaves) s_w[lane] = y - t;
    if (lane == kSampWaves - 1) s_w[kSampWaves] = y;
  }
  __syncthreads();
  const int r = s_w[w] + x - v;
  *total = s_w[kSampWaves];
  __syncthreads();   // s_w reused by the next scan
  return r;
}

// BIG: top_k above TI_SAMPLE_MAX_K -- the survivor arrays live in the row's HBM workspace
// (the same steps on them; the sequential sums read them from global memory).
template <bool BIG>
__global__ __launch_bounds__(kSampThreads) void sample_kernel(const SampArgs a) {
  constexpr int LK = BIG ? 1 : TI_SAMPLE_MAX_K;   // LDS survivor capacity
  __shared__ uint32_t hist[256];
  __shared__ int s_w[kSampWaves + 1];
  __shared__ uint32_t s_prefix;
  __shared__ int s_left, s_tok;
  __shared__ float s_lp;
  __shared__ float l_val[LK];
  __shared__ __attribute__((aligned(16))) float l_p[LK], l_sorted[LK];
  __shared__ int s_cut;
  __shared__ int l_idx[LK];
  __shared__ int l_rank[LK];
  __shared__ unsigned long long l_key[LK];   // top-p sort keys
  __shared__ float s_mx[kSampWaves];
  constexpr int kCand = BIG ? 1 : 2048;
  __shared__ uint32_t s_ck[kCand];
  __shared__ int s_ci[kCand];
  __shared__ uint8_t s_cf[kCand];
  const int m = blockIdx.x, tid = threadIdx.x, V = a.V, k = a.top_k;
  const int CAP = BIG ? V : TI_SAMPLE_MAX_K;
  float *s_val = l_val, *s_p = l_p, *s_sorted = l_sorted;
  int *s_idx = l_idx, *s_rank = l_rank;
  unsigned long long* s_key = l_key;
  if constexpr (BIG) {
    char* w = a.ws + (size_t)m * a.ws_bytes;
    const size_t A = samp_ws_array(V);
    s_val = (float*)w;
    s_idx = (int*)(w + A);
    s_p = (float*)(w + 2 * A);
    s_sorted = (float*)(w + 3 * A);
    s_rank = (int*)(w + 4 * A);
    s_key = (unsigned long long*)(w + 5 * A);
  }
  const float* row = a.logits + (size_t)m * a.ldl;
  const bool temp = a.temperature != 1.0f && a.temperature > 0.0f;
  auto lg = [&](int i) { return temp ? row[i] / a.temperature : row[i]; };

  int t = 0;   // which draw (and logprob slot) this step's token is
  if (a.step_ctr) t = (*a.step_ctr - a.advance) - (a.n_in ? a.n_in[m] - 1 : 0);
  if (t < 0 || t >= a.draw_stride) return;   // a prompt step (its token is the prompt's) or past the budget
  const float u = a.draws[(size_t)m * a.draw_stride + t];

  // ---- k-th largest of per-thread keys: 8 bits per pass, most significant first; each pass
  // histograms the keys of `sweep_fn` that match the prefix so far (LDS atomics)
  auto select_kth = [&](auto&& sweep_fn, int kk, uint32_t* kth_out, int* need_eq_out) {
    if (tid == 0) {
      s_prefix = 0u;
      s_left = kk;
    }
    uint32_t mask = 0u;
    for (int shift = 24; shift >= 0; shift -= 8) {
      if (tid < 256) hist[tid] = 0u;
      __syncthreads();
      const uint32_t pre = s_prefix;
      sweep_fn([&](uint32_t key) {
        if ((key & mask) == pre) atomicAdd(&hist[(key >> shift) & 255u], 1u);
      });
      __syncthreads();
      // the bin holding the s_left-th largest key: counts above each bin by one block scan
      // over the bins in descending order (thread j <-> bin 255 - j)
      const int h = tid < 256 ? (int)hist[255 - tid] : 0, left = s_left;
      int tot_h;
      const int above = block_excl_scan(h, &tot_h, s_w);
      if (tid < 256 && h > 0 && above < left && left <= above + h) {
        s_prefix = pre | ((uint32_t)(255 - tid) << shift);
        s_left = left - above;
      }
      mask |= 255u << shift;
      __syncthreads();
    }
    *kth_out = s_prefix;
    *need_eq_out = s_left;
  };
  // wave wv owns the index segment [g0, g1), read 64 consecutive indices per wave load
  // (coalesced), 8 loads in flight per lane; f(i, key, ok) sees every wave-load slot in index
  // order with a wave-uniform trip count (ok = i inside the segment), so ballots can order it
  const int wv = tid >> 6, lane = tid & 63;
  const int SEG = (((V + kSampWaves - 1) / kSampWaves) + 63) & ~63;
  const int g0 = min(V, wv * SEG), g1 = min(V, g0 + SEG);
  // Rows up to kCacheV keep the lane's 32 keys in registers after the first sweep (one CU
  // streams the row at ~25 GB/s: each sweep from memory costs ~5 us at V = 32000).
  constexpr int kCacheV = kSampWaves * 64 * 32;
  const bool cached = V <= kCacheV;
  uint32_t rk[32];
  bool loaded = false;
  auto own = [&](auto&& f) {
    if (cached) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int b = g0 + c * 64 * 8;
        if (!loaded) {
          float v[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int i = b + 64 * j + lane;
            v[j] = i < g1 ? row[i] : 0.0f;
          }
#pragma unroll
          for (int j = 0; j < 8; ++j) rk[c * 8 + j] = samp_key(temp ? v[j] / a.temperature : v[j]);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int i = b + 64 * j + lane;
          f(i, rk[c * 8 + j], i < g1);
        }
      }
      loaded = true;
      return;
    }
    for (int b = g0; b < g1; b += 64 * 8) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = b + 64 * j + lane;
        v[j] = i < g1 ? row[i] : 0.0f;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = b + 64 * j + lane;
        f(i, samp_key(temp ? v[j] / a.temperature : v[j]), i < g1);
      }
    }
  };
  auto below = [&](unsigned long long mask) {   // set bits of mask in lanes below this one
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
  };
  // the wave's starting offset in a block-ordered compaction of per-thread counts
  auto wave_base = [&](int cnt, int* total) { return __shfl(block_excl_scan(cnt, total, s_w), 0, 64); };

  // ---- candidates: every key at or above tau0, the k-th largest of the threads' maxima
  // (k elements reach it; for smooth logits a few dozen more).  The k largest candidates,
  // ties lowest index first, are the survivors; with more than kCand candidates the full
  // row goes through the radix select instead.
  // (k above the thread count: no k-th maximum to bound with, straight to the radix select)
  int tot = kCand + 1, cbase = 0;
  uint32_t tau0 = 0u;
  if (!BIG && k <= kSampThreads) {
    uint32_t tmax = 0u;   // below every finite key
    own([&](int, uint32_t key, bool ok) { tmax = ok && key > tmax ? key : tmax; });
    int unused;
    select_kth([&](auto&& f) { f(tmax); }, k, &tau0, &unused);
    int ncand = 0;
    own([&](int, uint32_t key, bool ok) { ncand += ok && key >= tau0; });
    cbase = wave_base(ncand, &tot);
  }
  const int C_tot = tot;
  int n;
  if (!BIG && C_tot <= kCand) {
    int run = cbase;
    own([&](int i, uint32_t key, bool ok) {
      const bool c = ok && key >= tau0;
      const unsigned long long m = __ballot(c);
      if (c) {
        s_ck[run + below(m)] = key;
        s_ci[run + below(m)] = i;
      }
      run += __popcll(m);
    });
    __syncthreads();
    // rank among the candidates (they are in index order): survivors have rank < k
    for (int i = tid; i < C_tot; i += kSampThreads) {
      const uint32_t ki = s_ck[i];
      int r = 0;
      for (int j = 0; j < C_tot; ++j) r += s_ck[j] > ki || (s_ck[j] == ki && j < i);
      s_cf[i] = r < k;
    }
    __syncthreads();
    // survivors in index order: thread tid compacts candidates [q0, q1)
    const int Q = (C_tot + kSampThreads - 1) / kSampThreads, q0 = min(C_tot, tid * Q), q1 = min(C_tot, q0 + Q);
    int nk = 0;
    for (int i = q0; i < q1; ++i) nk += s_cf[i];
    int at = block_excl_scan(nk, &tot, s_w);
    for (int i = q0; i < q1; ++i)
      if (s_cf[i] && at < TI_SAMPLE_MAX_K) {
        const int idx = s_ci[i];
        s_val[at] = lg(idx);
        s_idx[at] = idx;
        ++at;
      }
    __syncthreads();
    n = min(tot, TI_SAMPLE_MAX_K);
  } else {
    uint32_t kth;
    int need_eq;
    select_kth(
        [&](auto&& f) {
          constexpr int U = 16;   // the whole row, strided, 16 loads in flight per thread
          for (int b = tid; b < V; b += U * kSampThreads) {
            float v[U];
#pragma unroll
            for (int j = 0; j < U; ++j) v[j] = b + j * kSampThreads < V ? row[b + j * kSampThreads] : 0.0f;
#pragma unroll
            for (int j = 0; j < U; ++j)
              if (b + j * kSampThreads < V) f(samp_key(temp ? v[j] / a.temperature : v[j]));
          }
        },
        k, &kth, &need_eq);
    // survivors in index order: keys above the k-th, and the lowest-index ties at it
    int ng = 0, ne = 0;
    own([&](int, uint32_t key, bool ok) {
      ng += ok && key > kth;
      ne += ok && key == kth;
    });
    int tot_e;
    const int eq_base = wave_base(ne, &tot_e);                 // equal keys before this wave
    const int ne_w = __reduce_add_sync(~0ull, ne);             // this wave's equal keys
    const int keep_eq_w = max(0, min(ne_w, need_eq - eq_base));
    const int ng_w = __reduce_add_sync(~0ull, ng);
    const int kbase = wave_base(lane == 0 ? ng_w + keep_eq_w : 0, &tot);
    int run = kbase, eq_run = eq_base;
    own([&](int i, uint32_t key, bool ok) {
      const bool eq = ok && key == kth;
      const unsigned long long me = __ballot(eq);
      const bool keep = (ok && key > kth) || (eq && eq_run + below(me) < need_eq);
      const unsigned long long mk = __ballot(keep);
      if (keep && run + below(mk) < CAP) {
        s_val[run + below(mk)] = temp ? row[i] / a.temperature : row[i];
        s_idx[run + below(mk)] = i;
      }
      run += __popcll(mk);
      eq_run += __popcll(me);
    });
    __syncthreads();
    n = min(tot, CAP);   // == k
  }

  // ---- softmax over the survivors (the others are exp(-inf) = 0 in the reference's loops)
  float mx = -INFINITY;   // exact in any order
  for (int i = tid; i < n; i += kSampThreads) mx = fmaxf(mx, s_val[i]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  if (lane == 0) s_mx[wv] = mx;
  __syncthreads();
#pragma unroll
  for (int w = 0; w < kSampWaves; ++w) mx = fmaxf(mx, s_mx[w]);
  for (int i = tid; i < n; i += kSampThreads) s_p[i] = expf(s_val[i] - mx);
  __syncthreads();
  // The sequential sums run in one thread (the reference's order), 16 values per step with
  // the next 16 already in flight (the adds are one dependent chain; the LDS latency hides
  // behind it).
  auto seq_scan = [&](const float* p, float target, bool find, float* sum_out) {
    float cum = 0.0f;
    int i = 0;
    if (n >= 16) {
      float4 c[4], nx[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) c[j] = *(const float4*)(p + 4 * j);
      for (;; i += 16) {
        const bool more = i + 32 <= n;
        if (more) {
#pragma unroll
          for (int j = 0; j < 4; ++j) nx[j] = *(const float4*)(p + i + 16 + 4 * j);
        }
        const float v[16] = {c[0].x, c[0].y, c[0].z, c[0].w, c[1].x, c[1].y, c[1].z, c[1].w,
                             c[2].x, c[2].y, c[2].z, c[2].w, c[3].x, c[3].y, c[3].z, c[3].w};
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          cum += v[j];
          if (find && target <= cum) return i + j;
        }
        if (!more) {
          i += 16;
          break;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) c[j] = nx[j];
      }
    }
    for (; i < n; ++i) {
      cum += p[i];
      if (find && target <= cum) return i;
    }
    *sum_out = cum;
    return -1;
  };
  auto seq_sum = [&](const float* p) {
    float sum;
    seq_scan(p, 0.0f, false, &sum);
    return sum;
  };
  // first r (in order) whose running sum reaches `target` (cmp: sum >= target / target <= sum), or -1
  auto seq_find = [&](const float* p, float target) {
    float sum;
    return seq_scan(p, target, true, &sum);
  };
  if (tid == 0) s_lp = seq_sum(s_p);
  __syncthreads();
  for (int i = tid; i < n; i += kSampThreads) s_p[i] = s_p[i] / s_lp;
  __syncthreads();

  // ---- top-p: rank by probability (descending, lower index first on ties), cut, renormalise.
  // Rank order = ascending (~bits(p), survivor position) for p >= 0: a bitonic sort of those
  // 64-bit keys in LDS, padded to a power of two with all-ones keys.
  if (a.top_p < 1.0f) {
    int P = 64;
    while (P < n) P <<= 1;
    for (int i = tid; i < P; i += kSampThreads)
      s_key[i] = i < n ? ((unsigned long long)~__float_as_uint(s_p[i]) << 32) | (uint32_t)i : ~0ull;
    __syncthreads();
    for (int size = 2; size <= P; size <<= 1)
      for (int stride = size >> 1; stride > 0; stride >>= 1) {
        for (int i = tid; i < P / 2; i += kSampThreads) {
          const int lo = 2 * stride * (i / stride) + (i % stride), hi = lo + stride;
          const unsigned long long x = s_key[lo], y = s_key[hi];
          if ((x > y) == ((lo & size) == 0)) {
            s_key[lo] = y;
            s_key[hi] = x;
          }
        }
        __syncthreads();
      }
    for (int r = tid; r < n; r += kSampThreads) {
      const unsigned long long key = s_key[r];
      s_sorted[r] = __uint_as_float(~(uint32_t)(key >> 32));
      s_rank[(uint32_t)key] = r;
    }
    __syncthreads();
    if (tid == 0) {
      const int r = seq_find(s_sorted, a.top_p);
      s_cut = r < 0 ? n : r + 1;
    }
    __syncthreads();
    for (int i = tid; i < n; i += kSampThreads)
      if (s_rank[i] >= s_cut) s_p[i] = 0.0f;
    __syncthreads();
    if (tid == 0) s_lp = seq_sum(s_p);
    __syncthreads();
    if (s_lp > 0.0f)
      for (int i = tid; i < n; i += kSampThreads) s_p[i] = s_p[i] / s_lp;
    __syncthreads();
  }

  // ---- the draw: running sum in index order
  if (tid == 0) {
    int tok = V - 1;
    float pt = s_idx[n - 1] == V - 1 ? s_p[n - 1] : 0.0f;
    if (u <= 0.0f) {   // the reference returns index 0 at its first comparison
      tok = 0;
      pt = s_idx[0] == 0 ? s_p[0] : 0.0f;
    } else {
      const int i = seq_find(s_p, u);
      if (i >= 0) {
        tok = s_idx[i];
        pt = s_p[i];
      }
    }
    s_tok = tok;
    s_lp = logf(pt);
  }
  __syncthreads();
  if (tid == 0) {
    const int tok = s_tok;
    if (a.tokens) a.tokens[m] = tok;
    if (a.logprobs) a.logprobs[(size_t)m * a.lp_stride + t] = s_lp;
    // feedback like the greedy argmax: a key above every logit key (high word all ones)
    if (a.argmax) a.argmax[(size_t)m * TI_ARGMAX_SLOTS] = (0xFFFFFFFFull << 32) | (unsigned long long)(0xFFFFFFFFu - (uint32_t)tok);
  }
}

}  // namespace ti

extern "C" size_t ti_sample_workspace_bytes(int V, int top_k) {
  return V >= 1 && top_k > TI_SAMPLE_MAX_K ? ti::samp_ws_row_bytes(V) : 0;
}

static int sample_launch(ti::SampArgs a, int M, ti_stream_t stream) {
  if (!a.logits || !a.draws || M < 1 || a.V < 1 || a.ldl < a.V || a.draw_stride < 1)
    return ti_set_error(TI_ERR_ARG, "ti_sample: bad arguments");
  if (a.top_k < 1 || a.top_k > a.V)
    return ti_set_error(TI_ERR_ARG, "ti_sample: top_k %d not in [1, V = %d]", a.top_k, a.V);
  if (a.top_k > TI_SAMPLE_MAX_K) {
    if (!a.ws)
      return ti_set_error(TI_ERR_ARG, "ti_sample: top_k %d > %d needs a workspace (ti_sample_workspace_bytes)", a.top_k,
                          TI_SAMPLE_MAX_K);
    a.ws_bytes = ti::samp_ws_row_bytes(a.V);
    hipLaunchKernelGGL(ti::sample_kernel<true>, dim3(M), dim3(ti::kSampThreads), 0, (hipStream_t)stream, a);
  } else {
    hipLaunchKernelGGL(ti::sample_kernel<false>, dim3(M), dim3(ti::kSampThreads), 0, (hipStream_t)stream, a);
  }
  TI_LAUNCH_CHECK("sample_kernel");
  ti_stamp_next(ti::STAMP_OTHER, 0);   // (unstamped; keeps the stamped step's launch list whole)
  return TI_OK;
}

extern "C" int ti_sample_device_ws(const float* logits, int ldl, int M, int V, float temperature, int top_k,
                                   float top_p, const float* draws, int32_t* tokens, float* logprobs, void* ws,
                                   ti_stream_t stream) {
  ti::SampArgs a{};
  a.ws = (char*)ws;
  a.logits = logits;
  a.ldl = ldl;
  a.V = V;
  a.top_k = top_k;
  a.temperature = temperature;
  a.top_p = top_p;
  a.draws = draws;
  a.draw_stride = 1;
  a.tokens = tokens;
  a.logprobs = logprobs;
  a.lp_stride = 1;
  if (!tokens) return ti_set_error(TI_ERR_ARG, "ti_sample_device: tokens required");
  return sample_launch(a, M, stream);
}

extern "C" int ti_sample_device(const float* logits, int ldl, int M, int V, float temperature, int top_k, float top_p,
                                const float* draws, int32_t* tokens, float* logprobs, ti_stream_t stream) {
  return ti_sample_device_ws(logits, ldl, M, V, temperature, top_k, top_p, draws, tokens, logprobs, nullptr, stream);
}

extern "C" int ti_sample_step_ws(const float* logits, int ldl, int M, int V, float temperature, int top_k,
                                 float top_p, const float* draws, int draw_stride, const int32_t* step_ctr, int advance,
                                 const int32_t* n_in, unsigned long long* argmax, float* logprobs, void* ws,
                                 ti_stream_t stream) {
  ti::SampArgs a{};
  a.ws = (char*)ws;
  a.logits = logits;
  a.ldl = ldl;
  a.V = V;
  a.top_k = top_k;
  a.temperature = temperature;
  a.top_p = top_p;
  a.draws = draws;
  a.draw_stride = draw_stride;
  a.step_ctr = step_ctr;
  a.advance = advance;
  a.n_in = n_in;
  a.argmax = argmax;
  a.logprobs = logprobs;
  a.lp_stride = draw_stride;
  if (!step_ctr || !argmax) return ti_set_error(TI_ERR_ARG, "ti_sample_step: step_ctr and argmax required");
  return sample_launch(a, M, stream);
}

extern "C" int ti_sample_step(const float* logits, int ldl, int M, int V, float temperature, int top_k, float top_p,
                              const float* draws, int draw_stride, const int32_t* step_ctr, int advance,
                              const int32_t* n_in, unsigned long long* argmax, float* logprobs, ti_stream_t stream) {
  return ti_sample_step_ws(logits, ldl, M, V, temperature, top_k, top_p, draws, draw_stride, step_ctr, advance, n_in,
                           argmax, logprobs, nullptr, stream);
}
