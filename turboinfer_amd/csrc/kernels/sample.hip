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
// Selection: a 4-pass 8-bit radix select of the k-th largest order key over the row (LDS
// histograms), then the survivors (keys above it, and the lowest-index ties at it) compacted
// with block scans.  Differences to the reference: exp / log are the device's (<= 1 ulp from
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
};

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
  if (threadIdx.x == 0) {
    int run = 0;
    for (int i = 0; i < kSampWaves; ++i) {
      const int t = s_w[i];
      s_w[i] = run;
      run += t;
    }
    s_w[kSampWaves] = run;
  }
  __syncthreads();
  const int r = s_w[w] + x - v;
  *total = s_w[kSampWaves];
  __syncthreads();   // s_w reused by the next scan
  return r;
}

__global__ __launch_bounds__(kSampThreads) void sample_kernel(const SampArgs a) {
  __shared__ uint32_t hist[256];
  __shared__ int s_w[kSampWaves + 1];
  __shared__ uint32_t s_prefix;
  __shared__ int s_left, s_tok;
  __shared__ float s_lp;
  __shared__ float s_val[TI_SAMPLE_MAX_K], s_p[TI_SAMPLE_MAX_K];
  __shared__ int s_idx[TI_SAMPLE_MAX_K], s_order[TI_SAMPLE_MAX_K];
  const int m = blockIdx.x, tid = threadIdx.x, V = a.V, k = a.top_k;
  const float* row = a.logits + (size_t)m * a.ldl;
  const bool temp = a.temperature != 1.0f && a.temperature > 0.0f;
  auto lg = [&](int i) { return temp ? row[i] / a.temperature : row[i]; };
  // f(i, key) over the row, 16 loads in flight per thread (the passes are latency-bound)
  auto sweep = [&](auto&& f) {
    constexpr int U = 16;
    for (int b = tid; b < V; b += U * kSampThreads) {
      float v[U];
#pragma unroll
      for (int j = 0; j < U; ++j) v[j] = b + j * kSampThreads < V ? row[b + j * kSampThreads] : 0.0f;
#pragma unroll
      for (int j = 0; j < U; ++j)
        if (b + j * kSampThreads < V) f(samp_key(temp ? v[j] / a.temperature : v[j]));
    }
  };

  int t = 0;   // which draw (and logprob slot) this step's token is
  if (a.step_ctr) t = (*a.step_ctr - a.advance) - (a.n_in ? a.n_in[m] - 1 : 0);
  if (t < 0 || t >= a.draw_stride) return;   // a prompt step (its token is the prompt's) or past the budget
  const float u = a.draws[(size_t)m * a.draw_stride + t];

  // ---- k-th largest order key: 8 bits per pass, most significant first
  if (tid == 0) {
    s_prefix = 0u;
    s_left = k;
  }
  uint32_t mask = 0u;
  for (int shift = 24; shift >= 0; shift -= 8) {
    if (tid < 256) hist[tid] = 0u;
    __syncthreads();
    const uint32_t pre = s_prefix;
    sweep([&](uint32_t key) {
      if ((key & mask) == pre) atomicAdd(&hist[(key >> shift) & 255u], 1u);
    });
    __syncthreads();
    // the bin holding the s_left-th largest key: counts above each bin by one block scan over
    // the bins in descending order (thread j <-> bin 255 - j)
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
  const uint32_t kth = s_prefix;
  const int need_eq = s_left;   // keys equal to the k-th that survive (lowest indices first)

  // ---- survivors in index order: thread tid owns indices [c0, c1)
  const int C = (V + kSampThreads - 1) / kSampThreads, c0 = min(V, tid * C), c1 = min(V, c0 + C);
  int ng = 0, ne = 0;
  for (int i0 = c0; i0 < c1; i0 += 16) {   // the thread's own contiguous run, 16 loads in flight
    float v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = i0 + j < c1 ? row[i0 + j] : 0.0f;
#pragma unroll
    for (int j = 0; j < 16; ++j)
      if (i0 + j < c1) {
        const uint32_t key = samp_key(temp ? v[j] / a.temperature : v[j]);
        ng += key > kth;
        ne += key == kth;
      }
  }
  int tot;
  const int eq_before = block_excl_scan(ne, &tot, s_w);
  const int keep_eq = max(0, min(ne, need_eq - eq_before));
  const int at = block_excl_scan(ng + keep_eq, &tot, s_w);
  int w = at, eq_seen = 0;
  for (int i = c0; i < c1; ++i) {
    const float v = lg(i);
    const uint32_t key = samp_key(v);
    const bool keep = key > kth || (key == kth && eq_seen++ < keep_eq);
    if (keep && w < TI_SAMPLE_MAX_K) {
      s_val[w] = v;
      s_idx[w] = i;
      ++w;
    }
  }
  __syncthreads();
  const int n = min(tot, TI_SAMPLE_MAX_K);   // == k

  // ---- softmax over the survivors (the others are exp(-inf) = 0 in the reference's loops)
  float mx = -INFINITY;
  for (int i = 0; i < n; ++i) mx = fmaxf(mx, s_val[i]);   // every thread, exact in any order
  if (tid < n) s_p[tid] = expf(s_val[tid] - mx);
  __syncthreads();
  if (tid == 0) {
    float sum = 0.0f;
    for (int i = 0; i < n; ++i) sum += s_p[i];
    s_lp = sum;
  }
  __syncthreads();
  if (tid < n) s_p[tid] = s_p[tid] / s_lp;
  __syncthreads();

  // ---- top-p: rank by probability (descending, lower index first on ties), cut, renormalise
  if (a.top_p < 1.0f) {
    if (tid < n) {
      const float p = s_p[tid];
      int r = 0;
      for (int j = 0; j < n; ++j) r += s_p[j] > p || (s_p[j] == p && j < tid);
      s_order[r] = tid;
    }
    __syncthreads();
    if (tid == 0) {
      float cum = 0.0f;
      int cut = n;
      for (int r = 0; r < n; ++r) {
        cum += s_p[s_order[r]];
        if (cum >= a.top_p) {
          cut = r + 1;
          break;
        }
      }
      for (int r = cut; r < n; ++r) s_p[s_order[r]] = 0.0f;
      float ns = 0.0f;
      for (int i = 0; i < n; ++i) ns += s_p[i];
      s_lp = ns;
    }
    __syncthreads();
    if (tid < n && s_lp > 0.0f) s_p[tid] = s_p[tid] / s_lp;
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
      float cum = 0.0f;
      for (int i = 0; i < n; ++i) {
        cum += s_p[i];
        if (u <= cum) {
          tok = s_idx[i];
          pt = s_p[i];
          break;
        }
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

static int sample_launch(const ti::SampArgs& a, int M, ti_stream_t stream) {
  if (!a.logits || !a.draws || M < 1 || a.V < 1 || a.ldl < a.V || a.draw_stride < 1)
    return ti_set_error(TI_ERR_ARG, "ti_sample: bad arguments");
  if (a.top_k < 1 || a.top_k > TI_SAMPLE_MAX_K || a.top_k > a.V)
    return ti_set_error(TI_ERR_UNSUPPORTED, "ti_sample: top_k %d not in [1, min(V, %d)]", a.top_k, TI_SAMPLE_MAX_K);
  hipLaunchKernelGGL(ti::sample_kernel, dim3(M), dim3(ti::kSampThreads), 0, (hipStream_t)stream, a);
  TI_LAUNCH_CHECK("sample_kernel");
  return TI_OK;
}

extern "C" int ti_sample_device(const float* logits, int ldl, int M, int V, float temperature, int top_k, float top_p,
                                const float* draws, int32_t* tokens, float* logprobs, ti_stream_t stream) {
  ti::SampArgs a{};
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

extern "C" int ti_sample_step(const float* logits, int ldl, int M, int V, float temperature, int top_k, float top_p,
                              const float* draws, int draw_stride, const int32_t* step_ctr, int advance,
                              const int32_t* n_in, unsigned long long* argmax, float* logprobs, ti_stream_t stream) {
  ti::SampArgs a{};
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
