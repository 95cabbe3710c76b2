// sampling.cpp -- host-side helpers of the decode engine that must follow the reference's
// host arithmetic exactly: the RoPE (cos, sin) table and the token sampler.
#include <algorithm>
#include <cmath>
#include <limits>
#include <utility>
#include <vector>

#include "ti_engine.h"
#include "ti_hip.h"

int ti_set_error(int code, const char* fmt, ...);

extern "C" int ti_rope_table(const float* pos, int npos, int head_dim, float theta, float* out) {
  if (!pos || !out || npos < 1 || head_dim < 2 || (head_dim & 1))
    return ti_set_error(TI_ERR_ARG, "ti_rope_table: bad arguments");
  // TensorEngine::apply_rope (src/core/tensor_engine.cpp:1561-1566, 1595-1597):
  // freq_i = 1 / pow(theta, 2i / d); angle = pos * freq_i; (cos, sin) in fp32 via libm.
  const int half = head_dim / 2;
  std::vector<float> freq((size_t)half);
  for (int i = 0; i < half; ++i) freq[i] = 1.0f / std::pow(theta, (float)(2 * i) / (float)head_dim);
  for (int p = 0; p < npos; ++p)
    for (int i = 0; i < half; ++i) {
      const float ang = pos[p] * freq[i];
      out[((size_t)p * half + i) * 2] = std::cos(ang);
      out[((size_t)p * half + i) * 2 + 1] = std::sin(ang);
    }
  return TI_OK;
}

// InferenceEngine::sample_next_token (src/model/inference_engine.cpp:1554-1673) with the
// uniform draw u passed in (the engine owns the mt19937).  Equal logits are ordered by
// libstdc++'s std::sort exactly as in the reference, which decides ties under top-k.
extern "C" int ti_sample_token(const float* logits_in, int V, float temperature, int top_k, float top_p, float u,
                               int* token, float* logprob) {
  if (!logits_in || !token || V < 1) return ti_set_error(TI_ERR_ARG, "ti_sample_token: bad arguments");
  const size_t n = (size_t)V;
  std::vector<float> lg(logits_in, logits_in + n);
  if (temperature != 1.0f && temperature > 0.0f)
    for (float& l : lg) l /= temperature;
  if (top_k > 0 && (size_t)top_k < n) {
    std::vector<std::pair<float, int>> pr;
    pr.reserve(n);
    for (size_t i = 0; i < n; ++i) pr.emplace_back(lg[i], (int)i);
    std::sort(pr.begin(), pr.end(), [](const auto& a, const auto& b) { return a.first > b.first; });
    for (size_t i = (size_t)top_k; i < n; ++i) lg[pr[i].second] = -std::numeric_limits<float>::infinity();
  }
  const float mx = *std::max_element(lg.begin(), lg.end());
  std::vector<float> p(n);
  float sum = 0.0f;
  for (size_t i = 0; i < n; ++i) {
    p[i] = std::exp(lg[i] - mx);
    sum += p[i];
  }
  for (float& x : p) x /= sum;
  if (top_p < 1.0f) {
    std::vector<std::pair<float, int>> pr;
    pr.reserve(n);
    for (size_t i = 0; i < n; ++i) pr.emplace_back(p[i], (int)i);
    std::sort(pr.begin(), pr.end(), [](const auto& a, const auto& b) { return a.first > b.first; });
    float cum = 0.0f;
    size_t cut = n;
    for (size_t i = 0; i < n; ++i) {
      cum += pr[i].first;
      if (cum >= top_p) {
        cut = i + 1;
        break;
      }
    }
    for (size_t i = cut; i < n; ++i) p[pr[i].second] = 0.0f;
    float ns = 0.0f;
    for (float x : p) ns += x;
    if (ns > 0.0f)
      for (float& x : p) x /= ns;
  }
  float cum = 0.0f;
  for (size_t i = 0; i < n; ++i) {
    cum += p[i];
    if (u <= cum) {
      *token = (int)i;
      if (logprob) *logprob = std::log(p[i]);
      return TI_OK;
    }
  }
  *token = V - 1;
  if (logprob) *logprob = std::log(p[n - 1]);
  return TI_OK;
}
