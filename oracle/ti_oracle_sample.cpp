// ti_oracle_sample.cpp -- TEST INFRASTRUCTURE ONLY.
//
// Restatement of InferenceEngine::sample_next_token (src/model/inference_engine.cpp:1554-1673)
// with the uniform draw supplied by the caller instead of the clock-seeded mt19937
// (:470-473, :1651-1652).  The top-k and top-p stages rank (value, index) pairs with
// std::sort and the reference comparator `a.first > b.first` (:1591-1592, :1621-1622);
// the ORDER OF EQUAL LOGITS is therefore whatever libstdc++'s introsort produces
// (third-party dependency: libstdc++ from GCC 11.4.0, Ubuntu 22.04, the toolchain the
// reference is built with here) -- so this file calls the same std::sort rather than
// restating its internals.  Ties are real on the reference's plumbing model, whose
// lm_head repeats every 500 columns (benchmark_inference.cpp:214-219).
#include <algorithm>
#include <cmath>
#include <limits>
#include <utility>
#include <vector>

#include "ti_oracle.h"

// The distribution sample_next_token draws from (everything before :1651), into probs[V].
extern "C" void or_sample_probs(const float* logits_in, size_t V, float temperature, size_t top_k, float top_p,
                                float* probs_out) {
  std::vector<float> logits(logits_in, logits_in + V);
  if (temperature != 1.0f && temperature > 0.0f)                       // :1594-1599
    for (float& l : logits) l /= temperature;
  if (top_k > 0 && top_k < V) {                                        // :1602-1616
    std::vector<std::pair<float, int>> pairs;
    for (size_t i = 0; i < V; ++i) pairs.emplace_back(logits[i], static_cast<int>(i));
    std::sort(pairs.begin(), pairs.end(), [](const auto& a, const auto& b) { return a.first > b.first; });
    for (size_t i = top_k; i < V; ++i) logits[pairs[i].second] = -std::numeric_limits<float>::infinity();
  }
  const float mx = *std::max_element(logits.begin(), logits.end());   // :1619-1630
  std::vector<float> probs(V);
  float sum = 0.0f;
  for (size_t i = 0; i < V; ++i) {
    probs[i] = std::exp(logits[i] - mx);
    sum += probs[i];
  }
  for (float& p : probs) p /= sum;
  if (top_p < 1.0f) {                                                  // :1633-1664
    std::vector<std::pair<float, int>> pairs;
    for (size_t i = 0; i < V; ++i) pairs.emplace_back(probs[i], static_cast<int>(i));
    std::sort(pairs.begin(), pairs.end(), [](const auto& a, const auto& b) { return a.first > b.first; });
    float cum = 0.0f;
    size_t cutoff = V;
    for (size_t i = 0; i < V; ++i) {
      cum += pairs[i].first;
      if (cum >= top_p) { cutoff = i + 1; break; }
    }
    for (size_t i = cutoff; i < V; ++i) probs[pairs[i].second] = 0.0f;
    float ns = 0.0f;
    for (float p : probs) ns += p;
    if (ns > 0.0f)
      for (float& p : probs) p /= ns;
  }
  std::copy(probs.begin(), probs.end(), probs_out);
}

extern "C" int or_sample_token(const float* logits_in, size_t V, float temperature, size_t top_k,
                               float top_p, float u, float* logprob_out) {
  std::vector<float> probs(V);
  or_sample_probs(logits_in, V, temperature, top_k, top_p, probs.data());
  float cum = 0.0f;                                                    // :1654-1672
  for (size_t i = 0; i < V; ++i) {
    cum += probs[i];
    if (u <= cum) {
      if (logprob_out) *logprob_out = std::log(probs[i]);
      return static_cast<int>(i);
    }
  }
  if (logprob_out) *logprob_out = std::log(probs[V - 1]);
  return static_cast<int>(V - 1);
}
