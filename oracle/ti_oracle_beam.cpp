// ti_oracle_beam.cpp -- TEST INFRASTRUCTURE ONLY.
//
// Restatement of InferenceEngine::beam_search_decode (src/model/inference_engine.cpp:1912-2069)
// and its helpers softmax / apply_top_k_filtering / apply_top_p_filtering (:1798-1910), with
// the forward pass supplied by the caller (a callback returning the distribution's logits for
// a token sequence).  The reference's ranking structures are used as it uses them: a
// std::priority_queue ordered by log_prob (:1924-1927), std::sort with its comparators on
// vectors built in the same order -- so equal probabilities / scores resolve exactly as in
// the reference (libstdc++ from GCC 11.4.0, the toolchain the reference is built with here).
//
// The callback decides which logits form "the distribution": the reference reads all
// seq_len x vocab logits of forward_pass as one (:1962-1966); the engine's parity test
// passes the last position's logits.  The oracle also reports the smallest decision gap
// (expansion cut, keep / drop cut) so a test can tell a robust comparison from a near-tie.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <limits>
#include <queue>
#include <utility>
#include <vector>

#include "ti_oracle.h"

namespace {

struct Cand {               // BeamCandidate (inference_engine.hpp:350-358)
  std::vector<int> tokens;
  float score = 0.0f;
  float log_prob = 0.0f;
  float normalized_score = 0.0f;
  bool finished = false;
};

std::vector<float> softmax(const std::vector<float>& lg) {                 // :1798-1818
  std::vector<float> p(lg.size());
  const float mx = *std::max_element(lg.begin(), lg.end());
  float sum = 0.0f;
  for (size_t i = 0; i < lg.size(); ++i) {
    p[i] = std::exp(lg[i] - mx);
    sum += p[i];
  }
  if (sum > 0.0f)
    for (auto& x : p) x /= sum;
  return p;
}

std::vector<float> top_k_filter(const std::vector<float>& probs, size_t k) {   // :1820-1856
  std::vector<float> f = probs;
  if (k >= probs.size()) return f;
  std::vector<std::pair<float, size_t>> pi;
  for (size_t i = 0; i < probs.size(); ++i) pi.emplace_back(probs[i], i);
  std::sort(pi.begin(), pi.end(), [](const auto& a, const auto& b) { return a.first > b.first; });
  for (size_t i = k; i < pi.size(); ++i) f[pi[i].second] = 0.0f;
  float sum = 0.0f;
  for (float x : f) sum += x;
  if (sum > 0.0f)
    for (auto& x : f) x /= sum;
  return f;
}

std::vector<float> top_p_filter(const std::vector<float>& probs, float p) {    // :1858-1910
  std::vector<float> f = probs;
  if (p >= 1.0f) return f;
  std::vector<std::pair<float, size_t>> pi;
  for (size_t i = 0; i < probs.size(); ++i) pi.emplace_back(probs[i], i);
  std::sort(pi.begin(), pi.end(), [](const auto& a, const auto& b) { return a.first > b.first; });
  float cum = 0.0f;
  std::vector<bool> in(probs.size(), false);
  for (const auto& pr : pi) {
    cum += pr.first;
    in[pr.second] = true;
    if (cum >= p) break;
  }
  for (size_t i = 0; i < probs.size(); ++i)
    if (!in[i]) f[i] = 0.0f;
  float sum = 0.0f;
  for (float x : f) sum += x;
  if (sum > 0.0f)
    for (auto& x : f) x /= sum;
  return f;
}

}  // namespace

extern "C" int or_beam_search(or_forward_fn fwd, void* ctx, const int32_t* prompt, size_t len, size_t max_new,
                              size_t beam_size, float temperature, size_t top_k, float top_p, float length_penalty,
                              int eos, int32_t* out_tokens, int32_t* out_ntok, float* out_log_prob, float* out_score,
                              int32_t* out_finished, float* min_gap) {
  if (beam_size == 0) return -1;
  auto cmp = [](const Cand& a, const Cand& b) { return a.log_prob < b.log_prob; };   // :1924-1927
  std::priority_queue<Cand, std::vector<Cand>, decltype(cmp)> beam(cmp);
  Cand init;
  init.tokens.assign(prompt, prompt + len);
  beam.push(init);
  std::vector<Cand> done;
  float gap = std::numeric_limits<float>::infinity();
  for (size_t step = 0; step < max_new; ++step) {                                 // :1937
    std::vector<Cand> cur;
    while (!beam.empty()) {
      cur.push_back(beam.top());
      beam.pop();
    }
    if (cur.empty()) break;
    std::vector<Cand> next;
    for (const auto& cand : cur) {
      if (cand.finished) {
        done.push_back(cand);
        continue;
      }
      const float* lgp = nullptr;
      const size_t V = fwd(ctx, cand.tokens.data(), cand.tokens.size(), &lgp);   // forward_pass (:1961)
      if (V == 0 || !lgp) return -2;
      std::vector<float> lg(lgp, lgp + V);
      if (temperature != 1.0f)
        for (auto& x : lg) x /= temperature;
      std::vector<float> probs = softmax(lg);
      if (top_k > 0 && top_k < probs.size()) probs = top_k_filter(probs, top_k);
      if (top_p < 1.0f) probs = top_p_filter(probs, top_p);
      std::vector<std::pair<float, int>> pt;
      for (size_t i = 0; i < probs.size(); ++i)
        if (probs[i] > 0.0f) pt.emplace_back(probs[i], static_cast<int>(i));
      std::sort(pt.begin(), pt.end(), [](const auto& a, const auto& b) { return a.first > b.first; });
      const size_t ex = std::min(beam_size, pt.size());
      if (ex < pt.size()) gap = std::min(gap, std::log(pt[ex - 1].first) - std::log(pt[ex].first));
      for (size_t i = 0; i < ex; ++i) {
        const float prob = pt[i].first;
        const int token = pt[i].second;
        if (prob <= 0.0f) continue;
        Cand nc = cand;
        nc.tokens.push_back(token);
        nc.log_prob += std::log(prob);
        nc.finished = token == eos || nc.tokens.size() >= len + max_new;
        next.push_back(nc);
      }
    }
    for (auto& c : next) c.normalized_score = c.log_prob / std::pow(static_cast<float>(c.tokens.size()), length_penalty);
    std::sort(next.begin(), next.end(), [](const auto& a, const auto& b) { return a.normalized_score > b.normalized_score; });
    const size_t keep = std::min(beam_size, next.size());
    if (keep < next.size()) gap = std::min(gap, next[keep - 1].normalized_score - next[keep].normalized_score);
    for (size_t i = 0; i < keep; ++i) {
      if (next[i].finished) done.push_back(next[i]);
      else beam.push(next[i]);
    }
    if (done.size() >= beam_size) break;
  }
  while (!beam.empty()) {                                                         // :2052-2057
    Cand c = beam.top();
    beam.pop();
    c.finished = true;
    done.push_back(c);
  }
  std::sort(done.begin(), done.end(), [](const auto& a, const auto& b) { return a.normalized_score > b.normalized_score; });
  const size_t n = std::min(beam_size, done.size());
  for (size_t r = 0; r < n; ++r) {
    const Cand& c = done[r];
    const size_t nt = c.tokens.size() > len ? c.tokens.size() - len : 0;
    out_ntok[r] = static_cast<int32_t>(nt);
    for (size_t t = 0; t < max_new; ++t) out_tokens[r * max_new + t] = t < nt ? c.tokens[len + t] : -1;
    out_log_prob[r] = c.log_prob;
    out_score[r] = c.normalized_score;
    out_finished[r] = c.finished ? 1 : 0;
  }
  if (min_gap) *min_gap = gap;
  return static_cast<int>(n);
}
