// ref_shim.cpp -- TEST INFRASTRUCTURE ONLY.
//
// extern "C" wrappers over the UNMODIFIED reference library (compiled from
// /root/reference/src by oracle/Makefile into oracle/_ref/).  Used to generate the
// golden vectors in tests/golden/ and as the "reference" CPU baseline in bench.py.
// Nothing here is part of the product and nothing here re-implements reference
// arithmetic: every call lands in the reference's own TensorEngine / Quantizer /
// InferenceEngine.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <fstream>
#include <cstdint>
#include <cstring>
#include <exception>
#include <string>
#include <vector>

#include "turboinfer/core/tensor_engine.hpp"
#include "turboinfer/model/inference_engine.hpp"
#include "turboinfer/model/model_loader.hpp"
#include "turboinfer/optimize/quantization.hpp"

using turboinfer::core::ComputeDevice;
using turboinfer::core::DataType;
using turboinfer::core::Tensor;
using turboinfer::core::TensorEngine;
using turboinfer::core::TensorShape;

namespace {
thread_local std::string g_err;

TensorEngine& engine() {
  static TensorEngine e(ComputeDevice::kCPU);
  return e;
}

Tensor make(const float* p, int ndim, const uint64_t* dims) {
  std::vector<size_t> d(dims, dims + ndim);
  return Tensor(TensorShape(d), p, DataType::kFloat32);
}

int out(const Tensor& t, float* dst) {
  std::memcpy(dst, t.data(), t.byte_size());
  return static_cast<int>(t.shape().total_size());
}

template <class F>
int guard(F&& f) {
  try {
    return f();
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
}
}  // namespace

// ModelData -> <out>.meta (text) + <out>.data (the tensors' raw bytes in the .meta order):
// the dump tests/test_gguf.py compares between this library, the reference and the oracle.
static void dump_model_data(const turboinfer::model::ModelData& md, const std::string& out) {
  const auto& m = md.metadata();
  std::ofstream meta(out + ".meta"), data(out + ".data", std::ios::binary);
  char rope[32];
  std::snprintf(rope, sizeof rope, "%.9g", (double)m.rope_theta);
  meta << m.name << "\n" << m.architecture << "\n" << m.version << "\n" << m.vocab_size << " " << m.hidden_size << " "
       << m.num_layers << " " << m.num_heads << " " << m.intermediate_size << " " << rope << "\n";
  std::vector<std::string> keys;
  for (const auto& kv : m.extra_params) keys.push_back(kv.first);
  std::sort(keys.begin(), keys.end());
  meta << keys.size() << "\n";
  for (const auto& k : keys) meta << k << "\t" << m.extra_params.at(k) << "\n";
  const auto names = md.tensor_names();
  meta << names.size() << "\n";
  for (const auto& n : names) {
    const auto* t = md.get_tensor(n);
    const bool h = t->dtype() == turboinfer::core::DataType::kFloat16;
    meta << n << " " << (h ? 3 : 0) << " " << t->shape().ndim();
    for (size_t d : t->shape().dimensions()) meta << " " << d;
    meta << "\n";
    if (t->byte_size()) data.write((const char*)t->data(), (std::streamsize)t->byte_size());
  }
}

extern "C" {

const char* ref_last_error() { return g_err.c_str(); }

int ref_matmul(const float* a, int an, const uint64_t* ad, const float* b, int bn,
               const uint64_t* bd, float* y) {
  return guard([&] { return out(engine().matmul(make(a, an, ad), make(b, bn, bd)), y); });
}

int ref_rms_norm(const float* x, int xn, const uint64_t* xd, const float* w, uint64_t n, float eps,
                 float* y) {
  return guard([&] {
    const uint64_t wd[1] = {n};
    return out(engine().rms_norm(make(x, xn, xd), make(w, 1, wd), eps), y);
  });
}

int ref_apply_rope(const float* x, int xn, const uint64_t* xd, const float* pos, int pn,
                   const uint64_t* pd, float theta, float* y) {
  return guard([&] { return out(engine().apply_rope(make(x, xn, xd), make(pos, pn, pd), theta), y); });
}

int ref_silu(const float* x, uint64_t n, float* y) {
  return guard([&] { const uint64_t d[1] = {n}; return out(engine().silu(make(x, 1, d)), y); });
}

int ref_relu(const float* x, uint64_t n, float* y) {
  return guard([&] { const uint64_t d[1] = {n}; return out(engine().relu(make(x, 1, d)), y); });
}

int ref_add(const float* a, const float* b, uint64_t n, float* y) {
  return guard([&] {
    const uint64_t d[1] = {n};
    return out(engine().add(make(a, 1, d), make(b, 1, d)), y);
  });
}

int ref_multiply(const float* a, const float* b, uint64_t n, float* y) {
  return guard([&] {
    const uint64_t d[1] = {n};
    return out(engine().multiply(make(a, 1, d), make(b, 1, d)), y);
  });
}

int ref_softmax(const float* x, uint64_t rows, uint64_t n, float temperature, float* y) {
  return guard([&] {
    const uint64_t d[2] = {rows, n};
    return out(engine().softmax(make(x, 2, d), temperature), y);
  });
}

int ref_attention_fast_incremental(const float* q, const float* k, const float* v, uint64_t B,
                                   uint64_t S, uint64_t D, float* y) {
  return guard([&] {
    const uint64_t qd[3] = {B, 1, D}, kd[3] = {B, S, D};
    return out(engine().attention_fast_incremental(make(q, 3, qd), make(k, 3, kd), make(v, 3, kd)), y);
  });
}

int ref_multi_head_attention(const float* q, const float* k, const float* v, uint64_t B, uint64_t S,
                             uint64_t H, uint64_t heads, float* y) {
  return guard([&] {
    const uint64_t qd[3] = {B, 1, H}, kd[3] = {B, S, H};
    return out(engine().multi_head_attention(make(q, 3, qd), make(k, 3, kd), make(v, 3, kd), heads), y);
  });
}

// TensorEngine::attention (heads 0) / multi_head_attention (heads > 0) with query length Sq
// and an optional float mask [B][Sq][Sk] (tensor_engine.cpp:1045-1147, 1149-1252).
int ref_attention_general(const float* q, const float* k, const float* v, const float* mask, uint64_t B,
                          uint64_t Sq, uint64_t Sk, uint64_t H, uint64_t heads, float* y) {
  return guard([&] {
    const uint64_t qd[3] = {B, Sq, H}, kd[3] = {B, Sk, H}, md[3] = {B, Sq, Sk};
    const uint64_t one[3] = {1, 1, 1};
    const float zero = 0.0f;
    Tensor m = mask ? make(mask, 3, md) : make(&zero, 3, one);
    const Tensor* mp = mask ? &m : nullptr;
    if (heads == 0) return out(engine().attention(make(q, 3, qd), make(k, 3, kd), make(v, 3, kd), mp), y);
    return out(engine().multi_head_attention(make(q, 3, qd), make(k, 3, kd), make(v, 3, kd), heads, mp), y);
  });
}

// Quantizer: bits 8 / 4, symmetric 0 / 1.  Writes q as int32 (int8 widened), scale, zp.
int ref_quantize(const float* x, uint64_t n, int bits, int symmetric, int32_t* q, float* scale,
                 float* zp) {
  return guard([&] {
    using namespace turboinfer::optimize;
    QuantizationConfig cfg;
    cfg.type = bits == 8 ? QuantizationType::kInt8 : QuantizationType::kInt4;
    cfg.symmetric = symmetric != 0;
    Quantizer qz(cfg);
    const uint64_t d[1] = {n};
    Tensor t = make(x, 1, d);
    QuantizationInfo info = qz.calculate_quantization_info(t);
    Tensor qt = qz.quantize_tensor(t);
    if (bits == 8) {
      const int8_t* p = static_cast<const int8_t*>(qt.data());
      for (uint64_t i = 0; i < n; ++i) q[i] = p[i];
    } else {
      std::memcpy(q, qt.data(), n * sizeof(int32_t));
    }
    *scale = info.scales[0];
    *zp = info.zero_points[0];
    return static_cast<int>(n);
  });
}

int ref_dequantize(const int32_t* q, uint64_t n, int bits, float scale, float zp, float* y) {
  return guard([&] {
    using namespace turboinfer::optimize;
    QuantizationInfo info{};
    info.type = bits == 8 ? QuantizationType::kInt8 : QuantizationType::kInt4;
    info.scales = {scale};
    info.zero_points = {zp};
    if (bits == 8) {
      std::vector<int8_t> b(n);
      for (uint64_t i = 0; i < n; ++i) b[i] = static_cast<int8_t>(q[i]);
      dequantize_from_int8(b.data(), y, n, info);
    } else {
      dequantize_from_int4(q, y, n, info);
    }
    return static_cast<int>(n);
  });
}

// InferenceEngine::generate on the benchmark's synthetic model
// (benchmarks/benchmark_inference.cpp:145-225 fill patterns), greedy (top_k = 1).
namespace {
// benchmark_inference.cpp:145-225 create_test_model fill patterns (data, not algorithm).
turboinfer::model::ModelData plumbing_model(uint64_t vocab, uint64_t hidden, uint64_t layers) {
    using namespace turboinfer::model;
    ModelMetadata md{};
    md.name = "synthetic_test_model";
    md.architecture = "llama";
    md.vocab_size = vocab;
    md.hidden_size = hidden;
    md.num_layers = layers;
    md.num_heads = hidden / 64;
    md.intermediate_size = hidden * 4;
    md.rope_theta = 10000.0f;
    ModelData data;
    data.metadata() = md;
    {
      Tensor e(TensorShape({vocab, hidden}), DataType::kFloat32);
      float* p = e.data_ptr<float>();
      for (uint64_t i = 0; i < vocab * hidden; ++i)
        p[i] = (static_cast<float>(i % 1000) / 1000.0f - 0.5f) * 0.1f;
      data.add_tensor("token_embeddings.weight", std::move(e));
    }
    for (uint64_t l = 0; l < layers; ++l) {
      const std::string pfx = "layers." + std::to_string(l) + ".";
      Tensor q(TensorShape({hidden, hidden})), k(TensorShape({hidden, hidden})),
          v(TensorShape({hidden, hidden}));
      for (uint64_t i = 0; i < hidden * hidden; ++i) {
        q.data_ptr<float>()[i] = (static_cast<float>(i % 100) / 100.0f - 0.5f) * 0.05f;
        k.data_ptr<float>()[i] = (static_cast<float>((i + 1) % 100) / 100.0f - 0.5f) * 0.05f;
        v.data_ptr<float>()[i] = (static_cast<float>((i + 2) % 100) / 100.0f - 0.5f) * 0.05f;
      }
      data.add_tensor(pfx + "attention.q_proj.weight", std::move(q));
      data.add_tensor(pfx + "attention.k_proj.weight", std::move(k));
      data.add_tensor(pfx + "attention.v_proj.weight", std::move(v));
      Tensor up(TensorShape({hidden, 4 * hidden})), down(TensorShape({4 * hidden, hidden}));
      for (uint64_t i = 0; i < hidden * 4 * hidden; ++i) {
        up.data_ptr<float>()[i] = (static_cast<float>(i % 200) / 200.0f - 0.5f) * 0.02f;
        down.data_ptr<float>()[i] = (static_cast<float>(i % 200) / 200.0f - 0.5f) * 0.02f;
      }
      data.add_tensor(pfx + "mlp.up_proj.weight", std::move(up));
      data.add_tensor(pfx + "mlp.down_proj.weight", std::move(down));
    }
    {
      Tensor lm(TensorShape({hidden, vocab}));
      for (uint64_t i = 0; i < hidden * vocab; ++i)
        lm.data_ptr<float>()[i] = (static_cast<float>(i % 500) / 500.0f - 0.5f) * 0.01f;
      data.add_tensor("lm_head.weight", std::move(lm));
    }
    return data;
}
}  // namespace

int ref_plumbing_generate(uint64_t vocab, uint64_t hidden, uint64_t layers, const int32_t* prompt,
                          uint64_t n_prompt, uint64_t max_new, int32_t* tokens_out,
                          uint64_t* n_out) {
  return guard([&] {
    using namespace turboinfer::model;
    ModelData data = plumbing_model(vocab, hidden, layers);
    InferenceConfig cfg;
    cfg.top_k = 1;
    cfg.temperature = 1.0f;
    cfg.device = ComputeDevice::kCPU;
    InferenceEngine eng(data, cfg);
    std::vector<int> p(prompt, prompt + n_prompt);
    GenerationResult r = eng.generate(p, max_new, false);
    for (size_t i = 0; i < r.tokens.size(); ++i) tokens_out[i] = r.tokens[i];
    *n_out = r.tokens.size();
    return static_cast<int>(r.tokens.size());
  });
}

// The reference's generate() contract on the plumbing model, greedy, with a chosen
// config.eos_token_id and max_sequence_length: tokens, stop_reason (0 eos_token, 1 max_length,
// 2 max_new_tokens), finished, and its total_time_ms / tokens_per_second (inference_engine.cpp:734-802).
int ref_plumbing_generate_cfg(uint64_t vocab, uint64_t hidden, uint64_t layers, const int32_t* prompt,
                              uint64_t n_prompt, uint64_t max_new, int32_t eos_token_id, uint64_t max_len,
                              int32_t* tokens_out, uint64_t* n_out, int32_t* stop_out, float* time_ms_out,
                              float* tps_out) {
  return guard([&] {
    using namespace turboinfer::model;
    ModelData data = plumbing_model(vocab, hidden, layers);
    InferenceConfig cfg;
    cfg.top_k = 1;
    cfg.temperature = 1.0f;
    cfg.eos_token_id = eos_token_id;
    cfg.max_sequence_length = max_len;
    cfg.device = ComputeDevice::kCPU;
    InferenceEngine eng(data, cfg);
    std::vector<int> p(prompt, prompt + n_prompt);
    GenerationResult r = eng.generate(p, max_new, false);
    for (size_t i = 0; i < r.tokens.size(); ++i) tokens_out[i] = r.tokens[i];
    *n_out = r.tokens.size();
    *stop_out = r.stop_reason == "eos_token" ? 0 : r.stop_reason == "max_length" ? 1 : r.stop_reason == "max_new_tokens" ? 2 : -1;
    *time_ms_out = r.total_time_ms;
    *tps_out = r.tokens_per_second;
    return r.finished ? 1 : 0;
  });
}

// The reference's generate() with a sampling configuration and include_logprobs = true on the
// plumbing model: every step runs the reference's own sample_next_token
// (inference_engine.cpp:1554-1673) with its clock-seeded mt19937 draw (:470-473), and the
// GenerationResult carries std::log(probs[token]) of each sampled token.  The draw is not
// observable; the (token, log-prob) pairs pin temperature, top-k (with tied logits: the
// plumbing lm_head repeats every 500 columns), softmax and top-p renormalisation.
int ref_plumbing_generate_sampled(uint64_t vocab, uint64_t hidden, uint64_t layers, const int32_t* prompt,
                                  uint64_t n_prompt, uint64_t max_new, float temperature, uint64_t top_k,
                                  float top_p, int32_t* tokens_out, float* logprobs_out, uint64_t* n_out) {
  return guard([&] {
    using namespace turboinfer::model;
    ModelData data = plumbing_model(vocab, hidden, layers);
    InferenceConfig cfg;
    cfg.top_k = top_k;
    cfg.top_p = top_p;
    cfg.temperature = temperature;
    cfg.device = ComputeDevice::kCPU;
    InferenceEngine eng(data, cfg);
    std::vector<int> p(prompt, prompt + n_prompt);
    GenerationResult r = eng.generate(p, max_new, true);
    for (size_t i = 0; i < r.tokens.size(); ++i) tokens_out[i] = r.tokens[i];
    for (size_t i = 0; i < r.logprobs.size(); ++i) logprobs_out[i] = r.logprobs[i];
    *n_out = r.tokens.size();
    return static_cast<int>(r.logprobs.size());
  });
}

// The reference's generate_beam_search (inference_engine.cpp:830-871 over beam_search_decode
// :1912-2069) on the plumbing model: deterministic (no draws).  Per result r: its new tokens
// (out_tokens[r * max_new ..], -1 padded, count in out_ntok[r]), finished flag, and the
// per-token log-prob the result carries (candidate.log_prob / n_new, :862-865).
int ref_plumbing_beam_search(uint64_t vocab, uint64_t hidden, uint64_t layers, const int32_t* prompt,
                             uint64_t n_prompt, uint64_t max_new, uint64_t beam_size, float temperature,
                             uint64_t top_k, float top_p, float length_penalty, int32_t* out_tokens, int32_t* out_ntok,
                             int32_t* out_finished, float* out_logprob, uint64_t* n_out) {
  return guard([&] {
    using namespace turboinfer::model;
    ModelData data = plumbing_model(vocab, hidden, layers);
    InferenceConfig cfg;
    cfg.top_k = top_k;
    cfg.top_p = top_p;
    cfg.temperature = temperature;
    cfg.length_penalty = length_penalty;
    cfg.device = ComputeDevice::kCPU;
    InferenceEngine eng(data, cfg);
    std::vector<int> p(prompt, prompt + n_prompt);
    std::vector<GenerationResult> rs = eng.generate_beam_search(p, max_new, beam_size, true);
    for (size_t r = 0; r < rs.size(); ++r) {
      out_ntok[r] = static_cast<int32_t>(rs[r].tokens.size());
      for (size_t t = 0; t < max_new; ++t) out_tokens[r * max_new + t] = t < rs[r].tokens.size() ? rs[r].tokens[t] : -1;
      out_finished[r] = rs[r].finished ? 1 : 0;
      out_logprob[r] = rs[r].logprobs.empty() ? 0.0f : rs[r].logprobs[0];
    }
    *n_out = rs.size();
    return static_cast<int>(rs.size());
  });
}

// Times the reference-composed decode layer (SURVEY 8(c) O2 composition, all calls
// into the reference TensorEngine) at a given shape: n_layers passes of one layer,
// plus one lm_head matmul.  weight_kind: 0 fp32, 1 int32-stored INT4 (what
// Quantizer::quantize_model hands the engine, quantization.cpp:45-46), 2 int8.
// Inputs are filled with a cheap LCG; only time is reported.
int ref_time_decode(uint64_t H, uint64_t heads, uint64_t I, uint64_t V, uint64_t L, int weight_kind,
                    int n_layers, double* layer_seconds, double* head_seconds) {
  return guard([&] {
    uint32_t st = 12345u;
    auto rnd = [&]() { st = st * 1664525u + 1013904223u; return (float)((st >> 8) & 0xffff) / 65536.0f - 0.5f; };
    auto weight = [&](uint64_t K, uint64_t N) {
      DataType dt = weight_kind == 0 ? DataType::kFloat32 : (weight_kind == 1 ? DataType::kInt32 : DataType::kInt8);
      Tensor t(TensorShape({K, N}), dt);
      for (uint64_t i = 0; i < K * N; ++i) {
        if (weight_kind == 0) t.data_ptr<float>()[i] = rnd() * 0.05f;
        else if (weight_kind == 1) t.data_ptr<int32_t>()[i] = (int32_t)(rnd() * 14.0f);
        else t.data_ptr<int8_t>()[i] = (int8_t)(rnd() * 254.0f);
      }
      return t;
    };
    auto vec = [&](std::initializer_list<size_t> d) {
      Tensor t{TensorShape(d)};
      for (size_t i = 0; i < t.shape().total_size(); ++i) t.data_ptr<float>()[i] = rnd();
      return t;
    };
    TensorEngine& e = engine();
    Tensor wq = weight(H, H), wk = weight(H, H), wv = weight(H, H), wo = weight(H, H);
    Tensor wg = weight(H, I), wu = weight(H, I), wd = weight(I, H);
    Tensor n1 = vec({H}), n2 = vec({H});
    Tensor kc = vec({1, L, H}), vc = vec({1, L, H});
    Tensor x = vec({1, 1, H});
    Tensor pos(TensorShape({1}));
    pos.data_ptr<float>()[0] = (float)(L - 1);
    const uint64_t hd = H / heads;
    auto t0 = std::chrono::steady_clock::now();
    for (int it = 0; it < n_layers; ++it) {
      Tensor xn = e.rms_norm(x, n1);
      Tensor q = e.matmul(xn, wq), k = e.matmul(xn, wk), v = e.matmul(xn, wv);
      Tensor q4 = e.apply_rope(q.reshape(TensorShape({1, heads, 1, hd})), pos);
      Tensor k4 = e.apply_rope(k.reshape(TensorShape({1, heads, 1, hd})), pos);
      std::memcpy(kc.data_ptr<float>() + (L - 1) * H, k4.data(), H * sizeof(float));
      std::memcpy(vc.data_ptr<float>() + (L - 1) * H, v.data(), H * sizeof(float));
      Tensor a = e.multi_head_attention(q4.reshape(TensorShape({1, 1, H})), kc, vc, heads);
      Tensor h1 = e.add(x, e.matmul(a, wo));
      Tensor xn2 = e.rms_norm(h1, n2);
      Tensor g = e.silu(e.matmul(xn2, wg));
      Tensor u = e.matmul(xn2, wu);
      x = e.add(h1, e.matmul(e.multiply(u, g), wd));
    }
    auto t1 = std::chrono::steady_clock::now();
    Tensor lm = weight(H, V);
    auto t2 = std::chrono::steady_clock::now();
    Tensor logits = e.matmul(x, lm);
    auto t3 = std::chrono::steady_clock::now();
    *layer_seconds = std::chrono::duration<double>(t1 - t0).count() / n_layers;
    *head_seconds = std::chrono::duration<double>(t3 - t2).count();
    return (int)logits.shape().total_size();
  });
}

// Quantizer::quantize_model + save_quantized_model (quantization.cpp:79-211) on a ModelData of
// fp32 tensors added in the given order: the TINQ fixtures of tests/golden/gen_tinq.py.
int ref_tinq_save(const char* path, int qtype, int symmetric, int n, const char* const* names,
                  const float* const* data, const int* ndims, const uint64_t* dims, const char* name,
                  const char* arch, const char* version, const uint64_t* sizes /* vocab hidden layers heads inter */,
                  float rope_theta) {
  return guard([&] {
    turboinfer::model::ModelData md;
    auto& m = md.metadata();
    m.name = name;
    m.architecture = arch;
    m.version = version;
    m.vocab_size = sizes[0];
    m.hidden_size = sizes[1];
    m.num_layers = sizes[2];
    m.num_heads = sizes[3];
    m.intermediate_size = sizes[4];
    m.rope_theta = rope_theta;
    const uint64_t* d = dims;
    for (int i = 0; i < n; ++i) {
      md.add_tensor(names[i], make(data[i], ndims[i], d));
      d += ndims[i];
    }
    turboinfer::optimize::QuantizationConfig qc;
    qc.type = qtype == 0 ? turboinfer::optimize::QuantizationType::kInt8 : turboinfer::optimize::QuantizationType::kInt4;
    qc.symmetric = symmetric != 0;
    turboinfer::optimize::Quantizer qz(qc);
    qz.save_quantized_model(qz.quantize_model(md), path);
    return 0;
  });
}

// ModelLoader::load (model_loader.cpp:710-873 for .gguf) of a file written by
// tests/golden/gen_gguf.py, dumped as api_check's gguf_load does.
int ref_gguf_dump(const char* in, const char* out) {
  return guard([&] {
    dump_model_data(turboinfer::model::ModelLoader::load(in), out);
    return 0;
  });
}

}  // extern "C"
