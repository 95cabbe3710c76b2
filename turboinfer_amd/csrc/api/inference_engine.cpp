// inference_engine.cpp -- turboinfer::model::InferenceEngine on MI355X.
//
// InferenceEngineImpl (the reference's pimpl, inference_engine.hpp:214) owns one
// ti_engine (include/ti_engine.h): weights resolved by the reference's names
// (inference_engine.cpp:483-563) and uploaded once, KV / activations / step graph on the
// device.  Host logic here: the generate() contract (:734-802), batch validation
// (:1409-1427), sampling (:1554-1673, via ti_sample_token), statistics (:1014-1150).
#include "turboinfer/model/inference_engine.hpp"

#include <algorithm>
#include <map>
#include <chrono>
#include <cstdlib>
#include <cmath>
#include <iomanip>
#include <random>
#include <sstream>
#include <stdexcept>

#include "api_common.hpp"
#include "ti_engine.h"
#include "ti_hip.h"

namespace turboinfer {
namespace model {

using api::check;

namespace {

// generate()'s end-of-sequence token: the reference tests `next_token == 2` (inference_engine.cpp:759-760),
// not config.eos_token_id (which only its beam search reads, :2015)
constexpr int kGenerateEos = 2;

// The reference's public layouts are kept (a program built against its headers links against
// this library): InferenceConfig has no room for the MI355X options, so they come from the model's
// extra_params, then the environment, then the default (inference_engine.hpp header note).
static_assert(sizeof(InferenceConfig) == 48 && sizeof(GenerationResult) == 96, "reference layout (LP64)");
static_assert(sizeof(InferenceEngine) == 400, "reference layout (LP64)");
int engine_option(const ModelMetadata& md, const char* key, const char* env, int dflt) {
  const auto it = md.extra_params.find(key);
  if (it != md.extra_params.end()) return std::atoi(it->second.c_str());
  if (const char* v = std::getenv(env)) return std::atoi(v);
  return dflt;
}

[[noreturn]] void off_path(const std::string& what, const char* row) {
  throw std::runtime_error("InferenceEngine::" + what + ": not part of the MI355X decode hot path (SURVEY.md 8(f) " +
                           row + ")");
}

const core::Tensor* find(const ModelData& m, std::initializer_list<std::string> names) {
  for (const auto& n : names)
    if (const core::Tensor* t = m.get_tensor(n)) return t;
  return nullptr;
}

const core::Tensor* layer_tensor(const ModelData& m, size_t l, const char* hf, const char* meta) {
  const std::string a = "model.layers." + std::to_string(l) + ".", b = "layers." + std::to_string(l) + ".";
  return find(m, {a + hf, b + meta, b + hf});
}

// A ModelData read from a llama GGUF (ModelLoader::load) carries llama.cpp's
// tensor names and [out][in] linear weights; the engine takes the reference's names and [in][out]
// (ti_engine.h slots).  llama.cpp's q / k rows are already ordered for adjacent-pair RoPE, the
// rotation apply_rope implements (tensor_engine.cpp:1602-1612), so only names and the transpose
// change.  A file without output.weight ties the lm_head to the embedding.
bool gguf_named(const ModelData& m) { return m.get_tensor("blk.0.ffn_up.weight") != nullptr; }

core::Tensor transposed_f32(const core::Tensor& t) {
  if (t.shape().ndim() != 2) throw std::runtime_error("InferenceEngine: GGUF linear weight is not 2-D");
  const size_t r = t.shape().size(0), c = t.shape().size(1);
  const std::vector<float> v = api::to_f32(t);
  core::Tensor o(core::TensorShape({c, r}), core::DataType::kFloat32);
  float* d = o.data_ptr<float>();
  for (size_t i = 0; i < r; ++i)
    for (size_t j = 0; j < c; ++j) d[j * r + i] = v[i * c + j];
  return o;
}

ModelData from_gguf_names(const ModelData& g) {
  ModelData m;
  m.metadata() = g.metadata();
  auto need = [&](const std::string& n) -> const core::Tensor& {
    const core::Tensor* t = g.get_tensor(n);
    if (!t) throw std::runtime_error("InferenceEngine: GGUF model lacks " + n);
    return *t;
  };
  m.add_tensor("token_embeddings.weight", need("token_embd.weight"));
  // older converters omit llama.vocab_size: the embedding's rows are the vocabulary
  const core::Tensor& emb = need("token_embd.weight");
  if (m.metadata().vocab_size == 0 && emb.shape().ndim() == 2) m.metadata().vocab_size = emb.shape().size(0);
  m.add_tensor("norm.weight", need("output_norm.weight"));
  const core::Tensor* out = g.get_tensor("output.weight");
  m.add_tensor("lm_head.weight", transposed_f32(out ? *out : need("token_embd.weight")));
  for (size_t l = 0; l < g.metadata().num_layers; ++l) {
    const std::string b = "blk." + std::to_string(l) + ".", r = "layers." + std::to_string(l) + ".";
    m.add_tensor(r + "attention.q_proj.weight", transposed_f32(need(b + "attn_q.weight")));
    m.add_tensor(r + "attention.k_proj.weight", transposed_f32(need(b + "attn_k.weight")));
    m.add_tensor(r + "attention.v_proj.weight", transposed_f32(need(b + "attn_v.weight")));
    m.add_tensor(r + "attention.o_proj.weight", transposed_f32(need(b + "attn_output.weight")));
    m.add_tensor(r + "feed_forward.w3.weight", transposed_f32(need(b + "ffn_gate.weight")));
    m.add_tensor(r + "feed_forward.w1.weight", transposed_f32(need(b + "ffn_up.weight")));
    m.add_tensor(r + "feed_forward.w2.weight", transposed_f32(need(b + "ffn_down.weight")));
    m.add_tensor(r + "attention_norm.weight", need(b + "attn_norm.weight"));
    m.add_tensor(r + "ffn_norm.weight", need(b + "ffn_norm.weight"));
  }
  return m;
}

// GGUF Q4_0 / Q8_0 checkpoints reach the engine as ggml dequantizes them (gguf.cpp): every
// 32-weight block along K of an output column is d * q with d fp16 and q an integer of
// [-8, 7] (Q4_0) or [-127, 127] (Q8_0).  Recover (q, d) exactly from the fp32 values so the
// engine holds the checkpoint's blocks as they are (group-32 tiles, TI_BITS_G32) instead of
// re-quantizing them per 128.  ggml's quantizers put the block's largest magnitude at q = -8
// (Q4_0, d = max / -8) or |q| = 127 (Q8_0), so the first candidate nearly always fits.
bool recover_g32(const std::vector<float>& w, size_t K, size_t N, int bits, std::vector<int8_t>& q,
                 std::vector<uint16_t>& d) {
  if (K % 32 || w.size() != K * N) return false;
  const int lo = bits == 4 ? -8 : -127, hi = bits == 4 ? 7 : 127;
  q.assign(K * N, 0);
  d.assign(K / 32 * N, 0);
  auto half_bits = [](float f) {
    const _Float16 h = (_Float16)f;
    uint16_t u;
    std::memcpy(&u, &h, 2);
    return u;
  };
  auto half_val = [](uint16_t u) {
    _Float16 h;
    std::memcpy(&h, &u, 2);
    return (float)h;
  };
  std::vector<float> cand;
  for (size_t n = 0; n < N; ++n)
    for (size_t b = 0; b < K / 32; ++b) {
      float xm = 0.0f;
      for (size_t k = 32 * b; k < 32 * b + 32; ++k)
        if (std::fabs(w[k * N + n]) > std::fabs(xm)) xm = w[k * N + n];
      if (xm == 0.0f) continue;   // all zero: q = 0, d = 0
      cand.clear();
      const float sgn = xm > 0.0f ? 1.0f : -1.0f, a = std::fabs(xm);
      if (bits == 4) {
        cand.push_back(-sgn * a / 8.0f);
        for (int j = 7; j >= 1; --j) {
          cand.push_back(sgn * a / (float)j);
          cand.push_back(-sgn * a / (float)j);
        }
      } else {
        for (int j = 127; j >= 1; --j) cand.push_back(a / (float)j);
      }
      bool found = false;
      for (float c : cand) {
        const uint16_t dh = half_bits(c);
        const float dd = half_val(dh);
        if (dd == 0.0f || !std::isfinite(dd)) continue;
        bool ok = true;
        for (size_t k = 32 * b; k < 32 * b + 32 && ok; ++k) {
          const float x = w[k * N + n], r = std::rint(x / dd);
          ok = r >= (float)lo && r <= (float)hi && r * dd == x;
        }
        if (!ok) continue;
        for (size_t k = 32 * b; k < 32 * b + 32; ++k) q[k * N + n] = (int8_t)std::rint(w[k * N + n] / dd);
        d[b * N + n] = dh;
        found = true;
        break;
      }
      if (!found) return false;
    }
  return true;
}

// GGUF Q4_1 checkpoints likewise: every block is fl(q * d + m) with q in [0, 15] and d, m fp16
// (gguf.cpp dequant_q4_1).  ggml's Q4_1 quantizer maps the block minimum to q = 0 (so m is the
// smallest value, exactly) and the maximum to q = 15; d is the fp16 nearest (max - m) / 15 or
// one of its neighbours.  Every candidate is verified weight by weight.
bool recover_q41(const std::vector<float>& w, size_t K, size_t N, std::vector<int8_t>& q, std::vector<uint16_t>& d,
                 std::vector<uint16_t>& m) {
  if (K % 32 || w.size() != K * N) return false;
  q.assign(K * N, 0);
  d.assign(K / 32 * N, 0);
  m.assign(K / 32 * N, 0);
  auto half_bits = [](float f) {
    const _Float16 h = (_Float16)f;
    uint16_t u;
    std::memcpy(&u, &h, 2);
    return u;
  };
  auto half_val = [](uint16_t u) {
    _Float16 h;
    std::memcpy(&h, &u, 2);
    return (float)h;
  };
  for (size_t n = 0; n < N; ++n)
    for (size_t b = 0; b < K / 32; ++b) {
      float lo = INFINITY, hi = -INFINITY;
      for (size_t k = 32 * b; k < 32 * b + 32; ++k) {
        lo = std::min(lo, w[k * N + n]);
        hi = std::max(hi, w[k * N + n]);
      }
      const uint16_t mh = half_bits(lo);
      if (half_val(mh) != lo) return false;
      m[b * N + n] = mh;
      if (hi == lo) continue;   // constant block: q = 0, d = 0
      const uint16_t d0 = half_bits((hi - lo) / 15.0f);
      bool found = false;
      for (int dj : {0, 1, -1, 2, -2}) {
        const uint16_t dh = (uint16_t)(d0 + dj);
        const float dd = half_val(dh);
        if (!(dd > 0.0f) || !std::isfinite(dd)) continue;
        bool ok = true;
        for (size_t k = 32 * b; k < 32 * b + 32 && ok; ++k) {
          const float x = w[k * N + n], r = std::rint((x - lo) / dd);
          ok = r >= 0.0f && r <= 15.0f && r * dd + lo == x;
        }
        if (!ok) continue;
        for (size_t k = 32 * b; k < 32 * b + 32; ++k) q[k * N + n] = (int8_t)std::rint((w[k * N + n] - lo) / dd);
        d[b * N + n] = dh;
        found = true;
        break;
      }
      if (!found) return false;
    }
  return true;
}

bool is_int(const core::Tensor& t) {
  return t.dtype() == core::DataType::kInt8 || t.dtype() == core::DataType::kInt32 ||
         t.dtype() == core::DataType::kInt16 || t.dtype() == core::DataType::kUInt8;
}

}  // namespace

class InferenceEngineImpl {
 public:
  ti_engine* eng = nullptr;
  ti_engine_config cfg{};
  int capacity = 1;      // streams one device call holds
  bool compat = false;
  std::mt19937 rng;
  size_t total_generations = 0, total_tokens = 0, total_forward_passes = 0;
  float total_time_ms = 0.0f, peak_tps = 0.0f;

  bool gguf_src = false;  // built from a GGUF-read ModelData (llama.cpp names)
  // group-32 blocks recovered per linear weight (recover_g32 / recover_q41), reused by upload()
  struct Blocks {
    std::vector<int8_t> q;
    std::vector<uint16_t> d, m;   // m: Q4_1 block minimums
  };
  std::map<const core::Tensor*, Blocks> g32;

  static bool recover(const std::vector<float>& w, size_t K, size_t N, int bits, Blocks& b) {
    return (bits & TI_BITS_AFF) ? recover_q41(w, K, N, b.q, b.d, b.m)
                                : recover_g32(w, K, N, bits & ~TI_BITS_G32, b.q, b.d);
  }

  InferenceEngineImpl() { rng.seed((unsigned)std::chrono::steady_clock::now().time_since_epoch().count()); }

  // every linear weight of the model is exact group-32 blocks of `bits` (4 | G32, 8 | G32 or
  // 4 | G32 | AFF; cached on success)
  bool all_g32(const ModelData& m, size_t L, size_t H, size_t qd, size_t kvd, size_t I, size_t V, int bits) {
    g32.clear();
    auto one = [&](const core::Tensor* t, size_t K, size_t N) {
      if (!t || t->shape().total_size() != K * N) return false;
      return recover(api::to_f32(*t), K, N, bits, g32[t]);
    };
    bool ok = one(find(m, {"lm_head.weight", "output.weight"}), H, V);
    for (size_t l = 0; l < L && ok; ++l)
      ok = one(layer_tensor(m, l, "self_attn.q_proj.weight", "attention.q_proj.weight"), H, qd) &&
           one(layer_tensor(m, l, "self_attn.k_proj.weight", "attention.k_proj.weight"), H, kvd) &&
           one(layer_tensor(m, l, "self_attn.v_proj.weight", "attention.v_proj.weight"), H, kvd) &&
           one(layer_tensor(m, l, "self_attn.o_proj.weight", "attention.o_proj.weight"), qd, H) &&
           one(layer_tensor(m, l, "mlp.gate_proj.weight", "feed_forward.w3.weight"), H, I) &&
           one(layer_tensor(m, l, "mlp.up_proj.weight", "feed_forward.w1.weight"), H, I) &&
           one(layer_tensor(m, l, "mlp.down_proj.weight", "feed_forward.w2.weight"), I, H);
    if (!ok) g32.clear();
    return ok;
  }
  ~InferenceEngineImpl() {
    if (eng) ti_engine_destroy(eng);
  }

  void upload(int slot, int layer, const core::Tensor& t, size_t K, size_t N, int bits) {
    if ((bits & TI_BITS_G32) && t.shape().total_size() == K * N) {   // exact blocks when the weight has them
      auto it = g32.find(&t);
      Blocks b;
      if (it != g32.end()) {
        b = std::move(it->second);
        g32.erase(it);
      }
      if (!b.q.empty() || recover(api::to_f32(t), K, N, bits, b)) {
        if (bits & TI_BITS_AFF)
          check(ti_engine_set_tensor_q1(eng, slot, layer, reinterpret_cast<const uint8_t*>(b.q.data()), b.d.data(),
                                        b.m.data()),
                "ti_engine_set_tensor_q1");
        else
          check(ti_engine_set_tensor_q(eng, slot, layer, b.q.data(), b.d.data()), "ti_engine_set_tensor_q");
        return;
      }
    }   // otherwise quantized below (ggml's Q4_1 rounding on affine engines, ti_wpack_host)
    if (t.shape().total_size() != K * N)
      throw std::runtime_error("InferenceEngine: weight for slot " + std::to_string(slot) + " layer " +
                               std::to_string(layer) + " has " + std::to_string(t.shape().total_size()) +
                               " elements, expected " + std::to_string(K) + "x" + std::to_string(N));
    const std::vector<float> v = api::to_f32(t);
    int mode = TI_SCALE_GROUP;
    if (is_int(t)) {
      mode = TI_SCALE_UNIT;   // Quantizer output: the reference multiplies the raw integers (convert_dtype)
      const float lo = bits == 4 ? -8.0f : -128.0f, hi = bits == 4 ? 7.0f : 127.0f;
      if (bits != 16)
        for (float x : v)
          if (x < lo || x > hi)
            throw std::runtime_error("InferenceEngine: integer weight value " + std::to_string(x) +
                                     " does not fit the " + std::to_string(bits) + "-bit tiles");
    }
    check(ti_engine_set_tensor(eng, slot, layer, v.data(), mode), "ti_engine_set_tensor");
  }

  void upload_vec(int slot, int layer, const core::Tensor& t, size_t n) {
    if (t.shape().total_size() != n)
      throw std::runtime_error("InferenceEngine: vector for slot " + std::to_string(slot) + " has " +
                               std::to_string(t.shape().total_size()) + " elements, expected " + std::to_string(n));
    const std::vector<float> v = api::to_f32(t);
    check(ti_engine_set_tensor(eng, slot, layer, v.data(), TI_SCALE_UNIT), "ti_engine_set_tensor");
  }

  // The device engine of cfg (filled in by the caller but for the stream capacity).
  void create(const InferenceConfig& c) {
    cfg.attn_splits = 0;
    // streams held at once: the configured batch, bounded to 64 GiB of fp16 KV
    const double kv_stream = 2.0 * cfg.layers * cfg.kv_heads * cfg.head_dim * 2.0 * cfg.max_seq;
    capacity = (int)std::max<size_t>(1, std::min<size_t>(c.max_batch_size, (size_t)(64.0 * (1ull << 30) / kv_stream)));
    capacity = std::min(capacity, 64);
    cfg.max_batch = compat ? 1 : capacity;
    check(ti_init(cfg.device), "ti_init");
    check(ti_engine_create(&cfg, &eng), "ti_engine_create");
    // generate() ends its device loop at EOS (token id 2, inference_engine.cpp:759-764)
    if (!compat) check(ti_engine_set_stop(eng, kGenerateEos), "ti_engine_set_stop");
  }

  // Metadata without tensors (the reference's own test programs build engines this way and run
  // them on its placeholder fallbacks, inference_engine.cpp:293-296, 377-380, 672-684): the
  // engine's seeded synthetic llama model of that shape (ti_engine_synth), INT4 unless the
  // weight_bits option says 8 or 16.
  void build_synthetic(const ModelMetadata& md, const InferenceConfig& c, int gpu) {
    const int H = (int)md.hidden_size, nh = (int)md.num_heads;
    cfg.vocab = (int)md.vocab_size;
    cfg.hidden = H;
    cfg.layers = (int)md.num_layers;
    cfg.heads = nh;
    cfg.kv_heads = nh;
    cfg.head_dim = H / nh;
    cfg.inter = md.intermediate_size ? (int)md.intermediate_size : 4 * H;
    cfg.rope_theta = md.rope_theta > 0.0f ? md.rope_theta : 10000.0f;
    cfg.eps = 1e-5f;
    const int bits = engine_option(md, "turboinfer.weight_bits", "TI_WEIGHT_BITS", 0);
    cfg.bits = bits == 8 || bits == 16 ? bits : 4;
    cfg.max_seq = (int)std::max<size_t>(1, c.max_sequence_length);
    cfg.compat = 0;
    cfg.device = gpu;
    compat = false;
    create(c);
    check(ti_engine_synth(eng, 0x7475726269ull, 0.0f), "ti_engine_synth");
  }

  void build(const ModelData& m, const InferenceConfig& c) {
    if (gguf_named(m)) {
      gguf_src = true;
      return build(from_gguf_names(m), c);
    }
    const ModelMetadata& md = m.metadata();
    const size_t H = md.hidden_size, L = md.num_layers, nh = md.num_heads, V = md.vocab_size;
    size_t I = md.intermediate_size;
    if (!H || !L || !nh || !V || H % nh) throw std::runtime_error("InferenceEngine: incomplete model metadata");
    const size_t hd = H / nh;
    const int gpu = engine_option(md, "turboinfer.gpu_index", "TI_GPU_INDEX", 0);
    if (m.num_tensors() == 0) {
      // a tensorless ModelData (what the reference's test programs build) runs the seeded synthetic
      // model of that shape only when asked: otherwise a checkpoint that failed to load would decode
      // plausible-looking tokens from random weights
      if (engine_option(md, "turboinfer.synthetic", "TI_SYNTHETIC", 0) != 1)
        throw std::runtime_error("InferenceEngine: the model has metadata but no tensors (set "
                                 "extra_params[\"turboinfer.synthetic\"] = \"1\" or TI_SYNTHETIC=1 for the "
                                 "seeded synthetic model of this shape)");
      return build_synthetic(md, c, gpu);
    }
    const core::Tensor* q0 = layer_tensor(m, 0, "self_attn.q_proj.weight", "attention.q_proj.weight");
    const core::Tensor* k0 = layer_tensor(m, 0, "self_attn.k_proj.weight", "attention.k_proj.weight");
    const core::Tensor* up0 = layer_tensor(m, 0, "mlp.up_proj.weight", "feed_forward.w1.weight");
    const core::Tensor* lm = find(m, {"lm_head.weight", "output.weight"});
    if (!up0 || !lm) throw std::runtime_error("InferenceEngine: model has no FFN up / lm_head weights");
    if (!I) I = up0->shape().total_size() / H;
    compat = (q0 == nullptr);

    // weight format
    int bits = engine_option(md, "turboinfer.weight_bits", "TI_WEIGHT_BITS", 0);
    if (bits == 0) {
      bits = 16;
      if (is_int(*up0)) {
        bits = up0->dtype() == core::DataType::kInt32 ? 4 : 8;
        const std::vector<float> v = api::to_f32(*up0);
        for (float x : v)
          if (x < -8.0f || x > 7.0f) bits = 8;
      } else if (gguf_src && q0) {   // Q4_0 / Q4_1 / Q8_0 checkpoint: keep its blocks
        const size_t kvd = k0 ? k0->shape().total_size() / H : H;
        if (all_g32(m, L, H, H, kvd, I, V, 4 | TI_BITS_G32)) bits = 4 | TI_BITS_G32;
        else if (all_g32(m, L, H, H, kvd, I, V, 4 | TI_BITS_G32 | TI_BITS_AFF)) bits = 4 | TI_BITS_G32 | TI_BITS_AFF;
        else if (all_g32(m, L, H, H, kvd, I, V, 8 | TI_BITS_G32)) bits = 8 | TI_BITS_G32;
      }
    }
    if (bits != 4 && bits != 8 && bits != 16 && bits != (4 | TI_BITS_G32) && bits != (8 | TI_BITS_G32) &&
        bits != (4 | TI_BITS_G32 | TI_BITS_AFF))
      throw std::runtime_error(
          "InferenceEngine: weight_bits must be 4, 8, 16, 4 / 8 | 32 (group-32 blocks) or 4 | 32 | 64 (Q4_1 blocks)");
    cfg.vocab = (int)V;
    cfg.hidden = (int)H;
    cfg.layers = (int)L;
    cfg.heads = (int)nh;
    cfg.head_dim = (int)hd;
    cfg.kv_heads = (int)nh;
    if (k0) {
      const size_t kvd = k0->shape().total_size() / H;
      if (kvd % hd || !kvd) throw std::runtime_error("InferenceEngine: k_proj width not a multiple of head_dim");
      cfg.kv_heads = (int)(kvd / hd);
    }
    cfg.inter = (int)I;
    cfg.rope_theta = md.rope_theta > 0.0f ? md.rope_theta : 10000.0f;
    cfg.eps = 1e-5f;
    cfg.bits = compat ? 16 : bits;
    cfg.max_seq = (int)std::max<size_t>(1, c.max_sequence_length);
    cfg.compat = compat ? 1 : 0;
    cfg.device = gpu;
    create(c);

    for (size_t l = 0; l < L; ++l) {
      const int li = (int)l;
      const core::Tensor* up = layer_tensor(m, l, "mlp.up_proj.weight", "feed_forward.w1.weight");
      const core::Tensor* down = layer_tensor(m, l, "mlp.down_proj.weight", "feed_forward.w2.weight");
      if (!up || !down) throw std::runtime_error("InferenceEngine: layer " + std::to_string(l) + " lacks FFN weights");
      upload(TI_W_UP, li, *up, H, I, cfg.bits);
      upload(TI_W_DOWN, li, *down, I, H, cfg.bits);
      if (compat) continue;
      const size_t qd = nh * hd, kvd = (size_t)cfg.kv_heads * hd;
      const core::Tensor* q = layer_tensor(m, l, "self_attn.q_proj.weight", "attention.q_proj.weight");
      const core::Tensor* k = layer_tensor(m, l, "self_attn.k_proj.weight", "attention.k_proj.weight");
      const core::Tensor* v = layer_tensor(m, l, "self_attn.v_proj.weight", "attention.v_proj.weight");
      const core::Tensor* o = layer_tensor(m, l, "self_attn.o_proj.weight", "attention.o_proj.weight");
      const core::Tensor* g = layer_tensor(m, l, "mlp.gate_proj.weight", "feed_forward.w3.weight");
      const core::Tensor* an = layer_tensor(m, l, "input_layernorm.weight", "attention_norm.weight");
      const core::Tensor* fn = layer_tensor(m, l, "post_attention_layernorm.weight", "ffn_norm.weight");
      if (!q || !k || !v || !o || !g || !an || !fn)
        throw std::runtime_error("InferenceEngine: layer " + std::to_string(l) +
                                 " lacks attention / gate / norm weights (a llama model needs all of them)");
      upload(TI_W_Q, li, *q, H, qd, cfg.bits);
      upload(TI_W_K, li, *k, H, kvd, cfg.bits);
      upload(TI_W_V, li, *v, H, kvd, cfg.bits);
      upload(TI_W_O, li, *o, qd, H, cfg.bits);
      upload(TI_W_GATE, li, *g, H, I, cfg.bits);
      upload_vec(TI_V_ATTN_NORM, li, *an, H);
      upload_vec(TI_V_FFN_NORM, li, *fn, H);
    }
    upload(TI_W_LM_HEAD, 0, *lm, H, V, cfg.bits);
    if (!compat) {
      const core::Tensor* norm = find(m, {"norm.weight", "model.norm.weight"});
      const core::Tensor* emb = find(m, {"token_embeddings.weight", "embed_tokens.weight"});
      if (!norm || !emb) throw std::runtime_error("InferenceEngine: llama model needs norm.weight and the token embeddings");
      upload_vec(TI_V_OUT_NORM, 0, *norm, H);
      upload_vec(TI_E_EMBED, 0, *emb, V * H);
    }
  }

  // sample_next_token (inference_engine.cpp:1554-1673) with the engine's mt19937 draw
  int sample(const float* logits, const InferenceConfig& c, std::vector<float>* logprobs) {
    std::uniform_real_distribution<float> dist(0.0f, 1.0f);
    const float u = dist(rng);
    int tok = 0;
    float lp = 0.0f;
    check(ti_sample_token(logits, cfg.vocab, c.temperature, (int)std::min<size_t>(c.top_k, (size_t)cfg.vocab), c.top_p,
                          u, &tok, &lp),
          "ti_sample_token");
    if (logprobs) logprobs->push_back(lp);
    return tok;
  }
};

InferenceEngine::InferenceEngine(const ModelData& model_data, const InferenceConfig& config)
    : model_metadata_(model_data.metadata()), config_(config), impl_(std::make_unique<InferenceEngineImpl>()) {
  if (config_.device == core::ComputeDevice::kCPU)
    throw std::runtime_error("InferenceEngine: this build runs on MI355X (gfx950) only; kCPU is the reference's path");
  impl_->build(model_data, config_);
}

InferenceEngine::InferenceEngine(const std::string& model_path, const InferenceConfig& config)
    : InferenceEngine(ModelLoader::load(model_path), config) {}

InferenceEngine::~InferenceEngine() = default;
InferenceEngine::InferenceEngine(InferenceEngine&&) noexcept = default;
InferenceEngine& InferenceEngine::operator=(InferenceEngine&&) noexcept = default;

void InferenceEngine::set_config(const InferenceConfig& config) {
  if (config.max_sequence_length != config_.max_sequence_length)
    throw std::runtime_error("InferenceEngine::set_config: max_sequence_length is fixed when the device engine is built");
  config_ = config;
}

void InferenceEngine::validate_input_tokens(const std::vector<int>& tokens) const {
  if (tokens.empty()) throw std::runtime_error("Input tokens cannot be empty");
  if (tokens.size() > config_.max_sequence_length)
    throw std::runtime_error("Input sequence length exceeds maximum allowed length");
  for (int t : tokens)
    if (t < 0 || t >= impl_->cfg.vocab) throw std::runtime_error("Input token id " + std::to_string(t) + " out of vocabulary");
}

void InferenceEngine::validate_batch_size(size_t batch_size) const {
  if (batch_size == 0) throw std::runtime_error("Batch size cannot be zero");
  if (batch_size > config_.max_batch_size) throw std::runtime_error("Batch size exceeds maximum allowed batch size");
}

GenerationResult InferenceEngine::generate(const std::string&, size_t, bool) {
  off_path("generate(std::string)", "-- the tokenizer; pass token ids");
}

GenerationResult InferenceEngine::generate(const std::vector<int>& input_tokens, size_t max_new_tokens,
                                           bool include_logprobs) {
  return generate_batch(std::vector<std::vector<int>>{input_tokens}, max_new_tokens, include_logprobs).at(0);
}

std::vector<GenerationResult> InferenceEngine::generate_batch(const std::vector<std::string>&, size_t, bool) {
  off_path("generate_batch(std::vector<std::string>)", "-- the tokenizer; pass token ids");
}

std::vector<GenerationResult> InferenceEngine::generate_batch(const std::vector<std::vector<int>>& batches,
                                                              size_t max_new_tokens, bool include_logprobs) {
  validate_batch_size(batches.size());
  for (const auto& b : batches) validate_input_tokens(b);
  InferenceEngineImpl& im = *impl_;
  const size_t maxlen = config_.max_sequence_length;
  const int V = im.cfg.vocab;
  std::vector<GenerationResult> results(batches.size());
  // The contract of generate() (inference_engine.cpp:734-802): stop after EOS or once the
  // sequence reaches max_sequence_length; otherwise stop_reason "max_new_tokens".  EOS is token
  // id 2 whatever config.eos_token_id says (:759-760 hard-codes it; only beam search reads the
  // config, :2015).  total_time_ms is whole milliseconds (duration_cast<milliseconds>, :778-780)
  // and tokens_per_second = generated / (total_time_ms / 1000), inf (or NaN) under 1 ms (:782).
  auto finish = [&](GenerationResult& r, const std::vector<int>& prompt, const std::vector<int>& fresh,
                    const std::vector<float>& lps, float ms) {
    r.tokens = prompt;
    r.finished = false;
    for (size_t i = 0; i < fresh.size(); ++i) {
      r.tokens.push_back(fresh[i]);
      if (i < lps.size()) r.logprobs.push_back(lps[i]);
      if (fresh[i] == kGenerateEos) {
        r.finished = true;
        r.stop_reason = "eos_token";
        break;
      }
      if (r.tokens.size() >= maxlen) {
        r.finished = true;
        r.stop_reason = "max_length";
        break;
      }
    }
    if (!r.finished) r.stop_reason = "max_new_tokens";
    r.total_time_ms = static_cast<float>(static_cast<long long>(ms));
    const size_t gen = r.tokens.size() - prompt.size();
    r.tokens_per_second = gen / (r.total_time_ms / 1000.0f);
    im.total_generations++;
    im.total_tokens += gen;
    im.total_time_ms += r.total_time_ms;
    im.peak_tps = std::max(im.peak_tps, r.tokens_per_second);
  };
  // new tokens a request can take before max_length stops it (at least one is sampled)
  auto budget = [&](size_t plen) {
    return std::max<size_t>(1, std::min(max_new_tokens, maxlen > plen ? maxlen - plen : 1));
  };
  if (max_new_tokens == 0) {
    for (size_t i = 0; i < batches.size(); ++i) finish(results[i], batches[i], {}, {}, 0.0f);
    return results;
  }

  if (im.compat) {
    // reference_compat: placeholder-embedding plumbing model, one request at a time
    std::vector<float> logits(V);
    for (size_t i = 0; i < batches.size(); ++i) {
      const auto t0 = std::chrono::steady_clock::now();
      const auto& p = batches[i];
      std::vector<int> fresh;
      std::vector<float> lps;
      check(ti_engine_compat_step(im.eng, (int)((p.size() - 1) * im.cfg.hidden), logits.data()), "ti_engine_compat_step");
      im.total_forward_passes++;
      const size_t n = budget(p.size());
      for (size_t s = 0; s < n; ++s) {
        const int tok = im.sample(logits.data(), config_, include_logprobs ? &lps : nullptr);
        fresh.push_back(tok);
        if (tok == kGenerateEos || p.size() + fresh.size() >= maxlen || s + 1 == n) break;
        check(ti_engine_compat_step(im.eng, 0, logits.data()), "ti_engine_compat_step");
        im.total_forward_passes++;
      }
      const float ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
      finish(results[i], p, fresh, lps, ms);
    }
    return results;
  }

  const bool greedy = config_.top_k == 1 && !include_logprobs;
  // Requests go to the device together, `capacity` at a time.  A greedy group advances in
  // lock step from position 0, so the longest prompt bounds everyone's KV room: when that
  // would cut a request short of its budget, the group is run one request at a time.
  size_t group = (size_t)im.capacity;
  if (greedy) {
    size_t longest = 0;
    for (const auto& b : batches) longest = std::max(longest, b.size());
    for (const auto& b : batches)
      if (budget(b.size()) > (size_t)im.cfg.max_seq + 1 - longest) group = 1;
  }
  for (size_t c0 = 0; c0 < batches.size(); c0 += group) {
    const int n = (int)std::min<size_t>(group, batches.size() - c0);
    const auto t0 = std::chrono::steady_clock::now();
    size_t stride = 1, want = 1;
    for (int m = 0; m < n; ++m) {
      stride = std::max(stride, batches[c0 + m].size());
      want = std::max(want, budget(batches[c0 + m].size()));
    }
    std::vector<std::vector<int>> fresh(n);
    std::vector<std::vector<float>> lps(n);
    // forward passes = the engine's decode steps + prompt chunks actually run (the device loop
    // stops at EOS in chunks, so this is not the planned step count)
    uint64_t d0 = 0, p0 = 0, d1 = 0, p1 = 0;
    check(ti_engine_counters(im.eng, &d0, &p0), "ti_engine_counters");
    const bool device_loop = greedy || (n == 1 && config_.top_k >= 1 && config_.top_k <= (size_t)V);
    if (greedy) {
      // the whole token loop on the device (argmax feedback); it stops once every request of the
      // group emitted EOS (ti_engine_set_stop), the length limit is applied after
      std::vector<int32_t> prompts((size_t)n * stride, 0), lens(n), out((size_t)n * want);
      for (int m = 0; m < n; ++m) {
        const auto& p = batches[c0 + m];
        std::copy(p.begin(), p.end(), prompts.begin() + (size_t)m * stride);
        lens[m] = (int32_t)p.size();
      }
      // the longest prompt sets the step count (steps = longest + new - 1 <= max_seq)
      const size_t steps_new = std::min(want, (size_t)im.cfg.max_seq + 1 - stride);
      check(ti_engine_generate(im.eng, n, prompts.data(), lens.data(), (int)stride, nullptr, (int)steps_new, out.data(),
                               nullptr),
            "ti_engine_generate");
      for (int m = 0; m < n; ++m) {
        const size_t b = budget(batches[c0 + m].size());
        for (size_t t = 0; t < std::min(b, steps_new); ++t) fresh[m].push_back(out[(size_t)m * steps_new + t]);
      }
    } else if (n == 1 && config_.top_k >= 1 && config_.top_k <= (size_t)V) {
      // one request with top-k sampling (any k up to the vocabulary): the whole loop on the device
      // (ti_engine_generate_sampled), fed the engine's mt19937 draws in the reference's order;
      // the generator then advances by the draws the request actually used (one per token)
      const auto& p = batches[c0];
      const size_t steps_new = std::min(want, (size_t)im.cfg.max_seq + 1 - p.size());
      std::mt19937 saved = im.rng;
      std::uniform_real_distribution<float> dist(0.0f, 1.0f);
      std::vector<float> draws(steps_new), lp(steps_new);
      for (float& d : draws) d = dist(im.rng);
      std::vector<int32_t> prompt(p.begin(), p.end()), out(steps_new);
      const int32_t len = (int32_t)p.size();
      check(ti_engine_generate_sampled(im.eng, 1, prompt.data(), &len, (int)p.size(), nullptr, (int)steps_new,
                                       config_.temperature, (int)config_.top_k, config_.top_p, draws.data(), out.data(),
                                       lp.data()),
            "ti_engine_generate_sampled");
      const size_t b = budget(p.size());
      for (size_t t = 0; t < std::min(b, steps_new); ++t) {
        fresh[0].push_back(out[t]);
        if (include_logprobs) lps[0].push_back(lp[t]);
        if (out[t] == kGenerateEos || p.size() + fresh[0].size() >= maxlen) break;
      }
      im.rng = saved;
      im.rng.discard(fresh[0].size());
    } else {
      // logits to the host every step: the reference sampler (temperature / top-k / top-p / draw)
      std::vector<float> logits((size_t)n * V);
      std::vector<int32_t> tok(n), pos(n, 0);
      std::vector<size_t> fed(n, 0);   // prompt tokens consumed
      std::vector<bool> done(n, false);
      const size_t steps = stride + want - 1;
      for (size_t s = 0; s < steps; ++s) {
        for (int m = 0; m < n; ++m) {
          const auto& p = batches[c0 + m];
          tok[m] = fed[m] < p.size() ? p[fed[m]] : (fresh[m].empty() ? 0 : fresh[m].back());
          pos[m] = (int32_t)std::min<size_t>(s, (size_t)im.cfg.max_seq - 1);
        }
        check(ti_engine_step(im.eng, n, tok.data(), pos.data(), logits.data()), "ti_engine_step");
        im.total_forward_passes++;
        bool all_done = true;
        for (int m = 0; m < n; ++m) {
          const auto& p = batches[c0 + m];
          if (fed[m] < p.size()) ++fed[m];
          if (fed[m] < p.size() || done[m]) {
            all_done = all_done && done[m];
            continue;
          }
          const int t = im.sample(&logits[(size_t)m * V], config_, include_logprobs ? &lps[m] : nullptr);
          fresh[m].push_back(t);
          if (t == kGenerateEos || fresh[m].size() >= budget(p.size())) done[m] = true;
          all_done = all_done && done[m];
        }
        if (all_done) break;
      }
    }
    const float ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (device_loop) {   // (the host-sampler loop counts its own steps)
      check(ti_engine_counters(im.eng, &d1, &p1), "ti_engine_counters");
      im.total_forward_passes += (size_t)((d1 - d0) + (p1 - p0));
    }
    for (int m = 0; m < n; ++m) finish(results[c0 + m], batches[c0 + m], fresh[m], lps[m], ms);
  }
  return results;
}

// generate_beam_search (inference_engine.cpp:830-871): the beam loop runs in ti_engine_beam_search
// (beams as KV stream slots, one batched device step per round, the reference's host ranking);
// results keep only the new tokens and, with include_logprobs, the beam's average log-probability
// per token.  max_new_tokens = 0 gives the prompt back as one finished result with no tokens.
std::vector<GenerationResult> InferenceEngine::generate_beam_search(const std::vector<int>& input_tokens,
                                                                   size_t max_new_tokens, size_t beam_size,
                                                                   bool include_logprobs) {
  if (beam_size == 0) throw std::runtime_error("Beam size must be greater than 0");
  validate_input_tokens(input_tokens);
  InferenceEngineImpl& im = *impl_;
  if (im.compat) off_path("generate_beam_search on the reference_compat plumbing model", "rank 4");
  std::vector<GenerationResult> results;
  const int nb = (int)beam_size, mn = (int)max_new_tokens;
  std::vector<int32_t> prompt(input_tokens.begin(), input_tokens.end()), out((size_t)nb * mn);
  std::vector<float> lp(nb);
  std::vector<int32_t> fin(nb);
  int count = 0;
  const auto t0 = std::chrono::steady_clock::now();
  check(ti_engine_beam_search(im.eng, prompt.data(), (int)prompt.size(), mn, nb, config_.temperature,
                              (int)std::min<size_t>(config_.top_k, (size_t)im.cfg.vocab), config_.top_p,
                              config_.length_penalty, config_.eos_token_id, out.data(), lp.data(), nullptr, fin.data(),
                              &count),
        "ti_engine_beam_search");
  const float ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
  for (int r = 0; r < count; ++r) {
    GenerationResult g;
    for (int t = 0; t < mn && out[(size_t)r * mn + t] >= 0; ++t) g.tokens.push_back(out[(size_t)r * mn + t]);
    g.finished = fin[r] != 0;
    if (include_logprobs && !g.tokens.empty()) g.logprobs.assign(g.tokens.size(), lp[r] / (float)g.tokens.size());
    g.total_time_ms = ms;
    results.push_back(std::move(g));
  }
  return results;
}
std::vector<float> InferenceEngine::compute_logprobs(const std::vector<int>&) { off_path("compute_logprobs", "rank 1"); }
std::vector<int> InferenceEngine::encode(const std::string&) { off_path("encode", "-- the tokenizer"); }
std::string InferenceEngine::decode(const std::vector<int>&) { off_path("decode", "-- the tokenizer"); }

void InferenceEngine::reset_state() {
  if (!impl_) return;
  impl_->total_generations = impl_->total_tokens = impl_->total_forward_passes = 0;
  impl_->total_time_ms = impl_->peak_tps = 0.0f;
  impl_->rng.seed((unsigned)std::chrono::steady_clock::now().time_since_epoch().count());
  // the KV cache needs no clearing: every request starts writing at position 0
}

size_t InferenceEngine::memory_usage() const {
  if (!impl_ || !impl_->eng) return 0;
  size_t w = 0, kv = 0;
  check(ti_engine_memory(impl_->eng, &w, &kv), "ti_engine_memory");
  return w + kv;
}

std::string InferenceEngine::performance_stats() const {
  if (!impl_) return "Performance statistics unavailable (engine not initialized)";
  const InferenceEngineImpl& im = *impl_;
  std::ostringstream os;
  os << std::fixed << std::setprecision(2);
  os << "=== TurboInfer Performance Statistics (MI355X) ===\n";
  os << "  Total Generations: " << im.total_generations << "\n";
  os << "  Total Tokens Generated: " << im.total_tokens << "\n";
  os << "  Total Generation Time: " << im.total_time_ms << " ms\n";
  os << "  Forward Passes: " << im.total_forward_passes << "\n";
  if (im.total_time_ms > 0.0f)
    os << "  Average Tokens/Second: " << (im.total_tokens / (im.total_time_ms / 1000.0f)) << "\n";
  os << "  Peak Tokens/Second: " << im.peak_tps << "\n";
  os << "  Device Memory: " << (memory_usage() / (1024.0 * 1024.0)) << " MB (weights " << (im.cfg.bits & ~(TI_BITS_G32 | TI_BITS_AFF))
     << "-bit" << ((im.cfg.bits & TI_BITS_AFF) ? " affine group-32 blocks" : (im.cfg.bits & TI_BITS_G32) ? " group-32 blocks" : "") << ", fp16 KV, " << im.capacity
     << " stream(s) x " << im.cfg.max_seq << " slots)\n";
  os << "  Mode: " << (im.compat ? "reference_compat (plumbing model)" : "llama decode") << "\n";
  return os.str();
}

std::unique_ptr<InferenceEngine> create_engine(const std::string& model_path, const InferenceConfig& config) {
  return std::make_unique<InferenceEngine>(model_path, config);
}

// Reference inference_engine.cpp:2075-2082: build an engine from the checkpoint, then
// generate(prompt) and decode().  The checkpoint loads (GGUF); the string prompt
// needs the tokenizer, which is out of scope, so this throws from generate(std::string) rather
// than returning text it cannot produce.
std::string quick_generate(const std::string& model_path, const std::string& prompt, size_t max_tokens,
                           float temperature) {
  InferenceConfig config;
  config.temperature = temperature;
  InferenceEngine engine(model_path, config);
  auto result = engine.generate(prompt, max_tokens);
  return engine.decode(result.tokens);
}

}  // namespace model
}  // namespace turboinfer
