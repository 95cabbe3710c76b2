// turboinfer/model/inference_engine.hpp -- the drop-in InferenceEngine on MI355X.
//
// Same names, signatures and semantics as the reference's turboinfer::model::InferenceEngine
// (include/turboinfer/model/inference_engine.hpp:65-208 there; behaviour of
// src/model/inference_engine.cpp:695-828, 1014-1150, 1401-1427, 1554-1673): build from a
// ModelData, generate() returns prompt + new tokens and stops at EOS (id 2) or
// max_sequence_length, generate_batch() runs independent requests, sampling follows
// sample_next_token (temperature, top-k with the reference's sort order, top-p,
// uniform draw from a clock-seeded mt19937).
//
// Behind it (the pimpl InferenceEngineImpl, reference hpp:214) is the device-resident
// decode engine of include/ti_engine.h on one MI355X: packed INT4/INT8/fp16 weights and a
// fp16 KV cache in HBM, the whole decode step captured in a hipGraph.  Greedy requests
// (top_k == 1) run their token loop on the device; other sampling settings and logprobs
// take the logits to the host each step unless the device sampler runs them.  Prompts are
// prefilled in chunks of up to 1024 rows through the tile GEMM and the MFMA causal attention
// (DESIGN 4.6).
//
// Binary layout: every public class has the reference's layout (InferenceConfig 48 bytes, the
// engine's private members mirrored: tensor_engine_, impl_, the vocabulary maps), so a program
// compiled against the reference's headers links and runs against this library unchanged
// (tests/test_source_compat.py).  The two MI355X options live outside InferenceConfig, in the
// model's metadata or the environment (ModelMetadata::extra_params first, then the variable):
//   * "turboinfer.weight_bits" / TI_WEIGHT_BITS: the weight format below (default 0 = auto);
//   * "turboinfer.gpu_index" / TI_GPU_INDEX: the HIP device the engine binds (default 0).
//   * "turboinfer.synthetic" / TI_SYNTHETIC: "1" lets a ModelData with metadata but no tensors (the
//     reference's test programs) build the engine's seeded synthetic INT4 model of that shape
//     (ti_engine_synth; the reference runs such a model on its placeholder fallbacks); without it
//     such a ModelData throws std::runtime_error.
// TensorEngine binds the device TI_GPU_INDEX names (default 0).
//
// Model forms accepted (reference weight names, inference_engine.cpp:483-563):
//   * llama: token_embeddings / embed_tokens, per-layer q/k/v/o, gate/up/down, both norms,
//     final norm, lm_head / output; k/v narrower than q select GQA.
//   * plumbing (the reference benchmark's model, no attention / gate / norm weights): the
//     reference_compat path -- placeholder embeddings, attention bypass, ReLU FFN, fp32.
// Weight formats: fp32 tensors are packed as `weight_bits` (4/8: symmetric group-128
// quantization, 16: fp16); int8 / int32 tensors from Quantizer::quantize_model keep their
// integer values with unit scale (the reference's raw-cast semantics).  GGUF Q4_0 / Q4_1 / Q8_0
// checkpoints keep their 32-weight blocks exactly (weight_bits 0 picks 4 | 32, 4 | 32 | 64 or
// 8 | 32: TI_BITS_G32, TI_BITS_AFF of ti_hip.h).
#pragma once

#include <cstddef>
#include <memory>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "../core/tensor.hpp"
#include "../core/tensor_engine.hpp"
#include "model_loader.hpp"

namespace turboinfer {
namespace model {

struct InferenceConfig {
  size_t max_sequence_length = 2048;
  size_t max_batch_size = 32;
  float temperature = 1.0f;
  float top_p = 0.9f;
  size_t top_k = 50;
  float length_penalty = 1.0f;
  int eos_token_id = 2;
  bool use_cache = true;
  core::ComputeDevice device = core::ComputeDevice::kAuto;
};

struct GenerationResult {
  std::vector<int> tokens;
  std::vector<float> logprobs;
  float total_time_ms = 0.0f;
  float tokens_per_second = 0.0f;
  bool finished = false;
  std::string stop_reason;
};

class InferenceEngine {
 public:
  explicit InferenceEngine(const ModelData& model_data, const InferenceConfig& config = InferenceConfig{});
  explicit InferenceEngine(const std::string& model_path, const InferenceConfig& config = InferenceConfig{});
  ~InferenceEngine();
  InferenceEngine(const InferenceEngine&) = delete;
  InferenceEngine& operator=(const InferenceEngine&) = delete;
  InferenceEngine(InferenceEngine&&) noexcept;
  InferenceEngine& operator=(InferenceEngine&&) noexcept;

  const ModelMetadata& model_metadata() const noexcept { return model_metadata_; }
  const InferenceConfig& config() const noexcept { return config_; }
  void set_config(const InferenceConfig& config);

  GenerationResult generate(const std::string& prompt, size_t max_new_tokens, bool include_logprobs = false);
  GenerationResult generate(const std::vector<int>& input_tokens, size_t max_new_tokens,
                            bool include_logprobs = false);
  std::vector<GenerationResult> generate_batch(const std::vector<std::string>& prompts, size_t max_new_tokens,
                                               bool include_logprobs = false);
  std::vector<GenerationResult> generate_batch(const std::vector<std::vector<int>>& input_token_batches,
                                               size_t max_new_tokens, bool include_logprobs = false);
  std::vector<GenerationResult> generate_beam_search(const std::vector<int>& input_tokens, size_t max_new_tokens,
                                                     size_t beam_size = 4, bool include_logprobs = false);
  std::vector<float> compute_logprobs(const std::vector<int>& tokens);
  std::vector<int> encode(const std::string& text);
  std::string decode(const std::vector<int>& tokens);
  void reset_state();
  size_t memory_usage() const;
  std::string performance_stats() const;

 private:
  // the reference's data members in its order (inference_engine.hpp:211-214, 318-320 there)
  ModelMetadata model_metadata_;
  InferenceConfig config_;
  std::unique_ptr<core::TensorEngine> tensor_engine_;
  std::unique_ptr<class InferenceEngineImpl> impl_;
  std::unordered_map<std::string, int> vocab_map_;      // (tokenizer: out of scope, kept empty)
  std::unordered_map<int, std::string> id_to_token_;
  std::vector<std::pair<std::string, std::string>> bpe_merges_;
  void validate_input_tokens(const std::vector<int>& tokens) const;
  void validate_batch_size(size_t batch_size) const;
};

std::unique_ptr<InferenceEngine> create_engine(const std::string& model_path,
                                               const InferenceConfig& config = InferenceConfig{});
std::string quick_generate(const std::string& model_path, const std::string& prompt, size_t max_tokens = 50,
                           float temperature = 1.0f);

}  // namespace model
}  // namespace turboinfer
