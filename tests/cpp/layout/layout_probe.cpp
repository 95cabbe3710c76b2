// layout_probe.cpp -- prints sizeof / alignof / offsetof of the public TurboInfer classes.
// tests/test_source_compat.py compiles it once against the reference's include/ and once against
// this repository's include/: the two outputs must be identical (binary-layout drop-in).
#include <turboinfer/turboinfer.hpp>

#include <cstddef>
#include <cstdio>

using namespace turboinfer;
#define SIZE(T) std::printf("%-34s size %4zu align %2zu\n", #T, sizeof(T), alignof(T));
#define OFF(T, m) std::printf("  %-32s @%zu\n", #T "::" #m, offsetof(T, m));

int main() {
  SIZE(core::TensorShape) SIZE(core::Tensor) SIZE(core::TensorEngine) SIZE(model::ModelMetadata) SIZE(model::ModelData)
  SIZE(model::InferenceConfig) SIZE(model::GenerationResult) SIZE(model::InferenceEngine)
  SIZE(optimize::QuantizationConfig) SIZE(optimize::Quantizer) SIZE(optimize::QuantizationInfo)
  OFF(model::InferenceConfig, max_sequence_length) OFF(model::InferenceConfig, max_batch_size)
  OFF(model::InferenceConfig, temperature) OFF(model::InferenceConfig, top_p) OFF(model::InferenceConfig, top_k)
  OFF(model::InferenceConfig, length_penalty) OFF(model::InferenceConfig, eos_token_id)
  OFF(model::InferenceConfig, use_cache) OFF(model::InferenceConfig, device)
  OFF(model::GenerationResult, tokens) OFF(model::GenerationResult, logprobs) OFF(model::GenerationResult, total_time_ms)
  OFF(model::GenerationResult, tokens_per_second) OFF(model::GenerationResult, finished)
  OFF(model::GenerationResult, stop_reason)
  OFF(model::ModelMetadata, name) OFF(model::ModelMetadata, architecture) OFF(model::ModelMetadata, version)
  OFF(model::ModelMetadata, vocab_size) OFF(model::ModelMetadata, hidden_size) OFF(model::ModelMetadata, num_layers)
  OFF(model::ModelMetadata, num_heads) OFF(model::ModelMetadata, intermediate_size)
  OFF(model::ModelMetadata, rope_theta) OFF(model::ModelMetadata, extra_params)
  OFF(optimize::QuantizationConfig, type) OFF(optimize::QuantizationConfig, symmetric)
  OFF(optimize::QuantizationConfig, per_channel) OFF(optimize::QuantizationConfig, calibration_ratio)
  OFF(optimize::QuantizationConfig, calibration_dataset)
  OFF(optimize::QuantizationInfo, type) OFF(optimize::QuantizationInfo, scales) OFF(optimize::QuantizationInfo, zero_points)
  OFF(optimize::QuantizationInfo, original_size_bytes) OFF(optimize::QuantizationInfo, quantized_size_bytes)
  OFF(optimize::QuantizationInfo, compression_ratio)
  return 0;
}
