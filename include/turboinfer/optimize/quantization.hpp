// turboinfer/optimize/quantization.hpp -- the drop-in Quantizer.
//
// Names, fields and arithmetic of the reference's turboinfer::optimize API
// (include/turboinfer/optimize/quantization.hpp:94-135, 244-271 there;
// src/optimize/quantization.cpp:36-118, 335-394, 662-713): per-tensor symmetric or
// asymmetric INT8 / INT4 (INT4 held unpacked in int32), round-half-away-from-zero, the
// reference's clamping.  These are host-side weight-ingestion routines; the MI355X decode
// path re-packs the result into group-128 device tiles (include/ti_hip.h ti_wpack_host)
// when an InferenceEngine is built.  The TINQ file format (save/load) is SURVEY.md 8(f)
// rank 3 and throws.
#pragma once

#include <cstddef>
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "../core/tensor.hpp"
#include "../model/model_loader.hpp"

namespace turboinfer {
namespace optimize {

enum class QuantizationType {
  kInt8,
  kInt4,
  kFloat16,
  kNone
};

struct QuantizationConfig {
  QuantizationType type = QuantizationType::kInt8;
  bool symmetric = true;
  bool per_channel = true;
  float calibration_ratio = 0.1f;
  std::string calibration_dataset;
};

struct QuantizationInfo {
  QuantizationType type = QuantizationType::kNone;
  std::vector<float> scales;
  std::vector<float> zero_points;
  size_t original_size_bytes = 0;
  size_t quantized_size_bytes = 0;
  float compression_ratio = 1.0f;
};

class Quantizer {
 public:
  explicit Quantizer(const QuantizationConfig& config = QuantizationConfig{});
  ~Quantizer();

  const QuantizationConfig& config() const noexcept { return config_; }
  void set_config(const QuantizationConfig& config);

  core::Tensor quantize_tensor(const core::Tensor& input);
  core::Tensor dequantize_tensor(const core::Tensor& quantized, const QuantizationInfo& info);
  model::ModelData quantize_model(const model::ModelData& model_data);
  void save_quantized_model(const model::ModelData& quantized_model, const std::string& output_path);
  static model::ModelData load_quantized_model(const std::string& model_path);
  QuantizationInfo calculate_quantization_info(const core::Tensor& input);
  float estimate_compression_ratio(const model::ModelData& model_data);
  float validate_quantization_accuracy(const model::ModelData& original_model,
                                       const model::ModelData& quantized_model,
                                       const std::vector<core::Tensor>& test_inputs);

 private:
  QuantizationConfig config_;
  std::unique_ptr<class QuantizerImpl> impl_;   ///< (layout of the reference's class; unused here)
};

const char* quantization_type_to_string(QuantizationType type);
size_t get_quantization_bits(QuantizationType type);
float calculate_theoretical_compression(core::DataType from_type, QuantizationType to_type);
void quantize_model_file(const std::string& input_path, const std::string& output_path,
                         const QuantizationConfig& config = QuantizationConfig{});

void quantize_to_int8(const float* input, int8_t* output, size_t count, const QuantizationInfo& info);
void quantize_to_int4(const float* input, int32_t* output, size_t count, const QuantizationInfo& info);
void dequantize_from_int8(const int8_t* input, float* output, size_t count, const QuantizationInfo& info);
void dequantize_from_int4(const int32_t* input, float* output, size_t count, const QuantizationInfo& info);

}  // namespace optimize
}  // namespace turboinfer
