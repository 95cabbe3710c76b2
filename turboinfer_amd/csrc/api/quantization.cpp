// quantization.cpp -- turboinfer::optimize::Quantizer (host weight ingestion).
// Arithmetic of the reference's src/optimize/quantization.cpp (:36-118 tensor / model
// quantization, :335-394 calculate_quantization_info, :662-713 the element kernels);
// compiled with -ffp-contract=off so x / s + zp rounds exactly like the reference build.
#include "turboinfer/optimize/quantization.hpp"

#include <cmath>
#include <stdexcept>

namespace turboinfer {
namespace optimize {

namespace {
// std::max(lo, std::min(hi, v)) with the std operand order (a NaN lands on hi, then lo).
inline float clamp_ref(float v, float lo, float hi) {
  const float t = (v < hi) ? v : hi;   // std::min(hi, v)
  return (lo < t) ? t : lo;            // std::max(lo, t)
}
[[noreturn]] void file_off_path(const char* what) {
  throw std::runtime_error(std::string("Quantizer::") + what +
                           ": the TINQ file format is not built in this MI355X decode-path library "
                           "(SURVEY.md 8(f) rank 3)");
}
}  // namespace

Quantizer::Quantizer(const QuantizationConfig& config) : config_(config) {}
Quantizer::~Quantizer() = default;
void Quantizer::set_config(const QuantizationConfig& config) { config_ = config; }

QuantizationInfo Quantizer::calculate_quantization_info(const core::Tensor& input) {
  QuantizationInfo info;
  info.type = config_.type;
  info.original_size_bytes = input.byte_size();
  const size_t n = input.shape().total_size();
  const float* x = static_cast<const float*>(input.data());
  if (!x || n == 0) throw std::runtime_error("calculate_quantization_info: empty tensor");
  float mn = x[0], mx = x[0];
  for (size_t i = 1; i < n; ++i) {
    mn = (x[i] < mn) ? x[i] : mn;
    mx = (mx < x[i]) ? x[i] : mx;
  }
  const float amn = std::fabs(mn), amx = std::fabs(mx);
  const float absmax = (amn < amx) ? amx : amn;
  if (config_.type == QuantizationType::kInt8 || config_.type == QuantizationType::kInt4) {
    const bool i8 = config_.type == QuantizationType::kInt8;
    float scale, zp;
    if (config_.symmetric) {
      scale = absmax / (i8 ? 127.0f : 7.0f);
      zp = 0.0f;
    } else {
      scale = (mx - mn) / (i8 ? 255.0f : 15.0f);
      zp = -mn / scale;
    }
    info.scales = {scale};
    info.zero_points = {zp};
    info.quantized_size_bytes = i8 ? n : (n + 1) / 2;
    info.compression_ratio = (float)info.original_size_bytes / (float)info.quantized_size_bytes;
  } else {
    info.quantized_size_bytes = info.original_size_bytes;
    info.compression_ratio = 1.0f;
  }
  return info;
}

core::Tensor Quantizer::quantize_tensor(const core::Tensor& input) {
  if (config_.type == QuantizationType::kNone) return input;
  const QuantizationInfo info = calculate_quantization_info(input);
  const size_t n = input.shape().total_size();
  const float* x = static_cast<const float*>(input.data());
  if (config_.type == QuantizationType::kInt8) {
    core::Tensor q(input.shape(), core::DataType::kInt8);
    quantize_to_int8(x, q.data_ptr<int8_t>(), n, info);
    return q;
  }
  if (config_.type == QuantizationType::kInt4) {
    core::Tensor q(input.shape(), core::DataType::kInt32);   // int4 values held unpacked, as in the reference
    quantize_to_int4(x, q.data_ptr<int32_t>(), n, info);
    return q;
  }
  throw std::runtime_error("Unsupported quantization type");
}

core::Tensor Quantizer::dequantize_tensor(const core::Tensor& quantized, const QuantizationInfo& info) {
  if (info.type == QuantizationType::kNone) return quantized;
  core::Tensor y(quantized.shape(), core::DataType::kFloat32);
  const size_t n = quantized.shape().total_size();
  if (info.type == QuantizationType::kInt8) {
    dequantize_from_int8(quantized.data_ptr<int8_t>(), y.data_ptr<float>(), n, info);
  } else if (info.type == QuantizationType::kInt4) {
    dequantize_from_int4(quantized.data_ptr<int32_t>(), y.data_ptr<float>(), n, info);
  } else {
    throw std::runtime_error("Unsupported quantization type for dequantization");
  }
  return y;
}

model::ModelData Quantizer::quantize_model(const model::ModelData& model_data) {
  model::ModelData out;
  out.metadata() = model_data.metadata();
  for (const auto& name : model_data.tensor_names()) {
    const core::Tensor* t = model_data.get_tensor(name);
    if (!t) continue;
    if (t->dtype() == core::DataType::kFloat32) {
      try {
        out.add_tensor(name, quantize_tensor(*t));
      } catch (const std::exception&) {
        out.add_tensor(name, *t);   // a tensor that cannot be quantized is kept as is
      }
    } else {
      out.add_tensor(name, *t);
    }
  }
  return out;
}

void Quantizer::save_quantized_model(const model::ModelData&, const std::string&) { file_off_path("save_quantized_model"); }
model::ModelData Quantizer::load_quantized_model(const std::string&) { file_off_path("load_quantized_model"); }

float Quantizer::estimate_compression_ratio(const model::ModelData& model_data) {
  if (model_data.num_tensors() == 0) return 1.0f;
  size_t orig = 0, comp = 0;
  for (const auto& name : model_data.tensor_names()) {
    const core::Tensor* t = model_data.get_tensor(name);
    if (!t) continue;
    size_t n = 1;
    for (size_t d : t->shape().dimensions()) n *= d;
    orig += n * sizeof(float);
    switch (config_.type) {
      case QuantizationType::kInt4: comp += (n + 1) / 2; break;
      case QuantizationType::kInt8: comp += n; break;
      case QuantizationType::kFloat16: comp += n * 2; break;
      case QuantizationType::kNone: comp += n * sizeof(float); break;
    }
    if (config_.type != QuantizationType::kNone) comp += sizeof(float) + sizeof(int32_t);
  }
  return orig == 0 ? 1.0f : (float)orig / (float)comp;
}

float Quantizer::validate_quantization_accuracy(const model::ModelData& original_model,
                                                const model::ModelData& quantized_model,
                                                const std::vector<core::Tensor>& test_inputs) {
  if (original_model.num_tensors() == 0 || quantized_model.num_tensors() == 0) return 0.0f;
  if (!test_inputs.empty())
    throw std::runtime_error("Quantizer::validate_quantization_accuracy: inference-based validation needs "
                             "prefill (SURVEY.md 8(f)); pass no test inputs for the element-wise form");
  float total = 0.0f;
  size_t count = 0;
  for (const auto& name : original_model.tensor_names()) {
    const core::Tensor* a = original_model.get_tensor(name);
    const core::Tensor* b = quantized_model.get_tensor(name);
    if (!a || !b || a->shape() != b->shape()) continue;
    const size_t n = a->shape().total_size();
    const float* pa = a->data_ptr<float>();
    const float* pb = b->data_ptr<float>();
    for (size_t i = 0; i < n; ++i) {
      const float err = std::fabs(pa[i] - pb[i]);
      total += (pa[i] != 0.0f) ? err / std::fabs(pa[i]) : err;
    }
    count += n;
  }
  return count ? total / count : 0.0f;
}

const char* quantization_type_to_string(QuantizationType type) {
  switch (type) {
    case QuantizationType::kInt8: return "int8";
    case QuantizationType::kInt4: return "int4";
    case QuantizationType::kFloat16: return "float16";
    case QuantizationType::kNone: return "none";
  }
  return "unknown";
}

size_t get_quantization_bits(QuantizationType type) {
  switch (type) {
    case QuantizationType::kInt8: return 8;
    case QuantizationType::kInt4: return 4;
    case QuantizationType::kFloat16: return 16;
    case QuantizationType::kNone: return 32;
  }
  return 0;
}

float calculate_theoretical_compression(core::DataType from_type, QuantizationType to_type) {
  return (float)(core::get_dtype_size(from_type) * 8) / (float)get_quantization_bits(to_type);
}

void quantize_model_file(const std::string&, const std::string&, const QuantizationConfig&) {
  file_off_path("quantize_model_file");
}

void quantize_to_int8(const float* input, int8_t* output, size_t count, const QuantizationInfo& info) {
  const float s = info.scales.at(0), zp = info.zero_points.at(0);
  for (size_t i = 0; i < count; ++i) output[i] = (int8_t)clamp_ref(std::round(input[i] / s + zp), -128.0f, 127.0f);
}

void quantize_to_int4(const float* input, int32_t* output, size_t count, const QuantizationInfo& info) {
  const float s = info.scales.at(0), zp = info.zero_points.at(0);
  for (size_t i = 0; i < count; ++i) {
    const float v = std::round(input[i] / s - zp);
    output[i] = (int32_t)(zp == 0.0f ? clamp_ref(v, -7.0f, 7.0f) : clamp_ref(v, 0.0f, 15.0f));
  }
}

void dequantize_from_int8(const int8_t* input, float* output, size_t count, const QuantizationInfo& info) {
  const float s = info.scales.at(0), zp = info.zero_points.at(0);
  for (size_t i = 0; i < count; ++i) output[i] = s * ((float)input[i] - zp);
}

void dequantize_from_int4(const int32_t* input, float* output, size_t count, const QuantizationInfo& info) {
  const float s = info.scales.at(0), zp = info.zero_points.at(0);
  for (size_t i = 0; i < count; ++i) output[i] = s * ((float)input[i] + zp);
}

}  // namespace optimize
}  // namespace turboinfer
