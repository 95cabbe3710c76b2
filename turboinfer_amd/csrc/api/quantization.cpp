// quantization.cpp -- turboinfer::optimize::Quantizer (host weight ingestion).
// Arithmetic of the reference's src/optimize/quantization.cpp (:36-118 tensor / model
// quantization, :335-394 calculate_quantization_info, :662-713 the element kernels);
// compiled with -ffp-contract=off so x / s + zp rounds exactly like the reference build.
#include "turboinfer/optimize/quantization.hpp"

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <fstream>
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
                           ": not built in this MI355X decode-path library (SURVEY.md 8(f) rank 3)");
}

// ------------------------------------------------------------------ TINQ file format
// The reference's quantized-model file (quantization.cpp:120-333, write_string / read_string
// :716-735): little-endian host-order fields, written field by field.
template <class T>
void put(std::ofstream& f, const T& v) {
  f.write(reinterpret_cast<const char*>(&v), sizeof(T));
}
template <class T>
T get(std::ifstream& f) {
  T v{};
  f.read(reinterpret_cast<char*>(&v), sizeof(T));
  return v;
}
void put_string(std::ofstream& f, const std::string& s) {
  put<uint32_t>(f, (uint32_t)s.size());
  if (!s.empty()) f.write(s.data(), (std::streamsize)s.size());
}
std::string get_string(std::ifstream& f) {
  const uint32_t n = get<uint32_t>(f);
  std::string s(n, '\0');
  if (n) f.read(&s[0], n);
  return s;
}

// calculate_quantization_info_for_saved_tensor (quantization.cpp:737-817): the per-file
// scale / zero point the reference records for an int8 or int4-in-int32 tensor.
QuantizationInfo saved_tensor_info(const core::Tensor& t, QuantizationType type) {
  QuantizationInfo info;
  info.type = type;
  info.quantized_size_bytes = t.byte_size();
  const size_t n = t.shape().total_size();
  if (t.dtype() == core::DataType::kInt8 || t.dtype() == core::DataType::kInt32) {
    info.original_size_bytes = n * sizeof(float);
    info.compression_ratio = (float)info.original_size_bytes / (float)info.quantized_size_bytes;
    const bool i8 = t.dtype() == core::DataType::kInt8;
    if (n > 0) {
      int32_t mn, mx;
      if (i8) {
        const int8_t* d = t.data_ptr<int8_t>();
        int8_t a = d[0], b = d[0];
        for (size_t i = 1; i < n; ++i) {
          a = std::min(a, d[i]);
          b = std::max(b, d[i]);
        }
        mn = a;
        mx = b;
      } else {
        const int32_t* d = t.data_ptr<int32_t>();
        mn = d[0];
        mx = d[0];
        for (size_t i = 1; i < n; ++i) {
          mn = std::min(mn, d[i]);
          mx = std::max(mx, d[i]);
        }
        mn = std::max(mn, (int32_t)-8);
        mx = std::min(mx, (int32_t)7);
      }
      const float range = (float)(mx - mn);
      if (range > 0) {
        info.scales.push_back(range / (i8 ? 255.0f : 15.0f));
        info.zero_points.push_back((float)(-mn));
      } else {
        info.scales.push_back(i8 ? 1.0f / 127.0f : 1.0f / 7.0f);
        info.zero_points.push_back(0.0f);
      }
    } else {
      info.scales.push_back(i8 ? 1.0f / 127.0f : 1.0f / 7.0f);
      info.zero_points.push_back(0.0f);
    }
  } else {
    info.original_size_bytes = t.byte_size();
    info.compression_ratio = 1.0f;
  }
  return info;
}
}  // namespace

// (the reference's pimpl, kept for its class layout; this Quantizer needs no state beyond config_)
class QuantizerImpl {};
static_assert(sizeof(Quantizer) == 56, "reference layout (LP64)");

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

// save_quantized_model (quantization.cpp:120-211): the same bytes as the reference for the
// same ModelData (tensors in the container's iteration order).
void Quantizer::save_quantized_model(const model::ModelData& m, const std::string& path) {
  std::ofstream f(path, std::ios::binary);
  if (!f.is_open()) throw std::runtime_error("Failed to open file for writing: " + path);
  try {
    put<uint32_t>(f, 0x54494E51u);   // "TINQ"
    put<uint32_t>(f, 1u);
    put(f, config_.type);
    put(f, config_.symmetric);
    put(f, config_.per_channel);
    const auto& md = m.metadata();
    put_string(f, md.name);
    put_string(f, md.architecture);
    put_string(f, md.version);
    put(f, md.vocab_size);
    put(f, md.hidden_size);
    put(f, md.num_layers);
    put(f, md.num_heads);
    put(f, md.intermediate_size);
    put(f, md.rope_theta);
    const auto names = m.tensor_names();
    put<uint32_t>(f, (uint32_t)names.size());
    for (const auto& name : names) {
      const core::Tensor* t = m.get_tensor(name);
      if (!t) continue;
      put_string(f, name);
      put<uint32_t>(f, (uint32_t)t->dtype());
      put<uint32_t>(f, (uint32_t)t->shape().ndim());
      for (size_t i = 0; i < t->shape().ndim(); ++i) put<uint64_t>(f, (uint64_t)t->shape().size(i));
      const size_t bytes = t->byte_size();
      put(f, bytes);
      f.write(static_cast<const char*>(t->data()), (std::streamsize)bytes);
      if (t->dtype() == core::DataType::kInt8 || t->dtype() == core::DataType::kInt32) {
        const QuantizationInfo qi = saved_tensor_info(*t, config_.type);
        put<uint32_t>(f, (uint32_t)qi.scales.size());
        if (!qi.scales.empty()) f.write(reinterpret_cast<const char*>(qi.scales.data()), qi.scales.size() * sizeof(float));
        put<uint32_t>(f, (uint32_t)qi.zero_points.size());
        if (!qi.zero_points.empty())
          f.write(reinterpret_cast<const char*>(qi.zero_points.data()), qi.zero_points.size() * sizeof(float));
        put(f, qi.original_size_bytes);
        put(f, qi.quantized_size_bytes);
        put(f, qi.compression_ratio);
      }
    }
  } catch (const std::exception& e) {
    throw std::runtime_error("Failed to save quantized model: " + std::string(e.what()));
  }
}

// load_quantized_model (quantization.cpp:213-333): metadata and tensors back into a
// ModelData; the recorded scales are read past (the reference keeps them nowhere either).
// The int8 / int32 tensors then reach the engine with unit scale, the reference's raw cast.
model::ModelData Quantizer::load_quantized_model(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f.is_open()) throw std::runtime_error("Failed to open file for reading: " + path);
  try {
    if (get<uint32_t>(f) != 0x54494E51u) throw std::runtime_error("Invalid file format - not a TurboInfer quantized model");
    const uint32_t version = get<uint32_t>(f);
    if (version != 1) throw std::runtime_error("Unsupported quantized model version: " + std::to_string(version));
    (void)get<QuantizationType>(f);
    (void)get<bool>(f);
    (void)get<bool>(f);
    model::ModelData m;
    auto& md = m.metadata();
    md.name = get_string(f);
    md.architecture = get_string(f);
    md.version = get_string(f);
    md.vocab_size = get<size_t>(f);
    md.hidden_size = get<size_t>(f);
    md.num_layers = get<size_t>(f);
    md.num_heads = get<size_t>(f);
    md.intermediate_size = get<size_t>(f);
    md.rope_theta = get<float>(f);
    const uint32_t count = get<uint32_t>(f);
    for (uint32_t i = 0; i < count; ++i) {
      const std::string name = get_string(f);
      const auto dtype = (core::DataType)get<uint32_t>(f);
      const uint32_t nd = get<uint32_t>(f);
      if (!f || nd > 8) throw std::runtime_error("corrupt tensor header for: " + name);
      std::vector<size_t> dims(nd);
      for (auto& d : dims) d = (size_t)get<uint64_t>(f);
      core::Tensor t{core::TensorShape(dims), dtype};
      const size_t bytes = get<size_t>(f);
      if (bytes != t.byte_size()) throw std::runtime_error("Tensor size mismatch for: " + name);
      f.read(static_cast<char*>(t.data()), (std::streamsize)bytes);
      if (dtype == core::DataType::kInt8 || dtype == core::DataType::kInt32) {
        const uint32_t ns = get<uint32_t>(f);
        f.seekg((std::streamoff)ns * 4, std::ios::cur);
        const uint32_t nz = get<uint32_t>(f);
        f.seekg((std::streamoff)nz * 4, std::ios::cur);
        (void)get<size_t>(f);
        (void)get<size_t>(f);
        (void)get<float>(f);
      }
      if (!f) throw std::runtime_error("truncated file at tensor: " + name);
      m.add_tensor(name, std::move(t));
    }
    return m;
  } catch (const std::exception& e) {
    throw std::runtime_error("Failed to load quantized model: " + std::string(e.what()));
  }
}

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
