// turboinfer/model/model_loader.hpp -- model containers of the drop-in C++ API.
//
// ModelMetadata and ModelData keep the reference's names and semantics
// (include/turboinfer/model/model_loader.hpp:35-153 there): a name -> Tensor map plus the
// architecture numbers InferenceEngine is built from.  File ingestion (ModelLoader: GGUF,
// SafeTensors, PyTorch, ONNX) is weight loading, ranked 3rd in SURVEY.md 8(f): the loader
// entry points exist and throw std::runtime_error until that row is built.
#pragma once

#include <cstddef>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "../core/tensor.hpp"

namespace turboinfer {
namespace model {

enum class ModelFormat {
  kGGUF,
  kSafeTensors,
  kPyTorch,
  kONNX,
  kAuto
};

struct ModelMetadata {
  std::string name;
  std::string architecture;
  std::string version;
  size_t vocab_size = 0;
  size_t hidden_size = 0;
  size_t num_layers = 0;
  size_t num_heads = 0;
  size_t intermediate_size = 0;
  float rope_theta = 10000.0f;
  std::unordered_map<std::string, std::string> extra_params;
};

class ModelData {
 public:
  ModelData() = default;

  const ModelMetadata& metadata() const noexcept { return metadata_; }
  ModelMetadata& metadata() noexcept { return metadata_; }

  const core::Tensor* get_tensor(const std::string& name) const;
  core::Tensor* get_tensor(const std::string& name);
  void add_tensor(const std::string& name, core::Tensor tensor);
  std::vector<std::string> tensor_names() const;
  size_t num_tensors() const noexcept { return tensors_.size(); }
  bool has_tensor(const std::string& name) const;
  size_t total_memory_usage() const;
  std::string get_model_summary() const;
  bool validate() const;
  std::string get_memory_usage_string() const;
  void set_config_param(const std::string& key, const std::string& value);
  std::string get_config_param(const std::string& key, const std::string& default_value = "") const;

 private:
  ModelMetadata metadata_;
  std::unordered_map<std::string, core::Tensor> tensors_;
};

class ModelLoader {
 public:
  static ModelData load(const std::string& file_path);
  static ModelData load(const std::string& file_path, ModelFormat format);
  static ModelFormat detect_format(const std::string& file_path);
  static bool validate_file(const std::string& file_path);
  static ModelMetadata get_model_info(const std::string& file_path);
  static bool validate_model(const ModelData& model_data, const ModelMetadata& metadata);

 private:
  // GGUF v3 (reference model_loader.hpp:216); turboinfer_amd/csrc/api/gguf.cpp
  static ModelData load_gguf(const std::string& file_path);
};

const char* format_to_string(ModelFormat format);
const char* format_to_extension(ModelFormat format);
bool has_valid_model_extension(const std::string& file_path);

}  // namespace model
}  // namespace turboinfer
