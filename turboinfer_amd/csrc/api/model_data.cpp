// model_data.cpp -- turboinfer::model::ModelData (name -> Tensor container) and the
// ModelLoader entry points.  Container semantics follow the reference's
// src/model/model_loader.cpp:186-311; file parsing is SURVEY.md 8(f) rank 3 (not built).
#include <algorithm>
#include <fstream>
#include <sstream>
#include <stdexcept>

#include "turboinfer/model/model_loader.hpp"

namespace turboinfer {
namespace model {

const core::Tensor* ModelData::get_tensor(const std::string& name) const {
  auto it = tensors_.find(name);
  return it == tensors_.end() ? nullptr : &it->second;
}

core::Tensor* ModelData::get_tensor(const std::string& name) {
  auto it = tensors_.find(name);
  return it == tensors_.end() ? nullptr : &it->second;
}

void ModelData::add_tensor(const std::string& name, core::Tensor tensor) { tensors_[name] = std::move(tensor); }

std::vector<std::string> ModelData::tensor_names() const {
  std::vector<std::string> names;
  names.reserve(tensors_.size());
  for (const auto& kv : tensors_) names.push_back(kv.first);
  return names;
}

bool ModelData::has_tensor(const std::string& name) const { return tensors_.count(name) != 0; }

size_t ModelData::total_memory_usage() const {
  size_t total = 0;
  for (const auto& kv : tensors_) total += kv.second.byte_size();
  return total;
}

std::string ModelData::get_memory_usage_string() const {
  const double b = (double)total_memory_usage();
  std::ostringstream os;
  os.setf(std::ios::fixed);
  os.precision(2);
  if (b >= 1024.0 * 1024.0 * 1024.0) os << b / (1024.0 * 1024.0 * 1024.0) << " GB";
  else if (b >= 1024.0 * 1024.0) os << b / (1024.0 * 1024.0) << " MB";
  else if (b >= 1024.0) os << b / 1024.0 << " KB";
  else os << (size_t)b << " bytes";
  return os.str();
}

std::string ModelData::get_model_summary() const {
  std::ostringstream os;
  os << "Model: " << metadata_.name << " (" << metadata_.architecture << ")\n"
     << "  vocab " << metadata_.vocab_size << ", hidden " << metadata_.hidden_size << ", layers "
     << metadata_.num_layers << ", heads " << metadata_.num_heads << ", intermediate " << metadata_.intermediate_size
     << ", rope_theta " << metadata_.rope_theta << "\n"
     << "  tensors " << tensors_.size() << ", " << get_memory_usage_string();
  return os.str();
}

bool ModelData::validate() const {
  if (metadata_.name.empty() || metadata_.architecture.empty() || tensors_.empty()) return false;
  for (const auto& kv : tensors_) {
    const auto& d = kv.second.shape().dimensions();
    if (d.empty() || std::find(d.begin(), d.end(), size_t(0)) != d.end()) return false;
  }
  if (metadata_.vocab_size > 1000000 || metadata_.hidden_size > 32768) return false;
  return true;
}

void ModelData::set_config_param(const std::string& key, const std::string& value) {
  metadata_.extra_params[key] = value;
}

std::string ModelData::get_config_param(const std::string& key, const std::string& default_value) const {
  auto it = metadata_.extra_params.find(key);
  return it == metadata_.extra_params.end() ? default_value : it->second;
}

namespace {
[[noreturn]] void loader_off_path(const std::string& what) {
  throw std::runtime_error("ModelLoader::" + what +
                           ": checkpoint ingestion is not built in this MI355X decode-path library "
                           "(SURVEY.md 8(f) rank 3); build a ModelData in memory instead");
}
bool ends_with(const std::string& s, const std::string& suffix) {
  return s.size() >= suffix.size() && s.compare(s.size() - suffix.size(), suffix.size(), suffix) == 0;
}
}  // namespace

// load (reference model_loader.cpp load/:load(path, format)): GGUF is read (gguf.cpp); the
// other formats stay outside this library.
ModelData ModelLoader::load(const std::string& file_path) { return load(file_path, detect_format(file_path)); }
ModelData ModelLoader::load(const std::string& file_path, ModelFormat format) {
  if (format == ModelFormat::kGGUF) return load_gguf(file_path);
  loader_off_path("load(" + file_path + ")");
}
// get_model_info (reference model_loader.cpp:596-633): for GGUF the header is checked and the
// reference's fixed defaults are returned (it does not parse the key/value pairs there).
ModelMetadata ModelLoader::get_model_info(const std::string& file_path) {
  if (detect_format(file_path) != ModelFormat::kGGUF) loader_off_path("get_model_info(" + file_path + ")");
  std::ifstream f(file_path, std::ios::binary);
  if (!f.is_open()) throw std::runtime_error("Failed to extract model metadata: Could not open GGUF file for metadata reading");
  char magic[4] = {0, 0, 0, 0};
  uint32_t version = 0;
  f.read(magic, 4);
  f.read(reinterpret_cast<char*>(&version), 4);
  if (std::string(magic, 4) != "GGUF") throw std::runtime_error("Failed to extract model metadata: Invalid GGUF magic number");
  ModelMetadata m;
  const std::string base = file_path.substr(file_path.find_last_of('/') + 1);
  m.name = base.substr(0, base.rfind('.'));
  m.architecture = "GGUF";
  m.version = std::to_string(version);
  m.vocab_size = 32000;
  m.hidden_size = 4096;
  m.num_layers = 32;
  m.num_heads = 32;
  m.intermediate_size = 11008;
  m.rope_theta = 10000.0f;
  return m;
}

ModelFormat ModelLoader::detect_format(const std::string& file_path) {
  if (ends_with(file_path, ".gguf")) return ModelFormat::kGGUF;
  if (ends_with(file_path, ".safetensors")) return ModelFormat::kSafeTensors;
  if (ends_with(file_path, ".pt") || ends_with(file_path, ".pth")) return ModelFormat::kPyTorch;
  if (ends_with(file_path, ".onnx")) return ModelFormat::kONNX;
  throw std::runtime_error("Unknown model format: " + file_path);
}

bool ModelLoader::validate_file(const std::string& file_path) { return has_valid_model_extension(file_path); }

bool ModelLoader::validate_model(const ModelData& model_data, const ModelMetadata& metadata) {
  const ModelMetadata& m = model_data.metadata();
  return model_data.validate() && m.vocab_size == metadata.vocab_size && m.hidden_size == metadata.hidden_size &&
         m.num_layers == metadata.num_layers && m.num_heads == metadata.num_heads;
}

const char* format_to_string(ModelFormat format) {
  switch (format) {
    case ModelFormat::kGGUF: return "GGUF";
    case ModelFormat::kSafeTensors: return "SafeTensors";
    case ModelFormat::kPyTorch: return "PyTorch";
    case ModelFormat::kONNX: return "ONNX";
    case ModelFormat::kAuto: return "Auto";
  }
  return "Unknown";
}

const char* format_to_extension(ModelFormat format) {
  switch (format) {
    case ModelFormat::kGGUF: return ".gguf";
    case ModelFormat::kSafeTensors: return ".safetensors";
    case ModelFormat::kPyTorch: return ".pt";
    case ModelFormat::kONNX: return ".onnx";
    case ModelFormat::kAuto: return "";
  }
  return "";
}

bool has_valid_model_extension(const std::string& file_path) {
  for (const char* ext : {".gguf", ".safetensors", ".pt", ".pth", ".onnx"})
    if (ends_with(file_path, ext)) return true;
  return false;
}

}  // namespace model
}  // namespace turboinfer
