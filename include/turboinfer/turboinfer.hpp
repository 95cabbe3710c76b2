// turboinfer/turboinfer.hpp -- umbrella header of the drop-in C++ API (MI355X build).
//
// Mirrors the reference's include/turboinfer/turboinfer.hpp: the core / model / optimize
// headers, version and library init functions, and the short aliases.  The logging and
// profiler utilities (util/) are outside the decode hot path and not part of this build.
#pragma once

#include <cstddef>
#include <string>
#include <vector>

#include "core/tensor.hpp"
#include "core/tensor_engine.hpp"
#include "model/inference_engine.hpp"
#include "model/model_loader.hpp"
#include "optimize/quantization.hpp"

// The reference's umbrella header also pulls in util/profiler.hpp, hence <chrono>; reference
// programs rely on that transitively (tests/test_inference_engine.cpp, examples/basic_inference.cpp).
#include <chrono>

namespace turboinfer {

struct Version {
  static constexpr int kMajor = 1;
  static constexpr int kMinor = 0;
  static constexpr int kPatch = 0;
  static constexpr const char* kString = "1.0.0";
};

inline const char* version() { return Version::kString; }
/// Build description: gfx950 kernels, HIP runtime version, visible devices.
const char* build_info();
/// Binds the first visible MI355X; false when none is visible.
bool initialize(bool enable_logging = true);
void shutdown();
bool is_initialized();

using Tensor = core::Tensor;
using TensorShape = core::TensorShape;
using TensorEngine = core::TensorEngine;
using ModelData = model::ModelData;
using ModelLoader = model::ModelLoader;
using InferenceEngine = model::InferenceEngine;
using InferenceConfig = model::InferenceConfig;
using GenerationResult = model::GenerationResult;

inline ModelData load_model(const std::string& file_path) { return ModelLoader::load(file_path); }
std::vector<int> tokenize(const std::string& text, const std::string& model_path);
std::string detokenize(const std::vector<int>& tokens, const std::string& model_path);
inline std::string generate_text(const std::string& model_path, const std::string& prompt, size_t max_tokens = 50,
                                 float temperature = 1.0f) {
  return model::quick_generate(model_path, prompt, max_tokens, temperature);
}

}  // namespace turboinfer
