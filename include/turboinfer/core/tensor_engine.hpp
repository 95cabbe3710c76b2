// turboinfer/core/tensor_engine.hpp -- the drop-in TensorEngine on MI355X.
//
// Same class, enum and method names as the reference's turboinfer::core::TensorEngine
// (include/turboinfer/core/tensor_engine.hpp:42-264 there).  The decode-path ops run on the
// GPU through the C-ABI of include/ti_hip.h (fp32 op-level kernels: matmul, rms_norm,
// apply_rope, silu, relu, add, multiply, softmax, attention); each call uploads its
// operands, launches on the engine's HIP stream and returns a host Tensor, as the
// reference's ops return new tensors by value.
//
// Device policy: this library is built for gfx950 only.  kGPU and kAuto bind the GPU and
// throw std::runtime_error when no MI355X is visible; kCPU throws (the CPU path is the
// reference itself -- there is no CPU fallback here).  Operations outside the decode hot
// path (batch_matmul, gelu, layer_norm, concatenate, split, transpose, permute, add_bias,
// scale) throw std::runtime_error naming SURVEY.md 8(f).  attention / multi_head_attention take
// any query length and an optional float mask (the reference's sequence, on the device).
#pragma once

#include <cstddef>
#include <memory>
#include <string>
#include <vector>

#include "tensor.hpp"

namespace turboinfer {
namespace core {

enum class ComputeDevice {
  kCPU,
  kGPU,
  kAuto
};

class TensorEngine {
 public:
  explicit TensorEngine(ComputeDevice device = ComputeDevice::kAuto);
  ~TensorEngine();
  TensorEngine(const TensorEngine&) = delete;
  TensorEngine& operator=(const TensorEngine&) = delete;

  ComputeDevice device() const noexcept { return device_; }
  /// True when a gfx950 (MI355X) device is visible.
  bool gpu_available() const noexcept;
  std::string device_info() const;

  /// [M,K] x [K,N] -> [M,N];  [B,S,K] x [K,N] -> [B,S,N]  (fp32; k-ascending fma chain).
  Tensor matmul(const Tensor& a, const Tensor& b);
  Tensor batch_matmul(const Tensor& a, const Tensor& b);
  Tensor add_bias(const Tensor& input, const Tensor& bias);
  Tensor relu(const Tensor& input);
  Tensor gelu(const Tensor& input);
  Tensor silu(const Tensor& input);
  /// Row softmax over the last dimension with temperature.
  Tensor softmax(const Tensor& input, float temperature = 1.0f);
  /// Attention: query [B,Sq,D], key/value [B,S,D], optional float mask added to the scores
  /// (Sq == 1 without a mask is attention_fast_incremental).
  Tensor attention(const Tensor& query, const Tensor& key, const Tensor& value, const Tensor* mask = nullptr);
  Tensor attention_fast_incremental(const Tensor& query, const Tensor& key, const Tensor& value,
                                    const Tensor* mask = nullptr);
  /// query [B,Sq,H] (any Sq), key/value [B,S,H] with num_heads heads of H/num_heads interleaved
  /// in H, optional float mask [B,Sq,S] (0 = masked, the reference's -1e9 fill).
  Tensor multi_head_attention(const Tensor& query, const Tensor& key, const Tensor& value, size_t num_heads,
                              const Tensor* mask = nullptr);
  Tensor layer_norm(const Tensor& input, const Tensor& weight, const Tensor& bias, float eps = 1e-5f);
  /// x / sqrt(mean(x^2) + eps) * weight over the last dimension.
  Tensor rms_norm(const Tensor& input, const Tensor& weight, float eps = 1e-5f);
  /// Interleaved-pair RoPE of a [B,S,D] or [B,heads,S,D] input; position_ids fp32 [S] or [B,S].
  Tensor apply_rope(const Tensor& input, const Tensor& position_ids, float rope_theta = 10000.0f);
  Tensor add(const Tensor& a, const Tensor& b);
  Tensor multiply(const Tensor& a, const Tensor& b);
  Tensor scale(const Tensor& input, float scale);
  Tensor concatenate(const std::vector<Tensor>& tensors, size_t dim);
  std::vector<Tensor> split(const Tensor& input, const std::vector<size_t>& split_sizes, size_t dim);
  Tensor transpose(const Tensor& input);
  Tensor permute(const Tensor& input, const std::vector<size_t>& dims);

 private:
  ComputeDevice device_;
  std::unique_ptr<class TensorEngineImpl> impl_;
};

const char* device_to_string(ComputeDevice device);

}  // namespace core
}  // namespace turboinfer
