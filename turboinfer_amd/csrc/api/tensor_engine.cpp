// tensor_engine.cpp -- turboinfer::core::TensorEngine on MI355X through include/ti_hip.h.
//
// Every op: host checks with the reference's exception types (tensor_engine.cpp:490-528,
// 1452-1467, 1510-1540 in the reference), operands converted to fp32 like the reference's
// convert_dtype (:2218-2284: integer weights are a raw cast), upload, one gfx950 kernel on
// the engine stream, download.  No CPU arithmetic path exists.
#include "turboinfer/core/tensor_engine.hpp"

#include <cstdlib>
#include <cmath>
#include <cstring>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "api_common.hpp"
#include "ti_engine.h"
#include "ti_hip.h"

namespace turboinfer {
namespace core {

using api::check;
using api::DeviceBuffer;

class TensorEngineImpl {
 public:
  ti_stream_t stream = nullptr;
  int device = 0;
  explicit TensorEngineImpl(int dev) : device(dev) {
    check(ti_init(dev), "ti_init");
    check(ti_stream_create(&stream), "ti_stream_create");
  }
  ~TensorEngineImpl() {
    if (stream) ti_stream_destroy(stream);
  }
  DeviceBuffer upload(const std::vector<float>& v) {
    DeviceBuffer b(v.size() * sizeof(float));
    if (!v.empty()) check(ti_memcpy_h2d(b.ptr, v.data(), v.size() * sizeof(float), stream), "ti_memcpy_h2d");
    return b;
  }
  Tensor download(const DeviceBuffer& b, const TensorShape& shape) {
    Tensor t(shape, DataType::kFloat32);
    if (t.byte_size()) check(ti_memcpy_d2h(t.data(), b.ptr, t.byte_size(), stream), "ti_memcpy_d2h");
    check(ti_stream_sync(stream), "ti_stream_sync");
    return t;
  }
};

namespace {

[[noreturn]] void off_path(const char* op) {
  throw std::runtime_error(std::string("TensorEngine::") + op +
                           ": not part of the MI355X decode hot path of this build (SURVEY.md 8(f))");
}

void require_nonempty(const Tensor& t, const char* what) {
  if (t.empty()) throw std::runtime_error(std::string("Cannot apply ") + what + " to empty tensors");
}

void require_same_shape(const Tensor& a, const Tensor& b, const char* op) {
  if (a.shape() != b.shape())
    throw std::runtime_error(std::string("TensorEngine::") + op + ": tensor shapes must match");
}

}  // namespace

TensorEngine::TensorEngine(ComputeDevice device) : device_(device) {
  if (device == ComputeDevice::kCPU)
    throw std::runtime_error(
        "TensorEngine: this build runs on MI355X (gfx950) only; ComputeDevice::kCPU is the reference's own CPU path");
  int count = 0;
  if (ti_device_count(&count) != TI_OK || count < 1)
    throw std::runtime_error("GPU device requested but not available: no gfx950 (MI355X) device is visible");
  device_ = ComputeDevice::kGPU;
  // the device ordinal: TI_GPU_INDEX, as InferenceEngine reads it when its model's extra_params do
  // not name one (the reference binds device 0, tensor_engine.cpp:425-487)
  int gpu = 0;
  if (const char* v = std::getenv("TI_GPU_INDEX")) gpu = std::atoi(v);
  if (gpu < 0 || gpu >= count)
    throw std::runtime_error("TensorEngine: TI_GPU_INDEX=" + std::to_string(gpu) + " but " + std::to_string(count) +
                             " device(s) are visible");
  impl_ = std::make_unique<TensorEngineImpl>(gpu);
}

TensorEngine::~TensorEngine() = default;

bool TensorEngine::gpu_available() const noexcept {
  int count = 0;
  return ti_device_count(&count) == TI_OK && count > 0;
}

std::string TensorEngine::device_info() const {
  std::ostringstream os;
  int count = 0;
  ti_device_count(&count);
  os << "TensorEngine Device Information:\n";
  for (int d = 0; d < count; ++d) {
    char name[128] = {0};
    ti_device_name(d, name, sizeof(name));
    os << "  GPU " << d << ": " << name << "\n";
  }
  os << "  Active Device: " << device_to_string(device_) << " (HIP device " << (impl_ ? impl_->device : 0)
     << ", gfx950 kernels)";
  return os.str();
}

Tensor TensorEngine::matmul(const Tensor& a, const Tensor& b) {
  if (a.empty() || b.empty()) throw std::runtime_error("Cannot perform matrix multiplication on empty tensors");
  const auto& sa = a.shape();
  const auto& sb = b.shape();
  if (sb.ndim() != 2 || (sa.ndim() != 2 && sa.ndim() != 3))
    throw std::runtime_error("Matrix multiplication supports 2D and 3D tensors only. Got shapes: " +
                             std::to_string(sa.ndim()) + "D x " + std::to_string(sb.ndim()) + "D" +
                             (sb.ndim() == 3 ? " (batched 3D x 3D is not on the decode path)" : ""));
  const size_t K = sa.dimensions().back(), N = sb.size(1);
  if (sb.size(0) != K)
    throw std::runtime_error("Matrix dimensions incompatible for multiplication: " + std::to_string(K) + " vs " +
                             std::to_string(sb.size(0)));
  const size_t rows = sa.total_size() / K;
  DeviceBuffer da = impl_->upload(api::to_f32(a)), db = impl_->upload(api::to_f32(b)), dy(rows * N * 4);
  check(ti_matmul_f32((const float*)da.ptr, (const float*)db.ptr, (float*)dy.ptr, nullptr, (int)rows, (int)K, (int)N,
                      0, impl_->stream),
        "ti_matmul_f32");
  std::vector<size_t> od = sa.dimensions();
  od.back() = N;
  return impl_->download(dy, TensorShape(od));
}

Tensor TensorEngine::batch_matmul(const Tensor&, const Tensor&) { off_path("batch_matmul"); }
Tensor TensorEngine::add_bias(const Tensor&, const Tensor&) { off_path("add_bias"); }
Tensor TensorEngine::gelu(const Tensor&) { off_path("gelu"); }
Tensor TensorEngine::layer_norm(const Tensor&, const Tensor&, const Tensor&, float) { off_path("layer_norm"); }
Tensor TensorEngine::scale(const Tensor&, float) { off_path("scale"); }
Tensor TensorEngine::concatenate(const std::vector<Tensor>&, size_t) { off_path("concatenate"); }
std::vector<Tensor> TensorEngine::split(const Tensor&, const std::vector<size_t>&, size_t) { off_path("split"); }
Tensor TensorEngine::transpose(const Tensor&) { off_path("transpose"); }
Tensor TensorEngine::permute(const Tensor&, const std::vector<size_t>&) { off_path("permute"); }

static Tensor unary(TensorEngineImpl& impl, const Tensor& x, int (*fn)(const float*, float*, int64_t, ti_stream_t),
                    const char* name) {
  DeviceBuffer dx = impl.upload(api::to_f32(x)), dy(x.shape().total_size() * 4);
  check(fn((const float*)dx.ptr, (float*)dy.ptr, (int64_t)x.shape().total_size(), impl.stream), name);
  return impl.download(dy, x.shape());
}

static Tensor binary(TensorEngineImpl& impl, const Tensor& a, const Tensor& b,
                     int (*fn)(const float*, const float*, float*, int64_t, ti_stream_t), const char* name) {
  DeviceBuffer da = impl.upload(api::to_f32(a)), db = impl.upload(api::to_f32(b)), dy(a.shape().total_size() * 4);
  check(fn((const float*)da.ptr, (const float*)db.ptr, (float*)dy.ptr, (int64_t)a.shape().total_size(), impl.stream),
        name);
  return impl.download(dy, a.shape());
}

Tensor TensorEngine::relu(const Tensor& input) {
  require_nonempty(input, "ReLU");
  return unary(*impl_, input, ti_relu_f32, "ti_relu_f32");
}

Tensor TensorEngine::silu(const Tensor& input) {
  require_nonempty(input, "SiLU");
  return unary(*impl_, input, ti_silu_f32, "ti_silu_f32");
}

Tensor TensorEngine::add(const Tensor& a, const Tensor& b) {
  require_nonempty(a, "add");
  require_nonempty(b, "add");
  require_same_shape(a, b, "add");
  return binary(*impl_, a, b, ti_add_f32, "ti_add_f32");
}

Tensor TensorEngine::multiply(const Tensor& a, const Tensor& b) {
  require_nonempty(a, "multiply");
  require_nonempty(b, "multiply");
  require_same_shape(a, b, "multiply");
  return binary(*impl_, a, b, ti_mul_f32, "ti_mul_f32");
}

Tensor TensorEngine::softmax(const Tensor& input, float temperature) {
  if (input.empty()) throw std::runtime_error("Cannot apply softmax to empty tensor");
  const size_t n = input.shape().dimensions().back(), rows = input.shape().total_size() / n;
  DeviceBuffer dx = impl_->upload(api::to_f32(input)), dy(rows * n * 4);
  check(ti_softmax_f32((const float*)dx.ptr, (float*)dy.ptr, (int)rows, (int)n, temperature, impl_->stream),
        "ti_softmax_f32");
  return impl_->download(dy, input.shape());
}

Tensor TensorEngine::rms_norm(const Tensor& input, const Tensor& weight, float eps) {
  if (input.empty() || weight.empty()) throw std::runtime_error("Cannot apply RMS normalization to empty tensors");
  if (weight.shape().ndim() != 1) throw std::runtime_error("Weight must be a 1D tensor for RMS normalization");
  if (weight.shape().size(0) != input.shape().dimensions().back())
    throw std::runtime_error("Weight size must match the last dimension of input tensor");
  const size_t n = weight.shape().size(0), rows = input.shape().total_size() / n;
  DeviceBuffer dx = impl_->upload(api::to_f32(input)), dw = impl_->upload(api::to_f32(weight)), dy(rows * n * 4);
  check(ti_rms_norm_f32((const float*)dx.ptr, (const float*)dw.ptr, (float*)dy.ptr, (int)rows, (int)n, eps,
                        impl_->stream),
        "ti_rms_norm_f32");
  return impl_->download(dy, input.shape());
}

Tensor TensorEngine::apply_rope(const Tensor& input, const Tensor& position_ids, float rope_theta) {
  if (input.empty() || position_ids.empty()) throw std::runtime_error("Cannot apply RoPE to empty tensors");
  const auto& d = input.shape().dimensions();
  const auto& pd = position_ids.shape().dimensions();
  if (d.size() < 3) throw std::runtime_error("RoPE requires input tensor with at least 3 dimensions");
  if (pd.size() < 1 || pd.size() > 2) throw std::runtime_error("Position IDs must be 1D or 2D tensor");
  if (input.dtype() != DataType::kFloat32 || position_ids.dtype() != DataType::kFloat32)
    throw std::runtime_error("RoPE currently only supports Float32 data type");
  if (d.size() > 4) throw std::runtime_error("RoPE supports 3D or 4D input tensors only");
  const int B = (int)d[0], heads = d.size() == 4 ? (int)d[1] : 1, S = (int)d[d.size() - 2], D = (int)d.back();
  if (D % 2) throw std::runtime_error("Hidden dimension must be even for RoPE");
  const bool pos2d = pd.size() == 2;
  const size_t npos = pos2d ? (size_t)B * S : (size_t)S;
  if (position_ids.shape().total_size() < npos) throw std::runtime_error("RoPE: too few position ids");
  std::vector<float> cs(npos * D);
  check(ti_rope_table(position_ids.data_ptr<float>(), (int)npos, D, rope_theta, cs.data()), "ti_rope_table");
  DeviceBuffer dx = impl_->upload(api::to_f32(input)), dcs = impl_->upload(cs), dy(input.shape().total_size() * 4);
  check(ti_rope_f32((const float*)dx.ptr, (float*)dy.ptr, (const float*)dcs.ptr, B, heads, S, D, pos2d ? 1 : 0,
                    impl_->stream),
        "ti_rope_f32");
  return impl_->download(dy, input.shape());
}

// Query length > 1 (tensor_engine.cpp:1084-1147, per head as multi_head_attention :1149-1252
// slices the hidden dimension): scores = Q K^T, one matmul per batch entry (the reference's
// batch_matmul: one fma per k in ascending order = ti_matmul_f32), times 1/sqrt(d) (its scale:
// ti_mul_f32 by a filled operand), -1e9 added where a float mask is 0 (ti_add_f32 of 0 / -1e9),
// softmax over the keys (ti_softmax_f32), then P V.  Only the head slicing and the key
// transpose (the reference's own host loops) run on the host.
static Tensor attend_rows(TensorEngineImpl& impl, const std::vector<float>& q, const std::vector<float>& k,
                          const std::vector<float>& v, size_t B, size_t Sq, size_t Sk, size_t H, size_t heads,
                          const Tensor* mask) {
  const size_t hd = H / heads, n = B * Sq * Sk;
  const float scale_factor = 1.0f / std::sqrt(static_cast<float>(hd));   // :1116
  DeviceBuffer dscale = impl.upload(std::vector<float>(n, scale_factor));
  DeviceBuffer dmask;
  const bool masked = mask && mask->dtype() == DataType::kFloat32;   // other mask types: no effect (:1127)
  if (masked) {
    const float* md = mask->data_ptr<float>();
    std::vector<float> add(n);
    for (size_t i = 0; i < n; ++i) add[i] = md[i] == 0.0f ? -1e9f : 0.0f;   // ATTENTION_MASK_VALUE (:47)
    dmask = impl.upload(add);
  }
  std::vector<float> out(B * Sq * H);
  std::vector<float> qh(B * Sq * hd), kt(B * hd * Sk), vh(B * Sk * hd);
  for (size_t h = 0; h < heads; ++h) {
    for (size_t b = 0; b < B; ++b) {
      for (size_t s = 0; s < Sq; ++s)
        std::memcpy(&qh[(b * Sq + s) * hd], &q[(b * Sq + s) * H + h * hd], hd * sizeof(float));
      for (size_t s = 0; s < Sk; ++s)
        for (size_t d = 0; d < hd; ++d) {
          kt[(b * hd + d) * Sk + s] = k[(b * Sk + s) * H + h * hd + d];
          vh[(b * Sk + s) * hd + d] = v[(b * Sk + s) * H + h * hd + d];
        }
    }
    DeviceBuffer dq = impl.upload(qh), dk = impl.upload(kt), dv = impl.upload(vh);
    DeviceBuffer ds(n * 4), dp(n * 4), dy(B * Sq * hd * 4);
    float* fs = (float*)ds.ptr;
    float* fp = (float*)dp.ptr;
    for (size_t b = 0; b < B; ++b)
      check(ti_matmul_f32((const float*)dq.ptr + b * Sq * hd, (const float*)dk.ptr + b * hd * Sk, fs + b * Sq * Sk,
                          nullptr, (int)Sq, (int)hd, (int)Sk, 0, impl.stream),
            "ti_matmul_f32");
    check(ti_mul_f32(fs, (const float*)dscale.ptr, fs, (int64_t)n, impl.stream), "ti_mul_f32");
    if (masked) check(ti_add_f32(fs, (const float*)dmask.ptr, fs, (int64_t)n, impl.stream), "ti_add_f32");
    check(ti_softmax_f32(fs, fp, (int)(B * Sq), (int)Sk, 1.0f, impl.stream), "ti_softmax_f32");
    for (size_t b = 0; b < B; ++b)
      check(ti_matmul_f32(fp + b * Sq * Sk, (const float*)dv.ptr + b * Sk * hd, (float*)dy.ptr + b * Sq * hd, nullptr,
                          (int)Sq, (int)Sk, (int)hd, 0, impl.stream),
            "ti_matmul_f32");
    const Tensor y = impl.download(dy, TensorShape({B, Sq, hd}));
    const float* yd = y.data_ptr<float>();
    for (size_t r = 0; r < B * Sq; ++r) std::memcpy(&out[r * H + h * hd], &yd[r * hd], hd * sizeof(float));
  }
  Tensor t(TensorShape({B, Sq, H}), DataType::kFloat32);
  std::memcpy(t.data(), out.data(), out.size() * sizeof(float));
  return t;
}

static Tensor attend(TensorEngineImpl& impl, const Tensor& q, const Tensor& k, const Tensor& v, size_t heads,
                     const Tensor* mask, const char* op) {
  if (q.empty() || k.empty() || v.empty())
    throw std::runtime_error(std::string(op) + ": query, key and value must be non-empty");
  const auto& qd = q.shape().dimensions();
  const auto& kd = k.shape().dimensions();
  if (qd.size() != 3 || kd.size() != 3 || v.shape() != k.shape())
    throw std::runtime_error(std::string(op) + ": expects query [B,Sq,H] and key/value [B,S,H]");
  const size_t B = qd[0], H = qd[2], S = kd[1];
  if (kd[0] != B || kd[2] != H) throw std::runtime_error(std::string(op) + ": query / key shapes disagree");
  if (heads == 0 || H % heads) throw std::runtime_error(std::string(op) + ": hidden size not divisible by heads");
  if (qd[1] != 1) {
    if (mask && mask->shape().dimensions() != std::vector<size_t>{B, qd[1], S})
      throw std::runtime_error("Mask dimensions must match attention scores");   // :1123-1125
    return attend_rows(impl, api::to_f32(q), api::to_f32(k), api::to_f32(v), B, qd[1], S, H, heads, mask);
  }
  // one query: attention_fast_incremental (:1254-1388), which takes the mask and ignores it
  DeviceBuffer dq = impl.upload(api::to_f32(q)), dk = impl.upload(api::to_f32(k)), dv = impl.upload(api::to_f32(v));
  DeviceBuffer dy(B * H * 4), scratch(B * heads * S * 4);
  check(ti_attention_f32((const float*)dq.ptr, (const float*)dk.ptr, (const float*)dv.ptr, (float*)dy.ptr,
                         (float*)scratch.ptr, (int)B, (int)S, (int)H, (int)heads, impl.stream),
        "ti_attention_f32");
  return impl.download(dy, q.shape());
}

Tensor TensorEngine::attention(const Tensor& query, const Tensor& key, const Tensor& value, const Tensor* mask) {
  return attend(*impl_, query, key, value, 1, mask, "TensorEngine::attention");
}

Tensor TensorEngine::attention_fast_incremental(const Tensor& query, const Tensor& key, const Tensor& value,
                                                const Tensor* mask) {
  return attend(*impl_, query, key, value, 1, mask, "TensorEngine::attention_fast_incremental");
}

Tensor TensorEngine::multi_head_attention(const Tensor& query, const Tensor& key, const Tensor& value,
                                          size_t num_heads, const Tensor* mask) {
  return attend(*impl_, query, key, value, num_heads, mask, "TensorEngine::multi_head_attention");
}

const char* device_to_string(ComputeDevice device) {
  switch (device) {
    case ComputeDevice::kCPU: return "CPU";
    case ComputeDevice::kGPU: return "GPU";
    case ComputeDevice::kAuto: return "Auto";
  }
  return "Unknown";
}

}  // namespace core
}  // namespace turboinfer
