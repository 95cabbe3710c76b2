// api_common.hpp -- shared helpers of the C++ API layer (not installed): the C-ABI error
// mapping, an RAII device buffer and the reference's dtype conversion to fp32.
#pragma once

#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "ti_hip.h"
#include "turboinfer/core/tensor.hpp"

namespace turboinfer {
namespace api {

/// Any non-zero C-ABI code becomes std::runtime_error("ti_hip: <fn>: <message>").
inline void check(int rc, const char* what) {
  if (rc != TI_OK) throw std::runtime_error(std::string("ti_hip: ") + what + ": " + ti_last_error());
}

/// Device allocation owned by the API object that made it (never caller memory).
struct DeviceBuffer {
  void* ptr = nullptr;
  size_t bytes = 0;
  DeviceBuffer() = default;
  explicit DeviceBuffer(size_t n) : bytes(n) {
    if (n) check(ti_malloc(&ptr, n), "ti_malloc");
  }
  DeviceBuffer(const DeviceBuffer&) = delete;
  DeviceBuffer& operator=(const DeviceBuffer&) = delete;
  DeviceBuffer(DeviceBuffer&& o) noexcept : ptr(o.ptr), bytes(o.bytes) { o.ptr = nullptr; o.bytes = 0; }
  DeviceBuffer& operator=(DeviceBuffer&& o) noexcept {
    if (this != &o) {
      if (ptr) ti_free(ptr);
      ptr = o.ptr;
      bytes = o.bytes;
      o.ptr = nullptr;
      o.bytes = 0;
    }
    return *this;
  }
  ~DeviceBuffer() {
    if (ptr) ti_free(ptr);
  }
};

inline float half_to_float(uint16_t h) {
  const uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
  uint32_t e = (h >> 10) & 0x1fu, m = h & 0x3ffu, bits;
  if (e == 0) {
    if (m == 0) {
      bits = sign;
    } else {   // subnormal: renormalise
      int sh = 0;
      while (!(m & 0x400u)) { m <<= 1; ++sh; }
      bits = sign | ((uint32_t)(113 - sh) << 23) | ((m & 0x3ffu) << 13);
    }
  } else if (e == 31) {
    bits = sign | 0x7f800000u | (m << 13);
  } else {
    bits = sign | ((e + 112) << 23) | (m << 13);
  }
  float f;
  std::memcpy(&f, &bits, 4);
  return f;
}

/// Elements as fp32, the reference's convert_dtype (tensor_engine.cpp:2218-2284): integer
/// tensors are a raw value cast, fp16 is widened.
inline std::vector<float> to_f32(const core::Tensor& t) {
  using core::DataType;
  const size_t n = t.shape().total_size();
  std::vector<float> v(n);
  if (t.empty()) return v;
  switch (t.dtype()) {
    case DataType::kFloat32: std::memcpy(v.data(), t.data(), n * 4); break;
    case DataType::kFloat16: { const uint16_t* p = t.data_ptr<uint16_t>(); for (size_t i = 0; i < n; ++i) v[i] = half_to_float(p[i]); break; }
    case DataType::kInt32: { const int32_t* p = t.data_ptr<int32_t>(); for (size_t i = 0; i < n; ++i) v[i] = (float)p[i]; break; }
    case DataType::kInt16: { const int16_t* p = t.data_ptr<int16_t>(); for (size_t i = 0; i < n; ++i) v[i] = (float)p[i]; break; }
    case DataType::kInt8: { const int8_t* p = t.data_ptr<int8_t>(); for (size_t i = 0; i < n; ++i) v[i] = (float)p[i]; break; }
    case DataType::kUInt8: { const uint8_t* p = t.data_ptr<uint8_t>(); for (size_t i = 0; i < n; ++i) v[i] = (float)p[i]; break; }
  }
  return v;
}

}  // namespace api
}  // namespace turboinfer
