// tensor.cpp -- turboinfer::core::Tensor (host container of the drop-in C++ API).
// Semantics follow the reference's src/core/tensor.cpp (construction zero-fills, copies are
// deep, reshape/slice copy, total_size of a dimensionless shape is 0).
#include "turboinfer/core/tensor.hpp"

#include <cstring>
#include <string>

namespace turboinfer {
namespace core {

TensorShape::TensorShape(std::initializer_list<size_t> dimensions) : dims_(dimensions) { recompute(); }
TensorShape::TensorShape(const std::vector<size_t>& dimensions) : dims_(dimensions) { recompute(); }

void TensorShape::recompute() {
  if (dims_.empty()) {
    total_ = 0;
    return;
  }
  size_t t = 1;
  for (size_t d : dims_) t *= d;
  total_ = t;
}

size_t TensorShape::size(size_t dim) const {
  if (dim >= dims_.size())
    throw std::out_of_range("TensorShape::size: dimension " + std::to_string(dim) + " of a " +
                            std::to_string(dims_.size()) + "-dimensional shape");
  return dims_[dim];
}

Tensor::Tensor(const TensorShape& shape, DataType dtype) : shape_(shape), dtype_(dtype) { allocate(); }

Tensor::Tensor(const TensorShape& shape, const void* data, DataType dtype) : shape_(shape), dtype_(dtype) {
  allocate();
  if (data && bytes_) std::memcpy(bytes_.get(), data, byte_size());
}

Tensor::Tensor(const Tensor& other) : shape_(other.shape_), dtype_(other.dtype_) {
  allocate();
  if (other.bytes_ && bytes_) std::memcpy(bytes_.get(), other.bytes_.get(), byte_size());
}

Tensor::Tensor(Tensor&& other) noexcept
    : shape_(std::move(other.shape_)), dtype_(other.dtype_), bytes_(std::move(other.bytes_)) {}

Tensor& Tensor::operator=(const Tensor& other) {
  if (this == &other) return *this;
  shape_ = other.shape_;
  dtype_ = other.dtype_;
  allocate();
  if (other.bytes_ && bytes_) std::memcpy(bytes_.get(), other.bytes_.get(), byte_size());
  return *this;
}

Tensor& Tensor::operator=(Tensor&& other) noexcept {
  if (this == &other) return *this;
  shape_ = std::move(other.shape_);
  dtype_ = other.dtype_;
  bytes_ = std::move(other.bytes_);
  return *this;
}

size_t Tensor::element_size() const noexcept {
  switch (dtype_) {
    case DataType::kFloat32: case DataType::kInt32: return 4;
    case DataType::kFloat16: case DataType::kInt16: return 2;
    case DataType::kInt8: case DataType::kUInt8: return 1;
  }
  return 0;
}

size_t Tensor::byte_size() const noexcept { return shape_.total_size() * element_size(); }

void Tensor::allocate() {
  const size_t n = byte_size();
  if (n == 0) {
    bytes_.reset();
    return;
  }
  bytes_.reset(new uint8_t[n]());   // value-initialised: zero-filled
}

void Tensor::check_type(size_t type_size) const {
  if (type_size != element_size())
    throw std::runtime_error("Tensor::data_ptr: element type of " + std::to_string(type_size) +
                             " bytes does not match the tensor's " + std::to_string(element_size()) + "-byte " +
                             dtype_to_string(dtype_));
}

Tensor Tensor::clone() const { return Tensor(*this); }

Tensor Tensor::reshape(const TensorShape& new_shape) const {
  if (new_shape.total_size() != shape_.total_size())
    throw std::runtime_error("Tensor::reshape: " + std::to_string(new_shape.total_size()) + " elements requested, " +
                             std::to_string(shape_.total_size()) + " present");
  return Tensor(new_shape, bytes_.get(), dtype_);
}

Tensor Tensor::slice(const std::vector<size_t>& start, const std::vector<size_t>& end) const {
  const size_t nd = shape_.ndim();
  if (start.size() != nd || end.size() != nd)
    throw std::runtime_error("Tensor::slice: start/end need one index per dimension");
  std::vector<size_t> out_dims(nd);
  for (size_t d = 0; d < nd; ++d) {
    if (start[d] >= shape_.size(d) || end[d] > shape_.size(d) || start[d] >= end[d])
      throw std::runtime_error("Tensor::slice: invalid bounds in dimension " + std::to_string(d));
    out_dims[d] = end[d] - start[d];
  }
  Tensor out{TensorShape(out_dims), dtype_};
  if (empty() || out.empty()) return out;
  // Copy contiguous runs along the innermost dimension; an odometer walks the outer ones.
  const size_t es = element_size(), run = out_dims[nd - 1] * es;
  std::vector<size_t> src_stride(nd, 1);
  for (size_t d = nd - 1; d-- > 0;) src_stride[d] = src_stride[d + 1] * shape_.size(d + 1);
  std::vector<size_t> idx(nd, 0);
  const uint8_t* src = bytes_.get();
  uint8_t* dst = out.bytes_.get();
  const size_t runs = out.shape_.total_size() / out_dims[nd - 1];
  for (size_t r = 0; r < runs; ++r) {
    size_t off = start[nd - 1];
    for (size_t d = 0; d + 1 < nd; ++d) off += (start[d] + idx[d]) * src_stride[d];
    std::memcpy(dst + r * run, src + off * es, run);
    for (size_t d = nd - 1; d-- > 0;) {   // advance the outer-dimension odometer
      if (++idx[d] < out_dims[d]) break;
      idx[d] = 0;
    }
  }
  return out;
}

size_t get_dtype_size(DataType dtype) {
  switch (dtype) {
    case DataType::kFloat32: case DataType::kInt32: return 4;
    case DataType::kFloat16: case DataType::kInt16: return 2;
    case DataType::kInt8: case DataType::kUInt8: return 1;
  }
  throw std::runtime_error("get_dtype_size: unknown data type");
}

const char* dtype_to_string(DataType dtype) {
  switch (dtype) {
    case DataType::kFloat32: return "float32";
    case DataType::kFloat16: return "float16";
    case DataType::kInt32: return "int32";
    case DataType::kInt16: return "int16";
    case DataType::kInt8: return "int8";
    case DataType::kUInt8: return "uint8";
  }
  return "unknown";
}

}  // namespace core
}  // namespace turboinfer
