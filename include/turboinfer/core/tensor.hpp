// turboinfer/core/tensor.hpp -- host tensor container of the drop-in C++ API.
//
// Same names, signatures and semantics as the reference's turboinfer::core::Tensor /
// TensorShape / DataType (include/turboinfer/core/tensor.hpp:23-269 in the reference):
// an owning, zero-initialised host buffer; copy is deep; reshape and slice return new
// tensors; data_ptr<T>() checks only sizeof(T) against the element size.  Device memory
// never appears here: the MI355X engines keep their own device-resident state.
#pragma once

#include <cstddef>
#include <cstdint>
#include <initializer_list>
#include <memory>
#include <stdexcept>
#include <vector>

namespace turboinfer {
namespace core {

enum class DataType {
  kFloat32,
  kFloat16,
  kInt32,
  kInt16,
  kInt8,
  kUInt8
};

class TensorShape {
 public:
  TensorShape() = default;
  explicit TensorShape(std::initializer_list<size_t> dimensions);
  explicit TensorShape(const std::vector<size_t>& dimensions);

  size_t ndim() const noexcept { return dims_.size(); }
  /// Size of dimension `dim`; std::out_of_range past the last dimension.
  size_t size(size_t dim) const;
  /// Product of the dimensions (0 for a shape without dimensions).
  size_t total_size() const noexcept { return total_; }
  const std::vector<size_t>& dimensions() const noexcept { return dims_; }

  bool operator==(const TensorShape& other) const noexcept { return dims_ == other.dims_; }
  bool operator!=(const TensorShape& other) const noexcept { return dims_ != other.dims_; }

 private:
  std::vector<size_t> dims_;
  size_t total_ = 0;
  void recompute();
};

class Tensor {
 public:
  Tensor() = default;
  Tensor(const TensorShape& shape, DataType dtype = DataType::kFloat32);
  Tensor(const TensorShape& shape, const void* data, DataType dtype = DataType::kFloat32);
  Tensor(const Tensor& other);
  Tensor(Tensor&& other) noexcept;
  Tensor& operator=(const Tensor& other);
  Tensor& operator=(Tensor&& other) noexcept;
  ~Tensor() = default;

  const TensorShape& shape() const noexcept { return shape_; }
  DataType dtype() const noexcept { return dtype_; }
  size_t element_size() const noexcept;
  size_t byte_size() const noexcept;
  void* data() noexcept { return bytes_.get(); }
  const void* data() const noexcept { return bytes_.get(); }

  template <typename T>
  T* data_ptr() {
    check_type(sizeof(T));
    return reinterpret_cast<T*>(bytes_.get());
  }
  template <typename T>
  const T* data_ptr() const {
    check_type(sizeof(T));
    return reinterpret_cast<const T*>(bytes_.get());
  }

  bool empty() const noexcept { return !bytes_ || shape_.total_size() == 0; }

  template <typename T>
  void fill(T value) {
    check_type(sizeof(T));
    if (empty()) return;
    T* p = reinterpret_cast<T*>(bytes_.get());
    for (size_t i = 0, n = shape_.total_size(); i < n; ++i) p[i] = value;
  }

  Tensor clone() const;
  /// Same elements under `new_shape` (a copy); std::runtime_error if the sizes differ.
  Tensor reshape(const TensorShape& new_shape) const;
  /// Elements [start, end) along every dimension (a copy); std::runtime_error on bad bounds.
  Tensor slice(const std::vector<size_t>& start, const std::vector<size_t>& end) const;

 private:
  TensorShape shape_;
  DataType dtype_ = DataType::kFloat32;
  std::unique_ptr<uint8_t[]> bytes_;
  void allocate();
  void check_type(size_t type_size) const;
};

size_t get_dtype_size(DataType dtype);
const char* dtype_to_string(DataType dtype);

}  // namespace core
}  // namespace turboinfer
