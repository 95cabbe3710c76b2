// gguf.cpp -- ModelLoader::load_gguf (reference src/model/model_loader.cpp:710-873), SURVEY 8(f)
// rank 3: GGUF v3 checkpoints into the ModelData the engine is built from.
//
// The container walk follows the reference: header (magic "GGUF", version 3), the metadata
// key/value pairs mapped onto ModelMetadata exactly as :745-770 maps them (every value as the
// string the reference's read_gguf_value produces, :60-153: std::to_string for numbers,
// "true"/"false", strings verbatim, "[array]" for arrays), tensor infos with the dimensions
// reversed to row-major (:801), fp32 and fp16 tensors kept in their type (:165-170).
// Where the reference is wrong for real files, this follows the published GGUF / ggml layout
// instead (the differences are the point of the row):
//   * arrays are walked element by element (the reference skips count * 8 bytes, :142, which
//     loses the stream on the tokenizer's string arrays every llama GGUF carries);
//   * tensor data starts at the first general.alignment (default 32) boundary after the
//     tensor infos and tensor i sits at data_start + offset_i (the reference seeks each offset
//     relative to where the previous read ended, :842, correct for the first tensor only);
//   * Q4_0, Q4_1 and Q8_0 blocks are dequantized to fp32 (ggml's block formats: 32 weights per
//     block, an fp16 scale d (and min m), y = (q - 8) d, q d + m, q d); the reference declares
//     these types fp32 and reads the packed bytes as floats (:165-182, 817-829).  BF16 is
//     widened to fp32.  Other types raise.
// The CPU restatement is oracle/gguf_oracle.py (tests/test_cpp_api.py gguf cases).
#include <algorithm>
#include <cstring>
#include <filesystem>
#include <fstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "turboinfer/model/model_loader.hpp"

namespace turboinfer {
namespace model {

namespace {

constexpr uint32_t kGgufMagic = 0x46554747u;   // "GGUF"
constexpr uint32_t kGgufVersion = 3;
enum GgufValue : uint32_t {
  kU8 = 0, kI8 = 1, kU16 = 2, kI16 = 3, kU32 = 4, kI32 = 5, kF32 = 6, kBool = 7, kStr = 8, kArr = 9,
  kU64 = 10, kI64 = 11, kF64 = 12
};
enum GgmlType : uint32_t { kTF32 = 0, kTF16 = 1, kTQ4_0 = 2, kTQ4_1 = 3, kTQ8_0 = 8, kTBF16 = 30 };

struct Reader {
  std::ifstream f;
  std::string path;
  template <class T>
  T get() {
    T v{};
    f.read(reinterpret_cast<char*>(&v), sizeof(T));
    if (!f.good()) throw std::runtime_error("GGUF: unexpected end of file: " + path);
    return v;
  }
  std::string str() {
    const uint64_t n = get<uint64_t>();
    if (n > (1u << 20)) throw std::runtime_error("GGUF string too long");   // reference :45-47
    std::string s(n, '\0');
    f.read(s.data(), (std::streamsize)n);
    if (!f.good()) throw std::runtime_error("Failed to read GGUF string");
    return s;
  }
  void skip(uint32_t type) {   // one array element
    switch (type) {
      case kU8: case kI8: case kBool: get<uint8_t>(); break;
      case kU16: case kI16: get<uint16_t>(); break;
      case kU32: case kI32: case kF32: get<uint32_t>(); break;
      case kU64: case kI64: case kF64: get<uint64_t>(); break;
      case kStr: str(); break;
      case kArr: {
        const uint32_t t = get<uint32_t>();
        const uint64_t n = get<uint64_t>();
        for (uint64_t i = 0; i < n; ++i) skip(t);
        break;
      }
      default: throw std::runtime_error("Unsupported GGUF value type: " + std::to_string(type));
    }
  }
  // value as the reference's read_gguf_value string; *u32 receives a uint32 value (alignment)
  std::string value(uint32_t type, uint64_t* num = nullptr) {
    switch (type) {
      case kU8: { const auto v = get<uint8_t>(); if (num) *num = v; return std::to_string(v); }
      case kI8: return std::to_string(get<int8_t>());
      case kU16: { const auto v = get<uint16_t>(); if (num) *num = v; return std::to_string(v); }
      case kI16: return std::to_string(get<int16_t>());
      case kU32: { const auto v = get<uint32_t>(); if (num) *num = v; return std::to_string(v); }
      case kI32: return std::to_string(get<int32_t>());
      case kU64: { const auto v = get<uint64_t>(); if (num) *num = v; return std::to_string(v); }
      case kI64: return std::to_string(get<int64_t>());
      case kF32: return std::to_string(get<float>());
      case kF64: return std::to_string(get<double>());
      case kBool: return get<uint8_t>() ? "true" : "false";
      case kStr: return str();
      case kArr: {
        const uint32_t t = get<uint32_t>();
        const uint64_t n = get<uint64_t>();
        for (uint64_t i = 0; i < n; ++i) skip(t);
        return "[array]";
      }
      default: throw std::runtime_error("Unsupported GGUF value type: " + std::to_string(type));
    }
  }
};

float half_to_float(uint16_t h) {
  const uint32_t s = (uint32_t)(h & 0x8000u) << 16, e = (h >> 10) & 0x1f, m = h & 0x3ffu;
  uint32_t bits;
  if (e == 0) {
    if (m == 0) {
      bits = s;
    } else {   // subnormal: normalise
      int ee = -1;
      uint32_t mm = m;
      do { ++ee; mm <<= 1; } while (!(mm & 0x400u));
      bits = s | ((uint32_t)(127 - 15 - ee) << 23) | ((mm & 0x3ffu) << 13);
    }
  } else if (e == 31) {
    bits = s | 0x7f800000u | (m << 13);
  } else {
    bits = s | ((e + 127 - 15) << 23) | (m << 13);
  }
  float f;
  std::memcpy(&f, &bits, 4);
  return f;
}

// ggml block layouts (32 weights per block)
void dequant_q4_0(const uint8_t* b, size_t nblk, float* y) {
  for (size_t i = 0; i < nblk; ++i, b += 18, y += 32) {
    uint16_t dh;
    std::memcpy(&dh, b, 2);
    const float d = half_to_float(dh);
    for (int j = 0; j < 16; ++j) {
      y[j] = (float)((int)(b[2 + j] & 0x0f) - 8) * d;
      y[j + 16] = (float)((int)(b[2 + j] >> 4) - 8) * d;
    }
  }
}
void dequant_q4_1(const uint8_t* b, size_t nblk, float* y) {
  for (size_t i = 0; i < nblk; ++i, b += 20, y += 32) {
    uint16_t dh, mh;
    std::memcpy(&dh, b, 2);
    std::memcpy(&mh, b + 2, 2);
    const float d = half_to_float(dh), m = half_to_float(mh);
    for (int j = 0; j < 16; ++j) {
      y[j] = (float)(b[4 + j] & 0x0f) * d + m;
      y[j + 16] = (float)(b[4 + j] >> 4) * d + m;
    }
  }
}
void dequant_q8_0(const uint8_t* b, size_t nblk, float* y) {
  for (size_t i = 0; i < nblk; ++i, b += 34, y += 32) {
    uint16_t dh;
    std::memcpy(&dh, b, 2);
    const float d = half_to_float(dh);
    for (int j = 0; j < 32; ++j) y[j] = (float)(int8_t)b[2 + j] * d;
  }
}

struct Info {
  std::string name;
  std::vector<size_t> dims;   // reversed: row-major
  uint32_t type = 0;
  uint64_t offset = 0;
};

size_t stored_bytes(uint32_t type, size_t n, const std::string& name) {
  switch (type) {
    case kTF32: return n * 4;
    case kTF16: case kTBF16: return n * 2;
    case kTQ4_0: case kTQ4_1: case kTQ8_0:
      if (n % 32) throw std::runtime_error("GGUF: tensor " + name + " is not a whole number of 32-weight blocks");
      return n / 32 * (type == kTQ4_0 ? 18 : type == kTQ4_1 ? 20 : 34);
    default:
      throw std::runtime_error("GGUF: tensor " + name + " has unsupported ggml type " + std::to_string(type) +
                               " (supported: F32, F16, BF16, Q4_0, Q4_1, Q8_0)");
  }
}

}  // namespace

ModelData ModelLoader::load_gguf(const std::string& file_path) {
  if (!std::filesystem::exists(file_path)) throw std::runtime_error("GGUF file does not exist: " + file_path);
  Reader r;
  r.path = file_path;
  r.f.open(file_path, std::ios::binary);
  if (!r.f.is_open()) throw std::runtime_error("Cannot open GGUF file: " + file_path);
  const uint32_t magic = r.get<uint32_t>(), version = r.get<uint32_t>();
  const uint64_t n_tensors = r.get<uint64_t>(), n_kv = r.get<uint64_t>();
  if (magic != kGgufMagic) throw std::runtime_error("Invalid GGUF magic number");
  if (version != kGgufVersion) throw std::runtime_error("Unsupported GGUF version: " + std::to_string(version));

  ModelData md;
  ModelMetadata& meta = md.metadata();
  meta.name = std::filesystem::path(file_path).stem().string();
  meta.architecture = "unknown";
  meta.version = "gguf_v" + std::to_string(version);
  uint64_t alignment = 32;
  for (uint64_t i = 0; i < n_kv; ++i) {
    const std::string key = r.str();
    const uint32_t type = r.get<uint32_t>();
    uint64_t num = 0;
    const std::string value = r.value(type, &num);
    if (key == "general.alignment" && type == kU32) alignment = num;
    // model_loader.cpp:747-770
    if (key == "general.architecture") meta.architecture = value;
    else if (key == "general.name") meta.name = value;
    else if (key == "llama.vocab_size" || key == "gpt2.vocab_size") meta.vocab_size = std::stoull(value);
    else if (key == "llama.embedding_length" || key == "gpt2.embedding_length") meta.hidden_size = std::stoull(value);
    else if (key == "llama.block_count" || key == "gpt2.block_count") meta.num_layers = std::stoull(value);
    else if (key == "llama.attention.head_count" || key == "gpt2.attention.head_count") meta.num_heads = std::stoull(value);
    else if (key == "llama.feed_forward_length" || key == "gpt2.feed_forward_length")
      meta.intermediate_size = std::stoull(value);
    else if (key == "llama.rope.theta") meta.rope_theta = std::stof(value);
    else meta.extra_params[key] = value;
  }
  if (alignment == 0 || (alignment & (alignment - 1)))
    throw std::runtime_error("GGUF: general.alignment " + std::to_string(alignment) + " is not a power of two");

  std::vector<Info> infos((size_t)n_tensors);
  for (auto& t : infos) {
    t.name = r.str();
    const uint32_t nd = r.get<uint32_t>();
    if (nd == 0 || nd > 8) throw std::runtime_error("GGUF: tensor " + t.name + " has " + std::to_string(nd) + " dims");
    t.dims.resize(nd);
    for (uint32_t j = 0; j < nd; ++j) t.dims[j] = (size_t)r.get<uint64_t>();
    t.type = r.get<uint32_t>();
    t.offset = r.get<uint64_t>();
    std::reverse(t.dims.begin(), t.dims.end());
  }
  const uint64_t pos = (uint64_t)r.f.tellg();
  const uint64_t data_start = (pos + alignment - 1) / alignment * alignment;
  r.f.seekg(0, std::ios::end);
  const uint64_t file_size = (uint64_t)r.f.tellg();

  std::vector<uint8_t> raw;
  for (const auto& t : infos) {
    size_t n = 1;
    for (size_t d : t.dims) n *= d;
    const size_t bytes = stored_bytes(t.type, n, t.name);
    if (data_start + t.offset + bytes > file_size)
      throw std::runtime_error("Failed to read tensor data for: " + t.name + " (past the end of the file)");
    r.f.seekg((std::streamoff)(data_start + t.offset));
    const bool keep = t.type == kTF32 || t.type == kTF16;
    core::Tensor out(core::TensorShape(t.dims), t.type == kTF16 ? core::DataType::kFloat16 : core::DataType::kFloat32);
    if (keep) {
      if (bytes) r.f.read(reinterpret_cast<char*>(out.data()), (std::streamsize)bytes);
    } else {
      raw.resize(bytes);
      r.f.read(reinterpret_cast<char*>(raw.data()), (std::streamsize)bytes);
    }
    if (!r.f.good()) throw std::runtime_error("Failed to read tensor data for: " + t.name);
    float* y = keep ? nullptr : out.data_ptr<float>();
    if (t.type == kTQ4_0) dequant_q4_0(raw.data(), n / 32, y);
    else if (t.type == kTQ4_1) dequant_q4_1(raw.data(), n / 32, y);
    else if (t.type == kTQ8_0) dequant_q8_0(raw.data(), n / 32, y);
    else if (t.type == kTBF16)
      for (size_t i = 0; i < n; ++i) {
        const uint32_t bits = (uint32_t)(raw[2 * i] | (raw[2 * i + 1] << 8)) << 16;
        std::memcpy(y + i, &bits, 4);
      }
    md.add_tensor(t.name, std::move(out));
  }
  return md;
}

}  // namespace model
}  // namespace turboinfer
