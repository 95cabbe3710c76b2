// api_check.cpp -- drives the drop-in C++ API (turboinfer::core / model / optimize) for the
// pytest suite (tests/test_cpp_api.py), which supplies inputs and checks outputs against the
// golden fixtures.  Arrays travel as small binary files:
//   u32 dtype (0 f32, 1 i32, 2 i8) | u32 ndim | u64 dims[ndim] | raw little-endian data
//
//   api_check tensor                                  Tensor / TensorShape semantics (self-checking)
//   api_check quant  <x> <bits> <sym> <out>           Quantizer: out = [scale, zp] ++ q ++ dequantized
//   api_check op <name> <out> <in...> [param]         TensorEngine op on the GPU
//   api_check generate <model_dir> <prompts> <n_new> <top_k> <weight_bits> <out>
//                                                     InferenceEngine::generate_batch on the GPU
//   api_check tinq_save <model_dir> <bits> <sym> <out.tinq>
//                                                     Quantizer::quantize_model + save_quantized_model
//   api_check tinq_load <in.tinq> <out_dir>           Quantizer::load_quantized_model -> meta.txt,
//                                                     names.txt and <i>.bin in the file's order
//   api_check gguf_load <in.gguf> <out>               ModelLoader::load -> <out>.meta + <out>.data
//   api_check generate_gguf <in.gguf> <prompts> <n_new> <top_k> <weight_bits> <out>
//                                                     generate_batch on a model read from a GGUF file
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "turboinfer/turboinfer.hpp"

using namespace turboinfer;
using core::DataType;
using core::Tensor;
using core::TensorShape;

static Tensor read_array(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("cannot open " + path);
  uint32_t code = 0, nd = 0;
  f.read((char*)&code, 4);
  f.read((char*)&nd, 4);
  std::vector<size_t> dims(nd);
  for (auto& d : dims) {
    uint64_t v = 0;
    f.read((char*)&v, 8);
    d = (size_t)v;
  }
  const DataType dt = code == 0 ? DataType::kFloat32 : code == 1 ? DataType::kInt32 : DataType::kInt8;
  Tensor t(TensorShape(dims), dt);
  if (t.byte_size()) f.read((char*)t.data(), (std::streamsize)t.byte_size());
  if (!f) throw std::runtime_error("short read " + path);
  return t;
}

static void write_array(const std::string& path, const Tensor& t) {
  std::ofstream f(path, std::ios::binary);
  const uint32_t code = t.dtype() == DataType::kFloat32 ? 0 : t.dtype() == DataType::kInt32 ? 1 : 2;
  const uint32_t nd = (uint32_t)t.shape().ndim();
  f.write((const char*)&code, 4);
  f.write((const char*)&nd, 4);
  for (size_t d : t.shape().dimensions()) {
    const uint64_t v = d;
    f.write((const char*)&v, 8);
  }
  if (t.byte_size()) f.write((const char*)t.data(), (std::streamsize)t.byte_size());
}

#define EXPECT(cond)                                                              \
  do {                                                                            \
    if (!(cond)) {                                                                \
      std::cerr << "FAILED " << __FILE__ << ":" << __LINE__ << ": " #cond "\n"; \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

template <class E, class F>
static bool throws(F f) {
  try {
    f();
  } catch (const E&) {
    return true;
  } catch (...) {
    return false;
  }
  return false;
}

static int tensor_checks() {
  TensorShape s({2, 3, 4});
  EXPECT(s.ndim() == 3 && s.total_size() == 24 && s.size(2) == 4);
  EXPECT(throws<std::out_of_range>([&] { (void)s.size(3); }));
  EXPECT(TensorShape(std::vector<size_t>{}).total_size() == 0);
  Tensor t(s);
  EXPECT(t.byte_size() == 96 && t.element_size() == 4 && !t.empty());
  for (size_t i = 0; i < 24; ++i) EXPECT(t.data_ptr<float>()[i] == 0.0f);   // zero-filled
  t.fill(1.5f);
  Tensor c = t;                                                                // deep copy
  c.data_ptr<float>()[0] = 7.0f;
  EXPECT(t.data_ptr<float>()[0] == 1.5f);
  EXPECT(throws<std::runtime_error>([&] { (void)t.data_ptr<int8_t>(); }));     // element size check
  EXPECT(throws<std::runtime_error>([&] { (void)t.reshape(TensorShape({5, 5})); }));
  for (size_t i = 0; i < 24; ++i) t.data_ptr<float>()[i] = (float)i;
  Tensor r = t.reshape(TensorShape({4, 6}));
  EXPECT(r.shape().size(0) == 4 && r.data_ptr<float>()[23] == 23.0f);
  Tensor sl = t.slice({1, 1, 2}, {2, 3, 4});                                   // [1,2,2]
  EXPECT(sl.shape().total_size() == 4);
  EXPECT(sl.data_ptr<float>()[0] == 12 + 4 + 2 && sl.data_ptr<float>()[3] == 12 + 8 + 3);
  EXPECT(throws<std::runtime_error>([&] { (void)t.slice({0, 0, 0}, {1, 1}); }));
  EXPECT(throws<std::runtime_error>([&] { (void)t.slice({0, 2, 0}, {1, 2, 1}); }));
  Tensor m = std::move(c);
  EXPECT(m.data_ptr<float>()[0] == 7.0f && c.empty());
  Tensor e;
  EXPECT(e.empty());
  EXPECT(std::string(core::dtype_to_string(DataType::kInt8)) == "int8" && core::get_dtype_size(DataType::kFloat16) == 2);
  // ModelData container
  model::ModelData md;
  md.add_tensor("a", Tensor(TensorShape({2, 2})));
  EXPECT(md.has_tensor("a") && md.num_tensors() == 1 && md.get_tensor("b") == nullptr && md.total_memory_usage() == 16);
  EXPECT(!md.validate());   // no name / architecture
  md.metadata().name = "m";
  md.metadata().architecture = "llama";
  EXPECT(md.validate());
  EXPECT(throws<std::runtime_error>([&] { (void)model::ModelLoader::load("x.gguf"); }));
  EXPECT(model::ModelLoader::detect_format("w.safetensors") == model::ModelFormat::kSafeTensors);
  std::cout << "ok\n";
  return 0;
}

static int quant(const std::string& xin, int bits, int sym, const std::string& out) {
  const Tensor x = read_array(xin);
  optimize::QuantizationConfig qc;
  qc.type = bits == 8 ? optimize::QuantizationType::kInt8 : optimize::QuantizationType::kInt4;
  qc.symmetric = sym != 0;
  optimize::Quantizer qz(qc);
  const optimize::QuantizationInfo info = qz.calculate_quantization_info(x);
  const Tensor q = qz.quantize_tensor(x);
  const Tensor y = qz.dequantize_tensor(q, info);
  const size_t n = x.shape().total_size();
  Tensor o(TensorShape({2 + 2 * n}), DataType::kFloat32);
  float* p = o.data_ptr<float>();
  p[0] = info.scales.at(0);
  p[1] = info.zero_points.at(0);
  for (size_t i = 0; i < n; ++i) {
    const float qv = bits == 8 ? (float)q.data_ptr<int8_t>()[i] : (float)q.data_ptr<int32_t>()[i];
    p[2 + i] = qv;
    p[2 + n + i] = y.data_ptr<float>()[i];
  }
  write_array(out, o);
  return 0;
}

static int op(int argc, char** argv) {
  const std::string name = argv[2], out = argv[3];
  core::TensorEngine te(core::ComputeDevice::kGPU);
  auto in = [&](int i) { return read_array(argv[4 + i]); };
  Tensor y;
  if (name == "matmul") y = te.matmul(in(0), in(1));
  else if (name == "rms_norm") y = te.rms_norm(in(0), in(1), std::stof(argv[6]));
  else if (name == "rope") y = te.apply_rope(in(0), in(1), std::stof(argv[6]));
  else if (name == "relu") y = te.relu(in(0));
  else if (name == "silu") y = te.silu(in(0));
  else if (name == "add") y = te.add(in(0), in(1));
  else if (name == "mul") y = te.multiply(in(0), in(1));
  else if (name == "softmax") y = te.softmax(in(0), std::stof(argv[5]));
  else if (name == "attention") y = te.attention_fast_incremental(in(0), in(1), in(2));
  else if (name == "mha") y = te.multi_head_attention(in(0), in(1), in(2), (size_t)std::stoul(argv[7]));
  else if (name == "attn_general") {   // heads (0: TensorEngine::attention), mask file or "-"
    const size_t heads = (size_t)std::stoul(argv[7]);
    const bool masked = std::string(argv[8]) != "-";
    const Tensor mask = masked ? read_array(argv[8]) : Tensor(TensorShape({1}), DataType::kFloat32);
    const Tensor* mp = masked ? &mask : nullptr;
    y = heads == 0 ? te.attention(in(0), in(1), in(2), mp) : te.multi_head_attention(in(0), in(1), in(2), heads, mp);
  }
  else throw std::runtime_error("unknown op " + name);
  (void)argc;
  write_array(out, y);
  return 0;
}

// model_dir/manifest.txt: "meta vocab hidden layers heads inter rope_theta" then "<name> <file>" lines
static int run_generate(const model::ModelData& md, const std::string& prompts_file, int n_new, int top_k, int bits,
                        const std::string& out);

static int generate(const std::string& dir, const std::string& prompts_file, int n_new, int top_k, int bits,
                    const std::string& out) {
  model::ModelData md;
  std::ifstream man(dir + "/manifest.txt");
  std::string tag;
  man >> tag >> md.metadata().vocab_size >> md.metadata().hidden_size >> md.metadata().num_layers >>
      md.metadata().num_heads >> md.metadata().intermediate_size >> md.metadata().rope_theta;
  if (tag != "meta") throw std::runtime_error("manifest: expected meta line");
  md.metadata().name = "api_check";
  md.metadata().architecture = "llama";
  std::string name, file;
  while (man >> name >> file) md.add_tensor(name, read_array(dir + "/" + file));
  return run_generate(md, prompts_file, n_new, top_k, bits, out);
}

// the same from a GGUF file (ModelLoader::load; llama.cpp tensor names)
static int generate_gguf(const std::string& path, const std::string& prompts_file, int n_new, int top_k, int bits,
                         const std::string& out) {
  return run_generate(model::ModelLoader::load(path), prompts_file, n_new, top_k, bits, out);
}

static int run_generate(const model::ModelData& md_in, const std::string& prompts_file, int n_new, int top_k, int bits,
                        const std::string& out) {
  model::ModelData md = md_in;
  md.metadata().extra_params["turboinfer.weight_bits"] = std::to_string(bits);   // (the MI355X option)
  const Tensor pt = read_array(prompts_file);   // i32 [n][len]
  const size_t n = pt.shape().size(0), len = pt.shape().size(1);
  std::vector<std::vector<int>> prompts(n);
  for (size_t i = 0; i < n; ++i) prompts[i].assign(pt.data_ptr<int32_t>() + i * len, pt.data_ptr<int32_t>() + (i + 1) * len);
  model::InferenceConfig cfg;
  cfg.top_k = (size_t)top_k;
  cfg.max_sequence_length = 256;
  cfg.max_batch_size = 8;
  // generate() contract checks (tests/test_cpp_api.py::test_generate_contract_matches_reference)
  if (const char* v = std::getenv("TI_TEST_EOS")) cfg.eos_token_id = std::atoi(v);
  if (const char* v = std::getenv("TI_TEST_MAXLEN")) cfg.max_sequence_length = (size_t)std::atoi(v);
  model::InferenceEngine eng(md, cfg);
  const auto res = eng.generate_batch(prompts, (size_t)n_new);
  size_t width = 0;
  for (const auto& r : res) width = std::max(width, r.tokens.size());
  Tensor o(TensorShape({n, width}), DataType::kInt32);
  o.fill<int32_t>(-1);
  for (size_t i = 0; i < n; ++i)
    for (size_t j = 0; j < res[i].tokens.size(); ++j) o.data_ptr<int32_t>()[i * width + j] = res[i].tokens[j];
  write_array(out, o);
  std::cout << res[0].stop_reason << "\n";
  std::printf("finished %d time_ms %.9g tokens_per_second %.9g\n", res[0].finished ? 1 : 0, (double)res[0].total_time_ms,
              (double)res[0].tokens_per_second);
  std::cout << eng.performance_stats();
  return 0;
}

// model_dir/tinq_manifest.txt: "meta <name> <arch> <version> <vocab> <hidden> <layers> <heads> <inter>
// <rope_theta>" then "<tensor name> <file>" lines, added in that order
static int tinq_save(const std::string& dir, int bits, int sym, const std::string& out) {
  model::ModelData md;
  std::ifstream man(dir + "/tinq_manifest.txt");
  std::string tag;
  auto& m = md.metadata();
  man >> tag >> m.name >> m.architecture >> m.version >> m.vocab_size >> m.hidden_size >> m.num_layers >> m.num_heads >>
      m.intermediate_size >> m.rope_theta;
  if (tag != "meta") throw std::runtime_error("tinq_manifest: expected meta line");
  std::string name, file;
  while (man >> name >> file) md.add_tensor(name, read_array(dir + "/" + file));
  optimize::QuantizationConfig qc;
  qc.type = bits == 8 ? optimize::QuantizationType::kInt8 : optimize::QuantizationType::kInt4;
  qc.symmetric = sym != 0;
  optimize::Quantizer qz(qc);
  qz.save_quantized_model(qz.quantize_model(md), out);
  return 0;
}

// ModelData -> <out>.meta (text) + <out>.data (the tensors' raw bytes in the .meta order):
// the dump tests/test_gguf.py compares between this library, the reference and the oracle.
static void dump_model_data(const turboinfer::model::ModelData& md, const std::string& out) {
  const auto& m = md.metadata();
  std::ofstream meta(out + ".meta"), data(out + ".data", std::ios::binary);
  char rope[32];
  std::snprintf(rope, sizeof rope, "%.9g", (double)m.rope_theta);
  meta << m.name << "\n" << m.architecture << "\n" << m.version << "\n" << m.vocab_size << " " << m.hidden_size << " "
       << m.num_layers << " " << m.num_heads << " " << m.intermediate_size << " " << rope << "\n";
  std::vector<std::string> keys;
  for (const auto& kv : m.extra_params) keys.push_back(kv.first);
  std::sort(keys.begin(), keys.end());
  meta << keys.size() << "\n";
  for (const auto& k : keys) meta << k << "\t" << m.extra_params.at(k) << "\n";
  const auto names = md.tensor_names();
  meta << names.size() << "\n";
  for (const auto& n : names) {
    const auto* t = md.get_tensor(n);
    const bool h = t->dtype() == turboinfer::core::DataType::kFloat16;
    meta << n << " " << (h ? 3 : 0) << " " << t->shape().ndim();
    for (size_t d : t->shape().dimensions()) meta << " " << d;
    meta << "\n";
    if (t->byte_size()) data.write((const char*)t->data(), (std::streamsize)t->byte_size());
  }
}

static int gguf_load(const std::string& in, const std::string& out) {
  dump_model_data(model::ModelLoader::load(in), out);
  return 0;
}

static int tinq_load(const std::string& in, const std::string& dir) {
  const model::ModelData md = optimize::Quantizer::load_quantized_model(in);
  const auto& m = md.metadata();
  std::ofstream meta(dir + "/meta.txt"), names(dir + "/names.txt");
  meta << m.name << " " << m.architecture << " " << m.version << " " << m.vocab_size << " " << m.hidden_size << " "
       << m.num_layers << " " << m.num_heads << " " << m.intermediate_size << " " << m.rope_theta << "\n";
  int i = 0;
  for (const auto& n : md.tensor_names()) {
    names << n << "\n";
    write_array(dir + "/" + std::to_string(i++) + ".bin", *md.get_tensor(n));
  }
  return 0;
}

// A ModelData with metadata and no tensors: the engine's synthetic model only when asked
// ("turboinfer.synthetic" in extra_params or TI_SYNTHETIC=1), otherwise InferenceEngine throws.
static int tensorless(int ask) {
  model::ModelData md;
  auto& m = md.metadata();
  m.name = "tensorless";
  m.architecture = "llama";
  m.vocab_size = 512;
  m.hidden_size = 256;
  m.num_layers = 2;
  m.num_heads = 4;
  m.intermediate_size = 512;
  if (ask) m.extra_params["turboinfer.synthetic"] = "1";
  model::InferenceConfig cfg;
  cfg.max_sequence_length = 64;
  try {
    model::InferenceEngine eng(md, cfg);
    const auto r = eng.generate(std::vector<int>{1, 2, 3}, 4);
    std::cout << "built " << r.tokens.size() << "\n";
  } catch (const std::runtime_error& e) {
    std::cout << "threw " << e.what() << "\n";
  }
  return 0;
}

// TensorEngine's device (TI_GPU_INDEX) and one op on it
static int tensor_engine_device() {
  core::TensorEngine te(core::ComputeDevice::kGPU);
  std::cout << te.device_info() << "\n";
  Tensor a(TensorShape({4}), DataType::kFloat32), b(TensorShape({4}), DataType::kFloat32);
  for (int i = 0; i < 4; ++i) a.data_ptr<float>()[i] = b.data_ptr<float>()[i] = (float)i;
  const Tensor c = te.add(a, b);
  std::cout << "add " << c.data_ptr<float>()[3] << "\n";
  return 0;
}

int main(int argc, char** argv) {
  try {
    if (argc < 2) throw std::runtime_error("usage: api_check tensor|quant|op|generate ...");
    const std::string mode = argv[1];
    if (mode == "tensor") return tensor_checks();
    if (mode == "tensorless" && argc == 3) return tensorless(std::atoi(argv[2]));
    if (mode == "tensor_engine_device") return tensor_engine_device();
    if (mode == "quant" && argc == 6) return quant(argv[2], std::atoi(argv[3]), std::atoi(argv[4]), argv[5]);
    if (mode == "op" && argc >= 5) return op(argc, argv);
    if (mode == "tinq_save" && argc == 6) return tinq_save(argv[2], std::atoi(argv[3]), std::atoi(argv[4]), argv[5]);
    if (mode == "tinq_load" && argc == 4) return tinq_load(argv[2], argv[3]);
    if (mode == "gguf_load" && argc == 4) return gguf_load(argv[2], argv[3]);
    if (mode == "generate_gguf" && argc == 8)
      return generate_gguf(argv[2], argv[3], std::atoi(argv[4]), std::atoi(argv[5]), std::atoi(argv[6]), argv[7]);
    if (mode == "generate" && argc == 8)
      return generate(argv[2], argv[3], std::atoi(argv[4]), std::atoi(argv[5]), std::atoi(argv[6]), argv[7]);
    throw std::runtime_error("bad arguments for mode " + mode);
  } catch (const std::exception& e) {
    std::cerr << "api_check: " << e.what() << "\n";
    return 2;
  }
}
