// library.cpp -- turboinfer:: library functions of the umbrella header (turboinfer.hpp).
#include <stdexcept>
#include <string>

#include "ti_hip.h"
#include "turboinfer/turboinfer.hpp"

namespace turboinfer {

namespace {
bool g_initialized = false;
}

const char* build_info() {
  static std::string info;
  int count = 0;
  ti_device_count(&count);
  info = std::string("turboinfer-mi355x ") + Version::kString + " (HIP kernels for gfx950, " + std::to_string(count) +
         " device(s) visible)";
  return info.c_str();
}

bool initialize(bool) {
  int count = 0;
  if (ti_device_count(&count) != TI_OK || count < 1) return false;
  g_initialized = ti_init(0) == TI_OK;
  return g_initialized;
}

void shutdown() { g_initialized = false; }
bool is_initialized() { return g_initialized; }

std::vector<int> tokenize(const std::string&, const std::string&) {
  throw std::runtime_error("turboinfer::tokenize: the tokenizer is not part of the MI355X decode hot path");
}
std::string detokenize(const std::vector<int>&, const std::string&) {
  throw std::runtime_error("turboinfer::detokenize: the tokenizer is not part of the MI355X decode hot path");
}

}  // namespace turboinfer
