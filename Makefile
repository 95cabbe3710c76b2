# Builds the product library turboinfer_amd/lib/libturboinfer_amd.so for gfx950 (MI355X):
#   HIP kernels (turboinfer_amd/csrc/kernels/*.hip) + the C-ABI shim and the C++20 host
#   library (turboinfer_amd/csrc/host/*.cpp, public headers under include/).
# `make test-bins` builds the C++ API tests under tests/cpp/.
# The test oracle is built separately by oracle/Makefile (never linked in here).
HIPCC   ?= /opt/rocm/bin/hipcc
ARCH    ?= gfx950
JOBS    ?= 8
BUILD   ?= build
LIBDIR  := turboinfer_amd/lib
LIB     ?= $(LIBDIR)/libturboinfer_amd.so

COMMON  := -std=c++20 -O3 -fPIC -Iinclude -Iturboinfer_amd/csrc/kernels -Wall -Wno-unused-result -Wno-unused-value
EXTRA   ?=
DEVFLAGS:= $(COMMON) --offload-arch=$(ARCH) -fno-gpu-rdc $(EXTRA)

KERN    := $(wildcard turboinfer_amd/csrc/kernels/*.hip)
HOST    := $(wildcard turboinfer_amd/csrc/host/*.cpp)
API     := $(wildcard turboinfer_amd/csrc/api/*.cpp)
KOBJ    := $(patsubst turboinfer_amd/csrc/kernels/%.hip,$(BUILD)/k_%.o,$(KERN))
HOBJ    := $(patsubst turboinfer_amd/csrc/host/%.cpp,$(BUILD)/h_%.o,$(HOST))
AOBJ    := $(patsubst turboinfer_amd/csrc/api/%.cpp,$(BUILD)/a_%.o,$(API))
HDRS    := $(wildcard include/*.h) $(wildcard include/turboinfer/*/*.hpp) $(wildcard include/turboinfer/*.hpp) \
           $(wildcard turboinfer_amd/csrc/kernels/*.hpp) $(wildcard turboinfer_amd/csrc/host/*.hpp) \
           $(wildcard turboinfer_amd/csrc/api/*.hpp)

all: $(LIB)

$(BUILD)/k_ops_exact.o: turboinfer_amd/csrc/kernels/ops_exact.hip $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(DEVFLAGS) -ffp-contract=off -c $< -o $@

# gemv: preload its leading kernel arguments into SGPRs (gfx950 kernarg preload).
# gemv, attention and qkv_attn compile without fp contraction (the rounding sequence the parity tests pin).
$(BUILD)/k_gemv.o: turboinfer_amd/csrc/kernels/gemv.hip $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(DEVFLAGS) -ffp-contract=off -mllvm -amdgpu-kernarg-preload-count=16 -c $< -o $@

$(BUILD)/k_attention.o: turboinfer_amd/csrc/kernels/attention.hip $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(DEVFLAGS) -ffp-contract=off -c $< -o $@

$(BUILD)/k_qkv_attn.o: turboinfer_amd/csrc/kernels/qkv_attn.hip $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(DEVFLAGS) -ffp-contract=off -c $< -o $@

$(BUILD)/k_%.o: turboinfer_amd/csrc/kernels/%.hip $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(DEVFLAGS) -c $< -o $@

$(BUILD)/h_%.o: turboinfer_amd/csrc/host/%.cpp $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(COMMON) -ffp-contract=off -x hip --offload-arch=$(ARCH) -c $< -o $@

# C++20 drop-in API (turboinfer::core / model / optimize): host code over the C-ABI only
$(BUILD)/a_%.o: turboinfer_amd/csrc/api/%.cpp $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(COMMON) -ffp-contract=off -c $< -o $@

$(LIB): $(KOBJ) $(HOBJ) $(AOBJ)
	@mkdir -p $(dir $@)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $(KOBJ) $(HOBJ) $(AOBJ) -Wl,-soname,libturboinfer_amd.so

# C++ API test drivers (tests/cpp/*.cpp -> tests/cpp/bin/), linked against the in-tree library
CPPTESTS := $(patsubst tests/cpp/%.cpp,tests/cpp/bin/%,$(wildcard tests/cpp/*.cpp))
test-bins: $(CPPTESTS)
tests/cpp/bin/%: tests/cpp/%.cpp $(HDRS) | $(LIB)
	@mkdir -p tests/cpp/bin
	$(HIPCC) -std=c++20 -O2 -Iinclude $< -o $@ -L$(LIBDIR) -lturboinfer_amd -Wl,-rpath,'$$ORIGIN/../../../$(LIBDIR)'

.PHONY: all clean test-bins
