# Build of the MI355X-native Gauss-Jordan framework (reference build: Makefile:1-6, mpicxx -Ofast).
#
#   make            -> build/gj (CLI) + mpi_jordan_crazy_acceleration_amd/_C<ext>.so (Python module)
#   make cli | py   -> one of them
#   make clean
#
# Everything is compiled for gfx950 only.  Code object v5 keeps the objects loadable by the HIP
# runtime bundled with torch (ROCm 7.0) as well as by /opt/rocm (7.2).
ROCM      ?= /opt/rocm
HIPCC     ?= $(ROCM)/bin/hipcc
ARCH      ?= gfx950
PYTHON    ?= python3
BUILD     := build
PKG       := mpi_jordan_crazy_acceleration_amd

CXXSTD    := -std=c++17
COMMON    := -O3 -fPIC $(CXXSTD) -Icsrc/include -Wall -Wno-unused-result
HIPFLAGS  := $(COMMON) --offload-arch=$(ARCH) -mcode-object-version=5 -munsafe-fp-atomics
HOSTFLAGS := $(COMMON) -x c++ -D__HIP_PLATFORM_AMD__ -I$(ROCM)/include
LDLIBS    := -L$(ROCM)/lib -lrccl -lamdhip64 -lrocprofiler-sdk-roctx -lpthread

KERNELS   := gemm blockinv blockinv_mfma blockinv_big blockinv_huge misc
HOST_SRC  := solver/engine solver/runner runtime/host_device runtime/hip_device \
             runtime/loopback_comm runtime/async_loopback_comm runtime/async_host_device \
             runtime/shadow_comm runtime/rccl_comm runtime/comm runtime/race_check io/matrix_io

KOBJ      := $(patsubst %,$(BUILD)/kernels/%.o,$(KERNELS))
HOBJ      := $(patsubst %,$(BUILD)/%.o,$(HOST_SRC))
CORE      := $(KOBJ) $(HOBJ)

PYEXT     := $(shell $(PYTHON) -c "import sysconfig;print(sysconfig.get_config_var('EXT_SUFFIX'))")
PYINC     := $(shell $(PYTHON) -c "import sysconfig,pybind11;print('-I'+sysconfig.get_paths()['include'],'-I'+pybind11.get_include())")
PYMOD     := $(PKG)/_C$(PYEXT)

HEADERS   := $(wildcard csrc/include/gj/*.hpp) $(wildcard csrc/kernels/*.hpp)

# Host-code sanitizer build: the host runtime, engine, communicators and I/O
# under ASan + UBSan; device code is not instrumented (GPU sanitizers are not available here).
SANFLAGS  := -fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer -fno-gpu-sanitize
ASANOBJ   := $(patsubst %,$(BUILD)/asan/%.o,$(HOST_SRC) cli/main)

.PHONY: all cli py clean asan
all: cli py
cli: $(BUILD)/gj
py: $(PYMOD)

$(BUILD)/kernels/%.o: csrc/kernels/%.hip $(HEADERS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/%.o: csrc/%.cpp $(HEADERS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HOSTFLAGS) -c $< -o $@

$(BUILD)/cli/main.o: csrc/cli/main.cpp $(HEADERS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HOSTFLAGS) -c $< -o $@

$(BUILD)/python/module.o: csrc/python/module.cpp $(HEADERS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HOSTFLAGS) $(PYINC) -fvisibility=hidden -c $< -o $@

$(BUILD)/gj: $(CORE) $(BUILD)/cli/main.o
	$(HIPCC) --offload-arch=$(ARCH) -o $@ $^ $(LDLIBS) -Wl,-rpath,$(ROCM)/lib

$(PYMOD): $(CORE) $(BUILD)/python/module.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $^ $(LDLIBS)

asan: $(BUILD)/gj_asan
$(BUILD)/asan/%.o: csrc/%.cpp $(HEADERS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HOSTFLAGS) -O1 $(SANFLAGS) -c $< -o $@
$(BUILD)/gj_asan: $(KOBJ) $(ASANOBJ)
	$(HIPCC) --offload-arch=$(ARCH) -fsanitize=address,undefined -fno-gpu-sanitize -o $@ $^ $(LDLIBS) -Wl,-rpath,$(ROCM)/lib

clean:
	rm -rf $(BUILD) $(PKG)/_C*.so
