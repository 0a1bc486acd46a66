# Top-level build of the MI355X (gfx950) numerics library and the C++ host layer.
# `make -j8` (also driven by __graft_entry__.build()).
HIPCC    ?= /opt/rocm/bin/hipcc
CXX      ?= g++
ARCH     ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-function -Wno-unused-result -Wno-unused-value
BUILD    := build
LIBDIR   := gpr_amd/lib

HIP_SRCS := $(wildcard gpr_amd/csrc/*.hip)
CPP_SRCS := $(wildcard gpr_amd/csrc/*.cpp)
HIP_OBJS := $(patsubst gpr_amd/csrc/%.hip,$(BUILD)/%.o,$(HIP_SRCS))
CPP_OBJS := $(patsubst gpr_amd/csrc/%.cpp,$(BUILD)/%.o,$(CPP_SRCS))
HDRS     := $(wildcard gpr_amd/csrc/*.h) include/gprx.h

all: $(LIBDIR)/libgprx.so oracle

$(BUILD)/%.o: gpr_amd/csrc/%.hip $(HDRS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/%.o: gpr_amd/csrc/%.cpp $(HDRS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

$(LIBDIR)/libgprx.so: $(HIP_OBJS) $(CPP_OBJS) | $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $^ -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib

oracle:
	$(MAKE) -s -C oracle

$(BUILD) $(LIBDIR):
	mkdir -p $@

clean:
	rm -rf $(BUILD) $(LIBDIR)/*.so
	$(MAKE) -s -C oracle clean

.PHONY: all oracle clean
