# Build librdeic_hip.so (HIP kernels for gfx950 + host C++ coders) in-tree.
HIPCC ?= /opt/rocm/bin/hipcc
CXX ?= g++
ARCH ?= gfx950
BUILD ?= build
LIBDIR ?= rdeic_amd/lib
LIB := $(LIBDIR)/librdeic_hip.so
HIP_SRCS := $(wildcard rdeic_amd/csrc/*.hip)
CPP_SRCS := $(wildcard rdeic_amd/csrc/*.cpp)
HIP_OBJS := $(patsubst rdeic_amd/csrc/%.hip,$(BUILD)/%.hip.o,$(HIP_SRCS))
CPP_OBJS := $(patsubst rdeic_amd/csrc/%.cpp,$(BUILD)/%.cpp.o,$(CPP_SRCS))
HIPFLAGS := -O3 -fPIC -std=c++17 --offload-arch=$(ARCH) -Wall -Wno-unused-variable -Wno-unused-but-set-variable $(EXTRA_HIPFLAGS)
CXXFLAGS := -O3 -fPIC -std=c++17 -Wall -pthread

all: $(LIB) oracle

$(BUILD)/%.hip.o: rdeic_amd/csrc/%.hip rdeic_amd/csrc/common.h rdeic_amd/csrc/conv_common.h rdeic_amd/csrc/prof.h include/rdeic_hip.h
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/%.cpp.o: rdeic_amd/csrc/%.cpp include/rdeic_hip.h
	@mkdir -p $(BUILD)
	$(CXX) $(CXXFLAGS) -c $< -o $@

$(LIB): $(HIP_OBJS) $(CPP_OBJS)
	@mkdir -p $(LIBDIR)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $^ -lpthread

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf $(BUILD) $(LIB)
	$(MAKE) -C oracle clean

.PHONY: all clean oracle

# attention: MFMA results in VGPRs (the softmax reads every score; in AGPRs each one costs a
# v_accvgpr_read/write pair per tile, ~180 extra VALU instructions per 64-key tile)
$(BUILD)/attention.hip.o: HIPFLAGS += -mllvm -amdgpu-mfma-vgpr-form=1

# parity-sensitive scalar kernels: no fma contraction anywhere in these TUs (headers included)
$(BUILD)/elementwise.hip.o $(BUILD)/entropy.hip.o: HIPFLAGS += -ffp-contract=off

# conv kernels: no SLP vectorisation (packed-f32 VALU beside MFMAs is an anti-lever on gfx950,
# MI355X_MICROARCH.md constants table; measured r04 on the halo conv: -1 to -2% time)
$(BUILD)/conv_gemm.hip.o $(BUILD)/conv_dma.hip.o $(BUILD)/conv_halo.hip.o $(BUILD)/conv_edge.hip.o: HIPFLAGS += -fno-slp-vectorize
