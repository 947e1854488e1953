# Build for gfx950 (MI355X). Everything lands in-tree so it travels with the gpurun snapshot.
#   make            -> libyart.so (HIP, C ABI of include/yart.h), libyart_host.so (C++ host
#                      layer of include/yart_host.h), bin/yart (CLI), oracle/liboracle.so
ROOT := $(abspath .)
PKG := $(ROOT)/yet-another-raytracer_amd
LIB := $(PKG)/lib
BIN := $(PKG)/bin
GEN := $(ROOT)/build/gen
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
# -ffp-contract=off everywhere: the reference is IEEE f64 with no fused multiply-add.
CXXFLAGS := -O2 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wall -Wextra -Wno-unused-parameter
HIPFLAGS := -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -ffp-contract=off -fno-fast-math \
            -fno-gpu-rdc -Wall -Wno-unused-parameter -I$(GEN)

HOST_SRCS := $(PKG)/host/scene.cpp $(PKG)/host/presets.cpp $(PKG)/host/capi.cpp $(PKG)/host/png.cpp
HOST_HDRS := $(PKG)/host/scene.hpp $(PKG)/host/camera_impl.h $(ROOT)/include/yart.h $(ROOT)/include/yart_host.h
DEV_SRCS := $(wildcard $(PKG)/csrc/*.hip) $(wildcard $(PKG)/csrc/*.cpp)
DEV_HDRS := $(wildcard $(PKG)/csrc/*.h) $(ROOT)/include/yart.h $(PKG)/host/camera_impl.h

all: host device cli oracle
host: $(LIB)/libyart_host.so
device: $(LIB)/libyart.so
cli: $(BIN)/yart
oracle:
	$(MAKE) -C $(ROOT)/oracle

$(GEN)/cie_xyz.inc $(GEN)/smits.inc $(GEN)/srgb_steps.inc: $(ROOT)/tables/cie1931_xyz_1nm_360_830.f64 $(ROOT)/tables/smits_basis_36bin.f64 $(ROOT)/tables/srgb_u8_steps.f64 $(ROOT)/tools/gen_tables_inc.py
	python3 $(ROOT)/tools/gen_tables_inc.py $(GEN)

$(LIB)/libyart_host.so: $(HOST_SRCS) $(HOST_HDRS)
	@mkdir -p $(LIB)
	g++ $(CXXFLAGS) -shared -o $@ $(HOST_SRCS)

# build/gen/build_id.h: sha256 of the sources (yart/buildid.py), returned by yart_build_id(); the
# Python side refuses a libyart.so whose id is not the tree's (a stale prebuilt library)
$(LIB)/libyart.so: $(DEV_SRCS) $(DEV_HDRS) $(GEN)/cie_xyz.inc $(GEN)/smits.inc $(GEN)/srgb_steps.inc $(ROOT)/Makefile
	@mkdir -p $(LIB)
	python3 $(PKG)/yart/buildid.py --header $(GEN)/build_id.h
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(DEV_SRCS) -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib

$(BIN)/yart: $(PKG)/host/main.cpp $(LIB)/libyart.so $(LIB)/libyart_host.so
	@mkdir -p $(BIN)
	g++ $(CXXFLAGS) -o $@ $(PKG)/host/main.cpp -L$(LIB) -lyart -lyart_host -Wl,-rpath,'$$ORIGIN/../lib' -lpthread

clean:
	rm -rf $(LIB) $(BIN) $(GEN)
	$(MAKE) -C $(ROOT)/oracle clean
.PHONY: all host device cli oracle clean

# A/B builds for tools/ab.py: make variant NAME=x DEFS="-DYART_FOO"
variant: $(GEN)/cie_xyz.inc $(GEN)/smits.inc $(GEN)/srgb_steps.inc
	@mkdir -p $(LIB)/variants
	python3 $(PKG)/yart/buildid.py --header $(GEN)/build_id.h
	$(HIPCC) $(HIPFLAGS) $(DEFS) -shared -o $(LIB)/variants/libyart_$(NAME).so $(DEV_SRCS) -L/opt/rocm/lib -lrccl
.PHONY: variant
