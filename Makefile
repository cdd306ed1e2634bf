# Top-level build: the product library (gfx950 HIP) and the CPU oracle (tests only).
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-function

LIB := grapevine_amd/libgvstore.so
SRCS := grapevine_amd/csrc/gvs_engine.hip
HDRS := grapevine_amd/csrc/gvs_kernels.h grapevine_amd/csrc/gvs_device.h grapevine_amd/csrc/gvs_route.h grapevine_amd/csrc/gvs_crypto.h grapevine_amd/csrc/gvs_seal_dev.h include/gvstore.h

all: $(LIB) oracle

$(LIB): $(SRCS) $(HDRS)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(SRCS) -lrccl

oracle:
	$(MAKE) -C oracle

clean:
	rm -f $(LIB)
	$(MAKE) -C oracle clean

.PHONY: all oracle clean
