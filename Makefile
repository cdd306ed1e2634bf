# Top-level build: the product library (gfx950 HIP), the same engine with the
# test hooks of include/gvstore_test.h, and the CPU oracle (tests only).
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
# bitwise & and | on bools are deliberate in the kernels: no short-circuit
# branches that skip code by the data (DESIGN.md §3 rule 6)
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-function -Wno-bitwise-instead-of-logical

LIB := grapevine_amd/libgvstore.so
TESTLIB := grapevine_amd/libgvstore_test.so
SRCS := grapevine_amd/csrc/gvs_engine.hip
HDRS := $(wildcard grapevine_amd/csrc/*.h) include/gvstore.h include/gvstore_test.h

SRHOST := tests/libsrhost.so

all: $(LIB) $(TESTLIB) $(SRHOST) oracle

$(LIB): $(SRCS) $(HDRS)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(SRCS) -lrccl

$(TESTLIB): $(SRCS) $(HDRS)
	$(HIPCC) $(HIPFLAGS) -DGVS_TEST_HOOKS -shared -o $@ $(SRCS) -lrccl

# the device signature-check arithmetic built for the CPU (tests/test_sr_host.py)
$(SRHOST): tests/sr_host.cpp grapevine_amd/csrc/gvs_sr25519.h grapevine_amd/csrc/gvs_device.h
	$(HIPCC) -O2 -std=c++17 -fPIC -shared --offload-arch=$(ARCH) -o $@ tests/sr_host.cpp

oracle:
	$(MAKE) -C oracle

clean:
	rm -f $(LIB) $(TESTLIB) $(SRHOST)
	$(MAKE) -C oracle clean

.PHONY: all oracle clean
