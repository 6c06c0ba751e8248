# Builds the product library (gfx950) and the test-only oracle.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -Wno-unused-value
SRC := mgen_amd/csrc/mgenx_api.hip mgen_amd/csrc/mgenx_unpack.hip mgen_amd/csrc/mgenx_pack.hip \
       mgen_amd/csrc/mgenx_scan.hip mgen_amd/csrc/mgenx_analytic.hip
HDR := include/mgenx.h mgen_amd/csrc/mgenx_common.hpp mgen_amd/csrc/mgenx_kernels.hpp

all: mgen_amd/libmgenx.so oracle

mgen_amd/libmgenx.so: $(SRC) $(HDR)
	$(HIPCC) --offload-arch=$(ARCH) $(HIPFLAGS) -shared -Iinclude -Imgen_amd/csrc $(SRC) -o $@

oracle:
	$(MAKE) -s -C oracle

clean:
	rm -f mgen_amd/libmgenx.so
	$(MAKE) -s -C oracle clean

.PHONY: all oracle clean
