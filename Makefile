# Builds the product library (gfx950) and the test-only oracle.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -Wno-unused-value
SRC := mgen_amd/csrc/mgenx_api.hip mgen_amd/csrc/mgenx_unpack.hip mgen_amd/csrc/mgenx_pack.hip \
       mgen_amd/csrc/mgenx_scan.hip mgen_amd/csrc/mgenx_analytic.hip \
       mgen_amd/csrc/mgenx_log.hip
HDR := include/mgenx.h mgen_amd/csrc/mgenx_common.hpp mgen_amd/csrc/mgenx_kernels.hpp

all: mgen_amd/libmgenx.so oracle tests/cpp/host_roundtrip tests/cpp/loopback

mgen_amd/libmgenx.so: $(SRC) $(HDR)
	$(HIPCC) --offload-arch=$(ARCH) $(HIPFLAGS) -shared -Iinclude -Imgen_amd/csrc $(SRC) -o $@

# C++ host-layer test program (include/mgenx.hpp), plain g++ against the C ABI
tests/cpp/host_roundtrip: tests/cpp/host_roundtrip.cpp include/mgenx.hpp include/mgenx.h mgen_amd/libmgenx.so
	g++ -O2 -std=c++17 -D__HIP_PLATFORM_AMD__ -Iinclude -I/opt/rocm/include $< -o $@ \
	    -Lmgen_amd -lmgenx -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,'$$ORIGIN/../../mgen_amd' \
	    -Wl,-rpath,/opt/rocm/lib

# config 1 (UDP over loopback): CPU path through the test-only oracle, GPU path through libmgenx
tests/cpp/loopback: tests/cpp/loopback.cpp include/mgenx.hpp include/mgenx_io.hpp include/mgenx.h \
		mgen_amd/libmgenx.so oracle
	g++ -O2 -std=c++17 -D__HIP_PLATFORM_AMD__ -Iinclude -Ioracle -I/opt/rocm/include $< -o $@ \
	    -Lmgen_amd -lmgenx -Loracle/build -loracle -L/opt/rocm/lib -lamdhip64 \
	    -Wl,-rpath,'$$ORIGIN/../../mgen_amd' -Wl,-rpath,'$$ORIGIN/../../oracle/build' \
	    -Wl,-rpath,/opt/rocm/lib

oracle:
	$(MAKE) -s -C oracle

clean:
	rm -f mgen_amd/libmgenx.so
	$(MAKE) -s -C oracle clean

.PHONY: all oracle clean
