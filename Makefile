# Builds the product library (gfx950), the diagnostics library and the test-only oracle.
#   mgen_amd/libmgenx.so       product: the C ABI of include/mgenx.h (nothing else exported)
#   mgen_amd/libmgenx_diag.so  the same kernels plus the ablation variants and memory probes
#                              of include/mgenx_diag.h (benchmark scripts only)
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -Wno-unused-value -Wno-int-to-pointer-cast
NAMES := mgenx_api mgenx_unpack mgenx_pack mgenx_scan mgenx_analytic mgenx_log mgenx_comm mgenx_worker \
         mgenx_flowtab mgenx_tcp mgenx_rx mgenx_pcap
HDR := include/mgenx.h include/mgenx_diag.h mgen_amd/csrc/mgenx_common.hpp mgen_amd/csrc/mgenx_kernels.hpp \
       mgen_amd/csrc/mgenx_flowsm.hpp \
       mgen_amd/csrc/mgenx_parse.hpp
OBJ := $(addprefix build/product/,$(addsuffix .o,$(NAMES)))
DOBJ := $(addprefix build/diag/,$(addsuffix .o,$(NAMES)))
LIBS := -L/opt/rocm/lib -lrccl -lhsa-runtime64 -Wl,-rpath,/opt/rocm/lib

all: mgen_amd/libmgenx.so mgen_amd/libmgenx_diag.so oracle tests/cpp/host_roundtrip \
     tests/cpp/loopback tests/cpp/compat_shapes tests/cpp/compat_shapes_pl tests/cpp/shim_latency \
     tests/cpp/shard_scan tools/pcap2mgen

build/product/%.o: mgen_amd/csrc/%.hip $(HDR)
	@mkdir -p build/product
	$(HIPCC) --offload-arch=$(ARCH) $(HIPFLAGS) -DMGENX_DIAG=0 -Iinclude -Imgen_amd/csrc -c $< -o $@

build/diag/%.o: mgen_amd/csrc/%.hip $(HDR)
	@mkdir -p build/diag
	$(HIPCC) --offload-arch=$(ARCH) $(HIPFLAGS) -DMGENX_DIAG=1 -Iinclude -Imgen_amd/csrc -c $< -o $@

mgen_amd/libmgenx.so: $(OBJ)
	$(HIPCC) --offload-arch=$(ARCH) -shared $(OBJ) -o $@ $(LIBS)

mgen_amd/libmgenx_diag.so: $(DOBJ)
	$(HIPCC) --offload-arch=$(ARCH) -shared $(DOBJ) -o $@ $(LIBS)

HOSTCXX := g++ -O2 -std=c++17 -D__HIP_PLATFORM_AMD__ -Iinclude -I/opt/rocm/include
HOSTLD := -Lmgen_amd -lmgenx -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,'$$ORIGIN/../../mgen_amd' \
          -Wl,-rpath,/opt/rocm/lib

# C++ host-layer test program (include/mgenx.hpp), plain g++ against the C ABI
tests/cpp/host_roundtrip: tests/cpp/host_roundtrip.cpp include/mgenx.hpp include/mgenx.h mgen_amd/libmgenx.so
	$(HOSTCXX) $< -o $@ $(HOSTLD)

# config 1 (UDP over loopback): CPU path through the test-only oracle, GPU path through libmgenx
tests/cpp/loopback: tests/cpp/loopback.cpp include/mgenx.hpp include/mgenx_io.hpp include/mgenx.h \
		mgen_amd/libmgenx.so oracle
	$(HOSTCXX) -Ioracle $< -o $@ -Loracle/build -loracle -Wl,-rpath,'$$ORIGIN/../../oracle/build' \
	    $(HOSTLD)

# the reference's own call shapes compiled against the MgenMsg/MgenPayload/MgenAnalytic shim
COMPAT := $(wildcard include/mgenx_compat/*.h include/mgenx_compat/*.hpp) \
          include/mgenx_compat/mgenx_compat.cpp
tests/cpp/compat_shapes: tests/cpp/compat_shapes.cpp $(COMPAT) include/mgenx.h mgen_amd/libmgenx.so
	$(HOSTCXX) -Iinclude/mgenx_compat $< include/mgenx_compat/mgenx_compat.cpp -o $@ $(HOSTLD)

# mgenx::ShardedScan over simulated ranks (threads) and a one-rank RCCL communicator
tests/cpp/shard_scan: tests/cpp/shard_scan.cpp include/mgenx.hpp include/mgenx.h mgen_amd/libmgenx.so
	$(HOSTCXX) $< -o $@ $(HOSTLD) -lpthread

# per-call latency of the shim's single-message calls (batches of one) and batch forms
tests/cpp/shim_latency: tests/cpp/shim_latency.cpp $(COMPAT) include/mgenx.h mgen_amd/libmgenx.so
	$(HOSTCXX) -Iinclude/mgenx_compat $< include/mgenx_compat/mgenx_compat.cpp -o $@ $(HOSTLD)

# the same program through the shim's MGENX_WITH_PROTOLIB branch (what an MGEN build compiles),
# against protolib / Mgen-shaped test headers (tests/cpp/protolib_shape)
PLSHAPE := $(wildcard tests/cpp/protolib_shape/*)
tests/cpp/compat_shapes_pl: tests/cpp/compat_shapes.cpp $(COMPAT) $(PLSHAPE) include/mgenx.h \
		mgen_amd/libmgenx.so
	$(HOSTCXX) -DMGENX_WITH_PROTOLIB -Iinclude/mgenx_compat -Itests/cpp/protolib_shape $< \
	    include/mgenx_compat/mgenx_compat.cpp tests/cpp/protolib_shape/mgen_shape.cpp -o $@ $(HOSTLD)

# the reference's pcap2mgen command line over mgenx::Pcap2Mgen (include/mgenx_pcap.hpp)
tools/pcap2mgen: tools/pcap2mgen.cpp include/mgenx_pcap.hpp include/mgenx.hpp include/mgenx.h \
		mgen_amd/libmgenx.so
	$(HOSTCXX) $< -o $@ -Lmgen_amd -lmgenx -L/opt/rocm/lib -lamdhip64 \
	    -Wl,-rpath,'$$ORIGIN/../mgen_amd' -Wl,-rpath,/opt/rocm/lib

oracle:
	$(MAKE) -s -C oracle

clean:
	rm -rf build mgen_amd/libmgenx.so mgen_amd/libmgenx_diag.so
	$(MAKE) -s -C oracle clean

.PHONY: all oracle clean
