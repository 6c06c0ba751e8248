#!/bin/bash
# Builds of the product library with other detect geometries (MGENX_SCAN_BLOCK bytes per
# workgroup, MGENX_SCAN_THREADS threads) into mgen_amd/exp/, for scripts/scan_time.py with
# MGENX_LIB_OVERRIDE=mgen_amd/exp/libmgenx_<tag>.so.  CPU side (hipcc cross-compiles).
set -eu
cd "$(dirname "$0")/.."
geoms=("$@")
[ ${#geoms[@]} -eq 0 ] && geoms=(65536:512 32768:256 65536:1024 131072:512)
for g in "${geoms[@]}"; do
  blk=${g%%:*}; thr=${g##*:}; tag=b${blk}_t${thr}
  mkdir -p build/exp_$tag
  objs=""
  for n in mgenx_api mgenx_unpack mgenx_pack mgenx_scan mgenx_analytic mgenx_log mgenx_comm \
           mgenx_flowtab mgenx_tcp mgenx_rx mgenx_pcap; do
    if [ $n = mgenx_scan ]; then
      /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -DMGENX_DIAG=0 \
        -DMGENX_SCAN_BLOCK=$blk -DMGENX_SCAN_THREADS=$thr -Iinclude -Imgen_amd/csrc \
        -c mgen_amd/csrc/$n.hip -o build/exp_$tag/$n.o
      objs="$objs build/exp_$tag/$n.o"
    else
      objs="$objs build/product/$n.o"
    fi
  done
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared $objs -o mgen_amd/exp/libmgenx_$tag.so \
    -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
  echo built mgen_amd/exp/libmgenx_$tag.so
done
