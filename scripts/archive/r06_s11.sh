#!/bin/bash
# round 6: pack grid sweep (diagnostics build; workgroups per CU)
set -u
export TMPDIR=/tmp
D=$PWD/mgen_amd/libmgenx_diag.so
for g in 256 384 512 1024; do
  echo "grid $g"; MGENX_PACK_GRID=$g MGENX_LIB_OVERRIDE=$D timeout -k 10 120 python3 scripts/pack_time.py || exit 1
  MGENX_PACK_GRID=$g MGENX_LIB_OVERRIDE=$D timeout -k 10 120 python3 scripts/tcp_time.py || exit 1
done
