#!/bin/bash
# round 6: config-2 pack store-wave count (diagnostics variant 10: no meta-wave help)
set -u
export TMPDIR=/tmp
timeout -k 10 300 python3 -u scripts/pack_c2_variants.py 0 10 || exit 1
MGENX_PACK_GRID=512 timeout -k 10 300 python3 -u scripts/pack_c2_variants.py 0 10 || exit 1
