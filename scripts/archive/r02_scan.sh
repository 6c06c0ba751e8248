#!/bin/bash
# scan timing variants + rocprof kernel stats
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python scripts/scan_profile.py read > gpurun_out/scan_v0.log 2>&1 || exit 3

timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/scanprof3 -o scan -- python scripts/scan_profile.py > gpurun_out/scanprof3.log 2>&1 || exit 3

grep -h "scan_ms\|stream_read_ms" gpurun_out/scan_v0.log
