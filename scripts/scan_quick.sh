set -u
mkdir -p gpurun_out
timeout -k 10 120 python -u scripts/scan_time.py > gpurun_out/scan_time.log 2>&1; rc=$?; tail -5 gpurun_out/scan_time.log; exit $rc
