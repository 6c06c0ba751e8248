set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_scan.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/scan_chain_tests.log 2>&1; rc=$?; tail -5 gpurun_out/scan_chain_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_scan.py -m gpu -x -q --timeout 120 --timeout-method thread -k "chain or pruned or config5" > gpurun_out/scan_chain_tests2.log 2>&1; rc=$?; tail -3 gpurun_out/scan_chain_tests2.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u scripts/scan_time.py > gpurun_out/scan_time.log 2>&1; rc=$?; grep -E "scan_ms|c_call|interleaved" gpurun_out/scan_time.log; exit $rc
