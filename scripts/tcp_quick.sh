# TCP transmit: the byte-exact tests (tests/test_gpu_tcp_tx.py, config-5 scans over the
# built stream), config 5's transmit timing, and a rocprofv3 kernel summary of the timing
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_tcp_tx.py tests/test_gpu_scan.py -m gpu -x -q --timeout 120 --timeout-method thread -k "tcp_tx or config5" > gpurun_out/tcp_tests.log 2>&1; rc=$?; tail -3 gpurun_out/tcp_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u scripts/tcp_time.py > gpurun_out/tcp_time.log 2>&1; rc=$?; grep tcp_tx gpurun_out/tcp_time.log; [ $rc -ne 0 ] && exit $rc
rm -rf gpurun_out/tcp_prof
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tcp_prof -o tcp -- python3 scripts/tcp_time.py > gpurun_out/tcp_prof.log 2>&1; rc=$?
grep tcp_tx gpurun_out/tcp_prof.log; exit $rc
