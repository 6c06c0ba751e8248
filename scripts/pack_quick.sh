set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pack_layout.py tests/test_gpu_pack_msgs.py tests/test_gpu_tcp_tx.py tests/test_compat_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pack_tests.log 2>&1; rc=$?; tail -3 gpurun_out/pack_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/pack_time.py 1 > gpurun_out/pack_time.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/pack_time.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u scripts/fill_probe.py > gpurun_out/fill_probe.log 2>&1; rc=$?; tail -2 gpurun_out/fill_probe.log; exit $rc
