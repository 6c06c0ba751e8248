set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/pack_time.py 1 > gpurun_out/pack_time.log 2>&1; rc=$?; cat gpurun_out/pack_time.log | grep -v amdgpu.ids; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u scripts/fill_probe.py > gpurun_out/fill_probe.log 2>&1; rc=$?; tail -5 gpurun_out/fill_probe.log; exit $rc
