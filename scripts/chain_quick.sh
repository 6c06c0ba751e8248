set -u
mkdir -p gpurun_out
timeout -k 10 120 python -u scripts/chain_prof.py > gpurun_out/chain_prof.log 2>&1; rc=$?; tail -8 gpurun_out/chain_prof.log; exit $rc
