#!/bin/bash
# Round 6, late (update loop and tail): the whole -m gpu suite, the default bench line, the headline-only kernel stats,
# the pcap2mgen stage timing
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/suite_r06g.log 2>&1; rc=$?
tail -4 gpurun_out/suite_r06g.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench.py > gpurun_out/bench_r06g.log 2>&1 || { tail -5 gpurun_out/bench_r06g.log; exit 1; }
tail -c 600 gpurun_out/bench_r06g.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/benchprof_r06g -o bench -- python3 -u bench.py --no-extras --steps 50 --warmup 5 > gpurun_out/benchprof_r06g.log 2>&1 || exit $?
python3 scripts/kstats.py gpurun_out/benchprof_r06g 4 || true
timeout -k 10 300 python3 scripts/pcap_time.py || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c4prof_r06g -o c4 -- python3 -u scripts/c4_only.py > gpurun_out/c4prof_r06g.log 2>&1 || exit $?
python3 scripts/kstats.py gpurun_out/c4prof_r06g 12 || true
