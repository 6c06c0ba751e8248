#!/bin/bash
# round 6: kernel-trace summaries of the extras (config 3 / 4 / 5, FindFlow, TCP transmit)
set -u
export TMPDIR=/tmp
OUT=gpurun_out
for s in c3_only c4_only c5_only ft_time tcp_time; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_r06_$s -o $s -- \
    python3 scripts/$s.py > $OUT/prof_r06_$s.log 2>&1 || { tail -20 $OUT/prof_r06_$s.log; exit 1; }
  echo "== $s"; python3 scripts/kstats.py $OUT/prof_r06_$s 8 || true
done
