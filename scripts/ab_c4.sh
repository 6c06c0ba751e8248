# A/B: the working tree's libmgenx.so against mgen_amd/libmgenx_ab.so (a baseline build),
# interleaved runs of scripts/c4_only.py (config 4: reduce_ms and rank 0's share at N = 8)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/ab_c4.log
for k in 1 2 3; do
  for side in new old; do
    if [ $side = old ]; then export MGENX_LIB_OVERRIDE=$PWD/mgen_amd/libmgenx_ab.so; else unset MGENX_LIB_OVERRIDE; fi
    timeout -k 10 200 python -u scripts/c4_only.py 2>/dev/null | python3 -c "
import json,sys
d=json.loads(sys.stdin.read().strip().splitlines()[-1])
r=d.get('rank_share_at_8') or {}
print('$side', d['reduce_ms'], r.get('reduce_ms') if isinstance(r, dict) else r)" >> gpurun_out/ab_c4.log || exit 1
  done
done
cat gpurun_out/ab_c4.log
