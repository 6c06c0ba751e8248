# A/B: the working tree's libmgenx.so against mgen_amd/libmgenx_ab.so (a baseline build),
# interleaved runs of scripts/tcp_time.py (config 5's TCP transmit)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/ab_tcp.log
for k in 1 2 3; do
  for side in new old; do
    if [ $side = old ]; then export MGENX_LIB_OVERRIDE=$PWD/mgen_amd/libmgenx_ab.so; else unset MGENX_LIB_OVERRIDE; fi
    timeout -k 10 120 python -u scripts/tcp_time.py 2>/dev/null | sed "s/^/$side /" >> gpurun_out/ab_tcp.log || exit 1
  done
done
cat gpurun_out/ab_tcp.log
