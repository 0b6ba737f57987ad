#!/bin/bash
# The per-pop ABI (kbhost: sync / pipelined) beside kbhip_allocate at C4, C3
# and C5 (logs equal), and the C5 what-if sessions alone / 16 in flight,
# grouped and not.
set -o pipefail
TAG=${1:-r04h}
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
for CFG in c3 c5 c4; do
  timeout -k 10 600 python -u profiles/host_loop.py --config $CFG --reps 3 --out gpurun_out/$TAG/host_loop_$CFG.json \
      > gpurun_out/$TAG/host_loop_$CFG.log 2>&1 || { tail -20 gpurun_out/$TAG/host_loop_$CFG.log; exit 1; }
  tail -1 gpurun_out/$TAG/host_loop_$CFG.log | cut -c1-600
done
timeout -k 10 400 python -u bench_c5.py --concurrent 1 --sessions 5 --warmup 1 --cpu-baseline 0 > gpurun_out/$TAG/c5_alone.json 2> gpurun_out/$TAG/c5_alone.err || exit 1
cat gpurun_out/$TAG/c5_alone.json
for G in 0 1; do
  timeout -k 10 400 python -u bench_c5.py --concurrent 16 --sessions 16 --warmup 1 --group $G --cpu-baseline 0 \
      > gpurun_out/$TAG/c5_g${G}_c16.json 2> gpurun_out/$TAG/c5_g${G}_c16.err || exit 1
  cat gpurun_out/$TAG/c5_g${G}_c16.json
done
