#!/bin/bash
# r06: the engine's polling shape: the C4 bench line for
# the product library (8 loads in flight, s_sleep 1) and the tuning builds of
# profiles/build_poll_variants.sh, twice each, alternating, on one box.
# usage: bash profiles/r06_poll.sh TAG "p1_s1 p2_s0 ..."
set -o pipefail
TAG=${1:-r06p}
VARS=${2:-"p1_s1 p2_s0 p8_s0 p4_s2"}
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for v in product $VARS; do
    if [ $v = product ]; then LIBV=""; else LIBV=kube-batch-1_amd/_build/libkbhip_$v.so; fi
    KBHIP_LIB=$LIBV timeout -k 10 200 python3 -u bench.py --steps 10 --warmup 2 --cpu-baseline 0 --sweep-nodes 0 \
        > gpurun_out/${TAG}_$v.$r.json 2>> gpurun_out/${TAG}.err || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_$v.$r.json').read().strip().splitlines()[-1]); print('$v', round(d['value']/1e6,3), round(d['p50_session_ms'],1), round(d['config']['device_period_us'],3))"
  done
done
