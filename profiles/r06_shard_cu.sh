#!/bin/bash
# r06: the node-sharded C4 session rehearsed on one MI355X with W rank threads
# (profiles/shard_threads.py), each rank's streams on its own 256/W CUs
# (option cu_split), W = 2, 4, 8, and W = 2 unsplit.
# usage: bash profiles/r06_shard_cu.sh TAG
set -o pipefail
TAG=${1:-r06sh}
export TMPDIR=/tmp
mkdir -p gpurun_out
# every rank's streams on their own hardware queues (the ranks' chained kernels
# spin on each other; the library refuses a rank group that would share queues)
export GPU_MAX_HW_QUEUES=32
for spec in "2 1" "2 0" "4 1" "8 1"; do
  set -- $spec
  timeout -k 10 400 python3 -u profiles/shard_threads.py $TAG $1 2 1 $2 > gpurun_out/${TAG}_w$1_cu$2.json \
      2> gpurun_out/${TAG}_w$1_cu$2.err || { tail -20 gpurun_out/${TAG}_w$1_cu$2.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['device_period_us'], d['p50_session_ms'], d['all_digests_ok'])" gpurun_out/${TAG}_w$1_cu$2.json
done
