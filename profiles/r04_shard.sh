#!/bin/bash
# Overlapped shard pops (k_shard_sweep_ov) on one MI355X: the shard tests,
# then the C4 rehearsal with rank threads (W = 2, 4; overlap on and off).
# usage: bash profiles/r04_shard.sh TAG
set -o pipefail
TAG=${1:-r04sh}
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 900 python -u -m pytest tests/test_shard.py -x -q --timeout 450 --timeout-method thread \
    -k "batched_random or c4_scaled or c4_full_size or close_messages or carry" > gpurun_out/$TAG/pytest.log 2>&1 \
    || { tail -40 gpurun_out/$TAG/pytest.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest.log
fi
# the rank threads' streams (3 per rank) must map to distinct hardware queues: the chained
# kernels of one rank spin on each other (HIP's default is 4 queues per process)
export GPU_MAX_HW_QUEUES=16
for W in 2 4; do
  for OV in 1 0; do
    timeout -k 10 300 python -u profiles/shard_threads.py $TAG $W 2 $OV > gpurun_out/$TAG/st_w${W}_ov${OV}.json \
        2> gpurun_out/$TAG/st_w${W}_ov${OV}.err || { tail -20 gpurun_out/$TAG/st_w${W}_ov${OV}.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['device_period_us'], d['p50_session_ms'], d['all_digests_ok'])" gpurun_out/$TAG/st_w${W}_ov${OV}.json
  done
done
