#!/bin/bash
# End-of-round measurements on one MI355X (each step under its own limit):
# GPU suite, the C4 bench line, rocprofv3 stats + FETCH_SIZE of the bench,
# the per-pop ABI at C4, C5 what-if sessions (lockstep group on / off at 8 and
# 16 in flight), C3 whole sessions.  usage: bash profiles/r03_final.sh TAG
set -o pipefail
TAG=${1:-r03final}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit $?
cat gpurun_out/${TAG}_bench.json
bash profiles/run_profile.sh ${TAG} > gpurun_out/${TAG}_prof.log 2>&1 || exit $?
timeout -k 10 400 python -u profiles/host_loop.py --reps 3 --depth 2 --out gpurun_out/${TAG}_host_loop.json \
    > gpurun_out/${TAG}_host_loop.log 2>&1 || exit $?
for g in 0 1; do
  for c in 8 16; do
    timeout -k 10 300 python -u bench_c5.py --sessions 16 --concurrent $c --group $g --cpu-baseline 0 \
        > gpurun_out/${TAG}_c5_g${g}_c${c}.json 2> gpurun_out/${TAG}_c5_g${g}_c${c}.err || exit $?
  done
done
timeout -k 10 600 python -u profiles/baseline_table.py gpurun_out/${TAG}_c3_table.json --only=C3 \
    > gpurun_out/${TAG}_c3.log 2>&1 || exit $?
echo done
