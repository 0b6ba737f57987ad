#!/bin/bash
# What-if lockstep group with per-task chunks batched (k_sweep_argmax_multi):
# parity tests, then C5 sessions at 16 in flight, group on / off.
# usage: bash profiles/r03_sweepgroup.sh TAG
set -o pipefail
TAG=${1:-sweepgroup}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_whatif.py tests/test_gpu_evict.py tests/test_gpu_backfilled.py tests/test_gpu_pertask_abi.py \
    tests/test_gpu_parity.py tests/test_gpu_place_job.py tests/test_gpu_fit_error.py \
    > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
for g in 1 0; do
  timeout -k 10 300 python -u bench_c5.py --sessions 16 --concurrent 16 --group $g --cpu-baseline 0 \
      > gpurun_out/${TAG}_c5_g${g}_c16.json 2> gpurun_out/${TAG}_c5_g${g}_c16.err || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['value'], 2), round(d['p50_session_ms']), d.get('sessions_per_pop_launch'), d.get('sessions_per_rank_launch'), d.get('sweep_chunk_requests'), d.get('sessions_per_sweep_launch'))" gpurun_out/${TAG}_c5_g${g}_c16.json
done
