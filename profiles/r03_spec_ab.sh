#!/bin/bash
# C4 bench lines over (overlap, speculate), alternating; parity tests first.
# usage: bash profiles/r03_spec_ab.sh TAG
set -o pipefail
TAG=${1:-spec}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_placement_levels.py tests/test_gpu_parity.py tests/test_gpu_fit_error.py tests/test_gpu_fullsize.py tests/test_shard.py \
    > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
for r in 1 2; do
  for ds in "1 2" "2 2" "2 3"; do
    set -- $ds
    timeout -k 10 300 python -u bench.py --steps 6 --warmup 1 --cpu-baseline 0 --overlap $1 --speculate $2 \
        > gpurun_out/${TAG}_ov$1_sp$2_${r}.json 2> gpurun_out/${TAG}_ov$1_sp$2_${r}.err || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['value']), d['config']['device_period_us'], d['config']['allocate_s'], d['p50_session_ms'])" gpurun_out/${TAG}_ov$1_sp$2_${r}.json
  done
done
