#!/bin/bash
# Parity of the overlapped pops at depths 1 and 2, then the C4 bench line at
# each depth, alternating (box noise).  usage: bash profiles/r03_overlap_ab.sh TAG
set -o pipefail
TAG=${1:-ab}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_placement_levels.py tests/test_gpu_parity.py tests/test_gpu_fit_error.py \
    tests/test_gpu_fullsize.py tests/test_gpu_async_abi.py \
    > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
for r in 1 2; do
  for d in 1 2; do
    timeout -k 10 300 python -u bench.py --steps 6 --warmup 1 --cpu-baseline 0 --overlap $d \
        > gpurun_out/${TAG}_ov${d}_${r}.json 2> gpurun_out/${TAG}_ov${d}_${r}.err || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['value']), d['config']['device_period_us'], d['config']['allocate_s'])" gpurun_out/${TAG}_ov${d}_${r}.json
  done
done
