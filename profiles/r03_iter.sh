#!/bin/bash
# Iteration check on one MI355X: the placement / what-if parity tests, then
# the C4 bench line and (optionally) the C5 what-if group bench.
# usage: bash profiles/r03_iter.sh TAG [c5]
set -o pipefail
TAG=${1:-iter}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_placement_levels.py tests/test_gpu_parity.py tests/test_gpu_fit_error.py \
    tests/test_gpu_whatif.py tests/test_gpu_fullsize.py tests/test_gpu_async_abi.py \
    > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-baseline 0 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit $?
cat gpurun_out/${TAG}_bench.json
if [ "$2" = "c5" ]; then
  timeout -k 10 300 python -u bench_c5.py --sessions 16 --concurrent 8 --group 1 --cpu-baseline 0 \
      > gpurun_out/${TAG}_c5_group1.json 2> gpurun_out/${TAG}_c5_group1.err || exit $?
  cat gpurun_out/${TAG}_c5_group1.json
fi
