#!/bin/bash
# Quick iteration on one MI355X: the parity tests of the batched / per-task
# paths plus the full-size digests, a short C4 bench and the sweep probe.
# usage: bash profiles/r04_iter.sh TAG [steps]
set -o pipefail
TAG=${1:-r04i}
STEPS=${2:-10}
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_pertask_abi.py \
    tests/test_gpu_placement_levels.py tests/test_gpu_fit_error.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/$TAG/pytest.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest.log
timeout -k 10 300 python -u bench.py --steps $STEPS --warmup 3 --cpu-baseline 0 > gpurun_out/$TAG/bench.json \
    2> gpurun_out/$TAG/bench.err || { tail -20 gpurun_out/$TAG/bench.err; exit 1; }
cat gpurun_out/$TAG/bench.json
timeout -k 10 300 python -u profiles/sweep_probe.py 512 > gpurun_out/$TAG/probe.json 2> gpurun_out/$TAG/probe.err || exit 1
cat gpurun_out/$TAG/probe.json
