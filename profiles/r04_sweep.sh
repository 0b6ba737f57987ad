#!/bin/bash
# The standalone sweep kernel at C4 size: its parity tests, the probe's HIP-event
# numbers, and rocprofv3 kernel stats of the same probe (kernel durations).
# usage: bash profiles/r04_sweep.sh TAG
set -o pipefail
TAG=${1:-r04s}
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest tests/test_gpu_pertask_abi.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/$TAG/pytest.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest.log
timeout -k 10 300 python -u profiles/sweep_probe.py 512 > gpurun_out/$TAG/probe.json 2> gpurun_out/$TAG/probe.err || exit 1
cat gpurun_out/$TAG/probe.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/trace -o run --output-format csv -- \
    python3 profiles/sweep_probe.py 512 > gpurun_out/$TAG/probe_trace.json 2> gpurun_out/$TAG/trace.err || exit 1
grep -E "score_sweep|Name" gpurun_out/$TAG/trace/run_kernel_stats.csv > gpurun_out/$TAG/sweep_stats.csv || true
cp gpurun_out/$TAG/trace/run_kernel_stats.csv gpurun_out/$TAG/kernel_stats.csv
rm -rf gpurun_out/$TAG/trace
cat gpurun_out/$TAG/sweep_stats.csv
