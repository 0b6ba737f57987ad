#!/bin/bash
# Carry-over on one MI355X: the carry / carry_events / carry_snapshot tests,
# bench_carry (C4 carry and C4 with 1% arrivals), the sweep probe.
# usage: bash profiles/r04_carry.sh TAG
set -o pipefail
TAG=${1:-r04c}
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 700 python -u -m pytest tests/test_gpu_carry.py tests/test_gpu_carry_snapshot.py tests/test_gpu_async_abi.py tests/test_gpu_aff_batch.py \
    tests/test_gpu_fullsize.py::test_c3_full_size_parity \
    -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { tail -40 gpurun_out/$TAG/pytest.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest.log
timeout -k 10 400 python -u bench_carry.py --rounds 3 > gpurun_out/$TAG/carry.json 2> gpurun_out/$TAG/carry.err || { tail -20 gpurun_out/$TAG/carry.err; exit 1; }
cat gpurun_out/$TAG/carry.json
timeout -k 10 300 python -u profiles/sweep_probe.py 512 > gpurun_out/$TAG/probe.json 2> gpurun_out/$TAG/probe.err || exit 1
cat gpurun_out/$TAG/probe.json
timeout -k 10 300 python -u profiles/c3_probe.py 3 > gpurun_out/$TAG/c3.json 2> gpurun_out/$TAG/c3.err || exit 1
cat gpurun_out/$TAG/c3.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/c3trace -o run --output-format csv -- \
    python3 profiles/c3_probe.py 1 > gpurun_out/$TAG/c3_trace.json 2> gpurun_out/$TAG/c3_trace.err || exit 1
cp gpurun_out/$TAG/c3trace/run_kernel_stats.csv gpurun_out/$TAG/c3_kernel_stats.csv
rm -rf gpurun_out/$TAG/c3trace
head -12 gpurun_out/$TAG/c3_kernel_stats.csv
timeout -k 10 400 python -u bench_c5.py --concurrent 1 --sessions 3 --warmup 1 --cpu-baseline 0 > gpurun_out/$TAG/c5.json 2> gpurun_out/$TAG/c5.err || exit 1
cat gpurun_out/$TAG/c5.json
