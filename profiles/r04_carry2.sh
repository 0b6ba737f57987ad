#!/bin/bash
# Carry fast path check: the carry suites, then bench_carry with the per-phase host marks.
# usage: bash profiles/r04_carry2.sh TAG
set -o pipefail
TAG=${1:-r04k}
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 700 python -u -m pytest tests/test_gpu_carry.py tests/test_gpu_carry_snapshot.py \
    -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { tail -40 gpurun_out/$TAG/pytest.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest.log
KBHIP_OPEN_PROFILE=1 timeout -k 10 400 python -u bench_carry.py --rounds 3 > gpurun_out/$TAG/carry.json 2> gpurun_out/$TAG/carry.err || { tail -20 gpurun_out/$TAG/carry.err; exit 1; }
cat gpurun_out/$TAG/carry.json
grep "^\[carry\]" gpurun_out/$TAG/carry.err | tail -13
