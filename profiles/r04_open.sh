#!/bin/bash
# Session open by pod ranges: the GPU suite, then C4 and C5 with the open's phase marks.
set -o pipefail
TAG=${1:-r04o}
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/$TAG/pytest.log 2>&1 || { tail -40 gpurun_out/$TAG/pytest.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest.log
KBHIP_OPEN_PROFILE=1 timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/$TAG/bench.json \
    2> gpurun_out/$TAG/bench.err || { tail -20 gpurun_out/$TAG/bench.err; exit 1; }
cut -c1-400 gpurun_out/$TAG/bench.json
grep "^\[open\]" gpurun_out/$TAG/bench.err | tail -11
KBHIP_OPEN_PROFILE=1 timeout -k 10 400 python -u bench_c5.py --concurrent 1 --sessions 5 --warmup 1 --cpu-baseline 0 \
    > gpurun_out/$TAG/c5.json 2> gpurun_out/$TAG/c5.err || exit 1
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['p50_session_ms'], d['phases_ms'])" gpurun_out/$TAG/c5.json
grep "^\[open\]" gpurun_out/$TAG/c5.err | tail -11
