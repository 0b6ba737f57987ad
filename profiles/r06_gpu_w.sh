#!/bin/bash
# r06: after a change to the shared evaluation (kbhip_eval.h): the whole GPU
# suite, the C4 bench line (no CPU baseline), the standalone sweep's shapes
# against N with read eviction, and the write-eviction line at 4M for
# comparison.  usage: bash profiles/r06_gpu_w.sh TAG
set -o pipefail
TAG=${1:-r06w}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/${TAG}_pytest.txt 2>&1 || { tail -40 gpurun_out/${TAG}_pytest.txt; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.txt
timeout -k 10 240 python3 -u bench.py --steps 10 --warmup 2 --cpu-baseline 0 > gpurun_out/${TAG}_bench.json \
    2> gpurun_out/${TAG}_bench.err || exit 1
timeout -k 10 400 python3 -u profiles/sweep_scaling.py --variants 0 2 3 4 \
    > gpurun_out/${TAG}_sweep_scaling.jsonl 2> gpurun_out/${TAG}_sweep.err || exit 1
timeout -k 10 120 python3 -u profiles/sweep_scaling.py --nodes 4000000 --variants 0 --evict 1 --mode cold \
    >> gpurun_out/${TAG}_sweep_scaling.jsonl 2>> gpurun_out/${TAG}_sweep.err || exit 1
cat gpurun_out/${TAG}_sweep_scaling.jsonl | cut -c1-400
echo done
