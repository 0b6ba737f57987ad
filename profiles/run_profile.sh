#!/bin/bash
# Profile the C4 bench with rocprofv3 on the GPU box (kernel trace + stats),
# then a separate PMC pass for HBM traffic of the sweep kernel.
# Usage (from the repo root on the box): bash profiles/run_profile.sh <tag>
set -eo pipefail
TAG=${1:-r01}
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
    python3 bench.py --steps 1 --warmup 0 --cpu-baseline 0 > $OUT/bench_trace.json
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc -o run --output-format csv -- \
    python3 bench.py --steps 1 --warmup 0 --cpu-baseline 0 --time-every 0 > $OUT/bench_pmc.json
