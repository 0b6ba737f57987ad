#!/bin/bash
# Occupancy / stall counters of the C4 bench kernels (rocprofv3 PMC, one pass;
# SQ block only: at most 8 SQ counters per pass on gfx950), plus the stamps
# build's per-phase breakdown of one pop at a time.
# Usage (repo root, on the GPU box): bash profiles/run_sq.sh <tag>
set -eo pipefail
TAG=${1:-r02}
export TMPDIR=/tmp
OUT=gpurun_out/sq_$TAG
mkdir -p $OUT
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
WANT="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES"
PMC=""
N=0
for c in $WANT; do
    if grep -qw "$c" $OUT/counters.txt && [ $N -lt 8 ]; then PMC="$PMC $c"; N=$((N+1)); fi
done
echo "pmc:$PMC" > $OUT/pmc_used.txt
timeout -k 10 300 python3 -u profiles/phases.py 2 1 > $OUT/phases_ov.json
timeout -k 10 300 python3 -u profiles/phases.py 2 0 > $OUT/phases.json
if [ -n "$PMC" ]; then
    timeout -s KILL 600 rocprofv3 --pmc $PMC --kernel-trace -d $OUT/pmc -o run --output-format csv -- \
        python3 bench.py --steps 1 --warmup 0 --cpu-baseline 0 > $OUT/bench_pmc.json
fi
