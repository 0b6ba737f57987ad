#!/bin/bash
# r06: the standalone sweep (k_score_sweep) against N: the HIP-event line for
# N = 100k .. 4M nodes, then per N (100k, 1M, 4M) rocprofv3 kernel stats, a
# FETCH_SIZE pass and a WRITE_SIZE pass of the warm and the cold sweep, each
# in its own run (summarize.py: <tag>_<N>_<warm|cold>_summary.json under
# gpurun_out/).  Cold = a 512 MB read before each launch (--evict 2: no dirty
# lines whose write-back would overlap the sweep).
set -o pipefail
TAG=${1:-r06s}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u profiles/sweep_scaling.py > gpurun_out/${TAG}_sweep_scaling.jsonl 2> gpurun_out/${TAG}_sweep.err || exit 1
cat gpurun_out/${TAG}_sweep_scaling.jsonl
for N in 100000 1000000 4000000; do
  for M in warm cold; do
    OUT=gpurun_out/prof_${TAG}_${N}_${M}
    mkdir -p $OUT
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
        python3 profiles/sweep_scaling.py --nodes $N --mode $M > $OUT/probe_trace.json 2> $OUT/trace.err || exit 1
    timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc -o run --output-format csv -- \
        python3 profiles/sweep_scaling.py --nodes $N --mode $M > $OUT/probe_pmc.json 2> $OUT/pmc.err || exit 1
    timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/pmcw -o run --output-format csv -- \
        python3 profiles/sweep_scaling.py --nodes $N --mode $M > $OUT/probe_pmcw.json 2> $OUT/pmcw.err || exit 1
    python3 profiles/summarize.py $OUT ${TAG}_${N}_${M} gpurun_out > $OUT/summary.log 2>&1 || exit 1
    rm -rf $OUT/trace $OUT/pmc $OUT/pmcw
  done
done
echo done
