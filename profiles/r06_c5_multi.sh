#!/bin/bash
# r06: the what-if sessions' preempt sweep batched over S sessions per launch
# (profiles/c5_multi_sweep.py): the HIP-event line for S = 1 .. 64, then at
# S = 64 rocprofv3 kernel stats, FETCH_SIZE and WRITE_SIZE of the cold chain
# (descriptors in device memory), each pass its own run.
# usage: bash profiles/r06_c5_multi.sh TAG
set -o pipefail
TAG=${1:-r06m}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_whatif.py tests/test_gpu_evict.py -x -q -m gpu --timeout 200 \
    --timeout-method thread > gpurun_out/${TAG}_pytest.txt 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.txt; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.txt
timeout -k 10 300 python3 -u profiles/c5_multi_sweep.py > gpurun_out/${TAG}_c5_multi.jsonl 2> gpurun_out/${TAG}_c5_multi.err || exit 1
cat gpurun_out/${TAG}_c5_multi.jsonl
OUT=gpurun_out/prof_${TAG}_s64
mkdir -p $OUT
ARGS="--sessions 64 --mapped 0 --reps 16"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
    python3 profiles/c5_multi_sweep.py $ARGS > $OUT/probe_trace.json 2> $OUT/trace.err || exit 1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc -o run --output-format csv -- \
    python3 profiles/c5_multi_sweep.py $ARGS > $OUT/probe_pmc.json 2> $OUT/pmc.err || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/pmcw -o run --output-format csv -- \
    python3 profiles/c5_multi_sweep.py $ARGS > $OUT/probe_pmcw.json 2> $OUT/pmcw.err || exit 1
python3 profiles/summarize.py $OUT ${TAG}_s64 gpurun_out > $OUT/summary.log 2>&1 || exit 1
rm -rf $OUT/trace $OUT/pmc $OUT/pmcw
echo done
