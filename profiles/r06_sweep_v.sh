#!/bin/bash
# r06: the standalone sweep's kernel shapes against N (option sweep_variant:
# 0 one node per thread, 4 / 5 / 6 the prefetching grid with 8 / 4 / 16 blocks
# per CU): parity of every shape, the HIP-event line per (N, shape), then at
# N = 4M an SQ-counter pass of shapes 0 and 4 (cold: every launch from HBM).
# usage: bash profiles/r06_sweep_v.sh TAG
set -o pipefail
TAG=${1:-r06v}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_pertask_abi.py -x -q -m gpu -k sweep --timeout 120 \
    --timeout-method thread > gpurun_out/${TAG}_pytest.txt 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.txt; exit 1; }
tail -3 gpurun_out/${TAG}_pytest.txt
timeout -k 10 500 python3 -u profiles/sweep_scaling.py --variants 0 4 5 6 \
    > gpurun_out/${TAG}_sweep_scaling.jsonl 2> gpurun_out/${TAG}_sweep.err || exit 1
cat gpurun_out/${TAG}_sweep_scaling.jsonl
for V in 0 4; do
  OUT=gpurun_out/prof_${TAG}_4000000_v${V}
  mkdir -p $OUT
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
      python3 profiles/sweep_scaling.py --nodes 4000000 --mode cold --variants $V > $OUT/probe_trace.json 2> $OUT/trace.err || exit 1
  timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
      SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-trace -d $OUT/sq -o run --output-format csv -- \
      python3 profiles/sweep_scaling.py --nodes 4000000 --mode cold --variants $V > $OUT/probe_sq.json 2> $OUT/sq.err || exit 1
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc -o run --output-format csv -- \
      python3 profiles/sweep_scaling.py --nodes 4000000 --mode cold --variants $V > $OUT/probe_pmc.json 2> $OUT/pmc.err || exit 1
  python3 profiles/summarize.py $OUT ${TAG}_4000000_v${V} gpurun_out > $OUT/summary.log 2>&1 || exit 1
  rm -rf $OUT/trace $OUT/pmc $OUT/sq
done
echo done
