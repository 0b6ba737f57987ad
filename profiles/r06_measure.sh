#!/bin/bash
# r06 measurement pass (each GPU step under its own limit, chained so that a
# failure ends the script): the GPU suite (optional), the C4 bench line (with
# the CPU baseline and the at-scale sweep), the engine timeline, rocprofv3
# kernel stats of the bench, a FETCH_SIZE pass and an SQ-counter pass
# (separate runs: counters never share a run with tracing domains).
# usage: bash profiles/r06_measure.sh TAG [tests=1]
set -o pipefail
TAG=${1:-r06f}
TESTS=${2:-1}
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "$TESTS" = 1 ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
      > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
  tail -1 gpurun_out/${TAG}_pytest.log
fi
timeout -k 10 500 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json \
    2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cut -c1-300 gpurun_out/${TAG}_bench.json
timeout -k 10 200 python3 -u profiles/engine_tl.py --out gpurun_out/${TAG}_engine_tl.json > /dev/null 2>&1 || exit 1
OUT=gpurun_out/prof_${TAG}
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
    python3 bench.py --steps 2 --warmup 0 --cpu-baseline 0 --sweep-nodes 0 > $OUT/bench_trace.json 2> $OUT/trace.err || exit 1
echo trace done
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc -o run --output-format csv -- \
    python3 bench.py --steps 1 --warmup 0 --cpu-baseline 0 --sweep-nodes 0 --time-every 0 > $OUT/bench_pmc.json 2> $OUT/pmc.err || exit 1
echo pmc done
timeout -s KILL 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-trace -d $OUT/sq -o run --output-format csv -- \
    python3 bench.py --steps 1 --warmup 0 --cpu-baseline 0 --sweep-nodes 0 --time-every 0 > $OUT/bench_sq.json 2> $OUT/sq.err || exit 1
echo sq done
python3 profiles/summarize.py $OUT ${TAG} gpurun_out > $OUT/summary.log 2>&1 || exit 1
rm -rf $OUT/trace $OUT/pmc $OUT/sq
echo done
