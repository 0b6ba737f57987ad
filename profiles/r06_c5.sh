#!/bin/bash
# r06: what-if sessions (C5) — the group tests, then 16 sessions in flight
# ungrouped / grouped (combining), three times each, on one box, and one
# session alone.
# usage: bash profiles/r06_c5.sh TAG
set -o pipefail
TAG=${1:-r06c}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_whatif.py tests/test_gpu_evict.py -x -q -m gpu --timeout 200 \
    --timeout-method thread > gpurun_out/${TAG}_pytest.txt 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.txt; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.txt
for G in 0 1 0 1 0 1; do
  timeout -k 10 200 python3 -u bench_c5.py --sessions 16 --concurrent 16 --group $G --cpu-baseline 0 \
      >> gpurun_out/${TAG}_c5_g${G}.jsonl 2>> gpurun_out/${TAG}_c5.err || exit 1
  tail -1 gpurun_out/${TAG}_c5_g${G}.jsonl | cut -c1-300
done
timeout -k 10 200 python3 -u bench_c5.py --sessions 8 --concurrent 1 > gpurun_out/${TAG}_c5_alone.json 2>> gpurun_out/${TAG}_c5.err || exit 1
cut -c1-400 gpurun_out/${TAG}_c5_alone.json
echo done
