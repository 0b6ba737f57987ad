#!/bin/bash
# r06: engine change check with the front's timeline — the engine parity tests,
# the sweep-mode timeline, then the C4 bench line twice.
# usage: bash profiles/r06_eng_tl.sh TAG
set -o pipefail
TAG=${1:-r06e}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_engine.py tests/test_gpu_multiblock.py -x -q --timeout 200 \
    --timeout-method thread > gpurun_out/${TAG}_pytest.txt 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.txt; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.txt
timeout -k 10 200 python3 -u profiles/engine_tl_lists.py --lists 0 --out gpurun_out/${TAG}_tl_sweep.json > gpurun_out/${TAG}_tl.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 200 python3 -u bench.py --steps 10 --warmup 2 --cpu-baseline 0 --sweep-nodes 0 > gpurun_out/${TAG}_bench.$r.json \
      2>> gpurun_out/${TAG}_bench.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_bench.$r.json').read().strip().splitlines()[-1]); print(round(d['value']/1e6,3), round(d['p50_session_ms'],1), round(d['config']['device_period_us'],3))"
done
