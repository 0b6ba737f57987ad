#!/bin/bash
# r06: the whole GPU suite, then smoke() and a short bench line.
# usage: bash profiles/r06_gpu_suite.sh TAG
set -o pipefail
TAG=${1:-r06g}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 800 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/${TAG}_pytest.txt 2>&1 || { tail -40 gpurun_out/${TAG}_pytest.txt; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.txt
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.txt 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.txt; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.txt
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --cpu-baseline 0 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_bench.json').read().strip().splitlines()[-1]); print(d['value'], d['p50_session_ms'], d['roofline']['frac'], d['roofline']['sweep']['at_scale']['cold'])"
