#!/bin/bash
# Same-box A/B of two builds of the library at C4 (bench lines alternating,
# KBHIP_LIB selects the build), then the event timeline of the new build.
# usage: bash profiles/r03_ab_lib.sh TAG OLD_LIB [TESTS...]
set -o pipefail
TAG=${1:-ab}
OLD=$2
shift 2
mkdir -p gpurun_out
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu "$@" \
      > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
  tail -2 gpurun_out/${TAG}_pytest.log
fi
for r in 1 2 3; do
  for v in old new; do
    if [ $v = old ]; then export KBHIP_LIB=$OLD; else unset KBHIP_LIB; fi
    timeout -k 10 300 python -u bench.py --steps 6 --warmup 1 --cpu-baseline 0 \
        > gpurun_out/${TAG}_${v}_${r}.json 2> gpurun_out/${TAG}_${v}_${r}.err || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['value']), d['config']['device_period_us'], d['config']['allocate_s'], d['p50_session_ms'])" gpurun_out/${TAG}_${v}_${r}.json
  done
done
unset KBHIP_LIB
timeout -k 10 300 python -u profiles/timeline.py --overlap 1 --out gpurun_out/${TAG}_timeline_ov1.json > /dev/null || exit $?
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); [print(k, v) for k, v in d.items() if not isinstance(v, dict)]" gpurun_out/${TAG}_timeline_ov1.json
