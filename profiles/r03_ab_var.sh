#!/bin/bash
# Same-box A/B of library builds / bench options at C4, alternating.
# usage: bash profiles/r03_ab_var.sh TAG "name|lib|args" ...   (lib "-" = the in-tree build)
set -o pipefail
TAG=$1
shift
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in "$@"; do
    IFS='|' read -r name lib args <<< "$v"
    if [ "$lib" = "-" ]; then unset KBHIP_LIB; else export KBHIP_LIB=$lib; fi
    timeout -k 10 300 python -u bench.py --steps 6 --warmup 1 --cpu-baseline 0 $args \
        > gpurun_out/${TAG}_${name}_${r}.json 2> gpurun_out/${TAG}_${name}_${r}.err || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['value']), round(d['config']['device_period_us'], 3), d['config']['allocate_s'], round(d['p50_session_ms'], 1))" gpurun_out/${TAG}_${name}_${r}.json
  done
done
