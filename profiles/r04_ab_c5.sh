# Same-box A/B of the C5 session (a: this tree's libkbhip.so, b: _build/libkbhip_b.so built
# from another revision of kbhip_session.cpp), alternating.
set -o pipefail
mkdir -p gpurun_out/r04ab
if [ -n "$AB_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $AB_TESTS -x -q --timeout 300 --timeout-method thread > gpurun_out/r04ab/tests.log 2>&1 || { tail -30 gpurun_out/r04ab/tests.log; exit 1; }
  tail -3 gpurun_out/r04ab/tests.log
fi
for R in 1 2 3; do
  for V in a b; do
    if [ $V = b ]; then export KBHIP_LIB=kube-batch-1_amd/_build/libkbhip_b.so; else unset KBHIP_LIB; fi
    timeout -k 10 300 python -u bench_c5.py --concurrent 1 --sessions 3 --warmup 1 --cpu-baseline 0 > gpurun_out/r04ab/c5_${V}${R}.json 2> gpurun_out/r04ab/c5_${V}${R}.err || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['phases_ms'], d['launches_last_session']['reclaim'])" gpurun_out/r04ab/c5_${V}${R}.json
  done
done
