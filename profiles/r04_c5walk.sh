# C5 reclaim walk check: eviction parity suites, then the walk split (diagnostic build) and the product bench.
set -o pipefail
mkdir -p gpurun_out/r04wk
timeout -k 10 600 python -u -m pytest tests/test_gpu_evict.py tests/test_gpu_whatif.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04wk/tests.log 2>&1 || { tail -30 gpurun_out/r04wk/tests.log; exit 1; }
tail -2 gpurun_out/r04wk/tests.log
KBHIP_LIB=kube-batch-1_amd/_build/libkbhip_wp.so timeout -k 10 300 python -u bench_c5.py --concurrent 1 --sessions 3 --warmup 1 --cpu-baseline 0 > gpurun_out/r04wk/c5_wp.json 2> gpurun_out/r04wk/c5_wp.err || exit 1
grep walkprof gpurun_out/r04wk/c5_wp.err
for R in 1 2; do
  timeout -k 10 300 python -u bench_c5.py --concurrent 1 --sessions 3 --warmup 1 --cpu-baseline 0 > gpurun_out/r04wk/c5_$R.json 2> gpurun_out/r04wk/c5_$R.err || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['p50_session_ms'], d['phases_ms'], d['launches_last_session']['reclaim'])" gpurun_out/r04wk/c5_$R.json
done
