set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_evict.py tests/test_gpu_backfilled.py tests/test_gpu_engine.py tests/test_gpu_whatif.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06i_pytest.log 2>&1 || { tail -30 gpurun_out/r06i_pytest.log; exit 1; }
tail -1 gpurun_out/r06i_pytest.log
KBHIP_OPEN_PROFILE=1 timeout -k 10 300 python3 -u bench.py --steps 8 --warmup 2 --cpu-baseline 0 --sweep-nodes 0 > gpurun_out/r06i_bench.json 2> gpurun_out/r06i_bench.err || { tail -20 gpurun_out/r06i_bench.err; exit 1; }
cut -c1-400 gpurun_out/r06i_bench.json
grep -E "^\[alloc\]" gpurun_out/r06i_bench.err | tail -12
