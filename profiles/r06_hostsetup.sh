# host-side session setup check: the parity suites touching the open / allocate
# setup, then 8 C4 sessions with the host phase prints (KBHIP_OPEN_PROFILE=1)
# usage: bash profiles/r06_hostsetup.sh TAG [test files...]
set -o pipefail
TAG=${1:-r06i}
shift
TESTS=${@:-tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_evict.py tests/test_gpu_backfilled.py tests/test_gpu_engine.py tests/test_gpu_whatif.py}
mkdir -p gpurun_out
timeout -k 10 700 python3 -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
KBHIP_OPEN_PROFILE=1 timeout -k 10 300 python3 -u bench.py --steps 8 --warmup 2 --cpu-baseline 0 --sweep-nodes 0 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cut -c1-400 gpurun_out/${TAG}_bench.json
grep -E "^\[(alloc|open|close)\]" gpurun_out/${TAG}_bench.err | tail -20
