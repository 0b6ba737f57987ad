# the GPU suite, then C5 alone and C4 with the host phase prints (KBHIP_OPEN_PROFILE=1)
# usage: bash profiles/r06_spare.sh TAG
set -o pipefail
TAG=${1:-r06o}
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
KBHIP_OPEN_PROFILE=1 timeout -k 10 300 python3 -u bench_c5.py --sessions 6 --warmup 1 --concurrent 1 --cpu-baseline 0 > gpurun_out/${TAG}_c5.json 2> gpurun_out/${TAG}_c5.err || { tail -20 gpurun_out/${TAG}_c5.err; exit 1; }
cut -c1-700 gpurun_out/${TAG}_c5.json
grep -E "^\[(close|alloc)\]" gpurun_out/${TAG}_c5.err | tail -8
KBHIP_OPEN_PROFILE=1 timeout -k 10 300 python3 -u bench.py --steps 8 --warmup 2 --cpu-baseline 0 --sweep-nodes 0 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cut -c1-400 gpurun_out/${TAG}_bench.json
grep -E "^\[(alloc|open|close)\]" gpurun_out/${TAG}_bench.err | tail -18
