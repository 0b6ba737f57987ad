# C3 (20k nodes, affinity) and C5-allocate path counters, and the C4 carry-over
# chain, on the current build (each step under its own limit, chained).
# usage: bash profiles/r06_c3_carry.sh TAG
set -o pipefail
TAG=${1:-r06k}
mkdir -p gpurun_out
timeout -k 10 300 python3 -u profiles/c3_probe.py 5 > gpurun_out/${TAG}_c3.json 2> gpurun_out/${TAG}_c3.err || { tail -20 gpurun_out/${TAG}_c3.err; exit 1; }
cat gpurun_out/${TAG}_c3.json
timeout -k 10 300 python3 -u profiles/c3_probe.py 3 --c5 > gpurun_out/${TAG}_c5alloc.json 2> gpurun_out/${TAG}_c5alloc.err || { tail -20 gpurun_out/${TAG}_c5alloc.err; exit 1; }
cat gpurun_out/${TAG}_c5alloc.json
timeout -k 10 400 python3 -u bench_carry.py > gpurun_out/${TAG}_carry.json 2> gpurun_out/${TAG}_carry.err || { tail -20 gpurun_out/${TAG}_carry.err; exit 1; }
cut -c1-1500 gpurun_out/${TAG}_carry.json
