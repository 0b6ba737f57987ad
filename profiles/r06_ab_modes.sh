# Round-6: list mode vs sweep mode on one box (bench without the CPU baseline, then timelines)
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r06ab}
for m in 0 1 0 1; do
  timeout -k 10 240 python -u bench.py --steps 5 --warmup 1 --cpu-baseline 0 --engine-lists $m >> gpurun_out/${tag}_bench_$m.jsonl 2>> gpurun_out/${tag}_bench.err || exit 1
done
timeout -k 10 200 python -u profiles/engine_tl_lists.py --lists 0 --out gpurun_out/${tag}_tl0.json > /dev/null 2>> gpurun_out/${tag}_tl.err && \
timeout -k 10 200 python -u profiles/engine_tl_lists.py --lists 1 --out gpurun_out/${tag}_tl1.json > /dev/null 2>> gpurun_out/${tag}_tl.err
