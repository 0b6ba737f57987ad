# Round-6: the round-5 library (sweep engine) vs this round's, sweep and list mode, on one box
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r06ab}
for i in 1 2; do
  KBHIP_LIB=$PWD/kube-batch-1_amd/_build/libkbhip_r05.so timeout -k 10 240 python -u bench.py --steps 5 --warmup 1 --cpu-baseline 0 >> gpurun_out/${tag}_bench_r05.jsonl 2>> gpurun_out/${tag}_bench.err || exit 1
  timeout -k 10 240 python -u bench.py --steps 5 --warmup 1 --cpu-baseline 0 --engine-lists 0 >> gpurun_out/${tag}_bench_0.jsonl 2>> gpurun_out/${tag}_bench.err || exit 1
  timeout -k 10 240 python -u bench.py --steps 5 --warmup 1 --cpu-baseline 0 --engine-lists 1 >> gpurun_out/${tag}_bench_1.jsonl 2>> gpurun_out/${tag}_bench.err || exit 1
done
