# A/B of the engine's candidate copies (KBHIP_CAND_COPIES, whole-library
# tuning builds loaded with KBHIP_LIB): 8 (the product), 16, 4, alternating
# on one box; the bench's device period per pop and throughput.
set -o pipefail
mkdir -p gpurun_out
for v in 8 16 4 8 16 4; do
  if [ $v = 8 ]; then unset KBHIP_LIB; else export KBHIP_LIB=$PWD/kube-batch-1_amd/_build/libkbhip_c$v.so; fi
  timeout -k 10 300 python3 -u bench.py --steps 8 --warmup 2 --cpu-baseline 0 --sweep-nodes 0 > gpurun_out/r06cc_$v.json 2> gpurun_out/r06cc_$v.err || { tail -20 gpurun_out/r06cc_$v.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/r06cc_$v.json').read().strip().splitlines()[-1]);c=d['config'];print('copies $v', round(d['value']), round(d['p50_session_ms'],1), round(c['device_period_us'],3), c['engine_pops'])"
done
