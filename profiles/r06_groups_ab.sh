# A/B of the engine's merger blocks (option engine_groups; the library's
# default 8), alternating on one box: the bench's device period per pop.
set -o pipefail
mkdir -p gpurun_out
for g in 8 4 6 2 8 4 6 2; do
  timeout -k 10 300 python3 -u bench.py --steps 6 --warmup 2 --cpu-baseline 0 --sweep-nodes 0 --engine-groups $g > gpurun_out/r06g_$g.json 2> gpurun_out/r06g_$g.err || { tail -20 gpurun_out/r06g_$g.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/r06g_$g.json').read().strip().splitlines()[-1]);c=d['config'];print('groups $g', round(d['value']), round(d['p50_session_ms'],1), round(c['device_period_us'],3), c['engine_pops'])"
done
