#!/bin/bash
# The standalone sweep's latency floor (profiles/micro/sweep_floor.hip, built
# in-tree): rocprofv3 kernel stats of the empty / loads-only / long-stream
# kernels, warm and cold.  usage: bash profiles/r05_floor.sh TAG
set -o pipefail
TAG=${1:-r05floor}
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/trace -o run --output-format csv -- \
    profiles/micro/sweep_floor 100000 64 > gpurun_out/$TAG/run.json 2> gpurun_out/$TAG/run.err || exit 1
cp gpurun_out/$TAG/trace/run_kernel_stats.csv gpurun_out/$TAG/kernel_stats.csv
python3 - gpurun_out/$TAG <<'PY' || exit 1
import csv, json, sys, collections
d = sys.argv[1]
rows = collections.defaultdict(list)
with open(d + "/trace/run_kernel_trace.csv") as f:
    for r in csv.DictReader(f):
        rows[r["Kernel_Name"].split("(")[0]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
out = {}
for k, iv in rows.items():
    iv.sort()
    du = [(e - s) / 1e3 for s, e in iv]
    out[k] = {"calls": len(du), "durations_us": du}
loads = out.get("f_loads", {}).get("durations_us", [])
n = len(loads) // 2
res = {"empty_us": sum(out["f_empty"]["durations_us"]) / len(out["f_empty"]["durations_us"]),
       "loads_warm_us": sum(loads[:n]) / max(n, 1), "loads_cold_us": sum(loads[n:]) / max(len(loads) - n, 1),
       "stream_us": sum(out["f_stream"]["durations_us"]) / len(out["f_stream"]["durations_us"])}
res["stream_GBs"] = 100000 * 32 * 113 / (res["stream_us"] * 1e-6) / 1e9
res["loads_cold_GBs"] = 100000 * 113 / (res["loads_cold_us"] * 1e-6) / 1e9
res["loads_warm_GBs"] = 100000 * 113 / (res["loads_warm_us"] * 1e-6) / 1e9
json.dump(res, open(d + "/floor.json", "w"), indent=1)
print(json.dumps(res))
PY
rm -rf gpurun_out/$TAG/trace
