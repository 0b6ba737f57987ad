#!/usr/bin/env python3
"""Summarise a run_profile.sh output directory into the files committed under
profiles/: <tag>_kernel_stats.csv (rocprofv3 --stats, verbatim) and
<tag>_summary.json (per kernel: calls, mean duration, the union busy period
of overlapping launches, FETCH_SIZE per launch and the gfx950-corrected HBM
bytes per launch, SQ occupancy / stall counters per launch with VGPR / SGPR /
LDS of the kernel).

FETCH_SIZE is reported in KB by rocprofv3; on gfx950 it counts exactly half
the bytes of wide coalesced streaming reads (MI355X_MICROARCH.md, HBM section),
so the corrected traffic is 2 x FETCH_SIZE x 1024 bytes.

Usage: python profiles/summarize.py gpurun_out/prof_<tag> <tag> [dest dir, default profiles/]
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

HERE = os.path.dirname(os.path.abspath(__file__))


def short(name):
    return name.split("(")[0].replace("void ", "")


def main(src, tag, dest=None):
    stats_csv = os.path.join(src, "trace", "run_kernel_stats.csv")
    pmc_csv = os.path.join(src, "pmc", "run_counter_collection.csv")
    out = {"tag": tag, "kernels": {}}
    with open(stats_csv) as f:
        for row in csv.DictReader(f):
            out["kernels"][short(row["Name"])] = {"calls": int(row["Calls"]),
                                                  "mean_us": float(row["AverageNs"]) / 1e3,
                                                  "min_us": float(row["MinNs"]) / 1e3,
                                                  "max_us": float(row["MaxNs"]) / 1e3}
    trace_csv = os.path.join(src, "trace", "run_kernel_trace.csv")
    if os.path.exists(trace_csv):  # overlapped pop kernels: per-launch device period from the timeline
        by = defaultdict(list)
        with open(trace_csv) as f:
            for row in csv.DictReader(f):
                by[short(row["Kernel_Name"])].append((int(row["Start_Timestamp"]), int(row["End_Timestamp"])))
        for k, iv in by.items():
            if len(iv) < 2:
                continue
            iv.sort()
            span = iv[-1][1] - iv[0][0]
            busy, cur_s, cur_e = 0, iv[0][0], iv[0][1]  # union of the kernel intervals
            for s0, e0 in iv[1:]:
                if s0 > cur_e:
                    busy += cur_e - cur_s
                    cur_s, cur_e = s0, e0
                else:
                    cur_e = max(cur_e, e0)
            busy += cur_e - cur_s
            d = out["kernels"].setdefault(k, {})
            d["timeline_span_us"] = span / 1e3
            d["period_us"] = span / 1e3 / len(iv)          # launches overlap: span / launches
            d["busy_period_us"] = busy / 1e3 / len(iv)     # union of their intervals / launches
    if os.path.exists(pmc_csv):
        acc = defaultdict(lambda: [0.0, 0])
        with open(pmc_csv) as f:
            for row in csv.DictReader(f):
                if row["Counter_Name"] != "FETCH_SIZE":
                    continue
                a = acc[short(row["Kernel_Name"])]
                a[0] += float(row["Counter_Value"])
                a[1] += 1
        pops = None  # the persistent engine: one dispatch serves a session's pops (the PMC pass's bench line)
        bj = os.path.join(src, "bench_pmc.json")
        if os.path.exists(bj):
            try:
                with open(bj) as f:
                    line = [ln for ln in f.read().splitlines() if ln.startswith("{")][-1]
                pops = json.loads(line)["config"].get("engine_pops") or None
            except (IndexError, ValueError, KeyError):
                pops = None
        for k, (tot, n) in acc.items():
            d = out["kernels"].setdefault(k, {})
            d["fetch_size_kb_per_launch"] = tot / n
            d["hbm_bytes_per_launch_corrected"] = 2.0 * tot / n * 1024.0
            d["pmc_launches"] = n
            if k.startswith("kbhip::k_engine") and pops:
                d["engine_pops"] = pops
                d["hbm_bytes_per_pop_corrected"] = 2.0 * tot * 1024.0 / pops
    w_csv = os.path.join(src, "pmcw", "run_counter_collection.csv")
    if os.path.exists(w_csv):  # WRITE_SIZE (its own pass: FETCH_SIZE and WRITE_SIZE do not fit one)
        acc = defaultdict(lambda: [0.0, 0])
        with open(w_csv) as f:
            for row in csv.DictReader(f):
                if row["Counter_Name"] != "WRITE_SIZE":
                    continue
                a = acc[short(row["Kernel_Name"])]
                a[0] += float(row["Counter_Value"])
                a[1] += 1
        for k, (tot, n) in acc.items():
            d = out["kernels"].setdefault(k, {})
            d["write_size_kb_per_launch"] = tot / n  # KB as reported; no gfx950 calibration for writes
    sq_csv = os.path.join(src, "sq", "run_counter_collection.csv")
    if os.path.exists(sq_csv):  # occupancy / stall counters, per launch, with the kernel's resources
        acc = defaultdict(lambda: defaultdict(float))
        res, disp = {}, defaultdict(set)
        with open(sq_csv) as f:
            for row in csv.DictReader(f):
                k = short(row["Kernel_Name"])
                acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
                disp[k].add(row.get("Dispatch_Id") or row.get("Correlation_Id"))
                res[k] = {"grid": int(row.get("Grid_Size", 0) or 0), "wg": int(row.get("Workgroup_Size", 0) or 0),
                          "lds": int(row.get("LDS_Block_Size", 0) or 0), "vgpr": int(row.get("VGPR_Count", 0) or 0),
                          "agpr": int(row.get("Accum_VGPR_Count", 0) or 0), "sgpr": int(row.get("SGPR_Count", 0) or 0)}
        for k, c in acc.items():
            n = max(len(disp[k]), 1)
            per = {name: v / n for name, v in sorted(c.items())}
            d = out["kernels"].setdefault(k, {})
            d["sq"] = {"launches": n, **res[k], "per_launch": per}
            wc = per.get("SQ_WAVE_CYCLES", 0.0)
            if wc > 0:
                for key, name in (("wait_any_frac", "SQ_WAIT_ANY"), ("wait_inst_frac", "SQ_WAIT_INST_ANY"),
                                  ("active_inst_frac", "SQ_ACTIVE_INST_ANY"), ("valu_frac", "SQ_ACTIVE_INST_VALU")):
                    if name in per:
                        d["sq"][key] = round(per[name] / wc, 3)
    for name in ("bench_trace.json", "bench_pmc.json"):
        p = os.path.join(src, name)
        if os.path.exists(p):
            with open(p) as f:
                lines = [ln for ln in f.read().splitlines() if ln.startswith("{")]
            if lines:
                out[name.replace(".json", "")] = json.loads(lines[-1])
    dest = dest or HERE
    shutil.copy(stats_csv, os.path.join(dest, f"{tag}_kernel_stats.csv"))
    with open(os.path.join(dest, f"{tag}_summary.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out["kernels"], indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None)
