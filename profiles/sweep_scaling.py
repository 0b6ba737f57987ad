#!/usr/bin/env python3
"""The standalone predicate + score sweep (k_score_sweep, kbhip_sweep_scores'
kernel: every node's PredicateFn + NodeOrderFn key for one task,
preempt.go:270-287) against the node count N (VERDICT r05 "next" 5):
C4-shaped clusters (its SKU mix and task classes, no running pods) of N nodes,
`launches` tasks swept back to back (warm: the columns stay in the caches
while they fit the 256 MB Infinity Cache, N x 113 B) and one at a time behind
512 MB read (or written, --evict 1) before each launch (cold: every launch
reads HBM; a write leaves dirty lines whose write-back overlaps the sweep).  Prints one JSON
line per N (and kernel shape, option sweep_variant) with the HIP-event time
per launch and the roofline fraction on the kernel's algorithmic bytes: the
41 B per node its keys depend on (flags, acpu / amem / nzc / nzm, pods,
maxtasks; PredicateFn + NodeOrderFn read no fit column) plus the 8-byte key
written, 49 B per node (bench.SWEEP_B_NODE).  Run one N per process under
rocprofv3 --kernel-trace --stats for the kernel's own duration and under
--pmc FETCH_SIZE for its HBM bytes (profiles/r06_sweep_scaling.sh)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kube-batch-1_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import bench  # noqa: E402
import kbgen  # noqa: E402
import kbhip  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, nargs="+", default=[100_000, 400_000, 1_000_000, 4_000_000])
    ap.add_argument("--pending", type=int, default=20_000)
    ap.add_argument("--launches", type=int, default=256)
    ap.add_argument("--cold", type=int, default=32)
    ap.add_argument("--mode", choices=("both", "warm", "cold"), default="both")
    ap.add_argument("--variants", type=int, nargs="+", default=[0])
    ap.add_argument("--evict", type=int, default=2, help="cold launches: 1 = behind a 512 MB write, 2 = read")
    ap.add_argument("--cache", default="/tmp/kbhip_bench")
    a = ap.parse_args()
    os.makedirs(a.cache, exist_ok=True)
    for n in a.nodes:
        path = os.path.join(a.cache, f"sweep_{n}_{a.pending}.kbs")
        if not os.path.exists(path):
            kbgen.gen_c4(path, n_nodes=n, n_pending=a.pending, running_per_node=0)
        with open(path, "rb") as f:
            buf = f.read()
        B = bench.SWEEP_B_NODE
        with kbhip.Session(buf) as s:
            ids = np.arange(0, a.pending, max(1, a.pending // a.launches), dtype=np.int32)[: a.launches]
            for v in a.variants:
                s.set_option("sweep_variant", v)
                rec = {"nodes": n, "variant": v, "bytes_per_launch": n * B,
                       "fits_infinity_cache": n * B < 256 << 20}
                if a.mode in ("both", "warm"):
                    s.set_option("time_sweeps_cold", 0)
                    s.time_sweeps(ids[:16])  # warm up
                    us = s.time_sweeps(ids)
                    gbs = n * B / (us * 1e-6) / 1e9
                    rec["warm"] = {"launches": int(len(ids)), "mean_us": us, "gbs": gbs,
                                   "frac": gbs / bench.HBM_PEAK_GBS}
                if a.mode in ("both", "cold"):
                    s.set_option("time_sweeps_cold", a.evict)
                    us = s.time_sweeps(ids[: a.cold])
                    gbs = n * B / (us * 1e-6) / 1e9
                    rec["cold"] = {"launches": int(a.cold), "mean_us": us, "gbs": gbs,
                                   "frac": gbs / bench.HBM_PEAK_GBS,
                                   "evict": "512 MB " + ("write" if a.evict == 1 else "read") + " before each launch",
                                   "timing": "HIP events around each launch alone (dispatch and drain included)"}
                print(json.dumps(rec), flush=True)
            s.set_option("sweep_variant", 0)


if __name__ == "__main__":
    main()
