#!/usr/bin/env python3
"""The standalone predicate + score sweep (k_score_sweep, kbhip_sweep_scores'
kernel) at C4 size with cold caches: n launches, each behind a 512 MB write
that evicts L2 and the Infinity Cache (option time_sweeps_cold), so that every
launch reads its node columns from HBM.  Prints one JSON line (HIP-event span
per launch); run under rocprofv3 --kernel-trace --stats for the kernel's own
duration and under --pmc FETCH_SIZE for its HBM bytes (profiles/r05_measure.sh)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kube-batch-1_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import bench  # noqa: E402
import kbhip  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    path = bench.snapshot_path(bench.argparse.Namespace(cache="/tmp/kbhip_bench", nodes=100_000, pending=800_000))
    with open(path, "rb") as f:
        buf = f.read()
    with kbhip.Session(buf) as s:  # pending tasks of the session (the ones it places)
        pend, _, _ = s.allocate()
    ids = np.ascontiguousarray(pend[:: max(1, len(pend) // n)][:n], np.int32)
    with kbhip.Session(buf) as s:
        s.set_option("time_sweeps_cold", 1)
        cold_us = s.time_sweeps(ids)
        nodes = s.stats()["nodes"]
    gbs = nodes * bench.B_NODE / (cold_us * 1e-6) / 1e9
    print(json.dumps({"kernel": "k_score_sweep", "launches": int(len(ids)), "cold_span_us": cold_us,
                      "bytes_per_launch": nodes * bench.B_NODE, "achieved_gbs": gbs,
                      "frac": gbs / bench.HBM_PEAK_GBS}))


if __name__ == "__main__":
    main()
