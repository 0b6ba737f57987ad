#!/usr/bin/env python3
"""The what-if sessions' preempt sweep batched over S sessions per launch
("S = 64 what-if sessions per launch", §8(f) row 2; VERDICT
r05 item 5): kbhip_time_rank_multi over S sessions of C5 (50k nodes ~90 %
filled), each on its own node columns in HBM, one multi-session launch chain
(k_rank_bucket_multi: the PredicateFn + NodeOrderFn sweep and the histogram;
k_rank_scan_multi; k_rank_scatter_multi: the stable counting sort).  Prints
one JSON line per (S, descriptor placement) with warm and cold (behind a
512 MB read) microseconds per chain and the HBM fraction on the chain's
algorithmic bytes: per node and session 41 B read + 8 B key written by the
sweep, 8 B key read + 8 B sorted key written by the scatter (65 B).  Run under
rocprofv3 for the kernels' own durations and FETCH_SIZE / WRITE_SIZE
(profiles/r06_c5_multi.sh)."""
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

B_CHAIN = 41 + 8 + 8 + 8


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sessions", type=int, nargs="+", default=[1, 8, 16, 32, 64])
    ap.add_argument("--snapshots", type=int, default=4, help="distinct C5 snapshots the sessions cycle over")
    ap.add_argument("--nodes", type=int, default=50_000)
    ap.add_argument("--pending", type=int, default=2000)
    ap.add_argument("--reps", type=int, default=32)
    ap.add_argument("--mapped", type=int, nargs="+", default=[0, 1])
    ap.add_argument("--cache", default=os.environ.get("KBHIP_BENCH_CACHE", "/tmp/kbhip_bench"))
    a = ap.parse_args()
    os.makedirs(a.cache, exist_ok=True)
    bufs = []
    for k in range(a.snapshots):  # bench_c5.py's snapshots (same names)
        p = os.path.join(a.cache, f"c5_{a.nodes}_{a.pending}_{k}.kbs")
        if not os.path.exists(p):
            kbgen.gen_c5(p + ".tmp", seed=kbgen.BASE_SEED + 5 + k, n_nodes=a.nodes, n_pending=a.pending)
            os.replace(p + ".tmp", p)
        with open(p, "rb") as f:
            bufs.append(f.read())
    smax = max(a.sessions)
    sessions = [kbhip.Session(bufs[i % len(bufs)]) for i in range(smax)]
    try:
        ids = []
        for i, s in enumerate(sessions):
            cls = s.table("pod_class")
            pend = np.nonzero(cls >= 0)[0]
            ids.append(int(pend[(7 * i) % pend.size]))  # a different pending task per session
        n = sessions[0].stats()["nodes"]
        for S in a.sessions:
            for m in a.mapped:
                rec = {"sessions": S, "nodes_per_session": n, "desc": "mapped host" if m else "device",
                       "bytes_per_chain": S * n * B_CHAIN}
                for name, ev in (("warm", 0), ("cold", 2)):
                    kbhip.time_rank_multi(sessions[:S], ids[:S], reps=2, evict=0, mapped=m)  # warm up
                    us = kbhip.time_rank_multi(sessions[:S], ids[:S], reps=a.reps, evict=ev, mapped=m)
                    gbs = S * n * B_CHAIN / (us * 1e-6) / 1e9
                    rec[name] = {"us_per_chain": us, "gbs": gbs, "frac": gbs / bench.HBM_PEAK_GBS}
                print(json.dumps(rec), flush=True)
    finally:
        for s in sessions:
            s.close()


if __name__ == "__main__":
    main()
