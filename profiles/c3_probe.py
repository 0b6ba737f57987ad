"""C3 (20k nodes, selectors, taints, zone anti-affinity, 8 queues) — or with
--c5, C5's allocate (50k nodes with Backfilled resources, after reclaim): one
session's allocate with the engine's path counters — batched pops, the
sequential placements (6: Backfilled nodes, 7: pod anti-affinity classes) and
how they ended, per-task sweeps, unassigned pops, FitDelta recounts — plus
open / allocate times (--engine0: the persistent engine off; --aff: C3 with keyless nodes,
required pod affinity and preferred inter-pod terms).  Prints one JSON line; run under rocprofv3
--kernel-trace --stats for the kernel split."""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kube-batch-1_amd"))
import kbgen  # noqa: E402
import kbhip  # noqa: E402


def main():
    c5 = "--c5" in sys.argv
    engine = 0 if "--engine0" in sys.argv else 1
    aff = "--aff" in sys.argv  # C3 with keyless nodes, required pod affinity, preferred inter-pod terms
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    reps = int(args[0]) if args else 3
    p = "/tmp/kbhip_bench/c5_50000_2000_0.kbs" if c5 else "/tmp/kbhip_bench/c3aff.kbs" if aff else "/tmp/kbhip_bench/c3.kbs"
    if not os.path.exists(p):
        os.makedirs(os.path.dirname(p), exist_ok=True)
        if c5:
            kbgen.gen_c5(p + ".tmp", seed=kbgen.BASE_SEED + 5, n_nodes=50_000, n_pending=2000)
        elif aff:
            kbgen.gen_c3(keyless=0.1, pod_affinity=0.15, ipa=0.15).write(p + ".tmp")
        else:
            kbgen.gen_c3().write(p + ".tmp")
        os.replace(p + ".tmp", p)
    with open(p, "rb") as f:
        buf = f.read()
    opens, allocs, st = [], [], None
    for _ in range(reps):
        t0 = time.perf_counter()
        s = kbhip.Session(buf)
        s.set_option("engine", engine)
        t1 = time.perf_counter()
        if c5:
            s.reclaim()  # the shipped actions' order: allocate runs after reclaim (not timed)
            t0 += time.perf_counter() - t1
            t1 = time.perf_counter()
        pod, node, kind = s.allocate()
        t2 = time.perf_counter()
        st = s.stats()
        s.close()
        opens.append(t1 - t0)
        allocs.append(t2 - t1)
    keys = ("pops", "tasks", "placed", "sweeps", "batched_pops", "pertask_sweeps", "seq_launches", "seq_cut",
            "seq_none", "unassigned_pops", "spec_hits", "spec_missed", "fit_syncs", "alloc_setup_s", "alloc_device_s", "host_launch_s",
            "host_wait_s", "engine_pops", "engine_launches")
    print(json.dumps({"config": "C5 allocate" if c5 else "C3aff" if aff else "C3", "engine": engine, "placements": int(len(pod)), "open_ms": statistics.median(opens) * 1e3,
                      "allocate_ms": statistics.median(allocs) * 1e3, **{k: st[k] for k in keys}}))


if __name__ == "__main__":
    main()
