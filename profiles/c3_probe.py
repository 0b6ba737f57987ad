"""C3 (20k nodes, selectors, taints, zone anti-affinity, 8 queues): one
session's allocate with the engine's path counters — batched pops, the
sequential placements (7: pod anti-affinity classes) and how they ended,
per-task sweeps, unassigned pops — plus open / allocate times.  Prints one
JSON line; run under rocprofv3 --kernel-trace --stats for the kernel split."""
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
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    p = "/tmp/kbhip_bench/c3.kbs"
    if not os.path.exists(p):
        os.makedirs(os.path.dirname(p), exist_ok=True)
        kbgen.gen_c3().write(p + ".tmp")
        os.replace(p + ".tmp", p)
    with open(p, "rb") as f:
        buf = f.read()
    opens, allocs, st = [], [], None
    for _ in range(reps):
        t0 = time.perf_counter()
        s = kbhip.Session(buf)
        t1 = time.perf_counter()
        pod, node, kind = s.allocate()
        t2 = time.perf_counter()
        st = s.stats()
        s.close()
        opens.append(t1 - t0)
        allocs.append(t2 - t1)
    keys = ("pops", "tasks", "placed", "sweeps", "batched_pops", "pertask_sweeps", "seq_launches", "seq_cut",
            "seq_none", "unassigned_pops", "spec_hits", "spec_missed", "alloc_device_s", "host_launch_s",
            "host_wait_s")
    print(json.dumps({"config": "C3", "placements": int(len(pod)), "open_ms": statistics.median(opens) * 1e3,
                      "allocate_ms": statistics.median(allocs) * 1e3, **{k: st[k] for k in keys}}))


if __name__ == "__main__":
    main()
