"""Standalone predicate + score sweep at C4 size (100k nodes): kbhip_time_sweeps
over pending tasks of the C4 session, plus the C4 session's batched pops for
reference.  Prints one JSON line.  Run under rocprofv3 --kernel-trace --stats
to get the kernel's own duration (profiles/r04_sweep.sh)."""
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
    n_tasks = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    path = bench.snapshot_path(bench.argparse.Namespace(cache="/tmp/kbhip_bench", nodes=100_000, pending=800_000))
    with open(path, "rb") as f:
        buf = f.read()
    with kbhip.Session(buf) as s:
        pod, node, kind = s.allocate()
    res = bench.sweep_roofline(buf, 0, pod, n_tasks)
    variants, same = {}, {}
    ref = None
    for v in range(4):  # the kernel shapes of option "sweep_variant"
        with kbhip.Session(buf) as s:
            s.set_option("sweep_variant", v)
            got = [s.sweep_scores(int(p), 0)[1] if False else s.sweep_scores(int(p), 100_000)
                   for p in pod[:: max(1, len(pod) // 4)][:4]]
            if ref is None:
                ref = got
            same[v] = all(a[0] == b[0] and np.array_equal(a[1], b[1]) for a, b in zip(got, ref))
            step = max(1, len(pod) // n_tasks)
            ids = np.ascontiguousarray(pod[::step][:n_tasks], np.int32)
            s.time_sweeps(ids[:16])
            variants[v] = round(s.time_sweeps(ids), 3)
            s.set_option("sweep_variant", 0)
    res["variants_us"] = variants
    res["variants_equal_keys"] = same
    with kbhip.Session(buf) as s:  # per-launch event timing of single sweeps (includes launch latency)
        s.set_option("time_every", 1)
        for p in pod[:: max(1, len(pod) // 64)][:64]:
            s.sweep_scores(int(p), 0, keys=False)
        st = s.stats()
    res["single_launch_event_us"] = st["score_sweep_s"] / max(st["score_sweeps"], 1) * 1e6
    print(json.dumps(res))


if __name__ == "__main__":
    main()
