"""Fills BASELINE.md §3: whole-session GPU and CPU lines for C1-C4, plus the
faithful restatement's complexity fit.

For each config it records:
  - GPU: kbhip sessions (open + allocate + close, from the snapshot bytes already
    in host memory, as bench.py), placements/s and p50 session latency;
  - CPU-hoisted: oracle/kbfast.cpp whole sessions at 16 threads, placements/s and
    p50 (the checker's allocate phase; snapshot parse reported separately);
  - parity: the GPU log equals the CPU log, record for record.
Then kbref (the faithful restatement, per-(task,node) recomputation) on the C2
generator at N in {100, 300, 1000} nodes x T = 1000 pending tasks, and a power
fit of its allocate time in N.

Usage (repo root, GPU box): python3 profiles/baseline_table.py [out.json] [--fit] [--only=C3,C4]
Test infrastructure: the oracle here is the checker and the CPU baseline only.
"""
import json
import os
import statistics
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "kube-batch-1_amd"), os.path.join(ROOT, "oracle")]
import kbgen  # noqa: E402
import kbhip  # noqa: E402
import oracle  # noqa: E402  (checker / CPU baseline only)

THREADS = 16


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def gpu_sessions(buf, reps):
    times, n, phases = [], 0, []
    for _ in range(reps):
        t0 = time.perf_counter()
        s = kbhip.Session(buf)
        t1 = time.perf_counter()
        pod, node, kind = s.allocate(cap=1 << 21)
        t2 = time.perf_counter()
        s.close()
        t3 = time.perf_counter()
        times.append(t3 - t0)
        phases.append((t1 - t0, t2 - t1, t3 - t2))
        n = len(pod)
    p50 = statistics.median(times)
    return dict(placements=n, p50_session_ms=p50 * 1e3, placements_per_s=n / p50, sessions=reps,
                p50_allocate_ms=statistics.median(p[1] for p in phases) * 1e3,
                p50_open_ms=statistics.median(p[0] for p in phases) * 1e3), (pod, node, kind)


def cpu_sessions(path, reps):
    alloc, parse, n, pl = [], [], 0, None
    for _ in range(reps):
        st = {}
        pl = oracle.fast_allocate(path, threads=THREADS, stats=st)
        alloc.append(st["allocate_s"])
        parse.append(st["open_s"] + st.get("load_s", 0.0))
        n = len(pl)
    p50 = statistics.median(alloc)
    return dict(placements=n, p50_session_ms=p50 * 1e3, placements_per_s=n / p50, sessions=reps, threads=THREADS,
                p50_parse_ms=statistics.median(parse) * 1e3, host_cpus=os.cpu_count()), pl


def same(gl, pl):
    pod, node, kind = gl
    return bool(np.array_equal(pod, pl.pod) and np.array_equal(node, pl.node) and
                np.array_equal(np.array([0, 4, 8, 128])[kind], pl.status))


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    out_path = args[0] if args else os.path.join(ROOT, "gpurun_out", "baseline_table.json")
    tmp = tempfile.mkdtemp(prefix="kbbase")
    res = {"configs": {}}
    cfgs = [
        ("C1", lambda p: kbgen.gen_c1().write(p), 5, 5),
        ("C2", lambda p: kbgen.gen_c2(p), 5, 3),
        ("C3", lambda p: kbgen.gen_c3().write(p), 3, 1),
        ("C4", lambda p: kbgen.gen_c4(p), 3, 1),
    ]
    only = [a.split("=", 1)[1] for a in sys.argv[1:] if a.startswith("--only=")]
    for name, gen, greps, creps in cfgs:
        if only and name not in only[0].split(","):
            continue
        p = os.path.join(tmp, name + ".kbs")
        t = time.perf_counter()
        gen(p)
        log(f"{name}: generated in {time.perf_counter() - t:.1f}s")
        with open(p, "rb") as f:
            buf = f.read()
        g, gl = gpu_sessions(buf, greps)
        log(f"{name}: gpu {g}")
        c, pl = cpu_sessions(p, creps)
        log(f"{name}: cpu {c}")
        res["configs"][name] = dict(gpu=g, cpu_hoisted=c, parity=same(gl, pl),
                                    speedup_p50=c["p50_session_ms"] / g["p50_session_ms"])
        os.remove(p)
        with open(out_path, "w") as f:
            json.dump(res, f, indent=1)
    if "--fit" not in sys.argv:  # the faithful fit takes ~10 min (N = 1000); committed as profiles/r02_faithful_fit.json
        print(json.dumps(res))
        return
    fit = []
    for n in (100, 300, 1000):
        p = os.path.join(tmp, f"fit{n}.kbs")
        kbgen.gen_c2(p, n_nodes=n, n_pending=1000)
        t = time.perf_counter()
        pl = oracle.ref_allocate(p)
        dt = time.perf_counter() - t
        fit.append(dict(nodes=n, tasks=1000, placements=len(pl), seconds=dt))
        log(f"fit N={n}: {dt:.2f}s, {len(pl)} placements")
        os.remove(p)
    x = np.log([f["nodes"] for f in fit])
    y = np.log([f["seconds"] for f in fit])
    k, c0 = np.polyfit(x, y, 1)
    res["faithful_fit"] = dict(points=fit, exponent=float(k),
                               note="kbref (per-(task,node) recomputation, oracle/kbref.cpp) on the C2 generator; "
                                    "seconds = wall time of the whole call incl. snapshot parse; "
                                    "seconds ~ a * N^exponent at T = 1000",
                               extrapolated_c2_s=float(np.exp(c0) * 5000 ** k) * 50,
                               extrapolated_c2_note="N = 5000 at T = 1000, x 50 for T = 50k (linear in T)")
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
