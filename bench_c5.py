"""C5 what-if sessions (a parity-test config, not the
headline bench line — bench.py measures C4).  Each session: open a 50k-node
snapshot (~90 % filled, 5 % backfill pods) with a different 2k-task
high-priority pending set, run the shipped conf's actions
"reclaim, allocate, backfill, preempt", close.  Prints one JSON line: sessions/s,
p50 session latency, per-action wall times, records (evictions, pipelines,
allocations) per session, and the node-ranking sweeps (one per reclaim /
preempt task) with their mean wall time.

Usage: python bench_c5.py [--sessions S] [--warmup W] [--nodes N] [--pending T] [--concurrent C]
(--concurrent 1: one session at a time with per-action wall times)
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "kube-batch-1_amd"))
import numpy as np  # noqa: E402

import kbgen  # noqa: E402
import kbhip  # noqa: E402

ACTIONS = ("reclaim", "allocate", "backfill", "preempt")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sessions", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--nodes", type=int, default=50_000)
    ap.add_argument("--pending", type=int, default=2000)
    ap.add_argument("--cache", default=os.environ.get("KBHIP_BENCH_CACHE", "/tmp/kbhip_bench"))
    ap.add_argument("--cpu-baseline", type=int, default=1, help="1 = time the hoisted CPU restatement on one session")
    ap.add_argument("--group", type=int, default=1,
                    help="1 = option rank_group on the concurrent sessions: their allocate pops, per-task chunks "
                         "and reclaim / preempt rankings go out as multi-session launches, each request at once "
                         "with whatever other sessions' requests are pending; 0 = every session launches alone")
    ap.add_argument("--concurrent", type=int, default=8,
                    help="what-if sessions in flight (host threads); their node rankings share launches")
    args = ap.parse_args()
    os.makedirs(args.cache, exist_ok=True)
    bufs = []
    for k in range(args.warmup + args.sessions):
        p = os.path.join(args.cache, f"c5_{args.nodes}_{args.pending}_{k}.kbs")
        if not os.path.exists(p):
            print(f"generating C5 snapshot {k}", file=sys.stderr, flush=True)
            kbgen.gen_c5(p + ".tmp", seed=kbgen.BASE_SEED + 5 + k, n_nodes=args.nodes, n_pending=args.pending)
            os.replace(p + ".tmp", p)
        with open(p, "rb") as f:
            bufs.append(f.read())
    lat, phases, recs, sweeps = [], {a: [] for a in ("open",) + ACTIONS + ("close",)}, [], []
    if args.concurrent > 1:
        return concurrent(args, bufs)
    for k, buf in enumerate(bufs):
        t0 = time.perf_counter()
        s = kbhip.Session(buf, device=0)
        t = [time.perf_counter()]
        counts = {1: 0, 2: 0, 3: 0}
        kinds = []  # counted after the session (outside the timed phases)
        n_rank = 0
        launches = {}
        for a in ACTIONS:
            st0 = s.stats()
            t.append(time.perf_counter())
            _, _, kind = getattr(s, a)()
            t[-1] = (t[-1], time.perf_counter())
            kinds.append(kind)
            st1 = s.stats()
            if a in ("reclaim", "preempt"):
                n_rank += st1["sweeps"] - st0["sweeps"]  # one node-ranking sweep per reclaim / preempt task
                launches[a] = {k: st1[k] - st0[k] for k in ("evict_rank_s", "evict_walk_s", "evict_visits",
                                                            "evict_cands", "evict_setup_s")}
            else:  # batched pops (one launch places a chunk) vs per-task sweeps
                bp = st1["batched_pops"] - st0["batched_pops"]
                launches[a] = {"batched_pops": bp, "per_task_sweeps": st1["sweeps"] - st0["sweeps"] - bp}
        s.close()
        t_end = time.perf_counter()
        for kind in kinds:
            bc = np.bincount(kind, minlength=4)
            for v in (1, 2, 3):
                counts[v] += int(bc[v])
        if k < args.warmup:
            continue
        lat.append(t_end - t0)
        phases["open"].append(t[0] - t0)
        for i, a in enumerate(ACTIONS):
            phases[a].append(t[i + 1][1] - t[i + 1][0])
        phases["close"].append(t_end - t[-1][1])
        recs.append(counts)
        sweeps.append(n_rank)
        last_launches = launches
    evict_s = sum(statistics.mean(phases[a]) for a in ("reclaim", "preempt"))
    out = {
        "metric": "C5 what-if sessions/s (reclaim, allocate, backfill, preempt)",
        "value": len(lat) / sum(lat),
        "unit": "sessions/s",
        "n_gpus": 1,
        "sessions": len(lat),
        "p50_session_ms": statistics.median(lat) * 1e3,
        "higher_is_better": True,
        "data": "synthetic (kbgen.gen_c5, seeds 20261015+5+k)",
        "config": {"workload": "C5: 50k nodes ~90% filled, 5% backfill pods, 2k-task high-priority pending set per "
                               "session, 4 queues, shipped conf", "nodes": args.nodes, "pending": args.pending},
        "phases_ms": {a: round(statistics.mean(v) * 1e3, 3) for a, v in phases.items()},
        "records_per_session": {"evicted": statistics.mean(r[3] for r in recs),
                                "pipelined": statistics.mean(r[2] for r in recs),
                                "allocated": statistics.mean(r[1] for r in recs)},
        "rank_sweeps_per_session": statistics.mean(sweeps),
        "launches_last_session": last_launches,
        "reclaim_preempt_us_per_rank_sweep": evict_s / max(statistics.mean(sweeps), 1) * 1e6,
    }
    if args.cpu_baseline:  # the hoisted C++ restatement (oracle/kbfast.cpp): one session, same actions
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle  # the checker / CPU baseline only (test infrastructure)
        threads = min(16, os.cpu_count() or 1)
        p0 = os.path.join(args.cache, f"c5_{args.nodes}_{args.pending}_{args.warmup}.kbs")
        st = {}
        pl = oracle.fast_allocate(p0, threads=threads, actions=", ".join(ACTIONS), stats=st)
        sess_s = st["open_s"] + st["allocate_s"]  # plugin open + the four actions (snapshot load excluded)
        out["cpu_baseline"] = {"value": 1.0 / sess_s, "unit": "sessions/s", "cores": threads, "kind": "port",
                               "sample": f"one C5 session ({len(pl)} records), actions {', '.join(ACTIONS)}, "
                                         f"hoisted C++ restatement oracle/kbfast.cpp, {threads} threads on "
                                         f"{os.cpu_count()} host cpus, snapshot parse excluded"}
    print(json.dumps(out))


GROUP = [1]


def one_session(buf, group, barrier=None):
    t0 = time.perf_counter()
    s = kbhip.Session(buf, device=0)
    if group and GROUP[0]:
        s.set_option("rank_group", GROUP[0])
    if barrier is not None:
        barrier.wait()
    kinds = []
    for a in ACTIONS:
        _, _, kind = getattr(s, a)()
        kinds.append(kind)
    st = s.stats()
    s.close()
    dt = time.perf_counter() - t0
    counts = {1: 0, 2: 0, 3: 0}  # counted outside the timed session
    for kind in kinds:
        bc = np.bincount(kind, minlength=4)
        for v in (1, 2, 3):
            counts[v] += int(bc[v])
    return dt, counts, st


def concurrent(args, bufs):
    """S what-if sessions in flight from S host threads (the engine releases the
    GIL); with --group their reclaim / preempt node rankings, allocate pops
    and per-task chunks go out as shared multi-session launches (option
    rank_group, session/session.h StepBatcher)."""
    from concurrent.futures import ThreadPoolExecutor
    # the sessions of one wave of `concurrent` start together (a barrier after
    # their opens), as a what-if sweep over one cluster state would
    warm, timed = bufs[:args.warmup], bufs[args.warmup:]
    GROUP[0] = args.group
    import threading

    def waves(ex, bs):
        out = []
        for w in range(0, len(bs), args.concurrent):
            chunk = bs[w:w + args.concurrent]
            bar = threading.Barrier(len(chunk))
            out += list(ex.map(lambda b: one_session(b, True, bar), chunk))
        return out

    with ThreadPoolExecutor(args.concurrent) as ex:
        waves(ex, warm)
        t0 = time.perf_counter()
        res = waves(ex, timed)
        wall = time.perf_counter() - t0
    lat = [r[0] for r in res]
    req = sum(r[2]["rank_requests"] for r in res)
    bsum = sum(r[2]["rank_batch_sum"] for r in res)
    preq = sum(r[2]["pop_requests"] for r in res)  # allocate pops batched across sessions
    pbsum = sum(r[2]["pop_batch_sum"] for r in res)
    sreq = sum(r[2]["sweep_requests"] for r in res)  # per-task chunks (general path, backfill) batched
    sbsum = sum(r[2]["sweep_batch_sum"] for r in res)
    seq_lat, _, _ = one_session(timed[0], False)  # one session alone, for the latency beside the throughput
    out = {
        "metric": "C5 what-if sessions/s (reclaim, allocate, backfill, preempt)",
        "value": len(timed) / wall,
        "unit": "sessions/s",
        "n_gpus": 1,
        "sessions": len(timed),
        "concurrent_sessions": args.concurrent,
        "p50_session_ms": statistics.median(lat) * 1e3,
        "alone_session_ms": seq_lat * 1e3,
        "higher_is_better": True,
        "data": "synthetic (kbgen.gen_c5, seeds 20261015+5+k)",
        "config": {"workload": "C5: 50k nodes ~90% filled, 5% backfill pods, 2k-task high-priority pending set per "
                               "session, 4 queues, shipped conf", "nodes": args.nodes, "pending": args.pending},
        "records_per_session": {"evicted": statistics.mean(r[1][3] for r in res),
                                "pipelined": statistics.mean(r[1][2] for r in res),
                                "allocated": statistics.mean(r[1][1] for r in res)},
        "rank_launch_requests": req,
        "sessions_per_rank_launch": bsum / max(req, 1),
        "group": args.group,
        "pop_launch_requests": preq,
        "sessions_per_pop_launch": pbsum / max(preq, 1),
        "sweep_chunk_requests": sreq,
        "sessions_per_sweep_launch": sbsum / max(sreq, 1),
    }
    if args.cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle  # the checker / CPU baseline only (test infrastructure)
        threads = min(16, os.cpu_count() or 1)
        p0 = os.path.join(args.cache, f"c5_{args.nodes}_{args.pending}_{args.warmup}.kbs")
        st = {}
        pl = oracle.fast_allocate(p0, threads=threads, actions=", ".join(ACTIONS), stats=st)
        sess_s = st["open_s"] + st["allocate_s"]
        out["cpu_baseline"] = {"value": 1.0 / sess_s, "unit": "sessions/s", "cores": threads, "kind": "port",
                               "sample": f"one C5 session ({len(pl)} records), actions {', '.join(ACTIONS)}, "
                                         f"hoisted C++ restatement oracle/kbfast.cpp, {threads} threads on "
                                         f"{os.cpu_count()} host cpus, snapshot parse excluded"}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
