#!/usr/bin/env python3
"""bench.py — kube-batch allocate action on MI355X: pod placements/sec and p50
session latency on the C4 workload (100k nodes x 1M pods, BASELINE.json).

A step is one scheduling session over the same synthetic snapshot: open the
session from the in-memory KBS1 buffer (decode + encode + upload to HBM),
run the allocate action (host ordering plugins + HIP placement kernels),
close.  ``value`` = placements of all timed sessions on all ranks / max-over-
ranks wall time.  Inputs are resident in host memory when the timed region
starts (the session upload is part of every step, as in the reference where
every session re-snapshots the cache).

N > 1: one process per GPU (torch.distributed over RCCL for the barrier and
the max-over-ranks time).  Default --mode shard: ONE C4 session node-sharded
over the GPUs: per batched pop each rank sweeps its node
range to its top-64 with rows and writes them into every rank's mailbox over
xGMI (--exchange mailbox, default; --exchange rccl: one ncclAllGather), and
every rank runs the same placement (strong scaling).  --mode replicas: N
independent sessions.

Also reported:
* roofline of the batched pop path: with the persistent pop engine (default,
  --engine 1: k_engine, one resident kernel serving every eligible pop from a
  descriptor ring) or the fused pop kernel (--engine 0: k_pop_batch_ov, sweep
  + top-64 + placement per launch): algorithmic bytes = nodes x 113 B
   per pop / the device busy period per pop (allocate's
  device span, HIP events on the session streams, / batched pops); beside it
  the standalone predicate + score sweep (`sweep`: the product kernel
  k_score_sweep behind kbhip_sweep_scores, one launch over all nodes; 41 B
  read + 8 B written per node), warm (HIP events around back-to-back
  launches) and cold (each launch alone behind a cache-evicting read), on the
  C4 session and on a C4-shaped cluster of --sweep-nodes nodes (`at_scale`),
  each beside the committed rocprofv3 counter bytes of that size;
* cpu_baseline: the hoisted C++ restatement (oracle/kbfast.cpp) on the host
  cores, timed on a stratified sample of the same session: pop windows early,
  mid and late in the session, the pops between them fast-forwarded from the
  engine's placement log (the swept decisions are checked against it); the
  whole-session CPU allocate time is extrapolated per stratum.
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

METRIC = "pod placements/sec + p50 session latency, 100k nodes × 1M pods"
B_NODE = 113  # algorithmic bytes per node per sweep
# the standalone predicate + score sweep (kbhip_sweep_scores): its keys depend on
# 41 B of each node (flags, acpu / amem / nzc / nzm, pods, maxtasks: PredicateFn
# + NodeOrderFn read no Idle / Releasing / Backfilled column) + the 8-byte key
SWEEP_B_READ, SWEEP_B_WRITE = 41, 8
SWEEP_B_NODE = SWEEP_B_READ + SWEEP_B_WRITE
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--nodes", type=int, default=100_000)
    ap.add_argument("--pending", type=int, default=800_000)
    ap.add_argument("--cache", default=os.environ.get("KBHIP_BENCH_CACHE", "/tmp/kbhip_bench"))
    ap.add_argument("--cpu-baseline", type=int, default=1, help="1 = time the CPU restatement on rank 0")
    ap.add_argument("--sweep-nodes", type=int, default=4_000_000,
                    help="node count of the standalone sweep's at-scale line (roofline.sweep.at_scale; 0 = none)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="target CPU baseline sample length")
    ap.add_argument("--time-every", type=int, default=50,
                    help="HIP-event time every k-th batched pop launch on its own stream (the roofline's kernel "
                         "duration; 0 = off)")
    ap.add_argument("--speculate", type=int, default=4, choices=range(7),
                    help="predicted job pops queued ahead of the running one")
    ap.add_argument("--overlap", type=int, default=1, choices=(0, 1, 2),
                    help="1: batched pops alternate over two streams, a pop's sweep beside the previous pop's "
                         "placement (device-side chaining); 0 = one pop kernel at a time")
    ap.add_argument("--engine", type=int, default=1, choices=(0, 1),
                    help="1: batched pops go to the persistent pop engine (one resident kernel, DESIGN.md §4.10); "
                         "0 = one launched kernel per pop")
    ap.add_argument("--engine-workers", type=int, default=0, help="engine worker blocks (0: as many as stay resident)")
    ap.add_argument("--engine-groups", type=int, default=-1,
                    help="engine merger blocks (-1: the library's default, 8)")
    ap.add_argument("--engine-lists", type=int, default=0, choices=(0, 1),
                    help="1 = the engine's list mode when every class fits (class owners, DESIGN.md §4.11), 0 = sweep mode")
    ap.add_argument("--mode", choices=("replicas", "shard"), default="shard",
                    help="N>1: one C4 session node-sharded over the GPUs (default; SURVEY.md §8e: per batched pop "
                         "each shard sweeps its node range to its top-64, one RCCL all-gather, identical placement "
                         "on every shard), or N independent replica sessions")
    ap.add_argument("--exchange", choices=("mailbox", "rccl"), default="mailbox",
                    help="shard mode: batched pops exchange their top-64 lists through peer mailboxes written by "
                         "the kernels over xGMI (default; kbhip_shard_connect_mailbox), or one ncclAllGather per pop")
    args = ap.parse_args()
    EXCHANGE_MODE[0] = args.exchange
    return args


EXCHANGE_MODE = ["mailbox"]


# Rehearsal knobs (not used by the driver's runs): KBHIP_BENCH_BACKEND=gloo and
# KBHIP_BENCH_ONE_DEVICE=1 run the N-rank path with every rank on GPU 0 (the
# engine's RCCL communicator then cannot form and the exchange falls back to
# the torch.distributed callbacks).
BACKEND = os.environ.get("KBHIP_BENCH_BACKEND", "nccl")
ONE_DEVICE = os.environ.get("KBHIP_BENCH_ONE_DEVICE", "0") == "1"


def dist_setup(n):
    if n <= 1:
        return 0, 1, 0, None
    import torch
    import torch.distributed as dist
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    local = 0 if ONE_DEVICE else int(os.environ.get("LOCAL_RANK", rank))
    torch.cuda.set_device(local)
    dist.init_process_group(BACKEND)
    return rank, world, local, dist


def _dev(local):
    return f"cuda:{local}" if BACKEND == "nccl" else "cpu"


def barrier(dist, local):
    if dist is None:
        return
    import torch
    t = torch.zeros(1, device=_dev(local))
    dist.all_reduce(t)
    torch.cuda.synchronize(local)


def allmax(dist, local, x):
    if dist is None:
        return x
    import torch
    t = torch.tensor([x], dtype=torch.float64, device=_dev(local))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def allmin(dist, local, x):
    import torch
    t = torch.tensor([x], dtype=torch.float64, device=_dev(local))
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return float(t.item())


def allsum(dist, local, x):
    if dist is None:
        return x
    import torch
    t = torch.tensor([x], dtype=torch.float64, device=_dev(local))
    dist.all_reduce(t)
    return float(t.item())


def snapshot_path(args):
    os.makedirs(args.cache, exist_ok=True)
    p = os.path.join(args.cache, f"c4_{args.nodes}_{args.pending}_{kbgen.BASE_SEED + 4}.kbs")
    if not os.path.exists(p):
        tmp = p + f".tmp{os.getpid()}"
        kbgen.gen_c4(tmp, n_nodes=args.nodes, n_pending=args.pending)
        os.replace(tmp, p)
    return p


def pmc_traffic(engine=False):
    """HBM bytes per k_pop_batch launch (engine: per pop of k_engine, whose one
    dispatch serves a session's pops) from the newest committed rocprofv3 PMC
    summary (profiles/<tag>_summary.json: FETCH_SIZE x 2, the gfx950 correction
    of MI355X_MICROARCH.md).  PMC counters cannot be read inside a timed run,
    so this comes from the profiling pass of profiles/run_profile.sh."""
    import glob
    best = None
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_summary.json"))):  # tags sort by round
        with open(p) as f:
            d = json.load(f)
        for name, k in d.get("kernels", {}).items():
            if engine and name.startswith("kbhip::k_engine") and "hbm_bytes_per_pop_corrected" in k:
                best = (k["hbm_bytes_per_pop_corrected"], os.path.basename(p))
            elif not engine and name.startswith("kbhip::k_pop_batch") and "hbm_bytes_per_launch_corrected" in k:
                best = (k["hbm_bytes_per_launch_corrected"], os.path.basename(p))
    return best


EXCHANGE = ["rccl"]
RCCL_ID = [None]  # one unique id per run: every session's connect reuses the engine's pooled communicator


def open_sharded(buf, device, rank, world, dist):
    """The shard of the session on this rank's GPU, connected over RCCL (the
    engine's own communicator: ncclAllGather / ncclAllReduce on the session
    stream).  If that communicator cannot be created, the exchange goes
    through torch.distributed's RCCL process group as host callbacks instead
    (same placements; reported in config.exchange)."""
    s = kbhip.ShardedSession(buf, device, rank, world)
    if ONE_DEVICE:  # RCCL forms no communicator with two ranks on one GPU
        EXCHANGE[0] = f"torch.distributed {BACKEND} (host callbacks)"
    if EXCHANGE[0] == "rccl":
        if RCCL_ID[0] is None:  # ncclCommInitRank once per run, not per session (kbhip CommPool)
            box = [kbhip.ShardedSession.rccl_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(box, src=0)
            RCCL_ID[0] = box[0]
        try:
            s.connect_rccl(RCCL_ID[0])
            ok = 1.0
        except kbhip.KbhipError as e:
            print(f"rank {rank}: engine RCCL communicator failed ({e}); torch.distributed callbacks", file=sys.stderr)
            ok = 0.0
        if allmin(dist, device, ok) < 1.0:
            EXCHANGE[0] = f"torch.distributed {BACKEND} (host callbacks)"
            if ok:  # this rank's engine communicator formed: drop it, so every rank exchanges the same way
                s.close()
                s = kbhip.ShardedSession(buf, device, rank, world)
    dev = f"cuda:{device}" if BACKEND == "nccl" else None
    if EXCHANGE[0] != "rccl":
        s.connect_host(kbhip.torch_exchange(device=dev), kbhip.torch_gather(device=dev))
    if EXCHANGE_MODE[0] == "mailbox":  # batched pops: peer mailboxes; the all-reduce above stays for per-task pops
        s.connect_mailbox(kbhip.torch_gather(device=dev))
    return s


def run_session(buf, device, time_every, shard=None, overlap=1, speculate=4, keep_log=False, engine=1,
                engine_workers=0, engine_lists=0, engine_groups=-1):
    t0 = time.perf_counter()
    s = open_sharded(buf, device, *shard) if shard else kbhip.Session(buf, device=device)
    s.set_option("time_every", time_every)
    s.set_option("overlap", overlap)
    s.set_option("speculate", speculate)
    s.set_option("engine", engine)
    s.set_option("engine_workers", engine_workers)
    if engine_groups >= 0:
        s.set_option("engine_groups", engine_groups)
    s.set_option("engine_lists", engine_lists)
    t1 = time.perf_counter()
    pod, node, kind = s.allocate(cap=1 << 21)
    t2 = time.perf_counter()
    st = s.stats()
    s.close()
    t3 = time.perf_counter()
    st["phases_ms"] = {"open": (t1 - t0) * 1e3, "allocate": (t2 - t1) * 1e3, "close": (t3 - t2) * 1e3}
    if keep_log:
        st["log"] = (pod, node, kind)
    return t3 - t0, len(pod), st


def sweep_counters(nodes):
    """The newest committed rocprofv3 summary of the standalone sweep at this
    node count, cold (profiles/<tag>_<nodes>_cold_summary.json, written by
    profiles/r06_sweep_scaling.sh): the kernel's own mean duration and its
    FETCH_SIZE x 2 read bytes per launch (PMC cannot be read in a timed run)."""
    import glob
    best = None
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_{nodes}_cold_summary.json"))):
        with open(p) as f:
            d = json.load(f)
        for name, k in d.get("kernels", {}).items():
            if name.startswith("kbhip::k_score_sweep") and "hbm_bytes_per_launch_corrected" in k:
                best = (k, os.path.basename(p))
    if best is None:
        return None
    k, src = best
    rd = k["hbm_bytes_per_launch_corrected"]
    wr = k["write_size_kb_per_launch"] * 1024.0 if "write_size_kb_per_launch" in k else nodes * SWEEP_B_WRITE
    gbs = (rd + wr) / (k["mean_us"] * 1e-6) / 1e9
    return {"source": f"profiles/{src}", "kernel_mean_us": k["mean_us"], "read_bytes_per_launch": rd,
            "write_bytes_per_launch": wr, "achieved": gbs, "frac": gbs / HBM_PEAK_GBS,
            "note": "over the kernel's own rocprofv3 duration, cold; read = FETCH_SIZE x 2 (the gfx950 "
                    "correction: 41 B/node, what the kernel addresses), write = WRITE_SIZE (8.1 B/node: the keys)"}


def sweep_line(s, nodes, ids, warm_n, cold_n):
    s.set_option("time_sweeps_cold", 0)
    s.time_sweeps(ids[:16])  # warm
    mean_us = s.time_sweeps(ids[:warm_n])
    s.set_option("time_sweeps_cold", 2)
    cold_us = s.time_sweeps(ids[:cold_n])
    s.set_option("time_sweeps_cold", 0)
    b = nodes * SWEEP_B_NODE
    warm = b / (mean_us * 1e-6) / 1e9 if mean_us > 0 else 0.0
    cold = b / (cold_us * 1e-6) / 1e9 if cold_us > 0 else 0.0
    return {"nodes": nodes, "bytes_per_launch": b, "launches": int(min(warm_n, len(ids))), "mean_us": mean_us,
            "achieved": warm, "frac": warm / HBM_PEAK_GBS,
            "cold": {"launches": int(min(cold_n, len(ids))), "mean_us": cold_us, "achieved": cold,
                     "frac": cold / HBM_PEAK_GBS},
            "counters": sweep_counters(nodes)}


SWEEP_TIMING = ("warm: HIP events around back-to-back launches (kbhip_time_sweeps) / launches, the columns "
                "staying in the 256 MB Infinity Cache; cold: HIP events around each launch alone behind a 512 MB "
                "read that evicts L2 and the Infinity Cache (option time_sweeps_cold = 2), dispatch and drain "
                "included; bytes = 41 B read (flags, acpu / amem / nzc / nzm, pods, maxtasks) + 8 B key written "
                "per node")


def sweep_roofline(buf, device, pods, cache, big_nodes, n_tasks=512):
    """The standalone predicate + score sweep: kbhip_sweep_scores' kernel
    (k_score_sweep: every node's PredicateFn + NodeOrderFn key,
    preempt.go:270-287) for pending tasks of the session, on the C4 session
    itself (100k nodes: bounded by the launch) and on a
    C4-shaped cluster of big_nodes nodes (same SKU mix and task classes, no
    running pods), where one launch is long enough to be bounded by HBM
    (outside the timed steps)."""
    with kbhip.Session(buf, device=device) as s:
        step = max(1, len(pods) // n_tasks)
        ids = np.ascontiguousarray(pods[::step][:n_tasks], np.int32)
        out = sweep_line(s, s.stats()["nodes"], ids, n_tasks, 64)
    out["kernel"] = "k_score_sweep (kbhip_sweep_scores)"
    out["timing"] = SWEEP_TIMING
    if big_nodes:
        path = os.path.join(cache, f"sweep_{big_nodes}_20000.kbs")
        if not os.path.exists(path):
            os.makedirs(cache, exist_ok=True)
            tmp = f"{path}.{os.getpid()}.tmp"
            kbgen.gen_c4(tmp, n_nodes=big_nodes, n_pending=20_000, running_per_node=0)
            os.replace(tmp, path)
        with open(path, "rb") as f:
            big = f.read()
        with kbhip.Session(big, device=device) as s:
            ids = np.arange(0, 20_000, 20_000 // 128, dtype=np.int32)[:128]
            out["at_scale"] = sweep_line(s, big_nodes, ids, 128, 32)
        del big
    return out


def cpu_baseline(path, target_s, log):
    """The hoisted restatement on a stratified sample of the same session:
    three windows of the session's task sequence (around 1/6, 1/2 and 5/6 of
    the tasks tried) swept and timed; every other task fast-forwarded from
    the engine's log."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # the checker / CPU baseline only (test infrastructure)
    threads = min(16, os.cpu_count() or 1)
    pod, node, kind = log
    status = np.where(kind == kbhip.ALLOCATED, 4, 8).astype(np.int32)  # api.Allocated / api.Pipelined
    probe = oracle.fast_allocate_sampled(path, pod, node, status, [(0, 200)], threads=threads)
    T = probe["session_tasks"]
    per_task = probe["timed_s"] / max(probe["tasks_swept"], 1)
    W = int(max(50, min(T // 6, target_s / 3 / max(per_task, 1e-9))))
    strata, placed, secs, swept, mism = [], 0, 0.0, 0, probe["mismatches"]
    est_alloc_s = 0.0
    for c in (T // 6, T // 2, 5 * T // 6):
        lo = max(0, c - W // 2)
        r = oracle.fast_allocate_sampled(path, pod, node, status, [(lo, lo + W)], threads=threads)
        strata.append({"tasks": [lo, lo + r["tasks_swept"]], "placed": r["placed"], "s": round(r["timed_s"], 3)})
        placed += r["placed"]
        swept += r["tasks_swept"]
        secs += r["timed_s"]
        mism += r["mismatches"]
        est_alloc_s += r["timed_s"] / max(r["tasks_swept"], 1) * (T / 3)  # this stratum's third of the tasks
    return {"value": placed / secs, "unit": "placements/s", "cores": threads, "kind": "port",
            "p50_allocate_ms_est": est_alloc_s * 1e3,
            "session_placements_per_s_est": len(pod) / est_alloc_s,
            "strata": strata, "log_mismatches": mism,
            "sample": f"3 windows of {W} tasks (around 1/6, 1/2, 5/6 of the {T} tasks the session tries) of the "
                      f"same C4 session, swept and timed ({swept} tasks, {placed} placements); every other task "
                      f"fast-forwarded from the engine's placement log (the swept decisions are checked against it: "
                      f"{mism} differ); allocate action only, hoisted C++ restatement oracle/kbfast.cpp, {threads} "
                      f"threads on {os.cpu_count()} host cpus; p50_allocate_ms_est = the whole session's allocate "
                      f"extrapolated per stratum"}


def main():
    args = parse()
    rank, world, local, dist = dist_setup(args.gpus)
    path = snapshot_path(args) if rank == 0 or dist is None else None
    barrier(dist, local)
    if path is None:
        path = snapshot_path(args)
    with open(path, "rb") as f:
        buf = f.read()
    device = local
    shard = (rank, world, dist) if (args.mode == "shard" and world > 1) else None
    for _ in range(args.warmup):
        run_session(buf, device, 0, shard, args.overlap, args.speculate, engine=args.engine,
                    engine_workers=args.engine_workers, engine_lists=args.engine_lists,
                    engine_groups=args.engine_groups)
    barrier(dist, local)
    t0 = time.perf_counter()
    lat, placed, sweeps_ms, sweeps_n, st_last = [], 0, 0.0, 0, None
    dev_s, dev_pops = 0.0, 0
    for i in range(args.steps):
        dt, n, st = run_session(buf, device, args.time_every, shard, args.overlap,
                                args.speculate, keep_log=(i == 0 and rank == 0), engine=args.engine,
                                engine_workers=args.engine_workers, engine_lists=args.engine_lists,
                                engine_groups=args.engine_groups)
        lat.append(dt)
        placed += n
        sweeps_ms += st["device_s"] * 1e3
        sweeps_n += st["timed_launches"]
        dev_s += st["alloc_device_s"]
        dev_pops += st["batched_pops"]
        if "log" in st:
            log0 = st.pop("log")
        st_last = st
    barrier(dist, local)
    wall = time.perf_counter() - t0
    wall = allmax(dist, local, wall)
    # replicas: every rank schedules its own session; shard: one session shared by all ranks
    total_placed = placed if shard else allsum(dist, local, placed)
    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return
    nodes = st_last["nodes"]
    traffic = None if shard else pmc_traffic(st_last["engine_pops"] > 0)
    sweep = None if shard else sweep_roofline(buf, device, log0[0], args.cache, args.sweep_nodes)
    nodes_per_launch = (nodes + world - 1) // world if shard else nodes  # a shard sweeps its own range
    # the hot kernel's mean duration: HIP events around every batched pop launch on the stream it runs on
    # (overlapped pops: the duration includes the wait for the previous pop's write-back, as rocprof's does)
    launch_us = (sweeps_ms / max(sweeps_n, 1)) * 1e3 if sweeps_n else 0.0
    engine_on = st_last["engine_pops"] > 0
    kernel = "k_pop_batch (shard sweep, placement 3)" if shard else (
        "k_engine (persistent pop engine)" if engine_on else "k_pop_batch_ov" if args.overlap else "k_pop_batch")
    period_us = dev_s / dev_pops * 1e6 if dev_pops else 0.0
    # the kernel's busy period per launch: allocate's device span (HIP events on the engine streams) / launches
    achieved = nodes_per_launch * B_NODE / (period_us * 1e-6) / 1e9 if period_us > 0 else 0.0
    span_achieved = nodes_per_launch * B_NODE / (launch_us * 1e-6) / 1e9 if launch_us > 0 else 0.0
    out = {
        "metric": METRIC,
        "value": total_placed / wall,
        "unit": "placements/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": wall / args.steps * 1e3,
        "p50_session_ms": statistics.median(lat) * 1e3,
        "higher_is_better": True,
        "scaling": "strong" if shard else "weak",
        "vs_baseline": None,
        "dtype": "int64",
        "data": "synthetic (kbgen seed 20261015+4, C4 SKU mix, gang jobs minMember 8-64)",
        "config": {"workload": "C4: 100k nodes x 1M pods (200k running, 800k pending), 1 allocate session per "
                               "step, default kube-batch-conf tiers", "nodes": nodes, "pending": args.pending,
                   "placements_per_session": placed // args.steps, "pops_per_session": st_last["pops"],
                   "sweeps_per_session": st_last["sweeps"], "batched_pops": st_last["batched_pops"],
                   "open_s": st_last["open_s"], "allocate_s": st_last["allocate_s"],
                   "overlap": args.overlap, "speculate": args.speculate, "alloc_device_s": st_last["alloc_device_s"],
                   "engine_pops": st_last["engine_pops"], "engine_launches": st_last["engine_launches"],
                   "engine_workers": st_last["engine_workers"],
                   "engine_owners": st_last["engine_owners"],
                   "host_launch_s": st_last["host_launch_s"], "host_wait_s": st_last["host_wait_s"],
                   "spec_hits": st_last["spec_hits"], "spec_missed": st_last["spec_missed"],
                   "unassigned_pops": st_last["unassigned_pops"], "collectives": st_last["collectives"],
                   "session_phases_ms": {k: round(v, 2) for k, v in st_last["phases_ms"].items()},
                   "device_period_us": period_us,  # allocate's device span / batched launches (launches overlap)
                   "parallelism": (f"node-sharded x{world}" if shard else f"replicas x{world}") if world > 1
                   else "1 GPU",
                   "exchange": (f"peer mailboxes (per-task pops: {EXCHANGE[0]})" if EXCHANGE_MODE[0] == "mailbox"
                                else EXCHANGE[0]) if shard else None},
        "roofline": {"kernel": kernel, "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                     "traffic": traffic[0] if traffic else None,
                     "traffic_source": (f"profiles/{traffic[1]} (rocprofv3 FETCH_SIZE x2, bytes per "
                                        f"{'pop' if engine_on else 'launch'})") if traffic else None,
                     "busy_period_us": period_us,
                     "timing": ("busy period = allocate's device span (HIP events on the session stream around the "
                                "allocate action, summed over the timed sessions) / batched pops: the engine's one "
                                "dispatch per session serves them all, each pop's nodes evaluated once")
                     if engine_on else
                     ("busy period = allocate's device span (HIP events on the engine streams around the "
                      "allocate action, summed over the timed sessions) / batched pop launches: the launches "
                      "overlap, so this is the device time each one adds; the sum over launches = the span"),
                     "bytes_per_launch": nodes_per_launch * B_NODE,
                     "sweep": sweep},
    }
    if not engine_on:
        out["roofline"]["span_us"] = launch_us
        out["roofline"]["span_frac"] = span_achieved / HBM_PEAK_GBS
        out["roofline"]["span_timing"] = (f"each launch's own start-to-end span (HIP events around every "
                                          f"{args.time_every}-th launch on its stream, {sweeps_n} launches): it "
                                          f"includes the wait for the previous pop, so consecutive spans overlap")
    if args.cpu_baseline and world == 1:
        out["cpu_baseline"] = cpu_baseline(path, args.cpu_seconds, log0)
        out["cpu_baseline"]["gpu_p50_session_ms"] = out["p50_session_ms"]
    print(json.dumps(out))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
