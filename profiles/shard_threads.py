"""Rehearsal of the node-sharded C4 session (bench.py --mode shard, mailbox
exchange) with its W ranks as threads of ONE process on ONE GPU: every rank
has its own session, streams and node shard; the peer mailboxes are plain
device pointers between them (kbhip_shard_connect_mailbox's same-process
case), so the GPU runs the ranks' kernels side by side instead of
time-slicing between processes — what W GPUs over xGMI see, minus the link
latency, with the W sweeps sharing one chip.  Every rank's placement log is
checked against the C4 digest (tests/golden/fullsize.json).

usage (on the box, repo root): python3 profiles/shard_threads.py <tag> [W] [sessions] [shard_overlap] [cu_split]
(shard_overlap 1, the default: a shard's sweep of pop e beside pop e-1's
placement; 0: sweep, exchange and placement one after another; cu_split 1:
rank r's streams run on CUs [r C / W, (r + 1) C / W) only — option
"cu_split" — so that each rank has its own share of the chip, as W GPUs
would, instead of all ranks' kernels spreading over every CU)
"""
import hashlib
import json
import os
import statistics
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kube-batch-1_amd"))
import kbgen  # noqa: E402
import kbhip  # noqa: E402


class Gather:
    """An all-gather among the W rank threads of this process."""

    def __init__(self, w):
        self.w, self.bar, self.slots = w, threading.Barrier(w), [None] * w

    def fn(self, rank):
        def g(send, recv):
            self.slots[rank] = bytes(send)
            self.bar.wait()
            recv[:] = np.frombuffer(b"".join(self.slots), np.uint8)
            self.bar.wait()
        return g


class Reduce:
    def __init__(self, w):
        self.w, self.bar, self.slots = w, threading.Barrier(w), [None] * w

    def fn(self, rank):
        def r(vals, op):
            v = vals.view(np.int64).copy()
            if op == kbhip.RED_MAX_U64:
                v = (vals.copy()).astype(np.uint64)
            self.slots[rank] = v
            self.bar.wait()
            a = np.stack(self.slots)
            if op == kbhip.RED_MAX_U64:
                out = a.max(axis=0).astype(np.uint64)
            elif op == kbhip.RED_MIN_I64:
                out = a.min(axis=0).view(np.uint64)
            elif op == kbhip.RED_SUM_I64:
                out = a.sum(axis=0).view(np.uint64)
            else:
                out = a.max(axis=0).view(np.uint64)
            self.bar.wait()
            vals[:] = out
        return r


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r03"
    w = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    sessions = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    shov = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    cus = int(sys.argv[5]) if len(sys.argv) > 5 else 0
    cache = os.environ.get("KBHIP_BENCH_CACHE", "/tmp/kbhip_bench")
    os.makedirs(cache, exist_ok=True)
    path = os.path.join(cache, f"c4_100000_800000_{kbgen.BASE_SEED + 4}.kbs")
    if not os.path.exists(path):
        kbgen.gen_c4(path)
    buf = open(path, "rb").read()
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "fullsize.json")))["c4"]
    rows = []
    for it in range(sessions + 1):  # the first session warms up
        gat, red = Gather(w), Reduce(w)
        res = [None] * w

        def run(rank):
            t0 = time.perf_counter()
            s = kbhip.ShardedSession(buf, 0, rank, w)
            if cus:
                s.set_option("cu_split", rank * 256 + w)
            s.connect_host(red.fn(rank))
            s.connect_mailbox(gat.fn(rank))
            s.set_option("shard_overlap", shov)
            t1 = time.perf_counter()
            pod, node, kind = s.allocate(cap=1 << 21)
            t2 = time.perf_counter()
            st = s.stats()
            s.close()
            status = np.where(np.asarray(kind) == 1, 4, 8)
            dig = hashlib.sha256(np.stack([pod, node, status]).astype(np.int32).tobytes()).hexdigest()
            res[rank] = dict(open_s=t1 - t0, allocate_s=t2 - t1, session_s=time.perf_counter() - t0,
                             placed=len(pod), digest_ok=dig == gold["log_sha256"], pops=st["batched_pops"],
                             collectives=st["collectives"], alloc_device_s=st["alloc_device_s"],
                             period_us=st["alloc_device_s"] / max(st["batched_pops"], 1) * 1e6)
        th = [threading.Thread(target=run, args=(r,)) for r in range(w)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        if it > 0:
            rows.append(res)
        print(json.dumps({"session": it, "ranks": res}), file=sys.stderr, flush=True)
    out = {"what": f"C4 (100k nodes x 1M pods) node-sharded over {w} rank threads of one process on one MI355X, "
                   "peer-mailbox exchange (kbhip_shard_connect_mailbox)",
           "ranks": w, "sessions": sessions, "shard_overlap": shov, "cu_split": cus,
           "all_digests_ok": all(r["digest_ok"] for res in rows for r in res),
           "p50_session_ms": statistics.median(max(r["session_s"] for r in res) for res in rows) * 1e3,
           "p50_allocate_ms": statistics.median(max(r["allocate_s"] for r in res) for res in rows) * 1e3,
           "placements_per_s": rows[-1][0]["placed"] / statistics.median(max(r["session_s"] for r in res)
                                                                         for res in rows),
           "device_period_us": statistics.median(max(r["period_us"] for r in res) for res in rows),
           "one_exchange_per_pop": all(r["collectives"] == r["pops"] for res in rows for r in res),
           "last": rows[-1]}
    os.makedirs("gpurun_out", exist_ok=True)
    with open(f"gpurun_out/{tag}_shard_threads_w{w}_ov{shov}_cu{cus}.json", "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
