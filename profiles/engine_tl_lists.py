#!/usr/bin/env python3
"""Event timeline of the persistent pop engine in list mode (diagnostic;
option "engine_timeline", kbhip_engine.hip ETL stamps, 100 MHz): one C4
session, then per-phase medians.  Prints one JSON line.

Placer events as in engine_tl.py (0 iteration start .. 8 granules stored, 15
the next pop's package in LDS).  The owner of pop p's class:
20 pop p seen among the descriptors, 10 package start (rows applied up to pop
p-4), 11 pop p-2's candidates seen, 12 entries sorted, 13 package stored, 18
FitDelta counts stored.  28: dispatcher forwarded."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kube-batch-1_amd"))
import kbgen  # noqa: E402
import kbhip  # noqa: E402

SLOTS, EV = 32768, 64


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=100_000)
    ap.add_argument("--pending", type=int, default=800_000)
    ap.add_argument("--lists", type=int, default=1)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    path = f"/tmp/kbhip_bench/c4_{a.nodes}_{a.pending}_{kbgen.BASE_SEED + 4}.kbs"
    if not os.path.exists(path):
        os.makedirs(os.path.dirname(path), exist_ok=True)
        kbgen.gen_c4(path, n_nodes=a.nodes, n_pending=a.pending)
    buf = open(path, "rb").read()
    with kbhip.Session(buf) as s:  # warm
        s.set_option("engine_lists", a.lists)
        s.allocate()
    with kbhip.Session(buf) as s:
        s.set_option("engine_lists", a.lists)
        s.set_option("engine_timeline", 1)
        s.allocate()
        st = s.stats()
        raw = np.zeros(SLOTS * EV, np.uint64)
        n = kbhip.lib().kbhip_debug_table(s._h, b"engine_tl", raw.ctypes.data, raw.nbytes)
        assert n == raw.nbytes
    t = raw.reshape(SLOTS, EV).astype(np.int64)
    pops = t[:, 31]
    order = np.argsort(pops)
    t, pops = t[order], pops[order]
    need = [0, 1, 3, 4, 5, 6, 7, 8, 15, 28] + ([10, 11, 12, 13, 20] if a.lists else [])
    keep = (pops > 100) & np.all(t[:, need] > 0, axis=1)
    t = t[keep]
    pops = t[:, 31]
    cont = np.diff(pops) == 1
    us = lambda x: round(float(np.median(x)) / 100.0, 3)  # 100 MHz ticks -> us
    prev = lambda k: (pops[k:] - pops[:-k]) == k
    per = {}
    per["period"] = us(np.diff(t[:, 0])[cont])
    per["placer 0->3 P2"] = us(t[:, 3] - t[:, 0])
    per["placer 3->4 P3"] = us(t[:, 4] - t[:, 3])
    per["placer 5->6 decided"] = us(t[:, 6] - t[:, 5])
    per["placer 6->7 rows written"] = us(t[:, 7] - t[:, 6])
    per["placer 7 -> next 0"] = us((t[1:, 0] - t[:-1, 7])[cont])
    per["placer 5->15 next package in LDS"] = us(t[:, 15] - t[:, 5])
    for ev, name in ((19, "wave 1 (pop p-1 cands key)"), (29, "wave 5 (host out + eval)"), (16, "wave 7 (eval + package)"),
                     (17, "wave 6 (eval + package)"), (14, "wave 4 (eval + package)"), (23, "wave 2 (hash)")):
        ok = t[:, ev] > 0
        if ok.any():
            per[f"placer 5->{ev} front {name}"] = us((t[:, ev] - t[:, 5])[ok])
    per["P2 wave0 drop (0->1)"] = us(t[:, 1] - t[:, 0])
    per["P3: 3->44 merge"] = us(t[:, 44] - t[:, 3])
    per["P3: 44->45 publish done (vmcnt)"] = us(t[:, 45] - t[:, 44])
    per["P3: 45->46 cands / log stores"] = us(t[:, 46] - t[:, 45])
    per["P3: 46->4 rc_find, srcslot"] = us(t[:, 4] - t[:, 46])
    per["finish: 6->47 fit counts"] = us(t[:, 47] - t[:, 6])
    per["finish: 47->27 rows_seq"] = us(t[:, 27] - t[:, 47])
    per["finish: 27->7 write-back issued"] = us(t[:, 7] - t[:, 27])
    for st_, nm in ((0, "set 0 (pop p cands)"), (1, "set 1"), (2, "set 2")):
        b = 32 + 4 * st_
        ok = np.all(t[:, [b, b + 1, b + 2, b + 3]] > 0, axis=1)
        if ok.any():
            per[f"front {nm}: start(5)->rows ready"] = us((t[:, b] - t[:, 5])[ok])
            per[f"front {nm}: eval"] = us((t[:, b + 1] - t[:, b])[ok])
            per[f"front {nm}: ->hashed"] = us((t[:, b + 2] - t[:, b + 1])[ok])
            per[f"front {nm}: sort"] = us((t[:, b + 3] - t[:, b + 2])[ok])
            per[f"front {nm}: end - 5"] = us((t[:, b + 3] - t[:, 5])[ok])
    if a.lists:
        per["owner seen(20) - placer start(0)"] = us(t[:, 20] - t[:, 0])
        per["owner seen(20) -> start(10)"] = us(t[:, 10] - t[:, 20])
        per["owner start(10) - placer start(0)"] = us(t[:, 10] - t[:, 0])
        per["owner start(10,p) - placer P3(4,p-3) (done p-4)"] = us((t[3:, 10] - t[:-3, 4])[prev(3)])
        per["owner 10 -> 21 (p-3 cands, hash)"] = us(t[:, 21] - t[:, 10])
        per["owner 21 -> 24 (threshold, wave 0)"] = us(t[:, 24] - t[:, 21])
        per["owner 24 -> 26 (scan)"] = us(t[:, 26] - t[:, 24])
        per["owner 26 -> 12 (sort)"] = us(t[:, 12] - t[:, 26])
        per["owner sorted(12) - placer P3(4,p-2)"] = us((t[2:, 12] - t[:-2, 4])[prev(2)])
        per["owner p-2 cands seen(11,p) - placer P3(4,p-2)"] = us((t[2:, 11] - t[:-2, 4])[prev(2)])
        per["owner p-2 seen(11) -> stored(13)"] = us(t[:, 13] - t[:, 11])
        per["owner stored(13) - placer start(0)"] = us(t[:, 13] - t[:, 0])
    res_extra = {} if not a.lists else {"active_segments_quantiles": [float(np.quantile(t[:, 25] & 0xff, q)) for q in (0.1, 0.5, 0.9)],
                 "thr_quantiles": [float(np.quantile(t[:, 25] >> 8, q)) for q in (0.1, 0.5, 0.9)]}
    if a.lists:
        per["owner stored(13,p) - placer 5(p-1) front start"] = us((t[1:, 13] - t[:-1, 5])[cont])
        per["owner stored(13,p) - placer 15(p-1) package in LDS"] = us((t[1:, 13] - t[:-1, 15])[cont])
    for k, wv in enumerate((3, 4, 6, 7)):  # the package-loading waves of the front (r06 events)
        for ev, nm in ((56 + k, "eval done"), (48 + k, "package in registers"), (52 + k, "package in LDS")):
            ok = t[:, ev] > 0
            if ok.any():
                per[f"front wave {wv}: {nm} - 5"] = us((t[:, ev] - t[:, 5])[ok])
    for ev, nm in ((63, "wave 2: hash built"), (62, "wave 3: hash seen"), (60, "wave 3: stale dropped"),
                   (61, "wave 3: pre-merged")):
        ok = t[:, ev] > 0
        if ok.any():
            per[f"front {nm} - 5"] = us((t[:, ev] - t[:, 5])[ok])
    per["dispatch(28) - placer start(0)"] = us(t[:, 28] - t[:, 0])
    per_all = np.diff(t[:, 0])[cont] / 100.0
    res = {"pops": int(len(t)), "lists": a.lists,
           "stats": {k: st[k] for k in ("engine_pops", "engine_launches", "engine_workers", "engine_owners",
                                        "alloc_device_s", "batched_pops", "host_wait_s")},
           "median_us": per, "extra": res_extra,
           "period_us": {"mean": round(float(per_all.mean()), 3),
                         "quantiles_10_50_90_99": [round(float(np.quantile(per_all, q)), 2) for q in (0.1, 0.5, 0.9, 0.99)]}}
    print(json.dumps(res))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
