#!/usr/bin/env python3
"""Event timeline of the persistent pop engine (diagnostic; option
"engine_timeline", kbhip_engine.hip ETL stamps, 100 MHz): one C4 session,
then per-phase medians over the last kEngTlSlots pops.  Prints one JSON line.

Placer events: 0 iteration start, 1 descriptor, 2 package loaded, 3 drop +
patch done, 4 list published + rows, 5 placement start, 6 decided, 7 rows
written (stores issued), 8 granules stored (wave 5).  Final merger: 20
descriptor, 21 lists merged, 22 package flag.  Workers (blocks 0 and nw/2: 10.. / 16..): descriptor, done(p-3),
evaluated, list published, counts published.  Merger 0: 24 descriptor, 25
lists in, 26 group list published, 27 counts.  28: dispatcher forwarded."""
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
    ap.add_argument("--workers", type=int, default=0)
    ap.add_argument("--groups", type=int, default=-1)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    path = f"/tmp/kbhip_bench/c4_{a.nodes}_{a.pending}_{kbgen.BASE_SEED + 4}.kbs"
    if not os.path.exists(path):
        os.makedirs(os.path.dirname(path), exist_ok=True)
        kbgen.gen_c4(path, n_nodes=a.nodes, n_pending=a.pending)
    buf = open(path, "rb").read()
    with kbhip.Session(buf) as s:  # warm
        s.allocate()
    with kbhip.Session(buf) as s:
        s.set_option("engine_workers", a.workers)
        s.set_option("engine_groups", a.groups)
        s.set_option("engine_timeline", 1)
        s.allocate()
        st = s.stats()
        raw = np.zeros(SLOTS * EV, np.uint64)
        n = kbhip.lib().kbhip_debug_table(s._h, b"engine_tl", raw.ctypes.data, raw.nbytes)
        assert n == raw.nbytes
    t = raw.reshape(SLOTS, EV).astype(np.int64)
    pops = t[:, 31]
    order = np.argsort(pops)
    t = t[order]
    pops = pops[order]
    keep = (pops > 100) & np.all(t[:, [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 15, 28]] > 0, axis=1)
    t = t[keep]
    pops = t[:, 31]
    cont = np.diff(pops) == 1
    us = lambda x: float(np.median(x)) / 100.0  # 100 MHz ticks -> us
    res = {"pops": int(len(t)), "workers": a.workers, "groups": a.groups, "all_stats": {k: (v if isinstance(v, (int, float)) else str(v)) for k, v in st.items()}, "stats": {k: st[k] for k in ("engine_pops", "engine_launches", "engine_workers",
                                                             "alloc_device_s", "batched_pops", "host_wait_s")}}
    per = {}
    per["period"] = us(np.diff(t[:, 0])[cont])
    per["placer 0->3 drop+patch"] = us(t[:, 3] - t[:, 0])
    per["placer 3->4 final list + rows"] = us(t[:, 4] - t[:, 3])
    per["placer 4->5 barrier"] = us(t[:, 5] - t[:, 4])
    per["placer 5->6 decided"] = us(t[:, 6] - t[:, 5])
    per["placer 6->7 rows written"] = us(t[:, 7] - t[:, 6])
    per["placer 6->8 granules (wave 5)"] = us(t[:, 8] - t[:, 6])
    per["placer 5->15 front of next (wave 3, package)"] = us(t[:, 15] - t[:, 5])
    for ev, name in ((19, "wave 1 (pop p-1 cands key)"), (29, "wave 5 (host out + eval)"), (16, "wave 7 (eval + package)"),
                     (17, "wave 6 (eval + package)"), (14, "wave 4 (eval + package)"), (23, "wave 2 (hash)")):
        ok = t[:, ev] > 0
        if ok.any():
            per[f"placer 5->{ev} front {name}"] = us((t[:, ev] - t[:, 5])[ok])
    per["P2 wave0 drop (0->1)"] = us(t[:, 1] - t[:, 0])
    per["P2 wave1 start (0->2)"] = us(t[:, 2] - t[:, 0])
    per["P2 wave1 sort (2->9)"] = us(t[:, 9] - t[:, 2])
    per["placer 7 -> next 0"] = us((t[1:, 0] - t[:-1, 7])[cont])
    # when do the lists of pop p arrive, relative to the placer's start of pop p
    fin = np.all(t[:, [20, 21, 22]] > 0, axis=1)
    if fin.any():
        per["final: package flag (22) - placer start (0)"] = us((t[:, 22] - t[:, 0])[fin])
        per["final: desc(20)->merged(21)"] = us((t[:, 21] - t[:, 20])[fin])
        per["final: merged(21)->flag(22)"] = us((t[:, 22] - t[:, 21])[fin])
        f29 = fin & (t[:, 29] > 0)
        if f29.any():
            per["final: merged(21)->cands p-2 seen(29)"] = us((t[:, 29] - t[:, 21])[f29])
            per["final: cands p-2 seen(29,p) - placer P3(4,p-2)"] = us(
                (t[2:, 29] - t[:-2, 4])[((pops[2:] - pops[:-2]) == 2) & f29[2:]])
    lw = t[:, 18] > 0
    if lw.any():
        per["last worker published (18) - worker0 published (13)"] = us((t[:, 18] - t[:, 13])[lw])
        per["last worker published (18) - placer start (0)"] = us((t[:, 18] - t[:, 0])[lw])
    mg = np.all(t[:, [24, 25, 26]] > 0, axis=1)
    if mg.any():
        per["merger0 published (26) - placer start (0)"] = us((t[:, 26] - t[:, 0])[mg])
        per["merger0 lists in (25) - placer start (0)"] = us((t[:, 25] - t[:, 0])[mg])
        per["merger0 desc(24)->lists in(25)"] = us((t[:, 25] - t[:, 24])[mg])
        per["merger0 lists in(25)->pub(26)"] = us((t[:, 26] - t[:, 25])[mg])
        per["merger0 pub(26)->counts(27)"] = us((t[:, 27] - t[:, 26])[mg])
    per["worker0 published (13) - placer start (0)"] = us(t[:, 13] - t[:, 0])
    per["worker0 desc(10)->done(11)"] = us(t[:, 11] - t[:, 10])
    per["worker0 done(11)->eval(12)"] = us(t[:, 12] - t[:, 11])
    per["worker0 eval(12)->pub(13)"] = us(t[:, 13] - t[:, 12])
    per["worker0 pub(13) -> next desc(10)"] = us((t[1:, 10] - t[:-1, 13])[cont])
    per["worker0 published (13, p) - placer P3 (4, p-2)"] = us((t[2:, 13] - t[:-2, 4])[(pops[2:] - pops[:-2]) == 2])
    per["dispatch(28) - placer start(0)"] = us(t[:, 28] - t[:, 0])
    res["median_us"] = {k: round(v, 3) for k, v in per.items()}
    stop = (t[:, 30] >> 8) & 0xff
    res["stop_hist"] = {int(k): int(v) for k, v in zip(*np.unique(stop, return_counts=True))}
    # the whole session: placer starts of every pop (pop -> start), and where the time between them goes
    t0all = t[:, 0]
    span = (t0all[-1] - t0all[0]) / 100.0
    dif = np.diff(t0all) / 100.0
    big = np.argsort(dif)[-12:][::-1]
    res["session"] = {"pops_seen": int(len(t0all)), "span_us": round(span, 1), "mean_us": round(span / max(1, len(t0all) - 1), 3),
                      "largest_gaps": [(int(pops[i]), round(float(dif[i]), 1)) for i in big],
                      "gaps_over_20us_total": round(float(dif[dif > 20].sum()), 1), "n_over_20": int((dif > 20).sum())}
    per_all = np.diff(t[:, 0])[cont] / 100.0
    res["period_us"] = {"mean": round(float(per_all.mean()), 3),
                        "quantiles_10_50_90_99": [round(float(np.quantile(per_all, q)), 2) for q in (0.1, 0.5, 0.9, 0.99)],
                        "gaps_over_20us": int((per_all > 20).sum()), "gap_time_over_20us": round(float(per_all[per_all > 20].sum()), 1)}
    # placer waiting at the loop top for the package / descriptor (front done late): 7 -> next 0
    dec = (t[:, 6] - t[:, 5]) / 100.0
    res["decide_us_quantiles"] = [round(float(np.quantile(dec, q)), 2) for q in (0.1, 0.25, 0.5, 0.75, 0.9, 0.99)]
    print(json.dumps(res))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
