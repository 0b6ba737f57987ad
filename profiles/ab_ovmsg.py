"""A/B of the overlapped pops' rows hand-off (option "ov_msg") on the C4 bench
session: alternating sessions with the option off / on, placements/s and the
per-pop device period of each.  Usage: python profiles/ab_ovmsg.py [rounds]"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "kube-batch-1_amd"))
import kbhip  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    path = os.path.join(os.environ.get("TMPDIR", "/tmp"), "kbhip_ab_c4.kbs")
    if not os.path.exists(path):
        os.makedirs(os.path.dirname(path), exist_ok=True)
        import kbgen
        kbgen.gen_c4(path)
    buf = open(path, "rb").read()
    res = {0: [], 1: []}
    for r in range(rounds + 1):
        for msg in (0, 1):
            t0 = time.perf_counter()
            s = kbhip.Session(buf, device=0)
            s.set_option("ov_msg", msg)
            pod, _, _ = s.allocate(cap=1 << 21)
            st = s.stats()
            s.close()
            dt = time.perf_counter() - t0
            if r:
                res[msg].append({"placements_per_s": len(pod) / dt, "session_ms": dt * 1e3,
                                 "period_us": st["alloc_device_s"] / st["batched_pops"] * 1e6,
                                 "msg_pops": st["msg_pops"], "batched_pops": st["batched_pops"]})
            print(json.dumps({"ov_msg": msg, "round": r, "s": dt}), flush=True)
    out = {str(m): {"median_placements_per_s": statistics.median(x["placements_per_s"] for x in v),
                    "median_period_us": statistics.median(x["period_us"] for x in v), "runs": v}
           for m, v in res.items()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
