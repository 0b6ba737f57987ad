"""Per-pop ABI at full size (C4; --config c3 / c5): kube-batch-1_amd/_build/kbhost (the C++ host
loop a Go shim keeps — allocate.go:41-201 over kbhip_place_job, or over
kbhip_place_job_submit / _wait / _cancel with `depth` predicted pops in
flight) timed beside kbhip_allocate on the same snapshot; all three logs must
be identical.  Writes one JSON line (stdout and --out).

usage: python profiles/host_loop.py [--nodes 100000] [--pending 800000] [--reps 3] [--depth 2] [--out F]"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kube-batch-1_amd"))
import kbgen  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", choices=("c4", "c3", "c5"), default="c4",
                    help="c4: --nodes x --pending; c3 / c5: the full-size generators (allocate on the snapshot)")
    ap.add_argument("--nodes", type=int, default=100_000)
    ap.add_argument("--pending", type=int, default=800_000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--depth", type=int, default=2)
    ap.add_argument("--modes", default="allocate,sync,async")
    ap.add_argument("--cache", default="/tmp")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    if a.config == "c4":
        p = os.path.join(a.cache, f"c4_{a.nodes}_{a.pending}_{kbgen.BASE_SEED + 4}.kbs")
    else:
        p = os.path.join(a.cache, f"{a.config}_full.kbs")
    if not os.path.exists(p):
        t0 = time.time()
        tmp = p + f".{os.getpid()}.tmp"
        if a.config == "c4":
            kbgen.gen_c4(tmp, n_nodes=a.nodes, n_pending=a.pending)
        elif a.config == "c3":
            kbgen.gen_c3().write(tmp)
        else:
            kbgen.gen_c5(tmp)
        os.replace(tmp, p)
        print(f"generated {p} in {time.time() - t0:.1f}s", flush=True)
    exe = os.path.join(ROOT, "kube-batch-1_amd", "_build", "kbhost")
    r = subprocess.run([exe, p, "--modes", a.modes, "--reps", str(a.reps), "--depth", str(a.depth)],
                       capture_output=True, text=True, timeout=900)
    sys.stderr.write(r.stderr)
    if r.returncode != 0:
        print(r.stdout)
        sys.exit(r.returncode)
    rec = json.loads(r.stdout.strip().splitlines()[-1])
    rec["config"] = ({"workload": "C4", "nodes": a.nodes, "pending": a.pending} if a.config == "c4" else
                     {"workload": a.config.upper() + " (allocate action on the full-size snapshot)"})
    if "allocate" in rec:
        for m in ("sync", "async"):
            if m in rec:
                rec[m]["vs_allocate"] = rec[m]["ms"] / rec["allocate"]["ms"]
    line = json.dumps(rec)
    print(line)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
