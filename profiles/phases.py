"""Diagnostic: per-phase in-kernel time of k_pop_batch on C4 (stamps build).
Shares only; the stamps build is never used for timing claims."""
import ctypes, os, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kube-batch-1_amd"))
import kbhip
kbhip.LIB_PATH = os.path.join(ROOT, "kube-batch-1_amd", "_build", "libkbhip_stamps.so")
import kbgen
p = "/tmp/kbhip_bench/c4_100000_800000_%d.kbs" % (kbgen.BASE_SEED + 4)
if not os.path.exists(p):
    os.makedirs(os.path.dirname(p), exist_ok=True)
    kbgen.gen_c4(p)
L = kbhip.lib()
overlap = int(sys.argv[1]) if len(sys.argv) > 1 else 0  # 1: the overlapped kernel, one pop at a time
with kbhip.Session(p) as s:
    s.set_option("overlap", overlap)
    s.set_option("speculate", 0)  # stamps are read per launch
    s.allocate()
    out = (ctypes.c_double * 20)()
    n = L.kbhip_debug_phases(s._h, out, 20)
    names = ["block sweep+sort", "block merge+store", "span to all block lists stored",
             "group merge tail to final start", "final merge", "chain precompute", "placement loop",
             "write back", "kernel span", "tasks per launch", "placement: rows loaded", "placement: round-0 eval",
             "placement: round-0 sort+merge", "wb: ranks+stop", "wb: LDS counts", "ov: wait for previous pop",
             "ov: patch (eval previous candidates + merge)", "placement: rows fetched", "placement: LDS init + barrier"]
    print(json.dumps({"pops": n, "overlap": overlap, **{names[i]: round(out[i], 3) for i in range(len(names))}},
                     indent=1))
