"""Placement 7 (pod anti-affinity classes) phase split with the stamps build
(kube-batch-1_amd/_build/libkbhip_stamps.so, KBHIP_LIB; diagnostic only, never
used for timing claims): a C3-like cluster where every gang is zone-self-anti-
affine (24 zones, gangs of 8..24), so every batched pop is a placement-7 pop.
Prints kbhip_debug_phases' per-launch averages (us): per-block sweep, block
merge, first block start -> all lists stored, -> final merger, final merge,
final merge end -> placement start, placement, placement end -> end, total."""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kube-batch-1_amd"))
import kbgen  # noqa: E402
import kbhip  # noqa: E402


def main():
    rng = np.random.default_rng(77)
    c = kbgen.Cluster()
    zones = [f"z{i:02d}" for i in range(24)]
    for i in range(int(sys.argv[1]) if len(sys.argv) > 1 else 20000):
        name = f"n{i:06d}"
        c.add_node(name, 32000, 128 << 30, 0, 110, labels={"zone": zones[int(rng.integers(24))],
                                                           "kubernetes.io/hostname": name})
    c.add_queue("q0", 1)
    for j in range(300):
        jn = f"g{j:04d}"
        size = int(rng.integers(8, 25))
        c.add_job("default", jn, "q0", min_member=size, ts=j)
        for k in range(size):
            c.add_pod("default", f"{jn}-{k}", uid=f"p{j:04d}{k:03d}", group=jn, ts=j, labels={"job": jn},
                      containers=[kbgen.res(cpu=500, mem=1 << 30)],
                      affinity={"anti": {"required": [{"selector": {"ml": {"job": jn}}, "topology_key": "zone"}]}})
    p = "/tmp/aff_phases.kbs"
    c.write(p)
    with kbhip.Session(p) as s:
        s.set_option("speculate", 0)
        s.set_option("overlap", 0)
        pod, node, kind = s.allocate()
        st = s.stats()
        out = (ctypes.c_double * 20)()
        n = kbhip.lib().kbhip_debug_phases(s._h, out, 20)
    names = ["sweep_block", "merge_block", "lists_stored", "to_final", "final_merge", "to_place", "place",
             "place_to_end", "total"]
    print(json.dumps({"launches": n, "placements": int(len(pod)), "seq_launches": st["seq_launches"],
                      "seq_cut": st["seq_cut"], "phases_us": {k: round(out[i], 3) for i, k in enumerate(names)}}))


if __name__ == "__main__":
    main()
