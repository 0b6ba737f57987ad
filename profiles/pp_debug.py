"""Development aid: one snapshot through the persistent placer and the
overlapped kernel, first differing record and the engine's PP debug log."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "kube-batch-1_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import kbgen  # noqa: E402
import kbhip  # noqa: E402
from test_gpu_parity import NO_POD_AFFINITY  # noqa: E402

seed = int(sys.argv[1]) if len(sys.argv) > 1 else 13
tiers = [None, [["priority", "gang"], ["drf", "predicates", "proportion", "nodeorder"]],
         [["gang"], ["predicates", "nodeorder"]]][seed % 3]
c = kbgen.gen_random(9300 + seed, n_nodes=6 + 9 * (seed % 12), n_jobs=5 + seed % 9, max_tasks=2 + seed % 14,
                     features=tuple(f for f in NO_POD_AFFINITY if f != "backfill"), tiers=tiers)
p = c.write("/tmp/ppd.kbs")
res = {}
for pp in (0, 1):
    for spec in ((2,) if pp else (2, 0)):
        with kbhip.Session(p) as s:
            s.set_option("pp", pp)
            s.set_option("speculate", spec)
            pod, node, kind = s.allocate()
            res[(pp, spec)] = list(zip(pod.tolist(), node.tolist(), kind.tolist()))
            st = s.stats()
            print("pp", pp, "spec", spec, {k: st[k] for k in ("spec_hits", "spec_missed", "pp_retries", "batched_pops")},
                  file=sys.stderr, flush=True)
ref = res[(0, 2)]
for k, v in res.items():
    d = next((i for i, (a, b) in enumerate(zip(v, ref)) if a != b), None)
    print(k, len(v), "first diff", d, v[d] if d is not None else None, ref[d] if d is not None else None)
    print(k, v[:24])
