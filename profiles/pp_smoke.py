"""Quick check of the persistent placer (option "pp") against the overlapped
pop kernel and the CPU restatement on a few snapshots (development aid)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "kube-batch-1_amd"), os.path.join(ROOT, "oracle")]
import kbgen  # noqa: E402
import kbhip  # noqa: E402
import oracle  # noqa: E402


def run(p, **opts):
    with kbhip.Session(p) as s:
        for k, v in opts.items():
            s.set_option(k, v)
        t = time.perf_counter()
        pod, node, kind = s.allocate()
        dt = time.perf_counter() - t
        st = s.stats()
    return (pod, node, kind), dt, st


def main():
    tmp = "/tmp/pp_smoke"
    os.makedirs(tmp, exist_ok=True)
    cases = []
    for seed in range(6):
        c = kbgen.gen_random(9100 + seed, n_nodes=8 + 13 * seed, n_jobs=6 + seed, max_tasks=3 + 2 * seed,
                             features=("labels", "taints", "ports", "init", "running", "releasing", "selector",
                                       "nodeaffinity", "unsched", "bestEffort"))
        cases.append(c.write(f"{tmp}/r{seed}.kbs"))
    p2 = f"{tmp}/c2.kbs"
    kbgen.gen_c2(p2)
    cases.append(p2)
    p4 = f"{tmp}/c4s.kbs"
    kbgen.gen_c4(p4, n_nodes=20000, n_pending=160000)
    cases.append(p4)
    for p in cases:
        a, ta, sa = run(p, pp=1)
        b, tb, sb = run(p, pp=0)
        same = all(np.array_equal(x, y) for x, y in zip(a, b))
        ok = None
        if os.path.getsize(p) < 2_000_000:
            exp = oracle.ref_allocate(p)
            ok = bool(np.array_equal(a[0], exp.pod) and np.array_equal(a[1], exp.node))
        print(f"{os.path.basename(p)}: placed {len(a[0])} same_as_ov={same} oracle={ok} pp {ta*1e3:.1f} ms "
              f"ov {tb*1e3:.1f} ms retries {sa['pp_retries']} pops {sa['batched_pops']}", flush=True)


if __name__ == "__main__":
    main()
