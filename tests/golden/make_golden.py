"""Generate the golden fixtures in tests/golden/.

Two kinds of fixture:

* ``ka_*`` — known answers transcribed from the reference's own Go unit tests
  (inputs and expected outputs are data copied from the test tables, cited
  below).  These pin the oracle: tests/test_golden.py checks the faithful
  restatement (and the GPU engine, where the case is a placement) against them.
* ``c1_*`` / ``rnd_*`` — regression vectors: small snapshots and the placements
  the oracle produced for them when this script was run.  They are checked on
  CPU (oracle) and on GPU (engine) so a later change in either is caught.

Run:  python tests/golden/make_golden.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "kube-batch-1_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import kbgen  # noqa: E402
from kbgen import Cluster, res  # noqa: E402

G = 10 ** 9          # resource.MustParse("1G")
GI = kbgen.GI        # "1Gi"


def ka_allocate():
    """allocate_test.go:154-247 (TestAllocate), session tiers [drf, proportion]."""
    out = {}
    # case 1: "one Job with two Pods on one node" (:154-188)
    c = Cluster(tiers=kbgen.TEST_TIERS)
    c.add_node("n1", 2000, 4 * GI, 0, 0)                   # buildNode(n1, 2 CPU / 4Gi), no "pods"
    c.add_queue("c1", 1)
    c.add_job("c1", "pg1", "c1")
    for p in ("p1", "p2"):
        c.add_pod("c1", p, group="pg1", containers=[res(1000, G, 0)])
    c.write(os.path.join(HERE, "ka_allocate_1.kbs"))
    out["ka_allocate_1"] = {"expected_binds": {"c1/p1": "n1", "c1/p2": "n1"}}
    # case 2: "two Jobs on one node" (:189-247)
    c = Cluster(tiers=kbgen.TEST_TIERS)
    c.add_node("n1", 2000, 4 * G, 0, 0)
    c.add_queue("c1", 1)
    c.add_queue("c2", 1)
    c.add_job("c1", "pg1", "c1")
    c.add_job("c2", "pg2", "c2")
    for ns, g in (("c1", "pg1"), ("c2", "pg2")):
        for p in ("p1", "p2"):
            c.add_pod(ns, p, group=g, containers=[res(1000, G, 0)])
    c.write(os.path.join(HERE, "ka_allocate_2.kbs"))
    out["ka_allocate_2"] = {"expected_binds": {"c2/p1": "n1", "c1/p1": "n1"}}
    return out


def ka_node_info():
    """node_info_test.go:35-193: NodeInfo.AddTask arithmetic and GetAccessibleResource."""
    out = {}
    c = Cluster(tiers=kbgen.TEST_TIERS)
    c.add_node("n1", 8000, 10 * G, 0, 0)
    c.add_queue("default", 1)
    c.add_pod("c1", "p1", node="n1", phase="Running", containers=[res(1000, G)])
    c.add_pod("c1", "p2", node="n1", phase="Running", containers=[res(2000, 2 * G)])
    c.write(os.path.join(HERE, "ka_nodeinfo_add.kbs"))
    out["ka_nodeinfo_add"] = {"idle": [5000, 7 * G, 0], "used": [3000, 3 * G, 0], "releasing": [0, 0, 0],
                              "backfilled": [0, 0, 0]}
    c = Cluster(tiers=kbgen.TEST_TIERS)
    c.add_node("n1", 8000, 10 * G, 0, 0)
    c.add_queue("default", 1)
    c.add_pod("c1", "p1", node="n1", phase="Running", containers=[res(1000, G)])
    c.add_pod("c1", "p2", node="n1", phase="Running", backfill=True, containers=[res(2000, 2 * G)])
    c.write(os.path.join(HERE, "ka_nodeinfo_backfill.kbs"))
    out["ka_nodeinfo_backfill"] = {"idle": [5000, 7 * G, 0], "used": [3000, 3 * G, 0], "releasing": [0, 0, 0],
                                   "backfilled": [2000, 2 * G, 0], "accessible": [7000, 9 * G, 0]}
    return out


def ka_pod_info():
    """pod_info_test.go:26-162: GetPodResourceRequest / GetPodResourceWithoutInitContainers."""
    c = Cluster(tiers=kbgen.TEST_TIERS)
    c.add_node("n1", 8000, 10 * G, 0, 0)
    c.add_queue("default", 1)
    c.add_pod("c1", "a", containers=[res(1000, G), res(2000, G)])
    c.add_pod("c1", "b", containers=[res(1000, G), res(2000, G)],
              init_containers=[res(2000, 5 * G), res(2000, G)])
    c.write(os.path.join(HERE, "ka_podinfo.kbs"))
    # rows in pod order (c1-a, c1-b): Resreq, InitResreq
    return {"ka_podinfo": {"requests": [[3000, 2 * G, 0, 3000, 2 * G, 0], [3000, 2 * G, 0, 3000, 5 * G, 0]]}}


def ka_gang():
    """gang_test.go:14-43 with buildJob (:85-110): MinAvailable 2."""
    return {"ka_gang": {"cases": [
        {"min": 2, "statuses": ["Allocated", "Allocated"], "expected": "Ready"},
        {"min": 2, "statuses": ["Allocated", "AllocatedOverBackfill"], "expected": "AlmostReady"},
        {"min": 2, "statuses": [], "expected": "NotReady"},
    ]}}


def regression(oracle):
    out = {}
    cases = {"c1_default": kbgen.gen_c1(), "c1_testtiers": kbgen.gen_c1(tiers=kbgen.TEST_TIERS)}
    for seed in range(12):
        cases[f"rnd_{seed:02d}"] = kbgen.gen_random(
            5000 + seed, n_nodes=6 + seed % 5, n_jobs=5 + seed % 4, max_tasks=4,
            features=[f for f in ("labels", "taints", "ports", "init", "running", "releasing", "backfill",
                                  "selector", "nodeaffinity", "unsched", "bestEffort")])
    for seed in range(6):
        cases[f"rndaff_{seed:02d}"] = kbgen.gen_random(7000 + seed, n_nodes=7, n_jobs=6, max_tasks=4)
    for name, c in cases.items():
        path = os.path.join(HERE, f"{name}.kbs")
        c.write(path)
        pl = oracle.ref_allocate(path)
        out[name] = {"placements": pl.as_list(), "n_nodes": len(c.nodes)}
    return out


EVICT_ACTIONS = "reclaim, allocate, backfill, preempt"


def evict_regression(oracle):
    """Regression vectors of the reclaim / preempt actions (the shipped action list):
    preemption-shaped snapshots (kbgen.gen_preempt) and the records the faithful
    oracle produced (pod, node, status: 128 evicted, 8 pipelined, 4 allocated)."""
    out = {}
    for seed in range(8):
        c = kbgen.gen_preempt(9000 + seed, n_nodes=5 + seed % 4, n_queues=2 + seed % 3, n_run_jobs=6 + seed % 5,
                              n_pend_jobs=3 + seed % 3, max_tasks=4,
                              features=("selector", "taints", "ports", "init", "bestEffort") if seed % 2 else ())
        name = f"evict_{seed:02d}"
        path = os.path.join(HERE, f"{name}.kbs")
        c.write(path)
        pl = oracle.ref_allocate(path, actions=EVICT_ACTIONS)
        out[name] = {"records": pl.as_list(), "actions": EVICT_ACTIONS, "n_nodes": len(c.nodes)}
    return out


if __name__ == "__main__":
    import oracle
    oracle.build()
    golden = {}
    golden.update(ka_allocate())
    golden.update(ka_node_info())
    golden.update(ka_pod_info())
    golden.update(ka_gang())
    golden.update(regression(oracle))
    golden.update(evict_regression(oracle))
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(golden, f, indent=1, sort_keys=True)
    print("wrote", len(golden), "fixtures")
