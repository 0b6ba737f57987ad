"""GPU parity of the reclaim and preempt actions:
the engine's records — evictions that reach the cache and pipelined
preemptors, in decision order — and the device node state afterwards equal
the faithful restatement's (oracle/kbref.cpp reclaimExecute / preemptExecute)
on the same snapshot.  Records are compared as (pod, node, status) with the
oracle's TaskStatus codes: 4 Allocated, 8 Pipelined, 128 Releasing (evicted)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

STATUS = {1: 4, 2: 8, 3: 128}
FEATURES = ("selector", "taints", "ports", "init", "bestEffort", "unsched")
TIERS = [
    None,                                                          # shipped kube-batch-conf.yaml
    [["priority", "gang", "drf", "predicates", "proportion", "nodeorder"]],  # one tier: drf / proportion intersect
    [["drf", "predicates", "nodeorder"], ["gang", "proportion"]],
    [["priority", "conformance"], ["drf", "proportion", "predicates", "nodeorder"]],
]
ACTIONS = ["reclaim", "preempt", "reclaim, allocate, backfill, preempt", "allocate, preempt"]


def _engine(engine, path, actions):
    with engine.Session(path) as s:
        pod, node, kind = s.run_actions(actions)
        n_nodes = s.stats()["nodes"]
        ns = s.read_nodes(n_nodes)
    return [(int(p), int(n), STATUS[int(k)]) for p, n, k in zip(pod, node, kind)], ns


def _check(engine, oracle_mod, path, actions):
    exp, ons = oracle_mod.ref_allocate(path, actions=actions, with_nodes=True)
    got, ns = _engine(engine, path, actions)
    assert got == exp.as_list()
    assert np.array_equal(ns.astype(np.float64), ons[:ns.shape[0]])
    return got


def _hand(kbgen, pend_queue, pend_min):
    GI = 1 << 30
    c = kbgen.Cluster()
    c.add_node("n0", 4000, 8 * GI, 0, 110)
    c.add_queue("q0", 1)
    c.add_queue("q1", 1)
    c.add_job("ns1", "r0", "q0", min_member=1)
    c.add_pod("ns1", "r0-0", uid="a0", group="r0", node="n0", phase="Running", containers=[kbgen.res(cpu=4000, mem=GI)])
    c.add_job("ns2", "p0", pend_queue, min_member=pend_min)
    c.add_pod("ns2", "p0-0", uid="b0", group="p0", priority=10, containers=[kbgen.res(cpu=2000, mem=GI)])
    return c


@pytest.mark.parametrize("case", [("q1", 1, "reclaim", [(0, 0, 128), (1, 0, 8)]),
                                  ("q0", 0, "preempt", [(0, 0, 128), (1, 0, 8)]),
                                  ("q0", 1, "preempt", [])])
def test_known_answers(engine, oracle_mod, kbgen_mod, tmp_path, case):
    q, mn, actions, exp = case
    p = _hand(kbgen_mod, q, mn).write(str(tmp_path / "h.kbs"))
    assert _check(engine, oracle_mod, p, actions) == exp


@pytest.mark.parametrize("seed", range(48))
def test_random_preempt_snapshots(engine, oracle_mod, kbgen_mod, tmp_path, seed):
    c = kbgen_mod.gen_preempt(500 + seed, n_nodes=4 + seed % 10, n_queues=1 + seed % 4, n_run_jobs=4 + seed % 9,
                              n_pend_jobs=2 + seed % 5, max_tasks=1 + seed % 6, tiers=TIERS[seed % len(TIERS)],
                              features=FEATURES if seed % 2 else ())
    p = c.write(str(tmp_path / "s.kbs"))
    _check(engine, oracle_mod, p, ACTIONS[seed % len(ACTIONS)])


@pytest.mark.parametrize("seed", range(40))
def test_random_preempt_pod_affinity(engine, oracle_mod, kbgen_mod, tmp_path, seed):
    """Pod (anti-)affinity and inter-pod priority terms on running and pending
    pods: evicting a predicate target withdraws it from the count tables, an
    unevict restores it, a pipelined preemptor counts for the inter-pod
    priority at the fallback node (predicates.go:59-94, nodeorder.go:78-93)."""
    c = kbgen_mod.gen_preempt(1500 + seed, n_nodes=4 + seed % 10, n_queues=1 + seed % 4, n_run_jobs=4 + seed % 9,
                              n_pend_jobs=2 + seed % 5, max_tasks=1 + seed % 6, tiers=TIERS[seed % len(TIERS)],
                              features=("podaffinity",) + (FEATURES if seed % 2 else ()))
    if seed % 3 == 0:
        c.args = {"nodeorder": {"podaffinity.weight": str(1 + seed % 4)}}
    p = c.write(str(tmp_path / "a.kbs"))
    _check(engine, oracle_mod, p, ACTIONS[seed % len(ACTIONS)])


@pytest.mark.parametrize("first", [1, 3])
def test_chunked_readback(engine, oracle_mod, kbgen_mod, tmp_path, first):
    """Passing-node lists longer than the keys read back with the count (option
    rank_first, 2048 by default) are fetched in a second copy."""
    exp_all = []
    for seed in range(6):
        c = kbgen_mod.gen_preempt(900 + seed, n_nodes=24, n_queues=3, n_run_jobs=14, n_pend_jobs=5, max_tasks=5)
        p = c.write(str(tmp_path / f"c{seed}.kbs"))
        actions = "reclaim, allocate, backfill, preempt"
        exp, ons = oracle_mod.ref_allocate(p, actions=actions, with_nodes=True)
        with engine.Session(p) as s:
            s.set_option("rank_first", first)
            pod, node, kind = s.run_actions(actions)
            ns = s.read_nodes(24)
        assert [(int(a), int(b), STATUS[int(k)]) for a, b, k in zip(pod, node, kind)] == exp.as_list()
        assert np.array_equal(ns.astype(np.float64), ons[:24])
        exp_all += exp.as_list()
    assert any(k == 128 for _, _, k in exp_all)


def test_pod_affinity_hand(engine, oracle_mod, kbgen_mod, tmp_path):
    """A pending pod with required anti-affinity against the running pod's
    labels (by hostname) beside a plain reclaimer: records equal the faithful
    restatement's (the pod-affinity lister lists AllocatedStatuses tasks only,
    predicates.go:59-94)."""
    c = _hand(kbgen_mod, "q1", 1)
    term = {"selector": {"ml": {"job": "r0"}, "me": []}, "topology_key": "kubernetes.io/hostname"}
    c.add_job("ns2", "p1", "q1", min_member=1)
    c.add_pod("ns2", "p1-0", uid="b1", group="p1", priority=10, containers=[kbgen_mod.res(cpu=100, mem=1 << 20)],
              affinity={"anti": {"required": [term]}})
    p = c.write(str(tmp_path / "a.kbs"))
    got = _check(engine, oracle_mod, p, "reclaim")
    assert (0, 0, 128) in got


# ---- C5: the what-if session shape -----------------------------
C5_ACTIONS = "reclaim, allocate, backfill, preempt"


@pytest.mark.parametrize("seed", range(3))
def test_c5_scaled_parity(engine, oracle_mod, kbgen_mod, tmp_path, seed):
    """C5's generator at a size the faithful restatement finishes in seconds."""
    p = str(tmp_path / "c5s.kbs")
    kbgen_mod.gen_c5(p, seed=kbgen_mod.BASE_SEED + 5 + seed, n_nodes=90, n_pending=80, best_effort=8)
    got = _check(engine, oracle_mod, p, C5_ACTIONS)
    assert any(k == 128 for _, _, k in got)


def test_c5_full_size_parity(engine, oracle_mod, kbgen_mod, tmp_path):
    """C5 at full size (50k nodes x 1.45M running pods, 2k pending) against the hoisted
    restatement (oracle/kbfast.cpp), record for record (~728k records)."""
    p = str(tmp_path / "c5.kbs")
    kbgen_mod.gen_c5(p)
    exp = oracle_mod.fast_allocate(p, threads=16, actions=C5_ACTIONS)
    with engine.Session(p) as s:
        pod, node, kind = s.run_actions(C5_ACTIONS)
    assert np.array_equal(pod, exp.pod) and np.array_equal(node, exp.node)
    assert np.array_equal(np.array([0, 4, 8, 128])[kind], exp.status)
    assert (kind == 3).sum() > 100_000


def test_c5_full_size_invariants(engine, kbgen_mod, tmp_path):
    """50k nodes x 1.45M running pods, 2k pending: properties that hold at any size —
    evicted pods were Running on the recorded node and are evicted once; pipelined /
    allocated pods were Pending (or BestEffort-backfilled); a second session on the
    same snapshot reproduces the records exactly."""
    p = str(tmp_path / "c5.kbs")
    meta = kbgen_mod.gen_c5(p)
    runs = []
    for _ in range(2):
        with engine.Session(p) as s:
            pod, node, kind = s.run_actions(C5_ACTIONS)
        runs.append((pod, node, kind))
    pod, node, kind = runs[0]
    assert all(np.array_equal(a, b) for a, b in zip(runs[0], runs[1]))
    n_run = meta["running"]
    ev = kind == 3
    assert ev.any() and (kind == 2).any() and (kind == 1).any()
    assert (pod[ev] < n_run).all()                       # running pods sort first (kbgen._bulk)
    assert np.unique(pod[ev]).size == int(ev.sum())       # never evicted twice
    assert (pod[~ev] >= n_run).all()                      # only pending pods are placed
    # the recorded node of an eviction is the victim's node (running pods are laid out node by node)
    run_node = np.repeat(np.arange(meta["nodes"]), meta["rpn"])
    assert (run_node[pod[ev]] == node[ev]).all()


def _evict_golden():
    import json
    import os
    gold = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    with open(os.path.join(gold, "golden.json")) as f:
        g = json.load(f)
    return [(os.path.join(gold, k + ".kbs"), g[k]) for k in sorted(g) if k.startswith("evict_")]


@pytest.mark.parametrize("case", _evict_golden(), ids=lambda c: os.path.basename(c[0]) if isinstance(c, tuple) else "")
def test_evict_golden_vectors_gpu(engine, case):
    path, g = case
    got, _ = _engine(engine, path, g["actions"])
    assert got == [tuple(x) for x in g["records"]]


@pytest.mark.parametrize("radix", [0, 1])
@pytest.mark.parametrize("seed", range(4))
def test_rank_sort_paths(engine, oracle_mod, kbgen_mod, tmp_path, radix, seed):
    """The walk order of reclaim / preempt: the hand-written counting sort over a
    class's score range (default) and the wide-range radix passes (option rank_radix,
    kept for score ranges beyond 256 values) both give the oracle's records, on
    node counts that span many sort blocks and waves."""
    c = kbgen_mod.gen_preempt(700 + seed, n_nodes=300 + 170 * seed, n_queues=2 + seed % 3, n_run_jobs=40,
                              n_pend_jobs=6, max_tasks=6, tiers=TIERS[seed % len(TIERS)],
                              features=FEATURES if seed % 2 else ())
    p = c.write(str(tmp_path / "r.kbs"))
    actions = ACTIONS[seed % len(ACTIONS)]
    exp, ons = oracle_mod.ref_allocate(p, actions=actions, with_nodes=True)
    with engine.Session(p) as s:
        s.set_option("rank_radix", radix)
        pod, node, kind = s.run_actions(actions)
        ns = s.read_nodes(s.stats()["nodes"])
    assert [(int(a), int(b), STATUS[int(k)]) for a, b, k in zip(pod, node, kind)] == exp.as_list()
    assert np.array_equal(ns.astype(np.float64), ons[:ns.shape[0]])


@pytest.mark.parametrize("seed", range(4))
def test_rank_wide_score_range(engine, oracle_mod, kbgen_mod, tmp_path, seed):
    """Large nodeorder weights (plain Atoi arguments, nodeorder.go:209-246):
    a class's score range exceeds the counting sort's 256 values, so preempt's
    walk order comes from the radix passes without any option; records and
    node state equal the oracle's."""
    c = kbgen_mod.gen_preempt(760 + seed, n_nodes=200 + 90 * seed, n_queues=2, n_run_jobs=30, n_pend_jobs=5,
                              max_tasks=5, tiers=TIERS[seed % len(TIERS)])
    c.args = {"nodeorder": {"leastrequested.weight": str([1000, 70000, 3, 123456][seed]),
                            "balancedresource.weight": str([-7, 500, 1000000, 2][seed])}}
    p = c.write(str(tmp_path / "w.kbs"))
    exp, ons = oracle_mod.ref_allocate(p, actions="preempt, reclaim", with_nodes=True)
    with engine.Session(p) as s:
        pod, node, kind = s.run_actions("preempt, reclaim")
        ns = s.read_nodes(s.stats()["nodes"])
    assert [(int(a), int(b), STATUS[int(k)]) for a, b, k in zip(pod, node, kind)] == exp.as_list()
    assert np.array_equal(ns.astype(np.float64), ons[:ns.shape[0]])

