"""The faithful restatement (kbref) and the hoisted CPU baseline (kbfast)
must place identically on random snapshots that exercise every predicate and
priority of the path, and under alternative tier configurations."""
import os

import pytest

TIERS = [
    None,                                                        # shipped kube-batch-conf.yaml
    [["drf", "proportion"]],                                     # allocate_test.go session
    [["gang"], ["predicates", "nodeorder"]],
    [["priority", "gang", "drf"], ["predicates", "proportion", "nodeorder", "nodeorder"]],
]


@pytest.mark.parametrize("seed", range(60))
def test_faithful_vs_hoisted(oracle_mod, kbgen_mod, tmp_path, seed):
    c = kbgen_mod.gen_random(seed, n_nodes=3 + seed % 10, n_jobs=3 + seed % 7, max_tasks=1 + seed % 6,
                             tiers=TIERS[seed % len(TIERS)])
    if seed % 3 == 0:
        c.args = {"nodeorder": {"leastrequested.weight": "2", "podaffinity.weight": "3",
                                "nodeaffinity.weight": "-1"}}
    if seed % 11 == 0:
        c.flags = {"gang": ["disableJobReady"], "predicates": ["disablePredicate"]}
    p = str(tmp_path / "s.kbs")
    c.write(p)
    a = oracle_mod.ref_allocate(p).as_list()
    b = oracle_mod.fast_allocate(p, threads=3).as_list()
    assert a == b


def test_c3_shape_small(oracle_mod, kbgen_mod, tmp_path):
    """C3 features (labels, taints, selectors, zone anti-affinity, 8 queues) at small size."""
    c = kbgen_mod.gen_c3(n_nodes=60, n_pending=300)
    p = str(tmp_path / "c3.kbs")
    c.write(p)
    a = oracle_mod.ref_allocate(p).as_list()
    b = oracle_mod.fast_allocate(p, threads=4).as_list()
    assert a == b and len(a) > 100


def test_c2_shape_small(oracle_mod, kbgen_mod, tmp_path):
    p = str(tmp_path / "c2.kbs")
    kbgen_mod.gen_c2(p, n_nodes=40, n_pending=400)
    a = oracle_mod.ref_allocate(p).as_list()
    b = oracle_mod.fast_allocate(p, threads=4).as_list()
    assert a == b and len(a) > 100


@pytest.mark.parametrize("seed", range(40))
def test_backfill_faithful_vs_hoisted(oracle_mod, kbgen_mod, tmp_path, seed):
    """allocate then backfill (actions/backfill/backfill.go:40-70): BestEffort
    tasks go to the first node passing the predicates."""
    c = kbgen_mod.gen_random(500 + seed, n_nodes=3 + seed % 10, n_jobs=3 + seed % 7, max_tasks=1 + seed % 6,
                             tiers=TIERS[seed % len(TIERS)], best_effort_p=0.35)
    p = str(tmp_path / "b.kbs")
    c.write(p)
    acts = "allocate, backfill"
    a = oracle_mod.ref_allocate(p, actions=acts).as_list()
    b = oracle_mod.fast_allocate(p, threads=3, actions=acts).as_list()
    assert a == b
    alloc_only = oracle_mod.ref_allocate(p).as_list()
    assert a[:len(alloc_only)] == alloc_only


def test_backfill_places_best_effort(oracle_mod, kbgen_mod, tmp_path):
    n_bf = 0
    for seed in range(30):
        c = kbgen_mod.gen_random(700 + seed, n_nodes=6, n_jobs=6, max_tasks=5, best_effort_p=0.4)
        p = str(tmp_path / f"b{seed}.kbs")
        c.write(p)
        n_bf += len(oracle_mod.ref_allocate(p, actions="allocate, backfill")) - len(oracle_mod.ref_allocate(p))
    assert n_bf > 20


def test_unknown_action_rejected(oracle_mod, kbgen_mod, tmp_path):
    p = str(tmp_path / "u.kbs")
    kbgen_mod.gen_c1().write(p)
    with pytest.raises(RuntimeError):
        oracle_mod.ref_allocate(p, actions="allocate, enqueue")


# ---- gang OnSessionClose messages, hand-derived ---------
def test_gang_close_fit_error_known_answer(tmp_path):
    """Two nodes of 2 CPU / 4 GiB, a gang of 5 pods x (1 CPU, 1 GiB) with
    minMember 5: four pods fit, the fifth finds no node.  Its walk visits both
    nodes: Idle cpu 0 - (1000 + 10) < 0 on each, memory 2 GiB - (1 GiB + 10 MiB)
    >= 0, so FitError = '0/2 nodes are available, 2 insufficient cpu.'; 5 - 4
    = 1 task short of 5 (allocate.go:164-167, job_info.go:343-372,
    gang.go:166-187).  Then a gang whose only node fails the predicates:
    NodesFitDelta stays empty, '0 nodes are available'."""
    import kbgen
    import oracle
    c = kbgen.Cluster()
    c.add_queue("default", 1)
    for i in range(2):
        c.add_node(f"n{i}", 2000, 4 * kbgen.GI, 0)
    c.add_job("ns", "g", "default", min_member=5)
    for k in range(5):
        c.add_pod("ns", f"g-{k}", uid=f"u{k}", group="g", containers=[kbgen.res(1000, kbgen.GI)])
    p = str(tmp_path / "ka.kbs")
    c.write(p)
    assert oracle.ref_gang_close(p) == {"ns/g": "1/5 tasks in gang unschedulable: 0/2 nodes are available, "
                                                "2 insufficient cpu."}
    c2 = kbgen.Cluster()
    c2.add_queue("default", 1)
    c2.add_node("n0", 2000, 4 * kbgen.GI, 0, unschedulable=True)
    c2.add_job("ns", "g", "default", min_member=1)
    c2.add_pod("ns", "g-0", uid="u0", group="g", containers=[kbgen.res(1000, kbgen.GI)])
    p2 = str(tmp_path / "ka2.kbs")
    c2.write(p2)
    assert oracle.ref_gang_close(p2) == {"ns/g": "1/1 tasks in gang unschedulable: 0 nodes are available"}


def _backfill_gang_cluster():
    """A gang of 3 pods (minMember 3) on one 2-CPU node: two fit, the third
    does not, so the job stays not Ready.  One of its pods carries the backfill
    annotation (TaskInfo.IsBackfill)."""
    import kbgen
    c = kbgen.Cluster()
    c.add_queue("default", 1)
    c.add_node("n0", 2000, 4 * kbgen.GI, 0)
    c.add_job("ns", "g", "default", min_member=3)
    for k in range(3):
        c.add_pod("ns", f"g-{k}", uid=f"u{k}", group="g", containers=[kbgen.res(1000, kbgen.GI)], backfill=k == 2)
    c.add_job("ns", "h", "default", min_member=2)
    for k in range(2):
        c.add_pod("ns", f"h-{k}", uid=f"v{k}", group="h", containers=[kbgen.res(4000, kbgen.GI)])
    return c


def test_gang_close_backfilled_known_answer(tmp_path):
    """gang.go:189-199: a not-Ready job with an IsBackfill task gets the
    PodGroupBackfilled condition (no message) instead of Unschedulable; the
    other not-Ready job keeps its FitError message."""
    import oracle
    p = str(tmp_path / "bf.kbs")
    _backfill_gang_cluster().write(p)
    got = oracle.ref_gang_close(p)
    assert got["ns/g"] == "Backfilled"
    assert got["ns/h"].startswith("2/2 tasks in gang unschedulable: 0/1 nodes are available")
