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
        oracle_mod.ref_allocate(p, actions="allocate, preempt")
