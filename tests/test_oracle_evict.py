"""Known answers for the faithful restatement's reclaim and preempt actions
(oracle/kbref.cpp: reclaimExecute, preemptExecute, Statement), hand-derived
from actions/reclaim/reclaim.go:41-196, actions/preempt/preempt.go:43-353 and
framework/statement.go.  Log entries: (pod, node, status) with status 128 =
evicted (Releasing), 8 = Pipelined, 4 = Allocated."""
import pytest

GI = 1 << 30
EVICT, PIPE, ALLOC = 128, 8, 4


def _cluster(kbgen, pend_queue, pend_min, *, victim_min=1, victim_ns="ns1", victim_class=""):
    c = kbgen.Cluster()
    c.add_node("n0", 4000, 8 * GI, 0, 110)
    c.add_queue("q0", 1)
    c.add_queue("q1", 1)
    c.add_job(victim_ns, "r0", "q0", min_member=victim_min)
    c.add_pod(victim_ns, "r0-0", uid="a0", group="r0", node="n0", phase="Running",
              priority_class=victim_class, containers=[kbgen.res(cpu=4000, mem=GI)])
    c.add_job("ns2", "p0", pend_queue, min_member=pend_min)
    c.add_pod("ns2", "p0-0", uid="b0", group="p0", priority=10, containers=[kbgen.res(cpu=2000, mem=GI)])
    return c


def test_reclaim_other_queue(oracle_mod, kbgen_mod, tmp_path):
    """q1's pending task reclaims q0's running pod (gang: MinAvailable == 1 makes it
    a victim; proportion is in tier 2 and never consulted), then pipelines there."""
    p = _cluster(kbgen_mod, "q1", 1).write(str(tmp_path / "r.kbs"))
    assert oracle_mod.ref_allocate(p, actions="reclaim").as_list() == [(0, 0, EVICT), (1, 0, PIPE)]


@pytest.mark.parametrize("kw", [dict(victim_min=2), dict(victim_ns="kube-system"),
                                dict(victim_class="system-node-critical")])
def test_reclaim_protected_victims(oracle_mod, kbgen_mod, tmp_path, kw):
    """gang (MinAvailable 2 > ready-1) or conformance (kube-system, critical class)
    empties tier 1's intersection; the next tier starts from that nil set."""
    p = _cluster(kbgen_mod, "q1", 1, **kw).write(str(tmp_path / "r.kbs"))
    assert oracle_mod.ref_allocate(p, actions="reclaim").as_list() == []


def test_reclaim_same_queue_no_victims(oracle_mod, kbgen_mod, tmp_path):
    p = _cluster(kbgen_mod, "q0", 1).write(str(tmp_path / "r.kbs"))
    assert oracle_mod.ref_allocate(p, actions="reclaim").as_list() == []


def test_preempt_commit_when_ready(oracle_mod, kbgen_mod, tmp_path):
    """Same queue, MinAvailable 0: the job is Ready after the pipeline, the statement
    commits (evict, then pipeline, in operation order)."""
    p = _cluster(kbgen_mod, "q0", 0).write(str(tmp_path / "p.kbs"))
    pl, ns = oracle_mod.ref_allocate(p, actions="preempt", with_nodes=True)
    assert pl.as_list() == [(0, 0, EVICT), (1, 0, PIPE)]
    # n0: Releasing 4000 (evicted) - 2000 (pipelined); Used 6000; Idle 0
    assert list(ns[0, 0:3]) == [0, 7 * GI, 0]
    assert list(ns[0, 3:6]) == [6000, 2 * GI, 0]
    assert list(ns[0, 6:9]) == [2000, 0, 0]


def test_preempt_discard_keeps_node_releasing(oracle_mod, kbgen_mod, tmp_path):
    """MinAvailable 1: a Pipelined task does not make the job Ready, so the statement
    is discarded: nothing is logged, the victim is Running again in its job, but
    unevict's node.AddTask fails (the node still holds the task) so the node keeps
    it as Releasing (statement.go:81-105)."""
    p = _cluster(kbgen_mod, "q0", 1).write(str(tmp_path / "p.kbs"))
    pl, ns = oracle_mod.ref_allocate(p, actions="preempt", with_nodes=True)
    assert pl.as_list() == []
    assert list(ns[0, 0:3]) == [0, 7 * GI, 0]        # Idle
    assert list(ns[0, 3:6]) == [4000, GI, 0]         # Used
    assert list(ns[0, 6:9]) == [4000, GI, 0]         # Releasing


def test_preempt_random_smoke(oracle_mod, kbgen_mod, tmp_path):
    """The full default action list runs on random preemption-shaped snapshots and
    produces every record kind."""
    kinds = set()
    for seed in range(30):
        c = kbgen_mod.gen_preempt(seed, n_run_jobs=10, features=("selector", "taints", "ports", "init",
                                                                   "bestEffort", "unsched"))
        p = c.write(str(tmp_path / f"s{seed}.kbs"))
        kinds |= {k for _, _, k in oracle_mod.ref_allocate(p, actions="reclaim, allocate, backfill, preempt").as_list()}
    assert kinds == {EVICT, PIPE, ALLOC}


TIERS = [
    None,
    [["priority", "gang", "drf", "predicates", "proportion", "nodeorder"]],
    [["drf", "predicates", "nodeorder"], ["gang", "proportion"]],
    [["priority", "conformance"], ["drf", "proportion", "predicates", "nodeorder"]],
]
ACTIONS = ["reclaim", "preempt", "reclaim, allocate, backfill, preempt", "allocate, preempt"]


@pytest.mark.parametrize("seed", range(60))
def test_evict_faithful_vs_hoisted(oracle_mod, kbgen_mod, tmp_path, seed):
    """The two independent restatements (kbref: per-pair recomputation; kbfast:
    hoisted, threaded) agree on every reclaim / preempt record."""
    c = kbgen_mod.gen_preempt(700 + seed, n_nodes=4 + seed % 10, n_queues=1 + seed % 4, n_run_jobs=4 + seed % 9,
                              n_pend_jobs=2 + seed % 5, max_tasks=1 + seed % 6, tiers=TIERS[seed % len(TIERS)],
                              features=("selector", "taints", "ports", "init", "bestEffort", "unsched")
                              if seed % 2 else ())
    p = c.write(str(tmp_path / "s.kbs"))
    acts = ACTIONS[seed % len(ACTIONS)]
    a = oracle_mod.ref_allocate(p, actions=acts).as_list()
    b = oracle_mod.fast_allocate(p, threads=3, actions=acts).as_list()
    assert a == b


def test_evict_c5_scaled_faithful_vs_hoisted(oracle_mod, kbgen_mod, tmp_path):
    p = str(tmp_path / "c5.kbs")
    kbgen_mod.gen_c5(p, n_nodes=60, n_pending=60, best_effort=6)
    acts = "reclaim, allocate, backfill, preempt"
    a = oracle_mod.ref_allocate(p, actions=acts).as_list()
    b = oracle_mod.fast_allocate(p, threads=4, actions=acts).as_list()
    assert a == b and any(k == EVICT for _, _, k in a)
