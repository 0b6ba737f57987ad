"""Parity at sizes where the engine's worker blocks, mergers and several
placement lists run (VERDICT r05 "what's weak" 1 and "next" 7): 2-5k-node
random snapshots with the features the sweep evaluates (selectors, taints,
releasing, init containers, node affinity, unschedulable, BestEffort),
topology-keyless nodes (no zone label: a zone term never matches there,
predicates.go:1402-1458 — the case that hid placement 7's keyless-node bug in
round 4), and C3-shaped clusters with required pod affinity and preferred
inter-pod terms (interpod_affinity.go:119-240) beside the zone
anti-affinity.  The GPU logs, node state and gang close messages must equal
the hoisted restatement's; the restatement itself is checked against the
faithful one on small instances of the same generators (CPU tests below)."""
import numpy as np
import pytest

FEATURES = ("labels", "taints", "selector", "running", "releasing", "init", "nodeaffinity", "unsched",
            "bestEffort")


def _run(lib, path, **opts):
    with lib.Session(path) as s:
        for k, v in opts.items():
            s.set_option(k, v)
        pod, node, kind = s.allocate()
        st = s.stats()
        ns = s.read_nodes(st["nodes"])
        close = s.gang_unschedulable()
    return [(int(p), int(n), 4 if k == 1 else 8) for p, n, k in zip(pod, node, kind)], ns, st, close


# ---------------------------------------------------------------------------
# CPU: the generators' hardening options, faithful vs hoisted restatement
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("seed", range(6))
def test_keyless_random_restatements_agree(oracle_mod, kbgen_mod, tmp_path, seed):
    """gen_random with keyless nodes and pod affinity: kbref == kbfast."""
    c = kbgen_mod.gen_random(7100 + seed, n_nodes=10 + seed, n_jobs=6, max_tasks=6, keyless=0.4)
    p = str(tmp_path / "k.kbs")
    c.write(p)
    assert oracle_mod.fast_allocate(p, threads=2).as_list() == oracle_mod.ref_allocate(p).as_list()


@pytest.mark.parametrize("seed", range(3))
def test_c3_options_restatements_agree(oracle_mod, kbgen_mod, tmp_path, seed):
    """gen_c3 with keyless nodes, required pod affinity and preferred inter-pod
    terms, small: kbref == kbfast."""
    c = kbgen_mod.gen_c3(seed=7200 + seed, n_nodes=60, n_pending=160, keyless=0.2, pod_affinity=0.2, ipa=0.2)
    p = str(tmp_path / "c3.kbs")
    c.write(p)
    assert oracle_mod.fast_allocate(p, threads=2).as_list() == oracle_mod.ref_allocate(p).as_list()


def test_c3_default_stream_unchanged(kbgen_mod, tmp_path):
    """The options draw from a second generator: gen_c3() without them writes
    the same snapshot as with them set to 0."""
    a = str(tmp_path / "a.kbs")
    b = str(tmp_path / "b.kbs")
    kbgen_mod.gen_c3(seed=7300, n_nodes=50, n_pending=120).write(a)
    kbgen_mod.gen_c3(seed=7300, n_nodes=50, n_pending=120, keyless=0.0, pod_affinity=0.0, ipa=0.0).write(b)
    assert open(a, "rb").read() == open(b, "rb").read()


# ---------------------------------------------------------------------------
# GPU
# ---------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("lists", [0, 1])
@pytest.mark.parametrize("seed", range(4))
def test_engine_multiblock_features(engine, oracle_mod, kbgen_mod, tmp_path, seed, lists):
    """2-5k nodes, feature-rich classes, keyless nodes: many worker blocks and
    all mergers (sweep mode) or many class owners (list mode), against the
    hoisted restatement and the launched kernels."""
    c = kbgen_mod.gen_random(7400 + seed, n_nodes=2000 + 1000 * seed, n_jobs=60, max_tasks=48, features=FEATURES,
                             n_queues=1 + seed % 3, keyless=0.3)
    p = str(tmp_path / "mb.kbs")
    c.write(p)
    exp = oracle_mod.fast_allocate(p, threads=8).as_list()
    got, ns, st, close = _run(engine, p, engine_lists=lists)
    assert got == exp
    assert st["engine_pops"] > 0
    ref, ns0, st0, close0 = _run(engine, p, engine=0)
    assert ref == got and np.array_equal(ns0, ns) and close0 == close


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(4))
def test_pod_affinity_multiblock_keyless(engine, oracle_mod, kbgen_mod, tmp_path, seed):
    """Random pod (anti-)affinity on 2-3k nodes, 30 % of them without the zone
    label: the batched affinity pops (placement 7) and the per-task path
    against the restatement, and against each other (aff_batch = 0)."""
    c = kbgen_mod.gen_random(7500 + seed, n_nodes=2000 + 300 * seed, n_jobs=40, max_tasks=24,
                             features=FEATURES + ("podaffinity",), keyless=0.3)
    p = str(tmp_path / "pa.kbs")
    c.write(p)
    exp = oracle_mod.fast_allocate(p, threads=8).as_list()
    got, ns, st, close = _run(engine, p)
    assert got == exp
    got0, ns0, _, close0 = _run(engine, p, aff_batch=0)
    assert got0 == got and np.array_equal(ns0, ns) and close0 == close


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["keyless", "podaff", "ipa"])
def test_c3_hardened(engine, oracle_mod, kbgen_mod, tmp_path, variant):
    """C3's generator at 3k nodes x 6k pods with keyless nodes, required pod
    affinity, or preferred inter-pod terms beside its zone anti-affinity."""
    opts = {"keyless": dict(keyless=0.2), "podaff": dict(keyless=0.1, pod_affinity=0.15),
            "ipa": dict(keyless=0.1, ipa=0.15)}[variant]
    c = kbgen_mod.gen_c3(seed=7600, n_nodes=3000, n_pending=6000, **opts)
    p = str(tmp_path / "c3h.kbs")
    c.write(p)
    exp = oracle_mod.fast_allocate(p, threads=8).as_list()
    got, ns, st, close = _run(engine, p)
    assert got == exp
    assert len(got) > 1000
