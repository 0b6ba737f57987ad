"""GPU parity of the batched path's running-min level placement (parallel
levels, kbhip_batch.h place_parallel): placement logs equal the CPU oracle's
and the per-task path's.  The selection argument is checked exhaustively on
CPU in test_placement_levels_model below (it runs without a GPU)."""
import os
import random

import pytest

from test_gpu_parity import NO_POD_AFFINITY, _oracle_log


def _log(engine, path, **opts):
    with engine.Session(path) as s:
        for k, v in opts.items():
            s.set_option(k, v)
        pod, node, kind = s.allocate()
        st = s.stats()
    return [(int(p), int(n), 4 if k == 1 else 8) for p, n, k in zip(pod, node, kind)], st


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(30))
def test_levels_random_gpu(engine, oracle_mod, kbgen_mod, tmp_path, seed):
    c = kbgen_mod.gen_random(4100 + seed, n_nodes=4 + seed % 12, n_jobs=4 + seed % 8, max_tasks=2 + seed % 9,
                             features=NO_POD_AFFINITY)
    p = str(tmp_path / "l.kbs")
    c.write(p)
    exp = _oracle_log(oracle_mod, p)
    for opts in (dict(), dict(overlap=0)):
        got, st = _log(engine, p, **opts)
        assert got == exp, opts


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(12))
def test_parallel_levels_deep_gpu(engine, oracle_mod, kbgen_mod, tmp_path, seed):
    """Few nodes, big gangs: chains deeper than one round of 8 depths, Pipelined
    commits (releasing capacity) mid-chain."""
    c = kbgen_mod.gen_random(4300 + seed, n_nodes=2 + seed % 3, n_jobs=3 + seed % 4, max_tasks=20 + 4 * seed,
                             features=NO_POD_AFFINITY)
    p = str(tmp_path / "d.kbs")
    c.write(p)
    exp = _oracle_log(oracle_mod, p)
    for opts in (dict(), dict(overlap=0), dict(batched=0)):
        got, _ = _log(engine, p, **opts)
        assert got == exp, opts


@pytest.mark.gpu
def test_levels_c2_gpu(engine, oracle_mod, kbgen_mod, tmp_path):
    p = str(tmp_path / "c2.kbs")
    kbgen_mod.gen_c2(p)
    exp = _oracle_log(oracle_mod, p, fast=True)
    for opts in (dict(), dict(overlap=0)):
        got, st = _log(engine, p, **opts)
        assert st["batched_pops"] > 0
        assert got == exp, opts


@pytest.mark.gpu
def test_levels_c4_scaled_gpu(engine, kbgen_mod, tmp_path):
    p = str(tmp_path / "c4s.kbs")
    kbgen_mod.gen_c4(p, n_nodes=20000, n_pending=120000)
    a, _ = _log(engine, p)
    b, _ = _log(engine, p, overlap=0)
    c, _ = _log(engine, p, batched=0)
    assert a == b == c


# ---- CPU: the selection argument (no GPU) ----------------------------------
def _greedy(seqs, idx, m):
    c = [0] * len(seqs)
    out = []
    for _ in range(m):
        best = None
        for j, s in enumerate(seqs):
            if c[j] < len(s) and s[c[j]] is not None:
                key = (s[c[j]][0], -idx[j])
                if best is None or key > best[0]:
                    best = (key, j, s[c[j]][1])
        if best is None:
            out.append(None)
            break
        out.append((best[1], best[2]))
        c[best[1]] += 1
    return out


def _levels(seqs, idx, m):
    ents = []
    for j, s in enumerate(seqs):
        rm = None
        for d, e in enumerate(s):
            if e is None:
                break
            rm = e[0] if rm is None else min(rm, e[0])
            ents.append(((rm, -idx[j], -d), j, e[1]))
    ents.sort(reverse=True)
    out = [(j, k) for _, j, k in ents[:m]]
    return out + [None] if len(out) < m else out


def test_placement_levels_model():
    """Sorting (running-min score, -index, -depth) entries reproduces the
    sequential greedy, including scores that rise after a commit, ties and
    nodes that become infeasible."""
    rng = random.Random(7)
    for _ in range(20000):
        n, m = rng.randint(1, 6), rng.randint(1, 8)
        idx = rng.sample(range(50), n)
        seqs = []
        for _j in range(n):
            s = [None if rng.random() < 0.1 else (rng.randint(0, 5), rng.randint(1, 2))
                 for _d in range(rng.randint(1, m + 1))]
            if None in s:
                s = s[:s.index(None) + 1]
            elif len(s) <= m:
                s.append(None)
            seqs.append(s)
        g = _greedy(seqs, idx, m)
        assert g == _levels(seqs, idx, m)[:len(g)]


# ---- speculation: the predicted next pop queued behind the running one -----
def _log_spec(engine, path, speculate):
    with engine.Session(path) as s:
        s.set_option("speculate", speculate)
        pod, node, kind = s.allocate()
        st = s.stats()
    return [(int(p), int(n), int(k)) for p, n, k in zip(pod, node, kind)], st


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(16))
def test_speculation_random_gpu(engine, oracle_mod, kbgen_mod, tmp_path, seed):
    """Placements with speculation equal the oracle's; mispredictions (failed
    pops, pipelined tasks, non-batchable pops next) are retracted exactly."""
    tiers = [None, [["drf", "proportion"]], [["gang"], ["predicates", "nodeorder"]],
             [["priority", "gang", "drf"], ["predicates", "proportion", "nodeorder"]]][seed % 4]
    c = kbgen_mod.gen_random(4500 + seed, n_nodes=3 + seed % 10, n_jobs=6 + seed % 9, max_tasks=2 + seed % 9,
                             features=NO_POD_AFFINITY, tiers=tiers)
    p = str(tmp_path / "s.kbs")
    c.write(p)
    got, st = _log_spec(engine, p, 1)
    exp = _oracle_log(oracle_mod, p)
    assert [(a, b, 4 if k == 1 else 8) for a, b, k in got] == exp


@pytest.mark.gpu
def test_speculation_c2_gpu(engine, oracle_mod, kbgen_mod, tmp_path):
    p = str(tmp_path / "c2.kbs")
    kbgen_mod.gen_c2(p)
    a, sa = _log_spec(engine, p, 1)
    b, sb = _log_spec(engine, p, 0)
    assert a == b
    assert [(x, y, 4 if k == 1 else 8) for x, y, k in a] == _oracle_log(oracle_mod, p, fast=True)
    assert sa["spec_hits"] > 0 and sb["spec_hits"] == 0 and sb["spec_missed"] == 0


@pytest.mark.gpu
def test_speculation_c4_scaled_gpu(engine, kbgen_mod, tmp_path):
    p = str(tmp_path / "c4s.kbs")
    kbgen_mod.gen_c4(p, n_nodes=20000, n_pending=120000)
    a, sa = _log_spec(engine, p, 1)
    b, _ = _log_spec(engine, p, 0)
    assert a == b
    assert sa["spec_hits"] > sa["spec_missed"]


# ---- 32-bit selection keys in the batched sweep ------------------------------
def _log_opt(engine, path, **opts):
    with engine.Session(path) as s:
        for k, v in opts.items():
            s.set_option(k, v)
        pod, node, kind = s.allocate()
    return [(int(p), int(n), 4 if k == 1 else 8) for p, n, k in zip(pod, node, kind)]


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(12))
def test_keys32_random_gpu(engine, oracle_mod, kbgen_mod, tmp_path, seed):
    """Small and huge nodeorder weights: 32-bit keys where the score range fits,
    the 64-bit fallback where it does not; both equal the oracle."""
    c = kbgen_mod.gen_random(4700 + seed, n_nodes=4 + seed % 12, n_jobs=5 + seed % 8, max_tasks=2 + seed % 9,
                             features=NO_POD_AFFINITY)
    if seed % 3 == 1:
        c.args = {"nodeorder": {"leastrequested.weight": "100000000", "balancedresource.weight": "-3"}}
    elif seed % 3 == 2:
        c.args = {"nodeorder": {"nodeaffinity.weight": "-7", "balancedresource.weight": "5"}}
    p = str(tmp_path / "k.kbs")
    c.write(p)
    exp = _oracle_log(oracle_mod, p)
    assert _log_opt(engine, p, keys32=1) == exp
    assert _log_opt(engine, p, keys32=0) == exp


@pytest.mark.gpu
def test_keys32_c4_scaled_gpu(engine, kbgen_mod, tmp_path):
    p = str(tmp_path / "c4k.kbs")
    kbgen_mod.gen_c4(p, n_nodes=20000, n_pending=120000)
    assert _log_opt(engine, p, keys32=1) == _log_opt(engine, p, keys32=0)


# ---- overlapped pops (two / three streams, device-chained) x speculation depth -------
@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(16))
def test_overlap_speculation_random_gpu(engine, oracle_mod, kbgen_mod, tmp_path, seed):
    """Overlap on / off with speculation depths 0..3 place exactly as the
    oracle, including mispredicted pops retracted several deep."""
    tiers = [None, [["drf", "proportion"]], [["gang"], ["predicates", "nodeorder"]],
             [["priority", "gang", "drf"], ["predicates", "proportion", "nodeorder"]]][seed % 4]
    c = kbgen_mod.gen_random(4900 + seed, n_nodes=3 + seed % 10, n_jobs=6 + seed % 9, max_tasks=2 + seed % 9,
                             features=NO_POD_AFFINITY, tiers=tiers)
    p = str(tmp_path / "o.kbs")
    c.write(p)
    exp = _oracle_log(oracle_mod, p)
    for overlap, spec in ((0, 0), (0, 2), (1, 0), (1, 1), (1, 2), (1, 3), (0, 3), (2, 0), (2, 2), (2, 3)):
        assert _log_opt(engine, p, overlap=overlap, speculate=spec) == exp, (overlap, spec)


@pytest.mark.gpu
def test_overlap_c2_gpu(engine, oracle_mod, kbgen_mod, tmp_path):
    p = str(tmp_path / "c2o.kbs")
    kbgen_mod.gen_c2(p)
    exp = _oracle_log(oracle_mod, p, fast=True)
    for overlap, spec in ((1, 3), (1, 2), (0, 2), (2, 2), (2, 3)):
        assert _log_opt(engine, p, overlap=overlap, speculate=spec) == exp, (overlap, spec)


@pytest.mark.gpu
def test_overlap_c4_scaled_gpu(engine, kbgen_mod, tmp_path):
    """Overlapped (two and three streams), speculative pops on a C4-shaped
    session equal one pop at a time on one stream; the node state after the
    session too."""
    p = str(tmp_path / "c4o.kbs")
    kbgen_mod.gen_c4(p, n_nodes=20000, n_pending=120000)
    logs, nodes = [], []
    for overlap, spec in ((1, 3), (1, 2), (2, 2), (2, 3), (0, 0)):
        with engine.Session(p) as s:
            s.set_option("overlap", overlap)
            s.set_option("speculate", spec)
            pod, node, kind = s.allocate()
            st = s.stats()
            nodes.append(s.read_nodes(20000))
        logs.append([(int(a), int(b), int(k)) for a, b, k in zip(pod, node, kind)])
        if spec:
            assert st["spec_hits"] > st["spec_missed"]
        assert st["alloc_device_s"] > 0
    assert all(lg == logs[-1] for lg in logs)
    assert all((nd == nodes[-1]).all() for nd in nodes)
