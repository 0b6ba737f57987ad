"""The persistent placer (option "pp", kbhip_pp.hip): kbhip_allocate's batched
pops swept by one launch each and placed in order by one resident workgroup
that keeps its committed rows in LDS.  Records, node state and the gang
plugin's close messages equal the faithful restatement's and the overlapped
pop kernel's, including sweeps that read rows older than the placer's last
commits (the placer re-evaluates those nodes) and chunks the placer cuts at
its list's edge (the host sweeps the rest again)."""
import numpy as np
import pytest

from test_gpu_parity import NO_POD_AFFINITY

pytestmark = pytest.mark.gpu
STATUS = {1: 4, 2: 8}


def _run(engine, path, **opts):
    with engine.Session(path) as s:
        for k, v in opts.items():
            s.set_option(k, v)
        pod, node, kind = s.allocate()
        st = s.stats()
        ns = s.read_nodes(st["nodes"])
        close = s.gang_unschedulable()
    return [(int(p), int(n), int(k)) for p, n, k in zip(pod, node, kind)], ns, st, close


@pytest.mark.parametrize("seed", range(30))
def test_pp_random(engine, oracle_mod, kbgen_mod, tmp_path, seed):
    tiers = [None, [["priority", "gang"], ["drf", "predicates", "proportion", "nodeorder"]],
             [["gang"], ["predicates", "nodeorder"]]][seed % 3]
    c = kbgen_mod.gen_random(9300 + seed, n_nodes=6 + 9 * (seed % 12), n_jobs=5 + seed % 9, max_tasks=2 + seed % 14,
                             features=tuple(f for f in NO_POD_AFFINITY if f != "backfill"), tiers=tiers)
    p = c.write(str(tmp_path / "r.kbs"))
    exp, ons = oracle_mod.ref_allocate(p, with_nodes=True)
    got, ns, st, close = _run(engine, p, pp=1)
    assert [(a, b, STATUS[k]) for a, b, k in got] == exp.as_list()
    assert np.array_equal(ns.astype(np.float64), ons[:ns.shape[0]])
    assert close == oracle_mod.ref_gang_close(p)
    assert st["fit_inexact"] == 0


@pytest.mark.parametrize("spec", [0, 1, 2, 3])
def test_pp_c2(engine, kbgen_mod, tmp_path, spec):
    """C2 at full size, every speculation depth: equal to the overlapped kernel."""
    p = str(tmp_path / "c2.kbs")
    kbgen_mod.gen_c2(p)
    ref = _run(engine, p, pp=0)
    got = _run(engine, p, pp=1, speculate=spec)
    assert got[0] == ref[0] and np.array_equal(got[1], ref[1]) and got[3] == ref[3]
    assert got[2]["batched_pops"] > 1000


def test_pp_c4_scaled(engine, kbgen_mod, tmp_path):
    p = str(tmp_path / "c4s.kbs")
    kbgen_mod.gen_c4(p, n_nodes=20000, n_pending=160000)
    ref = _run(engine, p, pp=0)
    got = _run(engine, p, pp=1)
    assert got[0] == ref[0] and np.array_equal(got[1], ref[1]) and got[3] == ref[3]


def test_pp_then_other_actions(engine, oracle_mod, kbgen_mod, tmp_path):
    """The placer stops at the end of allocate: backfill / preempt after it see its rows."""
    for seed in range(4):
        c = kbgen_mod.gen_preempt(9500 + seed, n_nodes=30, n_queues=3, n_run_jobs=12, n_pend_jobs=6, max_tasks=6)
        p = c.write(str(tmp_path / f"a{seed}.kbs"))
        actions = "allocate, backfill, preempt"
        exp, ons = oracle_mod.ref_allocate(p, actions=actions, with_nodes=True)
        with engine.Session(p) as s:
            s.set_option("pp", 1)
            pod, node, kind = s.run_actions(actions)
            ns = s.read_nodes(30)
        st = {1: 4, 2: 8, 3: 128}
        assert [(int(a), int(b), st[int(k)]) for a, b, k in zip(pod, node, kind)] == exp.as_list()
        assert np.array_equal(ns.astype(np.float64), ons[:30])
