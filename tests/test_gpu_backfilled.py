"""Batched pops in sessions with Backfilled nodes (placement 6): every walk
visit adds a node's Backfilled to its Idle (GetAccessibleResource,
node_info.go:209-211; allocate.go:150-180), so nodes other than the winner
change between a pop's tasks.  The engine's records, node state and gang
close messages equal the faithful restatement's (oracle/kbref.cpp), and equal
the per-task path's (option bf_batch = 0)."""
import numpy as np
import pytest

from test_gpu_parity import NO_POD_AFFINITY

pytestmark = pytest.mark.gpu
GI = 1 << 30


def _run(engine, path, actions="allocate", **opts):
    with engine.Session(path) as s:
        for k, v in opts.items():
            s.set_option(k, v)
        pod, node, kind = s.run_actions(actions)
        st = s.stats()
        ns = s.read_nodes(st["nodes"])
        close = s.gang_unschedulable()
    return [(int(p), int(n), int(k)) for p, n, k in zip(pod, node, kind)], ns, st, close


def _visit_cluster(kbgen, seed, n_nodes, n_jobs):
    """Nodes whose Idle alone rarely fits a task but Idle + k x Backfilled does
    after k walk visits; gangs large enough that one pop spans many visits."""
    rng = np.random.default_rng(seed)
    c = kbgen.Cluster()
    c.add_queue("q0", 1)
    c.add_queue("q1", 2)
    for i in range(n_nodes):
        cpu = int(rng.choice([4000, 8000, 16000]))
        mem = int(rng.choice([8, 16, 32])) * GI
        c.add_node(f"n{i:03d}", cpu, mem, 0, int(rng.choice([6, 20, 110])))
        for k in range(int(rng.integers(0, 4))):  # running pods, some backfill-annotated
            bf = rng.random() < 0.6
            c.add_pod("run", f"r{i}-{k}", uid=f"r{i:03d}{k}", node=f"n{i:03d}", phase="Running", backfill=bf,
                      containers=[kbgen.res(cpu=int(rng.choice([500, 1000, 2000])), mem=int(rng.integers(1, 4)) * GI)])
    uid = 0
    for j in range(n_jobs):
        size = int(rng.integers(1, 24))
        jn = f"j{j:03d}"
        c.add_job("ns", jn, f"q{j % 2}", min_member=int(rng.integers(1, size + 1)), ts=j)
        req = kbgen.res(cpu=int(rng.choice([700, 1500, 2500, 3500])), mem=int(rng.choice([1, 2, 6])) * GI)
        for k in range(size):
            c.add_pod("ns", f"{jn}-{k}", uid=f"p{uid:05d}", group=jn, ts=j, containers=[dict(req)])
            uid += 1
    return c


def _check(engine, oracle_mod, p, actions="allocate"):
    exp, ons = oracle_mod.ref_allocate(p, actions=actions, with_nodes=True)
    exp_close = oracle_mod.ref_gang_close(p, actions=actions)
    status = {1: 4, 2: 8, 3: 128}
    got, ns, st, close = _run(engine, p, actions)
    assert [(a, b, status[k]) for a, b, k in got] == exp.as_list()
    assert np.array_equal(ns.astype(np.float64), ons[:ns.shape[0]])
    assert close == exp_close
    ref, ns0, st0, close0 = _run(engine, p, actions, bf_batch=0)
    assert ref == got and np.array_equal(ns0, ns) and close0 == close
    return st, st0


@pytest.mark.parametrize("seed", range(24))
def test_backfilled_visits(engine, oracle_mod, kbgen_mod, tmp_path, seed):
    c = _visit_cluster(kbgen_mod, 7100 + seed, n_nodes=6 + 7 * (seed % 10), n_jobs=4 + seed % 8)
    p = c.write(str(tmp_path / "v.kbs"))
    st, st0 = _check(engine, oracle_mod, p)
    assert st["batched_pops"] > 0
    if any(q.backfill and q.node for q in c.pods):  # Backfilled nodes: batched only with bf_batch
        assert st0["batched_pops"] == 0


@pytest.mark.parametrize("seed", range(24))
def test_backfilled_random(engine, oracle_mod, kbgen_mod, tmp_path, seed):
    c = kbgen_mod.gen_random(7300 + seed, n_nodes=4 + seed % 12, n_jobs=5 + seed % 9, max_tasks=2 + seed % 12,
                             features=NO_POD_AFFINITY)
    p = c.write(str(tmp_path / "r.kbs"))
    _check(engine, oracle_mod, p, ["allocate", "allocate, backfill", "backfill, allocate"][seed % 3])


def test_backfilled_many_nodes(engine, oracle_mod, kbgen_mod, tmp_path):
    """Lists that fill: more eligible nodes than a pop's 64 candidates, so pops
    end at the list's edge and go on in the next launch."""
    c = _visit_cluster(kbgen_mod, 7500, n_nodes=200, n_jobs=30)
    p = c.write(str(tmp_path / "m.kbs"))
    st, _ = _check(engine, oracle_mod, p)
    assert st["batched_pops"] > 0


@pytest.mark.parametrize("seed", range(2))
def test_c5_scaled_batched(engine, oracle_mod, kbgen_mod, tmp_path, seed):
    """C5's generator (5 % backfill pods), the what-if action list."""
    p = str(tmp_path / "c5.kbs")
    kbgen_mod.gen_c5(p, seed=kbgen_mod.BASE_SEED + 50 + seed, n_nodes=120, n_pending=150, best_effort=8)
    st, _ = _check(engine, oracle_mod, p, "reclaim, allocate, backfill, preempt")
    assert st["batched_pops"] > 0
