"""The persistent pop engine (kube-batch-1_amd/csrc/kbhip_engine.hip,
DESIGN.md §4.10): one resident grid serves the batched pops of
allocate.go:110-185 from a descriptor ring.  Its placement logs, node state and
gang close messages must equal the CPU oracle's and the launched kernels'
(option engine = 0), including the paths only the engine has: worker blocks
with several nodes per thread, pops whose candidates were left out or dropped
(the previous two pops'), a task that finds no node (the FitDelta histogram
from the group count words), runs interleaved with launched pops (classes the
engine does not serve), and a run that ends idle and is restarted."""
import time

import numpy as np
import pytest

from gohost import GoHost
from test_gpu_parity import NO_POD_AFFINITY

pytestmark = pytest.mark.gpu

TIERS = [None, [["drf", "proportion"]], [["gang"], ["predicates", "nodeorder"]],
         [["priority", "gang", "drf"], ["predicates", "proportion", "nodeorder", "nodeorder"]]]


def _run(lib, path, **opts):
    with lib.Session(path) as s:
        for k, v in opts.items():
            s.set_option(k, v)
        pod, node, kind = s.allocate()
        st = s.stats()
        ns = s.read_nodes(st["nodes"])
        close = s.gang_unschedulable()
    return [(int(p), int(n), 4 if k == 1 else 8) for p, n, k in zip(pod, node, kind)], ns, st, close


@pytest.mark.parametrize("lists", [1, 0])
@pytest.mark.parametrize("seed", range(32))
def test_engine_random_snapshots(engine, oracle_mod, kbgen_mod, tmp_path, seed, lists):
    """Feature-rich small snapshots: engine pops (resource / selector / taint
    classes) between launched ones (host ports, backfill annotation), against
    the faithful restatement and the launched path; list mode (class owners,
    DESIGN.md §4.11) and sweep mode."""
    c = kbgen_mod.gen_random(5100 + seed, n_nodes=4 + seed % 13, n_jobs=4 + seed % 9, max_tasks=1 + seed % 9,
                             features=NO_POD_AFFINITY, tiers=TIERS[seed % 4], n_queues=1 + seed % 3)
    p = str(tmp_path / "r.kbs")
    c.write(p)
    exp, ons = oracle_mod.ref_allocate(p, with_nodes=True)
    exp_close = oracle_mod.ref_gang_close(p)
    got, ns, st, close = _run(engine, p, engine_lists=lists)
    assert got == exp.as_list()
    assert np.array_equal(ns.astype(np.float64), ons[:ns.shape[0]])
    assert close == exp_close
    if st["engine_pops"]:
        assert (st["engine_owners"] > 0) == bool(lists)
    ref, ns0, st0, close0 = _run(engine, p, engine=0)
    assert ref == got and np.array_equal(ns0, ns) and close0 == close
    assert st0["engine_pops"] == 0


@pytest.mark.parametrize("workers", [1, 2, 5, 13])
def test_engine_worker_shapes(engine, oracle_mod, kbgen_mod, tmp_path, workers):
    """C2's generator at 3k nodes x 20k pods with few worker blocks: several
    nodes per thread (up to 3000 per block), groups of one or several workers."""
    p = str(tmp_path / "c2w.kbs")
    kbgen_mod.gen_c2(p, n_nodes=3000, n_pending=20000, seed=9300 + workers)
    exp = oracle_mod.fast_allocate(p, threads=8).as_list()
    got, ns, st, close = _run(engine, p, engine_workers=workers, engine_lists=0)
    assert got == exp
    assert st["engine_workers"] == workers and st["engine_pops"] == st["batched_pops"] > 100
    ref, ns0, _, close0 = _run(engine, p, engine=0)
    assert np.array_equal(ns0, ns) and close0 == close


@pytest.mark.parametrize("seed", range(8))
def test_engine_levels_only(engine, oracle_mod, kbgen_mod, tmp_path, seed):
    """engine_quick = 0: every decision by the levels over all the placer's
    waves (place_decide), not the single-wave path (place_decide_quick) —
    both must give the restatement's placements."""
    c = kbgen_mod.gen_random(5300 + seed, n_nodes=3 + seed % 5, n_jobs=6, max_tasks=12,
                             features=("labels", "running", "selector", "taints"), tiers=TIERS[seed % 4])
    p = str(tmp_path / "l.kbs")
    c.write(p)
    exp, ons = oracle_mod.ref_allocate(p, with_nodes=True)
    got, ns, st, close = _run(engine, p, engine_quick=0)
    assert got == exp.as_list()
    assert np.array_equal(ns.astype(np.float64), ons[:ns.shape[0]])
    assert close == oracle_mod.ref_gang_close(p)
    assert st["engine_pops"] > 0
    got1, ns1, _, close1 = _run(engine, p)
    assert got1 == got and np.array_equal(ns1, ns) and close1 == close


def test_engine_c2_levels_only(engine, oracle_mod, kbgen_mod, tmp_path):
    """C2's generator at 2k nodes x 12k pods, levels only vs the default."""
    p = str(tmp_path / "c2l.kbs")
    kbgen_mod.gen_c2(p, n_nodes=2000, n_pending=12000, seed=9350)
    exp = oracle_mod.fast_allocate(p, threads=8).as_list()
    got, ns, st, _ = _run(engine, p, engine_quick=0)
    assert got == exp and st["engine_pops"] > 50
    got1, ns1, _, _ = _run(engine, p)
    assert got1 == exp and np.array_equal(ns1, ns)


@pytest.mark.parametrize("lists", [1, 0])
@pytest.mark.parametrize("speculate", [2, 0])
def test_engine_unplaceable_gangs(engine, oracle_mod, kbgen_mod, tmp_path, speculate, lists):
    """A crowded cluster: many pops end on a task with no node, so the gang
    close messages carry the FitDelta histograms the engine counts (workers'
    counts without the previous pops' candidates, the placer's re-evaluated
    ones) — equal to the faithful restatement's.  speculate 0: the host sends
    the next descriptor only after such a pop's results (the counts it reads
    must not wait for it)."""
    GI = 1 << 30
    rng = np.random.default_rng(9400)
    c = kbgen_mod.Cluster()
    c.add_queue("q0", 1)
    for i in range(160):
        c.add_node(f"n{i:04d}", int(rng.choice([4000, 8000])), int(rng.choice([8, 16])) * GI,
                   int(rng.choice([0, 0, 4000])), 110)
    uid = 0
    for j in range(40):
        size = int(rng.integers(4, 30))
        jn = f"j{j:03d}"
        c.add_job("ns", jn, "q0", min_member=size, ts=j)
        req = kbgen_mod.res(cpu=int(rng.choice([1000, 2000, 3000])), mem=int(rng.choice([2, 4, 6])) * GI,
                            gpu=int(rng.choice([0, 0, 0, 1000])))
        for k in range(size):
            c.add_pod("ns", f"{jn}-{k}", uid=f"p{uid:05d}", group=jn, ts=j, containers=[dict(req)])
            uid += 1
    p = c.write(str(tmp_path / "u.kbs"))
    exp = oracle_mod.ref_allocate(p).as_list()
    exp_close = oracle_mod.ref_gang_close(p)
    t0 = time.time()
    got, ns, st, close = _run(engine, p, speculate=speculate, engine_lists=lists)
    assert time.time() - t0 < 20
    assert got == exp
    assert close == exp_close and len(close) > 5
    assert st["unassigned_pops"] > 5 and st["engine_pops"] > 20


@pytest.mark.parametrize("lists", [1, 0])
def test_engine_c4_scaled(engine, oracle_mod, kbgen_mod, tmp_path, lists):
    """C4's shape at 20k nodes x 120k pods through the engine (every pop)."""
    p = str(tmp_path / "c4s.kbs")
    kbgen_mod.gen_c4(p, n_nodes=20000, n_pending=120000)
    exp = oracle_mod.fast_allocate(p, threads=16).as_list()
    got, _, st, _ = _run(engine, p, engine_lists=lists)
    assert got == exp
    assert st["engine_pops"] == st["batched_pops"] and st["engine_launches"] <= 3
    assert (st["engine_owners"] > 0) == bool(lists)


def test_engine_idle_restart(engine, oracle_mod, kbgen_mod, tmp_path):
    """The per-pop ABI with the host idle for longer than the engine waits
    (1 s): the run ends on its own and the next pop starts a new one; pops
    submitted just before an idle end are served by the restart."""
    c = kbgen_mod.gen_random(9500, n_nodes=12, n_jobs=6, max_tasks=6, features=("labels", "running", "selector"))
    p = str(tmp_path / "i.kbs")
    c.write(p)
    exp = oracle_mod.ref_allocate(p).as_list()
    with engine.Session(p) as s:
        calls = [0]

        def place_job(ids, gm, min_avail, ready):
            calls[0] += 1
            if calls[0] in (2, 4):
                time.sleep(1.6)
            return s.place_job(ids, gm, min_avail, ready)
        got, _ = GoHost(c).allocate(place_job)
        st = s.stats()
    assert got == exp
    assert st["engine_launches"] >= 2


def test_engine_two_sessions_threads(engine, oracle_mod, kbgen_mod, tmp_path):
    """Two engine-eligible sessions allocating at once from two threads of one
    process: one device, one engine at a time (the in-process claim,
    eng_claim); the other session's pops take the launched path meanwhile.
    Both logs equal the hoisted restatement's, no KBHIP_EDEVICE, bounded
    time."""
    import threading
    paths, exps = [], []
    for i in range(2):
        p = str(tmp_path / f"c2t{i}.kbs")
        kbgen_mod.gen_c2(p, n_nodes=3000, n_pending=20000, seed=9600 + i)
        paths.append(p)
        exps.append(oracle_mod.fast_allocate(p, threads=8).as_list())
    out = [None, None]
    errs = []

    def run(i):
        try:
            for _ in range(3):  # several sessions each, so that the two overlap
                out[i] = _run(engine, paths[i])
        except Exception as e:  # noqa: BLE001 (reported below)
            errs.append(repr(e))
    t0 = time.time()
    th = [threading.Thread(target=run, args=(i,)) for i in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    assert not any(t.is_alive() for t in th)
    assert not errs, errs
    assert time.time() - t0 < 120
    for i in range(2):
        assert out[i][0] == exps[i]
    assert out[0][2]["engine_pops"] + out[1][2]["engine_pops"] > 0


def _proc_allocate(path, q):
    import kbhip
    with kbhip.Session(path) as s:
        pod, node, kind = s.allocate()
        st = s.stats()
    q.put(([(int(p), int(n), 4 if k == 1 else 8) for p, n, k in zip(pod, node, kind)],
           int(st["engine_pops"]), int(st["engine_not_resident"])))


def test_engine_two_processes(engine, oracle_mod, kbgen_mod, tmp_path):
    """Two processes on one GPU, each with an engine-eligible session: a grid
    that cannot become resident while the other holds the CUs ends serving
    nothing and is started again (eng_arrive, kEngErrResident) — both logs
    equal the restatement's."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    paths, exps = [], []
    for i in range(2):
        p = str(tmp_path / f"c2p{i}.kbs")
        kbgen_mod.gen_c2(p, n_nodes=3000, n_pending=20000, seed=9700 + i)
        paths.append(p)
        exps.append(oracle_mod.fast_allocate(p, threads=8).as_list())
    q = ctx.Queue()
    ps = [ctx.Process(target=_proc_allocate, args=(paths[i], q)) for i in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=180) for _ in range(2)]
    for p in ps:
        p.join(30)
        assert p.exitcode == 0
    logs = sorted(r[0] for r in res)
    assert logs == sorted(exps)
    assert all(r[1] > 0 for r in res)
