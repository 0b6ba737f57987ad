"""The asynchronous per-pop ABI (kbhip_place_job_submit / _wait / _cancel,
include/kbhip.h): pops submitted ahead of their wait run on the device state
their predecessors leave, exactly as a sequence of kbhip_place_job calls;
cancelled pops leave no trace.

Two drivers:
- the C++ host loop (kube-batch-1_amd/host/kbhost.cpp: allocate.go:41-201 with
  the ordering plugins and Go's heap, predicting `depth` pops ahead): its
  placement logs in sync and pipelined mode must equal the CPU oracle's;
- a recorded pop sequence (tests/gohost.py over kbhip_place_job) replayed
  through submit / wait / cancel in several interleavings."""
import json
import os
import subprocess

import numpy as np
import pytest

from gohost import GoHost
from test_gpu_parity import NO_POD_AFFINITY

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KBHOST = os.path.join(ROOT, "kube-batch-1_amd", "_build", "kbhost")
TIERS = [None, [["drf", "proportion"]], [["gang"], ["predicates", "nodeorder"]],
         [["priority", "gang", "drf"], ["predicates", "proportion", "nodeorder", "nodeorder"]]]


def _kbhost(path, tmp_path, modes="allocate,sync,async", depth=2, reps=1, timeout=300):
    if not os.path.exists(KBHOST):
        pytest.fail(f"{KBHOST} is missing: run __graft_entry__.build()")
    out = str(tmp_path / "log")
    r = subprocess.run([KBHOST, path, "--modes", modes, "--depth", str(depth), "--reps", str(reps),
                        "--log-out", out], capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout + r.stderr
    rec = json.loads(r.stdout.strip().splitlines()[-1])
    logs = {}
    for m in modes.split(","):
        a = np.fromfile(f"{out}.{m}.bin", dtype=np.int32).reshape(-1, 3)
        logs[m] = [tuple(int(x) for x in row) for row in a]
    return rec, logs


@pytest.mark.parametrize("seed", range(16))
def test_kbhost_random(engine, oracle_mod, kbgen_mod, tmp_path, seed):
    feats = NO_POD_AFFINITY if seed % 3 else ("labels", "taints", "ports", "affinity", "init", "running",
                                              "releasing", "selector", "nodeaffinity", "podaffinity", "unsched")
    c = kbgen_mod.gen_random(9300 + seed, n_nodes=4 + seed % 12, n_jobs=4 + seed % 9, max_tasks=1 + seed % 8,
                             features=feats, tiers=TIERS[seed % 4], n_queues=1 + seed % 3)
    p = str(tmp_path / "r.kbs")
    c.write(p)
    exp = oracle_mod.ref_allocate(p).as_list()
    rec, logs = _kbhost(p, tmp_path, depth=1 + seed % 3)
    assert rec["equal"], rec
    for m, got in logs.items():
        assert got == exp, m


def test_kbhost_c2(engine, oracle_mod, kbgen_mod, tmp_path):
    """C2 (5k nodes x 50k pods): the pipelined host loop against the oracle."""
    p = str(tmp_path / "c2.kbs")
    kbgen_mod.gen_c2(p)
    exp = oracle_mod.fast_allocate(p, threads=16).as_list()
    rec, logs = _kbhost(p, tmp_path, reps=1)
    assert rec["equal"], rec
    assert logs["async"] == exp
    assert rec["async"]["async_launched"] > 0
    print(json.dumps(rec))


def test_kbhost_c3_scaled(engine, oracle_mod, kbgen_mod, tmp_path):
    """C3-shaped (zone anti-affinity gangs, selectors, taints, 8 queues), 2k
    nodes: anti-affinity pops are launched at submit (placement 7); a launch
    whose candidate list runs out goes on synchronously inside its wait."""
    p = str(tmp_path / "c3.kbs")
    kbgen_mod.gen_c3(n_nodes=2000, n_pending=6000).write(p)
    exp = oracle_mod.fast_allocate(p, threads=8).as_list()
    rec, logs = _kbhost(p, tmp_path, reps=1)
    assert rec["equal"], rec
    assert logs["async"] == exp and logs["sync"] == exp
    assert rec["async"]["async_launched"] > 0


def test_kbhost_c5_scaled(engine, oracle_mod, kbgen_mod, tmp_path):
    """C5-shaped (Backfilled nodes: every pop's walk mutates Idle), 600 nodes:
    the pipelined host loop runs each pop inside its wait and equals the oracle."""
    p = str(tmp_path / "c5.kbs")
    kbgen_mod.gen_c5(p, n_nodes=600, n_pending=300, best_effort=20)
    exp = oracle_mod.fast_allocate(p, threads=8).as_list()
    rec, logs = _kbhost(p, tmp_path, reps=1)
    assert rec["equal"], rec
    assert logs["async"] == exp and logs["sync"] == exp


def _record(engine, path, cluster):
    """The pop sequence of a synchronous run: [(ids, gm, min, ready, (nodes, kinds, stop))]."""
    calls = []
    with engine.Session(path) as s:
        def place_job(ids, gm, min_avail, ready):
            r = s.place_job(ids, gm, min_avail, ready)
            calls.append((list(ids), gm, min_avail, ready, r))
            return r
        log, _ = GoHost(cluster).allocate(place_job)
        nodes = s.read_nodes(len(cluster.nodes))
    return calls, log, nodes


def _same(a, b):
    return list(a[0]) == list(b[0]) and list(a[1]) == list(b[1]) and a[2] == b[2]


@pytest.mark.parametrize("seed", range(8))
def test_submit_ahead_replays_sync_run(engine, kbgen_mod, tmp_path, seed):
    """The recorded pops submitted up to 6 ahead, waited in order: identical results."""
    c = kbgen_mod.gen_random(9400 + seed, n_nodes=6 + seed, n_jobs=6 + seed, max_tasks=2 + seed % 6,
                             features=NO_POD_AFFINITY, tiers=TIERS[seed % 4])
    p = str(tmp_path / "r.kbs")
    c.write(p)
    calls, _, nodes = _record(engine, p, c)
    ahead = 1 + seed % 6
    with engine.Session(p) as s:
        tix = []
        k = 0
        for i, (ids, gm, mn, rd, res) in enumerate(calls):
            while k < len(calls) and k <= i + ahead:
                tix.append(s.place_job_submit(calls[k][0], calls[k][1], calls[k][2], calls[k][3]))
                k += 1
            got = s.place_job_wait(tix[i])
            assert _same(got, res), (i, got, res)
        assert (s.read_nodes(len(c.nodes)) == nodes).all()
        st = s.stats()
        assert st["async_cancelled"] == 0 and st["async_retracted"] == 0


@pytest.mark.parametrize("seed", range(6))
def test_cancel_withdraws_device_updates(engine, kbgen_mod, tmp_path, seed):
    """Every pop after the first is submitted, then withdrawn and submitted
    again: the run ends exactly as the synchronous one."""
    c = kbgen_mod.gen_random(9500 + seed, n_nodes=6 + seed, n_jobs=5 + seed, max_tasks=2 + seed % 5,
                             features=NO_POD_AFFINITY, tiers=TIERS[seed % 4])
    p = str(tmp_path / "r.kbs")
    c.write(p)
    calls, _, nodes = _record(engine, p, c)
    if len(calls) < 2:
        pytest.skip("a single pop")
    with engine.Session(p) as s:
        for i, (ids, gm, mn, rd, res) in enumerate(calls):
            t = s.place_job_submit(ids, gm, mn, rd)
            nxt = calls[i + 1:i + 4]
            ahead = [s.place_job_submit(*x[:4]) for x in nxt]
            if ahead:  # a wrong guess: the later pops' arguments shifted by one
                bogus = s.place_job_submit(*calls[(i + 2) % len(calls)][:4])
                assert s.place_job_cancel(ahead[0]) == len(ahead) + 1
                del bogus
            got = s.place_job_wait(t)
            assert _same(got, res), (i, got, res)
        assert (s.read_nodes(len(c.nodes)) == nodes).all()
        st = s.stats()
        assert st["async_cancelled"] > 0


def test_ticket_rules(engine, kbgen_mod, tmp_path):
    c = kbgen_mod.gen_c1()
    p = str(tmp_path / "c1.kbs")
    c.write(p)
    calls, _, _ = _record(engine, p, c)
    assert len(calls) >= 2
    with engine.Session(p) as s:
        a = s.place_job_submit(*calls[0][:4])
        b = s.place_job_submit(*calls[1][:4])
        with pytest.raises(engine.KbhipError, match="oldest"):
            s.place_job_wait(b)
        with pytest.raises(engine.KbhipError, match="outstanding"):
            s.allocate()
        with pytest.raises(engine.KbhipError, match="outstanding"):
            s.place_job(*calls[0][:4])
        with pytest.raises(engine.KbhipError, match="no outstanding"):
            s.place_job_cancel(b + 5)
        assert _same(s.place_job_wait(a), calls[0][4])
        assert _same(s.place_job_wait(b), calls[1][4])
        with pytest.raises(engine.KbhipError, match="oldest"):
            s.place_job_wait(b)
        s.place_job_submit(*calls[0][:4])  # outstanding at close: dropped
    with engine.Session(p) as s:  # a fresh session after a close with tickets outstanding
        assert _same(s.place_job(*calls[0][:4]), calls[0][4])


def test_refused_wait_keeps_ticket(engine, kbgen_mod, tmp_path):
    """A wait refused with EINVAL (not the oldest ticket) leaves that ticket's
    result arrays sized for all its tasks: the retried wait of a multi-task
    pop reports every task (the binding lost the size)."""
    c = kbgen_mod.gen_random(9601, n_nodes=24, n_jobs=6, max_tasks=12, features=NO_POD_AFFINITY,
                             tiers=[["gang"], ["predicates", "nodeorder"]])
    p = str(tmp_path / "r.kbs")
    c.write(p)
    calls, _, _ = _record(engine, p, c)
    multi = [i for i, x in enumerate(calls) if len(x[4][0]) > 1]
    assert multi, "the generator gave no multi-task pop"
    i = multi[0]
    assert i + 1 < len(calls) or i > 0
    with engine.Session(p) as s:
        for x in calls[:i]:
            assert _same(s.place_job(*x[:4]), x[4])
        a = s.place_job_submit(*calls[i][:4])
        b = s.place_job_submit(*calls[i + 1][:4]) if i + 1 < len(calls) else None
        if b is not None:
            with pytest.raises(engine.KbhipError, match="oldest"):
                s.place_job_wait(b)  # refused: b's size stays in the binding
        assert _same(s.place_job_wait(a), calls[i][4])
        if b is not None:
            assert _same(s.place_job_wait(b), calls[i + 1][4])


def test_deferred_pops_keep_order(engine, kbgen_mod, tmp_path):
    """Pops longer than one chunk (or of mixed classes) run inside their wait;
    the pops behind them launch only after."""
    c = kbgen_mod.gen_random(9600, n_nodes=24, n_jobs=6, max_tasks=40, features=NO_POD_AFFINITY,
                             tiers=[["gang"], ["predicates", "nodeorder"]])
    p = str(tmp_path / "r.kbs")
    c.write(p)
    calls, _, nodes = _record(engine, p, c)
    assert any(len(x[0]) > 16 for x in calls)
    with engine.Session(p) as s:
        tix = [s.place_job_submit(*x[:4]) for x in calls[:48]]
        for i, t in enumerate(tix):
            assert _same(s.place_job_wait(t), calls[i][4]), i
        for x in calls[48:]:
            assert _same(s.place_job_wait(s.place_job_submit(*x[:4])), x[4])
        assert (s.read_nodes(len(c.nodes)) == nodes).all()
