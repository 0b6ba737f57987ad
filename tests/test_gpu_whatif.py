"""What-if sessions batched per launch:
sessions with option rank_group run from concurrent host threads and their
reclaim / preempt node rankings, allocate pops and per-task chunks go out as
multi-session launches (counting sort / pop kernel / sweep, blockIdx.y =
session), each request at once with whatever other sessions' requests are
pending.  Each session's records equal the faithful restatement's and the
same session run alone; every request went through the batcher."""
import threading
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ACTIONS = "reclaim, allocate, backfill, preempt"
STATUS = {1: 4, 2: 8, 3: 128}


def _run(engine, path, group, barrier=None, linger_us=0, actions=ACTIONS, before=None):
    with engine.Session(path) as s:
        if before:  # actions run alone before the grouped ones
            s.run_actions(before)
        if group:
            s.set_option("rank_group", group)
            s.set_option("group_linger_us", linger_us)
        if barrier is not None:  # the sessions start their actions together
            barrier.wait()
        pod, node, kind = s.run_actions(actions)
        st = s.stats()
    return [(int(a), int(b), STATUS[int(k)]) for a, b, k in zip(pod, node, kind)], st


class _linger:
    """group_linger_us is process-wide: back to 0 after the block."""

    def __init__(self, engine, path):
        self.engine, self.path = engine, path

    def __enter__(self):
        return self

    def __exit__(self, *a):
        with self.engine.Session(self.path) as s:
            s.set_option("group_linger_us", 0)


@pytest.mark.parametrize("linger_us", [0, 20000])
@pytest.mark.parametrize("n_sessions", [2, 6])
def test_whatif_sessions_batched(engine, oracle_mod, kbgen_mod, tmp_path, n_sessions, linger_us):
    """linger_us = 0: the product setting (requests share a launch when they
    coincide); 20 ms: a lane waits for every grouped session's request (or
    that long), so the concurrent sessions' rankings and pops meet."""
    paths = []
    for k in range(n_sessions):
        p = str(tmp_path / f"w{k}.kbs")
        kbgen_mod.gen_c5(p, seed=kbgen_mod.BASE_SEED + 70 + k, n_nodes=150, n_pending=120, best_effort=8)
        paths.append(p)
    alone = [_run(engine, p, False)[0] for p in paths]
    bar = threading.Barrier(n_sessions)
    with _linger(engine, paths[0]), ThreadPoolExecutor(n_sessions) as ex:
        res = list(ex.map(lambda p: _run(engine, p, 1, bar, linger_us), paths))
    for p, a, (got, st) in zip(paths, alone, res):
        assert got == a
        assert got == oracle_mod.ref_allocate(p, actions=ACTIONS).as_list()
    req = sum(st["rank_requests"] for _, st in res)
    bsum = sum(st["rank_batch_sum"] for _, st in res)
    assert req > 0 and bsum >= req
    sreq = sum(st["sweep_requests"] for _, st in res)  # per-task chunks (backfill first-fits, general path)
    sbsum = sum(st["sweep_batch_sum"] for _, st in res)
    assert sreq >= n_sessions and sbsum >= sreq  # every session's backfill chunk went through the group
    preq = sum(st["pop_requests"] for _, st in res)  # allocate pops batched across sessions
    pbsum = sum(st["pop_batch_sum"] for _, st in res)
    assert preq > 0 and pbsum >= preq
    if linger_us and n_sessions > 2:
        assert bsum > req  # some launch ranked more than one session's nodes
        assert pbsum > preq  # some pop launch served several sessions


def test_whatif_backfill_chunks_batched(engine, oracle_mod, kbgen_mod, tmp_path):
    """Six sessions allocate alone, then run backfill together under the
    linger: their first-fit chunks share k_sweep_argmax_multi launches (the
    assertion r05 dropped: without the linger sessions reach backfill at
    different times); records equal each session alone and the oracle."""
    paths = []
    for k in range(6):
        p = str(tmp_path / f"b{k}.kbs")
        kbgen_mod.gen_c5(p, seed=kbgen_mod.BASE_SEED + 90 + k, n_nodes=150, n_pending=120, best_effort=8)
        paths.append(p)
    alone = [_run(engine, p, False, actions="backfill", before="allocate")[0] for p in paths]
    bar = threading.Barrier(len(paths))
    with _linger(engine, paths[0]), ThreadPoolExecutor(len(paths)) as ex:
        res = list(ex.map(lambda p: _run(engine, p, 1, bar, 20000, "backfill", "allocate"), paths))
    for p, a, (got, st) in zip(paths, alone, res):
        assert got == a
    sreq = sum(st["sweep_requests"] for _, st in res)
    sbsum = sum(st["sweep_batch_sum"] for _, st in res)
    assert sreq >= len(paths) and sbsum > sreq


def test_whatif_full_size_grouped(engine, kbgen_mod, tmp_path):
    """C5 at full size (50k nodes ~90 % filled, 2k-task pending sets): four
    grouped sessions run concurrently record exactly what each records alone
    (tests/test_gpu_evict.py pins the session alone against the hoisted
    restatement at full size)."""
    import os
    cache = os.environ.get("KBHIP_BENCH_CACHE", "/tmp/kbhip_bench")
    os.makedirs(cache, exist_ok=True)
    paths = []
    for k in range(4):  # bench_c5.py's snapshots (same names): generated once per box
        p = os.path.join(cache, f"c5_50000_2000_{k}.kbs")
        if not os.path.exists(p):
            kbgen_mod.gen_c5(p + ".tmp", seed=kbgen_mod.BASE_SEED + 5 + k, n_nodes=50_000, n_pending=2000)
            os.replace(p + ".tmp", p)
        paths.append(p)
    alone = [_run(engine, p, False)[0] for p in paths]
    bar = threading.Barrier(len(paths))
    with ThreadPoolExecutor(len(paths)) as ex:
        res = list(ex.map(lambda p: _run(engine, p, 1, bar), paths))
    for a, (got, st) in zip(alone, res):
        assert len(got) > 100_000
        assert got == a
    assert sum(st["rank_batch_sum"] for _, st in res) >= sum(st["rank_requests"] for _, st in res)


def test_time_rank_multi(engine, kbgen_mod, tmp_path):
    """kbhip_time_rank_multi (the measurement entry of the multi-session
    ranking chain): positive device time with descriptors in device memory and
    in mapped host memory, warm and cold; a session listed twice is refused."""
    paths = []
    for k in range(3):
        p = str(tmp_path / f"r{k}.kbs")
        kbgen_mod.gen_c5(p, seed=kbgen_mod.BASE_SEED + 110 + k, n_nodes=300, n_pending=60)
        paths.append(p)
    ss = [engine.Session(p) for p in paths]
    try:
        ids = [int(np.nonzero(s.table("pod_class") >= 0)[0][0]) for s in ss]
        for mapped in (0, 1):
            for evict in (0, 2):
                assert engine.time_rank_multi(ss, ids, reps=3, evict=evict, mapped=mapped) > 0
        with pytest.raises(engine.KbhipError):
            engine.time_rank_multi([ss[0], ss[0]], ids[:2])
    finally:
        for s in ss:
            s.close()
