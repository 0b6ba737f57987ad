"""Node-array sharding.

CPU (gloo, world size 2 and 3): the exchange callback reduces selection keys
(u64, top bit set), and the IPA min/max (i64) exactly like the RCCL
all-reduce the GPU ranks use; shard ranges partition the node array.
GPU: ranks sharing the MI355X (gloo exchange) place exactly like the oracle
(tests/test_gpu_parity.py covers the one-GPU session)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _run_ranks(script, world, tmp_path, extra, timeout=300, env=None):
    import uuid
    init = str(tmp_path / f"init_{world}_{uuid.uuid4().hex}")  # a fresh rendezvous file per group
    outs = [str(tmp_path / f"out{r}.json") for r in range(world)]
    env = dict(os.environ, OMP_NUM_THREADS="1", **(env or {}))
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, script)] + extra(r, init, outs[r]), env=env)
             for r in range(world)]
    try:
        rcs = [p.wait(timeout=timeout) for p in procs]
    except subprocess.TimeoutExpired:
        pytest.fail(f"shard ranks did not finish within {timeout} s")
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert rcs == [0] * world, rcs
    res = []
    for o in outs:
        with open(o) as f:
            res.append(json.load(f))
    return res


@pytest.mark.parametrize("world", [2, 3])
def test_exchange_gloo(world, tmp_path):
    sys.path.insert(0, HERE)
    from exchange_worker import values
    res = _run_ranks("exchange_worker.py", world, tmp_path, lambda r, init, out: [str(r), str(world), init, out])
    keys = np.stack([values(r)[0] for r in range(world)])
    ints = np.stack([values(r)[1] for r in range(world)])
    for r in range(world):
        assert res[r]["max_u64"] == [int(x) for x in keys.max(axis=0)]
        assert res[r]["min_i64"] == [int(x) for x in ints.min(axis=0)]
        assert res[r]["max_i64"] == [int(x) for x in ints.max(axis=0)]
        assert res[r]["sum_i64"] == [int(x) for x in ints.sum(axis=0)]
        exp = np.concatenate([(np.arange(40, dtype=np.uint8) * (q + 1)).astype(np.uint8) for q in range(world)])
        assert res[r]["gather"] == [int(x) for x in exp]


def test_shard_ranges_partition(engine_lib):
    import kbhip
    for n in (0, 1, 7, 100, 100_000):
        for world in (1, 2, 3, 8):
            rs = [kbhip.shard_range(n, r, world) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))
            assert all(hi - lo in (n // world, n // world + 1) for lo, hi in rs)


def _shard_case(oracle_mod, tmp_path, c, world, actions="allocate", batched=1, exp=None, exchange="host"):
    p = str(tmp_path / "s.kbs")
    c.write(p)
    if exp is None:
        exp = oracle_mod.ref_allocate(p, actions=actions).as_list()
    # the gang plugin's close messages (FitError histograms summed over the shards)
    exp_close = oracle_mod.ref_gang_close(p) if actions == "allocate" else None
    res = _run_ranks("shard_worker.py", world, tmp_path,
                     lambda r, init, out: [p, str(r), str(world), init, out, actions, str(batched)], timeout=240,
                     env={"KBHIP_TEST_EXCHANGE": exchange})
    n_nodes = len(c.nodes)
    import kbhip
    for r in range(world):
        lo, hi = kbhip.shard_range(n_nodes, r, world)
        assert res[r]["info"] == [r, world, lo, hi]
        got = [(a, b, {1: 4, 2: 8, 3: 128}[k]) for a, b, k in res[r]["log"]]  # (3: evicted, Releasing)
        assert got == exp, f"rank {r}"
        if exp_close is not None:
            assert res[r]["close"] == exp_close, f"rank {r}"
    return res


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("batched", [1, 0])
def test_sharded_random_gpu(engine, oracle_mod, kbgen_mod, tmp_path, seed, batched):
    """2 or 3 ranks on one GPU, every feature (pod affinity, backfill, ports...);
    batched 1: per-pop all-gather path where the class allows it, 0: per-task only."""
    c = kbgen_mod.gen_random(2200 + seed, n_nodes=6 + seed * 3, n_jobs=6, max_tasks=5, best_effort_p=0.2)
    _shard_case(oracle_mod, tmp_path, c, 2 + seed % 2, actions="allocate, backfill", batched=batched)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(8))
@pytest.mark.parametrize("batched", [1, 0])
def test_sharded_close_messages_gpu(engine, oracle_mod, kbgen_mod, tmp_path, seed, batched):
    """FitError on shards: every feature (inter-pod priority classes, pod
    affinity, ports), gangs that cannot become Ready; the close messages of
    every rank equal the oracle's (walk histograms summed over the shards)."""
    c = kbgen_mod.gen_random(2700 + seed, n_nodes=5 + seed * 2, n_jobs=7, max_tasks=5, best_effort_p=0.1)
    for j in c.jobs[::2]:
        j.min_member += 2
    _shard_case(oracle_mod, tmp_path, c, 2 + seed % 2, batched=batched)


@pytest.mark.gpu
@pytest.mark.parametrize("exchange", ["host", "mailbox", "mailbox_serial", "mailbox_cu"])
@pytest.mark.parametrize("seed", range(8))
def test_sharded_batched_random_gpu(engine, oracle_mod, kbgen_mod, tmp_path, seed, exchange):
    """Batched-path features only (no pod affinity / backfill): every pop is
    one exchange — a host all-gather, or the peer mailboxes (kernels only;
    a shard's sweep of the next pop beside the placement, or serial; _cu:
    each rank's streams on its own share of the CUs, option cu_split)."""
    from test_gpu_parity import NO_POD_AFFINITY
    feats = tuple(f for f in NO_POD_AFFINITY if f != "backfill")
    c = kbgen_mod.gen_random(2400 + seed, n_nodes=10 + seed * 7, n_jobs=8, max_tasks=8, features=feats,
                             tiers=[["priority", "gang", "conformance"], ["drf", "predicates", "proportion",
                                                                           "nodeorder"]])
    res = _shard_case(oracle_mod, tmp_path, c, 2 + seed % 3, exchange=exchange)
    assert all(r["batched_pops"] > 0 for r in res)


EVICT_ACTIONS = ["reclaim", "preempt", "reclaim, allocate, backfill, preempt", "allocate, preempt"]


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(8))
def test_sharded_evict_gpu(engine, oracle_mod, kbgen_mod, tmp_path, seed):
    """Reclaim and preempt on node-array shards (reclaim.go:41-196,
    preempt.go:43-353): each rank ranks its own nodes, the sorted lists are
    all-gathered and merged, the replicated host model walks them; every
    rank's records equal the faithful restatement's.  Odd seeds add pod
    (anti-)affinity and inter-pod priority terms (replicated count tables,
    the inter-pod min / max reduced over the shards)."""
    feats = ("selector", "taints", "init", "bestEffort") + (("podaffinity",) if seed % 2 else ())
    c = kbgen_mod.gen_preempt(3100 + seed, n_nodes=6 + seed * 2, n_queues=1 + seed % 3, n_run_jobs=6 + seed % 5,
                              n_pend_jobs=3 + seed % 3, max_tasks=2 + seed % 4, features=feats)
    _shard_case(oracle_mod, tmp_path, c, 2 + seed % 2, actions=EVICT_ACTIONS[seed % len(EVICT_ACTIONS)])


@pytest.mark.gpu
def test_sharded_c5_scaled_gpu(engine, oracle_mod, kbgen_mod, tmp_path):
    """C5's what-if action sequence on 2 shards at a size the faithful
    restatement finishes in seconds."""
    p = str(tmp_path / "c5s.kbs")
    kbgen_mod.gen_c5(p, seed=kbgen_mod.BASE_SEED + 5, n_nodes=90, n_pending=80, best_effort=8)
    acts = "reclaim, allocate, backfill, preempt"
    exp = oracle_mod.ref_allocate(p, actions=acts).as_list()
    assert any(k == 128 for _, _, k in exp)
    res = _run_ranks("shard_worker.py", 2, tmp_path, lambda r, init, out: [p, str(r), "2", init, out, acts, "1"],
                     timeout=240)
    for r in range(2):
        assert [(a, b, {1: 4, 2: 8, 3: 128}[k]) for a, b, k in res[r]["log"]] == exp, f"rank {r}"


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(6))
def test_sharded_carry_gpu(engine, kbgen_mod, tmp_path, seed):
    """Session carry-over on shards: every rank carries its replicated host
    model and uploads its own rows; the second session's log equals the
    one-GPU session's after the same carry (tests/test_gpu_carry.py pins that
    one against the faithful oracle)."""
    from test_gpu_carry import NO_POD_AFFINITY
    c = kbgen_mod.gen_random(2900 + seed, n_nodes=6 + seed * 3, n_jobs=7, max_tasks=5, features=NO_POD_AFFINITY)
    p = str(tmp_path / "s.kbs")
    c.write(p)
    acts = "allocate, backfill"
    with engine.Session(p) as s:
        s.run_actions(acts)
        st = s.table("pod_status")
        dels = [int(i) for i in np.nonzero((st == 16) | (st == 64))[0][:4]]  # bound / running pods leave
        s.carry_events(dels, [1] * len(dels))  # KBHIP_EV_DELETE
        pod, node, kind = s.run_actions(acts)
    exp = [[int(a), int(b), int(k)] for a, b, k in zip(pod, node, kind)]
    world = 2 + seed % 2
    res = _run_ranks("shard_worker.py", world, tmp_path,
                     lambda r, init, out: [p, str(r), str(world), init, out, acts, "1"], timeout=240,
                     env={"KBHIP_TEST_CARRY": ",".join(map(str, dels))})
    for r in range(world):
        assert res[r]["log"] == exp, f"rank {r}"


@pytest.mark.gpu
@pytest.mark.parametrize("exchange", ["host", "mailbox", "mailbox_serial"])
def test_sharded_c4_scaled_gpu(engine, kbgen_mod, tmp_path, exchange):
    """C4 shape at 20k nodes (2 and 3 ranks sharing the GPU): the shard logs
    and close messages equal the one-GPU session's, and every batched pop is
    exactly one exchange (one all-gather over gloo, or one mailbox round)."""
    p = str(tmp_path / "c4s.kbs")
    kbgen_mod.gen_c4(p, n_nodes=20000, n_pending=60000)
    with engine.Session(p) as s:
        pod, node, kind = s.allocate(cap=1 << 20)
        st1 = s.stats()
        close1 = s.gang_unschedulable()
    exp = [(int(a), int(b), 4 if k == 1 else 8) for a, b, k in zip(pod, node, kind)]
    assert st1["batched_pops"] == st1["sweeps"] > 1000
    for world in (2, 3):
        res = _run_ranks("shard_worker.py", world, tmp_path,
                         lambda r, init, out: [p, str(r), str(world), init, out, "allocate", "1"], timeout=240,
                         env={"KBHIP_TEST_EXCHANGE": exchange})
        for r in range(world):
            got = [(a, b, 4 if k == 1 else 8) for a, b, k in res[r]["log"]]
            assert got == exp, f"world {world} rank {r}"
            assert res[r]["close"] == close1, f"world {world} rank {r}"
            assert res[r]["batched_pops"] == st1["batched_pops"]
            assert res[r]["collectives"] == res[r]["batched_pops"]  # one all-gather per pop, nothing else


@pytest.mark.gpu
@pytest.mark.parametrize("exchange", ["host", "mailbox"])
def test_sharded_c4_full_size_gpu(engine, kbgen_mod, tmp_path, exchange):
    """BASELINE.json's sharded config at full size: the bench snapshot (100k
    nodes x 1M pods) on 2 ranks sharing the GPU; every rank's placement log
    equals the pinned digest of the CPU oracle's (tests/golden/fullsize.json,
    as tests/test_gpu_fullsize.py checks the one-GPU session) and every
    batched pop is exactly one exchange."""
    import hashlib
    gold = json.load(open(os.path.join(HERE, "golden", "fullsize.json")))["c4"]
    p = str(tmp_path / "c4.kbs")
    kbgen_mod.gen_c4(p)
    with open(p, "rb") as f:
        assert hashlib.sha256(f.read()).hexdigest() == gold["snap_sha256"]
    res = _run_ranks("shard_worker.py", 2, tmp_path,
                     lambda r, init, out: [p, str(r), "2", init, out, "allocate", "1"], timeout=420,
                     env={"KBHIP_TEST_EXCHANGE": exchange, "KBHIP_TEST_DIGEST_ONLY": "1"})
    for r in range(2):
        assert res[r]["n"] == gold["n"]
        assert [[a, b, 4 if k == 1 else 8] for a, b, k in res[r]["head"]] == gold["head"][:64]
        assert res[r]["log_sha256"] == gold["log_sha256"], f"rank {r}"
        assert res[r]["batched_pops"] > 20000
        assert res[r]["collectives"] == res[r]["batched_pops"]


@pytest.mark.gpu
def test_sharded_c3_small_gpu(engine, oracle_mod, kbgen_mod, tmp_path):
    c = kbgen_mod.gen_c3(n_nodes=90, n_pending=400)
    _shard_case(oracle_mod, tmp_path, c, 2)


@pytest.mark.gpu
def test_sharded_rccl_two_devices(engine, oracle_mod, kbgen_mod, tmp_path):
    """The RCCL exchange (ncclAllGather / ncclAllReduce on the session stream):
    two ranks on two devices.  Skipped on a one-GPU box (RCCL does not run two
    ranks on one device)."""
    if engine.device_count() < 2:
        pytest.skip("needs two gfx950 devices")
    c = kbgen_mod.gen_random(2600, n_nodes=40, n_jobs=10, max_tasks=8, best_effort_p=0.2)
    p = str(tmp_path / "r.kbs")
    c.write(p)
    exp = oracle_mod.ref_allocate(p, actions="allocate, backfill").as_list()
    res = _run_ranks("rccl_worker.py", 2, tmp_path, lambda r, init, out: [p, str(r), "2", init, out], timeout=300)
    for r in range(2):
        assert [(a, b, 4 if k == 1 else 8) for a, b, k in res[r]["log"]] == exp


@pytest.mark.gpu
def test_rccl_communicator_pooled_across_sessions(engine, oracle_mod, kbgen_mod, tmp_path):
    """kbhip_shard_connect_rccl on one device (world 1, the only RCCL
    communicator a one-GPU box can form): the first session pays
    ncclCommInitRank, later sessions with the same unique id reuse the pooled
    communicator (return 1), and every session schedules like the oracle."""
    c = kbgen_mod.gen_random(2610, n_nodes=12, n_jobs=8, max_tasks=6)
    p = str(tmp_path / "w1.kbs")
    c.write(p)
    exp = oracle_mod.ref_allocate(p).as_list()
    uid = engine.ShardedSession.rccl_unique_id()
    buf = open(p, "rb").read()
    reused = []
    for _ in range(3):
        s = engine.ShardedSession(buf, 0, 0, 1)
        reused.append(s.connect_rccl(uid))
        pod, node, kind = s.allocate()
        s.close()
        assert [(int(a), int(b), 4 if k == 1 else 8) for a, b, k in zip(pod, node, kind)] == exp
    assert reused == [0, 1, 1]


@pytest.mark.gpu
def test_rccl_communicator_dropped_after_failure(engine, oracle_mod, kbgen_mod, tmp_path):
    """A session whose ABI call fails while its RCCL communicator is connected
    (here: kbhip_place_job with a task that is not pending) aborts the
    communicator at close instead of pooling it.  Its unique id is then
    refused (a second bootstrap on it would hang); the ranks connect with a
    new id — a new communicator (comm_reused 0), reused by the next session —
    and schedule like the oracle."""
    c = kbgen_mod.gen_random(2620, n_nodes=10, n_jobs=6, max_tasks=5)
    p = str(tmp_path / "w1f.kbs")
    c.write(p)
    exp = oracle_mod.ref_allocate(p).as_list()
    uid = engine.ShardedSession.rccl_unique_id()
    buf = open(p, "rb").read()
    s = engine.ShardedSession(buf, 0, 0, 1)
    assert s.connect_rccl(uid) == 0
    with pytest.raises(engine.KbhipError):
        s.place_job([-5], 1, 1, 0)
    s.close()
    s = engine.ShardedSession(buf, 0, 0, 1)
    with pytest.raises(engine.KbhipError, match="aborted"):
        s.connect_rccl(uid)
    s.close()
    uid2 = engine.ShardedSession.rccl_unique_id()
    reused = []
    for _ in range(2):
        s = engine.ShardedSession(buf, 0, 0, 1)
        reused.append(s.connect_rccl(uid2))
        pod, node, kind = s.allocate()
        s.close()
        assert [(int(a), int(b), 4 if k == 1 else 8) for a, b, k in zip(pod, node, kind)] == exp
    assert reused == [0, 1]


def test_mailbox_queue_rule(engine_lib):
    """kbhip_shard_mailbox_fits: the rule kbhip_shard_connect_mailbox applies to
    rank threads of one process sharing a device (each session has 3 streams;
    one process per GPU always fits)."""
    fits = engine_lib.kbhip_shard_mailbox_fits
    assert fits(1, 1) == 1 and fits(1, 4) == 1  # one rank per process and device
    assert fits(2, 4) == 0  # the r04 rank-thread rehearsal under the default 4 queues
    assert fits(2, 8) == 1 and fits(2, 7) == 0 and fits(2, 6) == 0  # two queues of headroom
    assert fits(8, 26) == 1 and fits(8, 24) == 0


@pytest.mark.gpu
def test_mailbox_refuses_shared_hw_queues(engine, oracle_mod, kbgen_mod, tmp_path):
    """Two shard ranks as threads of this process on one GPU, with the default
    hardware queues: kbhip_shard_connect_mailbox refuses on both ranks
    (KBHIP_EUNSUPPORTED, after the handle all-gather) instead of letting their
    mailbox kernels share a queue and wait on each other."""
    import threading
    kb = engine
    q = int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4)
    if kb.lib().kbhip_shard_mailbox_fits(2, q):
        pytest.skip(f"GPU_MAX_HW_QUEUES={q} fits two in-process ranks")
    c = kbgen_mod.gen_c3(n_nodes=90, n_pending=200)
    p = str(tmp_path / "c.kbs")
    c.write(p)
    buf = open(p, "rb").read()
    bar, slots, errs = threading.Barrier(2), [None, None], [None, None]

    def gather(rank):
        def g(send, recv):
            slots[rank] = bytes(send)
            bar.wait()
            recv[:] = np.frombuffer(b"".join(slots), np.uint8)
            bar.wait()
        return g

    red = [None, None]

    def reduce(rank):  # an in-process all-reduce over the two rank threads
        def f(vals, op):
            red[rank] = vals.copy()
            bar.wait()
            a, b = red[0], red[1]
            if op == kb.RED_MAX_U64:
                out = np.maximum(a, b)
            elif op == kb.RED_MIN_I64:
                out = np.minimum(a.view(np.int64), b.view(np.int64)).view(vals.dtype)
            elif op == kb.RED_SUM_I64:
                out = (a.view(np.int64) + b.view(np.int64)).view(vals.dtype)
            else:
                out = np.maximum(a.view(np.int64), b.view(np.int64)).view(vals.dtype)
            bar.wait()
            vals[:] = out
        return f

    logs = [None, None]

    def run(rank):
        s = kb.ShardedSession(buf, 0, rank, 2)
        try:
            try:
                s.connect_mailbox(gather(rank))
            except kb.KbhipError as e:
                errs[rank] = str(e)
            # the refusal left the session unconnected: the host exchange works after it
            s.connect_host(reduce(rank), gather(rank))
            pod, node, kind = s.allocate()
            logs[rank] = [(int(a), int(b), 4 if k == 1 else 8) for a, b, k in zip(pod, node, kind)]
        finally:
            s.close()

    th = [threading.Thread(target=run, args=(r,)) for r in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert all(e is not None and "error -3" in e and "hardware queues" in e for e in errs), errs
    assert logs[0] is not None and logs[0] == logs[1] == oracle_mod.ref_allocate(p).as_list()
