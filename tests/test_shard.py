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


def _run_ranks(script, world, tmp_path, extra, timeout=300):
    init = str(tmp_path / "init")
    outs = [str(tmp_path / f"out{r}.json") for r in range(world)]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, script)] + extra(r, init, outs[r]), env=env)
             for r in range(world)]
    try:
        rcs = [p.wait(timeout=timeout) for p in procs]
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


def test_shard_ranges_partition(engine_lib):
    import kbhip
    for n in (0, 1, 7, 100, 100_000):
        for world in (1, 2, 3, 8):
            rs = [kbhip.shard_range(n, r, world) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))
            assert all(hi - lo in (n // world, n // world + 1) for lo, hi in rs)


def _shard_case(oracle_mod, tmp_path, c, world, actions="allocate"):
    p = str(tmp_path / "s.kbs")
    c.write(p)
    exp = oracle_mod.ref_allocate(p, actions=actions).as_list()
    res = _run_ranks("shard_worker.py", world, tmp_path,
                     lambda r, init, out: [p, str(r), str(world), init, out, actions], timeout=600)
    n_nodes = len(c.nodes)
    import kbhip
    for r in range(world):
        lo, hi = kbhip.shard_range(n_nodes, r, world)
        assert res[r]["info"] == [r, world, lo, hi]
        got = [(a, b, 4 if k == 1 else 8) for a, b, k in res[r]["log"]]
        assert got == exp, f"rank {r}"


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(6))
def test_sharded_random_gpu(engine, oracle_mod, kbgen_mod, tmp_path, seed):
    """2 or 3 ranks on one GPU, every feature (pod affinity, backfill, ports...)."""
    c = kbgen_mod.gen_random(2200 + seed, n_nodes=6 + seed * 3, n_jobs=6, max_tasks=5, best_effort_p=0.2)
    _shard_case(oracle_mod, tmp_path, c, 2 + seed % 2, actions="allocate, backfill")


@pytest.mark.gpu
def test_sharded_c3_small_gpu(engine, oracle_mod, kbgen_mod, tmp_path):
    c = kbgen_mod.gen_c3(n_nodes=90, n_pending=400)
    _shard_case(oracle_mod, tmp_path, c, 2)
