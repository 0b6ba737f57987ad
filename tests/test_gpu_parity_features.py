"""GPU parity of the features added after the first device path: pod
(anti-)affinity + inter-pod affinity priority (count tables), the backfill
action, C3.  Same bar as tests/test_gpu_parity.py: placement logs bit-equal to
the CPU oracle's, both device paths."""
import json
import os

import numpy as np
import pytest

from test_gpu_parity import GOLD, _engine_log, _oracle_log

pytestmark = pytest.mark.gpu


def _aff_golden_cases():
    with open(os.path.join(GOLD, "golden.json")) as f:
        g = json.load(f)
    return sorted(k for k in g if k.startswith("rndaff_"))


@pytest.mark.parametrize("case", _aff_golden_cases())
@pytest.mark.parametrize("batched", [True, False])
def test_golden_affinity_gpu(engine, oracle_mod, case, batched):
    path = os.path.join(GOLD, case + ".kbs")
    got, _ = _engine_log(engine, path, batched)
    assert got == _oracle_log(oracle_mod, path)


@pytest.mark.parametrize("seed", range(60))
def test_random_pod_affinity_gpu(engine, oracle_mod, kbgen_mod, tmp_path, seed):
    """Every feature incl. pod (anti-)affinity and inter-pod affinity priority."""
    tiers = [None, [["drf", "proportion"]], [["gang"], ["predicates", "nodeorder"]],
             [["priority", "gang", "drf"], ["predicates", "proportion", "nodeorder", "nodeorder"]]][seed % 4]
    c = kbgen_mod.gen_random(900 + seed, n_nodes=4 + seed % 12, n_jobs=4 + seed % 8, max_tasks=1 + seed % 8,
                             tiers=tiers)
    if seed % 3 == 0:
        c.args = {"nodeorder": {"leastrequested.weight": "2", "podaffinity.weight": str(1 + seed % 4)}}
    p = str(tmp_path / "a.kbs")
    c.write(p)
    exp = _oracle_log(oracle_mod, p)
    for batched in (True, False):
        got, _ = _engine_log(engine, p, batched)
        assert got == exp, f"batched={batched}"


@pytest.mark.parametrize("seed", range(30))
def test_allocate_then_backfill_gpu(engine, oracle_mod, kbgen_mod, tmp_path, seed):
    """actions "allocate, backfill": BestEffort tasks first-fit after allocate."""
    tiers = [None, [["drf", "proportion"]], [["gang"], ["predicates", "nodeorder"]]][seed % 3]
    c = kbgen_mod.gen_random(1500 + seed, n_nodes=3 + seed % 12, n_jobs=3 + seed % 8, max_tasks=1 + seed % 7,
                             tiers=tiers, best_effort_p=0.35)
    p = str(tmp_path / "bf.kbs")
    c.write(p)
    acts = "allocate, backfill"
    exp = oracle_mod.ref_allocate(p, actions=acts).as_list()
    for batched in (True, False):
        with engine.Session(p) as s:
            s.set_option("batched", 1 if batched else 0)
            pod, node, kind = s.run_actions(acts)
        got = [(int(a), int(b), 4 if k == 1 else 8) for a, b, k in zip(pod, node, kind)]
        assert got == exp, f"batched={batched}"


def test_c3_scaled(engine, oracle_mod, kbgen_mod, tmp_path):
    """C3 shape (zone anti-affinity, selectors, taints, 8 queues) at 2k nodes x 8k pods."""
    c = kbgen_mod.gen_c3(n_nodes=2000, n_pending=8000)
    p = str(tmp_path / "c3.kbs")
    c.write(p)
    exp = _oracle_log(oracle_mod, p, fast=True)
    got, st = _engine_log(engine, p, True)
    assert len(got) > 1000
    assert got == exp
    assert st["batched_pops"] > 0




def _decode_max(k):
    k = int(k)
    if not k:
        return -1, 1
    return 0x7fffffff - ((k >> 1) & 0x7fffffff), 2 if k & 1 else 1


@pytest.mark.parametrize("seed", range(24))
def test_device_keys_match_host_replay(engine, kbgen_mod, tmp_path, seed):
    """Every per-task sweep's per-node keys and raw inter-pod counts on the
    device equal the host replay of the same __host__ __device__ arithmetic
    (kbhip_debug_replay) along the device's own decisions.  Catches device-only
    divergence (codegen, stale tables) independently of the oracle."""
    tiers = [None, [["gang"], ["predicates", "nodeorder"]],
             [["priority", "gang", "drf"], ["predicates", "proportion", "nodeorder", "nodeorder"]]][seed % 3]
    c = kbgen_mod.gen_random(7000 + seed, n_nodes=4 + seed % 13, n_jobs=4 + seed % 8, max_tasks=1 + seed % 8,
                             tiers=tiers)
    if seed % 2 == 0:
        c.args = {"nodeorder": {"podaffinity.weight": str(1 + seed % 4)}}
    p = str(tmp_path / "k.kbs")
    c.write(p)
    with engine.Session(p) as s:
        s.set_option("batched", 0)
        s.set_option("debug_keys", 1)
        s.allocate()
        pods, rows = s.debug_keys()
    with engine.EncodedSnapshot(p) as enc:
        n = int(enc.table("dims")[0])
        npad = (rows.shape[1] - 4) // 2 if len(pods) else n
        dec = [_decode_max(r[2 * npad + 3]) for r in rows]
        nodes = np.array([d[0] for d in dec], np.int32)
        kinds = np.array([d[1] for d in dec], np.uint8)
        keys = enc.replay(pods, np.zeros(len(pods), np.int32), nodes, kinds)
    for i in range(len(pods)):
        assert np.array_equal(rows[i][:n], keys[i]), f"sweep {i} (pod {pods[i]}): device keys differ from the replay"
