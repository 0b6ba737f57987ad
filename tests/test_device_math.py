"""CPU check of the device arithmetic (no GPU).

The kernels' per-node functions (kube-batch-1_amd/csrc/kbhip_eval.h:
predicates, LR/BRA/NA/inter-pod scores, fit, selection key, node-row and
pod-affinity commits, the GetAccessibleResource visit mutation) are
__host__ __device__.  kbhip_debug_replay runs them on the host over an
encode-only session's tables along the hoisted oracle's decision sequence;
before every task the oracle tried, the engine's selection key of every node
must equal the key the oracle's evaluation implies, and the oracle's decision
must be the argmax.  The device path end to end is tests/test_gpu_parity.py.
"""
import glob
import os

import numpy as np
import pytest

PIPELINED_ST = 8
ACTIONS = "allocate, backfill"


def check_keys(path, oracle_mod):
    import kbhip
    with kbhip.EncodedSnapshot(path) as enc:
        n_nodes = int(enc.table("dims")[0])
        tr = oracle_mod.fast_trace_affinity(path, n_nodes, cap_tasks=8192, actions=ACTIONS)
        kinds = np.where(tr["status"] == PIPELINED_ST, 2, 1).astype(np.uint8)
        keys = enc.replay(tr["pod"], tr["mode"], tr["node"], kinds)
    for i in range(len(tr["pod"])):
        bad = np.nonzero(keys[i] != tr["key"][i])[0]
        assert bad.size == 0, (f"step {i} (pod {tr['pod'][i]}, mode {tr['mode'][i]}): nodes {bad[:8]} "
                               f"engine {[hex(int(x)) for x in keys[i][bad[:4]]]} "
                               f"oracle {[hex(int(x)) for x in tr['key'][i][bad[:4]]]}")
        node = int(tr["node"][i])
        if node >= 0:
            assert int(np.argmax(keys[i])) == node
        else:
            assert n_nodes == 0 or keys[i].max() == 0
    return tr


TIERS = [None, [["drf", "proportion"]], [["gang"], ["predicates", "nodeorder"]],
         [["priority", "gang", "drf"], ["predicates", "proportion", "nodeorder", "nodeorder"]],
         [["priority", "gang"], ["predicates", "drf"]], [["gang"], ["nodeorder", "proportion"]]]


@pytest.mark.parametrize("seed", range(120))
def test_device_math_random(engine_lib, oracle_mod, kbgen_mod, tmp_path, seed):
    c = kbgen_mod.gen_random(5000 + seed, n_nodes=3 + seed % 15, n_jobs=3 + seed % 9, max_tasks=1 + seed % 7,
                             tiers=TIERS[seed % len(TIERS)], best_effort_p=0.2)
    if seed % 4 == 1:
        c.args = {"nodeorder": {"leastrequested.weight": "2", "balancedresource.weight": "3",
                                "nodeaffinity.weight": "-1", "podaffinity.weight": str(1 + seed % 3)}}
    if seed % 13 == 0:
        c.flags = {"gang": ["disableJobReady"], "predicates": ["disablePredicate"]}
    p = str(tmp_path / "m.kbs")
    c.write(p)
    check_keys(p, oracle_mod)


def test_device_math_c3_small(engine_lib, oracle_mod, kbgen_mod, tmp_path):
    c = kbgen_mod.gen_c3(n_nodes=150, n_pending=700)
    p = str(tmp_path / "c3.kbs")
    c.write(p)
    tr = check_keys(p, oracle_mod)
    assert (tr["node"] >= 0).sum() > 200


def test_device_math_c2_small(engine_lib, oracle_mod, kbgen_mod, tmp_path):
    p = str(tmp_path / "c2.kbs")
    kbgen_mod.gen_c2(p, n_nodes=80, n_pending=1200)
    tr = check_keys(p, oracle_mod)
    assert (tr["status"] == PIPELINED_ST).sum() >= 0 and (tr["node"] >= 0).sum() > 300


def test_device_math_golden(engine_lib, oracle_mod):
    files = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "*.kbs")))
    assert len(files) > 10
    for f in files:
        check_keys(f, oracle_mod)
