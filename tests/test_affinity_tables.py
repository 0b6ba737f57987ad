"""CPU cross-check of the engine's pod (anti-)affinity tables (no device).

The engine compiles pod affinity into per-topology-domain count tables and
per-task programs (kube-batch-1_amd/csrc/kbhip_affinity.h) that the kernels
read (aff_pred / ipa_count / commit_aff in kbhip_kernels.hip).  Here the
tables come from an encode-only session (kbhip_debug_encode) and are replayed
in numpy along the hoisted oracle's decision sequence: before every task the
oracle tried, the table view of the pod-affinity predicate and of the raw
inter-pod affinity count must equal the oracle's per-node values; after every
placement the task's commit updates are applied as the kernel applies them.
The device path itself is checked end to end by tests/test_gpu_parity.py.
"""
import numpy as np
import pytest

ALLOCATED_ST, PIPELINED_ST = 4, 8


def replay(enc, tr):
    n_nodes, npad, _, _ = (int(x) for x in enc.table("dims"))
    dom = enc.table("aff_dom").reshape(-1, npad)[:, :n_nodes].astype(np.int64)
    cnt = enc.table("aff_cnt").astype(np.int64)
    scal = enc.table("aff_scalar").astype(np.int64)
    items = enc.table("aff_items")
    ca = enc.table("class_aff").reshape(-1, 16)
    pod_class = enc.table("pod_class")
    fallback = -1
    checked = 0
    for t in range(len(tr["pod"])):
        p = int(tr["pod"][t])
        (aff, pred_err, ea_off, ea_n, pa_sp, pa_cnt, pa_tot, pa_self, paa_sp, paa_cnt, ipa_off, ipa_n,
         upd_off, upd_n, _score_err, _) = (int(x) for x in ca[pod_class[p]])
        flags = int(tr["flags"][t])
        # --- predicate (aff_pred)
        if flags & 1:
            assert pred_err == 1, f"task {t}: oracle fails every node, engine class has no pred_err"
        else:
            ok = np.ones(n_nodes, bool)
            for i in range(ea_n):
                sp, off = items[ea_off + 2 * i], items[ea_off + 2 * i + 1]
                d = dom[sp]
                ok &= ~((d >= 0) & (cnt[off + np.maximum(d, 0)] > 0))
            if pa_sp >= 0:
                d = dom[pa_sp]
                match = (d >= 0) & (cnt[pa_cnt + np.maximum(d, 0)] > 0)
                ok &= match | bool(pa_self and scal[pa_tot] == 0)
            if paa_sp >= 0:
                d = dom[paa_sp]
                ok &= ~((d >= 0) & (cnt[paa_cnt + np.maximum(d, 0)] > 0))
            exp = tr["ok"][t].astype(bool)
            assert np.array_equal(ok, exp), f"task {t} (pod {p}): affinity predicate {ok.astype(int)} != {exp.astype(int)}"
        # --- inter-pod affinity raw count (ipa_count) and its normalisation range
        if not flags & 2:
            raw = np.zeros(n_nodes, np.int64)
            for i in range(ipa_n):
                sp, off, sess, w = (int(x) for x in items[ipa_off + 4 * i: ipa_off + 4 * i + 4])
                d = dom[sp]
                x = np.where(d >= 0, cnt[off + np.maximum(d, 0)], 0)
                if fallback >= 0:
                    x = x + np.where((d >= 0) & (d == dom[sp, fallback]), scal[sess], 0)
                raw += w * x
            assert np.array_equal(raw.astype(np.float64), tr["raw"][t]), \
                f"task {t} (pod {p}): ipa raw {raw} != {tr['raw'][t]}"
            if flags & 4:
                lo, hi = min(0, int(raw.min())), max(0, int(raw.max()))
                assert (lo, hi) == tuple(tr["lohi"][t]), f"task {t}: ipa range"
        checked += 1
        # --- commit (commit_aff + fallback node)
        node = int(tr["node"][t])
        if node < 0:
            continue
        kind = 2 if int(tr["status"][t]) == PIPELINED_ST else 1
        for i in range(upd_n):
            typ, sp, off = (int(x) for x in items[upd_off + 3 * i: upd_off + 3 * i + 3])
            if typ == 0:
                if kind == 1 and dom[sp, node] >= 0:
                    cnt[off + dom[sp, node]] += 1
            elif typ == 1:
                if kind == 1:
                    scal[off] += 1
            else:
                scal[off] += 1
        if aff == 0:
            assert upd_n == 0
        if fallback < 0 or node < fallback:
            fallback = node
    return checked


def _check(engine_lib, oracle_mod, path):
    import kbhip
    with kbhip.EncodedSnapshot(path) as enc:
        n_nodes = int(enc.table("dims")[0])
        tr = oracle_mod.fast_trace_affinity(path, n_nodes)
        assert replay(enc, tr) == len(tr["pod"])
        return tr


TIERS = [None, [["drf", "proportion"]], [["gang"], ["predicates", "nodeorder"]],
         [["priority", "gang", "drf"], ["predicates", "proportion", "nodeorder", "nodeorder"]],
         [["priority", "gang"], ["predicates", "drf"]], [["gang"], ["nodeorder", "proportion"]]]


@pytest.mark.parametrize("seed", range(80))
def test_affinity_tables_random(engine_lib, oracle_mod, kbgen_mod, tmp_path, seed):
    c = kbgen_mod.gen_random(3000 + seed, n_nodes=3 + seed % 14, n_jobs=3 + seed % 9, max_tasks=1 + seed % 7,
                             tiers=TIERS[seed % len(TIERS)])
    if seed % 4 == 1:
        c.args = {"nodeorder": {"podaffinity.weight": str(1 + seed % 5)}}
    p = str(tmp_path / "a.kbs")
    c.write(p)
    _check(engine_lib, oracle_mod, p)


def test_affinity_tables_c3_small(engine_lib, oracle_mod, kbgen_mod, tmp_path):
    c = kbgen_mod.gen_c3(n_nodes=120, n_pending=600)
    p = str(tmp_path / "c3.kbs")
    c.write(p)
    tr = _check(engine_lib, oracle_mod, p)
    assert (tr["node"] >= 0).sum() > 100
    assert not tr["ok"].all()  # the zone anti-affinity does filter nodes


def test_affinity_tables_golden(engine_lib, oracle_mod):
    import glob
    import os
    files = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "rndaff_*.kbs")))
    assert files
    for f in files:
        _check(engine_lib, oracle_mod, f)
