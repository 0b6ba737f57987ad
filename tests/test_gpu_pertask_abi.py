"""The SURVEY §8(b) per-task entry points against the faithful oracle.

* kbhip_first_fit — backfill.go:51-65's node loop for given tasks
  (lowest-index node passing PredicateFn, then Session.Allocate): driven with
  the backfill action's own task list it must reproduce the oracle's backfill
  log; on arbitrary pending tasks the chosen node is the lowest index whose
  kbhip_sweep_scores key is non-zero.
* kbhip_sweep_scores — preempt.go:270-287's PredicateFn + NodeOrderFn sweep:
  the per-node packed keys equal kbref's (ref_sweep_scores) for every pending
  task, before and after an allocate action.
"""
import numpy as np
import pytest

from test_gpu_parity import NO_POD_AFFINITY

pytestmark = pytest.mark.gpu


class _variant:
    """sweep_variant is process-wide: set it for a block, back to 0 after."""

    def __init__(self, s, v):
        self.s, self.v = s, v

    def __enter__(self):
        self.s.set_option("sweep_variant", self.v)

    def __exit__(self, *a):
        self.s.set_option("sweep_variant", 0)


def _pending(c_path, oracle_mod):
    import kbhip
    enc = kbhip.EncodedSnapshot(c_path)
    cls = enc.table("pod_class")
    enc.close()
    return [int(i) for i in np.nonzero(cls >= 0)[0]]


@pytest.mark.parametrize("variant", [0, 4, 6])
@pytest.mark.parametrize("seed", range(16))
def test_sweep_scores_vs_oracle(engine, oracle_mod, kbgen_mod, tmp_path, seed, variant):
    """variant: option sweep_variant (0 one node per thread, 4 / 6 the
    prefetching grid of k_score_sweep_gs)."""
    feats = NO_POD_AFFINITY if seed % 2 else None
    kw = {} if feats is None else {"features": feats}
    c = kbgen_mod.gen_random(7100 + seed, n_nodes=5 + seed % 9, n_jobs=4 + seed % 5, max_tasks=1 + seed % 5, **kw)
    p = str(tmp_path / "s.kbs")
    c.write(p)
    n_nodes = len(c.nodes)
    pend = _pending(p, oracle_mod)
    assert pend
    for actions in ("", "allocate"):
        with engine.Session(p) as s, _variant(s, variant):
            todo = pend
            if actions:
                s.allocate()
                st = s.table("pod_status")
                todo = [q for q in pend if st[q] == 1]  # still Pending
            for pod in todo[:6]:
                n_exp, k_exp = oracle_mod.ref_sweep_scores(p, pod, n_nodes, actions)
                n_got, k_got = s.sweep_scores(pod, n_nodes)
                assert n_got == n_exp
                assert np.array_equal(k_got, k_exp), (actions, pod)


@pytest.mark.parametrize("seed", range(12))
def test_first_fit_is_backfill(engine, oracle_mod, kbgen_mod, tmp_path, seed):
    """first_fit over the backfill action's candidate list (Pending tasks with
    an empty InitResreq, jobs and tasks in UID order) = the backfill action."""
    c = kbgen_mod.gen_random(7300 + seed, n_nodes=3 + seed % 6, n_jobs=4 + seed % 5, max_tasks=2 + seed % 4,
                             features=NO_POD_AFFINITY)
    p = str(tmp_path / "b.kbs")
    c.write(p)
    exp = oracle_mod.ref_allocate(p, actions="allocate, backfill").as_list()
    with engine.Session(p) as s:
        pod_a, node_a, kind_a = s.allocate()
        # the backfill candidates: pending (after allocate) best-effort tasks, job order then task order
        status = s.table("pod_status")
        req = oracle_mod.ref_task_requests(p, len(status))
        cls = s.table("pod_class")
        # backfill.go:44-46 in the pinned order: jobs by UID (a pod without a
        # PodGroup is its own job, UID = pod UID), tasks by UID (= pod index)
        pods = sorted(c.pods, key=lambda q: q.uid)
        key = []
        for i, q in enumerate(pods):
            if status[i] == 1 and cls[i] >= 0 and (req[i, 3:] < [10, 10 * 2 ** 20, 10]).all():
                key.append((f"{q.ns}/{q.group}" if q.group is not None else q.uid, i))
        cand = [i for _, i in sorted(key)]
        nodes = s.first_fit(cand)
    got = [(int(a), int(b), 4 if k == 1 else 8) for a, b, k in zip(pod_a, node_a, kind_a)]
    got += [(i, int(n), 4) for i, n in zip(cand, nodes) if n >= 0]
    assert got == exp


@pytest.mark.parametrize("seed", range(8))
def test_first_fit_any_tasks(engine, kbgen_mod, tmp_path, seed):
    """On arbitrary pending tasks: each goes to the lowest-index node whose
    sweep key (PredicateFn + NodeOrderFn) is non-zero on the state it sees."""
    c = kbgen_mod.gen_random(7500 + seed, n_nodes=4 + seed % 5, n_jobs=3 + seed % 4, max_tasks=3,
                             features=NO_POD_AFFINITY, tiers=[["priority"], ["predicates"]])
    p = str(tmp_path / "a.kbs")
    c.write(p)
    n_nodes = len(c.nodes)
    import kbhip
    enc = kbhip.EncodedSnapshot(p)
    pend = [int(i) for i in np.nonzero(enc.table("pod_class") >= 0)[0]]
    enc.close()
    with engine.Session(p) as s:
        for pod in pend:
            _, keys = s.sweep_scores(pod, n_nodes)
            ok = np.nonzero(keys)[0]
            exp = int(ok[0]) if ok.size else -1
            got = int(s.first_fit([pod])[0])
            assert got == exp, pod


@pytest.mark.parametrize("n_nodes", [70_000, 300_000])
def test_sweep_variants_agree_large(engine, kbgen_mod, tmp_path, n_nodes):
    """At sizes where the prefetching grid walks several nodes per thread (and
    the last walk is ragged): every kernel shape writes the same keys and the
    same passing count as the one-node-per-thread grid."""
    p = str(tmp_path / "big.kbs")
    kbgen_mod.gen_c4(p, n_nodes=n_nodes, n_pending=2000, running_per_node=1)
    pend = _pending(p, None)
    with engine.Session(p) as s:
        for pod in pend[::397][:5]:
            ref = s.sweep_scores(pod, n_nodes)
            assert ref[0] > 0
            for v in (1, 2, 3, 4, 5, 6):
                with _variant(s, v):
                    got = s.sweep_scores(pod, n_nodes)
                assert got[0] == ref[0] and np.array_equal(got[1], ref[1]), (pod, v)
