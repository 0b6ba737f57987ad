"""FitError / NodesFitDelta: the gang plugin's
OnSessionClose messages after allocate — "<m>/<n> tasks in gang
unschedulable: <JobInfo.FitError>" for every job left not Ready — equal the
oracle's (kbref: allocate.go:124-126 / 164-167, job_info.go:343-372,
gang.go:166-187), on every device path: batched (in-kernel histogram, with and
without overlapped pops), per task, and the synchronous fallback (placement
(pops that place every task and stay not Ready), for every class including
those with inter-pod affinity priority terms.  Node-array shards are checked
in tests/test_shard.py."""
import pytest

from test_gpu_parity import NO_POD_AFFINITY

PATHS = [dict(), dict(overlap=0), dict(overlap=2), dict(batched=0), dict(speculate=0), dict(overlap=0, speculate=0)]


def _engine_close(engine, path, **opts):
    with engine.Session(path) as s:
        for k, v in opts.items():
            s.set_option(k, v)
        s.allocate()
        return s.gang_unschedulable(), s.stats()


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(40))
def test_fit_error_random_gpu(engine, oracle_mod, kbgen_mod, tmp_path, seed):
    tiers = [None, [["priority", "gang"], ["drf", "predicates", "proportion", "nodeorder"]],
             [["gang"], ["predicates", "nodeorder"]]][seed % 3]
    c = kbgen_mod.gen_random(5100 + seed, n_nodes=3 + seed % 10, n_jobs=5 + seed % 9, max_tasks=2 + seed % 9,
                             features=NO_POD_AFFINITY, tiers=tiers)
    p = str(tmp_path / "f.kbs")
    c.write(p)
    exp = oracle_mod.ref_gang_close(p)
    for opts in PATHS:
        got, st = _engine_close(engine, p, **opts)
        assert got == exp, opts


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(40))
def test_fit_error_full_features_gpu(engine, oracle_mod, kbgen_mod, tmp_path, seed):
    """Every feature, pod (anti-)affinity and inter-pod priority classes too
    (per-task path: in-kernel counts; pops that leave their job not Ready:
    the recount with the priority's min / max prepass on the task's state)."""
    c = kbgen_mod.gen_random(5300 + seed, n_nodes=4 + seed % 8, n_jobs=5 + seed % 7, max_tasks=2 + seed % 7)
    p = str(tmp_path / "ff.kbs")
    c.write(p)
    exp = oracle_mod.ref_gang_close(p)
    for opts in (dict(), dict(batched=0)):
        got, _ = _engine_close(engine, p, **opts)
        assert got == exp, opts


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(16))
def test_fit_error_interpod_priority_gpu(engine, oracle_mod, kbgen_mod, tmp_path, seed):
    """Sessions where most pending pods carry preferred pod (anti-)affinity
    terms (inter-pod priority classes) and gangs that cannot become Ready:
    the close messages come from walks ordered by the normalised inter-pod
    score."""
    c = kbgen_mod.gen_random(5500 + seed, n_nodes=3 + seed % 6, n_jobs=6 + seed % 5, max_tasks=3 + seed % 6,
                             features=("labels", "running", "podaffinity", "init"))
    for j in c.jobs:  # gangs larger than their pods: every pop ends not Ready
        j.min_member = j.min_member + 2
    p = str(tmp_path / "ip.kbs")
    c.write(p)
    exp = oracle_mod.ref_gang_close(p)
    assert exp
    for opts in (dict(), dict(batched=0)):
        got, _ = _engine_close(engine, p, **opts)
        assert got == exp, opts


@pytest.mark.gpu
def test_fit_error_c2_gpu(engine, kbgen_mod, tmp_path):
    """C2 at full size: the in-kernel histograms of the overlapped and the
    plain batched kernels equal the per-task kernel's."""
    p = str(tmp_path / "c2f.kbs")
    kbgen_mod.gen_c2(p)
    a, sa = _engine_close(engine, p)
    b, _ = _engine_close(engine, p, overlap=0)
    c, _ = _engine_close(engine, p, batched=0)
    assert sa["unassigned_pops"] > 0
    assert a == b == c
    assert any(not m.endswith("0 nodes are available") for m in a.values())


@pytest.mark.gpu
def test_fit_error_known_answer_gpu(engine, kbgen_mod, tmp_path):
    """The hand-derived case of tests/test_oracle.py on every device path."""
    c = kbgen_mod.Cluster()
    c.add_queue("default", 1)
    for i in range(2):
        c.add_node(f"n{i}", 2000, 4 * kbgen_mod.GI, 0)
    c.add_job("ns", "g", "default", min_member=5)
    for k in range(5):
        c.add_pod("ns", f"g-{k}", uid=f"u{k}", group="g", containers=[kbgen_mod.res(1000, kbgen_mod.GI)])
    p = str(tmp_path / "ka.kbs")
    c.write(p)
    for opts in PATHS:
        got, _ = _engine_close(engine, p, **opts)
        assert got == {"ns/g": "1/5 tasks in gang unschedulable: 0/2 nodes are available, 2 insufficient cpu."}, opts


@pytest.mark.gpu
def test_gang_close_backfilled_gpu(engine, oracle_mod, tmp_path):
    """The PodGroupBackfilled case (gang.go:189-199) on every device path."""
    from test_oracle import _backfill_gang_cluster
    p = str(tmp_path / "bf.kbs")
    _backfill_gang_cluster().write(p)
    exp = oracle_mod.ref_gang_close(p)
    assert exp["ns/g"] == "Backfilled"
    for opts in PATHS:
        got, _ = _engine_close(engine, p, **opts)
        assert got == exp, opts
