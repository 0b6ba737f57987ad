"""kbhip_session_carry_snapshot: a session carried
over to the scheduler cache's next snapshot after a mixed stream of informer
events — pod arrivals (new PodGroups with new task classes, pods joining
existing jobs, group-less pods, pods bound elsewhere), pod deletions (of a
PodGroup: gone; group-less: detached, event_handlers.go:119-165), pods
finishing, node updates (allocatable, unschedulable, labels), node add /
delete, PodGroup add / update (minMember, queue) — must schedule exactly like
the faithful oracle on that snapshot.  The snapshot is built by
tests/cachemodel.py, a restatement of the reference cache's handlers.

Shapes (seed % 4): 0 the fast path (node set, labels, taints, conf unchanged;
no pod affinity; plain arrivals); 1 node add / delete + label change (re-open
in place); 2 pod (anti-)affinity, arrivals with affinity terms (re-open); 3
arrivals with nodeSelector / host ports (re-open)."""
import numpy as np
import pytest

from cachemodel import CacheModel, clone, index_maps, snapshot_after_session

pytestmark = pytest.mark.gpu

STATUS = {1: 4, 2: 8, 3: 128}
RUNNING, BINDING, BOUND = 64, 16, 32
NO_POD_AFFINITY = ("labels", "taints", "ports", "init", "running", "releasing", "backfill", "selector",
                   "nodeaffinity", "unsched", "bestEffort")
ACTS = ["allocate", "allocate, backfill", "reclaim, allocate, backfill, preempt"]


def _events(M, rng, shape, seed, status_by_uid):
    c = M.c
    queues = sorted(q.name for q in c.queues)
    node_names = sorted(n.name for n in c.nodes if not n.name.startswith("aa-empty"))
    jobs = sorted(c.jobs, key=lambda j: j.uid)
    # arrivals: a new PodGroup with a new resource shape (a new task class)
    jn = f"arr{seed}"
    M.add_pod_group("default", jn, queues[int(rng.integers(len(queues)))], min_member=2, ts=10_000 + seed)
    for k in range(3):
        kw = {}
        if shape == 3:
            kw = {"node_selector": {"kubernetes.io/hostname": node_names[k % len(node_names)]}} if k == 0 else \
                {"containers": [{"cpu": 300 + 7 * seed, "mem": (3 << 20) + seed, "ports": [
                    {"port": 9000 + k, "ip": "", "proto": ""}]}]}
        if shape == 2:
            kw["labels"] = {"job": jn}
            kw["affinity"] = {"anti": {"required": [{"selector": {"ml": {"job": jn}},
                                                     "topology_key": "kubernetes.io/hostname"}]}}
        M.add_pod(ns="default", name=f"{jn}-{k}", uid=f"m{seed:03d}-{k}", group=jn, ts=10_000 + seed,
                  **({"containers": [{"cpu": 300 + 7 * seed, "mem": (3 << 20) + seed}]} if "containers" not in kw
                     else {}), **kw)
    # a pod joining an existing PodGroup, a group-less pending pod, a group-less pod bound elsewhere
    if jobs:
        j = jobs[int(rng.integers(len(jobs)))]
        M.add_pod(ns=j.ns, name=f"late{seed}", uid=f"b{seed:03d}-late", group=j.name, ts=20_000,
                  containers=[{"cpu": 200, "mem": 1 << 20}])
    M.add_pod(ns="default", name=f"solo{seed}", uid=f"k{seed:03d}-solo", group=None, ts=20_001,
              containers=[{"cpu": 150, "mem": 2 << 20}])
    M.add_pod(ns="default", name=f"ext{seed}", uid=f"e{seed:03d}-ext", group=None, ts=20_002,
              node=node_names[seed % len(node_names)], phase="Running", containers=[{"cpu": 100, "mem": 1 << 20}])
    # deletions, completions
    pods = sorted(c.pods, key=lambda q: q.uid)
    for q in pods:
        st = status_by_uid.get(q.uid)
        if st is None:
            continue
        r = rng.random()
        bound = st in (RUNNING, BINDING, BOUND)
        if q.group is None and (shape != 2 or not bound) and r < 0.5:
            M.delete_pod(q.uid)  # group-less: detached if bound, else unchanged
        elif q.group is not None and r < 0.08:
            M.delete_pod(q.uid)
        elif bound and r < 0.15:
            M.finish_pod(q.uid, "Succeeded" if rng.random() < 0.7 else "Failed")
    # node updates
    n0 = M.node(node_names[int(rng.integers(len(node_names)))])
    M.update_node(n0.name, cpu=n0.cpu + 2000)
    n1 = M.node(node_names[int(rng.integers(len(node_names)))])
    M.update_node(n1.name, unschedulable=not n1.unschedulable)
    if shape == 1:
        M.update_node(n0.name, labels=dict(n0.labels, tier=f"t{seed % 3}"))
        M.add_node(f"zz-new{seed}", 8000, 16 << 30, 0, 110, labels={"kubernetes.io/hostname": f"zz-new{seed}"})
        M.delete_node(f"aa-empty{seed}")
    # PodGroup updates
    if jobs:
        j = jobs[int(rng.integers(len(jobs)))]
        M.update_pod_group(j.uid, min_member=max(1, j.min_member - 1))
        j2 = jobs[int(rng.integers(len(jobs)))]
        M.update_pod_group(j2.uid, queue=queues[int(rng.integers(len(queues)))])


@pytest.mark.parametrize("seed", range(24))
def test_carry_snapshot_mixed_events(engine, oracle_mod, kbgen_mod, tmp_path, seed):
    rng = np.random.default_rng(9100 + seed)
    shape = seed % 4
    feats = tuple(NO_POD_AFFINITY) + (("podaffinity",) if shape == 2 else ())
    if seed % 2:
        c = kbgen_mod.gen_preempt(9200 + seed, n_nodes=4 + seed % 8, n_queues=1 + seed % 3, n_run_jobs=4 + seed % 7,
                                  n_pend_jobs=3 + seed % 5, max_tasks=2 + seed % 5,
                                  features=("selector", "taints", "ports", "init", "bestEffort")
                                  + (("podaffinity",) if shape == 2 else ()))
    else:
        c = kbgen_mod.gen_random(9300 + seed, n_nodes=4 + seed % 10, n_jobs=5 + seed % 8, max_tasks=2 + seed % 6,
                                 features=feats)
    if "default" not in {q.name for q in c.queues}:
        c.add_queue("default")
    if shape == 1:
        c.add_node(f"aa-empty{seed}", 4000, 8 << 30, 0, 110, unschedulable=True)  # deleted after the session
    acts = ACTS[seed % len(ACTS)]
    p1 = c.write(str(tmp_path / "s1.kbs"))
    old_pods = sorted(c.pods, key=lambda q: q.uid)
    old_nodes = sorted(n.name for n in c.nodes)
    with engine.Session(p1) as s:
        s.run_actions(acts)
        status, node = s.table("pod_status").copy(), s.table("pod_node").copy()
        c2 = snapshot_after_session(clone(c), status, node)
        M = CacheModel(c2)
        _events(M, rng, shape, seed, {q.uid: int(status[i]) for i, q in enumerate(old_pods)})
        op, on = index_maps(old_pods, old_nodes, c2)
        p2 = c2.write(str(tmp_path / "s2.kbs"))
        sent = s.carry_snapshot(p2, op, on)
        pod, nd, kind = s.run_actions(acts)
        n2 = len(c2.nodes)
        ns = s.read_nodes(n2)
        gang = s.gang_unschedulable()
    if shape == 0:
        assert sent >= 0, "the fast path re-opened the session"
    exp, ons = oracle_mod.ref_allocate(p2, actions=acts, with_nodes=True)
    assert [(int(a), int(b), STATUS[int(k)]) for a, b, k in zip(pod, nd, kind)] == exp.as_list()
    assert np.array_equal(ns.astype(np.float64), ons[:n2])
    assert gang == oracle_mod.ref_gang_close(p2, actions=acts)


def test_carry_snapshot_chain_equals_open(engine, kbgen_mod, tmp_path):
    """Three carried sessions in a row (plain arrivals each time, the fast
    path) schedule exactly like sessions opened from the same snapshots."""
    rng = np.random.default_rng(9400)
    c = kbgen_mod.gen_random(9401, n_nodes=12, n_jobs=10, max_tasks=6, features=NO_POD_AFFINITY)
    if "default" not in {q.name for q in c.queues}:
        c.add_queue("default")
    p = c.write(str(tmp_path / "s0.kbs"))
    with engine.Session(p) as s:
        for r in range(3):
            old_pods = sorted(c.pods, key=lambda q: q.uid)
            old_nodes = sorted(n.name for n in c.nodes)
            log = s.allocate()
            status, node = s.table("pod_status").copy(), s.table("pod_node").copy()
            with engine.Session(p) as f:  # the same snapshot opened fresh
                flog = f.allocate()
            assert all(np.array_equal(a, b) for a, b in zip(log, flog)), r
            c = snapshot_after_session(c, status, node)
            M = CacheModel(c)
            jn = f"wave{r}"
            M.add_pod_group("default", jn, sorted(q.name for q in c.queues)[0], min_member=1, ts=50_000 + r)
            for k in range(int(rng.integers(2, 6))):
                M.add_pod(ns="default", name=f"{jn}-{k}", uid=f"w{r}-{k:02d}", group=jn, ts=50_000 + r,
                          containers=[{"cpu": 250 * (k + 1), "mem": (k + 1) << 22}])
            op, on = index_maps(old_pods, old_nodes, c)
            p = c.write(str(tmp_path / f"s{r + 1}.kbs"))
            assert s.carry_snapshot(p, op, on) >= 0


def test_carry_snapshot_rejects_bad_maps(engine, kbgen_mod, tmp_path):
    c = kbgen_mod.gen_random(9501, n_nodes=4, n_jobs=4, max_tasks=3, features=NO_POD_AFFINITY)
    p = c.write(str(tmp_path / "s.kbs"))
    P, N = len(c.pods), len(c.nodes)
    with engine.Session(p) as s:
        s.allocate()
        for op, on in ((np.full(P, P, np.int32), np.arange(N, dtype=np.int32)),     # out of range
                       (np.zeros(P, np.int32), np.arange(N, dtype=np.int32)),       # one old pod twice
                       (np.arange(P, dtype=np.int32), np.full(N, -2, np.int32))):   # bad node index
            with pytest.raises(engine.KbhipError):
                s.carry_snapshot(p, op, on)
        assert s.carry_snapshot(p, np.arange(P, dtype=np.int32), np.arange(N, dtype=np.int32)) >= 0


@pytest.mark.parametrize("field", ["priority", "request", "backfill"])
def test_carry_snapshot_updated_pod_mapped(engine, kbgen_mod, tmp_path, field):
    """A pending pod updated between the sessions (updatePod rebuilds its
    TaskInfo, event_handlers.go:167-184) but mapped by UID: the carry must not
    keep its old priority, request or backfill flag — the next
    session schedules exactly like one opened fresh on the new snapshot."""
    c = kbgen_mod.gen_random(9601, n_nodes=10, n_jobs=10, max_tasks=6, features=NO_POD_AFFINITY)
    if "default" not in {q.name for q in c.queues}:
        c.add_queue("default")
    p1 = c.write(str(tmp_path / "s1.kbs"))
    old_pods = sorted(c.pods, key=lambda q: q.uid)
    old_nodes = sorted(n.name for n in c.nodes)
    with engine.Session(p1) as s:
        s.allocate()
        status, node = s.table("pod_status").copy(), s.table("pod_node").copy()
        c2 = snapshot_after_session(clone(c), status, node)
        pending = [q for q in sorted(c2.pods, key=lambda q: q.uid) if q.node is None and q.phase == "Pending"]
        assert pending
        for q in pending[:3]:
            if field == "priority":
                q.priority += 100
            elif field == "request":
                q.containers = [dict(q.containers[0], cpu=int(q.containers[0].get("cpu", 100)) + 1000)]
            else:
                q.backfill = not q.backfill
        op, on = index_maps(old_pods, old_nodes, c2)
        p2 = c2.write(str(tmp_path / "s2.kbs"))
        s.carry_snapshot(p2, op, on)
        got = s.allocate()
    with engine.Session(p2) as f:
        exp = f.allocate()
    assert all(np.array_equal(a, b) for a, b in zip(got, exp))


@pytest.mark.parametrize("variant", ["keyless", "podaff"])
def test_carry_snapshot_c3_affinity_arrivals(engine, oracle_mod, kbgen_mod, tmp_path, variant):
    """C3-shaped carry at 2k nodes: zone anti-affinity,
    topology-keyless nodes, required pod affinity (podaff); after allocate the
    cache model's next snapshot brings arrivals with hostname anti-affinity
    (the affinity shape of the events above, so the session re-opens in
    place), deletions, completions, node and PodGroup updates.  The carried
    session's allocate equals the hoisted restatement's on that snapshot (the
    faithful one, pinned against it on small instances, would take about half
    an hour at this size) and a session opened fresh on it."""
    opts = dict(keyless=0.2) if variant == "keyless" else dict(keyless=0.1, pod_affinity=0.15)
    c = kbgen_mod.gen_c3(seed=9700, n_nodes=2000, n_pending=3000, **opts)
    if "default" not in {q.name for q in c.queues}:
        c.add_queue("default")
    p1 = c.write(str(tmp_path / "c3a.kbs"))
    old_pods = sorted(c.pods, key=lambda q: q.uid)
    old_nodes = sorted(n.name for n in c.nodes)
    rng = np.random.default_rng(9701)
    with engine.Session(p1) as s:
        s.allocate()
        status, node = s.table("pod_status").copy(), s.table("pod_node").copy()
        c2 = snapshot_after_session(clone(c), status, node)
        M = CacheModel(c2)
        _events(M, rng, 2, 97, {q.uid: int(status[i]) for i, q in enumerate(old_pods)})
        op, on = index_maps(old_pods, old_nodes, c2)
        p2 = c2.write(str(tmp_path / "c3b.kbs"))
        s.carry_snapshot(p2, op, on)
        pod, nd, kind = s.allocate()
    got = [(int(a), int(b), STATUS[int(k)]) for a, b, k in zip(pod, nd, kind)]
    assert len(got) > 20  # (the first session placed most of the pending set)
    assert got == oracle_mod.fast_allocate(p2, threads=8).as_list()
    with engine.Session(p2) as s:
        pod, nd, kind = s.allocate()
    assert got == [(int(a), int(b), STATUS[int(k)]) for a, b, k in zip(pod, nd, kind)]
