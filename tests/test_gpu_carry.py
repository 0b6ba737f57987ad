"""kbhip_session_carry (the delta path between
sessions): a session carried over after its actions must schedule exactly
like a fresh session opened from the snapshot the scheduler cache would hold
then — dispatched tasks bound to their nodes, undispatched / pipelined tasks
pending again, evicted pods deleting (Releasing).  The fresh snapshot is
written from the engine's end state; its records and node state come from the
faithful oracle."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

STATUS = {1: 4, 2: 8, 3: 128}
BINDING, RELEASING, ALLOC, AOB, PIPE, RUNNING = 16, 128, 4, 2, 8, 64
NO_POD_AFFINITY = ("labels", "taints", "ports", "init", "running", "releasing", "backfill", "selector",
                   "nodeaffinity", "unsched", "bestEffort")
ACTS = ["allocate", "allocate, backfill", "reclaim, allocate, backfill, preempt"]


def _next_snapshot(c, status, node):
    """The cluster the cache holds after the session: binds and evictions applied."""
    pods = sorted(c.pods, key=lambda q: q.uid)
    names = sorted(n.name for n in c.nodes)
    for i, q in enumerate(pods):
        st = int(status[i])
        if st == BINDING:
            q.node, q.phase = names[int(node[i])], "Pending"  # bound: Pending with a node -> Bound
        elif st in (ALLOC, AOB, PIPE) or (st == 1 and q.node is None):
            q.node, q.phase = None, "Pending"
        elif st == RELEASING and not q.deleting and q.phase == "Running":
            q.deleting = True  # cache.Evict: the pod is being deleted
    return c


@pytest.mark.parametrize("seed", range(24))
def test_carry_equals_fresh_session(engine, oracle_mod, kbgen_mod, tmp_path, seed):
    if seed % 2:
        c = kbgen_mod.gen_preempt(300 + seed, n_nodes=4 + seed % 8, n_queues=1 + seed % 3, n_run_jobs=4 + seed % 7,
                                  n_pend_jobs=3 + seed % 5, max_tasks=2 + seed % 5,
                                  features=("selector", "taints", "ports", "init", "bestEffort"))
    else:
        c = kbgen_mod.gen_random(400 + seed, n_nodes=4 + seed % 10, n_jobs=5 + seed % 8, max_tasks=2 + seed % 6,
                                 features=NO_POD_AFFINITY)
    acts = ACTS[seed % len(ACTS)]
    p1 = c.write(str(tmp_path / "s1.kbs"))
    n_nodes = len(c.nodes)
    with engine.Session(p1) as s:
        s.run_actions(acts)
        status, node = s.table("pod_status").copy(), s.table("pod_node").copy()
        s.carry()
        pod, nd, kind = s.run_actions(acts)
        ns = s.read_nodes(n_nodes)
    p2 = _next_snapshot(c, status, node).write(str(tmp_path / "s2.kbs"))
    exp, ons = oracle_mod.ref_allocate(p2, actions=acts, with_nodes=True)
    assert [(int(a), int(b), STATUS[int(k)]) for a, b, k in zip(pod, nd, kind)] == exp.as_list()
    assert np.array_equal(ns.astype(np.float64), ons[:n_nodes])


@pytest.mark.parametrize("seed", range(16))
def test_carry_pod_affinity(engine, oracle_mod, kbgen_mod, tmp_path, seed):
    """Sessions with pod (anti-)affinity terms: the carried session's count
    tables are recounted from the carried pod states."""
    if seed % 2:
        c = kbgen_mod.gen_preempt(2300 + seed, n_nodes=4 + seed % 8, n_queues=1 + seed % 3, n_run_jobs=4 + seed % 7,
                                  n_pend_jobs=3 + seed % 5, max_tasks=2 + seed % 5, features=("podaffinity", "ports"))
    else:
        c = kbgen_mod.gen_random(2400 + seed, n_nodes=4 + seed % 10, n_jobs=5 + seed % 8, max_tasks=2 + seed % 6)
    if seed % 4 == 0:
        c.args = {"nodeorder": {"podaffinity.weight": "2"}}
    acts = ACTS[seed % len(ACTS)]
    p1 = c.write(str(tmp_path / "s1.kbs"))
    n_nodes = len(c.nodes)
    with engine.Session(p1) as s:
        s.run_actions(acts)
        status, node = s.table("pod_status").copy(), s.table("pod_node").copy()
        s.carry()
        pod, nd, kind = s.run_actions(acts)
        ns = s.read_nodes(n_nodes)
    p2 = _next_snapshot(c, status, node).write(str(tmp_path / "s2.kbs"))
    exp, ons = oracle_mod.ref_allocate(p2, actions=acts, with_nodes=True)
    assert [(int(a), int(b), STATUS[int(k)]) for a, b, k in zip(pod, nd, kind)] == exp.as_list()
    assert np.array_equal(ns.astype(np.float64), ons[:n_nodes])


def test_carry_c4_scaled_uploads_a_delta(engine, kbgen_mod, tmp_path):
    """C4-shaped, 20k nodes: the carry sends only the node rows the binds changed, and
    the carried session schedules only tasks that are still pending."""
    p1 = str(tmp_path / "c4.kbs")
    kbgen_mod.gen_c4(p1, n_nodes=20_000, n_pending=60_000)
    with engine.Session(p1) as s:
        s.allocate()
        st1 = s.table("pod_status").copy()
        sent = s.carry()
        st2 = s.table("pod_status").copy()
        pod, nd, kind = s.allocate()
    assert ((st1 == BINDING) == (st2 == 32)).all()           # dispatched -> Bound
    assert (st2[np.isin(st1, (ALLOC, PIPE))] == 1).all()     # undispatched / pipelined -> Pending
    assert len(pod) > 0 and (st2[pod] == 1).all()            # only pending tasks are placed again
    full = 20_000 * (12 * 8 + 4)                              # the dynamic node columns
    assert 0 < sent < full


EV_DELETE, EV_SUCCEEDED, EV_FAILED = 1, 2, 3


@pytest.mark.parametrize("seed", range(24))
def test_carry_events_equal_fresh_session(engine, oracle_mod, kbgen_mod, tmp_path, seed):
    """kbhip_session_carry_events: the session's own binds / evictions, then
    cache events on existing pods (event_handlers.go deletePod / updatePod to
    Succeeded or Failed) — evicted pods finishing, running pods completing,
    pending pods withdrawn, shadow (group-less) pods deleted.  The carried
    session must schedule like a fresh one opened from the snapshot the
    reference cache holds then: a deleted pod of a PodGroup is gone; a deleted
    group-less pod stays in its shadow job (deletePod's TaskInfo has an empty
    Job) — off its node if it had one (p_detached), unchanged (and allocated
    again) if it was pending.  The oracle's pod indices are mapped back
    through the UIDs."""
    rng = np.random.default_rng(7000 + seed)
    aff = seed % 4 in (0, 1)
    if seed % 2:
        c = kbgen_mod.gen_preempt(5300 + seed, n_nodes=4 + seed % 8, n_queues=1 + seed % 3, n_run_jobs=4 + seed % 7,
                                  n_pend_jobs=3 + seed % 5, max_tasks=2 + seed % 5,
                                  features=("selector", "taints", "ports", "init", "bestEffort")
                                  + (("podaffinity",) if seed % 4 == 1 else ()))
    else:
        c = kbgen_mod.gen_random(5400 + seed, n_nodes=4 + seed % 10, n_jobs=5 + seed % 8, max_tasks=2 + seed % 6,
                                 features=NO_POD_AFFINITY if seed % 4 else
                                 tuple(NO_POD_AFFINITY) + ("podaffinity",))
    queues = sorted(q.name for q in c.queues)
    if "default" not in queues:
        c.add_queue("default")
    node_names = sorted(n.name for n in c.nodes)
    for k in range(2 + seed % 3):  # shadow PodGroups: group-less pods, one job each
        running = k % 2 == 0
        c.add_pod("default", f"solo-{k}", uid=f"zsolo{seed:02d}{k}", group=None,
                  node=node_names[k % len(node_names)] if running else None,
                  phase="Running" if running else "Pending", containers=[{"cpu": 100, "mem": 1 << 20}])
    acts = ACTS[seed % len(ACTS)]
    p1 = c.write(str(tmp_path / "s1.kbs"))
    n_nodes = len(c.nodes)
    pods_sorted = sorted(c.pods, key=lambda q: q.uid)
    with engine.Session(p1) as s:
        s.run_actions(acts)
        status, node = s.table("pod_status").copy(), s.table("pod_node").copy()
        # events: every shadow pod deleted, evicted pods gone, some running pods done, some pending withdrawn
        ev = {}
        for i, q in enumerate(pods_sorted):
            st = int(status[i])
            if q.group is None:
                # a bound group-less pod is detached, which pod-affinity sessions refuse (tested below)
                on_node = st in (RUNNING, BINDING, 32, RELEASING)
                ev[i] = EV_SUCCEEDED if (aff and on_node) else EV_DELETE
            elif st == RELEASING and rng.random() < 0.7:
                ev[i] = EV_DELETE
            elif st in (RUNNING, BINDING, 32) and rng.random() < 0.15:
                ev[i] = EV_SUCCEEDED if rng.random() < 0.7 else EV_FAILED
            elif st == 1 and rng.random() < 0.1:
                ev[i] = EV_DELETE
        order = list(rng.permutation(sorted(ev)))
        s.carry_events(np.array(order, np.int32), np.array([ev[i] for i in order], np.uint8))
        st2 = s.table("pod_status").copy()
        pod, nd, kind = s.run_actions(acts)
        ns = s.read_nodes(n_nodes)
    c2 = _next_snapshot(c, status, node)
    for i, e in ev.items():
        q = pods_sorted[i]
        if e != EV_DELETE:
            q.phase = "Succeeded" if e == EV_SUCCEEDED else "Failed"
        elif q.group is None and q.node is not None and q.phase not in ("Succeeded", "Failed"):
            q.detached = True  # deletePod of a group-less pod: off its node, still in its shadow job
    gone = {pods_sorted[i].uid for i, e in ev.items() if e == EV_DELETE and pods_sorted[i].group is not None}
    c2.pods = [q for q in c2.pods if q.uid not in gone]
    p2 = c2.write(str(tmp_path / "s2.kbs"))
    exp, ons = oracle_mod.ref_allocate(p2, actions=acts, with_nodes=True)
    idx = {q.uid: i for i, q in enumerate(pods_sorted)}
    fresh = sorted(c2.pods, key=lambda q: q.uid)
    exp_engine = [(idx[fresh[a].uid], b, k) for a, b, k in exp.as_list()]
    assert all(int(st2[i]) == 2048 for i, e in ev.items() if e == EV_DELETE and pods_sorted[i].group is not None)
    assert all(int(st2[i]) != 2048 for i, e in ev.items() if e == EV_DELETE and pods_sorted[i].group is None)
    assert [(int(a), int(b), STATUS[int(k)]) for a, b, k in zip(pod, nd, kind)] == exp_engine
    assert np.array_equal(ns.astype(np.float64), ons[:n_nodes])


def test_carry_events_rejects_bad_input(engine, kbgen_mod, tmp_path):
    c = kbgen_mod.gen_random(77, n_nodes=4, n_jobs=4, max_tasks=3, features=NO_POD_AFFINITY)
    p1 = c.write(str(tmp_path / "s1.kbs"))
    n = len(c.pods)
    with engine.Session(p1) as s:
        s.allocate()
        before = s.table("pod_status").copy()
        for pods, evs in (([n], [EV_DELETE]), ([0], [9]), ([0, 0], [EV_DELETE, EV_SUCCEEDED])):
            with pytest.raises(engine.KbhipError):
                s.carry_events(np.array(pods, np.int32), np.array(evs, np.uint8))
            assert np.array_equal(s.table("pod_status"), before)  # nothing changed
        s.carry_events(np.array([0], np.int32), np.array([EV_DELETE], np.uint8))
        with pytest.raises(engine.KbhipError):  # already deleted
            s.carry_events(np.array([0], np.int32), np.array([EV_SUCCEEDED], np.uint8))


def test_carry_events_detach_refused_with_pod_affinity(engine, kbgen_mod, tmp_path):
    """Deleting a bound group-less pod detaches it (it stays in its shadow
    job); with pod (anti-)affinity terms in the session the predicate lister
    would leave it out at its own node only (NodeInfo.Filter), which the count
    tables do not model: KBHIP_EUNSUPPORTED, nothing changed."""
    c = kbgen_mod.gen_random(5501, n_nodes=6, n_jobs=5, max_tasks=3,
                             features=tuple(NO_POD_AFFINITY) + ("podaffinity",))
    if "default" not in {q.name for q in c.queues}:
        c.add_queue("default")
    node0 = sorted(n.name for n in c.nodes)[0]
    c.add_pod("default", "solo", uid="zsolo", group=None, node=node0, phase="Running",
              containers=[{"cpu": 100, "mem": 1 << 20}])
    c.add_job("default", "anti", sorted(q.name for q in c.queues)[0], min_member=1, ts=99)
    c.add_pod("default", "anti-0", uid="zanti", group="anti", ts=99, labels={"app": "anti"},
              containers=[{"cpu": 100, "mem": 1 << 20}],
              affinity={"anti": {"required": [{"selector": {"ml": {"app": "anti"}},
                                               "topology_key": "kubernetes.io/hostname"}]}})
    p1 = c.write(str(tmp_path / "s1.kbs"))
    solo = sorted(q.uid for q in c.pods).index("zsolo")
    with engine.Session(p1) as s:
        s.allocate()
        before = s.table("pod_status").copy()
        with pytest.raises(engine.KbhipError, match="affinity"):
            s.carry_events(np.array([solo], np.int32), np.array([EV_DELETE], np.uint8))
        assert np.array_equal(s.table("pod_status"), before)
