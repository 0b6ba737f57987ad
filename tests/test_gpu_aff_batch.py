"""Batched pops of pod-affinity classes (placement 7): classes whose pod
(anti-)affinity program only has required anti-affinity predicates — existing
pods' terms (predicates.go:1293-1360) and the pod's own (1405-1458) — with no
required affinity and no inter-pod priority terms.  A placement can only turn
nodes of the placed pod's domains infeasible, so one sweep's top-64 decides a
chunk down to the list's last key.  The engine's records, node state and gang
close messages equal the faithful restatement's (oracle/kbref.cpp) and the
per-task path's (option aff_batch = 0); C3's shape is checked against the
hoisted restatement."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
GI = 1 << 30


def _run(engine, path, actions="allocate", **opts):
    with engine.Session(path) as s:
        for k, v in opts.items():
            s.set_option(k, v)
        pod, node, kind = s.run_actions(actions)
        st = s.stats()
        ns = s.read_nodes(st["nodes"])
        close = s.gang_unschedulable()
    return [(int(p), int(n), int(k)) for p, n, k in zip(pod, node, kind)], ns, st, close


def _anti_cluster(kbgen, seed, n_nodes, n_jobs, n_zones):
    """Zones and hostnames as topology keys; running pods carrying required
    anti-affinity against app labels (existing pods' terms); pending gangs with
    self anti-affinity by zone or hostname, with app labels those running pods
    repel, or plain."""
    rng = np.random.default_rng(seed)
    c = kbgen.Cluster()
    c.add_queue("q0", 1)
    c.add_queue("q1", 3)
    zones = [f"z{i}" for i in range(n_zones)]
    apps = ["web", "db", "cache"]
    for i in range(n_nodes):
        name = f"n{i:04d}"
        c.add_node(name, int(rng.choice([8000, 16000, 32000])), int(rng.choice([16, 32, 64])) * GI, 0,
                   int(rng.choice([4, 12, 110])),
                   labels={"zone": zones[int(rng.integers(n_zones))], "kubernetes.io/hostname": name})
        if rng.random() < 0.15:  # a running pod repelling one app from its zone / host
            tk = ["zone", "kubernetes.io/hostname"][int(rng.integers(2))]
            c.add_pod("ns", f"run{i}", uid=f"r{i:05d}", node=name, phase="Running",
                      labels={"app": "guard"},
                      containers=[kbgen.res(cpu=1000, mem=GI)],
                      affinity={"anti": {"required": [{"selector": {"ml": {"app": apps[int(rng.integers(3))]}},
                                                        "topology_key": tk}]}})
    uid = 0
    for j in range(n_jobs):
        jn = f"j{j:03d}"
        size = int(rng.integers(1, 3 * n_zones + 2))
        kind = int(rng.integers(4))
        labels = {"job": jn}
        if rng.random() < 0.5:
            labels["app"] = apps[int(rng.integers(3))]
        aff = None
        if kind in (0, 1):
            tk = "zone" if kind == 0 else "kubernetes.io/hostname"
            aff = {"anti": {"required": [{"selector": {"ml": {"job": jn}}, "topology_key": tk}]}}
        c.add_job("ns", jn, f"q{j % 2}", min_member=int(rng.integers(1, size + 1)), ts=j)
        req = kbgen.res(cpu=int(rng.choice([500, 1000, 3000])), mem=int(rng.choice([1, 2, 4])) * GI)
        for k in range(size):
            c.add_pod("ns", f"{jn}-{k}", uid=f"p{uid:05d}", group=jn, ts=j, labels=dict(labels),
                      containers=[dict(req)], affinity=aff)
            uid += 1
    return c


def _check(engine, oracle_mod, p, actions="allocate"):
    exp, ons = oracle_mod.ref_allocate(p, actions=actions, with_nodes=True)
    exp_close = oracle_mod.ref_gang_close(p, actions=actions)
    status = {1: 4, 2: 8, 3: 128}
    got, ns, st, close = _run(engine, p, actions)
    assert [(a, b, status[k]) for a, b, k in got] == exp.as_list()
    assert np.array_equal(ns.astype(np.float64), ons[:ns.shape[0]])
    assert close == exp_close
    ref, ns0, st0, close0 = _run(engine, p, actions, aff_batch=0)
    assert ref == got and np.array_equal(ns0, ns) and close0 == close
    return st, st0


@pytest.mark.parametrize("seed", range(30))
def test_anti_affinity_batched(engine, oracle_mod, kbgen_mod, tmp_path, seed):
    c = _anti_cluster(kbgen_mod, 8100 + seed, n_nodes=5 + 9 * (seed % 8), n_jobs=4 + seed % 9,
                      n_zones=2 + seed % 5)
    p = c.write(str(tmp_path / "a.kbs"))
    st, st0 = _check(engine, oracle_mod, p, ["allocate", "allocate, backfill"][seed % 2])
    assert st["batched_pops"] >= st0["batched_pops"]


def test_anti_affinity_lists_fill(engine, oracle_mod, kbgen_mod, tmp_path):
    """More feasible nodes than a list holds, few zones: chunks end at the
    list's edge or when every list node is repelled, and go on in a new launch."""
    c = _anti_cluster(kbgen_mod, 8400, n_nodes=300, n_jobs=24, n_zones=6)
    p = c.write(str(tmp_path / "f.kbs"))
    st, st0 = _check(engine, oracle_mod, p)
    assert st["batched_pops"] > st0["batched_pops"]


@pytest.mark.parametrize("seed", range(20))
def test_random_pod_affinity_aff_batch(engine, oracle_mod, kbgen_mod, tmp_path, seed):
    """Every feature incl. pod affinity and inter-pod priority: eligible
    classes batched, the others on the per-task path, in one session."""
    c = kbgen_mod.gen_random(8600 + seed, n_nodes=4 + seed % 12, n_jobs=5 + seed % 8, max_tasks=2 + seed % 8)
    p = c.write(str(tmp_path / "r.kbs"))
    _check(engine, oracle_mod, p)


def test_c3_scaled_aff_batch(engine, oracle_mod, kbgen_mod, tmp_path):
    """C3's shape (zone anti-affinity on a quarter of the gangs) at 2k nodes x
    8k pods: records equal the hoisted restatement and the per-task path, and
    the anti-affine gangs go through batched pops."""
    c = kbgen_mod.gen_c3(n_nodes=2000, n_pending=8000)
    p = c.write(str(tmp_path / "c3.kbs"))
    exp = oracle_mod.fast_allocate(p, threads=8).as_list()
    got, ns, st, close = _run(engine, p)
    assert [(a, b, 4 if k == 1 else 8) for a, b, k in got] == exp
    ref, ns0, st0, close0 = _run(engine, p, aff_batch=0)
    assert ref == got and np.array_equal(ns0, ns) and close0 == close
    assert st["sweeps"] < st0["sweeps"]


@pytest.mark.parametrize("seed", range(12))
def test_per_domain_candidates_pipelined(engine, oracle_mod, kbgen_mod, tmp_path, seed):
    """Zone-self-anti-affine gangs (per-domain candidates, TaskClass dd_space)
    on nodes whose Idle is mostly taken by Releasing pods: many placements are
    Pipelined, which do not close their domain, so a launch ends after one and
    the host goes on.  Records, node state and close messages equal the
    faithful restatement's and the per-task path's."""
    rng = np.random.default_rng(8800 + seed)
    c = _anti_cluster(kbgen_mod, 8700 + seed, n_nodes=20 + 7 * (seed % 6), n_jobs=5 + seed % 6, n_zones=3 + seed % 4)
    guarded = {q.node for q in c.pods if q.node is not None}
    for i, n in enumerate(list(c.nodes)):
        if rng.random() < 0.85:  # a deleting pod holding most of the node: mostly Pipelined fits
            free = 1000 if n.name in guarded else 0
            c.add_pod("ns", f"rel{i}", uid=f"q{i:05d}", node=n.name, phase="Running", deleting=True,
                      containers=[kbgen_mod.res(cpu=n.cpu - free - 600 - 1000 * int(rng.integers(0, 2)),
                                                mem=n.mem - GI - GI // 2 - GI * int(rng.integers(0, 3)))])
    p = c.write(str(tmp_path / "p.kbs"))
    st, st0 = _check(engine, oracle_mod, p)
    assert st["batched_pops"] >= st0["batched_pops"]


@pytest.mark.parametrize("seed", range(3))
def test_per_domain_candidates_keyless_nodes(engine, oracle_mod, kbgen_mod, tmp_path, seed):
    """Per-domain candidates over many sweep blocks with nodes that lack the
    topology key: big nodes carry one of 24 zones (each block's
    list holds a node per zone, enough to fill a merged top-64 with keyed
    nodes), a third of the nodes — smaller, lower scores — have no zone label,
    so a zone-anti-affine gang of up to 64 pods must spill onto them once the
    zones are used.  Records equal the hoisted restatement's and the per-task
    path's."""
    rng = np.random.default_rng(9100 + seed)
    c = kbgen_mod.Cluster()
    c.add_queue("q0", 1)
    zones = [f"z{i:02d}" for i in range(24)]
    for i in range(3000 + 500 * seed):
        name = f"n{i:05d}"
        if rng.random() < 0.35:  # keyless: no zone label
            c.add_node(name, 8000, 16 * GI, 0, 110, labels={"kubernetes.io/hostname": name})
        else:
            c.add_node(name, 64000, 256 * GI, 0, 110,
                       labels={"zone": zones[int(rng.integers(24))], "kubernetes.io/hostname": name})
    uid = 0
    for j in range(24):
        jn = f"j{j:03d}"
        size = int(rng.integers(30, 65))
        aff = {"anti": {"required": [{"selector": {"ml": {"job": jn}}, "topology_key": "zone"}]}} \
            if j % 3 != 2 else None
        c.add_job("ns", jn, "q0", min_member=int(rng.integers(size // 2, size + 1)), ts=j)
        req = kbgen_mod.res(cpu=int(rng.choice([500, 1000])), mem=int(rng.choice([1, 2])) * GI)
        for k in range(size):
            c.add_pod("ns", f"{jn}-{k}", uid=f"p{uid:05d}", group=jn, ts=j, labels={"job": jn},
                      containers=[dict(req)], affinity=aff)
            uid += 1
    p = c.write(str(tmp_path / "k.kbs"))
    exp = oracle_mod.fast_allocate(p, threads=8).as_list()
    got, ns, st, close = _run(engine, p)
    assert [(a, b, 4 if k == 1 else 8) for a, b, k in got] == exp
    ref, ns0, st0, close0 = _run(engine, p, aff_batch=0)
    assert ref == got and np.array_equal(ns0, ns) and close0 == close
    assert st["batched_pops"] > 0
