"""Host ports beyond 256 distinct (ip, protocol, port) triples
(host_ports.go:96-125, predicates.go PodFitsHostPorts).  Port ids are
numbered in (protocol, port, IP) order and each task class reads a window of
four 64-bit words of the node port columns (TaskClass::pw_lo), so the session
may hold any number of distinct host ports; only a pod whose own ports and
their conflicts span more than 256 ids is refused (KBHIP_EUNSUPPORTED).
Records and node state equal the faithful restatement's on both device paths."""
import numpy as np
import pytest

GI = 1 << 30


def _port_cluster(kbgen, seed, n_nodes=30, n_jobs=24, n_ports=400):
    rng = np.random.default_rng(seed)
    c = kbgen.Cluster()
    c.add_queue("q0", 1)
    ports = 20000 + rng.permutation(n_ports)
    for i in range(n_nodes):
        name = f"n{i:03d}"
        c.add_node(name, 16000, 32 * GI, 0, 110)
        for k in range(int(rng.integers(0, 4))):  # running pods holding host ports
            pp = [{"port": int(ports[int(rng.integers(n_ports))]), "ip": ["", "10.0.0.1"][int(rng.integers(2))],
                   "proto": ["", "UDP"][int(rng.integers(2))]}]
            c.add_pod("run", f"r{i}-{k}", uid=f"r{i:03d}{k}", node=name, phase="Running",
                      containers=[dict(kbgen.res(cpu=500, mem=GI), ports=pp)])
    uid = 0
    for j in range(n_jobs):
        jn = f"j{j:03d}"
        size = int(rng.integers(1, 8))
        c.add_job("ns", jn, "q0", min_member=int(rng.integers(1, size + 1)), ts=j)
        p0 = int(rng.integers(n_ports - 1))
        pp = [{"port": int(ports[p0]), "ip": "", "proto": ""}]
        if rng.random() < 0.4:
            pp.append({"port": int(ports[p0]) + 100000, "ip": "10.0.0.2", "proto": "TCP"})
        req = kbgen.res(cpu=int(rng.choice([500, 1000])), mem=GI)
        for k in range(size):
            c.add_pod("ns", f"{jn}-{k}", uid=f"p{uid:05d}", group=jn, ts=j,
                      containers=[dict(req, ports=[dict(x) for x in pp])])
            uid += 1
    return c


def test_many_ports_encode(engine_lib, kbgen_mod, tmp_path):
    """More than 256 distinct host ports open (encode-only, no device)."""
    import kbhip
    c = _port_cluster(kbgen_mod, 1, n_ports=600)
    p = c.write(str(tmp_path / "p.kbs"))
    with kbhip.EncodedSnapshot(p) as e:
        assert int(e.table("dims")[0]) == 30


def test_port_window_refused(engine_lib, kbgen_mod, tmp_path):
    """A pod whose two ports lie more than 256 port ids apart is refused."""
    import kbhip
    c = _port_cluster(kbgen_mod, 2, n_ports=50)
    c.add_job("ns", "fill", "q0", min_member=1, ts=0)
    for k in range(300):  # 300 distinct ports between the wide pod's two
        c.add_pod("ns", f"fill-{k}", uid=f"f{k:04d}", group="fill",
                  containers=[dict(kbgen_mod.res(cpu=100, mem=GI), ports=[{"port": 30001 + k, "ip": "", "proto": ""}])])
    c.add_job("ns", "wide", "q0", min_member=1, ts=0)
    c.add_pod("ns", "wide-0", uid="w0", group="wide",
              containers=[dict(kbgen_mod.res(cpu=100, mem=GI),
                               ports=[{"port": 30000, "ip": "", "proto": ""}, {"port": 30400, "ip": "", "proto": ""}])])
    p = c.write(str(tmp_path / "w.kbs"))
    with pytest.raises(kbhip.KbhipError, match="host ports"):
        with kbhip.EncodedSnapshot(p):
            pass


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(8))
def test_many_ports_gpu(engine, oracle_mod, kbgen_mod, tmp_path, seed):
    c = _port_cluster(kbgen_mod, 3100 + seed, n_ports=300 + 60 * seed)
    p = c.write(str(tmp_path / "p.kbs"))
    exp, ons = oracle_mod.ref_allocate(p, with_nodes=True)
    for batched in (1, 0):
        with engine.Session(p) as s:
            s.set_option("batched", batched)
            pod, node, kind = s.allocate()
            ns = s.read_nodes(len(c.nodes))
        assert [(int(a), int(b), 4 if k == 1 else 8) for a, b, k in zip(pod, node, kind)] == exp.as_list()
        assert np.array_equal(ns.astype(np.float64), ons[:len(c.nodes)])
