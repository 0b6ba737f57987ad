"""kbgen — KBS1 snapshot writer and seeded synthetic cluster generator.

A KBS1 file (format: include/kbsnap.h) carries what kube-batch's
``SchedulerCache.Snapshot()`` hands a session (reference
pkg/scheduler/cache/cache.go:515-583): nodes, queues, pod groups, pods and the
tier configuration.  Two ways to build one:

* ``Cluster`` — an object-level builder for hand-written cases (the reference's
  unit-test fixtures, e.g. ``buildNode``/``buildPod`` in
  pkg/scheduler/actions/allocate/allocate_test.go:58-98) and medium synthetic
  configs with labels, taints, selectors and affinity.
* ``gen_c2`` / ``gen_c4`` — vectorised bulk generators for the resource-only
  configs (5k nodes x 50k pods, 100k nodes x 1M pods), written straight into
  columns.

Canonical order: nodes sorted by name, jobs by UID
("ns/name"), pods by UID, queues by name.  Every reference map iteration is
pinned to that order on every implementation.

Resource units are already the reference's: cpu and nvidia.com/gpu in milli,
memory in bytes, i.e. Quantity.MilliValue()/Value().
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

GI = 1 << 30
MI = 1 << 20

PHASES = {"Pending": 0, "Running": 1, "Succeeded": 2, "Failed": 3, "Unknown": 4}
OPS = {"In": 0, "NotIn": 1, "Exists": 2, "DoesNotExist": 3, "Gt": 4, "Lt": 5}
HAS_CPU, HAS_MEM, HAS_GPU = 1, 2, 4
AFF_NA, AFF_NA_REQ, AFF_PA, AFF_PAA = 1, 2, 4, 8
DIS = {"disableJobOrder": 1, "disableJobReady": 2, "disableTaskOrder": 4,
       "disablePreemptable": 8, "disableReclaimable": 16, "disableQueueOrder": 32,
       "disablePredicate": 64, "disableNodeOrder": 128}

# config/kube-batch-conf.yaml:1-10 (the reference's shipped conf)
DEFAULT_TIERS = [["priority", "gang", "conformance"],
                 ["drf", "predicates", "proportion", "nodeorder"]]
DEFAULT_ACTIONS = "reclaim, allocate, backfill, preempt"
# allocate_test.go:282-293 opens the session with tiers [drf, proportion] only.
TEST_TIERS = [["drf", "proportion"]]

_DT = {np.int8: (1, 1), np.uint8: (2, 1), np.int32: (3, 4), np.int64: (4, 8),
       np.float64: (5, 8)}


# ----------------------------------------------------------------------------
# low level: columns -> file
# ----------------------------------------------------------------------------
class StrTab:
    """NUL-terminated string table with interning."""

    def __init__(self):
        self._parts: List[bytes] = []
        self._size = 0
        self._ids: Dict[str, int] = {}

    def add(self, s: Optional[str]) -> int:
        if s is None:
            return -1
        off = self._ids.get(s)
        if off is not None:
            return off
        b = s.encode() + b"\0"
        off = self._size
        self._parts.append(b)
        self._size += len(b)
        self._ids[s] = off
        return off

    def add_bulk_unique(self, strings: Sequence[str]) -> np.ndarray:
        """Append strings known to be unique (no interning); returns offsets."""
        enc = [s.encode() for s in strings]
        lens = np.fromiter((len(b) + 1 for b in enc), dtype=np.int64, count=len(enc))
        offs = np.empty(len(enc), dtype=np.int64)
        if len(enc):
            offs[0] = 0
            np.cumsum(lens[:-1], out=offs[1:])
        offs += self._size
        blob = b"\0".join(enc) + (b"\0" if enc else b"")
        self._parts.append(blob)
        self._size += len(blob)
        if self._size >= 2 ** 31:
            raise ValueError("strtab exceeds 2 GiB")
        return offs.astype(np.int32)

    def bytes(self) -> bytes:
        return b"".join(self._parts)


def write_kbs(path: str, cols: Dict[str, np.ndarray], strtab: StrTab) -> None:
    """Write a KBS1 file: header, directory, 16-byte-aligned sections."""
    sections: List[Tuple[str, int, int, bytes]] = []
    st = strtab.bytes()
    if not st:
        st = b"\0"
    sections.append(("strtab", 6, 1, st))
    for name, arr in cols.items():
        arr = np.ascontiguousarray(arr)
        key = arr.dtype.type
        if key not in _DT:
            raise TypeError(f"column {name}: unsupported dtype {arr.dtype}")
        code, esz = _DT[key]
        if len(name) > 23:
            raise ValueError(f"column name too long: {name}")
        sections.append((name, code, esz, arr.tobytes()))
    nsec = len(sections)
    hdr = struct.pack("<4sIII", b"KBS1", 1, nsec, 0)
    dir_size = nsec * 48
    off = len(hdr) + dir_size
    off = (off + 15) & ~15
    dirents = []
    blobs = []
    for name, code, esz, data in sections:
        dirents.append(struct.pack("<24sIIQQ", name.encode(), code, esz, len(data) // esz, off))
        blobs.append((off, data))
        off += len(data)
        off = (off + 15) & ~15
    with open(path, "wb") as f:
        f.write(hdr)
        f.write(b"".join(dirents))
        for o, data in blobs:
            f.seek(o)
            f.write(data)
        f.truncate(off)


def _csr(lengths: Sequence[int]) -> np.ndarray:
    out = np.zeros(len(lengths) + 1, dtype=np.int32)
    if len(lengths):
        np.cumsum(np.asarray(lengths, dtype=np.int64), out=out[1:])
    return out


def read_kbs(path: str) -> Tuple[Dict[str, np.ndarray], bytes]:
    """Read a KBS1 file back: (columns, string table)."""
    inv = {v[0]: k for k, v in _DT.items()}
    with open(path, "rb") as f:
        data = f.read()
    magic, ver, nsec, _ = struct.unpack_from("<4sIII", data, 0)
    if magic != b"KBS1":
        raise ValueError("not a KBS1 file")
    cols, st = {}, b""
    for k in range(nsec):
        name, code, esz, n, off = struct.unpack_from("<24sIIQQ", data, 16 + 48 * k)
        name = name.rstrip(b"\0").decode()
        raw = data[off:off + n * esz]
        if name == "strtab":
            st = raw
        else:
            cols[name] = np.frombuffer(raw, dtype=inv[code]).copy()
    return cols, st


def cluster_from_kbs(path: str) -> "Cluster":
    """The object model of a KBS1 snapshot, as far as the host-side ordering
    needs it (tests/gohost.py): nodes (name, allocatable), queues, jobs and pods
    (UID, namespace, PodGroup, node, phase, priority, timestamp, container
    requests).  Labels, affinity, ports and tolerations are left out."""
    C, st = read_kbs(path)

    def s(off):
        if off < 0:
            return None
        return st[off:st.index(b"\0", off)].decode()
    c = Cluster(tiers=[], actions=s(int(C["conf_actions"][0])) if "conf_actions" in C else DEFAULT_ACTIONS)
    tiers: Dict[int, List[str]] = {}
    flags: Dict[str, List[str]] = {}
    inv_dis = {v: k for k, v in DIS.items()}
    for n, t, fl in zip(C["conf_plugin_name"], C["conf_plugin_tier"], C["conf_plugin_flags"]):
        tiers.setdefault(int(t), []).append(s(int(n)))
        for bit, name in inv_dis.items():
            if int(fl) & bit:
                flags.setdefault(s(int(n)), []).append(name)
    c.tiers = [tiers[k] for k in sorted(tiers)]
    c.flags = flags
    for q, w, ts in zip(C["q_name"], C["q_weight"], C["q_ts"]):
        c.add_queue(s(int(q)), int(w), int(ts))
    for i in range(len(C["n_name"])):
        c.add_node(s(int(C["n_name"][i])), int(C["n_alloc_cpu"][i]), int(C["n_alloc_mem"][i]),
                   int(C["n_alloc_gpu"][i]), int(C["n_alloc_pods"][i]))
    jname = [s(int(x)) for x in C["j_name"]]
    for k in range(len(jname)):
        c.add_job(s(int(C["j_ns"][k])), jname[k], s(int(C["j_queue"][k])), min_member=int(C["j_min"][k]),
                  ts=int(C["j_ts"][k]), pg_priority=int(C["j_pg_priority"][k]))
    inv_ph = {v: k for k, v in PHASES.items()}
    off = C["p_ctr_off"]
    dele = C.get("p_deleting")
    for i in range(len(C["p_uid"])):
        j = int(C["p_job"][i])
        ctrs = [dict(cpu=int(C["c_cpu"][q]), mem=int(C["c_mem"][q]), gpu=int(C["c_gpu"][q]))
                for q in range(int(off[i]), int(off[i + 1]))]
        c.add_pod(s(int(C["p_ns"][i])), s(int(C["p_name"][i])) if "p_name" in C else s(int(C["p_uid"][i])),
                  uid=s(int(C["p_uid"][i])), group=jname[j] if j >= 0 else None,
                  node=s(int(C["p_node"][i])) or None, phase=inv_ph[int(C["p_phase"][i])],
                  deleting=bool(dele[i]) if dele is not None else False, priority=int(C["p_priority"][i]),
                  ts=int(C["p_ts"][i]), containers=ctrs)
    return c


# ----------------------------------------------------------------------------
# object-level builder
# ----------------------------------------------------------------------------
@dataclass
class Node:
    name: str
    cpu: int
    mem: int
    gpu: int = 0
    pods: int = 110
    labels: Dict[str, str] = field(default_factory=dict)
    taints: List[Tuple[str, str, str]] = field(default_factory=list)  # (key, value, effect)
    unschedulable: bool = False
    cap: Optional[Tuple[int, int, int, int]] = None  # capacity; defaults to allocatable


@dataclass
class Queue:
    name: str
    weight: int = 1
    ts: int = 0


@dataclass
class Job:
    ns: str
    name: str
    queue: str
    min_member: int = 0
    ts: int = 0
    pg_priority: int = 0

    @property
    def uid(self) -> str:
        return f"{self.ns}/{self.name}"


@dataclass
class Pod:
    ns: str
    name: str
    uid: Optional[str] = None
    group: Optional[str] = None  # pod group name (annotation scheduling.k8s.io/group-name)
    node: Optional[str] = None
    phase: str = "Pending"
    deleting: bool = False
    # detached: the scheduler cache deleted this group-less pod, which takes it
    # off its node only (deletePod builds NewTaskInfo with an empty Job,
    # cache/event_handlers.go:119-165): the task stays in its shadow job with
    # its status and NodeName, but is not in the node's task list
    detached: bool = False
    priority: int = 0
    ts: int = 0
    backfill: bool = False
    priority_class: str = ""  # Spec.PriorityClassName (conformance plugin)
    labels: Dict[str, str] = field(default_factory=dict)
    # containers: dicts with optional keys cpu, mem, gpu (absent = not in Requests) and ports
    containers: List[dict] = field(default_factory=lambda: [{}])
    init_containers: List[dict] = field(default_factory=list)
    node_selector: Dict[str, str] = field(default_factory=dict)
    tolerations: List[dict] = field(default_factory=list)  # key, op, value, effect
    affinity: Optional[dict] = None

    def __post_init__(self):
        if self.uid is None:
            self.uid = f"{self.ns}-{self.name}"


def res(cpu=None, mem=None, gpu=None, ports=None) -> dict:
    d = {}
    if cpu is not None:
        d["cpu"] = cpu
    if mem is not None:
        d["mem"] = mem
    if gpu is not None:
        d["gpu"] = gpu
    if ports:
        d["ports"] = ports
    return d


class Cluster:
    """Object-level cluster description -> KBS1 columns."""

    def __init__(self, tiers=None, actions: str = DEFAULT_ACTIONS, args: Optional[dict] = None,
                 flags: Optional[dict] = None):
        self.tiers = [list(t) for t in (tiers if tiers is not None else DEFAULT_TIERS)]
        self.actions = actions
        self.args = dict(args or {})      # plugin -> {key: value}
        self.flags = dict(flags or {})    # plugin -> [flag names]
        self.nodes: List[Node] = []
        self.queues: List[Queue] = []
        self.jobs: List[Job] = []
        self.pods: List[Pod] = []

    def add_node(self, *a, **k) -> Node:
        n = Node(*a, **k)
        self.nodes.append(n)
        return n

    def add_queue(self, *a, **k) -> Queue:
        q = Queue(*a, **k)
        self.queues.append(q)
        return q

    def add_job(self, *a, **k) -> Job:
        j = Job(*a, **k)
        self.jobs.append(j)
        return j

    def add_pod(self, *a, **k) -> Pod:
        p = Pod(*a, **k)
        self.pods.append(p)
        return p

    # -- serialisation -------------------------------------------------------
    def columns(self) -> Tuple[Dict[str, np.ndarray], StrTab]:
        st = StrTab()
        C: Dict[str, np.ndarray] = {}
        i32 = lambda xs: np.asarray(xs, dtype=np.int32)
        i64 = lambda xs: np.asarray(xs, dtype=np.int64)
        u8 = lambda xs: np.asarray(xs, dtype=np.uint8)

        # conf
        C["conf_actions"] = i32([st.add(self.actions)])
        pn, pt, pf, ap, ak, av = [], [], [], [], [], []
        for ti, tier in enumerate(self.tiers):
            for name in tier:
                pidx = len(pn)
                pn.append(st.add(name))
                pt.append(ti)
                fl = 0
                for f in self.flags.get(name, []):
                    fl |= DIS[f]
                pf.append(fl)
                for k, v in sorted(self.args.get(name, {}).items()):
                    ap.append(pidx)
                    ak.append(st.add(k))
                    av.append(st.add(str(v)))
        C["conf_plugin_name"], C["conf_plugin_tier"], C["conf_plugin_flags"] = i32(pn), i32(pt), i32(pf)
        C["conf_arg_plugin"], C["conf_arg_key"], C["conf_arg_val"] = i32(ap), i32(ak), i32(av)

        queues = sorted(self.queues, key=lambda q: q.name)
        C["q_name"] = i32([st.add(q.name) for q in queues])
        C["q_weight"] = i32([q.weight for q in queues])
        C["q_ts"] = i64([q.ts for q in queues])

        nodes = sorted(self.nodes, key=lambda n: n.name)
        if len({n.name for n in nodes}) != len(nodes):
            raise ValueError("duplicate node names")
        C["n_name"] = i32([st.add(n.name) for n in nodes])
        C["n_alloc_cpu"] = i64([n.cpu for n in nodes])
        C["n_alloc_mem"] = i64([n.mem for n in nodes])
        C["n_alloc_gpu"] = i64([n.gpu for n in nodes])
        C["n_alloc_pods"] = i64([n.pods for n in nodes])
        caps = [n.cap if n.cap is not None else (n.cpu, n.mem, n.gpu, n.pods) for n in nodes]
        C["n_cap_cpu"] = i64([c[0] for c in caps])
        C["n_cap_mem"] = i64([c[1] for c in caps])
        C["n_cap_gpu"] = i64([c[2] for c in caps])
        C["n_cap_pods"] = i64([c[3] for c in caps])
        C["n_unsched"] = u8([1 if n.unschedulable else 0 for n in nodes])
        C["n_label_off"] = _csr([len(n.labels) for n in nodes])
        C["nl_key"] = i32([st.add(k) for n in nodes for k in sorted(n.labels)])
        C["nl_val"] = i32([st.add(n.labels[k]) for n in nodes for k in sorted(n.labels)])
        C["n_taint_off"] = _csr([len(n.taints) for n in nodes])
        C["nt_key"] = i32([st.add(t[0]) for n in nodes for t in n.taints])
        C["nt_val"] = i32([st.add(t[1] if t[1] != "" else None) for n in nodes for t in n.taints])
        C["nt_effect"] = i32([st.add(t[2]) for n in nodes for t in n.taints])

        jobs = sorted(self.jobs, key=lambda j: j.uid)
        jidx = {j.uid: i for i, j in enumerate(jobs)}
        if len(jidx) != len(jobs):
            raise ValueError("duplicate job uids")
        C["j_ns"] = i32([st.add(j.ns) for j in jobs])
        C["j_name"] = i32([st.add(j.name) for j in jobs])
        C["j_queue"] = i32([st.add(j.queue) for j in jobs])
        C["j_min"] = i32([j.min_member for j in jobs])
        C["j_pg_priority"] = i32([j.pg_priority for j in jobs])
        C["j_ts"] = i64([j.ts for j in jobs])

        pods = sorted(self.pods, key=lambda p: p.uid)
        if len({p.uid for p in pods}) != len(pods):
            raise ValueError("duplicate pod uids")
        C["p_uid"] = i32([st.add(p.uid) for p in pods])
        C["p_name"] = i32([st.add(p.name) for p in pods])
        C["p_ns"] = i32([st.add(p.ns) for p in pods])
        pj = []
        for p in pods:
            if p.group is None:
                pj.append(-1)
            else:
                uid = f"{p.ns}/{p.group}"
                if uid not in jidx:
                    raise ValueError(f"pod {p.uid}: unknown pod group {uid}")
                pj.append(jidx[uid])
        C["p_job"] = i32(pj)
        C["p_node"] = i32([st.add(p.node) if p.node else -1 for p in pods])
        C["p_phase"] = u8([PHASES[p.phase] for p in pods])
        C["p_deleting"] = u8([1 if p.deleting else 0 for p in pods])
        if any(p.detached for p in pods):
            C["p_detached"] = u8([1 if p.detached else 0 for p in pods])
        C["p_backfill"] = u8([1 if p.backfill else 0 for p in pods])
        C["p_pclass"] = i32([st.add(p.priority_class) if p.priority_class else -1 for p in pods])
        C["p_priority"] = i32([p.priority for p in pods])
        C["p_ts"] = i64([p.ts for p in pods])
        C["p_label_off"] = _csr([len(p.labels) for p in pods])
        C["pl_key"] = i32([st.add(k) for p in pods for k in sorted(p.labels)])
        C["pl_val"] = i32([st.add(p.labels[k]) for p in pods for k in sorted(p.labels)])
        C["p_nsel_off"] = _csr([len(p.node_selector) for p in pods])
        C["ps_key"] = i32([st.add(k) for p in pods for k in sorted(p.node_selector)])
        C["ps_val"] = i32([st.add(p.node_selector[k]) for p in pods for k in sorted(p.node_selector)])

        ctrs = [c for p in pods for c in p.containers]
        C["p_ctr_off"] = _csr([len(p.containers) for p in pods])
        C["c_cpu"] = i64([c.get("cpu", 0) for c in ctrs])
        C["c_mem"] = i64([c.get("mem", 0) for c in ctrs])
        C["c_gpu"] = i64([c.get("gpu", 0) for c in ctrs])
        C["c_has"] = u8([(HAS_CPU if "cpu" in c else 0) | (HAS_MEM if "mem" in c else 0)
                         | (HAS_GPU if "gpu" in c else 0) for c in ctrs])
        ports = [pt for c in ctrs for pt in c.get("ports", [])]
        C["c_port_off"] = _csr([len(c.get("ports", [])) for c in ctrs])
        C["pt_ip"] = i32([st.add(pt.get("ip") or None) for pt in ports])
        C["pt_proto"] = i32([st.add(pt.get("proto") or None) for pt in ports])
        C["pt_port"] = i32([pt.get("port", 0) for pt in ports])
        ictrs = [c for p in pods for c in p.init_containers]
        C["p_ictr_off"] = _csr([len(p.init_containers) for p in pods])
        C["ic_cpu"] = i64([c.get("cpu", 0) for c in ictrs])
        C["ic_mem"] = i64([c.get("mem", 0) for c in ictrs])
        C["ic_gpu"] = i64([c.get("gpu", 0) for c in ictrs])
        C["ic_has"] = u8([(HAS_CPU if "cpu" in c else 0) | (HAS_MEM if "mem" in c else 0)
                          | (HAS_GPU if "gpu" in c else 0) for c in ictrs])
        tols = [t for p in pods for t in p.tolerations]
        C["p_tol_off"] = _csr([len(p.tolerations) for p in pods])
        C["tl_key"] = i32([st.add(t.get("key") or None) for t in tols])
        C["tl_op"] = i32([st.add(t.get("op") or None) for t in tols])
        C["tl_val"] = i32([st.add(t.get("value") or None) for t in tols])
        C["tl_effect"] = i32([st.add(t.get("effect") or None) for t in tols])

        self._affinity_columns(pods, C, st)
        return C, st

    def _affinity_columns(self, pods, C, st):
        i32 = lambda xs: np.asarray(xs, dtype=np.int32)
        u8 = lambda xs: np.asarray(xs, dtype=np.uint8)
        nsr_key, nsr_op, nsr_len, nsrv = [], [], [], []
        e_start, e_cnt, f_start, f_cnt = [], [], [], []
        pst_w, pst_t = [], []
        ls_ml, ls_me, lkv_k, lkv_v = [], [], [], []
        lsr_key, lsr_op, lsr_len, lsrv = [], [], [], []
        pat_sel, pat_ns, patns, pat_topo = [], [], [], []
        wpat_w, wpat_t = [], []
        a_flags = []
        lists = {k: [] for k in ("nareq", "napref", "pareq", "papref", "paareq", "paapref")}
        p_aff = []

        def add_nsr(reqs):
            start = len(nsr_key)
            for (k, op, vs) in reqs:
                nsr_key.append(st.add(k))
                nsr_op.append(OPS.get(op, 15))
                nsr_len.append(len(vs))
                nsrv.extend(st.add(v) for v in vs)
            return start, len(reqs)

        def add_nst(term):
            idx = len(e_start)
            s, c = add_nsr(term.get("expr", []))
            e_start.append(s)
            e_cnt.append(c)
            s, c = add_nsr(term.get("fields", []))
            f_start.append(s)
            f_cnt.append(c)
            return idx

        def add_lsel(sel):
            if sel is None:
                return -1
            idx = len(ls_ml)
            ml = sel.get("ml", {})
            ls_ml.append(len(ml))
            for k in sorted(ml):
                lkv_k.append(st.add(k))
                lkv_v.append(st.add(ml[k]))
            me = sel.get("me", [])
            ls_me.append(len(me))
            for (k, op, vs) in me:
                lsr_key.append(st.add(k))
                lsr_op.append(OPS.get(op, 15))
                lsr_len.append(len(vs))
                lsrv.extend(st.add(v) for v in vs)
            return idx

        def add_pat(term):
            idx = len(pat_sel)
            pat_sel.append(add_lsel(term.get("selector")))
            nss = term.get("namespaces", [])
            pat_ns.append(len(nss))
            patns.extend(st.add(v) for v in nss)
            pat_topo.append(st.add(term.get("topology_key") or None))
            return idx

        for p in pods:
            a = p.affinity
            if a is None:
                p_aff.append(-1)
                continue
            p_aff.append(len(a_flags))
            fl = 0
            na, pa, paa = a.get("node"), a.get("pod"), a.get("anti")
            if na is not None:
                fl |= AFF_NA
                if na.get("required") is not None:
                    fl |= AFF_NA_REQ
            if pa is not None:
                fl |= AFF_PA
            if paa is not None:
                fl |= AFF_PAA
            a_flags.append(fl)
            lists["nareq"].append([add_nst(t) for t in ((na or {}).get("required") or [])])
            rows = []
            for (w, t) in ((na or {}).get("preferred") or []):
                rows.append(len(pst_w))
                pst_w.append(w)
                pst_t.append(add_nst(t))
            lists["napref"].append(rows)
            for key, src in (("pareq", pa), ("paareq", paa)):
                lists[key].append([add_pat(t) for t in ((src or {}).get("required") or [])])
            for key, src in (("papref", pa), ("paapref", paa)):
                rows = []
                for (w, t) in ((src or {}).get("preferred") or []):
                    t_idx = add_pat(t)
                    rows.append(len(wpat_w))
                    wpat_w.append(w)
                    wpat_t.append(t_idx)
                lists[key].append(rows)

        C["p_aff"] = i32(p_aff)
        C["a_flags"] = u8(a_flags)
        for key, rows in lists.items():
            # each pod's rows were appended consecutively: a contiguous run
            for lst in rows:
                if lst and lst != list(range(lst[0], lst[0] + len(lst))):
                    raise AssertionError(f"non-contiguous affinity rows for {key}")
            C[f"a_{key}_start"] = i32([lst[0] if lst else 0 for lst in rows])
            C[f"a_{key}_cnt"] = i32([len(lst) for lst in rows])
        C["nst_expr_start"], C["nst_expr_cnt"] = i32(e_start), i32(e_cnt)
        C["nst_field_start"], C["nst_field_cnt"] = i32(f_start), i32(f_cnt)
        C["nsr_key"], C["nsr_op"] = i32(nsr_key), u8(nsr_op)
        C["nsr_val_off"], C["nsrv"] = _csr(nsr_len), i32(nsrv)
        C["pst_weight"], C["pst_term"] = i32(pst_w), i32(pst_t)
        C["ls_ml_off"], C["lkv_key"], C["lkv_val"] = _csr(ls_ml), i32(lkv_k), i32(lkv_v)
        C["ls_me_off"] = _csr(ls_me)
        C["lsr_key"], C["lsr_op"] = i32(lsr_key), u8(lsr_op)
        C["lsr_val_off"], C["lsrv"] = _csr(lsr_len), i32(lsrv)
        C["pat_sel"], C["pat_topo"] = i32(pat_sel), i32(pat_topo)
        C["pat_ns_off"], C["patns"] = _csr(pat_ns), i32(patns)
        C["wpat_weight"], C["wpat_term"] = i32(wpat_w), i32(wpat_t)

    def write(self, path: str) -> str:
        C, st = self.columns()
        write_kbs(path, C, st)
        return path


# ----------------------------------------------------------------------------
# seeded synthetic configs; seed = 20261015 + config id
# ----------------------------------------------------------------------------
BASE_SEED = 20261015
SEC = 1_000_000_000  # timestamps are in ns; metav1.Time compares at full precision


def gen_c1(tiers=None) -> Cluster:
    """C1: the allocate-action unit-test shape (BASELINE configs[0]).

    3 nodes of 4 CPU / 8Gi / pods 110; queues q1, q2 (weight 1); job A in q1
    with minMember 4 and 4 pods of (1 CPU, 1Gi); job B in q2 with 2 pods,
    minMember 1.  Default tiers are the shipped conf; pass TEST_TIERS for the
    [drf, proportion] session of allocate_test.go:282-293.
    """
    c = Cluster(tiers=tiers)
    for i in range(3):
        c.add_node(f"n{i + 1}", 4000, 8 * GI, 0, 110)
    c.add_queue("q1", 1)
    c.add_queue("q2", 1)
    c.add_job("c1", "ja", "q1", min_member=4)
    c.add_job("c2", "jb", "q2", min_member=1)
    for i in range(4):
        c.add_pod("c1", f"a{i}", group="ja", containers=[res(1000, GI, 0)])
    for i in range(2):
        c.add_pod("c2", f"b{i}", group="jb", containers=[res(1000, GI, 0)])
    return c


# node SKUs (cpu milli, mem bytes, gpu milli) and their shares
SKUS = [(32000, 128 * GI, 0), (64000, 256 * GI, 0), (96000, 512 * GI, 8000)]
SKU_P = [0.3, 0.5, 0.2]
CPU_CHOICES = np.array([500, 1000, 2000, 4000], dtype=np.int64)
MEM_CHOICES = np.array([1, 2, 4, 8], dtype=np.int64) * GI
GPU_CHOICES = np.array([0, 1000, 2000, 4000, 8000], dtype=np.int64)
GPU_P = [0.75, 0.0625, 0.0625, 0.0625, 0.0625]


def _bulk(n_nodes: int, n_pending: int, running_per_node: np.ndarray, seed: int,
          n_queues: int = 1, tiers=None, gang_lo: int = 8, gang_hi: int = 64,
          running_gang: int = 8, run_res=None) -> Tuple[Dict[str, np.ndarray], StrTab, dict]:
    """Vectorised resource-only cluster (C2/C4 family) written straight to columns."""
    rng = np.random.default_rng(seed)
    st = StrTab()
    C: Dict[str, np.ndarray] = {}
    tiers = tiers if tiers is not None else DEFAULT_TIERS

    # conf: the shipped kube-batch-conf.yaml
    C["conf_actions"] = np.asarray([st.add(DEFAULT_ACTIONS)], dtype=np.int32)
    names = [p for t in tiers for p in t]
    C["conf_plugin_name"] = np.asarray([st.add(p) for p in names], dtype=np.int32)
    C["conf_plugin_tier"] = np.asarray([ti for ti, t in enumerate(tiers) for _ in t], dtype=np.int32)
    C["conf_plugin_flags"] = np.zeros(len(names), dtype=np.int32)

    qn = [f"q{i}" for i in range(n_queues)]
    C["q_name"] = np.asarray([st.add(q) for q in qn], dtype=np.int32)
    C["q_weight"] = np.arange(1, n_queues + 1, dtype=np.int32)
    C["q_ts"] = np.zeros(n_queues, dtype=np.int64)

    # nodes
    sku = rng.choice(len(SKUS), size=n_nodes, p=SKU_P)
    sk = np.asarray(SKUS, dtype=np.int64)
    C["n_name"] = st.add_bulk_unique([f"n{i:07d}" for i in range(n_nodes)])
    for j, k in enumerate(("cpu", "mem", "gpu")):
        C[f"n_alloc_{k}"] = sk[sku, j].copy()
        C[f"n_cap_{k}"] = sk[sku, j].copy()
    C["n_alloc_pods"] = np.full(n_nodes, 110, dtype=np.int64)
    C["n_cap_pods"] = np.full(n_nodes, 110, dtype=np.int64)
    C["n_unsched"] = np.zeros(n_nodes, dtype=np.uint8)
    C["n_label_off"] = np.zeros(n_nodes + 1, dtype=np.int32)
    C["n_taint_off"] = np.zeros(n_nodes + 1, dtype=np.int32)

    # running pods: running_per_node[i] pods on node i, grouped into running jobs
    r_node = np.repeat(np.arange(n_nodes), running_per_node)
    n_run = int(r_node.size)
    r_cpu = rng.choice(CPU_CHOICES, size=n_run)
    r_mem = rng.choice(MEM_CHOICES, size=n_run)
    if run_res is not None:  # caller-chosen running requests (gen_c5: within each node's allocatable)
        r_cpu, r_mem = run_res(r_node)
    n_rjobs = (n_run + running_gang - 1) // running_gang
    r_job = np.arange(n_run) // running_gang

    # pending gang jobs: tasks/job = minMember ~ U[gang_lo, gang_hi]
    sizes = []
    total = 0
    while total < n_pending:
        s = int(rng.integers(gang_lo, gang_hi + 1))
        s = min(s, n_pending - total)
        sizes.append(s)
        total += s
    sizes = np.asarray(sizes, dtype=np.int64)
    n_pjobs = sizes.size
    pj_cpu = rng.choice(CPU_CHOICES, size=n_pjobs)
    pj_mem = rng.choice(MEM_CHOICES, size=n_pjobs)
    pj_gpu = rng.choice(GPU_CHOICES, size=n_pjobs, p=GPU_P)
    pj_pri = np.where(rng.random(n_pjobs) < 0.1, 100, 0).astype(np.int32)
    pj_ts = (np.arange(n_pjobs, dtype=np.int64) // 3) * SEC + SEC  # ties of 3 -> UID order
    pj_q = rng.integers(0, n_queues, size=n_pjobs)
    p_job_local = np.repeat(np.arange(n_pjobs), sizes)

    # jobs: pending "jp%07d" sort before running "jr%07d"
    jnames = [f"jp{i:07d}" for i in range(n_pjobs)] + [f"jr{i:07d}" for i in range(n_rjobs)]
    J = len(jnames)
    C["j_ns"] = np.full(J, st.add("default"), dtype=np.int32)
    C["j_name"] = st.add_bulk_unique(jnames)
    qoff = np.asarray([st.add(q) for q in qn], dtype=np.int32)
    rj_q = rng.integers(0, n_queues, size=n_rjobs)
    C["j_queue"] = np.concatenate([qoff[pj_q], qoff[rj_q]]).astype(np.int32)
    rj_sizes = np.bincount(r_job, minlength=n_rjobs).astype(np.int32) if n_run else np.zeros(0, np.int32)
    C["j_min"] = np.concatenate([sizes.astype(np.int32), rj_sizes]).astype(np.int32)
    C["j_pg_priority"] = np.zeros(J, dtype=np.int32)
    C["j_ts"] = np.concatenate([pj_ts, np.zeros(n_rjobs, dtype=np.int64)])

    # pods: running "r%08d" sort before pending "u%08d"
    P = n_run + n_pending
    uids = [f"r{i:08d}" for i in range(n_run)] + [f"u{i:08d}" for i in range(n_pending)]
    C["p_uid"] = st.add_bulk_unique(uids)
    C["p_name"] = C["p_uid"]
    C["p_ns"] = np.full(P, st.add("default"), dtype=np.int32)
    C["p_job"] = np.concatenate([n_pjobs + r_job, p_job_local]).astype(np.int32)
    node_name_off = C["n_name"]
    C["p_node"] = np.concatenate([node_name_off[r_node], np.full(n_pending, -1, np.int32)]).astype(np.int32)
    C["p_phase"] = np.concatenate([np.full(n_run, 1, np.uint8), np.zeros(n_pending, np.uint8)])
    C["p_deleting"] = np.zeros(P, dtype=np.uint8)
    C["p_backfill"] = np.zeros(P, dtype=np.uint8)
    C["p_priority"] = np.concatenate([np.zeros(n_run, np.int32), pj_pri[p_job_local]]).astype(np.int32)
    C["p_ts"] = np.concatenate([np.zeros(n_run, np.int64), pj_ts[p_job_local]])
    z = np.zeros(P + 1, dtype=np.int32)
    C["p_label_off"] = z
    C["p_nsel_off"] = z
    C["p_ictr_off"] = z
    C["p_tol_off"] = z
    C["p_ctr_off"] = np.arange(P + 1, dtype=np.int32)
    C["c_cpu"] = np.concatenate([r_cpu, pj_cpu[p_job_local]]).astype(np.int64)
    C["c_mem"] = np.concatenate([r_mem, pj_mem[p_job_local]]).astype(np.int64)
    C["c_gpu"] = np.concatenate([np.zeros(n_run, np.int64), pj_gpu[p_job_local]]).astype(np.int64)
    C["c_has"] = np.full(P, HAS_CPU | HAS_MEM | HAS_GPU, dtype=np.uint8)
    C["c_port_off"] = np.zeros(P + 1, dtype=np.int32)
    C["p_aff"] = np.full(P, -1, dtype=np.int32)
    meta = dict(nodes=n_nodes, pending=n_pending, running=n_run, jobs=J, pending_jobs=n_pjobs)
    return C, st, meta


def gen_c2(path: str, seed: int = BASE_SEED + 2, n_nodes: int = 5000, n_pending: int = 50000) -> dict:
    """C2: 5k nodes x 50k pending pods in gang jobs, 20% of nodes pre-filled."""
    rng = np.random.default_rng(seed + 1000)
    rpn = np.where(rng.random(n_nodes) < 0.2, rng.integers(1, 5, size=n_nodes), 0)
    C, st, meta = _bulk(n_nodes, n_pending, rpn, seed)
    write_kbs(path, C, st)
    return meta


def gen_c4(path: str, seed: int = BASE_SEED + 4, n_nodes: int = 100_000,
           n_pending: int = 800_000, running_per_node: int = 2) -> dict:
    """C4: 100k nodes x 1M pods (200k Running pre-placed, 2/node; 800k pending)."""
    rpn = np.full(n_nodes, running_per_node, dtype=np.int64)
    C, st, meta = _bulk(n_nodes, n_pending, rpn, seed)
    write_kbs(path, C, st)
    return meta


def gen_c3(seed: int = BASE_SEED + 3, n_nodes: int = 20_000, n_pending: int = 50_000,
           n_queues: int = 8, keyless: float = 0.0, pod_affinity: float = 0.0, ipa: float = 0.0) -> Cluster:
    """C3: labels, taints/tolerations, selectors, zone anti-affinity, 8 queues.

    Hardening options (0 = the C3 of the bench; they draw from a second
    generator so the default stream is unchanged): ``keyless`` — the share of
    nodes without the zone label (topology-keyless nodes: a pod-affinity term
    by zone never matches there, predicates.go:1402-1458); ``pod_affinity`` —
    the share of gangs with a required pod-affinity term by zone to their own
    job (self-affine: the first pod goes anywhere, the rest follow it);
    ``ipa`` — the share of gangs with preferred inter-pod affinity / anti-
    affinity terms (interpod_affinity.go:119-240)."""
    rng = np.random.default_rng(seed)
    rng2 = np.random.default_rng(seed + 7919)
    c = Cluster()
    zones = [f"z{i:02d}" for i in range(48)]
    itypes = ["it-a", "it-b", "it-c", "it-d"]
    for i in range(n_nodes):
        s = SKUS[rng.choice(3, p=SKU_P)]
        name = f"n{i:07d}"
        labels = {"zone": zones[int(rng.integers(48))], "rack": f"r{i // 40:04d}",
                  "instance-type": itypes[int(rng.integers(4))],
                  "gen": str(int(rng.integers(1, 6))), "kubernetes.io/hostname": name}
        if keyless and rng2.random() < keyless:
            del labels["zone"]
        taints = [("dedicated", "gpu", "NoSchedule")] if rng.random() < 0.1 else []
        c.add_node(name, s[0], s[1], s[2], 110, labels=labels, taints=taints)
    for q in range(n_queues):
        c.add_queue(f"q{q}", q + 1)
    total, j = 0, 0
    while total < n_pending:
        size = min(int(rng.integers(8, 65)), n_pending - total)
        jn = f"jp{j:07d}"
        pri = 100 if rng.random() < 0.1 else 0
        ts = (j // 3 + 1) * SEC
        c.add_job("default", jn, f"q{int(rng.integers(n_queues))}", min_member=size, ts=ts)
        r = res(int(rng.choice(CPU_CHOICES)), int(rng.choice(MEM_CHOICES)),
                int(rng.choice(GPU_CHOICES, p=GPU_P)))
        nsel = {"instance-type": itypes[int(rng.integers(4))]} if rng.random() < 0.3 else {}
        tols = [{"key": "dedicated", "op": "Equal", "value": "gpu", "effect": "NoSchedule"}] \
            if rng.random() < 0.1 else []
        aff = None
        if rng.random() < 0.25:
            aff = {"anti": {"required": [{"selector": {"ml": {"job": jn}}, "topology_key": "zone"}]}}
        if rng.random() < 0.15:
            aff = dict(aff or {})
            aff["node"] = {"preferred": [(10, {"expr": [("gen", "Gt", ["3"])]}),
                                         (5, {"expr": [("zone", "In", zones[:8])]})]}
        if pod_affinity and rng2.random() < pod_affinity:
            aff = dict(aff or {})
            aff["pod"] = {"required": [{"selector": {"ml": {"job": jn}}, "topology_key": "zone"}]}
        if ipa and rng2.random() < ipa:
            aff = dict(aff or {})
            other = f"jp{int(rng2.integers(max(1, j))):07d}"
            aff["pod"] = dict(aff.get("pod") or {})
            aff["pod"]["preferred"] = [(int(rng2.integers(1, 50)),
                                        {"selector": {"ml": {"job": other}}, "topology_key": "zone"})]
            aff["anti"] = dict(aff.get("anti") or {})
            aff["anti"]["preferred"] = [(int(rng2.integers(1, 20)),
                                         {"selector": {"ml": {"job": jn}}, "topology_key": "rack"})]
        for k in range(size):
            c.add_pod("default", f"{jn}-{k:03d}", uid=f"u{total + k:08d}", group=jn, priority=pri, ts=ts,
                      labels={"job": jn}, containers=[dict(r)], node_selector=dict(nsel),
                      tolerations=list(tols), affinity=aff)
        total += size
        j += 1
    return c


def gen_random(seed: int, n_nodes: int = 8, n_jobs: int = 6, max_tasks: int = 5,
               features: Sequence[str] = ("labels", "taints", "ports", "affinity", "init",
                                          "running", "releasing", "backfill", "selector", "nodeaffinity",
                                          "podaffinity", "unsched", "bestEffort"),
               tiers=None, n_queues: int = 2, best_effort_p: float = 0.1, keyless: float = 0.0) -> Cluster:
    """Small random cluster exercising every feature of the hot path (parity tests).

    ``keyless``: the share of nodes without the zone label (a second generator:
    the default stream is unchanged)."""
    rng = np.random.default_rng(seed)
    rng2 = np.random.default_rng(seed + 7919)
    f = set(features)
    c = Cluster(tiers=tiers)
    zones = ["za", "zb", "zc"]
    itypes = ["small", "big"]
    for i in range(n_nodes):
        name = f"n{i:03d}"
        labels = {}
        if "labels" in f:
            labels = {"zone": zones[int(rng.integers(3))], "kubernetes.io/hostname": name}
            if keyless and rng2.random() < keyless:
                del labels["zone"]
            if rng.random() < 0.8:
                labels["itype"] = itypes[int(rng.integers(2))]
            if rng.random() < 0.7:
                labels["gen"] = str(int(rng.integers(1, 5)))
        taints = []
        if "taints" in f and rng.random() < 0.3:
            taints.append(("dedicated", ["a", "b"][int(rng.integers(2))],
                           ["NoSchedule", "NoExecute", "PreferNoSchedule"][int(rng.integers(3))]))
        cpu = int(rng.choice([2000, 4000, 8000]))
        mem = int(rng.choice([4, 8, 16])) * GI
        gpu = int(rng.choice([0, 0, 4000]))
        pods = int(rng.choice([3, 6, 110]))
        c.add_node(name, cpu, mem, gpu, pods, labels=labels, taints=taints,
                   unschedulable=("unsched" in f and rng.random() < 0.1))
    for q in range(n_queues):
        c.add_queue(f"q{q}", int(rng.integers(1, 4)), ts=int(rng.integers(0, 2)) * SEC)
    node_names = [n.name for n in c.nodes]
    uid = 0

    def rand_res():
        r = {}
        if rng.random() < 0.9:
            r["cpu"] = int(rng.choice([0, 250, 500, 1000, 1500]))
        if rng.random() < 0.9:
            r["mem"] = int(rng.choice([0, 256 * MI, GI, 2 * GI]))
        if rng.random() < 0.2:
            r["gpu"] = int(rng.choice([0, 1000, 2000]))
        return r

    def rand_sel(jn):
        me = []
        if rng.random() < 0.5:
            me.append(("app", ["In", "NotIn", "Exists", "DoesNotExist"][int(rng.integers(4))],
                       [] if rng.random() < 0.3 else ["x", "y"]))
        ml = {"job": jn} if rng.random() < 0.6 else {"app": ["x", "y"][int(rng.integers(2))]}
        # fix operator arity so selectors stay valid
        me = [(k, op, ([] if op in ("Exists", "DoesNotExist") else (vs or ["x"]))) for (k, op, vs) in me]
        return {"ml": ml, "me": me}

    for j in range(n_jobs):
        jn = f"j{j:03d}"
        ntask = int(rng.integers(1, max_tasks + 1))
        jq = f"q{int(rng.integers(n_queues))}"
        jts = int(rng.integers(0, 3)) * SEC
        pri = int(rng.choice([0, 0, 10]))
        c.add_job("ns1" if j % 2 else "ns2", jn, jq, min_member=int(rng.integers(0, ntask + 1)), ts=jts)
        ns = "ns1" if j % 2 else "ns2"
        for k in range(ntask):
            phase, node, deleting = "Pending", None, False
            if "running" in f and rng.random() < 0.35:
                phase, node = "Running", node_names[int(rng.integers(n_nodes))]
                if "releasing" in f and rng.random() < 0.3:
                    deleting = True
            ctrs = [rand_res()]
            if rng.random() < 0.3:
                ctrs.append(rand_res())
            if "bestEffort" in f and rng.random() < best_effort_p:
                ctrs = [{}]
            if "ports" in f and rng.random() < 0.2:
                ctrs[0]["ports"] = [{"port": int(rng.choice([80, 8080])),
                                     "ip": ["", "10.0.0.1"][int(rng.integers(2))],
                                     "proto": ["", "TCP", "UDP"][int(rng.integers(3))]}]
            inits = [rand_res()] if ("init" in f and rng.random() < 0.2) else []
            nsel = {}
            if "selector" in f and rng.random() < 0.2:
                nsel = {"itype": itypes[int(rng.integers(2))]}
            tols = []
            if "taints" in f and rng.random() < 0.4:
                tols.append({"key": "dedicated", "op": ["Equal", "Exists", ""][int(rng.integers(3))],
                             "value": ["a", "b"][int(rng.integers(2))],
                             "effect": ["", "NoSchedule", "NoExecute"][int(rng.integers(3))]})
                if tols[-1]["op"] == "Exists":
                    tols[-1]["value"] = ""
            aff = None
            if "nodeaffinity" in f and rng.random() < 0.25:
                ops = [("gen", "Gt", ["1"]), ("gen", "Lt", ["3"]), ("zone", "In", ["za", "zb"]),
                       ("itype", "NotIn", ["big"]), ("itype", "Exists", []), ("gen", "DoesNotExist", [])]
                req = None
                if rng.random() < 0.6:
                    req = [{"expr": [ops[int(rng.integers(len(ops)))]]}]
                    if rng.random() < 0.3:
                        req.append({"fields": [("metadata.name", "In", [node_names[int(rng.integers(n_nodes))]])]})
                    if rng.random() < 0.1:
                        req.append({})
                pref = [(int(rng.integers(0, 20)), {"expr": [ops[int(rng.integers(len(ops)))]]})
                        for _ in range(int(rng.integers(0, 3)))]
                aff = {"node": {"required": req, "preferred": pref}}
            if "podaffinity" in f and rng.random() < 0.35:
                aff = dict(aff or {})
                kind = int(rng.integers(3))
                tk = ["zone", "kubernetes.io/hostname"][int(rng.integers(2))]
                term = {"selector": rand_sel(jn), "topology_key": tk}
                if rng.random() < 0.3:
                    term["namespaces"] = ["ns1"]
                if kind == 0:
                    aff["pod"] = {"required": [term] if rng.random() < 0.6 else [],
                                  "preferred": [(int(rng.integers(1, 10)), term)] if rng.random() < 0.6 else []}
                elif kind == 1:
                    aff["anti"] = {"required": [term] if rng.random() < 0.6 else [],
                                   "preferred": [(int(rng.integers(1, 10)), term)] if rng.random() < 0.6 else []}
                else:
                    aff["pod"] = {"preferred": [(int(rng.integers(1, 10)), term)]}
                    aff["anti"] = {"required": [dict(term, selector=rand_sel(jn))]}
            labels = {"job": jn}
            if rng.random() < 0.5:
                labels["app"] = ["x", "y"][int(rng.integers(2))]
            c.add_pod(ns, f"{jn}-{k}", uid=f"u{uid:05d}", group=jn, node=node, phase=phase,
                      deleting=deleting, priority=pri, ts=jts + int(rng.integers(0, 2)) * SEC,
                      backfill=("backfill" in f and node is not None and rng.random() < 0.3),
                      labels=labels, containers=ctrs, init_containers=inits, node_selector=nsel,
                      tolerations=tols, affinity=aff)
            uid += 1
    return c


def gen_preempt(seed: int, n_nodes: int = 8, n_queues: int = 3, n_run_jobs: int = 6, n_pend_jobs: int = 4,
                max_tasks: int = 5, tiers=None, fill: float = 0.9, features: Sequence[str] = ()) -> Cluster:
    """Random cluster for the reclaim / preempt actions (SURVEY §3.5, config C5 in
    miniature): nodes mostly filled with Running pods of low-priority jobs spread over
    queues of unequal weight (so some queues sit above their proportion share),
    pending higher-priority jobs, gang sizes that make some victims protected, some
    kube-system / system-critical pods (conformance), releasing and backfill pods.
    Features: "selector", "taints", "ports", "init", "bestEffort", "unsched", "podaffinity"
    (zone labels; running and pending pods with app labels and required / preferred pod
    (anti-)affinity terms by zone or hostname)."""
    rng = np.random.default_rng(seed)
    f = set(features)
    c = Cluster(tiers=tiers)
    zones = ["za", "zb", "zc"]
    for i in range(n_nodes):
        name = f"n{i:03d}"
        taints = []
        if "taints" in f and rng.random() < 0.2:
            taints.append(("dedicated", "a", "NoSchedule"))
        labels = {"itype": ["small", "big"][int(rng.integers(2))], "kubernetes.io/hostname": name}
        c.add_node(name, int(rng.choice([4000, 8000])), int(rng.choice([8, 16])) * GI,
                   int(rng.choice([0, 0, 4000])), int(rng.choice([4, 110])),
                   labels=labels, taints=taints, unschedulable=("unsched" in f and rng.random() < 0.1))
        if "podaffinity" in f:
            labels["zone"] = zones[int(rng.integers(3))]

    def paff(own_job):
        """(labels, affinity) of a pod under the "podaffinity" feature."""
        labels = {"job": own_job}
        if rng.random() < 0.5:
            labels["app"] = ["x", "y"][int(rng.integers(2))]
        if rng.random() >= 0.45:
            return labels, None
        tk = ["zone", "kubernetes.io/hostname"][int(rng.integers(2))]
        sel = {"ml": {"app": ["x", "y"][int(rng.integers(2))]}} if rng.random() < 0.7 else {"ml": {"job": own_job}}
        term = {"selector": sel, "topology_key": tk}
        kind = int(rng.integers(4))
        if kind == 0:
            aff = {"anti": {"required": [term]}}
        elif kind == 1:
            aff = {"pod": {"required": [term]}}
        elif kind == 2:
            aff = {"pod": {"preferred": [(int(rng.integers(1, 10)), term)]}}
        else:
            aff = {"anti": {"preferred": [(int(rng.integers(1, 10)), term)], "required": [term]}}
        return labels, aff
    for q in range(n_queues):
        c.add_queue(f"q{q}", int(rng.integers(1, 5)), ts=int(rng.integers(0, 2)) * SEC)
    free = {n.name: [n.cpu, n.mem, n.gpu] for n in c.nodes}
    names = [n.name for n in c.nodes]
    uid = 0

    def rres():
        r = {"cpu": int(rng.choice([500, 1000, 2000])), "mem": int(rng.choice([1, 2, 4])) * GI}
        if rng.random() < 0.2:
            r["gpu"] = int(rng.choice([1000, 2000]))
        return r

    # running jobs: queue 0 gets the most (it is the one above its share)
    for j in range(n_run_jobs):
        jn, ns = f"r{j:03d}", ("kube-system" if rng.random() < 0.1 else "ns1")
        q = 0 if rng.random() < 0.6 else int(rng.integers(n_queues))
        ntask = int(rng.integers(1, max_tasks + 1))
        c.add_job(ns, jn, f"q{q}", min_member=int(rng.choice([1, max(1, ntask - 1), ntask])), ts=0)
        for k in range(ntask):
            r = rres()
            cands = [n for n in names if free[n][0] >= r["cpu"] and free[n][1] >= r["mem"]
                     and free[n][2] >= r.get("gpu", 0)]
            if not cands or rng.random() > fill:
                node, phase = None, "Pending"
            else:
                node, phase = cands[int(rng.integers(len(cands)))], "Running"
                free[node][0] -= r["cpu"]; free[node][1] -= r["mem"]; free[node][2] -= r.get("gpu", 0)
            pc = ["", "", "", "system-node-critical", "system-cluster-critical"][int(rng.integers(5))] \
                if rng.random() < 0.15 else ""
            labels, aff = paff(jn) if "podaffinity" in f else ({"job": jn}, None)
            c.add_pod(ns, f"{jn}-{k}", uid=f"u{uid:05d}", group=jn, node=node, phase=phase,
                      deleting=(node is not None and rng.random() < 0.05), priority=int(rng.choice([0, 1])),
                      ts=int(rng.integers(0, 2)) * SEC, backfill=(node is not None and rng.random() < 0.1),
                      priority_class=pc, labels=labels, containers=[r], affinity=aff)
            uid += 1
    # pending preemptor jobs
    for j in range(n_pend_jobs):
        jn = f"p{j:03d}"
        q = int(rng.integers(n_queues))
        ntask = int(rng.integers(1, max_tasks + 1))
        pri = int(rng.choice([5, 10]))
        c.add_job("ns2", jn, f"q{q}", min_member=int(rng.choice([0, 1, ntask])), ts=int(rng.integers(1, 3)) * SEC,
                  pg_priority=pri)
        for k in range(ntask):
            ctrs = [rres()]
            if "bestEffort" in f and rng.random() < 0.1:
                ctrs = [{}]
            if "ports" in f and rng.random() < 0.2:
                ctrs[0]["ports"] = [{"port": 80, "ip": "", "proto": ""}]
            inits = [rres()] if ("init" in f and rng.random() < 0.2) else []
            nsel = {"itype": "big"} if ("selector" in f and rng.random() < 0.2) else {}
            tols = [{"key": "dedicated", "op": "Exists", "value": "", "effect": ""}] \
                if ("taints" in f and rng.random() < 0.5) else []
            labels, aff = paff(jn) if "podaffinity" in f else ({"job": jn}, None)
            c.add_pod("ns2", f"{jn}-{k}", uid=f"u{uid:05d}", group=jn, priority=pri,
                      ts=int(rng.integers(1, 3)) * SEC, labels=labels, containers=ctrs,
                      init_containers=inits, node_selector=nsel, tolerations=tols, affinity=aff)
            uid += 1
    return c


def gen_c5(path: str, seed: int = BASE_SEED + 5, n_nodes: int = 50_000, n_pending: int = 2000, n_queues: int = 4,
           fill: float = 0.9, backfill_frac: float = 0.05, best_effort: int = 200, run_min1: float = 0.5) -> dict:
    """C5: a what-if session for reclaim / allocate / backfill / preempt.
    Nodes of the C2 SKU mix filled with Running pods up to ~`fill` of their cpu and
    memory (a prefix of random C2-sized pods per node), 5 % of them backfill-annotated;
    running jobs of 8 pods spread over `n_queues` queues (weights 1..n), half of them
    with minMember 1 (their pods are gang-preemptable); `n_pending` pending tasks of
    priority-100 jobs (minMember = size / 1 / 0), the last `best_effort` of them BestEffort.
    Each seed is one session's pending set (the S what-if sessions differ by seed)."""
    rng0 = np.random.default_rng(seed)  # _bulk's first draw: the node SKUs
    sku = rng0.choice(len(SKUS), size=n_nodes, p=SKU_P)
    sk = np.asarray(SKUS, dtype=np.int64)
    rng = np.random.default_rng(seed + 2000)
    K = 64
    cpu = rng.choice(CPU_CHOICES, size=(n_nodes, K))
    mem = rng.choice(MEM_CHOICES, size=(n_nodes, K))
    ok = (np.cumsum(cpu, axis=1) <= fill * sk[sku, 0][:, None]) & (np.cumsum(mem, axis=1) <= fill * sk[sku, 1][:, None])
    rpn = np.minimum(ok.cumprod(axis=1).sum(axis=1), 100).astype(np.int64)  # pods cap 110
    keep = np.arange(K)[None, :] < rpn[:, None]
    run_cpu, run_mem = cpu[keep], mem[keep]  # row-major = node order, matching _bulk's r_node

    def run_res(r_node):
        assert r_node.size == run_cpu.size
        return run_cpu, run_mem

    C, st, meta = _bulk(n_nodes, n_pending, rpn, seed, n_queues=n_queues, run_res=run_res)
    n_run, n_pjobs = meta["running"], meta["pending_jobs"]
    n_rjobs = meta["jobs"] - n_pjobs
    C["p_backfill"][:n_run] = (rng.random(n_run) < backfill_frac).astype(np.uint8)
    C["p_priority"][n_run:] = 100
    C["p_priority"][:n_run] = 0
    C["j_pg_priority"][:n_pjobs] = 100
    jmin = C["j_min"]
    jmin[n_pjobs:] = np.where(rng.random(n_rjobs) < run_min1, 1, jmin[n_pjobs:])
    pick = rng.random(n_pjobs)
    jmin[:n_pjobs] = np.where(pick < 0.15, 0, np.where(pick < 0.3, 1, jmin[:n_pjobs]))
    if best_effort:
        be = np.arange(n_run + n_pending - best_effort, n_run + n_pending)
        for k in ("c_cpu", "c_mem", "c_gpu"):
            C[k][be] = 0
        C["c_has"][be] = 0
    write_kbs(path, C, st)
    meta.update(running_per_node=float(rpn.mean()), backfill_pods=int(C["p_backfill"].sum()), rpn=rpn)
    return meta
