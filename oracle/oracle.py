"""TEST ORACLE bindings (test infrastructure only).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this module, and only as the checker / CPU baseline — never as the measured or
shipped path.  The product library (kube-batch-1_amd/) must not import it.

Two restatements of kube-batch's allocate action live next to this file:

* ``kbref`` (kbref.cpp) — faithful: structured like the Go code, per-pair
  recomputation; small snapshots only.
* ``kbfast`` (kbfast.cpp) — hoisted: identical placements, per-task precompute
  and an O(N) multi-threaded sweep; the CPU baseline.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import Dict, List, Optional, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
BUILD = os.path.join(HERE, "_build")

# ref::TaskStatus codes (pkg/scheduler/api/types.go:22-61)
PENDING, ALLOCATED_OVER_BACKFILL, ALLOCATED, PIPELINED = 1, 2, 4, 8
BINDING, BOUND, RUNNING, RELEASING = 16, 32, 64, 128
SUCCEEDED, FAILED, UNKNOWN = 256, 512, 1024
READY, ALMOST_READY, NOT_READY = 1, 2, 4

_libs: Dict[str, ctypes.CDLL] = {}


def build() -> None:
    """Compile the oracle libraries (gcc only; no GPU)."""
    subprocess.run(["make", "-s", "-C", HERE, "all"], check=True)


def _lib(name: str) -> ctypes.CDLL:
    if name not in _libs:
        path = os.path.join(BUILD, f"lib{name}.so")
        if not os.path.exists(path):
            build()
        lib = ctypes.CDLL(path)
        _libs[name] = lib
    return _libs[name]


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


class Placement:
    """Placements in decision order: (pod index, node index, status code)."""

    def __init__(self, pod: np.ndarray, node: np.ndarray, status: np.ndarray):
        self.pod, self.node, self.status = pod, node, status

    def __len__(self):
        return int(self.pod.size)

    def as_list(self) -> List[Tuple[int, int, int]]:
        return list(zip(self.pod.tolist(), self.node.tolist(), self.status.tolist()))

    def kinds(self) -> np.ndarray:
        """1 = allocated (any Allocated* status), 2 = pipelined."""
        return np.where(self.status == PIPELINED, 2, 1).astype(np.int32)


def ref_allocate(path: str, cap: Optional[int] = None, with_nodes: bool = False, actions: str = "allocate"):
    """Faithful restatement: the conf actions (default: allocate only) on the
    snapshot; placement log in decision order."""
    lib = _lib("kbref")
    fn = lib.ref_allocate
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_char_p] + [ctypes.c_void_p] * 3 + [ctypes.c_int, ctypes.c_void_p, ctypes.c_char_p]
    cap = cap or 1 << 20
    pod = np.zeros(cap, np.int32)
    node = np.zeros(cap, np.int32)
    st = np.zeros(cap, np.int32)
    nstate = None
    if with_nodes:
        nstate = np.zeros((1 << 16, 12), np.float64)
    n = fn(path.encode(), _p(pod), _p(node), _p(st), cap, _p(nstate) if nstate is not None else None,
           actions.encode())
    if n < 0:
        lib.ref_last_error.restype = ctypes.c_char_p
        raise RuntimeError(lib.ref_last_error().decode())
    pl = Placement(pod[:n].copy(), node[:n].copy(), st[:n].copy())
    return (pl, nstate) if with_nodes else pl


def parse_gang_close(text: str) -> dict:
    """'<job uid>\\t<message>' lines -> {uid: message}."""
    out = {}
    for line in text.splitlines():
        if line:
            uid, msg = line.split("\t", 1)
            out[uid] = msg
    return out


def ref_gang_close(path: str, actions: str = "allocate") -> dict:
    """The gang plugin's OnSessionClose after the actions (gang.go:166-187):
    {job uid: Unschedulable condition message} for every job not Ready."""
    lib = _lib("kbref")
    fn = lib.ref_gang_close
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int]
    n = fn(path.encode(), actions.encode(), None, 0)
    if n < 0:
        lib.ref_last_error.restype = ctypes.c_char_p
        raise RuntimeError(lib.ref_last_error().decode())
    buf = ctypes.create_string_buffer(n + 1)
    fn(path.encode(), actions.encode(), buf, n + 1)
    return parse_gang_close(buf.value.decode())


def ref_open_nodes(path: str, n_nodes: int):
    lib = _lib("kbref")
    fn = lib.ref_open_nodes
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_void_p]
    st = np.zeros((n_nodes, 12), np.float64)
    acc = np.zeros((n_nodes, 3), np.float64)
    n = fn(path.encode(), _p(st), _p(acc))
    if n < 0:
        lib.ref_last_error.restype = ctypes.c_char_p
        raise RuntimeError(lib.ref_last_error().decode())
    return st[:n], acc[:n]


def ref_task_requests(path: str, n_pods: int) -> np.ndarray:
    lib = _lib("kbref")
    fn = lib.ref_task_requests
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_char_p, ctypes.c_void_p]
    out = np.zeros((n_pods, 6), np.float64)
    n = fn(path.encode(), _p(out))
    if n < 0:
        lib.ref_last_error.restype = ctypes.c_char_p
        raise RuntimeError(lib.ref_last_error().decode())
    return out[:n]


def ref_job_readiness(min_available: int, statuses: List[int]) -> int:
    lib = _lib("kbref")
    fn = lib.ref_job_readiness
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_int32, ctypes.c_void_p, ctypes.c_int]
    a = np.asarray(statuses, dtype=np.int32)
    return fn(min_available, _p(a), len(statuses))


def fast_allocate(path: str, threads: int = 16, cap: Optional[int] = None,
                  max_pops: int = -1, stats: Optional[dict] = None, actions: str = "allocate") -> Placement:
    """Hoisted restatement (CPU baseline).  ``max_pops`` bounds the number of
    job pops (a bounded sample of the session for timing)."""
    lib = _lib("kbfast")
    fn = lib.fast_allocate
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 3 + \
        [ctypes.c_int, ctypes.c_void_p, ctypes.c_char_p]
    cap = cap or (1 << 21)
    pod = np.zeros(cap, np.int32)
    node = np.zeros(cap, np.int32)
    st = np.zeros(cap, np.int32)
    tm = np.zeros(8, np.float64)
    n = fn(path.encode(), threads, max_pops, _p(pod), _p(node), _p(st), cap, _p(tm), actions.encode())
    if n < 0:
        lib.fast_last_error.restype = ctypes.c_char_p
        raise RuntimeError(lib.fast_last_error().decode())
    if stats is not None:
        stats.update(open_s=tm[0], allocate_s=tm[1], pops=int(tm[2]), tasks_tried=int(tm[3]),
                     load_s=tm[4])
    return Placement(pod[:n].copy(), node[:n].copy(), st[:n].copy())


def fast_allocate_sampled(path: str, log_pod, log_node, log_status, windows, threads: int = 16) -> dict:
    """Stratified timing of the hoisted allocate (bench.py's CPU baseline):
    the whole session runs, the tasks at positions [lo, hi) of the session's
    task sequence are swept for real and timed, every other task takes its decision from the given
    placement log (statuses ALLOCATED=4 / PIPELINED=8) without a sweep; the
    swept decisions are checked against the log (``mismatches``)."""
    lib = _lib("kbfast")
    fn = lib.fast_allocate_sampled
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 3 + \
        [ctypes.c_int] + [ctypes.c_void_p] * 3
    pod = np.ascontiguousarray(log_pod, np.int32)
    node = np.ascontiguousarray(log_node, np.int32)
    st = np.ascontiguousarray(log_status, np.int32)
    lo = np.ascontiguousarray([w[0] for w in windows], np.int32)
    hi = np.ascontiguousarray([w[1] for w in windows], np.int32)
    out = np.zeros(8, np.float64)
    if fn(path.encode(), threads, len(pod), _p(pod), _p(node), _p(st), len(lo), _p(lo), _p(hi), _p(out)) < 0:
        lib.fast_last_error.restype = ctypes.c_char_p
        raise RuntimeError(lib.fast_last_error().decode())
    return {"timed_s": out[0], "session_tasks": int(out[1]), "tasks_swept": int(out[2]), "placed": int(out[3]),
            "mismatches": int(out[4]), "session_pops": int(out[5]), "session_placements": int(out[6]),
            "load_s": out[7]}


def fast_trace_affinity(path: str, n_nodes: int, cap_tasks: int = 4096, actions: str = "allocate") -> dict:
    """Test support: run the hoisted restatement of the actions with a
    per-task trace.  For every task tried, in order: pod, result node (-1
    unassigned), status, per-node pod-affinity predicate verdict (ok), per-node
    raw inter-pod affinity count (raw), its [min, max] over nodes (lohi), flags
    (bit0 predicate error on every node, bit1 score error, bit2 IPA on), the
    per-node selection key the sweep implies (key: packed score / index /
    pipelined, 0 = not selectable) and the action (mode: 0 allocate, 1
    backfill)."""
    lib = _lib("kbfast")
    fn = lib.fast_trace_affinity
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 7 + [ctypes.c_char_p] + \
        [ctypes.c_void_p] * 2
    pod = np.zeros(cap_tasks, np.int32)
    node = np.zeros(cap_tasks, np.int32)
    st = np.zeros(cap_tasks, np.int32)
    ok = np.zeros((cap_tasks, n_nodes), np.uint8)
    raw = np.zeros((cap_tasks, n_nodes), np.float64)
    lohi = np.zeros((cap_tasks, 2), np.float64)
    flags = np.zeros(cap_tasks, np.uint8)
    key = np.zeros((cap_tasks, n_nodes), np.uint64)
    mode = np.zeros(cap_tasks, np.uint8)
    n = fn(path.encode(), cap_tasks, n_nodes, _p(pod), _p(node), _p(st), _p(ok), _p(raw), _p(lohi), _p(flags),
           actions.encode(), _p(key), _p(mode))
    if n < 0:
        lib.fast_last_error.restype = ctypes.c_char_p
        raise RuntimeError(lib.fast_last_error().decode())
    if n > cap_tasks:
        raise RuntimeError("trace larger than cap_tasks")
    return {"pod": pod[:n], "node": node[:n], "status": st[:n], "ok": ok[:n], "raw": raw[:n],
            "lohi": lohi[:n], "flags": flags[:n], "key": key[:n], "mode": mode[:n]}


def ref_sweep_scores(path: str, pod: int, n_nodes: int, actions: str = "") -> Tuple[int, np.ndarray]:
    """Faithful restatement of preempt()'s predicate + score sweep
    (preempt.go:270-287) for one task after the given actions: (passing nodes,
    per-node packed keys, 0 = node fails)."""
    lib = _lib("kbref")
    fn = lib.ref_sweep_scores
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_void_p]
    keys = np.zeros(max(n_nodes, 1), np.uint64)
    n = fn(path.encode(), actions.encode(), pod, _p(keys))
    if n < 0:
        lib.ref_last_error.restype = ctypes.c_char_p
        raise RuntimeError(lib.ref_last_error().decode())
    return n, keys[:n_nodes]
