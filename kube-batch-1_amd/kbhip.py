"""kbhip — Python binding of libkbhip.so (the MI355X placement engine).

This is the host-side mirror of the reference's plugin boundary for callers
that are not Go (tests, bench): it loads the in-tree ``_build/libkbhip.so`` and
exposes the C ABI of include/kbhip.h.  There is no fallback: if the library or
a gfx950 device is missing, calls raise ``KbhipError``.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import Optional, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("KBHIP_LIB") or os.path.join(HERE, "_build", "libkbhip.so")  # KBHIP_LIB: tuning builds

ALLOCATED, PIPELINED, EVICTED = 1, 2, 3
EV_DELETE, EV_SUCCEEDED, EV_FAILED = 1, 2, 3  # kbhip_session_carry_events
STOP_ALL, STOP_UNASSIGNED, STOP_READY = 0, 1, 2

# int kbhip_* entry points declared by include/kbhip.h
EXPORTS = ("kbhip_device_count", "kbhip_session_open", "kbhip_session_open_file", "kbhip_place_job",
           "kbhip_allocate", "kbhip_read_nodes", "kbhip_get_stats", "kbhip_set_option",
           "kbhip_session_close", "kbhip_last_error", "kbhip_debug_encode", "kbhip_debug_table",
           "kbhip_backfill", "kbhip_session_open_shard", "kbhip_shard_info", "kbhip_rccl_unique_id",
           "kbhip_shard_connect_rccl", "kbhip_shard_connect_host", "kbhip_debug_replay",
           "kbhip_gang_unschedulable", "kbhip_reclaim", "kbhip_preempt", "kbhip_session_carry",
           "kbhip_first_fit", "kbhip_sweep_scores", "kbhip_shard_connect_host_gather",
           "kbhip_session_carry_events", "kbhip_shard_connect_mailbox", "kbhip_shard_mailbox_fits", "kbhip_place_job_submit",
           "kbhip_place_job_wait", "kbhip_place_job_cancel", "kbhip_time_sweeps", "kbhip_time_rank_multi",
           "kbhip_session_carry_snapshot")

RED_MAX_U64, RED_MIN_I64, RED_MAX_I64, RED_SUM_I64 = 0, 1, 2, 3
ALLREDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int32,
                                ctypes.c_int32)
ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64)


class KbhipError(RuntimeError):
    pass


class Stats(ctypes.Structure):
    _fields_ = [("open_s", ctypes.c_double), ("allocate_s", ctypes.c_double), ("device_s", ctypes.c_double),
                ("pops", ctypes.c_int64), ("tasks", ctypes.c_int64), ("placed", ctypes.c_int64),
                ("sweeps", ctypes.c_int64), ("batched_pops", ctypes.c_int64), ("nodes", ctypes.c_int64),
                ("timed_launches", ctypes.c_int64), ("host_launch_s", ctypes.c_double),
                ("host_wait_s", ctypes.c_double), ("spec_hits", ctypes.c_int64), ("spec_missed", ctypes.c_int64),
                ("alloc_device_s", ctypes.c_double), ("unassigned_pops", ctypes.c_int64),
                ("collectives", ctypes.c_int64), ("rank_requests", ctypes.c_int64),
                ("rank_batch_sum", ctypes.c_int64), ("pop_requests", ctypes.c_int64),
                ("pop_batch_sum", ctypes.c_int64), ("comm_reused", ctypes.c_int64),
                ("async_launched", ctypes.c_int64), ("async_retracted", ctypes.c_int64),
                ("async_cancelled", ctypes.c_int64), ("sweep_requests", ctypes.c_int64),
                ("sweep_batch_sum", ctypes.c_int64), ("score_sweep_s", ctypes.c_double),
                ("score_sweeps", ctypes.c_int64), ("pertask_sweeps", ctypes.c_int64),
                ("seq_launches", ctypes.c_int64), ("seq_cut", ctypes.c_int64), ("seq_none", ctypes.c_int64),
                ("evict_rank_s", ctypes.c_double), ("evict_walk_s", ctypes.c_double),
                ("evict_visits", ctypes.c_int64), ("evict_cands", ctypes.c_int64), ("fit_syncs", ctypes.c_int64),
                ("alloc_setup_s", ctypes.c_double), ("evict_setup_s", ctypes.c_double),
                ("engine_pops", ctypes.c_int64), ("engine_launches", ctypes.c_int64),
                ("engine_workers", ctypes.c_int64), ("engine_owners", ctypes.c_int64),
                ("engine_not_resident", ctypes.c_int64)]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}


_lib: Optional[ctypes.CDLL] = None


def build() -> str:
    """Compile libkbhip.so for gfx950 in-tree (hipcc cross-compiles without a GPU)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise KbhipError(f"{LIB_PATH} is missing: run kbhip.build() (no CPU fallback exists)")
        L = ctypes.CDLL(LIB_PATH)
        vp, i32, i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
        L.kbhip_last_error.restype = ctypes.c_char_p
        L.kbhip_device_count.restype = ctypes.c_int
        L.kbhip_session_open.argtypes = [vp, ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(vp)]
        L.kbhip_session_open_file.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(vp)]
        L.kbhip_place_job.argtypes = [vp, vp, i32, i32, i32, i32, vp, vp, vp, vp]
        L.kbhip_place_job_submit.argtypes = [vp, vp, i32, i32, i32, i32]
        L.kbhip_place_job_submit.restype = i64
        L.kbhip_place_job_wait.argtypes = [vp, i64, vp, vp, vp, vp]
        L.kbhip_place_job_cancel.argtypes = [vp, i64]
        L.kbhip_allocate.argtypes = [vp, vp, vp, vp, i64]
        L.kbhip_backfill.argtypes = [vp, vp, vp, vp, i64]
        L.kbhip_first_fit.argtypes = [vp, vp, i32, vp]
        L.kbhip_sweep_scores.argtypes = [vp, i32, vp]
        L.kbhip_time_sweeps.argtypes = [vp, vp, i32, vp]
        L.kbhip_time_rank_multi.argtypes = [vp, i32, vp, i32, i32, i32, vp]
        L.kbhip_reclaim.argtypes = [vp, vp, vp, vp, i64]
        L.kbhip_session_carry.argtypes = [vp, vp]
        L.kbhip_session_carry_events.argtypes = [vp, vp, vp, i64, vp]
        L.kbhip_session_carry_snapshot.argtypes = [vp, vp, ctypes.c_size_t, vp, vp, vp]
        L.kbhip_preempt.argtypes = [vp, vp, vp, vp, i64]
        L.kbhip_session_open_shard.argtypes = [vp, ctypes.c_size_t, ctypes.c_int, i32, i32, ctypes.POINTER(vp)]
        L.kbhip_shard_info.argtypes = [vp, vp]
        L.kbhip_rccl_unique_id.argtypes = [vp, i64]
        L.kbhip_shard_connect_rccl.argtypes = [vp, vp, i64]
        L.kbhip_shard_connect_host.argtypes = [vp, ALLREDUCE_FN, vp]
        L.kbhip_shard_connect_host_gather.argtypes = [vp, ALLGATHER_FN, vp]
        L.kbhip_shard_connect_mailbox.argtypes = [vp, ALLGATHER_FN, vp]
        L.kbhip_shard_mailbox_fits.argtypes = [ctypes.c_int32, ctypes.c_int32]
        L.kbhip_shard_mailbox_fits.restype = ctypes.c_int
        L.kbhip_read_nodes.argtypes = [vp, vp, i64]
        L.kbhip_get_stats.argtypes = [vp, ctypes.POINTER(Stats)]
        L.kbhip_set_option.argtypes = [vp, ctypes.c_char_p, i64]
        L.kbhip_session_close.argtypes = [vp]
        L.kbhip_debug_encode.argtypes = [vp, ctypes.c_size_t, ctypes.POINTER(vp)]
        L.kbhip_debug_table.argtypes = [vp, ctypes.c_char_p, vp, i64]
        L.kbhip_debug_table.restype = i64
        L.kbhip_gang_unschedulable.argtypes = [vp, ctypes.c_char_p, i64]
        L.kbhip_gang_unschedulable.restype = i64
        L.kbhip_debug_replay.argtypes = [vp, i32, vp, vp, vp, vp, vp]
        _lib = L
    return _lib


def _check(rc: int) -> int:
    if rc < 0:
        raise KbhipError(f"kbhip error {rc}: {lib().kbhip_last_error().decode()}")
    return rc


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def device_count() -> int:
    return _check(lib().kbhip_device_count())


class Session:
    """One scheduling session on one GPU (framework.Session equivalent)."""

    def __init__(self, snapshot, device: int = 0):
        self._h = ctypes.c_void_p()
        if isinstance(snapshot, (bytes, bytearray, memoryview)):
            buf = bytes(snapshot)
            _check(lib().kbhip_session_open(ctypes.c_char_p(buf), len(buf), device, ctypes.byref(self._h)))
        else:
            _check(lib().kbhip_session_open_file(str(snapshot).encode(), device, ctypes.byref(self._h)))

    def close(self) -> None:
        if self._h:
            _check(lib().kbhip_session_close(self._h))
            self._h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_option(self, key: str, value: int) -> None:
        _check(lib().kbhip_set_option(self._h, key.encode(), int(value)))

    def allocate(self, cap: int = 1 << 21) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        """Run allocateAction.Execute; returns (pod, node, kind) in decision order."""
        pod = np.zeros(cap, np.int32)
        node = np.zeros(cap, np.int32)
        kind = np.zeros(cap, np.uint8)
        n = _check(lib().kbhip_allocate(self._h, _p(pod), _p(node), _p(kind), cap))
        if n > cap:
            raise KbhipError("placement log larger than cap")
        return pod[:n].copy(), node[:n].copy(), kind[:n].copy()

    def _action(self, fn, cap: int) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        pod = np.zeros(cap, np.int32)
        node = np.zeros(cap, np.int32)
        kind = np.zeros(cap, np.uint8)
        n = _check(fn(self._h, _p(pod), _p(node), _p(kind), cap))
        if n > cap:
            raise KbhipError("placement log larger than cap")
        return pod[:n].copy(), node[:n].copy(), kind[:n].copy()

    def backfill(self, cap: int = 1 << 21) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        """Run backfillAction.Execute on the current session state."""
        return self._action(lib().kbhip_backfill, cap)

    def first_fit(self, task_ids) -> np.ndarray:
        """kbhip_first_fit: backfill.go:51-65 for the given pending tasks, in
        order (lowest-index node passing the predicates, Session.Allocate);
        returns the node per task (-1: none)."""
        ids = np.ascontiguousarray(task_ids, dtype=np.int32)
        out = np.full(max(ids.size, 1), -1, np.int32)
        _check(lib().kbhip_first_fit(self._h, _p(ids), ids.size, _p(out)))
        return out[: ids.size].copy()

    def sweep_scores(self, task_id: int, n_nodes: int, keys: bool = True) -> Tuple[int, np.ndarray]:
        """kbhip_sweep_scores: preempt.go:270-287's predicate + score sweep of
        one task: (passing nodes, per-node packed keys; 0 = node fails).
        keys=False: the count only (no copy of the keys)."""
        if not keys:
            return _check(lib().kbhip_sweep_scores(self._h, int(task_id), None)), np.zeros(0, np.uint64)
        out = np.zeros(max(n_nodes, 1), np.uint64)
        n = _check(lib().kbhip_sweep_scores(self._h, int(task_id), _p(out)))
        return n, out[:n_nodes].copy()

    def time_sweeps(self, task_ids) -> float:
        """kbhip_time_sweeps: device time per launch (us) of the standalone sweep,
        one launch per task, back to back."""
        ids = np.ascontiguousarray(task_ids, dtype=np.int32)
        out = np.zeros(1, np.float64)
        _check(lib().kbhip_time_sweeps(self._h, _p(ids), ids.size, _p(out)))
        return float(out[0])

    def carry(self) -> int:
        """kbhip_session_carry: become the next session (binds / evictions applied); bytes uploaded."""
        out = np.zeros(1, np.int64)
        _check(lib().kbhip_session_carry(self._h, _p(out)))
        return int(out[0])

    def carry_events(self, pods, events) -> int:
        """kbhip_session_carry_events: carry, then the cache's events on existing pods
        (EV_DELETE / EV_SUCCEEDED / EV_FAILED per pod index); bytes uploaded."""
        p = np.ascontiguousarray(pods, np.int32)
        e = np.ascontiguousarray(events, np.uint8)
        if p.shape != e.shape:
            raise ValueError("pods and events differ in length")
        out = np.zeros(1, np.int64)
        _check(lib().kbhip_session_carry_events(self._h, _p(p), _p(e), int(p.size), _p(out)))
        return int(out[0])

    def carry_snapshot(self, snapshot, old_pod, old_node) -> int:
        """kbhip_session_carry_snapshot: become the session of the cache's next
        snapshot (KBS1 bytes or a path); old_pod / old_node map its pods / nodes
        to this session's indices (-1: new).  Bytes uploaded (-1: re-opened)."""
        if not isinstance(snapshot, (bytes, bytearray, memoryview)):
            with open(snapshot, "rb") as f:
                snapshot = f.read()
        buf = bytes(snapshot)
        op = np.ascontiguousarray(old_pod, np.int32)
        on = np.ascontiguousarray(old_node, np.int32)
        out = np.zeros(1, np.int64)
        _check(lib().kbhip_session_carry_snapshot(self._h, ctypes.c_char_p(buf), len(buf), _p(op) if op.size else None,
                                                  _p(on) if on.size else None, _p(out)))
        return int(out[0])

    def reclaim(self, cap: int = 1 << 21) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        """Run reclaimAction.Execute: (pod, node, EVICTED | PIPELINED) records in decision order."""
        return self._action(lib().kbhip_reclaim, cap)

    def preempt(self, cap: int = 1 << 21) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        """Run preemptAction.Execute: records of the committed statements, in operation order."""
        return self._action(lib().kbhip_preempt, cap)

    def run_actions(self, actions: str = "allocate") -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        """The conf's actions in order (scheduler.go:93-97): allocate, backfill, reclaim, preempt."""
        logs = []
        for a in (x.strip() for x in actions.split(",")):
            if a == "allocate":
                logs.append(self.allocate())
            elif a == "backfill":
                logs.append(self.backfill())
            elif a == "reclaim":
                logs.append(self.reclaim())
            elif a == "preempt":
                logs.append(self.preempt())
            else:
                raise KbhipError(f"action {a!r} is not implemented by this engine")
        if not logs:
            z = np.zeros(0, np.int32)
            return z, z.copy(), np.zeros(0, np.uint8)
        return tuple(np.concatenate([lg[k] for lg in logs]) for k in range(3))

    def place_job(self, task_ids, gang_mode: int, min_available: int, ready_count: int):
        ids = np.ascontiguousarray(task_ids, dtype=np.int32)
        n = ids.size
        node = np.full(max(n, 1), -1, np.int32)
        kind = np.zeros(max(n, 1), np.uint8)
        done = np.zeros(1, np.int32)
        stop = np.zeros(1, np.int32)
        _check(lib().kbhip_place_job(self._h, _p(ids), n, gang_mode, min_available, ready_count, _p(node),
                                     _p(kind), _p(done), _p(stop)))
        d = int(done[0])
        return node[:d].copy(), kind[:d].copy(), int(stop[0])

    def place_job_submit(self, task_ids, gang_mode: int, min_available: int, ready_count: int) -> int:
        """kbhip_place_job_submit: queue a job pop (run on the state the earlier submitted pops leave); a ticket."""
        ids = np.ascontiguousarray(task_ids, dtype=np.int32)
        t = int(lib().kbhip_place_job_submit(self._h, _p(ids), ids.size, gang_mode, min_available, ready_count))
        _check(t if t < 0 else 0)
        self._tix = getattr(self, "_tix", {})
        self._tix[t] = max(ids.size, 1)
        return t

    def place_job_wait(self, ticket: int):
        """kbhip_place_job_wait: results of the oldest outstanding ticket, as place_job."""
        # the result arrays hold every task of the ticket; its size leaves the
        # table only once the wait succeeded (a refused wait can be retried)
        tix = getattr(self, "_tix", {})
        # a ticket this binding does not hold is refused by the library (EINVAL): arrays as large as any held one
        n = tix.get(ticket, max(list(tix.values()) + [1]))
        node = np.full(n, -1, np.int32)
        kind = np.zeros(n, np.uint8)
        done = np.zeros(1, np.int32)
        stop = np.zeros(1, np.int32)
        _check(lib().kbhip_place_job_wait(self._h, int(ticket), _p(node), _p(kind), _p(done), _p(stop)))
        tix.pop(ticket, None)
        d = int(done[0])
        return node[:d].copy(), kind[:d].copy(), int(stop[0])

    def place_job_cancel(self, ticket: int) -> int:
        """kbhip_place_job_cancel: withdraw `ticket` and every later one; the number withdrawn."""
        k = _check(lib().kbhip_place_job_cancel(self._h, int(ticket)))
        for t in [t for t in getattr(self, "_tix", {}) if t >= ticket]:
            del self._tix[t]
        return k

    def read_nodes(self, n_nodes: int) -> np.ndarray:
        out = np.zeros((n_nodes, 12), np.int64)
        _check(lib().kbhip_read_nodes(self._h, _p(out), n_nodes))
        return out

    def debug_keys(self) -> Tuple[np.ndarray, np.ndarray]:
        """Test support (after set_option("debug_keys", 1) and a run): the pod of
        every per-task sweep and its row: per-node keys, per-node raw inter-pod
        counts (npad each), then ipa lo, ipa hi, fallback node, max key."""
        L = lib()
        n = int(L.kbhip_debug_table(self._h, b"dbg_keys", None, 0))
        _check(n if n < 0 else 0)
        keys = np.zeros(max(n // 8, 1), np.uint64)
        if n:
            _check(int(L.kbhip_debug_table(self._h, b"dbg_keys", _p(keys), keys.nbytes)))
        m = int(L.kbhip_debug_table(self._h, b"dbg_pods", None, 0))
        pods = np.zeros(max(m // 4, 1), np.int32)
        if m:
            _check(int(L.kbhip_debug_table(self._h, b"dbg_pods", _p(pods), pods.nbytes)))
        pods = pods[: m // 4]
        return pods, keys[: n // 8].reshape(len(pods), -1) if len(pods) else keys[:0]

    def table(self, name: str) -> np.ndarray:
        """Test support: a device table read back (kbhip_debug_table)."""
        n = lib().kbhip_debug_table(self._h, name.encode(), None, 0)
        _check(int(n) if n < 0 else 0)
        out = np.zeros(max(int(n) // 4, 1), np.int32)
        _check(int(lib().kbhip_debug_table(self._h, name.encode(), _p(out), out.nbytes)) if n > 0 else 0)
        return out[: int(n) // 4]

    def gang_unschedulable(self) -> dict:
        """The gang plugin's OnSessionClose messages: {job uid: message} for
        every job not Ready (kbhip_gang_unschedulable)."""
        L = lib()
        n = int(L.kbhip_gang_unschedulable(self._h, None, 0))
        _check(n if n < 0 else 0)
        buf = ctypes.create_string_buffer(n + 1)
        _check(int(L.kbhip_gang_unschedulable(self._h, buf, n + 1)))
        out = {}
        for line in buf.value.decode().splitlines():
            if line:
                uid, msg = line.split("\t", 1)
                out[uid] = msg
        return out

    def stats(self) -> dict:
        st = Stats()
        _check(lib().kbhip_get_stats(self._h, ctypes.byref(st)))
        return st.as_dict()


class EncodedSnapshot:
    """Test support: the engine's compiled host tables for a snapshot, built
    without a device (kbhip_debug_encode).  It cannot place anything."""

    def __init__(self, snapshot):
        if not isinstance(snapshot, (bytes, bytearray, memoryview)):
            with open(snapshot, "rb") as f:
                snapshot = f.read()
        buf = bytes(snapshot)
        self._h = ctypes.c_void_p()
        _check(lib().kbhip_debug_encode(ctypes.c_char_p(buf), len(buf), ctypes.byref(self._h)))

    def table(self, name: str) -> np.ndarray:
        n = lib().kbhip_debug_table(self._h, name.encode(), None, 0)
        _check(int(n) if n < 0 else 0)
        out = np.zeros(max(int(n) // 4, 1), np.int32)
        _check(int(lib().kbhip_debug_table(self._h, name.encode(), _p(out), out.nbytes)) if n > 0 else 0)
        return out[: int(n) // 4]

    def replay(self, pods, modes, nodes, kinds) -> np.ndarray:
        """Per-step, per-node selection keys along a given decision sequence
        (kbhip_debug_replay); kinds: KBHIP_ALLOCATED / KBHIP_PIPELINED."""
        pods = np.ascontiguousarray(pods, np.int32)
        modes = np.ascontiguousarray(modes, np.int32)
        nodes = np.ascontiguousarray(nodes, np.int32)
        kinds = np.ascontiguousarray(kinds, np.uint8)
        n_nodes = int(self.table("dims")[0])
        out = np.zeros((len(pods), max(n_nodes, 1)), np.uint64)
        _check(lib().kbhip_debug_replay(self._h, len(pods), _p(pods), _p(modes), _p(nodes), _p(kinds), _p(out)))
        return out[:, :n_nodes]

    def close(self) -> None:
        if self._h:
            _check(lib().kbhip_session_close(self._h))
            self._h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def time_rank_multi(sessions, task_ids, reps: int = 16, evict: int = 0, mapped: int = 0) -> float:
    """kbhip_time_rank_multi: device microseconds of one multi-session preempt
    ranking launch chain over the given sessions (session i for its pending
    task task_ids[i])."""
    hs = (ctypes.c_void_p * len(sessions))(*[s._h for s in sessions])
    ids = np.ascontiguousarray(task_ids, dtype=np.int32)
    if ids.size != len(sessions):
        raise ValueError("one task id per session")
    out = np.zeros(1, np.float64)
    _check(lib().kbhip_time_rank_multi(hs, len(sessions), _p(ids), reps, evict, mapped, _p(out)))
    return float(out[0])


def shard_range(n_nodes: int, rank: int, world: int) -> Tuple[int, int]:
    """Node range [lo, hi) of a shard (the library's partition)."""
    return n_nodes * rank // world, n_nodes * (rank + 1) // world


def torch_gather(group=None, device=None):
    """An all-gather callback for kbhip_shard_connect_host_gather over
    torch.distributed (gloo on CPU tensors; device = a cuda device for the
    nccl (RCCL) backend): recv <- every rank's `send` bytes in rank order."""
    import torch
    import torch.distributed as dist

    def fn(send: np.ndarray, recv: np.ndarray) -> None:
        world = dist.get_world_size(group)
        out = [torch.empty(send.size, dtype=torch.uint8, device=device) for _ in range(world)]
        dist.all_gather(out, torch.from_numpy(send.copy()).to(device) if device is not None
                        else torch.from_numpy(send.copy()), group=group)
        recv[:] = torch.cat(out).cpu().numpy()
    return fn


def torch_exchange(group=None, device=None):
    """An exchange callback for kbhip_shard_connect_host doing the all-reduce
    with torch.distributed (gloo on CPU tensors; device = a cuda device for the
    nccl backend).  u64 keys are mapped to i64 by flipping the top bit, which
    preserves their order."""
    import torch
    import torch.distributed as dist

    def fn(vals: np.ndarray, op: int) -> None:
        v = vals.view(np.int64).copy()
        if op == RED_MAX_U64:
            v ^= np.int64(-0x8000000000000000)
        t = torch.from_numpy(v)
        if device is not None:
            t = t.to(device)
        rop = {RED_MIN_I64: dist.ReduceOp.MIN, RED_SUM_I64: dist.ReduceOp.SUM}.get(op, dist.ReduceOp.MAX)
        dist.all_reduce(t, op=rop, group=group)
        out = t.cpu().numpy()
        if op == RED_MAX_U64:
            out = out ^ np.int64(-0x8000000000000000)
        vals.view(np.int64)[:] = out
    return fn


class ShardedSession(Session):
    """A node-array shard of a session (include/kbhip.h): this
    rank's device holds nodes [lo, hi); every rank runs the same host loop and
    gets the same placements.  Connect with RCCL (connect_rccl, one GPU per
    rank) or with a Python exchange (connect_host, e.g. torch_exchange())."""

    def __init__(self, snapshot, device: int, rank: int, world: int):
        if not isinstance(snapshot, (bytes, bytearray, memoryview)):
            with open(snapshot, "rb") as f:
                snapshot = f.read()
        buf = bytes(snapshot)
        self._h = ctypes.c_void_p()
        self._cb = None
        _check(lib().kbhip_session_open_shard(ctypes.c_char_p(buf), len(buf), device, rank, world,
                                              ctypes.byref(self._h)))

    def info(self) -> Tuple[int, int, int, int]:
        out = np.zeros(4, np.int32)
        _check(lib().kbhip_shard_info(self._h, _p(out)))
        return tuple(int(x) for x in out)

    @staticmethod
    def rccl_unique_id() -> bytes:
        buf = ctypes.create_string_buffer(512)
        n = _check(lib().kbhip_rccl_unique_id(buf, 512))
        return buf.raw[:n]

    def connect_rccl(self, unique_id: bytes) -> int:
        """1 when a pooled communicator of an earlier session was reused, 0 after a new init."""
        b = ctypes.create_string_buffer(unique_id, len(unique_id))
        _check(lib().kbhip_shard_connect_rccl(self._h, b, len(unique_id)))
        return int(self.stats()["comm_reused"])

    def connect_host(self, fn, gather=None) -> None:
        """fn(vals: np.ndarray[uint64], op) reduces vals in place across ranks
        (per-task pops); gather(send: np.ndarray[uint8], recv) fills recv with
        every rank's send bytes in rank order (batched pops; without it every
        pop takes the per-task path)."""
        def cb(_ctx, vals, n, op):
            try:
                fn(np.ctypeslib.as_array(vals, shape=(n,)), op)
                return 0
            except Exception:  # reported to the library as a failed exchange
                return 1
        self._cb = ALLREDUCE_FN(cb)  # keep the trampoline alive
        _check(lib().kbhip_shard_connect_host(self._h, self._cb, None))
        if gather is not None:
            world = self.info()[1]

            def gcb(_ctx, send, recv, nbytes):
                try:
                    s_arr = np.ctypeslib.as_array(ctypes.cast(send, ctypes.POINTER(ctypes.c_uint8)), shape=(nbytes,))
                    r_arr = np.ctypeslib.as_array(ctypes.cast(recv, ctypes.POINTER(ctypes.c_uint8)),
                                                  shape=(nbytes * world,))
                    gather(s_arr, r_arr)
                    return 0
                except Exception:
                    return 1
            self._gcb = ALLGATHER_FN(gcb)
            _check(lib().kbhip_shard_connect_host_gather(self._h, self._gcb, None))

    def connect_mailbox(self, gather) -> None:
        """Peer mailboxes for the batched pops (kbhip_shard_connect_mailbox):
        gather(send, recv) all-gathers the ranks' IPC handles once."""
        world = self.info()[1]

        def mcb(_ctx, send, recv, nbytes):
            try:
                s_arr = np.ctypeslib.as_array(ctypes.cast(send, ctypes.POINTER(ctypes.c_uint8)), shape=(nbytes,))
                r_arr = np.ctypeslib.as_array(ctypes.cast(recv, ctypes.POINTER(ctypes.c_uint8)), shape=(nbytes * world,))
                gather(s_arr.copy(), r_arr)
                return 0
            except Exception:
                return 1
        cb = ALLGATHER_FN(mcb)
        _check(lib().kbhip_shard_connect_mailbox(self._h, cb, None))
