"""A host-side allocate loop that drives the engine one job pop at a time
through kbhip_place_job — what the Go shim of INTEGRATION.md does inside
kube-batch, restated in Python for the tests (no Go toolchain here).

It mirrors pkg/scheduler/actions/allocate/allocate.go:41-201 with the
ordering plugins of the tiers (priority.go:38-79, gang.go:63-66 / 136-160,
drf.go:52-170, proportion.go:57-241) and Go's container/heap, and hands each
job pop — the job's remaining pending tasks in TaskOrderFn order — to the
engine, which runs PredicateFn / NodeOrderFn / SelectBestNode / the walk /
Session.Allocate|Pipeline node updates / the gang stop on the device.  Back on
the host the shim applies each decision to its own model (TaskStatus,
AllocateFunc event handlers), as ssn.Allocate / ssn.Pipeline would.

Inputs come from a kbgen.Cluster (the object the snapshot was written from):
pods by UID = the snapshot's pod index, nodes by name, jobs by UID.
"""
from typing import Callable, List

import kbgen

MIN_CPU, MIN_MEM, MIN_GPU = 10.0, 10.0 * 1024 * 1024, 10.0
PENDING, ALLOCATED, PIPELINED, BINDING, BOUND, RUNNING, RELEASING = "Pending", "Allocated", "Pipelined", \
    "Binding", "Bound", "Running", "Releasing"
ALLOCATED_STATUSES = (BOUND, BINDING, RUNNING, ALLOCATED)


class GoHeap:
    """Go container/heap with a less(a, b) callback (heap.go: up / down)."""

    def __init__(self, less: Callable):
        self.items: List = []
        self.less = less

    def _l(self, i, j):
        return self.less(self.items[i], self.items[j])

    def push(self, x):
        self.items.append(x)
        j = len(self.items) - 1
        while True:
            i = (j - 1) // 2
            if i == j or j == 0 or not self._l(j, i):
                break
            self.items[i], self.items[j] = self.items[j], self.items[i]
            j = i

    def pop(self):
        n = len(self.items) - 1
        self.items[0], self.items[n] = self.items[n], self.items[0]
        i = 0
        while True:
            j1 = 2 * i + 1
            if j1 >= n:
                break
            j = j1
            if j1 + 1 < n and self._l(j1 + 1, j1):
                j = j1 + 1
            if not self._l(j, i):
                break
            self.items[i], self.items[j] = self.items[j], self.items[i]
            i = j
        return self.items.pop()

    def empty(self):
        return not self.items


def _share(l, r):  # helpers.go:35-48
    if r == 0:
        return 0.0 if l == 0 else 1.0
    return l / r


def _le(a, b):  # Resource.LessEqual (resource_info.go:164-168)
    mins = (MIN_CPU, MIN_MEM, MIN_GPU)
    return all(x < y or abs(y - x) < m for x, y, m in zip(a, b, mins))


class GoHost:
    def __init__(self, c: "kbgen.Cluster"):
        dis = {p: set(f) for p, f in c.flags.items()}
        self.tiers = [[p for p in t] for t in c.tiers]

        def on(p, flag):
            return flag not in dis.get(p, ())
        names = [p for t in self.tiers for p in t]
        self.job_order = [p for p in names if p in ("priority", "gang", "drf") and on(p, "disableJobOrder")]
        self.queue_prop = any(p == "proportion" and on(p, "disableQueueOrder") for p in names)
        self.task_prio = any(p == "priority" and on(p, "disableTaskOrder") for p in names)
        self.gang_ready = any(p == "gang" and on(p, "disableJobReady") for p in names)
        self.drf_on = "drf" in names
        self.prop_on = "proportion" in names
        nodes = sorted(c.nodes, key=lambda n: n.name)
        self.total = [float(sum(n.cpu for n in nodes)), float(sum(n.mem for n in nodes)),
                      float(sum(n.gpu for n in nodes))]
        self.queues = {q.name: dict(name=q.name, weight=q.weight, ts=q.ts, share=0.0, deserved=[0.0] * 3,
                                    allocated=[0.0] * 3, request=[0.0] * 3, attr=False) for q in c.queues}
        pods = sorted(c.pods, key=lambda p: p.uid)
        jobs = {}
        for j in c.jobs:
            if j.queue in self.queues:  # cache.go:556-560
                jobs[j.uid] = dict(uid=j.uid, queue=j.queue, min=j.min_member, ts=j.ts, tasks=[])
        self.pods = []
        for i, p in enumerate(pods):
            juid = f"{p.ns}/{p.group}" if p.group is not None else p.uid
            if p.group is None and "default" in self.queues and juid not in jobs:  # shadow PodGroup
                jobs[juid] = dict(uid=juid, queue="default", min=1, ts=0, tasks=[])
            req = [sum(x.get(k, 0) for x in p.containers) for k in ("cpu", "mem", "gpu")]
            st = self._status(p)
            self.pods.append(dict(i=i, uid=p.uid, prio=p.priority, ts=p.ts, req=[float(x) for x in req], status=st,
                                  job=juid if juid in jobs else None))
            if juid in jobs:
                jobs[juid]["tasks"].append(i)
        self.jobs = [jobs[k] for k in sorted(jobs)]  # UID order
        for j in self.jobs:
            j["prio"] = self.pods[j["tasks"][-1]]["prio"] if j["tasks"] else 0  # job_info.go:242 (last task)
            j["alloc_n"] = sum(self.pods[t]["status"] in ALLOCATED_STATUSES for t in j["tasks"])
            j["drf_alloc"] = [0.0] * 3
            j["cursor"] = 0
            j["pending"] = None
        self._open_plugins()

    @staticmethod
    def _status(p):  # api/helpers.go:35-61
        if p.phase == "Running":
            return RELEASING if p.deleting else RUNNING
        if p.phase == "Pending":
            return RELEASING if p.deleting else (BOUND if p.node else PENDING)
        return p.phase

    def _open_plugins(self):
        for j in self.jobs:  # drf.go:65-82
            for t in j["tasks"]:
                if self.pods[t]["status"] in ALLOCATED_STATUSES:
                    j["drf_alloc"] = [a + b for a, b in zip(j["drf_alloc"], self.pods[t]["req"])]
            j["drf"] = max(_share(a, b) for a, b in zip(j["drf_alloc"], self.total))
        if not self.prop_on:
            return
        for j in self.jobs:  # proportion.go:65-101
            q = self.queues[j["queue"]]
            q["attr"] = True
            for t in j["tasks"]:
                p = self.pods[t]
                if p["status"] in ALLOCATED_STATUSES:
                    q["allocated"] = [a + b for a, b in zip(q["allocated"], p["req"])]
                    q["request"] = [a + b for a, b in zip(q["request"], p["req"])]
                elif p["status"] == PENDING:
                    q["request"] = [a + b for a, b in zip(q["request"], p["req"])]
        order = [self.queues[n] for n in sorted(self.queues) if self.queues[n]["attr"]]
        remaining = list(self.total)
        meet = set()
        while True:  # proportion.go:104-136
            tw = sum(q["weight"] for q in order if q["name"] not in meet)
            if tw == 0:
                break
            deserved = [0.0] * 3
            for q in order:
                if q["name"] in meet:
                    continue
                ratio = q["weight"] / tw
                q["deserved"] = [a + r * ratio for a, r in zip(q["deserved"], remaining)]
                if not _le(q["deserved"], q["request"]):
                    q["deserved"] = [min(a, b) for a, b in zip(q["deserved"], q["request"])]
                    meet.add(q["name"])
                self._prop_share(q)
                deserved = [a + b for a, b in zip(deserved, q["deserved"])]
            remaining = [a - b for a, b in zip(remaining, deserved)]
            if all(x < m for x, m in zip(remaining, (MIN_CPU, MIN_MEM, MIN_GPU))):
                break

    @staticmethod
    def _prop_share(q):  # proportion.go:229-241
        q["share"] = max(_share(a, d) for a, d in zip(q["allocated"], q["deserved"]))

    # ---- order functions (session_plugins.go:244-329) ----
    def _ready(self, j):
        return j["alloc_n"] >= j["min"]

    def job_less(self, l, r):
        L, R = self.jobs[l], self.jobs[r]
        for p in self.job_order:
            if p == "priority":
                c = -1 if L["prio"] > R["prio"] else (1 if L["prio"] < R["prio"] else 0)
            elif p == "gang":
                lr, rr = self._ready(L), self._ready(R)
                c = 0 if lr and rr else (1 if lr else (-1 if rr else 0))
            else:
                c = 0 if L["drf"] == R["drf"] else (-1 if L["drf"] < R["drf"] else 1)
            if c:
                return c < 0
        if L["ts"] == R["ts"]:
            return L["uid"] < R["uid"]
        return L["ts"] < R["ts"]

    def queue_less(self, l, r):
        L, R = self.queues[l], self.queues[r]
        if self.queue_prop and L["share"] != R["share"]:
            return L["share"] < R["share"]
        if L["ts"] == R["ts"]:
            return L["name"] < R["name"]
        return L["ts"] < R["ts"]

    def _task_key(self, t):
        p = self.pods[t]
        return (-p["prio"] if self.task_prio else 0, p["ts"], p["uid"])

    def _overused(self, qn):  # proportion.go:186-197
        if not self.prop_on:
            return False
        q = self.queues[qn]
        return _le(q["deserved"], q["allocated"])

    def _on_allocate(self, t):  # drf.go:134-143, proportion.go:200-210
        p = self.pods[t]
        j = self._job_of[p["job"]]
        if self.drf_on:
            j["drf_alloc"] = [a + b for a, b in zip(j["drf_alloc"], p["req"])]
            j["drf"] = max(_share(a, b) for a, b in zip(j["drf_alloc"], self.total))
        if self.prop_on:
            q = self.queues[j["queue"]]
            q["allocated"] = [a + b for a, b in zip(q["allocated"], p["req"])]
            self._prop_share(q)

    def allocate(self, place_job):
        """allocate.go:41-201 with place_job(ids, gang_mode, min_available,
        ready_count) -> (nodes, kinds, stop) per job pop.  Returns the
        placement log [(pod, node, 4 Allocated | 8 Pipelined)] and the pop count."""
        self._job_of = {j["uid"]: j for j in self.jobs}
        qheap = GoHeap(self.queue_less)
        jheaps = {}
        for k, j in enumerate(self.jobs):
            qheap.push(j["queue"])
            jheaps.setdefault(j["queue"], GoHeap(self.job_less)).push(k)
        log, pops = [], 0
        gm = 1 if self.gang_ready else 0
        while not qheap.empty():
            qn = qheap.pop()
            if self._overused(qn):
                continue
            jh = jheaps.get(qn)
            if jh is None or jh.empty():
                continue
            k = jh.pop()
            j = self.jobs[k]
            pops += 1
            if j["pending"] is None:  # allocate.go:91-104: BestEffort tasks are skipped
                j["pending"] = sorted((t for t in j["tasks"] if self.pods[t]["status"] == PENDING and
                                       not all(x < m for x, m in zip(self.pods[t]["req"],
                                                                     (MIN_CPU, MIN_MEM, MIN_GPU)))),
                                      key=self._task_key)
            ids = j["pending"][j["cursor"]:]
            if ids:
                nodes, kinds, stop = place_job(ids, gm, j["min"], j["alloc_n"])
                for t, n, kd in zip(ids, nodes, kinds):
                    if n < 0:
                        continue
                    p = self.pods[t]
                    p["status"] = ALLOCATED if kd == 1 else PIPELINED
                    if kd == 1:
                        j["alloc_n"] += 1
                    j["prio"] = p["prio"]  # UpdateTaskStatus -> AddTaskInfo (job_info.go:242)
                    self._on_allocate(t)
                    log.append((t, int(n), 4 if kd == 1 else 8))
                j["cursor"] += len(nodes)
                if stop == 2:  # JobReady: the job goes back (allocate.go:191-195)
                    jh.push(k)
            qheap.push(qn)
        return log, pops
