"""Test support: the reference scheduler cache's informer event handlers
(pkg/scheduler/cache/event_handlers.go) restated on a kbgen.Cluster — the
cluster state the cache holds, whose KBS1 snapshot is what cache.Snapshot
(cache.go:515-583) gives the next session.  Used to build "the snapshot the
reference cache would hold" after a mixed event stream, which the oracle
schedules and the engine must reproduce through kbhip_session_carry_snapshot.

Handlers (the cache's own, in the reference's terms):
  add_pod     addPod -> addTask (:63-86): the task joins its job (a shadow
              PodGroup for a pod without one) and, if bound and not
              terminated, its node.
  delete_pod  deletePod (:119-165) -> deleteTask on NewTaskInfo(pod): a pod of
              a PodGroup leaves its job and its node; a group-less pod's
              TaskInfo has an empty Job (api/job_info.go:60-70), so its shadow
              job keeps it and only the node drops it (kbgen Pod.detached);
              jobs are never deleted (JobTerminated needs a nil PodGroup).
  finish_pod  updatePod to Succeeded / Failed (:112-117): delete + add of the
              terminated pod: it stays in its job, off its node.
  add_node / update_node / delete_node (:250-290): NewNodeInfo / SetNode /
              delete (the tests drain a node before deleting it: pods bound to a
              node absent from the snapshot are refused by both sides).
  add_pod_group / update_pod_group (:385-425).
"""
import copy
from typing import Dict, List, Optional


class CacheModel:
    def __init__(self, cluster):
        self.c = cluster

    # --- pods -------------------------------------------------------------------
    def pod(self, uid):
        for q in self.c.pods:
            if q.uid == uid:
                return q
        raise KeyError(uid)

    def add_pod(self, **kw):
        return self.c.add_pod(**kw)

    def delete_pod(self, uid):
        q = self.pod(uid)
        if q.group is not None:
            self.c.pods.remove(q)
        elif q.node is not None and q.phase not in ("Succeeded", "Failed"):
            q.detached = True  # off its node, still a task of its shadow job

    def finish_pod(self, uid, phase):
        assert phase in ("Succeeded", "Failed")
        self.pod(uid).phase = phase

    # --- nodes ------------------------------------------------------------------
    def node(self, name):
        for n in self.c.nodes:
            if n.name == name:
                return n
        raise KeyError(name)

    def add_node(self, *a, **kw):
        return self.c.add_node(*a, **kw)

    def update_node(self, name, **fields):
        n = self.node(name)
        for k, v in fields.items():
            setattr(n, k, v)

    def delete_node(self, name):
        assert not any(q.node == name and not q.detached for q in self.c.pods), "drain the node first"
        self.c.nodes.remove(self.node(name))

    # --- pod groups -------------------------------------------------------------
    def add_pod_group(self, *a, **kw):
        return self.c.add_job(*a, **kw)

    def update_pod_group(self, uid, **fields):
        for j in self.c.jobs:
            if j.uid == uid:
                for k, v in fields.items():
                    setattr(j, k, v)
                return j
        raise KeyError(uid)


def index_maps(old_cluster_pods: List, old_node_names: List[str], new_cluster) -> tuple:
    """old_pod / old_node maps of kbhip_session_carry_snapshot: for every pod /
    node of the new snapshot (canonical order: pods by UID, nodes by name), its
    index in the old session (-1: new).  old_cluster_pods: the old session's
    pods in its canonical order."""
    import numpy as np
    old_pod_idx: Dict[str, int] = {q.uid: i for i, q in enumerate(old_cluster_pods)}
    old_node_idx = {n: i for i, n in enumerate(old_node_names)}
    new_pods = sorted(new_cluster.pods, key=lambda q: q.uid)
    new_nodes = sorted(n.name for n in new_cluster.nodes)
    op = np.array([old_pod_idx.get(q.uid, -1) for q in new_pods], np.int32)
    on = np.array([old_node_idx.get(n, -1) for n in new_nodes], np.int32)
    return op, on


def snapshot_after_session(c, status, node):
    """The cluster the cache holds after a session: binds and evictions applied
    (the session's other decisions are session-only)."""
    BINDING, RELEASING, ALLOC, AOB, PIPE = 16, 128, 4, 2, 8
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


def clone(c):
    return copy.deepcopy(c)
