/*
 * kbref.h — TEST ORACLE (faithful restatement), shared header of kbref.cpp and
 * kbref_plugins.cpp.  Test infrastructure only (see kbref.cpp).
 */
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <set>
#include <stdexcept>
#include <string>
#include <vector>

#include "../include/kbsnap.h"

namespace ref {

using std::map;
using std::string;
using std::vector;

/* ------------------------------------------------------------------------ */
/* k8s object model subset                                                   */
/* ------------------------------------------------------------------------ */
enum Op { OpIn = 0, OpNotIn = 1, OpExists = 2, OpDoesNotExist = 3, OpGt = 4, OpLt = 5, OpEquals = 6,
          OpInvalid = 15 };

struct Requirement {  // labels.Requirement (apimachinery/pkg/labels/selector.go)
    string key;
    int op;
    vector<string> values;
};

struct LabelSelector {  // metav1.LabelSelector
    map<string, string> ml;
    vector<Requirement> me;
};

struct NodeSelectorTerm {
    vector<Requirement> expr, fields;
};

struct PodAffinityTerm {
    std::shared_ptr<LabelSelector> sel;  // nil-able
    vector<string> namespaces;
    string topologyKey;
};

struct WeightedPodAffinityTerm {
    int32_t weight;
    PodAffinityTerm term;
};

struct Affinity {
    bool hasNA = false, hasNAReq = false, hasPA = false, hasPAA = false;
    vector<NodeSelectorTerm> naReq;
    vector<std::pair<int32_t, NodeSelectorTerm>> naPref;
    vector<PodAffinityTerm> paReq, paaReq;
    vector<WeightedPodAffinityTerm> paPref, paaPref;
};

struct ContainerPort {
    string ip, proto;
    int32_t port;
};

struct Container {
    int64_t cpu = 0, mem = 0, gpu = 0;
    int has = 0;  // KBS_HAS_* : key present in Requests
    vector<ContainerPort> ports;
};

struct Toleration {
    string key, op, value, effect;
};

struct Taint {
    string key, value, effect;
};

struct Pod {
    int index = 0;
    string uid, name, ns;
    map<string, string> labels;
    string nodeName;  // Spec.NodeName
    int phase = KBS_PENDING;
    bool deleting = false;
    bool detached = false;  // p_detached (kbsnap.h): in its job, off its node's task list
    int32_t priority = 0;
    int64_t ts = 0;
    bool backfill = false;
    string priorityClassName;  // Spec.PriorityClassName (conformance.go:40-45)
    vector<Container> containers, initContainers;
    map<string, string> nodeSelector;
    vector<Toleration> tolerations;
    std::shared_ptr<Affinity> affinity;
    int job = -1;  // snapshot job row
};

struct KNode {  // v1.Node
    int index = 0;
    string name;
    map<string, string> labels;
    vector<Taint> taints;
    bool unschedulable = false;
    int64_t a_cpu, a_mem, a_gpu, a_pods, c_cpu, c_mem, c_gpu, c_pods;
};

/* ------------------------------------------------------------------------ */
/* kube-batch api (pkg/scheduler/api)                                        */
/* ------------------------------------------------------------------------ */
static const double minMilliCPU = 10, minMilliGPU = 10, minMemory = 10 * 1024 * 1024;  // resource_info.go:54-56

struct Resource {  // resource_info.go:26-33
    double MilliCPU = 0, Memory = 0, MilliGPU = 0;
    int MaxTaskNum = 0;
    Resource& Add(const Resource& r) { MilliCPU += r.MilliCPU; Memory += r.Memory; MilliGPU += r.MilliGPU; return *this; }
    Resource& Sub(const Resource& r) { MilliCPU -= r.MilliCPU; Memory -= r.Memory; MilliGPU -= r.MilliGPU; return *this; }
    Resource& Multi(double ratio) { MilliCPU *= ratio; Memory *= ratio; MilliGPU *= ratio; return *this; }
    bool IsEmpty() const { return MilliCPU < minMilliCPU && Memory < minMemory && MilliGPU < minMilliGPU; }  // :75-77
    bool Less(const Resource& rr) const {  // :156-158 — strict in every dimension
        return MilliCPU < rr.MilliCPU && Memory < rr.Memory && MilliGPU < rr.MilliGPU;
    }
    bool LessEqual(const Resource& rr) const {  // :164-168
        return (MilliCPU < rr.MilliCPU || std::fabs(rr.MilliCPU - MilliCPU) < minMilliCPU) &&
               (Memory < rr.Memory || std::fabs(rr.Memory - Memory) < minMemory) &&
               (MilliGPU < rr.MilliGPU || std::fabs(rr.MilliGPU - MilliGPU) < minMilliGPU);
    }
    void SetMaxResource(const Resource& rr) {  // :114-128
        if (rr.MilliCPU > MilliCPU) MilliCPU = rr.MilliCPU;
        if (rr.Memory > Memory) Memory = rr.Memory;
        if (rr.MilliGPU > MilliGPU) MilliGPU = rr.MilliGPU;
    }
    double Get(int rn) const { return rn == 0 ? MilliCPU : rn == 1 ? Memory : MilliGPU; }
};

static Resource MinRes(const Resource& l, const Resource& r) {  // api/helpers/helpers.go:25-33
    Resource res;
    res.MilliCPU = std::fmin(l.MilliCPU, r.MilliCPU);
    res.MilliGPU = std::fmin(l.MilliGPU, r.MilliGPU);
    res.Memory = std::fmin(l.Memory, r.Memory);
    return res;
}

static double Share(double l, double r) {  // helpers.go:35-48
    if (r == 0) return l == 0 ? 0 : 1;
    return l / r;
}

enum TaskStatus {  // types.go:22-61
    Pending = 1 << 0, AllocatedOverBackfill = 1 << 1, Allocated = 1 << 2, Pipelined = 1 << 3,
    Binding = 1 << 4, Bound = 1 << 5, Running = 1 << 6, Releasing = 1 << 7, Succeeded = 1 << 8,
    Failed = 1 << 9, Unknown = 1 << 10
};
static const int AllocatedStatusesList[] = {Bound, Binding, Running, Allocated};  // types.go:82-84
static bool AllocatedStatus(int s) { return s == Bound || s == Binding || s == Running || s == Allocated; }

enum JobReadiness { Ready = 1, AlmostReady = 2, NotReady = 4 };

static int getTaskStatus(const Pod& p) {  // helpers.go:35-61
    switch (p.phase) {
        case KBS_RUNNING: return p.deleting ? Releasing : Running;
        case KBS_PENDING:
            if (p.deleting) return Releasing;
            if (p.nodeName.empty()) return Pending;
            return Bound;
        case KBS_UNKNOWN: return Unknown;
        case KBS_SUCCEEDED: return Succeeded;
        case KBS_FAILED: return Failed;
    }
    return Unknown;
}

static Resource ContainerRes(const Container& c) {  // NewResource(container.Resources.Requests)
    Resource r;
    r.MilliCPU = (double)c.cpu;
    r.Memory = (double)c.mem;
    r.MilliGPU = (double)c.gpu;
    return r;
}

static Resource GetPodResourceWithoutInitContainers(const Pod& p) {  // pod_info.go:64-71
    Resource r;
    for (auto& c : p.containers) r.Add(ContainerRes(c));
    return r;
}
static Resource GetPodResourceRequest(const Pod& p) {  // pod_info.go:51-60
    Resource r = GetPodResourceWithoutInitContainers(p);
    for (auto& c : p.initContainers) r.SetMaxResource(ContainerRes(c));
    return r;
}

struct TaskInfo {  // job_info.go:36-58
    int pod = -1;  // index of pod (also the pinned map-iteration key)
    string uid;
    int job = -1;  // session job slot (-1 = not in a session job)
    string jobUID;
    string name, ns;
    Resource Resreq, InitResreq;
    string NodeName;
    int Status = Pending;
    int32_t Priority = 1;
    Pod* P = nullptr;
    bool IsBackfill = false;
};

struct NodeInfo {  // node_info.go:27-45
    string Name;
    KNode* Node = nullptr;
    Resource Releasing, Idle, Used, Backfilled, Allocatable, Capability;
    map<int, TaskInfo> Tasks;  // keyed by pod index: pinned map order

    void init(KNode* n) {  // NewNodeInfo(node) :62-75
        Name = n->name;
        Node = n;
        Idle.MilliCPU = (double)n->a_cpu; Idle.Memory = (double)n->a_mem; Idle.MilliGPU = (double)n->a_gpu;
        Idle.MaxTaskNum = (int)n->a_pods;
        Allocatable = Idle;
        Capability.MilliCPU = (double)n->c_cpu; Capability.Memory = (double)n->c_mem;
        Capability.MilliGPU = (double)n->c_gpu; Capability.MaxTaskNum = (int)n->c_pods;
    }
    bool AddTask(const TaskInfo& task) {  // :113-145
        if (Tasks.count(task.pod)) return false;
        TaskInfo ti = task;  // task.Clone()
        if (Node) {
            if (task.IsBackfill) Backfilled.Add(task.Resreq);
            switch (ti.Status) {
                case ::ref::Releasing: Releasing.Add(ti.Resreq); Idle.Sub(ti.Resreq); break;
                case ::ref::Pipelined: Releasing.Sub(ti.Resreq); break;
                default: Idle.Sub(ti.Resreq);
            }
            Used.Add(ti.Resreq);
        }
        Tasks[task.pod] = ti;
        return true;
    }
    bool RemoveTask(const TaskInfo& ti) {  // :147-177
        auto it = Tasks.find(ti.pod);
        if (it == Tasks.end()) return false;
        const TaskInfo& task = it->second;
        if (Node) {
            if (task.IsBackfill) Backfilled.Sub(task.Resreq);
            switch (task.Status) {
                case ::ref::Releasing: Releasing.Sub(task.Resreq); Idle.Add(task.Resreq); break;
                case ::ref::Pipelined: Releasing.Add(task.Resreq); break;
                default: Idle.Add(task.Resreq);
            }
            Used.Sub(task.Resreq);
        }
        Tasks.erase(it);
        return true;
    }
    bool UpdateTask(const TaskInfo& ti) {  // :179-185
        if (!RemoveTask(ti)) return false;
        return AddTask(ti);
    }
    vector<Pod*> Pods() const {  // :201-207
        vector<Pod*> v;
        for (auto& kv : Tasks) v.push_back(kv.second.P);
        return v;
    }
    Resource GetAccessibleResource() {  // :209-211 — mutates Idle (Appendix A.1)
        Idle.Add(Backfilled);
        return Idle;
    }
};

struct JobInfo {  // job_info.go:140-167
    string UID, Name, Namespace, Queue;
    int32_t Priority = 0;
    int32_t MinAvailable = 0;
    map<int, map<int, TaskInfo*>> TaskStatusIndex;  // status -> pod index -> task
    map<int, TaskInfo*> Tasks;
    Resource Allocated, TotalRequest;
    int64_t CreationTimestamp = 0;
    map<string, Resource> NodesFitDelta;
    int slot = 0;

    void addTaskIndex(TaskInfo* ti) { TaskStatusIndex[ti->Status][ti->pod] = ti; }
    void AddTaskInfo(TaskInfo* ti) {  // :239-249
        Tasks[ti->pod] = ti;
        addTaskIndex(ti);
        Priority = ti->P->priority;
        TotalRequest.Add(ti->Resreq);
        if (AllocatedStatus(ti->Status)) Allocated.Add(ti->Resreq);
    }
    void deleteTaskIndex(TaskInfo* ti) {
        auto it = TaskStatusIndex.find(ti->Status);
        if (it != TaskStatusIndex.end()) {
            it->second.erase(ti->pod);
            if (it->second.empty()) TaskStatusIndex.erase(it);
        }
    }
    void DeleteTaskInfo(TaskInfo* ti) {  // :276-292
        auto it = Tasks.find(ti->pod);
        if (it == Tasks.end()) return;
        TaskInfo* task = it->second;
        TotalRequest.Sub(task->Resreq);
        if (AllocatedStatus(task->Status)) Allocated.Sub(task->Resreq);
        Tasks.erase(it);
        deleteTaskIndex(task);
    }
    void UpdateTaskStatus(TaskInfo* task, int status) {  // :251-264
        DeleteTaskInfo(task);
        task->Status = status;
        AddTaskInfo(task);
    }
    int count(int status) const {
        auto it = TaskStatusIndex.find(status);
        return it == TaskStatusIndex.end() ? 0 : (int)it->second.size();
    }
    int GetReadiness() const {  // :374-388
        int allocated = 0;
        for (int s : AllocatedStatusesList) allocated += count(s);
        if (allocated >= MinAvailable) return Ready;
        if (allocated + count(AllocatedOverBackfill) >= MinAvailable) return AlmostReady;
        return NotReady;
    }
};

struct QueueInfo {
    string UID, Name;
    int32_t Weight = 1;
    int64_t ts = 0;
    int slot = 0;
};

/* ------------------------------------------------------------------------ */
/* Go container/heap + util.PriorityQueue (util/priority_queue.go)           */
/* ------------------------------------------------------------------------ */
template <typename T>
struct PriorityQueue {
    vector<T*> items;
    std::function<bool(T*, T*)> lessFn;
    bool Less(int i, int j) { return lessFn(items[i], items[j]); }
    void Swap(int i, int j) { std::swap(items[i], items[j]); }
    void up(int j) {
        for (;;) {
            int i = (j - 1) / 2;  // parent
            if (i == j || !Less(j, i)) break;
            Swap(i, j);
            j = i;
        }
    }
    bool down(int i0, int n) {
        int i = i0;
        for (;;) {
            int j1 = 2 * i + 1;
            if (j1 >= n || j1 < 0) break;
            int j = j1;
            int j2 = j1 + 1;
            if (j2 < n && Less(j2, j1)) j = j2;
            if (!Less(j, i)) break;
            Swap(i, j);
            i = j;
        }
        return i > i0;
    }
    void Push(T* x) {
        items.push_back(x);
        up((int)items.size() - 1);
    }
    T* Pop() {
        if (items.empty()) return nullptr;
        int n = (int)items.size() - 1;
        Swap(0, n);
        down(0, n);
        T* it = items.back();
        items.pop_back();
        return it;
    }
    bool Empty() const { return items.empty(); }
    int Len() const { return (int)items.size(); }
};

/* ------------------------------------------------------------------------ */
/* labels / selectors (apimachinery/pkg/labels/selector.go)                  */
/* ------------------------------------------------------------------------ */
static bool parseInt64(const string& s, int64_t* out) {  // strconv.ParseInt(s, 10, 64)
    if (s.empty()) return false;
    size_t i = 0;
    bool neg = false;
    if (s[0] == '+' || s[0] == '-') {
        neg = s[0] == '-';
        i = 1;
        if (s.size() == 1) return false;
    }
    unsigned long long v = 0;
    const unsigned long long lim = neg ? 9223372036854775808ULL : 9223372036854775807ULL;
    for (; i < s.size(); ++i) {
        char ch = s[i];
        if (ch < '0' || ch > '9') return false;
        unsigned d = (unsigned)(ch - '0');
        if (v > (lim - d) / 10) return false;
        v = v * 10 + d;
    }
    *out = neg ? (int64_t)(0 - v) : (int64_t)v;
    return true;
}

typedef map<string, string> Labels;

static bool hasValue(const Requirement& r, const string& v) {
    for (auto& s : r.values) if (s == v) return true;
    return false;
}

static bool RequirementMatches(const Requirement& r, const Labels& ls) {  // selector.go:192-236
    auto it = ls.find(r.key);
    bool has = it != ls.end();
    switch (r.op) {
        case OpIn:
        case OpEquals:
            if (!has) return false;
            return hasValue(r, it->second);
        case OpNotIn:
            if (!has) return true;
            return !hasValue(r, it->second);
        case OpExists: return has;
        case OpDoesNotExist: return !has;
        case OpGt:
        case OpLt: {
            if (!has) return false;
            int64_t lv, rv = 0;
            if (!parseInt64(it->second, &lv)) return false;
            if (r.values.size() != 1) return false;
            for (auto& s : r.values) if (!parseInt64(s, &rv)) return false;
            return (r.op == OpGt && lv > rv) || (r.op == OpLt && lv < rv);
        }
    }
    return false;
}

/* labels.NewRequirement validation (selector.go:134-170), without the
 * key/value syntax checks (documented limitation). */
static bool ValidRequirement(const Requirement& r) {
    switch (r.op) {
        case OpIn:
        case OpNotIn: return !r.values.empty();
        case OpEquals: return r.values.size() == 1;
        case OpExists:
        case OpDoesNotExist: return r.values.empty();
        case OpGt:
        case OpLt: {
            if (r.values.size() != 1) return false;
            int64_t v;
            return parseInt64(r.values[0], &v);
        }
    }
    return false;
}

/* A compiled selector: kind 0 = internal (AND of reqs), 1 = Nothing. */
struct Selector {
    bool nothing = false;
    vector<Requirement> reqs;
    bool Matches(const Labels& ls) const {
        if (nothing) return false;
        for (auto& r : reqs) if (!RequirementMatches(r, ls)) return false;
        return true;
    }
};

/* metav1.LabelSelectorAsSelector (apimachinery/pkg/apis/meta/v1/helpers.go:31-67) */
static bool LabelSelectorAsSelector(const LabelSelector* ps, Selector* out) {
    *out = Selector();
    if (!ps) { out->nothing = true; return true; }
    if (ps->ml.size() + ps->me.size() == 0) return true;  // Everything
    for (auto& kv : ps->ml) {
        Requirement r{kv.first, OpEquals, {kv.second}};
        if (!ValidRequirement(r)) return false;
        out->reqs.push_back(r);
    }
    for (auto& e : ps->me) {
        if (e.op != OpIn && e.op != OpNotIn && e.op != OpExists && e.op != OpDoesNotExist) return false;
        if (!ValidRequirement(e)) return false;
        out->reqs.push_back(e);
    }
    // internalSelector.Add sorts by key; irrelevant for Matches (AND).
    return true;
}

/* v1helper.NodeSelectorRequirementsAsSelector (helper/helpers.go:222-252) */
static bool NodeSelectorRequirementsAsSelector(const vector<Requirement>& nsm, Selector* out) {
    *out = Selector();
    if (nsm.empty()) { out->nothing = true; return true; }
    for (auto& e : nsm) {
        if (e.op > OpLt) return false;
        if (!ValidRequirement(e)) return false;
        out->reqs.push_back(e);
    }
    return true;
}

/* NodeSelectorRequirementsAsFieldSelector (helper/helpers.go:255-283) + Matches
 * against fields.Set{metadata.name: node.Name} (algorithm/types.go:30-32). */
static bool FieldSelectorMatches(const vector<Requirement>& nsm, const string& nodeName, bool* err) {
    *err = false;
    if (nsm.empty()) return false;  // fields.Nothing()
    for (auto& e : nsm) {
        if ((e.op != OpIn && e.op != OpNotIn) || e.values.size() != 1) { *err = true; return false; }
    }
    for (auto& e : nsm) {
        string fv = e.key == "metadata.name" ? nodeName : string();
        bool eq = fv == e.values[0];
        if (e.op == OpIn && !eq) return false;
        if (e.op == OpNotIn && eq) return false;
    }
    return true;
}

/* v1helper.MatchNodeSelectorTerms (helper/helpers.go:302-333) */
static bool MatchNodeSelectorTerms(const vector<NodeSelectorTerm>& terms, const KNode& node) {
    for (auto& req : terms) {
        if (req.expr.empty() && req.fields.empty()) continue;
        if (!req.expr.empty()) {
            Selector sel;
            if (!NodeSelectorRequirementsAsSelector(req.expr, &sel) || !sel.Matches(node.labels)) continue;
        }
        if (!req.fields.empty()) {
            bool err;
            if (!FieldSelectorMatches(req.fields, node.name, &err) || err) continue;
        }
        return true;
    }
    return false;
}

/* predicates.podMatchesNodeSelectorAndAffinityTerms (predicates.go:807-850) */
static bool podMatchesNodeSelectorAndAffinityTerms(const Pod& pod, const KNode& node) {
    if (!pod.nodeSelector.empty()) {
        // labels.SelectorFromSet (selector.go:849-862): Equals requirements
        for (auto& kv : pod.nodeSelector) {
            auto it = node.labels.find(kv.first);
            if (it == node.labels.end() || it->second != kv.second) return false;
        }
    }
    bool nodeAffinityMatches = true;
    if (pod.affinity && pod.affinity->hasNA) {
        if (!pod.affinity->hasNAReq) return true;
        nodeAffinityMatches = nodeAffinityMatches && MatchNodeSelectorTerms(pod.affinity->naReq, node);
    }
    return nodeAffinityMatches;
}

/* Toleration.ToleratesTaint (vendor/k8s.io/api/core/v1/toleration.go:37-56) */
static bool ToleratesTaint(const Toleration& t, const Taint& taint) {
    if (!t.effect.empty() && t.effect != taint.effect) return false;
    if (!t.key.empty() && t.key != taint.key) return false;
    if (t.op.empty() || t.op == "Equal") return t.value == taint.value;
    if (t.op == "Exists") return true;
    return false;
}

/* ------------------------------------------------------------------------ */
/* vendored k8s scheduler cache NodeInfo (pkg/scheduler/cache/node_info.go)  */
/* ------------------------------------------------------------------------ */
struct PP {
    string proto;
    int32_t port;
    bool operator<(const PP& o) const { return proto != o.proto ? proto < o.proto : port < o.port; }
};
typedef map<string, std::set<PP>> HostPortInfo;  // host_ports.go:50-51

static void sanitize(string* ip, string* proto) {
    if (ip->empty()) *ip = "0.0.0.0";
    if (proto->empty()) *proto = "TCP";
}
static void HPAdd(HostPortInfo& h, string ip, string proto, int32_t port) {  // :53-72
    if (port <= 0) return;
    sanitize(&ip, &proto);
    h[ip].insert(PP{proto, port});
}
static bool HPCheckConflict(const HostPortInfo& h, string ip, string proto, int32_t port) {  // :96-125
    if (port <= 0) return false;
    sanitize(&ip, &proto);
    PP pp{proto, port};
    if (ip == "0.0.0.0") {
        for (auto& kv : h) if (kv.second.count(pp)) return true;
        return false;
    }
    for (const string& key : {string("0.0.0.0"), ip}) {
        auto it = h.find(key);
        if (it != h.end() && it->second.count(pp)) return true;
    }
    return false;
}

static void GetNonzeroRequests(const Container& c, int64_t* cpu, int64_t* mem) {  // util/non_zero.go:37-52
    *cpu = (c.has & KBS_HAS_CPU) ? c.cpu : 100;
    *mem = (c.has & KBS_HAS_MEM) ? c.mem : 200LL * 1024 * 1024;
}

struct K8sNodeInfo {
    KNode* node = nullptr;
    vector<Pod*> pods, podsWithAffinity;
    int64_t req_cpu = 0, req_mem = 0, nz_cpu = 0, nz_mem = 0;
    HostPortInfo usedPorts;
    int64_t alloc_cpu = 0, alloc_mem = 0;

    static bool hasPodAffinityConstraints(const Pod* p) {
        return p->affinity && (p->affinity->hasPA || p->affinity->hasPAA);
    }
    void AddPod(Pod* p) {  // :498-521
        for (auto& c : p->containers) {
            req_cpu += c.cpu;
            req_mem += c.mem;
            int64_t a, b;
            GetNonzeroRequests(c, &a, &b);
            nz_cpu += a;
            nz_mem += b;
        }
        pods.push_back(p);
        if (hasPodAffinityConstraints(p)) podsWithAffinity.push_back(p);
        for (auto& c : p->containers)
            for (auto& pt : c.ports) HPAdd(usedPorts, pt.ip, pt.proto, pt.port);
    }
    void SetNode(KNode* n) {  // :608-631
        node = n;
        alloc_cpu = n->a_cpu;
        alloc_mem = n->a_mem;
    }
    bool Filter(const Pod* p) const {  // :692-702
        if (p->nodeName != node->name) return true;
        for (auto* q : pods) if (q->name == p->name && q->ns == p->ns) return true;
        return false;
    }
};

static K8sNodeInfo BuildK8sNodeInfo(const NodeInfo& ni) {  // cache.NewNodeInfo(node.Pods()...) + SetNode
    K8sNodeInfo k;
    for (auto* p : ni.Pods()) k.AddPod(p);
    k.SetNode(ni.Node);
    return k;
}

/* ------------------------------------------------------------------------ */
/* framework.Session + plugins                                               */
/* ------------------------------------------------------------------------ */
struct PluginOption {
    string name;
    int flags = 0;
    map<string, string> args;
};
typedef vector<vector<PluginOption>> Tiers;

struct Session;
typedef std::function<int(void*, void*)> CompareFn;
typedef std::function<bool(TaskInfo*, NodeInfo*, string*)> PredicateFn;  // returns ok
typedef std::function<bool(TaskInfo*, NodeInfo*, int*)> NodeOrderFn;      // returns ok
typedef std::function<int(JobInfo*)> JobReadyFn;
typedef std::function<bool(QueueInfo*)> OverusedFn;

struct EventHandler {  // framework/event.go:27-30
    std::function<void(TaskInfo*)> AllocateFunc;
    std::function<void(TaskInfo*)> DeallocateFunc;
};
typedef std::function<vector<TaskInfo*>(TaskInfo*, const vector<TaskInfo*>&)> EvictableFn;  // api/types.go

struct Session {
    vector<JobInfo*> Jobs;          // pinned order (by job UID)
    map<string, JobInfo*> JobByUID;
    vector<NodeInfo*> Nodes;        // pinned order (by node name)
    map<string, NodeInfo*> NodeByName;
    vector<QueueInfo*> Queues;      // pinned order (by queue name)
    map<string, QueueInfo*> QueueByUID;
    Tiers tiers;
    map<string, CompareFn> jobOrderFns, queueOrderFns, taskOrderFns;
    map<string, PredicateFn> predicateFns;
    map<string, NodeOrderFn> nodeOrderFns;
    map<string, JobReadyFn> jobReadyFns;
    map<string, OverusedFn> overusedFns;
    vector<EventHandler> eventHandlers;
    map<string, EvictableFn> preemptableFns, reclaimableFns;
    std::deque<TaskInfo> clones;  // task.Clone() results (preempt.go:298-300, reclaim.go:138): the job keeps them after an eviction
    // observer: placement log
    vector<std::tuple<int, int, int>> log;  // (pod, node index, status)
    map<string, int> nodeIndex;

    bool JobOrderFn(JobInfo* l, JobInfo* r) {  // session_plugins.go:244-268
        for (auto& tier : tiers)
            for (auto& p : tier) {
                if (p.flags & KBS_DIS_JOBORDER) continue;
                auto it = jobOrderFns.find(p.name);
                if (it == jobOrderFns.end()) continue;
                int j = it->second(l, r);
                if (j != 0) return j < 0;
            }
        if (l->CreationTimestamp == r->CreationTimestamp) return l->UID < r->UID;
        return l->CreationTimestamp < r->CreationTimestamp;
    }
    bool QueueOrderFn(QueueInfo* l, QueueInfo* r) {  // :270-295
        for (auto& tier : tiers)
            for (auto& p : tier) {
                if (p.flags & KBS_DIS_QUEUEORDER) continue;
                auto it = queueOrderFns.find(p.name);
                if (it == queueOrderFns.end()) continue;
                int j = it->second(l, r);
                if (j != 0) return j < 0;
            }
        if (l->ts == r->ts) return l->UID < r->UID;
        return l->ts < r->ts;
    }
    bool TaskOrderFn(TaskInfo* l, TaskInfo* r) {  // :297-329
        for (auto& tier : tiers)
            for (auto& p : tier) {
                if (p.flags & KBS_DIS_TASKORDER) continue;
                auto it = taskOrderFns.find(p.name);
                if (it == taskOrderFns.end()) continue;
                int j = it->second(l, r);
                if (j != 0) return j < 0;
            }
        if (l->P->ts == r->P->ts) return l->uid < r->uid;
        return l->P->ts < r->P->ts;
    }
    bool PredicateFn_(TaskInfo* t, NodeInfo* n) {  // :331-348
        for (auto& tier : tiers)
            for (auto& p : tier) {
                if (p.flags & KBS_DIS_PREDICATE) continue;
                auto it = predicateFns.find(p.name);
                if (it == predicateFns.end()) continue;
                string err;
                if (!it->second(t, n, &err)) return false;
            }
        return true;
    }
    bool NodeOrderFn_(TaskInfo* t, NodeInfo* n, int* score) {  // :350-370
        int priorityScore = 0;
        for (auto& tier : tiers)
            for (auto& p : tier) {
                if (p.flags & KBS_DIS_NODEORDER) continue;
                auto it = nodeOrderFns.find(p.name);
                if (it == nodeOrderFns.end()) continue;
                int s = 0;
                if (!it->second(t, n, &s)) { *score = 0; return false; }
                priorityScore += s;
            }
        *score = priorityScore;
        return true;
    }
    bool JobReady(JobInfo* job) {  // :167-186 — `break` leaves the plugin loop only,
        int status = Ready;          // so the last tier with an enabled JobReadyFn decides
        for (auto& tier : tiers)
            for (auto& p : tier) {
                if (p.flags & KBS_DIS_JOBREADY) continue;
                auto it = jobReadyFns.find(p.name);
                if (it == jobReadyFns.end()) continue;
                status = it->second(job);
                break;
            }
        return status == Ready;
    }
    bool Overused(QueueInfo* q) {  // :150-164
        for (auto& tier : tiers)
            for (auto& p : tier) {
                auto it = overusedFns.find(p.name);
                if (it == overusedFns.end()) continue;
                if (it->second(q)) return true;
            }
        return false;
    }

    // Session.Reclaimable / Preemptable (session_plugins.go:67-148): per tier,
    // the intersection (in victim order) of the enabled plugins' candidates;
    // the first tier whose result is non-nil decides.  A nil result (no plugin
    // yet, or a plugin that returned nothing) lets the next tier decide.
    vector<TaskInfo*> evictable(map<string, EvictableFn>& fns, int disFlag, TaskInfo* evictor,
                                const vector<TaskInfo*>& evictees) {
        vector<TaskInfo*> victims;
        bool init = false, isNil = true;
        for (auto& tier : tiers) {
            for (auto& p : tier) {
                if (p.flags & disFlag) continue;
                auto it = fns.find(p.name);
                if (it == fns.end()) continue;
                vector<TaskInfo*> candidates = it->second(evictor, evictees);
                if (!init) {
                    victims = candidates;
                    isNil = candidates.empty();  // the plugins build their slices by append: empty == nil
                    init = true;
                } else {
                    vector<TaskInfo*> inter;
                    for (auto* v : victims)
                        for (auto* c : candidates)
                            if (v->uid == c->uid) inter.push_back(v);
                    victims = inter;
                    isNil = inter.empty();  // `var intersection []*TaskInfo` stays nil when nothing matches
                }
            }
            if (!isNil) return victims;
        }
        return victims;
    }
    vector<TaskInfo*> Reclaimable(TaskInfo* t, const vector<TaskInfo*>& es) {
        return evictable(reclaimableFns, KBS_DIS_RECLAIMABLE, t, es);
    }
    vector<TaskInfo*> Preemptable(TaskInfo* t, const vector<TaskInfo*>& es) {
        return evictable(preemptableFns, KBS_DIS_PREEMPTABLE, t, es);
    }
    // The session-side half of an eviction (session.go:331-356, statement.go:35-67):
    // job status -> Releasing, node copy updated, Deallocate handlers.
    void evictInSession(TaskInfo* reclaimee) {
        auto jit = JobByUID.find(reclaimee->jobUID);
        if (jit != JobByUID.end()) jit->second->UpdateTaskStatus(reclaimee, Releasing);
        auto nit = NodeByName.find(reclaimee->NodeName);
        if (nit != NodeByName.end()) nit->second->UpdateTask(*reclaimee);
        for (auto& eh : eventHandlers) if (eh.DeallocateFunc) eh.DeallocateFunc(reclaimee);
    }
    void logEvict(TaskInfo* t) { log.emplace_back(t->pod, nodeIndex[t->NodeName], Releasing); }  // cache.Evict
    void Evict(TaskInfo* reclaimee) {  // session.go:323-359 (the fake cache's Evict never fails)
        logEvict(reclaimee);
        evictInSession(reclaimee);
    }
    void Pipeline(TaskInfo* task, NodeInfo* node) {  // session.go:199-235
        auto jit = JobByUID.find(task->jobUID);
        if (jit != JobByUID.end()) jit->second->UpdateTaskStatus(task, Pipelined);
        task->NodeName = node->Name;
        node->AddTask(*task);
        for (auto& eh : eventHandlers) if (eh.AllocateFunc) eh.AllocateFunc(task);
        log.emplace_back(task->pod, nodeIndex[node->Name], Pipelined);
    }
    bool Allocate(TaskInfo* task, NodeInfo* node, bool usingBackfillTaskRes) {  // :237-297
        auto jit = JobByUID.find(task->jobUID);
        if (jit == JobByUID.end()) return false;
        JobInfo* job = jit->second;
        job->UpdateTaskStatus(task, usingBackfillTaskRes ? AllocatedOverBackfill : Allocated);
        task->NodeName = node->Name;
        if (!node->AddTask(*task)) return false;
        for (auto& eh : eventHandlers) if (eh.AllocateFunc) eh.AllocateFunc(task);
        log.emplace_back(task->pod, nodeIndex[node->Name], task->Status);
        if (JobReady(job)) {
            // dispatch every Allocated task (session.go:299-321): status -> Binding
            auto it = job->TaskStatusIndex.find(Allocated);
            if (it != job->TaskStatusIndex.end()) {
                vector<TaskInfo*> ts;
                for (auto& kv : it->second) ts.push_back(kv.second);
                for (auto* t : ts) job->UpdateTaskStatus(t, Binding);
            }
        }
        return true;
    }
};

/* the plugins' state shared with the session open (kbref_plugins.cpp) */
struct DrfState {
    Resource total;
    map<string, Resource> allocated;
    map<string, double> share;
};

struct QueueAttr {
    string queueID, name;
    int32_t weight = 0;
    double share = 0;
    Resource deserved, allocated, request;
};

struct PropState {
    Resource total;
    map<string, QueueAttr> opts;
    vector<string> order;  // pinned iteration order of queueOpts (by queue index)
};

/* plugin open functions (kbref_plugins.cpp) */
void priorityOpen(Session& ssn, const PluginOption&);
void gangOpen(Session& ssn, const PluginOption&);
void conformanceOpen(Session& ssn, const PluginOption&);
void drfOpen(Session& ssn, const PluginOption&, std::shared_ptr<DrfState> st);
void propOpen(Session& ssn, const PluginOption&, std::shared_ptr<PropState> st);
void predicatesOpen(Session& ssn, const PluginOption&);
void nodeorderOpen(Session& ssn, const PluginOption& opt);

}  // namespace ref
