/*
 * kbfast.h — TEST ORACLE (hoisted restatement, CPU baseline), shared header of
 * kbfast.cpp and kbfast_load.cpp.  Test infrastructure only (see kbfast.cpp).
 */
#pragma once
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../include/kbsnap.h"

namespace fast {

using std::string;
using std::vector;

static const int64_t kMinCPU = 10, kMinGPU = 10, kMinMem = 10LL * 1024 * 1024;  // resource_info.go:54-56

struct Res {
    int64_t cpu = 0, mem = 0, gpu = 0;
    Res& operator+=(const Res& o) { cpu += o.cpu; mem += o.mem; gpu += o.gpu; return *this; }
    Res& operator-=(const Res& o) { cpu -= o.cpu; mem -= o.mem; gpu -= o.gpu; return *this; }
};
// Resource.LessEqual on exact integers: r - rr < min per dimension (resource_info.go:164-168)
static inline bool le(const Res& r, const Res& rr) {
    return r.cpu - rr.cpu < kMinCPU && r.mem - rr.mem < kMinMem && r.gpu - rr.gpu < kMinGPU;
}
static inline bool le_sum(const Res& r, const Res& a, const Res& b) {
    return r.cpu - (a.cpu + b.cpu) < kMinCPU && r.mem - (a.mem + b.mem) < kMinMem && r.gpu - (a.gpu + b.gpu) < kMinGPU;
}
static inline bool isEmpty(const Res& r) { return r.cpu < kMinCPU && r.mem < kMinMem && r.gpu < kMinGPU; }

// float64 Resource for the ordering plugins (drf / proportion shares)
struct FRes {
    double c = 0, m = 0, g = 0;
    void add(const FRes& o) { c += o.c; m += o.m; g += o.g; }
    void sub(const FRes& o) { c -= o.c; m -= o.m; g -= o.g; }
    double get(int k) const { return k == 0 ? c : k == 1 ? m : g; }
    bool lessEqual(const FRes& rr) const {
        return (c < rr.c || std::fabs(rr.c - c) < (double)kMinCPU) &&
               (m < rr.m || std::fabs(rr.m - m) < (double)kMinMem) &&
               (g < rr.g || std::fabs(rr.g - g) < (double)kMinGPU);
    }
    bool isEmpty() const { return c < (double)kMinCPU && m < (double)kMinMem && g < (double)kMinGPU; }
};
static FRes toF(const Res& r) { return FRes{(double)r.cpu, (double)r.mem, (double)r.gpu}; }
static double share(double l, double r) { return r == 0 ? (l == 0 ? 0 : 1) : l / r; }

enum St { Pending = 1, AOB = 2, Allocated = 4, Pipelined = 8, Binding = 16, Bound = 32, Running = 64,
          Releasing = 128, Succeeded = 256, Failed = 512, Unknown = 1024 };
static inline bool allocSt(int s) { return s == Bound || s == Binding || s == Running || s == Allocated; }

/* --------------------------- dictionaries ------------------------------- */
struct Dict {
    std::unordered_map<string, int> ids;
    vector<string> strs;
    int get(const string& s) {
        auto it = ids.find(s);
        if (it != ids.end()) return it->second;
        int id = (int)strs.size();
        ids.emplace(s, id);
        strs.push_back(s);
        return id;
    }
    int find(const string& s) const {
        auto it = ids.find(s);
        return it == ids.end() ? -1 : it->second;
    }
};

static bool parseI64(const string& s, int64_t* out) {  // strconv.ParseInt(s, 10, 64)
    if (s.empty()) return false;
    size_t i = 0;
    bool neg = false;
    if (s[0] == '+' || s[0] == '-') { neg = s[0] == '-'; i = 1; if (s.size() == 1) return false; }
    unsigned long long v = 0, lim = neg ? 9223372036854775808ULL : 9223372036854775807ULL;
    for (; i < s.size(); ++i) {
        if (s[i] < '0' || s[i] > '9') return false;
        unsigned d = (unsigned)(s[i] - '0');
        if (v > (lim - d) / 10) return false;
        v = v * 10 + d;
    }
    *out = neg ? (int64_t)(0 - v) : (int64_t)v;
    return true;
}

/* A label set as a sorted (key id -> value id) vector. */
typedef vector<std::pair<int, int>> LSet;
static inline int lget(const LSet& l, int key) {
    auto it = std::lower_bound(l.begin(), l.end(), std::make_pair(key, INT32_MIN));
    return (it != l.end() && it->first == key) ? it->second : -1;
}

enum { OIn = 0, ONotIn = 1, OExists = 2, ODNE = 3, OGt = 4, OLt = 5, OEq = 6 };
struct Req {  // compiled labels.Requirement
    int key;
    int op;
    vector<int> vals;  // value ids (-1 for values never seen: they match nothing)
    int64_t rhs = 0;   // Gt/Lt
};
struct Sel {  // compiled selector: nothing / AND of reqs
    bool nothing = false;
    vector<Req> reqs;
};

struct World;
static bool reqMatch(const World& w, const Req& r, const LSet& ls);

/* --------------------------- model -------------------------------------- */
struct PATerm {  // compiled PodAffinityTerm
    Sel sel;
    bool selErr = false;
    vector<int> ns;  // namespace ids (empty => definer's namespace)
    int key = -1;    // topology key id (-1 == "")
};
struct WTerm {
    int32_t w;
    PATerm t;
};
struct NSTerm {
    vector<Req> expr;
    bool exprErr = false;
    vector<std::pair<int, string>> fields;  // (op, value) on metadata.name; key checked at compile
    vector<string> fieldKeys;
    bool fieldErr = false;
};
struct Aff {
    bool na = false, naReq = false, pa = false, paa = false;
    vector<NSTerm> naReqTerms;
    vector<std::pair<int32_t, NSTerm>> naPref;
    vector<PATerm> paReq, paaReq;
    vector<WTerm> paPref, paaPref;
};
struct Port {
    int ip, proto;  // sanitised ids
    int32_t port;
};
struct PodRec {
    string uid, name;
    int ns = -1;
    LSet labels;
    int nodeRaw = -1;  // node index of raw Spec.NodeName (-1 "")
    int status = Pending;
    int32_t priority = 0;
    int64_t ts = 0;
    bool backfill = false;
    Res req, initReq;
    int64_t nzc = 0, nzm = 0;
    vector<Port> ports;
    vector<std::pair<int, int>> nsel;  // (key, value) required
    vector<int> tolTaints;             // tolerated taint ids (computed later)
    std::shared_ptr<Aff> aff;
    int job = -1;  // session job slot
    string jobUID;
    int curNode = -1;  // task.NodeName (node index)
    bool detached = false;  // p_detached: in its job with its NodeName, off the node
    bool critical = false;  // kube-system or a system-*-critical priority class (conformance.go:40-45)
    bool nodeRel = false;   // the node's copy stayed Releasing after an unevict (statement.go:81-105)
    bool hasPodAff() const { return aff && (aff->pa || aff->paa); }
};
struct NodeRec {
    string name;
    LSet labels;
    vector<int> taints;  // NoSchedule/NoExecute taint ids
    bool unsched = false;
    int maxTasks = 0;
    Res alloc, idle, used, rel, bf;
    int64_t acpu = 0, amem = 0;  // k8s allocatable
    int64_t nzc = 0, nzm = 0;    // k8s nonzeroRequest over node.Pods()
    int pods = 0;
    vector<Port> used_ports;  // sanitised (ip, proto, port>0)
    vector<int> podList;      // pods on node (all statuses), pinned order by insertion
    bool hasEmptyNamePod = false;  // some pod on it has raw Spec.NodeName == ""
};
struct JobRec {
    string uid;
    int queue = -1;
    int32_t minAvail = 0, priority = 0;
    int64_t ts = 0;
    vector<int> tasks;  // pod indices, pinned order
    int cntAlloc = 0, cntAOB = 0;  // AllocatedStatuses count, AllocatedOverBackfill count
    FRes drfAlloc;
    double drfShare = 0;
};
struct QueueRec {
    string name;
    int32_t weight = 1;
    int64_t ts = 0;
    bool hasAttr = false;
    FRes deserved, allocated, request;
    double share = 0;
};
struct Plugin {
    string name;
    int flags = 0;
    std::map<string, string> args;
};

struct World {
    Dict keys, vals, nss, ips, protos;
    vector<std::map<int, int64_t>> intVal;  // not used
    vector<NodeRec> nodes;
    vector<PodRec> pods;
    vector<JobRec> jobs;
    vector<QueueRec> queues;
    vector<vector<Plugin>> tiers;
    vector<std::tuple<int, int, string>> taintDefs;  // (key id, value, effect)
    // value id -> parsed int64 (for Gt/Lt)
    vector<int64_t> valInt;
    vector<char> valIntOk;
    // plugin presence
    bool predOn = false, nodeorderOn = false, drfOn = false, propOn = false, gangOn = false, prioOn = false;
    int wLR = 1, wBRA = 1, wNA = 1, wPA = 1, noMult = 0;
    FRes total;
    // pod-affinity bookkeeping
    vector<int> affPods;  // pods (anywhere on nodes) with PodAffinity/PodAntiAffinity
    bool anyBackfilled = false;
    int fallbackNode = -1;  // lowest node index holding a pod with empty raw NodeName
    vector<std::tuple<int, int, int>> log;
};

static bool reqMatch(const World& w, const Req& r, const LSet& ls) {  // selector.go:192-236
    int v = lget(ls, r.key);
    switch (r.op) {
        case OIn:
        case OEq:
            if (v < 0) return false;
            for (int x : r.vals) if (x == v) return true;
            return false;
        case ONotIn:
            if (v < 0) return true;
            for (int x : r.vals) if (x == v) return false;
            return true;
        case OExists: return v >= 0;
        case ODNE: return v < 0;
        case OGt:
        case OLt: {
            if (v < 0 || !w.valIntOk[v]) return false;
            int64_t lv = w.valInt[v];
            return r.op == OGt ? lv > r.rhs : lv < r.rhs;
        }
    }
    return false;
}
static bool selMatch(const World& w, const Sel& s, const LSet& ls) {
    if (s.nothing) return false;
    for (auto& r : s.reqs) if (!reqMatch(w, r, ls)) return false;
    return true;
}

/* the snapshot into the World (kbfast_load.cpp) */
void load_world(const kbs::Snapshot& s, World& w);

}  // namespace fast
