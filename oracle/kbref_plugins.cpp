/*
 * kbref_plugins.cpp — TEST ORACLE: the plugins of the faithful restatement
 * (priority, gang, conformance, drf, proportion, predicates, nodeorder).  Test
 * infrastructure only (see kbref.cpp).
 */
#include "kbref.h"

namespace ref {

/* ---- priority plugin (plugins/priority/priority.go:38-79) ---------------- */
void priorityOpen(Session& ssn, const PluginOption&) {
    ssn.taskOrderFns["priority"] = [](void* l, void* r) {
        auto* lv = (TaskInfo*)l;
        auto* rv = (TaskInfo*)r;
        if (lv->Priority == rv->Priority) return 0;
        if (lv->Priority > rv->Priority) return -1;
        return 1;
    };
    ssn.jobOrderFns["priority"] = [](void* l, void* r) {
        auto* lv = (JobInfo*)l;
        auto* rv = (JobInfo*)r;
        if (lv->Priority > rv->Priority) return -1;
        if (lv->Priority < rv->Priority) return 1;
        return 0;
    };
}

/* ---- gang plugin (plugins/gang/gang.go:82-164) --------------------------- */
void gangOpen(Session& ssn, const PluginOption&) {
    ssn.jobOrderFns["gang"] = [](void* l, void* r) {
        bool lReady = ((JobInfo*)l)->GetReadiness() == Ready;
        bool rReady = ((JobInfo*)r)->GetReadiness() == Ready;
        if (lReady && rReady) return 0;
        if (lReady) return 1;
        if (rReady) return -1;
        return 0;
    };
    ssn.jobReadyFns["gang"] = [](JobInfo* j) { return j->GetReadiness(); };
    // preemptableFn (gang.go:107-129), registered as both Reclaimable and Preemptable
    Session* sp = &ssn;
    EvictableFn pf = [sp](TaskInfo*, const vector<TaskInfo*>& preemptees) {
        vector<TaskInfo*> victims;
        for (auto* preemptee : preemptees) {
            JobInfo* job = sp->JobByUID[preemptee->jobUID];
            int ready = 0;  // readyTaskNum (gang.go:212-222)
            for (auto& kv : job->TaskStatusIndex)
                if (AllocatedStatus(kv.first) || kv.first == Succeeded || kv.first == Pipelined)
                    ready += (int)kv.second.size();
            if (job->MinAvailable <= ready - 1 || job->MinAvailable == 1) victims.push_back(preemptee);
        }
        return victims;
    };
    ssn.reclaimableFns["gang"] = pf;
    ssn.preemptableFns["gang"] = pf;
}

/* ---- conformance plugin (plugins/conformance/conformance.go:37-61) ------- */
void conformanceOpen(Session& ssn, const PluginOption&) {
    EvictableFn ef = [](TaskInfo*, const vector<TaskInfo*>& evictees) {
        vector<TaskInfo*> victims;
        for (auto* e : evictees) {
            const string& cls = e->P->priorityClassName;
            if (cls == "system-cluster-critical" || cls == "system-node-critical" || e->ns == "kube-system") continue;
            victims.push_back(e);
        }
        return victims;
    };
    ssn.preemptableFns["conformance"] = ef;
    ssn.reclaimableFns["conformance"] = ef;
}

/* ---- drf plugin (plugins/drf/drf.go:59-170) ------------------------------ */
static double drfShare(const Resource& alloc, const Resource& total) {  // :160-170
    double res = 0;
    for (int rn = 0; rn < 3; ++rn) {
        double s = Share(alloc.Get(rn), total.Get(rn));
        if (s > res) res = s;
    }
    return res;
}
void drfOpen(Session& ssn, const PluginOption&, std::shared_ptr<DrfState> st) {
    for (auto* n : ssn.Nodes) st->total.Add(n->Allocatable);
    for (auto* job : ssn.Jobs) {
        Resource a;
        for (auto& kv : job->TaskStatusIndex)
            if (AllocatedStatus(kv.first))
                for (auto& t : kv.second) a.Add(t.second->Resreq);
        st->allocated[job->UID] = a;
        st->share[job->UID] = drfShare(a, st->total);
    }
    // preemptableFn (drf.go:84-109)
    ssn.preemptableFns["drf"] = [st](TaskInfo* preemptor, const vector<TaskInfo*>& preemptees) {
        vector<TaskInfo*> victims;
        Resource lalloc = st->allocated[preemptor->jobUID];
        lalloc.Add(preemptor->Resreq);
        double ls = drfShare(lalloc, st->total);
        map<string, Resource> allocations;
        for (auto* preemptee : preemptees) {
            if (!allocations.count(preemptee->jobUID)) allocations[preemptee->jobUID] = st->allocated[preemptee->jobUID];
            Resource& ralloc = allocations[preemptee->jobUID].Sub(preemptee->Resreq);
            double rs = drfShare(ralloc, st->total);
            if (ls < rs || std::fabs(ls - rs) <= 0.000001) victims.push_back(preemptee);  // shareDelta (drf.go:29)
        }
        return victims;
    };
    ssn.jobOrderFns["drf"] = [st](void* l, void* r) {
        double ls = st->share[((JobInfo*)l)->UID], rs = st->share[((JobInfo*)r)->UID];
        if (ls == rs) return 0;
        if (ls < rs) return -1;
        return 1;
    };
    EventHandler eh;
    eh.AllocateFunc = [st](TaskInfo* t) {
        Resource& a = st->allocated[t->jobUID];
        a.Add(t->Resreq);
        st->share[t->jobUID] = drfShare(a, st->total);
    };
    eh.DeallocateFunc = [st](TaskInfo* t) {  // drf.go:144-151
        Resource& a = st->allocated[t->jobUID];
        a.Sub(t->Resreq);
        st->share[t->jobUID] = drfShare(a, st->total);
    };
    ssn.eventHandlers.push_back(eh);
}

/* ---- proportion plugin (plugins/proportion/proportion.go:57-241) --------- */
static void propUpdateShare(QueueAttr& a) {  // :229-241
    double res = 0;
    for (int rn = 0; rn < 3; ++rn) {
        double s = Share(a.allocated.Get(rn), a.deserved.Get(rn));
        if (s > res) res = s;
    }
    a.share = res;
}
void propOpen(Session& ssn, const PluginOption&, std::shared_ptr<PropState> st) {
    for (auto* n : ssn.Nodes) st->total.Add(n->Allocatable);
    for (auto* job : ssn.Jobs) {
        if (!st->opts.count(job->Queue)) {
            QueueInfo* q = ssn.QueueByUID[job->Queue];
            QueueAttr a;
            a.queueID = q->UID;
            a.name = q->Name;
            a.weight = q->Weight;
            st->opts[job->Queue] = a;
        }
        QueueAttr& a = st->opts[job->Queue];
        for (auto& kv : job->TaskStatusIndex) {
            if (AllocatedStatus(kv.first)) {
                for (auto& t : kv.second) { a.allocated.Add(t.second->Resreq); a.request.Add(t.second->Resreq); }
            } else if (kv.first == Pending) {
                for (auto& t : kv.second) a.request.Add(t.second->Resreq);
            }
        }
    }
    for (auto* q : ssn.Queues) if (st->opts.count(q->UID)) st->order.push_back(q->UID);
    Resource remaining = st->total;
    std::set<string> meet;
    for (;;) {
        int32_t totalWeight = 0;
        for (auto& id : st->order) if (!meet.count(id)) totalWeight += st->opts[id].weight;
        if (totalWeight == 0) break;
        Resource deserved;
        for (auto& id : st->order) {
            QueueAttr& a = st->opts[id];
            if (meet.count(id)) continue;
            Resource r = remaining;
            a.deserved.Add(r.Multi((double)a.weight / (double)totalWeight));
            if (!a.deserved.LessEqual(a.request)) {
                a.deserved = MinRes(a.deserved, a.request);
                meet.insert(id);
            }
            propUpdateShare(a);
            deserved.Add(a.deserved);
        }
        remaining.Sub(deserved);
        if (remaining.IsEmpty()) break;
    }
    ssn.queueOrderFns["proportion"] = [st](void* l, void* r) {
        double ls = st->opts[((QueueInfo*)l)->UID].share, rs = st->opts[((QueueInfo*)r)->UID].share;
        if (ls == rs) return 0;
        if (ls < rs) return -1;
        return 1;
    };
    // reclaimableFn (proportion.go:159-183)
    ssn.reclaimableFns["proportion"] = [st, &ssn](TaskInfo*, const vector<TaskInfo*>& reclaimees) {
        vector<TaskInfo*> victims;
        map<string, Resource> allocations;
        for (auto* reclaimee : reclaimees) {
            JobInfo* job = ssn.JobByUID[reclaimee->jobUID];
            QueueAttr& attr = st->opts[job->Queue];
            if (!allocations.count(job->Queue)) allocations[job->Queue] = attr.allocated;
            Resource& allocated = allocations[job->Queue];
            if (allocated.Less(reclaimee->Resreq)) continue;
            allocated.Sub(reclaimee->Resreq);
            if (attr.deserved.LessEqual(allocated)) victims.push_back(reclaimee);
        }
        return victims;
    };
    ssn.overusedFns["proportion"] = [st](QueueInfo* q) {
        QueueAttr& a = st->opts[q->UID];
        return a.deserved.LessEqual(a.allocated);
    };
    Session* sp = &ssn;
    EventHandler eh;
    eh.AllocateFunc = [st, sp](TaskInfo* t) {
        JobInfo* job = sp->JobByUID[t->jobUID];
        QueueAttr& a = st->opts[job->Queue];
        a.allocated.Add(t->Resreq);
        propUpdateShare(a);
    };
    eh.DeallocateFunc = [st, sp](TaskInfo* t) {  // proportion.go:211-219
        JobInfo* job = sp->JobByUID[t->jobUID];
        QueueAttr& a = st->opts[job->Queue];
        a.allocated.Sub(t->Resreq);
        propUpdateShare(a);
    };
    ssn.eventHandlers.push_back(eh);
}

/* ---- predicates plugin (plugins/predicates/predicates.go:114-204) -------- */

// podLister.FilteredList (predicates.go:72-91): allocated-status tasks of all
// session jobs, copied with Spec.NodeName = task.NodeName.
struct ListedPod {
    Pod* pod;
    string nodeName;  // overridden Spec.NodeName
};
static vector<ListedPod> predFilteredList(Session& ssn, const K8sNodeInfo& ni) {
    vector<ListedPod> out;
    for (auto* job : ssn.Jobs)
        for (auto& kv : job->TaskStatusIndex) {
            if (!AllocatedStatus(kv.first)) continue;
            for (auto& t : kv.second) {
                TaskInfo* task = t.second;
                if (ni.Filter(task->P)) out.push_back({task->P, task->NodeName});
            }
        }
    return out;
}

// priorityutil.GetNamespacesFromPodAffinityTerm / PodMatchesTermsNamespaceAndSelector
static std::set<string> termNamespaces(const Pod& definer, const PodAffinityTerm& t) {
    std::set<string> s;
    if (t.namespaces.empty()) s.insert(definer.ns);
    else s.insert(t.namespaces.begin(), t.namespaces.end());
    return s;
}
static bool podMatchesTermsNamespaceAndSelector(const Pod& pod, const std::set<string>& nss, const Selector& sel) {
    if (!nss.count(pod.ns)) return false;
    return sel.Matches(pod.labels);
}

// priorityutil.NodesHaveSameTopologyKey (util/topologies.go:53-75)
static bool NodesHaveSameTopologyKey(const KNode* a, const KNode* b, const string& key) {
    if (key.empty()) return false;
    auto ia = a->labels.find(key), ib = b->labels.find(key);
    if (ia != a->labels.end() && ib != b->labels.end()) return ia->second == ib->second;
    return false;
}

struct PredErr {};

// predicates cachedNodeInfo.GetNodeInfo (predicates.go:97-104): no fallback
static KNode* predGetNode(Session& ssn, const string& name) {
    auto it = ssn.NodeByName.find(name);
    if (it == ssn.NodeByName.end()) throw PredErr();
    return it->second->Node;
}

// podMatchesPodAffinityTerms (predicates.go:1189-1215): returns {match, propsMatch}; throws on error
static std::pair<bool, bool> podMatchesPodAffinityTerms(Session& ssn, const Pod& pod, const ListedPod& target,
                                                        const K8sNodeInfo& ni,
                                                        const vector<PodAffinityTerm>& terms) {
    if (terms.empty()) throw PredErr();
    // getAffinityTermProperties + podMatchesAllAffinityTermProperties
    for (auto& term : terms) {
        Selector sel;
        if (!LabelSelectorAsSelector(term.sel.get(), &sel)) throw PredErr();
    }
    for (auto& term : terms) {
        Selector sel;
        LabelSelectorAsSelector(term.sel.get(), &sel);
        if (!podMatchesTermsNamespaceAndSelector(*target.pod, termNamespaces(pod, term), sel))
            return {false, false};
    }
    KNode* targetNode = predGetNode(ssn, target.nodeName);
    for (auto& term : terms) {
        if (term.topologyKey.empty()) throw PredErr();
        if (!NodesHaveSameTopologyKey(ni.node, targetNode, term.topologyKey)) return {false, true};
    }
    return {true, true};
}

static bool targetPodMatchesAffinityOfPod(const Pod& pod, const Pod& target) {  // metadata.go:498-509
    if (!pod.affinity || !pod.affinity->hasPA) return false;
    const auto& terms = pod.affinity->paReq;
    if (terms.empty()) return false;  // podMatchesAllAffinityTermProperties: no properties -> false
    for (auto& term : terms) {
        Selector sel;
        if (!LabelSelectorAsSelector(term.sel.get(), &sel)) return false;
        if (!podMatchesTermsNamespaceAndSelector(target, termNamespaces(pod, term), sel)) return false;
    }
    return true;
}

// InterPodAffinityMatches slow path (predicates.go:1155-1184, 1293-1334, 1402-1458)
static bool InterPodAffinityMatches(Session& ssn, const Pod& pod, const K8sNodeInfo& ni) {
    try {
        // satisfiesExistingPodsAntiAffinity
        vector<ListedPod> filtered = predFilteredList(ssn, ni);
        std::set<std::pair<string, string>> forbidden;
        for (auto& ep : filtered) {
            KNode* epNode = predGetNode(ssn, ep.nodeName);
            const Pod& existing = *ep.pod;
            if (!existing.affinity || !existing.affinity->hasPAA) continue;
            for (auto& term : existing.affinity->paaReq) {
                Selector sel;
                if (!LabelSelectorAsSelector(term.sel.get(), &sel)) throw PredErr();
                if (podMatchesTermsNamespaceAndSelector(pod, termNamespaces(existing, term), sel)) {
                    auto it = epNode->labels.find(term.topologyKey);
                    if (it != epNode->labels.end()) forbidden.insert({term.topologyKey, it->second});
                }
            }
        }
        for (auto& kv : ni.node->labels)
            if (forbidden.count({kv.first, kv.second})) return false;

        if (!pod.affinity || (!pod.affinity->hasPA && !pod.affinity->hasPAA)) return true;
        // satisfiesPodsAffinityAntiAffinity, meta == nil branch
        const vector<PodAffinityTerm> empty;
        const auto& affinityTerms = pod.affinity->hasPA ? pod.affinity->paReq : empty;
        const auto& antiAffinityTerms = pod.affinity->hasPAA ? pod.affinity->paaReq : empty;
        bool matchFound = false, termsSelectorMatchFound = false;
        for (auto& target : filtered) {
            if (!matchFound && !affinityTerms.empty()) {
                auto r = podMatchesPodAffinityTerms(ssn, pod, target, ni, affinityTerms);
                if (r.second) termsSelectorMatchFound = true;
                if (r.first) matchFound = true;
            }
            if (!antiAffinityTerms.empty()) {
                try {
                    auto r = podMatchesPodAffinityTerms(ssn, pod, target, ni, antiAffinityTerms);
                    if (r.first) return false;
                } catch (PredErr&) {
                    return false;
                }
            }
        }
        if (!matchFound && !affinityTerms.empty()) {
            if (termsSelectorMatchFound) return false;
            if (!targetPodMatchesAffinityOfPod(pod, pod)) return false;
        }
        return true;
    } catch (PredErr&) {
        return false;
    }
}

void predicatesOpen(Session& ssn, const PluginOption&) {
    Session* sp = &ssn;
    ssn.predicateFns["predicates"] = [sp](TaskInfo* task, NodeInfo* node, string* err) {
        K8sNodeInfo ni = BuildK8sNodeInfo(*node);
        if (node->Allocatable.MaxTaskNum <= (int)ni.pods.size()) { *err = "maxtasks"; return false; }
        const Pod& pod = *task->P;
        if (!podMatchesNodeSelectorAndAffinityTerms(pod, *node->Node)) { *err = "selector"; return false; }
        // PodFitsHostPorts (predicates.go:1031-1052)
        for (auto& c : pod.containers)
            for (auto& pt : c.ports)
                if (HPCheckConflict(ni.usedPorts, pt.ip, pt.proto, pt.port)) { *err = "ports"; return false; }
        // CheckNodeUnschedulable (predicates.go:107-112)
        if (node->Node->unschedulable) { *err = "unschedulable"; return false; }
        // PodToleratesNodeTaints (predicates.go:1489-1499, helper/helpers.go:425-440)
        for (auto& taint : node->Node->taints) {
            if (taint.effect != "NoSchedule" && taint.effect != "NoExecute") continue;
            bool tol = false;
            for (auto& t : pod.tolerations) if (ToleratesTaint(t, taint)) { tol = true; break; }
            if (!tol) { *err = "taints"; return false; }
        }
        if (!InterPodAffinityMatches(*sp, pod, ni)) { *err = "podaffinity"; return false; }
        return true;
    };
}

/* ---- nodeorder plugin (plugins/nodeorder/nodeorder.go:177-319) ----------- */
struct Weights {
    int leastReq = 1, nodeAffinity = 1, podAffinity = 1, balanced = 1;
};
static bool atoi_go(const string& s, int* out) {  // strconv.Atoi
    int64_t v;
    if (!parseInt64(s, &v)) return false;
    if (v < INT32_MIN || v > INT32_MAX) { /* Go int is 64-bit; keep within int */ }
    *out = (int)v;
    return true;
}
static Weights calculateWeight(const map<string, string>& args) {  // :177-249
    Weights w;
    auto get = [&](const char* k, int* dst) {
        auto it = args.find(k);
        if (it != args.end() && !it->second.empty()) {
            int v;
            if (atoi_go(it->second, &v)) *dst = v;
        }
    };
    get("nodeaffinity.weight", &w.nodeAffinity);
    get("podaffinity.weight", &w.podAffinity);
    get("leastrequested.weight", &w.leastReq);
    get("balancedresource.weight", &w.balanced);
    return w;
}

static int64_t leastRequestedScore(int64_t requested, int64_t capacity) {  // least_requested.go:44-53
    if (capacity == 0) return 0;
    if (requested > capacity) return 0;
    return ((capacity - requested) * 10) / capacity;
}
static double fractionOfCapacity(int64_t requested, int64_t capacity) {  // balanced_resource_allocation.go:72-77
    if (capacity == 0) return 1;
    return (double)requested / (double)capacity;
}

static void podNonZero(const Pod& p, int64_t* cpu, int64_t* mem) {  // resource_allocation.go:94-103
    *cpu = 0;
    *mem = 0;
    for (auto& c : p.containers) {
        int64_t a, b;
        GetNonzeroRequests(c, &a, &b);
        *cpu += a;
        *mem += b;
    }
}

// nodeorder cachedNodeInfo.GetNodeInfo with the empty-NodeName fallback (:78-93)
static KNode* noGetNode(Session& ssn, const string& name, bool* ok) {
    *ok = true;
    auto it = ssn.NodeByName.find(name);
    if (it != ssn.NodeByName.end()) return it->second->Node;
    for (auto* n : ssn.Nodes)
        for (auto* p : n->Pods())
            if (p->nodeName.empty()) return n->Node;
    *ok = false;
    return nullptr;
}

// CalculateInterPodAffinityPriority (interpod_affinity.go:119-240); returns false on error
static bool interPodAffinityScores(Session& ssn, const Pod& pod, map<string, int>* out) {
    const Affinity* aff = pod.affinity.get();
    bool hasAff = aff && aff->hasPA;
    bool hasAnti = aff && aff->hasPAA;
    map<string, double> counts;
    bool err = false;
    auto processTerm = [&](const PodAffinityTerm& term, const Pod& definer, const Pod& toCheck,
                           const KNode* fixed, double weight) {
        Selector sel;
        if (!LabelSelectorAsSelector(term.sel.get(), &sel)) { err = true; return; }
        if (podMatchesTermsNamespaceAndSelector(toCheck, termNamespaces(definer, term), sel)) {
            for (auto* n : ssn.Nodes)
                if (NodesHaveSameTopologyKey(n->Node, fixed, term.topologyKey)) counts[n->Name] += weight;
        }
    };
    auto processTerms = [&](const vector<WeightedPodAffinityTerm>& terms, const Pod& definer, const Pod& toCheck,
                            const KNode* fixed, int mult) {
        for (auto& t : terms) processTerm(t.term, definer, toCheck, fixed, (double)(t.weight * mult));
    };
    auto processPod = [&](const Pod& existing) {
        bool ok;
        KNode* epNode = noGetNode(ssn, existing.nodeName, &ok);
        if (!ok) { err = true; return; }
        const Affinity* ea = existing.affinity.get();
        bool eAff = ea && ea->hasPA, eAnti = ea && ea->hasPAA;
        if (hasAff) processTerms(aff->paPref, pod, existing, epNode, 1);
        if (hasAnti) processTerms(aff->paaPref, pod, existing, epNode, -1);
        if (eAff) {
            for (auto& term : ea->paReq) processTerm(term, existing, pod, epNode, 1.0);  // hardPodAffinityWeight
            processTerms(ea->paPref, existing, pod, epNode, 1);
        }
        if (eAnti) processTerms(ea->paaPref, existing, pod, epNode, -1);
    };
    for (auto* n : ssn.Nodes) {  // processNode over all nodes (16-way in the reference; sums are exact)
        K8sNodeInfo ni = BuildK8sNodeInfo(*n);
        const vector<Pod*>& pods = (hasAff || hasAnti) ? ni.pods : ni.podsWithAffinity;
        for (auto* p : pods) processPod(*p);
    }
    if (err) return false;
    double maxCount = 0, minCount = 0;
    for (auto* n : ssn.Nodes) {
        double c = counts[n->Name];
        if (c > maxCount) maxCount = c;
        if (c < minCount) minCount = c;
    }
    for (auto* n : ssn.Nodes) {
        double f = 0;
        if (maxCount - minCount > 0) f = 10.0 * ((counts[n->Name] - minCount) / (maxCount - minCount));
        (*out)[n->Name] = (int)f;
    }
    return true;
}

void nodeorderOpen(Session& ssn, const PluginOption& opt) {
    Session* sp = &ssn;
    map<string, string> args = opt.args;
    ssn.nodeOrderFns["nodeorder"] = [sp, args](TaskInfo* task, NodeInfo* node, int* out) {
        Weights weight = calculateWeight(args);
        Session& s = *sp;
        // generateNodeMapAndSlice(ssn.Nodes) is rebuilt inside the IPA below
        K8sNodeInfo ni = BuildK8sNodeInfo(*node);
        const Pod& pod = *task->P;
        int score = 0;
        int64_t rc, rm;
        podNonZero(pod, &rc, &rm);
        rc += ni.nz_cpu;
        rm += ni.nz_mem;
        // LeastRequestedPriorityMap
        int64_t lr = (leastRequestedScore(rc, ni.alloc_cpu) + leastRequestedScore(rm, ni.alloc_mem)) / 2;
        score += (int)lr * weight.leastReq;
        // BalancedResourceAllocationMap
        double cpuF = fractionOfCapacity(rc, ni.alloc_cpu), memF = fractionOfCapacity(rm, ni.alloc_mem);
        int64_t bra;
        if (cpuF >= 1 || memF >= 1) bra = 0;
        else {
            double diff = std::fabs(cpuF - memF);
            volatile double t = 1 - diff;  // no contraction: Go rounds each op
            bra = (int64_t)(t * 10.0);
        }
        score += (int)bra * weight.balanced;
        // CalculateNodeAffinityPriorityMap
        int32_t count = 0;
        if (pod.affinity && pod.affinity->hasNA) {
            for (auto& pt : pod.affinity->naPref) {
                if (pt.first == 0) continue;
                Selector sel;
                if (!NodeSelectorRequirementsAsSelector(pt.second.expr, &sel)) { *out = 0; return false; }
                if (sel.Matches(node->Node->labels)) count += pt.first;
            }
        }
        score += (int)count * weight.nodeAffinity;
        // CalculateInterPodAffinityPriority over all nodes, then lookup
        map<string, int> ipa;
        if (!interPodAffinityScores(s, pod, &ipa)) { *out = 0; return false; }
        auto it = ipa.find(node->Name);
        int hostScore = it == ipa.end() ? 0 : it->second;
        score += hostScore * weight.podAffinity;
        *out = score;
        return true;
    };
}

}  // namespace ref
