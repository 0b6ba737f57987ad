/*
 * kbfast_load.cpp — TEST ORACLE: the hoisted restatement's snapshot loader
 * (KBS1 -> World: dictionaries, compiled selectors, pods, nodes, jobs, queues,
 * plugin configuration).  Test infrastructure only (see kbfast.cpp).
 */
#include "kbfast.h"

namespace fast {

/* ---------------------------- loading ----------------------------------- */
static void ensureValInt(World& w) {
    size_t n = w.vals.strs.size();
    size_t o = w.valInt.size();
    w.valInt.resize(n);
    w.valIntOk.resize(n);
    for (size_t i = o; i < n; ++i) w.valIntOk[i] = parseI64(w.vals.strs[i], &w.valInt[i]);
}

// compile a requirement; returns false when labels.NewRequirement would error
static bool compileReq(World& w, const string& key, int op, const vector<string>& values, Req* out) {
    out->key = w.keys.get(key);
    out->op = op;
    out->vals.clear();
    switch (op) {
        case OIn:
        case ONotIn: if (values.empty()) return false; break;
        case OEq: if (values.size() != 1) return false; break;
        case OExists:
        case ODNE: if (!values.empty()) return false; break;
        case OGt:
        case OLt:
            if (values.size() != 1 || !parseI64(values[0], &out->rhs)) return false;
            break;
        default: return false;
    }
    for (auto& v : values) out->vals.push_back(w.vals.get(v));
    return true;
}

struct Loader {
    const kbs::Snapshot& s;
    World& w;
    vector<int32_t> nsr_key, lsr_key, nsr_voff, lsr_voff, nsrv, lsrv, ls_ml, ls_me, lkv_k, lkv_v, pat_sel, pat_topo,
        pat_ns, patns, es, ec, fs, fc;
    vector<uint8_t> nsr_op, lsr_op;
    Loader(const kbs::Snapshot& s_, World& w_) : s(s_), w(w_) {}

    vector<string> strs(const vector<int32_t>& off, const vector<int32_t>& tab, int row) {
        vector<string> v;
        for (int k = off[row]; k < off[row + 1]; ++k) v.push_back(s.s(tab[k]));
        return v;
    }
    bool nsReq(int row, Req* r) { return compileReq(w, s.s(nsr_key[row]), nsr_op[row], strs(nsr_voff, nsrv, row), r); }
    NSTerm nst(int row) {
        NSTerm t;
        for (int k = es[row]; k < es[row] + ec[row]; ++k) {
            Req r;
            if (!nsReq(k, &r)) t.exprErr = true;
            t.expr.push_back(r);
        }
        for (int k = fs[row]; k < fs[row] + fc[row]; ++k) {
            vector<string> vs = strs(nsr_voff, nsrv, k);
            int op = nsr_op[k];
            if ((op != OIn && op != ONotIn) || vs.size() != 1) t.fieldErr = true;
            t.fields.push_back({op, vs.empty() ? string() : vs[0]});
            t.fieldKeys.push_back(s.s(nsr_key[k]));
        }
        return t;
    }
    PATerm pat(int row) {
        PATerm t;
        int sr = pat_sel[row];
        if (sr < 0) t.sel.nothing = true;
        else {
            for (int k = ls_ml[sr]; k < ls_ml[sr + 1]; ++k) {
                Req r;
                if (!compileReq(w, s.s(lkv_k[k]), OEq, {s.s(lkv_v[k])}, &r)) t.selErr = true;
                t.sel.reqs.push_back(r);
            }
            for (int k = ls_me[sr]; k < ls_me[sr + 1]; ++k) {
                Req r;
                int op = lsr_op[k];
                if (op > ODNE || !compileReq(w, s.s(lsr_key[k]), op, strs(lsr_voff, lsrv, k), &r)) t.selErr = true;
                t.sel.reqs.push_back(r);
            }
        }
        for (int k = pat_ns[row]; k < pat_ns[row + 1]; ++k) t.ns.push_back(w.nss.get(s.s(patns[k])));
        string tk = s.s(pat_topo[row]);
        t.key = tk.empty() ? -1 : w.keys.get(tk);
        return t;
    }

    void load() {
        auto V32 = [&](const char* n) { return s.vec<int32_t>(n); };
        // conf
        auto pn = V32("conf_plugin_name"), pt = V32("conf_plugin_tier"), pf = V32("conf_plugin_flags"),
             ap = V32("conf_arg_plugin"), ak = V32("conf_arg_key"), av = V32("conf_arg_val");
        vector<Plugin> opts(pn.size());
        for (size_t i = 0; i < pn.size(); ++i) { opts[i].name = s.s(pn[i]); opts[i].flags = pf[i]; }
        for (size_t i = 0; i < ap.size(); ++i) opts[ap[i]].args[s.s(ak[i])] = s.s(av[i]);
        for (size_t i = 0; i < pn.size(); ++i) {
            if ((size_t)pt[i] >= w.tiers.size()) w.tiers.resize(pt[i] + 1);
            w.tiers[pt[i]].push_back(opts[i]);
        }
        // nodes
        auto nname = V32("n_name");
        size_t N = nname.size();
        auto acpu = s.vec<int64_t>("n_alloc_cpu"), amem = s.vec<int64_t>("n_alloc_mem"),
             agpu = s.vec<int64_t>("n_alloc_gpu"), apods = s.vec<int64_t>("n_alloc_pods");
        auto unsched = s.vec<uint8_t>("n_unsched");
        auto loff = s.offs("n_label_off", N);
        auto lk = V32("nl_key"), lv = V32("nl_val");
        auto toff = s.offs("n_taint_off", N);
        auto tk = V32("nt_key"), tv = V32("nt_val"), te = V32("nt_effect");
        w.nodes.resize(N);
        std::map<string, int> taintIds;
        for (size_t i = 0; i < N; ++i) {
            NodeRec& n = w.nodes[i];
            n.name = s.s(nname[i]);
            for (int k = loff[i]; k < loff[i + 1]; ++k) n.labels.push_back({w.keys.get(s.s(lk[k])), w.vals.get(s.s(lv[k]))});
            std::sort(n.labels.begin(), n.labels.end());
            for (int k = toff[i]; k < toff[i + 1]; ++k) {
                string eff = s.s(te[k]);
                if (eff != "NoSchedule" && eff != "NoExecute") continue;  // predicates.go:1494-1497
                string key = s.s(tk[k]) + '\x01' + s.s(tv[k]) + '\x01' + eff;
                auto it = taintIds.find(key);
                int id;
                if (it == taintIds.end()) {
                    id = (int)w.taintDefs.size();
                    taintIds[key] = id;
                    w.taintDefs.emplace_back(w.keys.get(s.s(tk[k])), w.vals.get(s.s(tv[k])), eff);
                } else id = it->second;
                n.taints.push_back(id);
            }
            n.unsched = !unsched.empty() && unsched[i];
            n.maxTasks = (int)apods[i];
            n.alloc = Res{acpu[i], amem[i], agpu[i]};
            n.idle = n.alloc;
            n.acpu = acpu[i];
            n.amem = amem[i];
        }
        // affinity tables
        nsr_key = V32("nsr_key"); nsr_op = s.vec<uint8_t>("nsr_op"); nsr_voff = s.offs("nsr_val_off", nsr_key.size());
        nsrv = V32("nsrv");
        lsr_key = V32("lsr_key"); lsr_op = s.vec<uint8_t>("lsr_op"); lsr_voff = s.offs("lsr_val_off", lsr_key.size());
        lsrv = V32("lsrv");
        ls_ml = V32("ls_ml_off"); ls_me = V32("ls_me_off"); lkv_k = V32("lkv_key"); lkv_v = V32("lkv_val");
        pat_sel = V32("pat_sel"); pat_topo = V32("pat_topo"); pat_ns = s.offs("pat_ns_off", pat_sel.size());
        patns = V32("patns");
        es = V32("nst_expr_start"); ec = V32("nst_expr_cnt"); fs = V32("nst_field_start"); fc = V32("nst_field_cnt");
        auto a_flags = s.vec<uint8_t>("a_flags");
        auto pst_w = V32("pst_weight"), pst_t = V32("pst_term"), wpat_w = V32("wpat_weight"), wpat_t = V32("wpat_term");
        auto S = [&](const char* n) { return V32(n); };
        auto nareq_s = S("a_nareq_start"), nareq_c = S("a_nareq_cnt"), napref_s = S("a_napref_start"),
             napref_c = S("a_napref_cnt"), pareq_s = S("a_pareq_start"), pareq_c = S("a_pareq_cnt"),
             papref_s = S("a_papref_start"), papref_c = S("a_papref_cnt"), paareq_s = S("a_paareq_start"),
             paareq_c = S("a_paareq_cnt"), paapref_s = S("a_paapref_start"), paapref_c = S("a_paapref_cnt");
        vector<std::shared_ptr<Aff>> affs(a_flags.size());
        for (size_t a = 0; a < a_flags.size(); ++a) {
            auto af = std::make_shared<Aff>();
            af->na = a_flags[a] & KBS_AFF_NA; af->naReq = a_flags[a] & KBS_AFF_NA_REQ;
            af->pa = a_flags[a] & KBS_AFF_PA; af->paa = a_flags[a] & KBS_AFF_PAA;
            for (int k = nareq_s[a]; k < nareq_s[a] + nareq_c[a]; ++k) af->naReqTerms.push_back(nst(k));
            for (int k = napref_s[a]; k < napref_s[a] + napref_c[a]; ++k) af->naPref.push_back({pst_w[k], nst(pst_t[k])});
            for (int k = pareq_s[a]; k < pareq_s[a] + pareq_c[a]; ++k) af->paReq.push_back(pat(k));
            for (int k = paareq_s[a]; k < paareq_s[a] + paareq_c[a]; ++k) af->paaReq.push_back(pat(k));
            for (int k = papref_s[a]; k < papref_s[a] + papref_c[a]; ++k) af->paPref.push_back({wpat_w[k], pat(wpat_t[k])});
            for (int k = paapref_s[a]; k < paapref_s[a] + paapref_c[a]; ++k) af->paaPref.push_back({wpat_w[k], pat(wpat_t[k])});
            affs[a] = af;
        }
        // pods
        auto puid = V32("p_uid");
        size_t P = puid.size();
        auto pname = V32("p_name"), pns = V32("p_ns"), pjob = V32("p_job"), pnode = V32("p_node"),
             ppri = V32("p_priority"), paff = V32("p_aff");
        auto pphase = s.vec<uint8_t>("p_phase"), pdel = s.vec<uint8_t>("p_deleting"), pbf = s.vec<uint8_t>("p_backfill");
        auto pdet = s.vec<uint8_t>("p_detached");  // optional (kbsnap.h)
        auto ppcls = s.vec<int32_t>("p_pclass"), pns_raw = s.vec<int32_t>("p_ns");
        auto pts = s.vec<int64_t>("p_ts");
        auto plo = s.offs("p_label_off", P);
        auto plk = V32("pl_key"), plv = V32("pl_val");
        auto pso = s.offs("p_nsel_off", P);
        auto psk = V32("ps_key"), psv = V32("ps_val");
        auto pco = s.offs("p_ctr_off", P);
        auto ccpu = s.vec<int64_t>("c_cpu"), cmem = s.vec<int64_t>("c_mem"), cgpu = s.vec<int64_t>("c_gpu");
        auto chas = s.vec<uint8_t>("c_has");
        auto cpo = s.offs("c_port_off", ccpu.size());
        auto ptip = V32("pt_ip"), ptpr = V32("pt_proto"), ptpo = V32("pt_port");
        auto pio = s.offs("p_ictr_off", P);
        auto iccpu = s.vec<int64_t>("ic_cpu"), icmem = s.vec<int64_t>("ic_mem"), icgpu = s.vec<int64_t>("ic_gpu");
        auto pto = s.offs("p_tol_off", P);
        auto tlk = V32("tl_key"), tlo = V32("tl_op"), tlv = V32("tl_val"), tle = V32("tl_effect");
        std::unordered_map<string, int> nodeIdx;
        for (size_t i = 0; i < N; ++i) nodeIdx[w.nodes[i].name] = (int)i;
        w.pods.resize(P);
        int defaultNs = -1;
        (void)defaultNs;
        for (size_t i = 0; i < P; ++i) {
            PodRec& p = w.pods[i];
            p.uid = s.s(puid[i]);
            p.name = s.s(pname[i]);
            p.ns = w.nss.get(s.s(pns[i]));
            for (int k = plo[i]; k < plo[i + 1]; ++k) p.labels.push_back({w.keys.get(s.s(plk[k])), w.vals.get(s.s(plv[k]))});
            std::sort(p.labels.begin(), p.labels.end());
            string nn = s.s(pnode[i]);
            if (!nn.empty()) {
                auto it = nodeIdx.find(nn);
                if (it == nodeIdx.end()) throw std::runtime_error("pod " + p.uid + " bound to unknown node " + nn);
                p.nodeRaw = it->second;
            }
            // getTaskStatus (api/helpers.go:35-61)
            int ph = pphase[i];
            bool del = pdel[i];
            if (ph == KBS_RUNNING) p.status = del ? Releasing : Running;
            else if (ph == KBS_PENDING) p.status = del ? Releasing : (nn.empty() ? Pending : Bound);
            else if (ph == KBS_SUCCEEDED) p.status = Succeeded;
            else if (ph == KBS_FAILED) p.status = Failed;
            else p.status = Unknown;
            p.priority = ppri[i];
            p.ts = pts[i];
            p.backfill = pbf[i];
            {
                const string pc = (!ppcls.empty() && ppcls[i] >= 0) ? s.s(ppcls[i]) : string();
                p.critical = s.s(pns_raw[i]) == "kube-system" || pc == "system-cluster-critical" ||
                             pc == "system-node-critical";
            }
            for (int k = pco[i]; k < pco[i + 1]; ++k) {
                p.req += Res{ccpu[k], cmem[k], cgpu[k]};
                p.nzc += (chas[k] & KBS_HAS_CPU) ? ccpu[k] : 100;                 // non_zero.go:43-47
                p.nzm += (chas[k] & KBS_HAS_MEM) ? cmem[k] : 200LL * 1024 * 1024;  // non_zero.go:48-52
                for (int q = cpo[k]; q < cpo[k + 1]; ++q) {
                    string ip = s.s(ptip[q]), pr = s.s(ptpr[q]);
                    if (ip.empty()) ip = "0.0.0.0";
                    if (pr.empty()) pr = "TCP";
                    p.ports.push_back({w.ips.get(ip), w.protos.get(pr), ptpo[q]});
                }
            }
            p.initReq = p.req;
            for (int k = pio[i]; k < pio[i + 1]; ++k) {  // SetMaxResource (resource_info.go:114-128)
                p.initReq.cpu = std::max(p.initReq.cpu, iccpu[k]);
                p.initReq.mem = std::max(p.initReq.mem, icmem[k]);
                p.initReq.gpu = std::max(p.initReq.gpu, icgpu[k]);
            }
            for (int k = pso[i]; k < pso[i + 1]; ++k) p.nsel.push_back({w.keys.get(s.s(psk[k])), w.vals.get(s.s(psv[k]))});
            // tolerations -> tolerated taint ids (toleration.go:37-56)
            for (size_t t = 0; t < w.taintDefs.size(); ++t) {
                const auto& td = w.taintDefs[t];
                bool tol = false;
                for (int k = pto[i]; k < pto[i + 1] && !tol; ++k) {
                    string key = s.s(tlk[k]), op = s.s(tlo[k]), val = s.s(tlv[k]), eff = s.s(tle[k]);
                    if (!eff.empty() && eff != std::get<2>(td)) continue;
                    if (!key.empty() && key != w.keys.strs[std::get<0>(td)]) continue;
                    if (op.empty() || op == "Equal") tol = val == w.vals.strs[std::get<1>(td)];
                    else if (op == "Exists") tol = true;
                }
                if (tol) p.tolTaints.push_back((int)t);
            }
            if (!paff.empty() && paff[i] >= 0) p.aff = affs[paff[i]];
        }
        ensureValInt(w);
        // queues
        auto qn = V32("q_name"), qw = V32("q_weight");
        auto qts = s.vec<int64_t>("q_ts");
        w.queues.resize(qn.size());
        std::map<string, int> qidx;
        for (size_t i = 0; i < qn.size(); ++i) {
            w.queues[i].name = s.s(qn[i]);
            w.queues[i].weight = qw[i];
            w.queues[i].ts = qts.empty() ? 0 : qts[i];
            qidx[w.queues[i].name] = (int)i;
        }
        // jobs: pod-group jobs + shadow jobs, sorted by UID; only jobs whose queue exists
        auto jns = V32("j_ns"), jname = V32("j_name"), jq = V32("j_queue"), jmin = V32("j_min"),
             jpri = V32("j_pg_priority");
        auto jts = s.vec<int64_t>("j_ts");
        struct Src { string uid; int row, pod; };
        vector<Src> srcs;
        for (size_t j = 0; j < jns.size(); ++j) srcs.push_back({s.s(jns[j]) + "/" + s.s(jname[j]), (int)j, -1});
        for (size_t i = 0; i < P; ++i) if (pjob[i] < 0) srcs.push_back({w.pods[i].uid, -1, (int)i});
        std::stable_sort(srcs.begin(), srcs.end(), [](const Src& a, const Src& b) { return a.uid < b.uid; });
        vector<int> rowSlot(jns.size(), -1);
        vector<int> shadowSlot(P, -1);
        for (auto& src : srcs) {
            string qname = src.row >= 0 ? s.s(jq[src.row]) : string("default");
            auto qit = qidx.find(qname);
            JobRec jr;
            jr.uid = src.uid;
            if (src.row >= 0) {
                jr.minAvail = jmin[src.row];
                jr.ts = jts[src.row];
                jr.priority = jpri[src.row];
            } else {
                jr.minAvail = 1;
                jr.ts = 0;
                jr.priority = 0;
            }
            int slot = -1;
            if (qit != qidx.end()) {
                jr.queue = qit->second;
                slot = (int)w.jobs.size();
                w.jobs.push_back(jr);
            }
            if (src.row >= 0) rowSlot[src.row] = slot;
            else shadowSlot[src.pod] = slot;
        }
        for (size_t i = 0; i < P; ++i) {
            int slot = pjob[i] >= 0 ? rowSlot[pjob[i]] : shadowSlot[i];
            w.pods[i].job = slot;
            if (slot >= 0) {
                w.jobs[slot].tasks.push_back((int)i);
                w.pods[i].jobUID = w.jobs[slot].uid;
            }
        }
        for (auto& j : w.jobs) {
            for (int t : j.tasks) {
                j.priority = w.pods[t].priority;  // AddTaskInfo: last task wins (job_info.go:242)
                if (allocSt(w.pods[t].status)) j.cntAlloc++;
                if (w.pods[t].status == AOB) j.cntAOB++;
            }
        }
        // place pods on nodes (cache addTask -> NodeInfo.AddTask; terminated pods skipped)
        bool anyDetached = false;
        for (size_t i = 0; i < P; ++i) {
            PodRec& p = w.pods[i];
            p.curNode = p.nodeRaw;
            // a detached pod (cache deletePod of a group-less pod) keeps its job and NodeName, off the node
            if (!pdet.empty() && pdet[i] && p.nodeRaw >= 0) { p.detached = true; anyDetached = true; continue; }
            if (p.nodeRaw < 0 || p.status == Succeeded || p.status == Failed) continue;
            NodeRec& n = w.nodes[p.nodeRaw];
            if (p.backfill) n.bf += p.req;
            if (p.status == Releasing) { n.rel += p.req; n.idle -= p.req; }
            else if (p.status == Pipelined) n.rel -= p.req;
            else n.idle -= p.req;
            n.used += p.req;
            n.pods++;
            n.nzc += p.nzc;
            n.nzm += p.nzm;
            for (auto& pt : p.ports) if (pt.port > 0) n.used_ports.push_back(pt);
            n.podList.push_back((int)i);
        }
        for (auto& n : w.nodes) if (n.bf.cpu || n.bf.mem || n.bf.gpu) w.anyBackfilled = true;
        for (size_t i = 0; i < P; ++i) if (w.pods[i].hasPodAff() && w.pods[i].curNode >= 0 && !w.pods[i].detached &&
                                             w.pods[i].status != Succeeded && w.pods[i].status != Failed)
            w.affPods.push_back((int)i);
        if (anyDetached)  // the predicate lister's NodeInfo.Filter excludes such a pod at its own node only
            for (auto& p : w.pods)
                if (p.aff && (p.aff->pa || p.aff->paa || !p.aff->paPref.empty() || !p.aff->paaPref.empty()))
                    throw std::runtime_error("detached pods with pod (anti-)affinity in the session: kbref only");
        // plugins (framework.go:33-48: one object per name, last entry's arguments;
        // dispatch loops over tier entries, so an enabled duplicate entry counts twice)
        for (auto& tier : w.tiers)
            for (auto& p : tier) {
                if (p.name == "predicates" && !(p.flags & KBS_DIS_PREDICATE)) w.predOn = true;
                if (p.name == "nodeorder" && !(p.flags & KBS_DIS_NODEORDER)) { w.nodeorderOn = true; w.noMult++; }
                if (p.name == "nodeorder") {
                    w.wLR = w.wBRA = w.wNA = w.wPA = 1;
                    auto get = [&](const char* k, int* dst) {
                        auto it = p.args.find(k);
                        int64_t v;
                        if (it != p.args.end() && !it->second.empty() && parseI64(it->second, &v)) *dst = (int)v;
                    };
                    get("nodeaffinity.weight", &w.wNA);
                    get("podaffinity.weight", &w.wPA);
                    get("leastrequested.weight", &w.wLR);
                    get("balancedresource.weight", &w.wBRA);
                }
                if (p.name == "drf") w.drfOn = true;
                if (p.name == "proportion") w.propOn = true;
                if (p.name == "gang") w.gangOn = true;
                if (p.name == "priority") w.prioOn = true;
            }
        for (auto& n : w.nodes) w.total.add(toF(n.alloc));
    }
};

void load_world(const kbs::Snapshot& s, World& w) {
    Loader L(s, w);
    L.load();
}

}  // namespace fast
