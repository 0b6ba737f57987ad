// kbhip session, part 02: session open (KBS1 decode, dictionary encoding, task classes, upload to HBM)
#include "session.h"

namespace kbhip {

// ---------------------------------------------------------------------------
// encoder
// ---------------------------------------------------------------------------
struct Encoder {
    const kbs::Snapshot& s;
    Session& S;
    Dict keys_all, vals, nss, taint_keys, port_keys, ip_dict, proto_dict;
    std::map<string, int> sel_keys;  // label key -> label column
    vector<Req> reqs;
    vector<Term> terms;
    vector<int32_t> vals_list;
    vector<uint64_t> masks;
    vector<int32_t> nl_off;                       // node labels, CSR: node i owns nl_kv[nl_off[i] .. nl_off[i+1])
    vector<std::pair<int, int>> nl_kv;            // (key id in keys_all, value id)
    vector<std::tuple<string, string, string>> taint_defs;
    vector<std::tuple<int, int, int32_t>> port_defs;  // (ip id, proto id, port)
    std::map<std::tuple<int, int, int32_t>, int> port_ids;
    int tw = 0, pw = 0;

    Encoder(const kbs::Snapshot& s_, Session& S_) : s(s_), S(S_) {}

    vector<int32_t> V32(const char* n) { return s.vec<int32_t>(n); }

    int sel_key(const string& k) {
        auto it = sel_keys.find(k);
        if (it != sel_keys.end()) return it->second;
        int id = (int)sel_keys.size();
        sel_keys[k] = id;
        return id;
    }

};

void fail_unsupported(const string& m) { throw Error(KBHIP_EUNSUPPORTED, m); }

// Host-port ids of pod i: run i of the session's port CSR, compared by value.
struct PortRun {
    const int32_t *b, *e;
    const int32_t* begin() const { return b; }
    const int32_t* end() const { return e; }
    bool empty() const { return b == e; }
    bool operator!=(const PortRun& o) const {
        return (e - b) != (o.e - o.b) || !std::equal(b, e, o.b);
    }
};
struct PortRuns {
    const int32_t* off;
    const vector<int32_t>& ids;
    PortRun operator[](int i) const { return {ids.data() + off[i], ids.data() + off[i + 1]}; }
};

// 32-bit selection keys per class (PopArgs, kbhip_kernels.hip): the score
// of a batched-path class is mult x (w_lr lr + w_bra bra + w_na na) with
// lr, bra in [0, 10] and na between the sums of its negative / positive
// preferred-term weights; it fits when (range + 1) < 2^(31 - index bits).
void class_key_format(const Session& S, const TaskClass& c, const vector<Term>& terms, int N, KeyFormat* kf_out,
                             std::pair<int64_t, int64_t>* range_out) {
    int ibits = 1;  // keys carry global node indices (shards too)
    while (ibits < 30 && ((int64_t)1 << ibits) < (int64_t)N) ++ibits;
    int64_t na_lo = 0, na_hi = 0;
    for (int i = 0; i < c.pref_term_n; ++i) {
        const int64_t w = terms[c.pref_term_off + i].weight;
        (w < 0 ? na_lo : na_hi) += w;
    }
    const int64_t mult = S.conf.score_mult;
    auto rng = [](int64_t a, int64_t b, int64_t* lo, int64_t* hi) {
        *lo += std::min(a, b);
        *hi += std::max(a, b);
    };
    int64_t lo = 0, hi = 0;
    rng(0, 10 * (int64_t)S.conf.w_lr, &lo, &hi);
    rng(0, 10 * (int64_t)S.conf.w_bra, &lo, &hi);
    rng(na_lo * S.conf.w_na, na_hi * S.conf.w_na, &lo, &hi);
    const int64_t slo = std::min(lo * mult, hi * mult), shi = std::max(lo * mult, hi * mult);
    *range_out = {slo, shi};
    {  // nodeorder.go:287-313 sums in Go's 64-bit int; the kernels' score is int32 (kbhip_eval.h
       // node_score): sessions whose score range (with the inter-pod term) leaves int32 are refused
        int64_t flo = lo, fhi = hi;
        rng(0, 10 * (int64_t)S.conf.w_pa, &flo, &fhi);
        const int64_t a = flo * mult, b = fhi * mult;
        if (std::min(a, b) < INT32_MIN || std::max(a, b) > INT32_MAX)
            fail_unsupported("nodeorder score range leaves int32 (weights x terms x tiers)");
    }
    KeyFormat& kf = *kf_out;
    kf = KeyFormat{};
    kf.use32 = ibits <= 25 && shi - slo + 1 < ((int64_t)1 << (31 - ibits)) && slo >= INT32_MIN && shi <= INT32_MAX;
    kf.ent32 = kf.use32 && ibits <= 24 && shi - slo + 1 < ((int64_t)1 << (26 - ibits));
    kf.base = (int32_t)slo;
    kf.shift = ibits + 1;
    kf.idxmax = (int32_t)(((int64_t)1 << ibits) - 1);
}

// FNV-1a digests of the snapshot parts kbhip_session_carry_snapshot's fast
// path takes over unchanged: the conf sections, and every node's labels and
// taints (as strings, in node order).
static uint64_t fnv(uint64_t h, const void* p, size_t n) {
    const unsigned char* b = (const unsigned char*)p;
    for (size_t i = 0; i < n; ++i) { h ^= b[i]; h *= 1099511628211ULL; }
    return h;
}
static uint64_t fnv_str(uint64_t h, const char* z) { return fnv(h, z, std::strlen(z) + 1); }
uint64_t conf_digest(const kbs::Snapshot& s) {
    uint64_t h = 1469598103934665603ULL;
    for (const char* n : {"conf_plugin_name", "conf_arg_key", "conf_arg_val", "conf_actions"})
        for (int32_t o : s.vec<int32_t>(n)) h = fnv_str(h, s.str(o));
    for (const char* n : {"conf_plugin_tier", "conf_plugin_flags", "conf_arg_plugin"}) {
        auto v = s.vec<int32_t>(n);
        h = fnv(h, v.data(), v.size() * sizeof(int32_t));
        h = fnv(h, "|", 1);
    }
    return h;
}
// (over kDigestParts fixed node ranges hashed in parallel, their digests then
// hashed in range order: the value depends on the snapshot only)
uint64_t node_spec_digest(const kbs::Snapshot& s) {
    constexpr int kDigestParts = 16;
    const size_t N = s.rows("n_name");
    auto loff = s.offs("n_label_off", N), toff = s.offs("n_taint_off", N);
    auto lk = s.span<int32_t>("nl_key"), lv = s.span<int32_t>("nl_val");
    auto tk = s.span<int32_t>("nt_key"), tv = s.span<int32_t>("nt_val"), te = s.span<int32_t>("nt_effect");
    uint64_t part[kDigestParts];
    auto range = [&](int r) {
        uint64_t h = 1469598103934665603ULL;
        for (size_t i = N * r / kDigestParts; i < N * (r + 1) / kDigestParts; ++i) {
            for (int k = loff[i]; k < loff[i + 1]; ++k) { h = fnv_str(h, s.str(lk[k])); h = fnv_str(h, s.str(lv[k])); }
            h = fnv(h, "|", 1);
            for (int k = toff[i]; k < toff[i + 1]; ++k) {
                h = fnv_str(h, s.str(tk[k]));
                h = fnv_str(h, s.str(tv[k]));
                h = fnv_str(h, s.str(te[k]));
            }
            h = fnv(h, "#", 1);
        }
        part[r] = h;
    };
    const int nth = N < (1u << 13) ? 1 : std::min(kDigestParts, host_threads());
    vector<std::thread> th;
    for (int t = 1; t < nth; ++t)
        th.emplace_back([&, t] { for (int r = t; r < kDigestParts; r += nth) range(r); });
    for (int r = 0; r < kDigestParts; r += nth) range(r);
    for (auto& x : th) x.join();
    return fnv(1469598103934665603ULL, part, sizeof(part));
}

void open_session(Session& S, const kbs::Snapshot& s, int device, bool encode_only, int rank,
                         int world) {
    if (world < 1 || world > 16 || rank < 0 || rank >= world) throw Error(KBHIP_EINVAL, "bad shard rank / world (1..16)");
    S.rank = rank;
    S.world = world;
    S.encode_only = encode_only;
    auto t0 = std::chrono::steady_clock::now();
    // KBHIP_OPEN_PROFILE=1: per-phase host times of the session open on stderr (diagnostic)
    static const bool prof = std::getenv("KBHIP_OPEN_PROFILE") != nullptr;
    auto tp = t0;
    auto mark = [&](const char* what) {
        if (!prof) return;
        auto now = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[open] %-10s %8.2f ms\n", what, std::chrono::duration<double>(now - tp).count() * 1e3);
        tp = now;
    };
    Encoder E(s, S);
    auto V32 = [&](const char* n) { return s.vec<int32_t>(n); };
    // ---------------- conf (framework.go:29-51) ----------------
    {
        auto pn = V32("conf_plugin_name"), pt = V32("conf_plugin_tier"), pf = V32("conf_plugin_flags"),
             ap = V32("conf_arg_plugin"), ak = V32("conf_arg_key"), av = V32("conf_arg_val");
        vector<Plugin> opts(pn.size());
        for (size_t i = 0; i < pn.size(); ++i) { opts[i].name = s.s(pn[i]); opts[i].flags = pf[i]; }
        for (size_t i = 0; i < ap.size(); ++i) {
            if (ap[i] < 0 || (size_t)ap[i] >= opts.size()) throw Error(KBHIP_EINVAL, "bad conf_arg_plugin");
            opts[ap[i]].args[s.s(ak[i])] = s.s(av[i]);
        }
        for (size_t i = 0; i < pn.size(); ++i) {
            if (pt[i] < 0 || pt[i] > 64) throw Error(KBHIP_EINVAL, "bad conf_plugin_tier");
            if ((size_t)pt[i] >= S.tiers.size()) S.tiers.resize(pt[i] + 1);
            S.tiers[pt[i]].push_back(opts[i]);
        }
        S.conf.w_lr = S.conf.w_bra = S.conf.w_na = S.conf.w_pa = 1;
        for (auto& tier : S.tiers)
            for (auto& p : tier) {
                if (p.name == "predicates" && !(p.flags & KBS_DIS_PREDICATE)) S.conf.pred_on = 1;
                if (p.name == "nodeorder" && !(p.flags & KBS_DIS_NODEORDER)) S.conf.score_mult++;
                if (p.name == "nodeorder") {  // the last entry's arguments win (framework.go:38-39)
                    int w[4] = {1, 1, 1, 1};
                    const char* names[4] = {"leastrequested.weight", "balancedresource.weight",
                                            "nodeaffinity.weight", "podaffinity.weight"};
                    for (int k = 0; k < 4; ++k) {  // nodeorder.go:177-249
                        auto it = p.args.find(names[k]);
                        int64_t v;
                        if (it != p.args.end() && !it->second.empty() && parse_int64(it->second, &v)) {
                            // Go's int is 64-bit; the device score is int32 (checked per class below)
                            if (v > INT32_MAX || v < INT32_MIN) fail_unsupported("nodeorder weight outside int32: " + it->second);
                            w[k] = (int)v;
                        }
                    }
                    S.conf.w_lr = w[0]; S.conf.w_bra = w[1]; S.conf.w_na = w[2]; S.conf.w_pa = w[3];
                }
                if (p.name == "drf") S.drf_on = true;
                if (p.name == "proportion") S.prop_on = true;
                if (p.name == "gang" && !(p.flags & KBS_DIS_JOBREADY)) S.gang_ready = true;
                if (p.name == "gang") S.gang_close = true;
            }
    }
    mark("conf");
    // ---------------- nodes ----------------
    auto nname = V32("n_name");
    const int N = (int)nname.size();
    const int npad = ((N + kBlock - 1) / kBlock) * kBlock;
    auto acpu = s.vec<int64_t>("n_alloc_cpu"), amem = s.vec<int64_t>("n_alloc_mem"), agpu = s.vec<int64_t>("n_alloc_gpu"),
         apods = s.vec<int64_t>("n_alloc_pods");
    if ((int)acpu.size() != N || (int)amem.size() != N || (int)agpu.size() != N || (int)apods.size() != N)
        throw Error(KBHIP_EINVAL, "node columns length mismatch");
    auto unsched = s.vec<uint8_t>("n_unsched");
    auto loff = s.offs("n_label_off", N);
    auto lk = V32("nl_key"), lv = V32("nl_val");
    auto toff = s.offs("n_taint_off", N);
    auto tk = V32("nt_key"), tv = V32("nt_val"), te = V32("nt_effect");
    // Name -> node: binary search when the names are strictly ascending (the
    // canonical snapshot order, kbsnap.h), else a map of views into the string table.
    bool names_sorted = true;
    for (int i = 1; i < N && names_sorted; ++i) names_sorted = std::strcmp(s.str(nname[i - 1]), s.str(nname[i])) < 0;
    std::unordered_map<std::string_view, int> node_idx;
    if (!names_sorted) {
        node_idx.reserve((size_t)N * 2);
        for (int i = 0; i < N; ++i) node_idx.emplace(std::string_view(s.str(nname[i])), i);
        if ((int)node_idx.size() != N) throw Error(KBHIP_EINVAL, "duplicate node names");
    }
    auto find_node = [&](std::string_view v) -> int {
        if (!names_sorted) {
            auto it = node_idx.find(v);
            return it == node_idx.end() ? -1 : it->second;
        }
        int lo = 0, hi = N;
        while (lo < hi) {
            const int m = (lo + hi) / 2;
            if (std::string_view(s.str(nname[m])) < v) lo = m + 1;
            else hi = m;
        }
        return lo < N && std::string_view(s.str(nname[lo])) == v ? lo : -1;
    };
    E.nl_off.assign(N + 1, 0);
    E.nl_kv.clear();
    E.nl_kv.reserve(lk.size());
    std::unordered_map<int32_t, int> key_by_off, val_by_off;  // strtab offset -> dictionary id
    vector<vector<int>> node_taints(N);
    std::map<std::tuple<string, string, string>, int> taint_ids;
    std::unordered_map<int32_t, int> node_by_off;  // strtab offset of the name -> node (fast path)
    node_by_off.reserve((size_t)N * 2);
    for (int i = 0; i < N; ++i) {
        node_by_off.emplace(nname[i], i);
        for (int k = loff[i]; k < loff[i + 1]; ++k) {
            auto ki = key_by_off.find(lk[k]);
            if (ki == key_by_off.end()) ki = key_by_off.emplace(lk[k], E.keys_all.get(s.s(lk[k]))).first;
            auto vi = val_by_off.find(lv[k]);
            if (vi == val_by_off.end()) vi = val_by_off.emplace(lv[k], E.vals.get(s.s(lv[k]))).first;
            E.nl_kv.push_back({ki->second, vi->second});
        }
        E.nl_off[i + 1] = (int32_t)E.nl_kv.size();
        for (int k = toff[i]; k < toff[i + 1]; ++k) {
            string eff = s.s(te[k]);
            if (eff != "NoSchedule" && eff != "NoExecute") continue;  // predicates.go:1494-1497
            auto key = std::make_tuple(s.s(tk[k]), s.s(tv[k]), eff);
            auto it = taint_ids.find(key);
            int id;
            if (it == taint_ids.end()) { id = (int)E.taint_defs.size(); taint_ids[key] = id; E.taint_defs.push_back(key); }
            else id = it->second;
            node_taints[i].push_back(id);
        }
    }
    // host-side node state (NewNodeInfo + AddTask replay, node_info.go:62-145)
    vector<R3> idle(N), rel(N), bf(N);
    vector<int64_t> nzc(N, 0), nzm(N, 0);
    vector<int32_t> podcnt(N, 0);
    vector<vector<int>> node_ports(N);
    S.used.assign(N, R3{});
    for (int i = 0; i < N; ++i) idle[i] = R3{acpu[i], amem[i], agpu[i]};

    mark("nodes");
    // ---------------- pods ----------------
    // per-pod columns are read in place (1M-row columns: no copies)
    auto S32 = [&](const char* n) { return s.span<int32_t>(n); };
    auto puid = S32("p_uid");
    const int P = (int)puid.size();
    auto pns = S32("p_ns"), pjob = S32("p_job"), pnode = S32("p_node"), ppri = S32("p_priority"), paff = S32("p_aff");
    auto pphase = s.span<uint8_t>("p_phase"), pdel = s.span<uint8_t>("p_deleting"), pbf = s.span<uint8_t>("p_backfill");
    auto pts = s.span<int64_t>("p_ts");
    auto ppc = s.span<int32_t>("p_pclass");  // optional: Spec.PriorityClassName
    auto pdet = s.span<uint8_t>("p_detached");  // optional: group-less pods the cache took off their node
    if ((int)pns.size() != P || (int)pjob.size() != P || (int)pnode.size() != P || (int)ppri.size() != P ||
        (int)pphase.size() != P || (int)pts.size() != P)
        throw Error(KBHIP_EINVAL, "pod columns length mismatch");
    auto pco = s.offs("p_ctr_off", P);
    auto ccpu = s.span<int64_t>("c_cpu"), cmem = s.span<int64_t>("c_mem"), cgpu = s.span<int64_t>("c_gpu");
    auto chas = s.span<uint8_t>("c_has");
    auto cpo = s.offs("c_port_off", ccpu.size());
    auto ptip = V32("pt_ip"), ptpr = V32("pt_proto"), ptpo = V32("pt_port");
    auto pio = s.offs("p_ictr_off", P);
    auto iccpu = s.span<int64_t>("ic_cpu"), icmem = s.span<int64_t>("ic_mem"), icgpu = s.span<int64_t>("ic_gpu");
    auto pso = s.offs("p_nsel_off", P);
    auto psk = S32("ps_key"), psv = S32("ps_val");
    auto pto = s.offs("p_tol_off", P);
    auto tlk = S32("tl_key"), tlo = S32("tl_op"), tlv = S32("tl_val"), tle = S32("tl_effect");
    auto a_flags = s.vec<uint8_t>("a_flags");
    auto acnt = [&](const char* n) { return V32(n); };
    auto pareq_c = acnt("a_pareq_cnt"), papref_c = acnt("a_papref_cnt"), paareq_c = acnt("a_paareq_cnt"),
         paapref_c = acnt("a_paapref_cnt");
    (void)pareq_c; (void)papref_c; (void)paareq_c; (void)paapref_c;

    spare_pods().take_keep(S.pods);  // old pods are reset in pass A below (in parallel)
    S.pods.resize(P);
    vector<int32_t> uid_rank_of;  // UID ranks when the pods are not in UID order
    {  // UID ranks: the canonical order (kbsnap.h) makes them the index; sort otherwise
        // strictly ascending? (checked in kThreads chunks: 1M string compares at C4)
        const int kThreads = host_threads();
        const int per = (P + kThreads - 1) / kThreads;
        std::atomic<bool> sorted{true};
        auto check = [&](int lo, int hi) {
            for (int i = std::max(lo, 1); i < hi; ++i)
                if (std::strcmp(s.str(puid[i - 1]), s.str(puid[i])) >= 0) { sorted = false; return; }
        };
        if (P < (1 << 16)) {
            check(0, P);
        } else {
            vector<std::thread> th;
            for (int t = 1; t < kThreads; ++t) th.emplace_back(check, t * per, std::min(P, (t + 1) * per));
            check(0, std::min(P, per));
            for (auto& x : th) x.join();
        }
        if (!sorted) {  // ranks assigned after pass A; sorted: rank = index, set there
            vector<int> ord(P);
            for (int i = 0; i < P; ++i) ord[i] = i;
            std::sort(ord.begin(), ord.end(),
                      [&](int a, int b) { return std::strcmp(s.str(puid[a]), s.str(puid[b])) < 0; });
            uid_rank_of.resize(P);
            for (int r = 0; r < P; ++r) uid_rank_of[ord[r]] = r;
        }
    }
    mark("pods:init");
    // host ports per pod: CSR built in pod order (S.pod_port_off / S.pod_port_ids)
    S.pod_port_off.assign(P + 1, 0);
    S.pod_port_ids.clear();
    const PortRuns pod_ports{S.pod_port_off.data(), S.pod_port_ids};
    // Pass A (parallel over pod ranges): the per-pod fields that need no
    // dictionary -- status, priority, requests, nonzero requests, node.
    auto pod_fields = [&](int lo, int hi) {
        for (int i = lo; i < hi; ++i) {
            HPod& p = S.pods[i];
            p = HPod{};
            p.uid_rank = uid_rank_of.empty() ? i : uid_rank_of[i];
            const bool has_node = pnode[i] >= 0 && s.str(pnode[i])[0] != '\0';
            int ph = pphase[i];
            bool del = !pdel.empty() && pdel[i];
            if (ph == KBS_RUNNING) p.status = del ? Releasing : Running;            // api/helpers.go:35-61
            else if (ph == KBS_PENDING) p.status = del ? Releasing : (!has_node ? Pending : Bound);
            else if (ph == KBS_SUCCEEDED) p.status = Succeeded;
            else if (ph == KBS_FAILED) p.status = Failed;
            else p.status = Unknown;
            p.priority = ppri[i];
            p.ts = pts[i];
            {
                const char* pc = (!ppc.empty() && ppc[i] >= 0) ? s.str(ppc[i]) : "";
                p.critical = std::strcmp(s.str(pns[i]), "kube-system") == 0 ||
                             std::strcmp(pc, "system-cluster-critical") == 0 || std::strcmp(pc, "system-node-critical") == 0;
            }
            p.backfill = !pbf.empty() && pbf[i];
            p.groupless = pjob[i] < 0;
            p.detached = has_node && !pdet.empty() && pdet[i];
            for (int k = pco[i]; k < pco[i + 1]; ++k) {  // pod_info.go:51-71, non_zero.go:37-52
                p.req.c += ccpu[k]; p.req.m += cmem[k]; p.req.g += cgpu[k];
                p.nzc += (chas[k] & KBS_HAS_CPU) ? ccpu[k] : 100;
                p.nzm += (chas[k] & KBS_HAS_MEM) ? cmem[k] : 200LL * 1024 * 1024;
            }
            p.ireq = p.req;
            for (int k = pio[i]; k < pio[i + 1]; ++k) {
                p.ireq.c = std::max(p.ireq.c, iccpu[k]);
                p.ireq.m = std::max(p.ireq.m, icmem[k]);
                p.ireq.g = std::max(p.ireq.g, icgpu[k]);
            }
            if (has_node) {
                auto ot = node_by_off.find(pnode[i]);
                if (ot != node_by_off.end()) {
                    p.node = ot->second;
                } else {
                    const int n = find_node(std::string_view(s.str(pnode[i])));
                    if (n < 0)
                        throw Error(KBHIP_EINVAL, "pod " + s.s(puid[i]) + " is bound to node " + s.s(pnode[i]) +
                                                      " which is not in the snapshot");
                    p.node = n;
                }
            }
        }
    };
    {
        const int kThreads = host_threads();
        if (P < (1 << 16)) {
            pod_fields(0, P);
        } else {  // the first failing range's error is rethrown (its lowest pod)
            const int per = (P + kThreads - 1) / kThreads;
            vector<std::exception_ptr> err(kThreads);
            auto run = [&](int t) {
                try { pod_fields(t * per, std::min(P, (t + 1) * per)); } catch (...) { err[t] = std::current_exception(); }
            };
            vector<std::thread> th;
            for (int t = 1; t < kThreads; ++t) th.emplace_back(run, t);
            run(0);
            for (auto& x : th) x.join();
            for (auto& e : err) if (e) std::rethrow_exception(e);
        }
    }
    mark("pods:A");
    // ---------------- queues & jobs ----------------
    auto qn = V32("q_name"), qw = V32("q_weight");
    auto qts = s.vec<int64_t>("q_ts");
    std::map<string, int> qidx;
    S.queues.resize(qn.size());
    for (size_t i = 0; i < qn.size(); ++i) {
        S.queues[i].name = s.s(qn[i]);
        S.queues[i].weight = qw[i];
        S.queues[i].ts = qts.empty() ? 0 : qts[i];
        qidx[S.queues[i].name] = (int)i;
    }
    {
        int r = 0;  // equal names share a rank (the map holds each name once, in string order)
        std::map<string, int> rank;
        for (auto& kv : qidx) rank[kv.first] = r++;
        for (auto& q : S.queues) q.rank = rank[q.name];
    }
    auto jns = V32("j_ns"), jname = V32("j_name"), jq = V32("j_queue"), jmin = V32("j_min"), jpri = V32("j_pg_priority");
    auto jts = s.vec<int64_t>("j_ts");
    // Job UIDs: "namespace/name" of a PodGroup, the pod UID of a shadow one
    // (cache/util.go:42-60); compared as those strings without building them.
    struct Src {
        const char* a;  // namespace, or the pod UID
        const char* b;  // PodGroup name (after '/'), or nullptr
        int row, pod;
    };
    auto src_less = [](const Src& x, const Src& y) {
        const char *p = x.a, *q = y.a;
        int sp = 0, sq = 0;  // part: 0 = a, 1 = '/', 2 = b, 3 = end
        for (;;) {
            if (sp == 0 && !*p) { sp = x.b ? 1 : 3; }
            if (sq == 0 && !*q) { sq = y.b ? 1 : 3; }
            if (sp == 2 && !*p) sp = 3;
            if (sq == 2 && !*q) sq = 3;
            const int cp = sp == 3 ? -1 : sp == 1 ? '/' : (unsigned char)*p;
            const int cq = sq == 3 ? -1 : sq == 1 ? '/' : (unsigned char)*q;
            if (cp != cq) return cp < cq;
            if (cp < 0) return false;
            if (sp == 1) { sp = 2; p = x.b; } else ++p;
            if (sq == 1) { sq = 2; q = y.b; } else ++q;
        }
    };
    vector<Src> srcs;
    srcs.reserve(jns.size() + 64);
    for (size_t j = 0; j < jns.size(); ++j) srcs.push_back({s.str(jns[j]), s.str(jname[j]), (int)j, -1});
    for (int i = 0; i < P; ++i) {
        if (pjob[i] >= (int)jns.size()) throw Error(KBHIP_EINVAL, "pod job index out of range");
        if (pjob[i] < 0) srcs.push_back({s.str(puid[i]), nullptr, -1, i});  // shadow PodGroup
    }
    const int jth = srcs.size() < (1u << 14) ? 1 : host_threads();
    auto par_j = [&](auto&& fn) {
        vector<std::thread> th;
        for (int t = 1; t < jth; ++t) th.emplace_back(fn, t);
        fn(0);
        for (auto& x : th) x.join();
    };
    {
        const size_t ns = srcs.size();
        std::atomic<bool> sorted{true};
        par_j([&](int t) {  // UID order checked by ranges
            for (size_t k = std::max<size_t>(1, ns * t / jth); k < ns * (t + 1) / jth; ++k)
                if (src_less(srcs[k], srcs[k - 1])) { sorted = false; return; }
        });
        if (!sorted) std::stable_sort(srcs.begin(), srcs.end(), src_less);
    }
    vector<int> row_slot(jns.size(), -1), shadow_slot(P, -1);
    std::unordered_map<int32_t, int> q_by_off;  // strtab offset of a job's queue name -> queue (-1: none)
    const auto default_q = qidx.find("default");
    vector<int32_t> uid_src;  // job slot -> its source (the UID strings are built after, in parallel)
    spare_jobs().take_keep(S.jobs);  // a predecessor's records: reset below, their task lists' buffers kept
    const size_t reuse = S.jobs.size();
    size_t nslot = 0;
    S.jobs.reserve(srcs.size());
    uid_src.reserve(srcs.size());
    for (size_t si = 0; si < srcs.size(); ++si) {
        const Src& src = srcs[si];
        std::map<string, int>::const_iterator qit;
        int qslot = -1;
        if (src.row >= 0) {
            auto qo = q_by_off.find(jq[src.row]);
            if (qo == q_by_off.end()) {
                qit = qidx.find(s.s(jq[src.row]));
                qo = q_by_off.emplace(jq[src.row], qit == qidx.end() ? -1 : qit->second).first;
            }
            qslot = qo->second;
        } else {
            qslot = default_q == qidx.end() ? -1 : default_q->second;
        }
        int slot = -1;
        if (qslot >= 0) {  // Snapshot drops jobs whose queue does not exist (cache.go:556-560)
            HJob j;
            j.queue = qslot;
            j.min_avail = src.row >= 0 ? jmin[src.row] : 1;
            j.ts = src.row >= 0 ? jts[src.row] : 0;
            j.priority = j.pg_priority = src.row >= 0 ? jpri[src.row] : 0;
            j.shadow = src.row < 0;
            slot = (int)nslot++;
            if ((size_t)slot < reuse) {  // keep the old record's task-list buffers (emptied)
                HJob& d = S.jobs[slot];
                j.tasks.swap(d.tasks);
                j.pending.swap(d.pending);
                j.tasks.clear();
                j.pending.clear();
                d = std::move(j);
            } else {
                S.jobs.push_back(std::move(j));
            }
            uid_src.push_back((int32_t)si);
        }
        if (src.row >= 0) row_slot[src.row] = slot;
        else shadow_slot[src.pod] = slot;
    }
    S.jobs.resize(nslot);
    {
        const size_t nj = uid_src.size();
        spare_uids().take_keep(S.job_uid);  // assigned in place: the strings' buffers are reused
        S.job_uid.resize(nj);
        par_j([&](int t) {
            for (size_t k = nj * t / jth; k < nj * (t + 1) / jth; ++k) {
                const Src& src = srcs[uid_src[k]];
                string& u = S.job_uid[k];
                u.assign(src.a);
                if (src.b) { u += '/'; u += src.b; }
            }
        });
    }
    mark("jobs:slots");
    // Pass B: namespace and host-port dictionaries (ids in first-seen pod order,
    // serial), job slots and counts, the affinity model's pod view (parallel
    // over pod ranges), node accumulation (parallel over node ranges, each
    // node's pods in pod order), job task lists (parallel over job ranges).
    // Integer sums only: the result does not depend on the split.
    const int bth = P < (1 << 16) ? 1 : host_threads();
    auto par_b = [&](auto&& fn) {
        vector<std::thread> th;
        for (int t = 1; t < bth; ++t) th.emplace_back(fn, t);
        fn(0);
        for (auto& x : th) x.join();
    };
    vector<int32_t> ntask(S.jobs.size(), 0), last_pod(S.jobs.size(), -1);
    // per pod (every element written in the first parallel pass: no serial fill)
    std::unique_ptr<int32_t[]> slot_of(new int32_t[P]), onode(new int32_t[P]);
    vector<AffPod> ap(P);  // the pod (anti-)affinity model's view of each pod
    {  // namespaces: each range's run heads, ids assigned in pod order, then filled in
        vector<vector<int32_t>> heads(bth);
        par_b([&](int t) {
            const int lo = (int)((int64_t)P * t / bth), hi = (int)((int64_t)P * (t + 1) / bth);
            int32_t last = -1;
            for (int i = lo; i < hi; ++i)
                if (i == lo || pns[i] != last) { last = pns[i]; heads[t].push_back(last); }
        });
        std::unordered_map<int32_t, int> ns_by_off;  // strtab offset -> namespace id
        for (auto& h : heads)
            for (int32_t off : h)
                if (!ns_by_off.count(off)) ns_by_off.emplace(off, E.nss.get(s.s(off)));
        par_b([&](int t) {
            const int lo = (int)((int64_t)P * t / bth), hi = (int)((int64_t)P * (t + 1) / bth);
            int32_t last_off = -1;
            int last_ns = -1;
            for (int i = lo; i < hi; ++i) {
                HPod& p = S.pods[i];
                if (pns[i] != last_off) { last_off = pns[i]; last_ns = ns_by_off.find(last_off)->second; }
                p.ns = last_ns;
                const int slot = pjob[i] >= 0 ? row_slot[pjob[i]] : shadow_slot[i];
                p.job = slot;
                slot_of[i] = slot;
                if (slot >= 0) {
                    HJob& j = S.jobs[slot];
                    __atomic_fetch_add(&ntask[slot], 1, __ATOMIC_RELAXED);
                    if (allocated_status(p.status)) __atomic_fetch_add(&j.cnt_alloc, 1, __ATOMIC_RELAXED);
                    if (p.status == AOB) __atomic_fetch_add(&j.cnt_aob, 1, __ATOMIC_RELAXED);
                    int32_t cur = __atomic_load_n(&last_pod[slot], __ATOMIC_RELAXED);
                    while (cur < i && !__atomic_compare_exchange_n(&last_pod[slot], &cur, i, true, __ATOMIC_RELAXED,
                                                                   __ATOMIC_RELAXED)) {
                    }
                }
                AffPod& a = ap[i];
                a.ns = p.ns;
                a.status = p.status;
                a.session_job = slot >= 0;
                const bool on_node = on_node_of(p);
                a.node = on_node ? p.node : -1;
                a.target = a.session_job && allocated_status(p.status) && on_node;
                a.pending = a.session_job && p.status == Pending;
                onode[i] = a.node;
            }
        });
        // JobInfo.AddTaskInfo: the last task's priority (job_info.go:242)
        for (size_t j = 0; j < S.jobs.size(); ++j)
            if (last_pod[j] >= 0) S.jobs[j].priority = S.pods[last_pod[j]].priority;
    }
    // host ports per pod (HostPortInfo.Add ignores port <= 0): dictionary ids in pod order
    bool any_ports = false;
    for (size_t q = 0; q < ptpo.size() && !any_ports; ++q) any_ports = ptpo[q] > 0;
    if (any_ports) {
        for (int i = 0; i < P; ++i) {
            S.pod_port_off[i] = (int32_t)S.pod_port_ids.size();
            for (int k = pco[i]; k < pco[i + 1]; ++k) {
                for (int q = cpo[k]; q < cpo[k + 1]; ++q) {
                    if (ptpo[q] <= 0) continue;
                    string ip = s.s(ptip[q]), pr = s.s(ptpr[q]);
                    if (ip.empty()) ip = "0.0.0.0";
                    if (pr.empty()) pr = "TCP";
                    auto key = std::make_tuple(E.ip_dict.get(ip), E.proto_dict.get(pr), (int32_t)ptpo[q]);
                    auto it = E.port_ids.find(key);
                    int id;
                    if (it == E.port_ids.end()) { id = (int)E.port_defs.size(); E.port_ids[key] = id; E.port_defs.push_back(key); }
                    else id = it->second;
                    S.pod_port_ids.push_back(id);
                }
            }
        }
    }
    S.pod_port_off[P] = (int32_t)S.pod_port_ids.size();
    // cache addTask -> NodeInfo.AddTask, per node in pod order
    par_b([&](int t) {
        const int nlo = (int)((int64_t)N * t / bth), nhi = (int)((int64_t)N * (t + 1) / bth);
        for (int i = 0; i < P; ++i) {
            const int n = onode[i];
            if (n < nlo || n >= nhi) continue;
            const HPod& p = S.pods[i];
            if (p.backfill) { bf[n].c += p.req.c; bf[n].m += p.req.m; bf[n].g += p.req.g; }
            if (p.status == Releasing) { rel[n].c += p.req.c; rel[n].m += p.req.m; rel[n].g += p.req.g; }
            idle[n].c -= p.req.c; idle[n].m -= p.req.m; idle[n].g -= p.req.g;
            S.used[n].c += p.req.c; S.used[n].m += p.req.m; S.used[n].g += p.req.g;
            podcnt[n]++;
            nzc[n] += p.nzc;
            nzm[n] += p.nzm;
            for (int k = S.pod_port_off[i]; k < S.pod_port_off[i + 1]; ++k) node_ports[n].push_back(S.pod_port_ids[k]);
        }
    });
    for (int i = 0; i < N; ++i) if (bf[i].c || bf[i].m || bf[i].g) S.any_bf = 1;
    S.h_alloc.resize(N);
    for (int i = 0; i < N; ++i) S.h_alloc[i] = R3{acpu[i], amem[i], agpu[i]};

    mark("pods:B");
    {  // each job's tasks in pod order
        const int nj = (int)S.jobs.size();
        par_b([&](int t) {
            const int jlo = (int)((int64_t)nj * t / bth), jhi = (int)((int64_t)nj * (t + 1) / bth);
            for (int j = jlo; j < jhi; ++j) S.jobs[j].tasks.reserve(ntask[j]);
            for (int i = 0; i < P; ++i) {
                const int sl = slot_of[i];
                if (sl < jlo || sl >= jhi) continue;
                HJob& j = S.jobs[sl];
                j.tasks.push_back(i);
                const HPod& p = S.pods[i];
                if (p.status == Pending && !(p.req.c < kMinCPU && p.req.m < kMinMem && p.req.g < kMinGPU))
                    j.maybe_pending = true;
            }
        });
    }

    mark("jobs");
    // ---------------- pod (anti-)affinity model (kbhip_affinity.h) ----------------
    S.aff.reset(new AffinityModel());
    AffinityModel& aff = *S.aff;
    vector<int> row_canon;  // canonical affinity row of every row (kbhip_affinity.h)
    {  // ap: filled in pass B
        try {
            row_canon = canon_aff_rows(s);
            aff.build(s, N, npad, ap, E.nss.strs, S.conf.pred_on != 0, S.conf.score_mult > 0 && S.conf.w_pa != 0,
                      row_canon);
        } catch (const std::invalid_argument& e) {
            fail_unsupported(e.what());
        }
        if (aff.active)  // the predicate lister's NodeInfo.Filter leaves such a pod out at its own node only
            for (int i = 0; i < P; ++i)
                if (S.pods[i].detached) fail_unsupported("detached pods (p_detached) in a session with pod (anti-)affinity");
    }
    vector<int32_t> aff_items;
    // domains per topology space (placement 7's per-domain candidates, dedup_space)
    vector<int> space_ndom(aff.active ? aff.n_spaces : 0, 0);
    for (int sp = 0; sp < (int)space_ndom.size(); ++sp)
        for (int n = 0; n < N; ++n) space_ndom[sp] = std::max(space_ndom[sp], aff.dom[(size_t)sp * npad + n] + 1);

    mark("affinity");
    // ---------------- task classes for pending tasks ----------------
    // label columns: keys referenced by selectors / node affinity of pending tasks
    auto es = V32("nst_expr_start"), ec = V32("nst_expr_cnt"), fs = V32("nst_field_start"), fc = V32("nst_field_cnt");
    auto nsr_key = V32("nsr_key");
    auto nsr_op = s.vec<uint8_t>("nsr_op");
    auto nsr_voff = s.offs("nsr_val_off", nsr_key.size());
    auto nsrv = V32("nsrv");
    auto pst_w = V32("pst_weight"), pst_t = V32("pst_term");
    auto nareq_s = acnt("a_nareq_start"), nareq_c = acnt("a_nareq_cnt"), napref_s = acnt("a_napref_start"),
         napref_c = acnt("a_napref_cnt");
    auto nsr_vals = [&](int row) {
        vector<string> v;
        for (int k = nsr_voff[row]; k < nsr_voff[row + 1]; ++k) v.push_back(s.s(nsrv[k]));
        return v;
    };
    // A task is compiled into local tables (offsets relative to the task),
    // hashed, and appended to the session tables only when its class is new.
    struct Local {
        vector<Req> reqs;
        vector<Term> terms;
        vector<int32_t> vals;
    };
    auto local_req = [&](Local& L, const string& key, int op, const vector<string>& values, Req* r) -> bool {
        r->key = E.sel_key(key);
        r->op = op;
        r->nvals = 0;
        r->val_off = (int32_t)L.vals.size();
        r->rhs = 0;
        switch (op) {  // labels.NewRequirement validation (selector.go:134-170)
            case OP_IN:
            case OP_NOTIN: if (values.empty()) return false; break;
            case OP_EXISTS:
            case OP_DNE: if (!values.empty()) return false; break;
            case OP_GT:
            case OP_LT: return values.size() == 1 && parse_int64(values[0], &r->rhs);
            default: return false;
        }
        for (auto& v : values) L.vals.push_back(E.vals.get(v));
        r->nvals = (int32_t)values.size();
        return true;
    };
    auto local_false = [&](Local& L, int weight) {
        Term t{(int32_t)L.reqs.size(), 1, weight, 0};
        L.reqs.push_back(Req{0, OP_FALSE, 0, 0, 0});
        L.terms.push_back(t);
    };
    // One NodeSelectorTerm.  required: MatchExpressions AND MatchFields
    // (helper/helpers.go:302-333); preferred: MatchExpressions only
    // (node_affinity.go:58-66).  *err: a preferred term's selector errors.
    auto local_nst = [&](Local& L, int row, bool required, int weight, bool* err) {
        if (required && ec[row] == 0 && fc[row] == 0) { local_false(L, weight); return; }  // empty term: nothing
        if (!required && ec[row] == 0) { local_false(L, weight); return; }                // labels.Nothing()
        vector<Req> rs;
        bool bad = false;
        for (int k = es[row]; k < es[row] + ec[row]; ++k) {
            Req r;
            int op = nsr_op[k];
            if (op > OP_LT || !local_req(L, s.s(nsr_key[k]), op, nsr_vals(k), &r)) bad = true;
            rs.push_back(r);
        }
        if (required) {
            for (int k = fs[row]; k < fs[row] + fc[row]; ++k) {
                vector<string> vs = nsr_vals(k);
                int op = nsr_op[k];
                if ((op != OP_IN && op != OP_NOTIN) || vs.size() != 1) { bad = true; continue; }
                if (s.s(nsr_key[k]) == "metadata.name") {
                    rs.push_back(Req{0, op == OP_IN ? OP_NAME_IN : OP_NAME_NOTIN, 0, find_node(vs[0]), 0});
                } else if ((op == OP_IN) != vs[0].empty()) {  // any other field reads ""
                    rs.push_back(Req{0, OP_FALSE, 0, 0, 0});
                }
            }
        }
        if (bad) {
            if (!required) { *err = true; return; }
            local_false(L, weight);  // NodeSelectorRequirementsAsSelector error: the term `continue`s
            return;
        }
        Term t{(int32_t)L.reqs.size(), (int32_t)rs.size(), weight, 0};
        for (auto& r : rs) L.reqs.push_back(r);
        L.terms.push_back(t);
    };

    std::unordered_map<string, int> class_ids;
    auto plo = s.offs("p_label_off", P);
    auto plk = S32("pl_key"), plv = S32("pl_val");
    using Col = kbs::Snapshot::Span<int32_t>;
    auto same_run = [](const vector<int32_t>& off, int a, int b, std::initializer_list<const Col*> cols) {
        const int na = off[a + 1] - off[a];
        if (na != off[b + 1] - off[b]) return false;
        for (const Col* c : cols)
            for (int k = 0; k < na; ++k)
                if ((*c)[off[a] + k] != (*c)[off[b] + k]) return false;
        return true;
    };
    auto same_prog = [&](int a, int b) {
        if (aff.program_id(a) == aff.program_id(b)) return true;
        const AffProgram *x = aff.program(a), *y = aff.program(b);
        if (!x || !y) return x == y;
        return x->ea == y->ea && x->pa_space == y->pa_space && x->pa_cnt == y->pa_cnt && x->pa_total == y->pa_total &&
               x->pa_self == y->pa_self && x->paa_space == y->paa_space && x->paa_cnt == y->paa_cnt &&
               x->ipa == y->ipa && x->upd == y->upd && x->pred_err == y->pred_err;
    };
    // Every input of the class of pod a equals pod b's (typical for the pods of
    // one job): the class is reused without building its signature.
    auto same_class_inputs = [&](int a, int b) {
        const HPod &A = S.pods[a], &B = S.pods[b];
        if (A.ns != B.ns || A.backfill != B.backfill) return false;
        if (A.req.c != B.req.c || A.req.m != B.req.m || A.req.g != B.req.g) return false;
        if (A.ireq.c != B.ireq.c || A.ireq.m != B.ireq.m || A.ireq.g != B.ireq.g) return false;
        if (A.nzc != B.nzc || A.nzm != B.nzm || pod_ports[a] != pod_ports[b]) return false;
        auto row = [&](int i) {  // equal contents, equal id
            const int r = paff.empty() ? -1 : paff[i];
            return r >= 0 && r < (int)row_canon.size() ? row_canon[r] : r;
        };
        if (row(a) != row(b)) return false;
        if (!same_run(pso, a, b, {&psk, &psv})) return false;
        if (!same_run(pto, a, b, {&tlk, &tlo, &tlv, &tle})) return false;
        if (aff.active && !(same_run(plo, a, b, {&plk, &plv}) && same_prog(a, b))) return false;
        return true;
    };
    vector<int> cls_pod;  // class -> its first pod
    // Pending pods of session jobs in pod order: a pod whose class inputs equal the
    // previous such pod's (kind 1) takes its class; the others (kind 2, run heads)
    // are looked up or built in pod order.  Compared and propagated in parallel over
    // pod ranges.
    // A run head whose class inputs (same_class_inputs' fields, as raw values and
    // string-table offsets) equal an earlier head's takes that head's class.
    std::unordered_map<string, int> input_cls;
    auto class_input_key = [&](int i) {
        const HPod& A = S.pods[i];
        string k;
        k.reserve(256);
        auto put = [&](auto v) { k.append((const char*)&v, sizeof v); };
        put(aff.active ? A.ns : -1);  // (a class depends on the namespace through its affinity program only)
        put((int)A.backfill);
        put(A.req.c); put(A.req.m); put(A.req.g); put(A.ireq.c); put(A.ireq.m); put(A.ireq.g);
        put(A.nzc); put(A.nzm);
        const int r = paff.empty() ? -1 : paff[i];
        put(r >= 0 && r < (int)row_canon.size() ? row_canon[r] : r);
        put(aff.active ? aff.program_id(i) : -1);
        auto run = [&](const vector<int32_t>& off, std::initializer_list<const Col*> cols) {
            put(off[i + 1] - off[i]);
            for (int q = off[i]; q < off[i + 1]; ++q)
                for (const Col* c : cols) put((*c)[q]);
        };
        run(pso, {&psk, &psv});
        run(pto, {&tlk, &tlo, &tlv, &tle});
        if (aff.active) run(plo, {&plk, &plv});
        const PortRun pr = pod_ports[i];
        for (const int32_t* q = pr.b; q != pr.e; ++q) put(*q);
        return k;
    };
    auto class_pod = [&](int i) { return S.pods[i].status == Pending && S.pods[i].job >= 0; };
    std::unique_ptr<uint8_t[]> ckind(new uint8_t[P]);
    vector<vector<int>> heads(bth);
    vector<vector<string>> head_keys(bth);  // class_input_key of each head
    par_b([&](int t) {
        const int lo = (int)((int64_t)P * t / bth), hi = (int)((int64_t)P * (t + 1) / bth);
        int prev = lo - 1;
        while (prev >= 0 && !class_pod(prev)) --prev;
        for (int i = lo; i < hi; ++i) {
            ckind[i] = 0;
            if (!class_pod(i)) continue;
            ckind[i] = prev >= 0 && same_class_inputs(prev, i) ? 1 : 2;
            if (ckind[i] == 2) { heads[t].push_back(i); head_keys[t].push_back(class_input_key(i)); }
            prev = i;
        }
    });
    std::unordered_map<string, vector<uint64_t>> tol_cache;  // toleration list -> tolerated taint ids
    for (int ht = 0; ht < bth; ++ht)
    for (size_t hk = 0; hk < heads[ht].size(); ++hk) {
        const int i = heads[ht][hk];
        HPod& p = S.pods[i];
        string& ikey = head_keys[ht][hk];
        if (auto ik = input_cls.find(ikey); ik != input_cls.end()) { p.cls = ik->second; continue; }
        TaskClass c{};
        c.ireq_cpu = p.ireq.c; c.ireq_mem = p.ireq.m; c.ireq_gpu = p.ireq.g;
        c.req_cpu = p.req.c; c.req_mem = p.req.m; c.req_gpu = p.req.g;
        c.nz_cpu = S.pods[i].nzc; c.nz_mem = S.pods[i].nzm;
        c.backfill = p.backfill;
        c.nsel_term = -1;
        c.req_term_n = -1;
        Local L;
        if (pso[i + 1] > pso[i]) {  // nodeSelector: labels.SelectorFromSet -> Equals requirements
            Term t{(int32_t)L.reqs.size(), 0, 0, 0};
            for (int k = pso[i]; k < pso[i + 1]; ++k) {
                Req r;
                local_req(L, s.s(psk[k]), OP_IN, {s.s(psv[k])}, &r);
                L.reqs.push_back(r);
                t.req_n++;
            }
            c.nsel_term = (int32_t)L.terms.size();
            L.terms.push_back(t);
        }
        int a = paff.empty() ? -1 : paff[i];
        if (a >= 0 && (a_flags[a] & KBS_AFF_NA)) {
            if (a_flags[a] & KBS_AFF_NA_REQ) {
                c.req_term_off = (int32_t)L.terms.size();
                for (int k = nareq_s[a]; k < nareq_s[a] + nareq_c[a]; ++k) local_nst(L, k, true, 0, nullptr);
                c.req_term_n = (int32_t)L.terms.size() - c.req_term_off;
            }
            c.pref_term_off = (int32_t)L.terms.size();
            bool err = false;
            for (int k = napref_s[a]; k < napref_s[a] + napref_c[a] && !err; ++k) {
                if (pst_w[k] == 0) continue;  // node_affinity.go:54-56
                local_nst(L, pst_t[k], false, pst_w[k], &err);
            }
            c.pref_term_n = (int32_t)L.terms.size() - c.pref_term_off;
            if (err) { c.score_err = 1; c.pref_term_n = 0; }
        }
        // tolerations -> tolerated taint ids (toleration.go:37-56)
        // (one mask per distinct toleration list: the string table is interned, equal offsets
        // are equal strings)
        E.tw = ((int)E.taint_defs.size() + 63) / 64;
        string tol_key;
        for (int k = pto[i]; k < pto[i + 1]; ++k)
            for (const Col* col : {&tlk, &tlo, &tlv, &tle}) tol_key.append((const char*)&(*col)[k], sizeof(int32_t));
        auto tit = tol_cache.find(tol_key);
        if (tit == tol_cache.end()) {
            vector<uint64_t> m(E.tw, 0);
            for (size_t t = 0; t < E.taint_defs.size(); ++t) {
                bool ok = false;
                for (int k = pto[i]; k < pto[i + 1] && !ok; ++k) {
                    string key = s.s(tlk[k]), op = s.s(tlo[k]), val = s.s(tlv[k]), eff = s.s(tle[k]);
                    if (!eff.empty() && eff != std::get<2>(E.taint_defs[t])) continue;
                    if (!key.empty() && key != std::get<0>(E.taint_defs[t])) continue;
                    if (op.empty() || op == "Equal") ok = val == std::get<1>(E.taint_defs[t]);
                    else if (op == "Exists") ok = true;
                }
                if (ok) m[t / 64] |= 1ULL << (t % 64);
            }
            tit = tol_cache.emplace(std::move(tol_key), std::move(m)).first;
        }
        const vector<uint64_t>& tol = tit->second;
        c.has_ports = pod_ports[i].empty() ? 0 : 1;
        const AffProgram* pg = aff.program(i);
        if (pg) {
            c.aff = 1;
            c.pred_err |= pg->pred_err;
            c.ea_n = (int32_t)pg->ea.size() / 2;
            c.pa_space = pg->pa_space; c.pa_cnt = pg->pa_cnt; c.pa_total = pg->pa_total; c.pa_self = pg->pa_self;
            c.paa_space = pg->paa_space; c.paa_cnt = pg->paa_cnt;
            c.ipa_n = (int32_t)pg->ipa.size() / 4;
            c.upd_n = (int32_t)pg->upd.size() / 3;
            c.dd_space = dedup_space(*pg, space_ndom);
            c.dd_ndom = c.dd_space >= 0 ? space_ndom[c.dd_space] : 0;
        } else {
            c.pa_space = c.paa_space = -1;
            c.dd_space = -1;
        }
        // class signature: the task-relative tables + the class fields (offsets are local)
        string sig((const char*)&c, sizeof(TaskClass));
        if (pg) {
            for (auto* v : {&pg->ea, &pg->ipa, &pg->upd}) {
                sig.append((const char*)v->data(), v->size() * sizeof(int32_t));
                sig.push_back('|');
            }
        }
        sig.append((const char*)L.reqs.data(), L.reqs.size() * sizeof(Req));
        sig.append((const char*)L.terms.data(), L.terms.size() * sizeof(Term));
        sig.append((const char*)L.vals.data(), L.vals.size() * sizeof(int32_t));
        sig.append((const char*)tol.data(), tol.size() * sizeof(uint64_t));
        for (int id : pod_ports[i]) sig.append((const char*)&id, sizeof id);
        auto it = class_ids.find(sig);
        if (it != class_ids.end()) {
            p.cls = it->second;
            input_cls.emplace(std::move(ikey), p.cls);
            continue;
        }
        // relocate into the session tables
        const int32_t req0 = (int32_t)E.reqs.size(), term0 = (int32_t)E.terms.size(), val0 = (int32_t)E.vals_list.size();
        for (Req r : L.reqs) {
            if (r.op <= OP_LT) r.val_off += val0;
            E.reqs.push_back(r);
        }
        for (Term t : L.terms) { t.req_off += req0; E.terms.push_back(t); }
        for (int32_t v : L.vals) E.vals_list.push_back(v);
        if (c.nsel_term >= 0) c.nsel_term += term0;
        c.req_term_off += term0;
        c.pref_term_off += term0;
        c.tol_off = (int32_t)E.masks.size();
        for (auto x : tol) E.masks.push_back(x);
        if (pg) {
            c.ea_off = (int32_t)aff_items.size();
            aff_items.insert(aff_items.end(), pg->ea.begin(), pg->ea.end());
            c.ipa_off = (int32_t)aff_items.size();
            aff_items.insert(aff_items.end(), pg->ipa.begin(), pg->ipa.end());
            c.upd_off = (int32_t)aff_items.size();
            aff_items.insert(aff_items.end(), pg->upd.begin(), pg->upd.end());
        }
        p.cls = (int)S.classes.size();
        class_ids.emplace(std::move(sig), p.cls);
        input_cls.emplace(std::move(ikey), p.cls);
        S.classes.push_back(c);
        cls_pod.push_back(i);  // classes are created in pod order: i is the class's first pod
    }
    par_b([&](int t) {  // the other pods: their run head's class
        const int lo = (int)((int64_t)P * t / bth), hi = (int)((int64_t)P * (t + 1) / bth);
        int cur = -1;
        for (int u = t - 1; u >= 0 && cur < 0; --u)
            if (!heads[u].empty()) cur = S.pods[heads[u].back()].cls;
        for (int i = lo; i < hi; ++i) {
            if (ckind[i] == 2) cur = S.pods[i].cls;
            else if (ckind[i] == 1) S.pods[i].cls = cur;
        }
    });
    mark("classes:loop");
    // port masks per class (conflict = CheckConflict, own = HostPortInfo.Add).
    // Port ids are renumbered in (protocol, port, IP) order, so the ids one
    // (protocol, port) can conflict with are contiguous; a class's masks then
    // cover a window of kPortWin words (TaskClass::pw_lo) of the node columns.
    {
        const size_t U = E.port_defs.size();
        vector<int> order(U), new_id(U);
        for (size_t u = 0; u < U; ++u) order[u] = (int)u;
        std::sort(order.begin(), order.end(), [&](int a, int b) {
            auto [aip, apr, aport] = E.port_defs[a];
            auto [bip, bpr, bport] = E.port_defs[b];
            return std::make_tuple(apr, aport, aip) < std::make_tuple(bpr, bport, bip);
        });
        vector<std::tuple<int, int, int32_t>> defs(U);
        for (size_t k = 0; k < U; ++k) { new_id[order[k]] = (int)k; defs[k] = E.port_defs[order[k]]; }
        E.port_defs.swap(defs);
        for (auto& id : S.pod_port_ids) id = new_id[id];
        for (auto& v : node_ports)
            for (auto& id : v) id = new_id[id];
        E.port_ids.clear();
    }
    E.pw = ((int)E.port_defs.size() + 63) / 64;
    {
        int zero_ip = E.ip_dict.get("0.0.0.0");
        for (size_t ci = 0; ci < S.classes.size(); ++ci) {
            TaskClass& c = S.classes[ci];
            int lo = INT32_MAX, hi = -1;  // ids the class's masks touch
            auto touch = [&](int id) { lo = std::min(lo, id); hi = std::max(hi, id); };
            for (int id : pod_ports[cls_pod[ci]]) {
                auto [ip, pr, port] = E.port_defs[id];
                touch(id);
                for (size_t u = 0; u < E.port_defs.size(); ++u) {
                    auto [uip, upr, uport] = E.port_defs[u];
                    if (upr != pr || uport != port) continue;
                    if (ip == zero_ip || uip == zero_ip || uip == ip) touch((int)u);
                }
            }
            c.pw_lo = hi < 0 ? 0 : lo / 64;
            if (hi >= 0 && hi / 64 - c.pw_lo >= kPortWin)
                fail_unsupported("a pod's host ports and their conflicts span more than " +
                                 std::to_string(kPortWin * 64) + " port ids");
            vector<uint64_t> conf(kPortWin, 0), own(kPortWin, 0);
            for (int id : pod_ports[cls_pod[ci]]) {
                auto [ip, pr, port] = E.port_defs[id];
                own[id / 64 - c.pw_lo] |= 1ULL << (id % 64);
                for (size_t u = 0; u < E.port_defs.size(); ++u) {
                    auto [uip, upr, uport] = E.port_defs[u];
                    if (upr != pr || uport != port) continue;
                    if (ip == zero_ip || uip == zero_ip || uip == ip) conf[u / 64 - c.pw_lo] |= 1ULL << (u % 64);
                }
            }
            c.pconf_off = (int32_t)E.masks.size();
            for (auto x : conf) E.masks.push_back(x);
            c.pown_off = (int32_t)E.masks.size();
            for (auto x : own) E.masks.push_back(x);
        }
    }
    S.n_spaces = aff.n_spaces;
    if (encode_only) {  // kbhip_debug_encode: keep copies of the compiled tables, touch no device
        S.h_dom = aff.dom;
        S.h_aff_cnt = aff.cnt;
        S.h_aff_scalar = aff.scalar;
        S.h_aff_items = aff_items;
    } else {
        HIPCHK(hipSetDevice(device));
        S.device = device;
        S.stream = MemPool::get().take_stream();
        S.ov_streams[0] = S.stream;
        for (int k = 1; k <= kMaxDep; ++k) S.ov_streams[k] = MemPool::get().take_stream();
    }
    mark("classes");
    // ---------------- upload ----------------
    // this session's node range: the whole array, or one contiguous shard
    const int lo = (int)((int64_t)N * S.rank / S.world), hi = (int)((int64_t)N * (S.rank + 1) / S.world);
    const int nl = hi - lo, npl = std::max(((nl + kBlock - 1) / kBlock) * kBlock, kBlock);
    vector<int64_t> col[13];
    for (int i = 0; i < 13; ++i) col[i].assign(npl, 0);
    for (int i = lo; i < hi; ++i) {
        const int r = i - lo;
        col[0][r] = idle[i].c; col[1][r] = idle[i].m; col[2][r] = idle[i].g;
        col[3][r] = rel[i].c; col[4][r] = rel[i].m; col[5][r] = rel[i].g;
        col[6][r] = bf[i].c; col[7][r] = bf[i].m; col[8][r] = bf[i].g;
        col[9][r] = acpu[i]; col[10][r] = amem[i]; col[11][r] = nzc[i]; col[12][r] = nzm[i];
    }
    int64_t** dst[13] = {&S.nc.idle_cpu, &S.nc.idle_mem, &S.nc.idle_gpu, &S.nc.rel_cpu, &S.nc.rel_mem, &S.nc.rel_gpu,
                         &S.nc.bf_cpu, &S.nc.bf_mem, &S.nc.bf_gpu, &S.nc.acpu, &S.nc.amem, &S.nc.nzc, &S.nc.nzm};
    for (int i = 0; i < 13; ++i) *dst[i] = upload(S, S.b_cols[i], col[i]);
    vector<int32_t> pods_col(npl, 0), max_col(npl, 0);
    vector<uint8_t> flags_col(npl, 0);
    for (int i = lo; i < hi; ++i) {
        pods_col[i - lo] = podcnt[i];
        max_col[i - lo] = (int32_t)apods[i];
        flags_col[i - lo] = (!unsched.empty() && unsched[i]) ? 1 : 0;
    }
    S.nc.pods = upload(S, S.b_cols[13], pods_col);
    S.nc.maxtasks = upload(S, S.b_cols[14], max_col);
    S.nc.flags = upload(S, S.b_cols[15], flags_col);
    const int K = (int)E.sel_keys.size();
    vector<int32_t> lab((size_t)std::max(K, 1) * npl, -1);
    for (auto& kv : E.sel_keys) {
        auto kit = E.keys_all.ids.find(kv.first);
        if (kit == E.keys_all.ids.end()) continue;  // no node has the key
        int kid = kit->second;
        for (int i = lo; i < hi; ++i)
            for (int q = E.nl_off[i]; q < E.nl_off[i + 1]; ++q)
                if (E.nl_kv[q].first == kid) lab[(size_t)kv.second * npl + (i - lo)] = E.nl_kv[q].second;
    }
    S.nc.labels = upload(S, S.b_labels, lab);
    vector<uint64_t> tcol((size_t)std::max(E.tw, 1) * npl, 0);
    for (int i = lo; i < hi; ++i)
        for (int id : node_taints[i]) tcol[(size_t)(id / 64) * npl + (i - lo)] |= 1ULL << (id % 64);
    S.nc.taints = upload(S, S.b_taints, tcol);
    vector<uint64_t> pcol((size_t)std::max(E.pw, 1) * npl, 0);
    for (int i = lo; i < hi; ++i)
        for (int id : node_ports[i]) pcol[(size_t)(id / 64) * npl + (i - lo)] |= 1ULL << (id % 64);
    S.nc.ports = upload(S, S.b_ports, pcol);
    S.n_aff_cnt = aff.active ? aff.cnt.size() : 1;
    S.n_aff_scalar = aff.active ? aff.scalar.size() : 1;
    if (aff.active) {  // domain columns cover every node on every shard (winners may be remote)
        S.nc.dom = upload(S, S.b_dom, aff.dom);
        if (aff_items.empty()) aff_items.push_back(0);
        S.tab.aff_items = upload(S, S.b_aff_items, aff_items);
        S.tab.aff_cnt = upload(S, S.b_aff_cnt, aff.cnt);
        S.tab.aff_scalar = upload(S, S.b_aff_scalar, aff.scalar);
    } else {
        vector<int32_t> one(1, 0);
        S.nc.dom = upload(S, S.b_dom, one);
        S.tab.aff_items = upload(S, S.b_aff_items, one);
        S.tab.aff_cnt = upload(S, S.b_aff_cnt, one);
        S.tab.aff_scalar = upload(S, S.b_aff_scalar, one);
    }
    S.nc.n = nl;
    S.nc.npad = npl;
    S.nc.base = lo;
    S.nc.dom_stride = npad;
    S.n_total = N;
    S.nc.n_keys = K;
    S.nc.taint_words = E.tw;
    S.nc.port_words = E.pw;
    // value tables (Gt/Lt parse per value id)
    vector<int64_t> valint(E.vals.strs.size() + 1, 0);
    vector<uint8_t> valok(E.vals.strs.size() + 1, 0);
    for (size_t v = 0; v < E.vals.strs.size(); ++v) valok[v] = parse_int64(E.vals.strs[v], &valint[v]);
    // 32-bit selection keys per class (class_key_format)
    S.class_kf.assign(S.classes.size(), KeyFormat{});
    S.class_srange.assign(S.classes.size(), {0, 0});
    for (size_t ci = 0; ci < S.classes.size(); ++ci)
        class_key_format(S, S.classes[ci], E.terms, N, &S.class_kf[ci], &S.class_srange[ci]);
    S.tab.classes = upload(S, S.b_classes, S.classes);
    S.tab.terms = upload(S, S.b_terms, E.terms);
    S.tab.reqs = upload(S, S.b_reqs, E.reqs);
    S.tab.vals = upload(S, S.b_vals, E.vals_list);
    S.tab.valint = upload(S, S.b_valint, valint);
    S.tab.valok = upload(S, S.b_valok, valok);
    S.tab.masks = upload(S, S.b_masks, E.masks);
    {
        static const vector<uint64_t> zero(kDedupMax, 0);  // (outlives the asynchronous copy)
        S.tab.dd_max = upload(S, S.b_dd_max, zero);
    }
    if (encode_only) {
        S.stats.nodes = N;
        S.stats.open_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        return;
    }
    hipStream_t st = S.stream;
    S.d_ctrl = S.b_ctrl.alloc<PopCtrl>(1);
    S.d_walk = S.b_walk.alloc<uint64_t>(npl);
    {
        int R2;
        const int nb2 = pop_blocks(nl, &R2);
        S.d_cand2 = S.b_cand2.alloc<uint64_t>((size_t)(std::max(nb2, 1) + kMaxGroups) * 64);
        S.d_arrive = S.b_arrive.alloc<uint32_t>((3 * kMaxGroups + 1) * 32);
        HIPCHK(hipMemsetAsync(S.d_arrive, 0, (3 * kMaxGroups + 1) * 32 * sizeof(uint32_t), st));
        S.d_fit4 = S.b_fit4.alloc<int32_t>(4 + 8);  // device counters + an int64[4] exchange slot
        if (S.world > 1) {
            S.d_shard_send = S.b_shard_send.alloc<ShardMsg>(1);
            S.d_shard_recv = S.b_shard_recv.alloc<ShardMsg>(S.world);
        }
        for (int k = 0; k <= kMaxDep; ++k) {
            const size_t cw = (size_t)(std::max(nb2, 1) + kMaxGroups) * kCandStride;  // tagged granules (seq >= 1)
            S.d_cand_ov[k] = S.b_cand_ov[k].alloc<uint64_t>(cw);
            HIPCHK(hipMemsetAsync(S.d_cand_ov[k], 0, cw * sizeof(uint64_t), st));
            S.d_arrive_ov[k] = S.b_arrive_ov[k].alloc<uint32_t>((3 * kMaxGroups + 1) * 32);
            HIPCHK(hipMemsetAsync(S.d_arrive_ov[k], 0, (3 * kMaxGroups + 1) * 32 * sizeof(uint32_t), st));
        }
        S.d_link = S.b_link.alloc<PopLink>(1);
        {
            PopLink init{};  // done 0; candidates of "pop 0": none, tagged 0
            for (auto& slot : init.touched)
                for (auto& g : slot) g = 0xffffffffull;
            HIPCHK(hipMemcpy(S.d_link, &init, sizeof(PopLink), hipMemcpyHostToDevice));
        }
        if (sizeof(PopOutHost) != pop_out_bytes()) throw Error(KBHIP_EINVAL, "PopOut layout mismatch");
        S.h_out = (PopOutHost*)MemPool::get().take(MemPool::kPinnedMapped, Session::kSlots * sizeof(PopOutHost),
                                                   &S.h_out_cap);
        HIPCHK(hipHostGetDevicePointer(&S.d_out, S.h_out, 0));
        std::memset(S.h_out, 0, Session::kSlots * sizeof(PopOutHost));
#ifdef KBHIP_STAMPS
        S.d_stamps = S.b_stamps.alloc<uint64_t>((size_t)nb2 * 4 + 16);
        HIPCHK(hipMemsetAsync(S.d_stamps, 0, ((size_t)nb2 * 4 + 16) * 8, st));
        HIPCHK(set_stamp_buffer(S.d_stamps));
#endif
    }
    HIPCHK(hipStreamSynchronize(st));
    mark("upload");
    // ---------------- kbhip_session_carry_snapshot's fast path ----------------
    S.keep.ok = S.world == 1 && !aff.active;
    if (S.keep.ok) {
        S.keep.class_ids = std::move(class_ids);
        S.keep.masks = E.masks;
        S.keep.taint_defs = E.taint_defs;
        S.keep.nss = E.nss;
        S.keep.conf_digest = conf_digest(s);
        S.keep.node_spec_digest = node_spec_digest(s);
    }
    // ---------------- ordering plugins OnSessionOpen ----------------
    for (int i = 0; i < N; ++i) S.total.add(R3{acpu[i], amem[i], agpu[i]});  // drf.go:61-63, proportion.go:59-61
    mark("keep");
    S.stats.nodes = N;
    S.stats.open_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

// Option "cu_split" (rehearsals of the node-sharded path on one GPU, DESIGN.md
// §6): the session's streams are replaced by streams restricted to CUs
// [part * C / parts, (part + 1) * C / parts) of the device's C, so that W
// ranks sharing one GPU each get their own share of the chip as W GPUs would.
void cu_split(Session& S, int part, int parts) {
    if (parts < 1 || part < 0 || part >= parts) throw Error(KBHIP_EINVAL, "cu_split: part must be in [0, parts)");
    if (S.encode_only || !S.stream) throw Error(KBHIP_EINVAL, "cu_split: the session has no streams");
    ov_quiesce(S);
    int cus = 0;
    HIPCHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, S.device));
    if (cus < parts) throw Error(KBHIP_EINVAL, "cu_split: more parts than CUs");
    vector<uint32_t> mask((cus + 31) / 32, 0u);
    for (int c = part * cus / parts; c < (part + 1) * cus / parts; ++c) mask[c / 32] |= 1u << (c % 32);
    HIPCHK(hipDeviceSynchronize());
    hipStream_t fresh[kMaxDep + 1] = {};
    for (int k = 0; k <= kMaxDep; ++k)
        HIPCHK(hipExtStreamCreateWithCUMask(&fresh[k], (uint32_t)mask.size(), mask.data()));
    for (int k = 0; k <= kMaxDep; ++k) {
        hipStream_t old = k == 0 ? S.stream : S.ov_streams[k];
        if (S.cu_masked) (void)hipStreamDestroy(old);
        else MemPool::get().give_stream(old, S.device);
        if (k == 0) S.stream = fresh[0];
        S.ov_streams[k] = fresh[k];
    }
    S.cu_masked = true;
}

}  // namespace kbhip
