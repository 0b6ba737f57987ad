// kbhip session, part 06: session carry-over from the scheduler cache
#include "session.h"

namespace kbhip {

// ---------------------------------------------------------------------------
// kbhip_session_carry_snapshot: the next session from the
// scheduler cache's snapshot of it (cache.go:515-583) — pod arrivals, deletions
// and phase changes, node updates, PodGroup and queue changes — re-deriving
// only what the changes touch.  old_pod[i] / old_node[n]: the index in this
// session of the new snapshot's pod i / node n (-1: new).  Fast path (the
// common shape: same node set, same labels / taints / conf, no pod affinity,
// new pods without host ports, nodeSelector or node affinity): mapped pods
// keep their dictionary ids, ports and task class; new pods are decoded and
// classed against the kept dictionaries; jobs, queues and node rows are
// re-derived; only changed node rows and the grown tables are uploaded.
// Anything else re-opens the session in place (same handle and options).
// ---------------------------------------------------------------------------
struct SavedOptions {
    bool batched, keys32, bf_batch, aff_batch, aff_fence, shard_overlap, rank_group, force_radix, debug_keys;
    int64_t time_every;
    int speculate, overlap, rank_first;
    bool engine, eng_quick, eng_lists, eng_timeline;  // the persistent engine's options
    int eng_nw_opt, eng_ng_opt;
};
static SavedOptions save_options(const Session& S) {
    return SavedOptions{S.batched, S.keys32, S.bf_batch, S.aff_batch, S.aff_fence, S.shard_overlap, S.rank_group,
                        S.force_radix,
                        S.debug_keys,
                        S.time_every, S.speculate, S.overlap, S.rank_first,
                        S.engine, S.eng_quick, S.eng_lists, S.d_eng_tl != nullptr,
                        S.eng_nw_opt, S.eng_ng_opt};
}
static void restore_options(Session& S, const SavedOptions& o) {
    S.batched = o.batched; S.keys32 = o.keys32; S.bf_batch = o.bf_batch; S.aff_batch = o.aff_batch;
    S.aff_fence = o.aff_fence;
    S.shard_overlap = o.shard_overlap;
    S.rank_group = o.rank_group; S.force_radix = o.force_radix; S.time_every = o.time_every;
    S.speculate = o.speculate; S.overlap = o.overlap; S.rank_first = o.rank_first;
    S.debug_keys = o.debug_keys;
    if (S.debug_keys && !S.d_dbg && !S.encode_only)
        S.d_dbg = S.b_dbg.alloc<uint64_t>((size_t)kMaxChunk * (2 * S.nc.npad + 4));
    S.engine = o.engine; S.eng_quick = o.eng_quick; S.eng_lists = o.eng_lists;
    S.eng_nw_opt = o.eng_nw_opt; S.eng_ng_opt = o.eng_ng_opt;
    S.eng_nw = 0;  // sized at the next engine pop
    if (o.eng_timeline && !S.d_eng_tl && !S.encode_only) {
        const size_t words = (size_t)kEngTlSlots * kEngTlEvents;
        S.d_eng_tl = S.b_eng_tl.alloc<uint64_t>(words);
        HIPCHK(hipMemset(S.d_eng_tl, 0, words * 8));
    }
}

// pass A of open_session for one pod (status, priority, requests, node)
struct PodView {
    const kbs::Snapshot& s;
    kbs::Snapshot::Span<int32_t> puid, pns, pjob, pnode, ppri, paff, ppc;
    kbs::Snapshot::Span<uint8_t> pphase, pdel, pbf, pdet;
    kbs::Snapshot::Span<int64_t> pts;
    vector<int32_t> pco, pio, pso, pto, cpo;
    kbs::Snapshot::Span<int64_t> ccpu, cmem, cgpu, iccpu, icmem, icgpu;
    kbs::Snapshot::Span<uint8_t> chas;
    int P;
    explicit PodView(const kbs::Snapshot& s_) : s(s_) {
        puid = s.span<int32_t>("p_uid");
        P = (int)puid.size();
        pns = s.span<int32_t>("p_ns"); pjob = s.span<int32_t>("p_job"); pnode = s.span<int32_t>("p_node");
        ppri = s.span<int32_t>("p_priority"); paff = s.span<int32_t>("p_aff"); ppc = s.span<int32_t>("p_pclass");
        pphase = s.span<uint8_t>("p_phase"); pdel = s.span<uint8_t>("p_deleting"); pbf = s.span<uint8_t>("p_backfill");
        pdet = s.span<uint8_t>("p_detached");
        pts = s.span<int64_t>("p_ts");
        if ((int)pns.size() != P || (int)pjob.size() != P || (int)pnode.size() != P || (int)ppri.size() != P ||
            (int)pphase.size() != P || (int)pts.size() != P)
            throw Error(KBHIP_EINVAL, "pod columns length mismatch");
        pco = s.offs("p_ctr_off", P);
        pio = s.offs("p_ictr_off", P);
        pso = s.offs("p_nsel_off", P);
        pto = s.offs("p_tol_off", P);
        ccpu = s.span<int64_t>("c_cpu"); cmem = s.span<int64_t>("c_mem"); cgpu = s.span<int64_t>("c_gpu");
        chas = s.span<uint8_t>("c_has");
        cpo = s.offs("c_port_off", ccpu.size());
        iccpu = s.span<int64_t>("ic_cpu"); icmem = s.span<int64_t>("ic_mem"); icgpu = s.span<int64_t>("ic_gpu");
    }
    bool has_node(int i) const { return pnode[i] >= 0 && s.str(pnode[i])[0] != '\0'; }
    int status(int i) const {  // api/helpers.go:35-61
        const int ph = pphase[i];
        const bool del = !pdel.empty() && pdel[i];
        if (ph == KBS_RUNNING) return del ? Releasing : Running;
        if (ph == KBS_PENDING) return del ? Releasing : (!has_node(i) ? Pending : Bound);
        if (ph == KBS_SUCCEEDED) return Succeeded;
        if (ph == KBS_FAILED) return Failed;
        return Unknown;
    }
    bool has_ports(int i) const {
        for (int k = pco[i]; k < pco[i + 1]; ++k)
            if (cpo[k + 1] > cpo[k]) return true;
        return false;
    }
    // the spec-derived fields (everything but status, node and the session ids)
    void spec(int i, HPod& p) const {
        p.priority = ppri[i];
        p.ts = pts[i];
        const char* pc = (!ppc.empty() && ppc[i] >= 0) ? s.str(ppc[i]) : "";
        p.critical = std::strcmp(s.str(pns[i]), "kube-system") == 0 ||
                     std::strcmp(pc, "system-cluster-critical") == 0 || std::strcmp(pc, "system-node-critical") == 0;
        p.backfill = !pbf.empty() && pbf[i];
        p.groupless = pjob[i] < 0;
        p.req = p.ireq = R3{};
        p.nzc = p.nzm = 0;
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
    }
};

void reopen_in_place(kb_session* ks, const kbs::Snapshot& s) {
    Session& S = ks->s;
    const SavedOptions o = save_options(S);
    const int dev = S.device;
    S.~Session();
    new (&S) Session();
    open_session(S, s, dev);
    restore_options(S, o);
    S.carry_bytes = -1;  // every table uploaded
}

// Whether the fast path can take the new snapshot (else: reopen_in_place).
static bool carry_fast_ok(const Session& S, const kbs::Snapshot& s, const PodView& v, const int32_t* old_pod,
                          const int32_t* old_node) {
    if (!S.keep.ok || S.world != 1) return false;
    const int N = (int)s.rows("n_name");
    if (N != (int)S.h_alloc.size()) return false;
    for (int n = 0; n < N; ++n) if (old_node[n] != n) return false;
    if (conf_digest(s) != S.keep.conf_digest || node_spec_digest(s) != S.keep.node_spec_digest) return false;
    auto a_flags = s.vec<uint8_t>("a_flags");
    for (uint8_t f : a_flags) if (f & (KBS_AFF_PA | KBS_AFF_PAA)) return false;  // pod (anti-)affinity
    for (int i = 0; i < v.P; ++i) {
        if (old_pod[i] >= 0) continue;
        if (v.pso[i + 1] > v.pso[i] || v.has_ports(i)) return false;   // nodeSelector / host ports
        if (!v.paff.empty() && v.paff[i] >= 0 && (a_flags[v.paff[i]] & KBS_AFF_NA)) return false;  // node affinity
    }
    return true;
}

void carry_snapshot(kb_session* ks, const kbs::Snapshot& s, const int32_t* old_pod, const int32_t* old_node) {
    Session& S = ks->s;
    if (S.world != 1) throw Error(KBHIP_EUNSUPPORTED, "kbhip_session_carry_snapshot on a node-sharded session");
    static const bool prof = std::getenv("KBHIP_OPEN_PROFILE") != nullptr;  // per-phase host times (diagnostic)
    auto tp = std::chrono::steady_clock::now();
    auto mark = [&](const char* what) {
        if (!prof) return;
        auto now = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[carry] %-10s %8.2f ms\n", what, std::chrono::duration<double>(now - tp).count() * 1e3);
        tp = now;
    };
    require_no_tickets(S);
    const PodView v(s);
    const int P = v.P, Pold = (int)S.pods.size(), N = (int)s.rows("n_name"), Nold = (int)S.h_alloc.size();
    {  // the maps: indices in range, each old pod / node at most once (the pod map by ranges in parallel)
        const size_t ns = (size_t)std::max(Pold, Nold);
        {
            std::unique_ptr<std::atomic<uint8_t>[]> seen_p(new std::atomic<uint8_t>[ns]());
            std::atomic<bool> bad{false};
            const int nth = P < (1 << 16) ? 1 : host_threads();
            auto chk = [&](int t) {
                for (int i = (int)((int64_t)P * t / nth); i < (int)((int64_t)P * (t + 1) / nth); ++i) {
                    const int o = old_pod[i];
                    if (o < -1 || o >= Pold || (o >= 0 && seen_p[o].fetch_or(1, std::memory_order_relaxed))) {
                        bad = true;
                        return;
                    }
                }
            };
            vector<std::thread> th;
            for (int t = 1; t < nth; ++t) th.emplace_back(chk, t);
            chk(0);
            for (auto& x : th) x.join();
            if (bad) throw Error(KBHIP_EINVAL, "bad old_pod map");
        }
        vector<char> seen(ns, 0);
        for (int n = 0; n < N; ++n) {
            const int o = old_node[n];
            if (o < -1 || o >= Nold || (o >= 0 && seen[o]++)) throw Error(KBHIP_EINVAL, "bad old_node map");
        }
    }
    mark("maps");
    ov_quiesce(S);
    HIPCHK(hipStreamSynchronize(S.stream));
    S.model_gen++;  // jobs are renumbered: per-pod caches of the host model are rebuilt
    if (!carry_fast_ok(S, s, v, old_pod, old_node)) {
        reopen_in_place(ks, s);
        return;
    }
    // UID order (kbsnap.h canonical order): the UID rank of a pod is its index
    {
        const int kThreads = host_threads();
        const int per = (P + kThreads - 1) / kThreads;
        std::atomic<bool> sorted{true};
        auto check = [&](int lo, int hi) {
            for (int i = std::max(lo, 1); i < hi; ++i)
                if (std::strcmp(s.str(v.puid[i - 1]), s.str(v.puid[i])) >= 0) { sorted = false; return; }
        };
        if (P < (1 << 16)) {
            check(0, P);
        } else {
            vector<std::thread> th;
            for (int t = 1; t < kThreads; ++t) th.emplace_back(check, t * per, std::min(P, (t + 1) * per));
            check(0, std::min(P, per));
            for (auto& x : th) x.join();
        }
        if (!sorted) {  // the fast path keeps UID ranks as indices
            reopen_in_place(ks, s);
            return;
        }
    }
    mark("checks");
    // the device node rows, read back into pinned memory while the host model is rebuilt
    // (compared with the new rows at the upload: only rows that differ are written)
    const int Nl = S.nc.n;
    struct ColRef { void* d; size_t elem, off; };
    vector<ColRef> dcols;
    size_t stage_bytes = 0;
    auto add_col = [&](void* d, size_t elem) {
        dcols.push_back({d, elem, stage_bytes});
        stage_bytes += ((size_t)Nl * elem + 255) & ~(size_t)255;
    };
    int64_t* dcol[13] = {S.nc.idle_cpu, S.nc.idle_mem, S.nc.idle_gpu, S.nc.rel_cpu, S.nc.rel_mem, S.nc.rel_gpu,
                         S.nc.bf_cpu, S.nc.bf_mem, S.nc.bf_gpu, S.nc.acpu, S.nc.amem, S.nc.nzc, S.nc.nzm};
    for (int k = 0; k < 13; ++k) add_col(dcol[k], sizeof(int64_t));
    add_col(S.nc.pods, sizeof(int32_t));
    add_col(S.nc.maxtasks, sizeof(int32_t));
    add_col(S.nc.flags, sizeof(uint8_t));
    for (int w = 0; w < S.nc.port_words; ++w) add_col(S.nc.ports + (size_t)w * S.nc.npad, sizeof(uint64_t));
    struct Stage {  // pooled pinned buffer, returned on every exit (after the stream has drained)
        uint8_t* p = nullptr;
        size_t cap = 0;
        int dev = 0;
        hipStream_t st = nullptr;
        ~Stage() {
            if (!p) return;
            (void)hipStreamSynchronize(st);
            MemPool::get().give(MemPool::kPinned, p, cap, dev);
        }
    } stage;
    stage.dev = S.device;
    stage.st = S.stream;
    stage.p = (uint8_t*)MemPool::get().take(MemPool::kPinned, std::max<size_t>(stage_bytes, 256), &stage.cap);
    for (auto& c : dcols)
        HIPCHK(hipMemcpyAsync(stage.p + c.off, c.d, (size_t)Nl * c.elem, hipMemcpyDeviceToHost, S.stream));
    // ---------------- nodes: allocatable, pods, unschedulable (labels / taints unchanged) ----------------
    auto acpu = s.vec<int64_t>("n_alloc_cpu"), amem = s.vec<int64_t>("n_alloc_mem"), agpu = s.vec<int64_t>("n_alloc_gpu"),
         apods = s.vec<int64_t>("n_alloc_pods");
    if ((int)acpu.size() != N || (int)amem.size() != N || (int)agpu.size() != N || (int)apods.size() != N)
        throw Error(KBHIP_EINVAL, "node columns length mismatch");
    auto unsched = s.vec<uint8_t>("n_unsched");
    auto nname = s.span<int32_t>("n_name");
    std::unordered_map<std::string_view, int> node_idx;  // names of the nodes new pods are bound to
    auto find_node = [&](std::string_view nm) -> int {
        if (node_idx.empty()) {
            node_idx.reserve((size_t)N * 2);
            for (int n = 0; n < N; ++n) node_idx.emplace(std::string_view(s.str(nname[n])), n);
        }
        auto it = node_idx.find(nm);
        return it == node_idx.end() ? -1 : it->second;
    };
    // ---------------- queues & jobs (as at open) ----------------
    auto qn = s.vec<int32_t>("q_name"), qw = s.vec<int32_t>("q_weight");
    auto qts = s.vec<int64_t>("q_ts");
    std::map<string, int> qidx;
    vector<HQueue> queues(qn.size());
    for (size_t i = 0; i < qn.size(); ++i) {
        queues[i].name = s.s(qn[i]);
        queues[i].weight = qw[i];
        queues[i].ts = qts.empty() ? 0 : qts[i];
        qidx[queues[i].name] = (int)i;
    }
    {
        int r = 0;
        std::map<string, int> rank;
        for (auto& kv : qidx) rank[kv.first] = r++;
        for (auto& q : queues) q.rank = rank[q.name];
    }
    auto jns = s.vec<int32_t>("j_ns"), jname = s.vec<int32_t>("j_name"), jq = s.vec<int32_t>("j_queue"),
         jmin = s.vec<int32_t>("j_min"), jpri = s.vec<int32_t>("j_pg_priority");
    auto jts = s.vec<int64_t>("j_ts");
    struct Src { string uid; int row, pod; };
    vector<Src> srcs;
    const int JN = (int)jns.size();
    const int jth = JN < (1 << 13) ? 1 : host_threads();
    srcs.resize(JN);
    auto par_j = [&](auto&& fn) {
        vector<std::thread> th;
        for (int t = 1; t < jth; ++t) th.emplace_back(fn, t);
        fn(0);
        for (auto& x : th) x.join();
    };
    par_j([&](int t) {  // job UIDs (namespace/name) by job ranges
        for (int j = (int)((int64_t)JN * t / jth); j < (int)((int64_t)JN * (t + 1) / jth); ++j)
            srcs[j] = {s.s(jns[j]) + "/" + s.s(jname[j]), j, -1};
    });
    for (int i = 0; i < P; ++i) {
        if (v.pjob[i] >= JN) throw Error(KBHIP_EINVAL, "pod job index out of range");
        if (v.pjob[i] < 0) srcs.push_back({s.s(v.puid[i]), -1, i});  // shadow PodGroup
    }
    {
        const int ns = (int)srcs.size();
        std::atomic<bool> sorted{true};
        if (jth == 1 || ns != JN) {
            sorted = std::is_sorted(srcs.begin(), srcs.end(), [](const Src& a, const Src& b) { return a.uid < b.uid; });
        } else {
            par_j([&](int t) {  // UID order checked by ranges
                for (int j = std::max(1, (int)((int64_t)ns * t / jth)); j < (int)((int64_t)ns * (t + 1) / jth); ++j)
                    if (srcs[j].uid < srcs[j - 1].uid) { sorted = false; return; }
            });
        }
        if (!sorted)
            std::stable_sort(srcs.begin(), srcs.end(), [](const Src& a, const Src& b) { return a.uid < b.uid; });
    }
    mark("jobs:srcs");
    vector<HJob> jobs;
    vector<string> job_uid;
    jobs.reserve(srcs.size());
    job_uid.reserve(srcs.size());
    vector<int> row_slot(jns.size(), -1), shadow_slot(P, -1);
    const auto default_q = qidx.find("default");
    std::unordered_map<int32_t, int> qslot_of;  // queue name (interned string offset) -> queue slot
    for (auto& src : srcs) {
        int qslot = -1;
        if (src.row >= 0) {
            auto qc = qslot_of.find(jq[src.row]);
            if (qc == qslot_of.end()) {
                auto qit = qidx.find(s.s(jq[src.row]));
                qc = qslot_of.emplace(jq[src.row], qit == qidx.end() ? -1 : qit->second).first;
            }
            qslot = qc->second;
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
            slot = (int)jobs.size();
            jobs.push_back(std::move(j));
            job_uid.push_back(std::move(src.uid));
        }
        if (src.row >= 0) row_slot[src.row] = slot;
        else shadow_slot[src.pod] = slot;
    }
    mark("jobs:slots");
    // ---------------- pods ----------------
    vector<HPod> pods;  // the pooled array (its pages already mapped): every element is assigned below
    spare_pods().take_keep(pods);
    pods.resize(P);
    mark("pods:array");
    vector<int32_t> port_off(P + 1, 0), port_ids;
    port_ids.reserve(S.pod_port_ids.size());
    const int tw = ((int)S.keep.taint_defs.size() + 63) / 64;
    auto pns = v.pns;
    auto tlk = s.span<int32_t>("tl_key"), tlo = s.span<int32_t>("tl_op"), tlv = s.span<int32_t>("tl_val"),
         tle = s.span<int32_t>("tl_effect");
    vector<int> new_classes;  // classes this carry appended
    // the pod pass's ranges; per range the tasks per job (the job task lists' offsets below)
    const int jth_p = P < (1 << 15) ? 1 : host_threads();
    const int per_p = (P + jth_p - 1) / jth_p;
    vector<vector<int32_t>> jcnt(jth_p, vector<int32_t>(jobs.size(), 0));
    {
        // node names of new bound pods and of pods whose node changed are looked up in a map
        // built up front (read-only in the parallel pass below)
        bool need_map = false;
        for (int i = 0; i < P && !need_map; ++i) need_map = old_pod[i] < 0 && v.has_node(i);
        if (need_map) find_node("");
        std::atomic<int> bad_pod{-1};
        std::atomic<bool> spec_changed{false};
        vector<int32_t> pcount(P, 0);
        auto pass = [&](int t, int lo, int hi) {  // the pods' records (kept or decoded), status, node, job
            int32_t* jc = jcnt[t].data();
            for (int i = lo; i < hi; ++i) {
                HPod& p = pods[i];
                const int o = old_pod[i];
                if (o >= 0) {
                    p = S.pods[o];  // spec-derived fields and session ids (namespace, class) kept
                    // ... once the cheap spec fields agree: an updated pod the caller mapped by UID
                    // (updatePod rebuilds its TaskInfo, event_handlers.go:167-184) must not keep a
                    // stale priority, backfill flag or request (its class): the session re-opens
                    R3 rq{};
                    for (int k = v.pco[i]; k < v.pco[i + 1]; ++k) { rq.c += v.ccpu[k]; rq.m += v.cmem[k]; rq.g += v.cgpu[k]; }
                    if (p.priority != v.ppri[i] || p.ts != v.pts[i] || p.backfill != (!v.pbf.empty() && v.pbf[i]) ||
                        rq.c != p.req.c || rq.m != p.req.m || rq.g != p.req.g)
                        spec_changed.store(true, std::memory_order_relaxed);
                } else {
                    p = HPod{};
                    v.spec(i, p);
                }
                p.job = v.pjob[i] >= 0 ? row_slot[v.pjob[i]] : shadow_slot[i];  // session job slot
                if (p.job >= 0) jc[p.job]++;
                p.uid_rank = i;
                p.status = v.status(i);
                p.node = -1;
                p.node_rel = false;
                p.detached = false;
                p.groupless = v.pjob[i] < 0;
                if (v.has_node(i)) {
                    int n = -1;
                    if (o >= 0 && S.pods[o].node >= 0 && S.pods[o].node < N &&
                        std::strcmp(s.str(nname[S.pods[o].node]), s.str(v.pnode[i])) == 0)
                        n = S.pods[o].node;
                    else if (!node_idx.empty()) {
                        auto it = node_idx.find(std::string_view(s.str(v.pnode[i])));
                        n = it == node_idx.end() ? -1 : it->second;
                    }
                    if (n < 0) {
                        int want = -1;
                        bad_pod.compare_exchange_strong(want, i);
                        continue;
                    }
                    p.node = n;
                    p.detached = !v.pdet.empty() && v.pdet[i];
                }
                pcount[i] = o >= 0 ? S.pod_port_off[o + 1] - S.pod_port_off[o] : 0;
            }
        };
        auto run = [&]() {
            for (auto& c : jcnt) std::fill(c.begin(), c.end(), 0);
            if (jth_p == 1) {
                pass(0, 0, P);
            } else {
                vector<std::thread> th;
                for (int t = 1; t < jth_p; ++t) th.emplace_back(pass, t, t * per_p, std::min(P, (t + 1) * per_p));
                pass(0, 0, std::min(P, per_p));
                for (auto& x : th) x.join();
            }
        };
        run();
        if (bad_pod >= 0 && node_idx.empty()) {  // a kept pod moved to another node: again, with the map
            find_node("");
            bad_pod = -1;
            run();
        }
        if (bad_pod >= 0) {
            const int i = bad_pod;
            throw Error(KBHIP_EINVAL, "pod " + s.s(v.puid[i]) + " is bound to node " + s.s(v.pnode[i]) +
                                          " which is not in the snapshot");
        }
        if (spec_changed) {  // nothing of the session has changed yet
            spare_pods().give(pods);
            reopen_in_place(ks, s);
            return;
        }
        for (int i = 0; i < P; ++i)  // namespace ids of new pods (the kept dictionary grows in order)
            if (old_pod[i] < 0) pods[i].ns = S.keep.nss.get(s.s(pns[i]));
        if (!S.pod_port_ids.empty()) {  // kept pods' host ports (none held: every offset stays 0)
            for (int i = 0; i < P; ++i) port_off[i + 1] = port_off[i] + pcount[i];
            port_ids.resize(port_off[P]);
            for (int i = 0; i < P; ++i)
                if (pcount[i])
                    std::copy(S.pod_port_ids.begin() + S.pod_port_off[old_pod[i]],
                              S.pod_port_ids.begin() + S.pod_port_off[old_pod[i] + 1], port_ids.begin() + port_off[i]);
        }
    }
    mark("pods");
    // From here the session's own state changes (classes, masks, node rows, then pods and jobs):
    // a failure part way leaves it unusable (every later call but close fails, kbhip.h)
    struct BreakOnThrow {
        Session& S;
        int pending = std::uncaught_exceptions();
        ~BreakOnThrow() {
            if (std::uncaught_exceptions() > pending)
                S.broken = "kbhip_session_carry_snapshot failed part way: close the session";
        }
    } break_on_throw{S};
    {
        // job task lists in pod order, filled by kThreads pod ranges: per-range counts per job
        // give every range its first position in each job's list
        // (each pod's job slot and the per-range counts: the pod pass above)
        const int J = (int)jobs.size();
        const int nth = jth_p;
        const int per = per_p;
        vector<vector<int32_t>>& cnt = jcnt;
        auto par = [&](auto&& fn) {
            vector<std::thread> th;
            for (int t = 1; t < nth; ++t) th.emplace_back(fn, t);
            fn(0);
            for (auto& x : th) x.join();
        };
        for (int j = 0; j < J; ++j) {  // per job: the ranges' offsets, the list's size
            int32_t off = 0;
            for (int t = 0; t < nth; ++t) {
                const int32_t k = cnt[t][j];
                cnt[t][j] = off;
                off += k;
            }
            jobs[j].tasks.resize(off);
        }
        par([&](int t) {
            const int lo = t * per, hi = std::min(P, lo + per);
            int32_t* c = cnt[t].data();
            for (int i = lo; i < hi; ++i) {
                const int slot = pods[i].job;
                if (slot >= 0) jobs[slot].tasks[c[slot]++] = i;
            }
        });
        par([&](int t) {  // job fields from their tasks (jobs split by ranges of job slots)
            const int jlo = (int)((int64_t)J * t / nth), jhi = (int)((int64_t)J * (t + 1) / nth);
            for (int j = jlo; j < jhi; ++j) {
                HJob& job = jobs[j];
                for (int i : job.tasks) {
                    const HPod& p = pods[i];
                    if (allocated_status(p.status)) job.cnt_alloc++;
                    if (p.status == AOB) job.cnt_aob++;
                    if (p.status == Pending && !(p.req.c < kMinCPU && p.req.m < kMinMem && p.req.g < kMinGPU))
                        job.maybe_pending = true;
                }
                // JobInfo.AddTaskInfo: the last task's priority (job_info.go:242)
                if (!job.tasks.empty()) job.priority = pods[job.tasks.back()].priority;
            }
        });
    }
    mark("jobs");
    // ---------------- task classes of pending tasks without one (new pods) ----------------
    int prev_new = -1;  // the last new pending pod classed here: a gang's pods share one spec
    auto same_spec = [&](int x, int y) {  // the class inputs the fast path reads (no selectors, ports, affinity)
        const HPod &X = pods[x], &Y = pods[y];
        if (X.job != Y.job || X.backfill != Y.backfill || X.nzc != Y.nzc || X.nzm != Y.nzm ||
            X.req.c != Y.req.c || X.req.m != Y.req.m || X.req.g != Y.req.g || X.ireq.c != Y.ireq.c ||
            X.ireq.m != Y.ireq.m || X.ireq.g != Y.ireq.g)
            return false;
        const int nx = v.pto[x + 1] - v.pto[x];
        if (nx != v.pto[y + 1] - v.pto[y]) return false;
        for (int k = 0; k < nx; ++k) {
            const int kx = v.pto[x] + k, ky = v.pto[y] + k;
            if (tlk[kx] != tlk[ky] || tlo[kx] != tlo[ky] || tlv[kx] != tlv[ky] || tle[kx] != tle[ky]) return false;
        }
        return true;
    };
    vector<int> need_cls;  // pending pods of a job without a class (new pods), in pod order
    {
        const int nth = P < (1 << 15) ? 1 : host_threads();
        vector<vector<int>> part(nth);
        auto scan = [&](int t) {
            const int lo = (int)((int64_t)P * t / nth), hi = (int)((int64_t)P * (t + 1) / nth);
            for (int i = lo; i < hi; ++i) {
                HPod& p = pods[i];
                if (p.status != Pending || p.job < 0) { if (old_pod[i] < 0) p.cls = -1; continue; }
                if (p.cls < 0) part[t].push_back(i);  // (else kept: the pod's spec did not change)
            }
        };
        vector<std::thread> th;
        for (int t = 1; t < nth; ++t) th.emplace_back(scan, t);
        scan(0);
        for (auto& x : th) x.join();
        for (auto& q : part) need_cls.insert(need_cls.end(), q.begin(), q.end());
    }
    for (int i : need_cls) {
        HPod& p = pods[i];
        if (prev_new >= 0 && same_spec(prev_new, i)) {  // (string offsets compared: the table is interned)
            p.cls = pods[prev_new].cls;
            prev_new = i;
            continue;
        }
        prev_new = i;
        TaskClass c{};
        c.ireq_cpu = p.ireq.c; c.ireq_mem = p.ireq.m; c.ireq_gpu = p.ireq.g;
        c.req_cpu = p.req.c; c.req_mem = p.req.m; c.req_gpu = p.req.g;
        c.nz_cpu = p.nzc; c.nz_mem = p.nzm;
        c.backfill = p.backfill;
        c.nsel_term = -1;
        c.req_term_n = -1;
        vector<uint64_t> tol(tw, 0);  // tolerations -> tolerated taint ids (toleration.go:37-56)
        for (size_t t = 0; t < S.keep.taint_defs.size(); ++t) {
            bool ok = false;
            for (int k = v.pto[i]; k < v.pto[i + 1] && !ok; ++k) {
                string key = s.s(tlk[k]), op = s.s(tlo[k]), val = s.s(tlv[k]), eff = s.s(tle[k]);
                if (!eff.empty() && eff != std::get<2>(S.keep.taint_defs[t])) continue;
                if (!key.empty() && key != std::get<0>(S.keep.taint_defs[t])) continue;
                if (op.empty() || op == "Equal") ok = val == std::get<1>(S.keep.taint_defs[t]);
                else if (op == "Exists") ok = true;
            }
            if (ok) tol[t / 64] |= 1ULL << (t % 64);
        }
        c.pa_space = c.paa_space = -1;
        c.dd_space = -1;
        // the class signature exactly as open_session builds it (no selector terms, no ports, no program)
        string sig((const char*)&c, sizeof(TaskClass));
        sig.append((const char*)tol.data(), tol.size() * sizeof(uint64_t));
        auto it = S.keep.class_ids.find(sig);
        if (it != S.keep.class_ids.end()) { p.cls = it->second; continue; }
        c.tol_off = (int32_t)S.keep.masks.size();
        for (auto x : tol) S.keep.masks.push_back(x);
        c.pconf_off = (int32_t)S.keep.masks.size();
        for (int w = 0; w < kPortWin; ++w) S.keep.masks.push_back(0);
        c.pown_off = (int32_t)S.keep.masks.size();
        for (int w = 0; w < kPortWin; ++w) S.keep.masks.push_back(0);
        p.cls = (int)S.classes.size();
        S.keep.class_ids.emplace(std::move(sig), p.cls);
        S.classes.push_back(c);
        new_classes.push_back(p.cls);
    }
    mark("classes");
    // ---------------- node rows from the pods (cache addTask -> NodeInfo.AddTask) ----------------
    vector<int64_t> col[13];
    for (auto& c : col) c.assign(N, 0);
    vector<int32_t> podcnt(N, 0), maxc(N, 0);
    vector<uint8_t> flg(N, 0);
    vector<uint64_t> pcol((size_t)std::max(S.nc.port_words, 1) * S.nc.npad, 0);
    S.used.assign(N, R3{});
    for (int n = 0; n < N; ++n) {
        col[0][n] = acpu[n]; col[1][n] = amem[n]; col[2][n] = agpu[n];
        col[9][n] = acpu[n]; col[10][n] = amem[n];
        maxc[n] = (int32_t)apods[n];
        flg[n] = (!unsched.empty() && unsched[n]) ? 1 : 0;
    }
    {
        // every thread scans all pods and adds the ones on its own node range (no shared writes;
        // per node the additions keep pod order, as the serial pass would)
        const int kThreads = host_threads();
        const int nth = P < (1 << 15) ? 1 : kThreads;
        // pods on a node, bucketed by (pod range, node range) in one parallel pass; then each
        // thread adds its node range's pods, pod ranges in order (per node: pod order)
        vector<int> nb(nth + 1);
        for (int t = 0; t <= nth; ++t) nb[t] = (int)((int64_t)N * t / nth);
        vector<vector<vector<int32_t>>> bucket(nth, vector<vector<int32_t>>(nth));
        auto fill = [&](int t) {
            const int lo = (int)((int64_t)P * t / nth), hi = (int)((int64_t)P * (t + 1) / nth);
            for (int i = lo; i < hi; ++i) {
                const HPod& p = pods[i];
                if (!on_node_of(p)) continue;
                int r = (int)((int64_t)p.node * nth / N);
                while (r > 0 && p.node < nb[r]) --r;
                while (r + 1 < nth && p.node >= nb[r + 1]) ++r;
                bucket[t][r].push_back(i);
            }
        };
        {
            vector<std::thread> th;
            for (int t = 1; t < nth; ++t) th.emplace_back(fill, t);
            fill(0);
            for (auto& x : th) x.join();
        }
        auto rows = [&](int t) {
            for (int b = 0; b < nth; ++b)
            for (int i : bucket[b][t]) {
                const HPod& p = pods[i];
                const int n = p.node;
                if (p.backfill) { col[6][n] += p.req.c; col[7][n] += p.req.m; col[8][n] += p.req.g; }
                if (p.status == Releasing) { col[3][n] += p.req.c; col[4][n] += p.req.m; col[5][n] += p.req.g; }
                col[0][n] -= p.req.c; col[1][n] -= p.req.m; col[2][n] -= p.req.g;
                S.used[n].c += p.req.c; S.used[n].m += p.req.m; S.used[n].g += p.req.g;
                podcnt[n]++;
                col[11][n] += p.nzc;
                col[12][n] += p.nzm;
                for (int k = port_off[i]; k < port_off[i + 1]; ++k) {
                    const int id = port_ids[k];
                    pcol[(size_t)(id / 64) * S.nc.npad + n] |= 1ULL << (id % 64);
                }
            }
        };
        vector<std::thread> th;
        for (int t = 1; t < nth; ++t) th.emplace_back(rows, t);
        rows(0);
        for (auto& x : th) x.join();
    }
    S.any_bf = 0;
    for (int n = 0; n < N; ++n) if (col[6][n] || col[7][n] || col[8][n]) S.any_bf = 1;
    mark("rows");
    // ---------------- device: the node rows that differ, the grown class tables ----------------
    int64_t uploaded = 0;
    HIPCHK(hipStreamSynchronize(S.stream));  // the read-back of the device rows
    size_t ci = 0;
    vector<RowPatch> patches;  // the differing elements, written by one k_row_patch launch
    auto sync_col = [&](void* dptr, const void* want, size_t elem) {
        if (ci >= dcols.size() || dcols[ci].d != dptr || dcols[ci].elem != elem)
            throw Error(KBHIP_EDEVICE, "carry: device row read-back out of order");
        const uint8_t* hv = stage.p + dcols[ci++].off;
        const uint8_t* w = (const uint8_t*)want;
        auto scan = [&](auto zero) {  // typed compares (a memcmp call per element costs more than the rows)
            using T = decltype(zero);
            const T* a = reinterpret_cast<const T*>(hv);
            const T* b = reinterpret_cast<const T*>(w);
            for (int n = 0; n < Nl; ++n) {
                if (a[n] == b[n]) continue;
                patches.push_back({(uint64_t)(uintptr_t)((T*)dptr + n), (uint64_t)b[n], (int32_t)sizeof(T), 0});
                uploaded += (int64_t)sizeof(T);
            }
        };
        if (elem == 8) scan(uint64_t{0});
        else if (elem == 4) scan(uint32_t{0});
        else scan(uint8_t{0});
    };
    for (int k = 0; k < 13; ++k) sync_col(dcol[k], col[k].data(), sizeof(int64_t));
    sync_col(S.nc.pods, podcnt.data(), sizeof(int32_t));
    sync_col(S.nc.maxtasks, maxc.data(), sizeof(int32_t));
    sync_col(S.nc.flags, flg.data(), sizeof(uint8_t));
    for (int w = 0; w < S.nc.port_words; ++w)
        sync_col(S.nc.ports + (size_t)w * S.nc.npad, pcol.data() + (size_t)w * S.nc.npad, sizeof(uint64_t));
    DevBuf d_patch;
    if (!patches.empty()) {
        RowPatch* dp = d_patch.alloc<RowPatch>(patches.size());
        HIPCHK(hipMemcpyAsync(dp, patches.data(), patches.size() * sizeof(RowPatch), hipMemcpyHostToDevice, S.stream));
        HIPCHK(launch_row_patch(dp, (int)patches.size(), S.stream));
    }
    if (!new_classes.empty()) {
        S.class_kf.resize(S.classes.size());
        S.class_srange.resize(S.classes.size());
        static const vector<Term> no_terms;
        for (int ci : new_classes) class_key_format(S, S.classes[ci], no_terms, N, &S.class_kf[ci], &S.class_srange[ci]);
        S.tab.classes = upload(S, S.b_classes, S.classes);
        S.tab.masks = upload(S, S.b_masks, S.keep.masks);
        uploaded += (int64_t)(S.classes.size() * sizeof(TaskClass) + S.keep.masks.size() * sizeof(uint64_t));
    }
    HIPCHK(hipStreamSynchronize(S.stream));  // the host sources above are about to go away
    mark("upload");
    // ---------------- the host model of the new session ----------------
    spare_pods().give(S.pods);
    S.pods.swap(pods);
    S.pod_port_off.swap(port_off);
    S.pod_port_ids.swap(port_ids);
    S.jobs.swap(jobs);
    S.job_uid.swap(job_uid);
    S.queues.swap(queues);
    for (int n = 0; n < N; ++n) S.h_alloc[n] = R3{acpu[n], amem[n], agpu[n]};
    S.total = F3{};
    for (int n = 0; n < N; ++n) S.total.add(S.h_alloc[n]);  // drf.go:61-63, proportion.go:59-61
    S.carry_bytes = uploaded;
    S.tab_delta.clear();
    S.plugins_opened = false;
    S.fallback = -1;
    S.sess_cnt.clear();
    S.node_tasks.clear();
    S.log.clear();
    S.last_fit_ok = false;
    S.stats.nodes = N;
    mark("swap");
}

int evict_action(kb_session* s, bool preempt, int32_t* out_pod, int32_t* out_node, uint8_t* out_kind,
                        int64_t cap) {
    ABI_GUARD_S(s, {
        check_log_args(s, out_pod, out_node, out_kind, cap);
        kbhip::require_no_tickets(s->s);
        HIPCHK(hipSetDevice(s->s.device));
        kbhip::ov_quiesce(s->s);
        s->s.log.clear();
        kbhip::evict_run(s->s, preempt);
        HIPCHK(hipStreamSynchronize(s->s.stream));
        const int64_t n = (int64_t)s->s.log.size();
        for (int64_t i = 0; i < n && i < cap; ++i) {
            out_pod[i] = std::get<0>(s->s.log[i]);
            out_node[i] = std::get<1>(s->s.log[i]);
            out_kind[i] = (uint8_t)std::get<2>(s->s.log[i]);
        }
        return (int)n;
    })
}

}  // namespace kbhip
