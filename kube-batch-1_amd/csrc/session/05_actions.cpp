// kbhip session, part 05: backfill, the standalone sweeps and the C-ABI entry points of the actions
#include "session.h"

namespace kbhip {


void backfill_run(Session& S) {
    vector<int32_t> cand;
    for (auto& j : S.jobs)
        for (int t : j.tasks) {
            const HPod& p = S.pods[t];
            if (p.status != Pending || p.cls < 0) continue;
            if (!(p.ireq.c < kMinCPU && p.ireq.m < kMinMem && p.ireq.g < kMinGPU)) continue;  // IsEmpty
            cand.push_back(t);
        }
    vector<int32_t> node(cand.size());
    first_fit(S, cand.data(), (int)cand.size(), node.data());
}

// The nodeorder sweep of one task as the preempt action uses it
// (preempt.go:270-287): per node, pack_key(score, index) when the node passes
// PredicateFn and has a NodeOrderFn score, 0 otherwise; sorting the keys
// descending gives util.SelectBestNode's order.  Reads the session state,
// changes nothing.  Returns the number of passing nodes.
int sweep_scores(Session& S, int pod, uint64_t* out_keys) {
    if (pod < 0 || pod >= (int)S.pods.size() || S.pods[pod].cls < 0)
        throw Error(KBHIP_EINVAL, "task id has no task class (not a pending task of the session)");
    if (S.world != 1) throw Error(KBHIP_EUNSUPPORTED, "sweep_scores on a node-sharded session");
    ov_quiesce(S);
    const int cls = S.pods[pod].cls;
    const int N = S.nc.n;
    if (!S.b_rank_keys.p) {
        S.b_rank_keys.alloc<uint64_t>(std::max(N, 1));
        S.b_rank_cnt.alloc<uint32_t>(4);
    }
    if (!S.b_sweep_cnt.p) S.b_sweep_cnt.alloc<uint32_t>(8 * 32);
    ctrl_setup(S, 1, &cls, 0, 0, 0, 0, -1, 0);
    const TaskClass& c = S.classes[cls];
    if (c.ipa_n > 0) HIPCHK(launch_ipa_minmax(S.nc, S.tab, S.d_ctrl, 0, S.stream));
    HIPCHK(hipMemsetAsync(S.b_sweep_cnt.p, 0, 8 * 32 * sizeof(uint32_t), S.stream));
    const bool timed = S.time_every > 0;  // the standalone sweep's own duration (bench.py's sweep roofline)
    if (timed) {
        if (!S.ev_sweep[0]) { HIPCHK(hipEventCreate(&S.ev_sweep[0])); HIPCHK(hipEventCreate(&S.ev_sweep[1])); }
        HIPCHK(hipEventRecord(S.ev_sweep[0], S.stream));
    }
    HIPCHK(launch_score_sweep(S.conf, S.nc, S.tab, c, S.d_ctrl, (uint64_t*)S.b_rank_keys.p,
                              (uint32_t*)S.b_sweep_cnt.p, S.stream));
    if (timed) HIPCHK(hipEventRecord(S.ev_sweep[1], S.stream));
    uint32_t cnt[8 * 32];
    HIPCHK(hipMemcpyAsync(cnt, S.b_sweep_cnt.p, sizeof cnt, hipMemcpyDeviceToHost, S.stream));
    if (out_keys && N)
        HIPCHK(hipMemcpyAsync(out_keys, S.b_rank_keys.p, (size_t)N * sizeof(uint64_t), hipMemcpyDeviceToHost,
                              S.stream));
    HIPCHK(hipStreamSynchronize(S.stream));
    if (timed) {
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, S.ev_sweep[0], S.ev_sweep[1]));
        S.stats.score_sweep_s += ms * 1e-3;
        S.stats.score_sweeps++;
    }
    S.stats.sweeps++;
    uint32_t total = 0;
    for (int g = 0; g < 8; ++g) total += cnt[32 * g];
    return (int)total;
}

// kbhip_time_sweeps: the standalone sweep of each task, launched back to back
// (option "time_sweeps_cold": one at a time behind a cache-evicting write)
// (no copies in between), one HIP-event pair around the whole sequence: the
// device time per sweep launch, boundaries between launches included.
double time_sweeps(Session& S, const int32_t* ids, int n) {
    if (S.world != 1) throw Error(KBHIP_EUNSUPPORTED, "time_sweeps on a node-sharded session");
    for (int i = 0; i < n; ++i)
        if (ids[i] < 0 || ids[i] >= (int)S.pods.size() || S.pods[ids[i]].cls < 0)
            throw Error(KBHIP_EINVAL, "task id has no task class (not a pending task of the session)");
    bool any_ipa = false;
    for (int i = 0; i < n; ++i) any_ipa |= S.classes[S.pods[ids[i]].cls].ipa_n > 0;
    if (any_ipa) throw Error(KBHIP_EUNSUPPORTED, "time_sweeps: classes with inter-pod terms need their prepass");
    ov_quiesce(S);
    const int N = S.nc.n;
    if (!S.b_rank_keys.p) {
        S.b_rank_keys.alloc<uint64_t>(std::max(N, 1));
        S.b_rank_cnt.alloc<uint32_t>(4);
    }
    if (!S.b_sweep_cnt.p) S.b_sweep_cnt.alloc<uint32_t>(8 * 32);
    // one control block per task (the kernel reads its class from ctrl->cls[0])
    DevBuf ctl;
    vector<PopCtrl> h(n);
    for (int i = 0; i < n; ++i) {
        std::memset(&h[i], 0, sizeof(PopCtrl));
        h[i].cls[0] = S.pods[ids[i]].cls;
        h[i].fallback = -1;
    }
    PopCtrl* d = ctl.alloc<PopCtrl>(std::max(n, 1));
    HIPCHK(hipMemcpyAsync(d, h.data(), (size_t)n * sizeof(PopCtrl), hipMemcpyHostToDevice, S.stream));
    HIPCHK(hipMemsetAsync(S.b_sweep_cnt.p, 0, 8 * 32 * sizeof(uint32_t), S.stream));
    if (!S.ev_sweep[0]) { HIPCHK(hipEventCreate(&S.ev_sweep[0])); HIPCHK(hipEventCreate(&S.ev_sweep[1])); }
    if (S.sweeps_cold) {
        // cold caches: 512 MB (twice the 256 MB Infinity Cache, far beyond the 8 x 4 MB of L2)
        // written (1) or read (2) before every launch, so that each sweep reads its columns
        // from HBM; HIP events around each launch alone.  A write leaves up to the Infinity
        // Cache's size of dirty lines whose write-back may overlap the sweep; a read does not.
        DevBuf flush;
        const size_t fb = (size_t)512 << 20;
        void* fp = flush.alloc<uint8_t>(fb);
        if (S.sweeps_cold == 2) {  // written once, then read twice so its write-back has drained
            HIPCHK(hipMemsetAsync(fp, 1, fb, S.stream));
            for (int k = 0; k < 2; ++k) HIPCHK(launch_evict_read(fp, fb, S.stream));
            HIPCHK(hipStreamSynchronize(S.stream));
        }
        double total_ms = 0;
        for (int i = 0; i < n; ++i) {
            if (S.sweeps_cold == 2) HIPCHK(launch_evict_read(fp, fb, S.stream));
            else HIPCHK(hipMemsetAsync(fp, i & 0xff, fb, S.stream));
            HIPCHK(hipEventRecord(S.ev_sweep[0], S.stream));
            HIPCHK(launch_score_sweep(S.conf, S.nc, S.tab, S.classes[h[i].cls[0]], d + i, (uint64_t*)S.b_rank_keys.p,
                                      (uint32_t*)S.b_sweep_cnt.p, S.stream));
            HIPCHK(hipEventRecord(S.ev_sweep[1], S.stream));
            HIPCHK(hipEventSynchronize(S.ev_sweep[1]));
            float ms = 0;
            HIPCHK(hipEventElapsedTime(&ms, S.ev_sweep[0], S.ev_sweep[1]));
            total_ms += ms;
        }
        flush.release();
        ctl.release();
        return n > 0 ? total_ms * 1e3 / n : 0.0;
    }
    HIPCHK(hipEventRecord(S.ev_sweep[0], S.stream));
    for (int i = 0; i < n; ++i) {
        HIPCHK(launch_score_sweep(S.conf, S.nc, S.tab, S.classes[h[i].cls[0]], d + i, (uint64_t*)S.b_rank_keys.p,
                                  (uint32_t*)S.b_sweep_cnt.p, S.stream));
    }
    HIPCHK(hipEventRecord(S.ev_sweep[1], S.stream));
    HIPCHK(hipStreamSynchronize(S.stream));
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, S.ev_sweep[0], S.ev_sweep[1]));
    ctl.release();
    return n > 0 ? (double)ms * 1e3 / n : 0.0;
}

// kbhip_time_rank_multi: the preempt node ranking (preempt.go:270-287's
// PredicateFn + NodeOrderFn sweep, then the stable counting sort) of n
// what-if sessions as ONE multi-session launch chain — k_rank_bucket_multi /
// k_rank_scan_multi / k_rank_scatter_multi, blockIdx.y = session, each on its
// own node columns: what the StepBatcher issues for coinciding rankings —
// session i ranking for its pending task ids[i].  The chain is launched reps
// times back to back (evict 0) or each time behind a 512 MB cache-evicting
// read (evict 2) on session 0's stream, HIP events around each; returns the
// microseconds per chain.  The descriptors are copied to device memory first
// (mapped = 0) or read by the kernels from pinned mapped host memory (1).
double time_rank_multi(Session* const* ss, int n, const int32_t* ids, int reps, int evict, int mapped) {
    if (n < 1 || reps < 1) throw Error(KBHIP_EINVAL, "time_rank_multi: n and reps must be positive");
    if (evict != 0 && evict != 2) throw Error(KBHIP_EINVAL, "time_rank_multi: evict must be 0 or 2");
    Session& S0 = *ss[0];
    int max_nblk = 1;
    vector<RankDesc> h(n);
    for (int i = 0; i < n; ++i) {
        Session& S = *ss[i];
        if (S.world != 1 || S.encode_only) throw Error(KBHIP_EUNSUPPORTED, "time_rank_multi: one-GPU sessions only");
        if (S.device != S0.device) throw Error(KBHIP_EINVAL, "time_rank_multi: sessions on different devices");
        for (int j = 0; j < i; ++j)
            if (ss[j] == ss[i]) throw Error(KBHIP_EINVAL, "time_rank_multi: a session appears twice");
        if (ids[i] < 0 || ids[i] >= (int)S.pods.size() || S.pods[ids[i]].cls < 0)
            throw Error(KBHIP_EINVAL, "task id has no task class (not a pending task of the session)");
        const int cls = S.pods[ids[i]].cls;
        const auto sr = S.class_srange[cls];
        if (S.classes[cls].ipa_n > 0 || sr.second - sr.first >= 256)
            throw Error(KBHIP_EUNSUPPORTED, "time_rank_multi: classes of the one-pass counting sort only");
        ov_quiesce(S);
        rank_buffers(S);
        flush_tables(S);
        ctrl_setup(S, 1, &cls, 0, 0, 0, 0, -1, 0);
        HIPCHK(hipMemsetAsync(S.b_rank_cnt.p, 0, 2 * sizeof(uint32_t), S.stream));
        HIPCHK(fill_rank_desc(&h[i], S.conf, S.nc, S.tab, S.classes[cls], S.d_ctrl, 1, (int)sr.first, (int)sr.second,
                              (uint64_t*)S.b_rank_keys.p, (uint32_t*)S.b_rank_tmp.p, (uint64_t*)S.b_rank_sorted.p,
                              (uint32_t*)S.b_rank_cnt.p));
        max_nblk = std::max(max_nblk, h[i].nblk);
        HIPCHK(hipStreamSynchronize(S.stream));  // every session's control block is in place
    }
    HIPCHK(hipSetDevice(S0.device));
    size_t cap = 0;
    RankDesc* hp = (RankDesc*)MemPool::get().take(MemPool::kPinnedMapped, (size_t)n * sizeof(RankDesc), &cap);
    std::memcpy(hp, h.data(), (size_t)n * sizeof(RankDesc));
    DevBuf dd;
    const RankDesc* desc = nullptr;
    if (mapped) {
        void* dp = nullptr;
        HIPCHK(hipHostGetDevicePointer(&dp, hp, 0));
        desc = (const RankDesc*)dp;
    } else {
        desc = dd.alloc<RankDesc>(n);
        HIPCHK(hipMemcpyAsync((void*)desc, hp, (size_t)n * sizeof(RankDesc), hipMemcpyHostToDevice, S0.stream));
    }
    DevBuf flush;
    const size_t fb = (size_t)512 << 20;
    void* fp = nullptr;
    if (evict) {
        fp = flush.alloc<uint8_t>(fb);
        HIPCHK(hipMemsetAsync(fp, 1, fb, S0.stream));
        for (int k = 0; k < 2; ++k) HIPCHK(launch_evict_read(fp, fb, S0.stream));
    }
    hipEvent_t ev[2];
    HIPCHK(hipEventCreate(&ev[0]));
    HIPCHK(hipEventCreate(&ev[1]));
    double total_ms = 0;
    HIPCHK(hipStreamSynchronize(S0.stream));
    for (int r = 0; r < reps; ++r) {
        if (evict) HIPCHK(launch_evict_read(fp, fb, S0.stream));
        HIPCHK(hipEventRecord(ev[0], S0.stream));
        HIPCHK(launch_rank_sorted_multi(desc, n, max_nblk, S0.stream));
        HIPCHK(hipEventRecord(ev[1], S0.stream));
        HIPCHK(hipEventSynchronize(ev[1]));
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, ev[0], ev[1]));
        total_ms += ms;
    }
    HIPCHK(hipEventDestroy(ev[0]));
    HIPCHK(hipEventDestroy(ev[1]));
    MemPool::get().give(MemPool::kPinnedMapped, hp, cap, S0.device);
    return total_ms * 1e3 / reps;
}

// JobInfo.FitError (job_info.go:343-372) from the histogram of the job's last walk.
string fit_error(const HJob& j) {
    if (j.fit[0] == 0) return "0 nodes are available";
    vector<string> rs;  // "%v insufficient %v", sort.Strings
    const std::pair<const char*, int32_t> rz[3] = {{"cpu", j.fit[1]}, {"memory", j.fit[2]}, {"GPU", j.fit[3]}};
    for (auto& r : rz)
        if (r.second > 0) rs.push_back(std::to_string(r.second) + " insufficient " + r.first);
    std::sort(rs.begin(), rs.end());
    string joined;
    for (size_t i = 0; i < rs.size(); ++i) joined += (i ? ", " : "") + rs[i];
    return "0/" + std::to_string(j.fit[0]) + " nodes are available, " + joined + ".";
}
// The gang plugin's OnSessionClose (plugins/gang/gang.go:166-187): the
// Unschedulable condition message of every job that is not Ready, one line
// "<job uid>\t<message>\n" per job in UID order; empty without gang.  A job
// with an IsBackfill task gets the PodGroupBackfilled condition instead, which
// has no message (gang.go:189-199): "<job uid>\tBackfilled\n".
string gang_close_text(const Session& S) {
    if (!S.gang_close) return "";
    string out;
    for (size_t i = 0; i < S.jobs.size(); ++i) {
        const HJob& j = S.jobs[i];
        if (j.cnt_alloc >= j.min_avail) continue;  // JobInfo.GetReadiness() == Ready
        int ready = 0;                              // readyTaskNum (gang.go:212-222)
        bool backfill = false;
        for (int t : j.tasks) {
            const int st = S.pods[t].status;
            ready += allocated_status(st) || st == Pipelined || st == Succeeded;
            backfill = backfill || S.pods[t].backfill;
        }
        if (backfill) {
            out += S.job_uid[i] + "\tBackfilled\n";
            continue;
        }
        out += S.job_uid[i] + "\t" + std::to_string(j.min_avail - ready) + "/" + std::to_string(j.tasks.size()) +
               " tasks in gang unschedulable: " + fit_error(j) + "\n";
    }
    return out;
}

int device_count() {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) {
        g_err = string("hipGetDeviceCount: ") + hipGetErrorString(e);
        return KBHIP_ENODEV;
    }
    int ok = 0;
    for (int i = 0; i < n; ++i) {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, i) != hipSuccess) continue;
        if (std::strncmp(prop.gcnArchName, "gfx950", 6) == 0) ok++;
    }
    return ok;
}



// kbhip_session_carry: the next scheduling session's
// start state from this one's end state, without a new snapshot — what the
// scheduler cache holds after the session's binds and evictions reached it
// (cache.go:515-583 snapshots it again):
//   dispatched (Binding) tasks  -> Bound on their node (the bind succeeded);
//   Allocated but not dispatched, Pipelined -> Pending, no node (session-only);
//   evicted (Releasing)         -> Releasing on their node (deleting pods);
//   an unevicted victim         -> Running (the node copy's Releasing is session-only);
// node rows (Idle, Releasing, Backfilled, pod count, nonzero requests, host
// ports) are recomputed from those pods — dropping the session-only
// GetAccessibleResource inflation of Idle — and only rows that changed are
// uploaded (contiguous runs); jobs, queues and plugin state are re-derived as
// at open.  Cache events of existing pods between the sessions follow
// (event_handlers.go): deletePod -> deleteTask on NewTaskInfo(pod) — a pod of
// a PodGroup leaves its job and its node; a group-less pod's TaskInfo has an
// empty Job, so it stays in its shadow job with its status and NodeName and
// only its node drops it (detached); no job is deleted — and updatePod to
// Succeeded / Failed (isTerminated: the task stays in its job, off its node).
// New pods, node and PodGroup changes: kbhip_session_carry_snapshot.
void session_carry(Session& S, const int32_t* ev_pod, const uint8_t* ev, int64_t n_ev) {
    S.model_gen++;  // per-pod caches of the host model (Session::pod_queue) are rebuilt
    // every node's row is recomputed on the host (a shard's host model holds
    // all of them); this device's rows [lo, lo + Nl) are compared and uploaded
    const int N = (int)S.h_alloc.size(), Nl = S.nc.n, lo = S.nc.base, P = (int)S.pods.size();
    {  // validate the events before anything changes
        vector<char> gone(P, 0);
        const bool aff = S.aff && S.aff->active;
        for (int64_t k = 0; k < n_ev; ++k) {
            const int32_t i = ev_pod[k];
            if (i < 0 || i >= P) throw Error(KBHIP_EINVAL, "event pod index out of range");
            if (ev[k] != KBHIP_EV_DELETE && ev[k] != KBHIP_EV_SUCCEEDED && ev[k] != KBHIP_EV_FAILED)
                throw Error(KBHIP_EINVAL, "unknown cache event");
            if (gone[i] || S.pods[i].status == Gone || S.pods[i].detached)
                throw Error(KBHIP_EINVAL, "event on a deleted pod");
            if (ev[k] == KBHIP_EV_DELETE) gone[i] = 1;
            const HPod& q = S.pods[i];
            // on a node once the carry's transitions ran (session-only Allocated / Pipelined: Pending again)
            const bool carried_on_node = q.node >= 0 && q.status != Allocated && q.status != AOB &&
                                         q.status != Pipelined && q.status != Pending && q.status != Succeeded &&
                                         q.status != Failed;
            if (aff && ev[k] == KBHIP_EV_DELETE && q.groupless && carried_on_node)
                throw Error(KBHIP_EUNSUPPORTED, "deleting a bound group-less pod (it stays in its shadow job, "
                                                "detached) in a session with pod (anti-)affinity");
        }
    }
    ov_quiesce(S);
    HIPCHK(hipStreamSynchronize(S.stream));
    for (auto& p : S.pods) {
        if (p.status == Binding) p.status = Bound;
        else if (p.status == Allocated || p.status == AOB || p.status == Pipelined) { p.status = Pending; p.node = -1; }
        else if (p.status == Pending) p.node = -1;  // an unpipelined task keeps its NodeName in the session only
        p.node_rel = false;
    }
    if (n_ev > 0) {
        vector<char> del(P, 0);
        bool any_del = false;
        for (int64_t k = 0; k < n_ev; ++k) {
            HPod& p = S.pods[ev_pod[k]];
            if (ev[k] == KBHIP_EV_DELETE) {
                // deletePod -> deleteTask on NewTaskInfo(pod) (event_handlers.go:119-165).  A pod of a
                // PodGroup leaves its job (JobInfo.DeleteTaskInfo) and its node.  A group-less pod's
                // TaskInfo has an empty Job (job_info.go:60-70): its shadow job keeps the task with
                // its status and NodeName, only the node drops it (a pending or terminated one is on
                // no node: nothing changes).  No job is ever deleted (JobTerminated needs a nil
                // PodGroup, job_info.go / event_handlers.go:165-168).
                if (p.groupless) {
                    if (on_node_of(p)) p.detached = true;
                } else {
                    p.status = Gone;
                    p.node = -1;
                    del[ev_pod[k]] = 1;
                    any_del = true;
                }
            } else {
                p.status = ev[k] == KBHIP_EV_SUCCEEDED ? Succeeded : Failed;  // keeps its NodeName
            }
        }
        if (any_del)
            for (auto& j : S.jobs) {  // JobInfo.DeleteTaskInfo
                size_t w = 0;
                for (int t : j.tasks) if (!del[t]) j.tasks[w++] = t;
                j.tasks.resize(w);
            }
    }
    vector<int64_t> col[9];
    for (auto& c : col) c.assign(N, 0);
    vector<int32_t> podcnt(N, 0);
    vector<int64_t> nzc(N, 0), nzm(N, 0);
    vector<uint64_t> pcol((size_t)std::max(S.nc.port_words, 1) * S.nc.npad, 0);  // this device's rows
    for (int n = 0; n < N; ++n) { col[0][n] = S.h_alloc[n].c; col[1][n] = S.h_alloc[n].m; col[2][n] = S.h_alloc[n].g; }
    S.used.assign(N, R3{});
    S.any_bf = 0;
    for (int i = 0; i < P; ++i) {  // cache addTask -> NodeInfo.AddTask, as at open
        const HPod& p = S.pods[i];
        if (!on_node_of(p)) continue;
        const int n = p.node;
        if (p.backfill) { col[6][n] += p.req.c; col[7][n] += p.req.m; col[8][n] += p.req.g; }
        if (p.status == Releasing) { col[3][n] += p.req.c; col[4][n] += p.req.m; col[5][n] += p.req.g; }
        col[0][n] -= p.req.c; col[1][n] -= p.req.m; col[2][n] -= p.req.g;
        S.used[n].c += p.req.c; S.used[n].m += p.req.m; S.used[n].g += p.req.g;
        podcnt[n]++;
        nzc[n] += p.nzc;
        nzm[n] += p.nzm;
        if (n < lo || n >= lo + Nl) continue;
        for (int k = S.pod_port_off[i]; k < S.pod_port_off[i + 1]; ++k) {
            const int id = S.pod_port_ids[k];
            pcol[(size_t)(id / 64) * S.nc.npad + (n - lo)] |= 1ULL << (id % 64);
        }
    }
    for (int n = 0; n < N; ++n) if (col[6][n] || col[7][n] || col[8][n]) S.any_bf = 1;
    // delta upload: read the device rows back, send only the runs that differ
    int64_t* dcol[9] = {S.nc.idle_cpu, S.nc.idle_mem, S.nc.idle_gpu, S.nc.rel_cpu, S.nc.rel_mem, S.nc.rel_gpu,
                        S.nc.bf_cpu, S.nc.bf_mem, S.nc.bf_gpu};
    int64_t uploaded = 0;
    auto sync_col = [&](void* dptr, const void* want, size_t elem) {  // want: this device's rows
        vector<uint8_t> have((size_t)Nl * elem);
        HIPCHK(hipMemcpy(have.data(), dptr, have.size(), hipMemcpyDeviceToHost));
        const uint8_t* w = (const uint8_t*)want;
        int n = 0;
        while (n < Nl) {
            if (std::memcmp(have.data() + (size_t)n * elem, w + (size_t)n * elem, elem) == 0) { ++n; continue; }
            int e = n + 1;
            while (e < Nl && std::memcmp(have.data() + (size_t)e * elem, w + (size_t)e * elem, elem) != 0) ++e;
            HIPCHK(hipMemcpyAsync((uint8_t*)dptr + (size_t)n * elem, w + (size_t)n * elem, (size_t)(e - n) * elem,
                                  hipMemcpyHostToDevice, S.stream));
            uploaded += (int64_t)(e - n) * (int64_t)elem;
            n = e;
        }
    };
    for (int k = 0; k < 9; ++k) sync_col(dcol[k], col[k].data() + lo, sizeof(int64_t));
    sync_col(S.nc.pods, podcnt.data() + lo, sizeof(int32_t));
    sync_col(S.nc.nzc, nzc.data() + lo, sizeof(int64_t));
    sync_col(S.nc.nzm, nzm.data() + lo, sizeof(int64_t));
    for (int w = 0; w < S.nc.port_words; ++w)
        sync_col(S.nc.ports + (size_t)w * S.nc.npad, pcol.data() + (size_t)w * S.nc.npad, sizeof(uint64_t));
    HIPCHK(hipStreamSynchronize(S.stream));  // the host sources above are about to go away
    S.carry_bytes = uploaded;
    // jobs, queues, plugins: as at open
    for (auto& j : S.jobs) {
        j.cnt_alloc = j.cnt_aob = 0;
        j.pending.clear();
        j.cursor = 0;
        j.pending_built = false;
        for (int q = 0; q < 4; ++q) j.fit[q] = 0;
        j.drf_alloc = F3{};
        j.drf_share = 0;
        j.priority = j.pg_priority;
        for (int t : j.tasks) {
            j.priority = S.pods[t].priority;
            if (allocated_status(S.pods[t].status)) j.cnt_alloc++;
        }
    }
    for (auto& q : S.queues) {
        q.has_attr = false;
        q.deserved = q.allocated = q.request = F3{};
        q.share = 0;
    }
    // pod (anti)-affinity count tables of the carried pod states (the term
    // classes and programs do not depend on statuses; their counts do)
    S.tab_delta.clear();
    if (S.aff && S.aff->active) {
        vector<AffPod> ap(P);
        for (int i = 0; i < P; ++i) {
            const HPod& p = S.pods[i];
            AffPod& a = ap[i];
            a.ns = p.ns;
            a.status = p.status;
            a.session_job = p.job >= 0;
            const bool on_node = on_node_of(p);
            a.node = on_node ? p.node : -1;
            a.target = a.session_job && allocated_status(p.status) && on_node;
            a.pending = a.session_job && p.status == Pending;
        }
        S.aff->recount(ap);
        HIPCHK(hipMemcpyAsync(S.tab.aff_cnt, S.aff->cnt.data(), S.aff->cnt.size() * sizeof(int32_t),
                              hipMemcpyHostToDevice, S.stream));
        HIPCHK(hipMemcpyAsync(S.tab.aff_scalar, S.aff->scalar.data(), S.aff->scalar.size() * sizeof(int32_t),
                              hipMemcpyHostToDevice, S.stream));
        HIPCHK(hipStreamSynchronize(S.stream));
        S.carry_bytes += (int64_t)(S.aff->cnt.size() + S.aff->scalar.size()) * (int64_t)sizeof(int32_t);
    }
    S.plugins_opened = false;
    S.fallback = -1;
    S.sess_cnt.clear();
    S.node_tasks.clear();
    S.log.clear();
    S.last_fit_ok = false;
}

}  // namespace kbhip

using namespace kbhip;

extern "C" {

const char* kbhip_last_error(void) { return kbhip::g_err.c_str(); }


int kbhip_device_count(void) { ABI_GUARD(return kbhip::device_count();) }

// Arguments of the actions that return a record log: a device session and,
// when cap > 0, three output arrays of at least cap entries.

static int open_common(const kbs::Snapshot& snap, int device, kb_session** out) {
    int nd = kbhip::device_count();
    if (nd <= 0) throw kbhip::Error(KBHIP_ENODEV, "no gfx950 HIP device available");
    if (device < 0 || device >= nd) throw kbhip::Error(KBHIP_EINVAL, "device index out of range");
    std::unique_ptr<kb_session> s(new kb_session());
    kbhip::open_session(s->s, snap, device);
    *out = s.release();
    return KBHIP_OK;
}

int kbhip_session_open(const void* bytes, size_t len, int device, kb_session** out) {
    ABI_GUARD({
        if (!bytes || !out) throw kbhip::Error(KBHIP_EINVAL, "null argument");
        kbs::Snapshot snap;
        snap.view_bytes(bytes, len);  // the caller's buffer outlives the call; nothing keeps a view after it
        return open_common(snap, device, out);
    })
}

int kbhip_session_open_file(const char* path, int device, kb_session** out) {
    ABI_GUARD({
        if (!path || !out) throw kbhip::Error(KBHIP_EINVAL, "null argument");
        kbs::Snapshot snap(path);
        return open_common(snap, device, out);
    })
}

int kbhip_place_job(kb_session* s, const int32_t* task_ids, int32_t n_tasks, int32_t gang_mode, int32_t min_available,
                    int32_t ready_count, int32_t* out_node, uint8_t* out_kind, int32_t* out_n_done,
                    int32_t* out_stop_reason) {
    ABI_GUARD_S(s, {
        if (!s || (!task_ids && n_tasks) || !out_node || !out_kind || !out_n_done || !out_stop_reason)
            throw kbhip::Error(KBHIP_EINVAL, "null argument");
        if (s->s.encode_only) throw kbhip::Error(KBHIP_EINVAL, "encode-only session has no device state");
        kbhip::require_no_tickets(s->s);
        HIPCHK(hipSetDevice(s->s.device));
        // results come back through the pinned result granules; device work still in flight (an
        // overlapped pop's write-back) is ordered before the next pop by the device chain, and
        // before anything else by ov_quiesce in the entry point that runs it
        return kbhip::place_job(s->s, task_ids, n_tasks, gang_mode, min_available, ready_count, out_node, out_kind,
                                out_n_done, out_stop_reason);
    })
}

int64_t kbhip_place_job_submit(kb_session* s, const int32_t* task_ids, int32_t n_tasks, int32_t gang_mode,
                               int32_t min_available, int32_t ready_count) {
    ABI_GUARD_S(s, {
        if (!s || (!task_ids && n_tasks) || n_tasks < 0) throw kbhip::Error(KBHIP_EINVAL, "null argument");
        if (s->s.encode_only) throw kbhip::Error(KBHIP_EINVAL, "encode-only session has no device state");
        // a shard's launch would block inside the exchange, and a retraction needs every rank to cancel
        // identically: node-sharded sessions use the synchronous kbhip_place_job
        if (s->s.world > 1)
            throw kbhip::Error(KBHIP_EUNSUPPORTED, "kbhip_place_job_submit on a node-sharded session (use kbhip_place_job)");
        HIPCHK(hipSetDevice(s->s.device));
        return kbhip::place_job_submit(s->s, task_ids, n_tasks, gang_mode, min_available, ready_count);
    })
}

int kbhip_place_job_wait(kb_session* s, int64_t ticket, int32_t* out_node, uint8_t* out_kind, int32_t* out_n_done,
                         int32_t* out_stop_reason) {
    ABI_GUARD_S(s, {
        if (!s || !out_node || !out_kind || !out_n_done || !out_stop_reason)
            throw kbhip::Error(KBHIP_EINVAL, "null argument");
        HIPCHK(hipSetDevice(s->s.device));
        return kbhip::place_job_wait(s->s, ticket, out_node, out_kind, out_n_done, out_stop_reason);
    })
}

int kbhip_place_job_cancel(kb_session* s, int64_t ticket) {
    ABI_GUARD_S(s, {
        if (!s) throw kbhip::Error(KBHIP_EINVAL, "null argument");
        HIPCHK(hipSetDevice(s->s.device));
        return kbhip::place_job_cancel(s->s, ticket);
    })
}

int kbhip_allocate(kb_session* s, int32_t* out_pod, int32_t* out_node, uint8_t* out_kind, int64_t cap) {
    ABI_GUARD_S(s, {
        check_log_args(s, out_pod, out_node, out_kind, cap);
        kbhip::require_no_tickets(s->s);
        HIPCHK(hipSetDevice(s->s.device));
        s->s.log.clear();
        kbhip::allocate_run(s->s);
        const int64_t n = (int64_t)s->s.log.size();
        for (int64_t i = 0; i < n && i < cap; ++i) {
            out_pod[i] = std::get<0>(s->s.log[i]);
            out_node[i] = std::get<1>(s->s.log[i]);
            out_kind[i] = (uint8_t)std::get<2>(s->s.log[i]);
        }
        return (int)n;
    })
}

int kbhip_backfill(kb_session* s, int32_t* out_pod, int32_t* out_node, uint8_t* out_kind, int64_t cap) {
    ABI_GUARD_S(s, {
        check_log_args(s, out_pod, out_node, out_kind, cap);
        kbhip::require_no_tickets(s->s);
        HIPCHK(hipSetDevice(s->s.device));
        kbhip::ov_quiesce(s->s);
        s->s.log.clear();
        kbhip::backfill_run(s->s);
        const int64_t n = (int64_t)s->s.log.size();
        for (int64_t i = 0; i < n && i < cap; ++i) {
            out_pod[i] = std::get<0>(s->s.log[i]);
            out_node[i] = std::get<1>(s->s.log[i]);
            out_kind[i] = (uint8_t)std::get<2>(s->s.log[i]);
        }
        return (int)n;
    })
}

int kbhip_first_fit(kb_session* s, const int32_t* task_ids, int32_t n, int32_t* out_node) {
    ABI_GUARD_S(s, {
        if (!s || n < 0 || (n > 0 && (!task_ids || !out_node))) throw kbhip::Error(KBHIP_EINVAL, "null argument");
        if (s->s.encode_only) throw kbhip::Error(KBHIP_EINVAL, "encode-only session has no device state");
        kbhip::require_no_tickets(s->s);
        HIPCHK(hipSetDevice(s->s.device));
        s->s.log.clear();
        kbhip::first_fit(s->s, task_ids, n, out_node);
        int placed = 0;
        for (int i = 0; i < n; ++i) placed += out_node[i] >= 0;
        return placed;
    })
}

int kbhip_time_sweeps(kb_session* s, const int32_t* task_ids, int32_t n, double* out_mean_us) {
    ABI_GUARD_S(s, {
        if (!s || (!task_ids && n) || n < 0 || !out_mean_us) throw kbhip::Error(KBHIP_EINVAL, "null argument");
        if (s->s.encode_only) throw kbhip::Error(KBHIP_EINVAL, "encode-only session has no device state");
        kbhip::require_no_tickets(s->s);
        HIPCHK(hipSetDevice(s->s.device));
        *out_mean_us = kbhip::time_sweeps(s->s, task_ids, n);
        return KBHIP_OK;
    })
}

int kbhip_time_rank_multi(kb_session* const* sessions, int32_t n, const int32_t* task_ids, int32_t reps,
                          int32_t evict, int32_t mapped, double* out_us) {
    ABI_GUARD({
        if (!sessions || !task_ids || n < 1 || n > 4096 || !out_us) throw kbhip::Error(KBHIP_EINVAL, "null argument");
        vector<kbhip::Session*> ss(n);
        for (int i = 0; i < n; ++i) {
            if (!sessions[i]) throw kbhip::Error(KBHIP_EINVAL, "null session");
            check_usable(sessions[i]);
            kbhip::require_no_tickets(sessions[i]->s);
            ss[i] = &sessions[i]->s;
        }
        HIPCHK(hipSetDevice(ss[0]->device));
        *out_us = kbhip::time_rank_multi(ss.data(), n, task_ids, reps, evict, mapped);
        return KBHIP_OK;
    })
}


int kbhip_sweep_scores(kb_session* s, int32_t task_id, uint64_t* out_keys) {
    ABI_GUARD_S(s, {
        if (!s) throw kbhip::Error(KBHIP_EINVAL, "null session");
        if (s->s.encode_only) throw kbhip::Error(KBHIP_EINVAL, "encode-only session has no device state");
        kbhip::require_no_tickets(s->s);
        HIPCHK(hipSetDevice(s->s.device));
        return kbhip::sweep_scores(s->s, task_id, out_keys);
    })
}

}  // extern "C"
