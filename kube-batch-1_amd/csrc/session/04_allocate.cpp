// kbhip session, part 04: the allocate / reclaim / preempt actions and the ordering plugins (C++ mirror)
#include "session.h"

namespace kbhip {

// ---------------------------------------------------------------------------
// allocate action with the Go framework's ordering (host mirror)
// ---------------------------------------------------------------------------
// Undo log of speculative heap operations: (heap items, position, old value);
// position -1 records the old size.
struct HeapJournal {
    bool on = false;
    struct Entry {
        vector<int>* v;
        int pos, val;
    };
    vector<Entry> e;
    void rollback() {
        for (auto it = e.rbegin(); it != e.rend(); ++it) {
            if (it->pos < 0) it->v->resize(it->val);
            else (*it->v)[it->pos] = it->val;
        }
        e.clear();
    }
};

template <typename L>
struct GoHeap {  // Go container/heap (up/down exactly as heap.go), with an optional undo log
    vector<int> items;
    L less;
    HeapJournal* jr = nullptr;
    explicit GoHeap(L l) : less(l) {}
    bool Less(int i, int j) { return less(items[i], items[j]); }
    void swap_at(int i, int j) {
        if (jr && jr->on) {
            jr->e.push_back({&items, i, items[i]});
            jr->e.push_back({&items, j, items[j]});
        }
        std::swap(items[i], items[j]);
    }
    void up(int j) {
        for (;;) {
            int i = (j - 1) / 2;
            if (i == j || !Less(j, i)) break;
            swap_at(i, j);
            j = i;
        }
    }
    void down(int i, int n) {
        for (;;) {
            int j1 = 2 * i + 1;
            if (j1 >= n || j1 < 0) break;
            int j = j1, j2 = j1 + 1;
            if (j2 < n && Less(j2, j1)) j = j2;
            if (!Less(j, i)) break;
            swap_at(i, j);
            i = j;
        }
    }
    void push(int x) {
        if (jr && jr->on) jr->e.push_back({&items, -1, (int)items.size()});
        items.push_back(x);
        up((int)items.size() - 1);
    }
    int pop() {
        int n = (int)items.size() - 1;
        swap_at(0, n);
        down(0, n);
        int x = items.back();
        if (jr && jr->on) {  // rolled back in reverse: size first, then the slot
            jr->e.push_back({&items, n, x});
            jr->e.push_back({&items, -1, n + 1});
        }
        items.pop_back();
        return x;
    }
    bool empty() const { return items.empty(); }
};

// A queue's job heap in allocate (allocate.go:48-63, 87): a job's order key
// (priority, gang readiness, DRF share, creation time, UID) changes only
// while the job is popped, so the heap never holds a stale key and pops in
// exact key order (a strict total order) whatever its layout.  Jobs with no
// pending task when the action starts are never pushed back and never change
// key: they wait in a list sorted by key, and a pop takes the smaller of its
// head and the heap's top.  Only the jobs with pending tasks pay heap work
// (C5: ~180k running jobs, a few hundred pending ones).
template <typename L>
struct JobQueue {
    GoHeap<L> heap;
    vector<int> idle;       // jobs without pending tasks, ascending key
    vector<int> head{0};    // next idle job (a vector: the speculation journal restores it)
    L less;
    explicit JobQueue(L l) : heap(l), less(l) {}
    void set_journal(HeapJournal* jr) { heap.jr = jr; }
    void push(int x) { heap.push(x); }
    bool empty() const { return head[0] >= (int)idle.size() && heap.empty(); }
    int pop() {
        const int h = head[0];
        if (h < (int)idle.size() && (heap.empty() || less(idle[h], heap.items[0]))) {
            if (heap.jr && heap.jr->on) heap.jr->e.push_back({&head, 0, h});
            head[0] = h + 1;
            return idle[h];
        }
        return heap.pop();
    }
};

// The node-ranking buffers of a session (keys, sorted keys, histogram,
// counters, the host copy), allocated on its first ranking.
void rank_buffers(Session& S) {
    if (S.b_rank_sorted.p) return;
    const int N = S.nc.n;
    S.b_rank_keys.alloc<uint64_t>(N);
    S.b_rank_sorted.alloc<uint64_t>(N);
    S.b_rank_cnt.alloc<uint32_t>(4);
    S.rank_tmp_bytes = std::max<size_t>((size_t)16, rank_hist_words(N) * sizeof(uint32_t));
    S.b_rank_tmp.alloc<uint8_t>(S.rank_tmp_bytes);
    S.b_rank_radix.alloc<uint64_t>(std::max(N, 1));
    S.h_rank = (uint64_t*)MemPool::get().take(MemPool::kPinned, (size_t)(N + 1) * sizeof(uint64_t), &S.h_rank_cap);
}

struct Allocator {
    Session& S;
    explicit Allocator(Session& s) : S(s) {}

    int readiness(const HJob& j) const {  // job_info.go:374-388
        if (j.cnt_alloc >= j.min_avail) return 1;
        if (j.cnt_alloc + j.cnt_aob >= j.min_avail) return 2;
        return 4;
    }
    bool job_ready(const HJob& j) const { return !S.gang_ready || readiness(j) == 1; }  // session_plugins.go:167-186
    // tier dispatch compiled once: enabled order functions in tier order
    // (session_plugins.go:244-329); codes 1 priority, 2 gang, 3 drf
    vector<int> job_order;
    bool queue_prop = false, task_prio = false;
    void compile_orders() {
        for (auto& tier : S.tiers)
            for (auto& p : tier) {
                if (!(p.flags & KBS_DIS_JOBORDER)) {
                    if (p.name == "priority") job_order.push_back(1);
                    else if (p.name == "gang") job_order.push_back(2);
                    else if (p.name == "drf") job_order.push_back(3);
                }
                if (!(p.flags & KBS_DIS_QUEUEORDER) && p.name == "proportion") queue_prop = true;
                if (!(p.flags & KBS_DIS_TASKORDER) && p.name == "priority") task_prio = true;
            }
    }
    bool job_less(int l, int r) const {  // session_plugins.go:244-268
        if (l == r) return false;
        const HJob &L = S.jobs[l], &R = S.jobs[r];
        for (int code : job_order) {
            int c;
            if (code == 1) c = L.priority > R.priority ? -1 : L.priority < R.priority ? 1 : 0;  // priority.go:60-76
            else if (code == 2) {  // gang.go:136-160
                bool lr = readiness(L) == 1, rr = readiness(R) == 1;
                c = (lr && rr) ? 0 : lr ? 1 : rr ? -1 : 0;
            } else c = L.drf_share == R.drf_share ? 0 : L.drf_share < R.drf_share ? -1 : 1;  // drf.go:113-129
            if (c != 0) return c < 0;
        }
        if (L.ts == R.ts) return l < r;  // UID order: jobs are numbered in UID order at open
        return L.ts < R.ts;
    }
    // jobs in job_less order, sorted on compact keys: job_less's comparisons in
    // turn as unsigned digits (priority descending, gang-ready last, DRF share
    // ascending — non-negative doubles order as their bits — creation time),
    // then the job index (UID order)
    void sort_jobs(vector<int>& v) const {
        struct K {
            uint64_t d[3];
            int64_t ts;
            int j;
        };
        const int nd = (int)job_order.size();
        bool neg = false;  // (DRF shares are sums of requests over totals: never negative)
        for (int j : v) neg = neg || S.jobs[j].drf_share < 0;
        if (nd > 3 || neg) {  // more order codes than digits (repeated plugins): the comparator itself
            std::sort(v.begin(), v.end(), [this](int a, int b) { return job_less(a, b); });
            return;
        }
        vector<K> k(v.size());
        auto keys = [&](size_t lo, size_t hi) {
            for (size_t i = lo; i < hi; ++i) {
                const HJob& J = S.jobs[v[i]];
                K& x = k[i];
                for (int c = 0; c < nd; ++c) {
                    const int code = job_order[c];
                    if (code == 1) x.d[c] = (uint64_t)((int64_t)INT32_MAX - (int64_t)J.priority);
                    else if (code == 2) x.d[c] = readiness(J) == 1 ? 1 : 0;
                    else {
                        uint64_t b = 0;
                        if (J.drf_share != 0) std::memcpy(&b, &J.drf_share, 8);
                        x.d[c] = b;
                    }
                }
                x.ts = J.ts;
                x.j = v[i];
            }
        };
        auto lt = [nd](const K& a, const K& b) {
            for (int c = 0; c < nd; ++c)
                if (a.d[c] != b.d[c]) return a.d[c] < b.d[c];
            if (a.ts != b.ts) return a.ts < b.ts;
            return a.j < b.j;
        };
        const size_t n = k.size();
        if (n < (1u << 14)) {
            keys(0, n);
            std::sort(k.begin(), k.end(), lt);
        } else {  // C4 / C5: 10 k - 180 k jobs without pending tasks: 8 runs keyed and sorted in parallel,
                  // merged pairwise (each level's merges in parallel)
            constexpr int kRuns = 8;
            vector<size_t> cut(kRuns + 1);
            for (int r = 0; r <= kRuns; ++r) cut[r] = n * r / kRuns;
            auto par = [](int cnt, auto&& fn) {
                vector<std::thread> th;
                for (int r = 1; r < cnt; ++r) th.emplace_back(fn, r);
                fn(0);
                for (auto& x : th) x.join();
            };
            par(kRuns, [&](int r) {
                keys(cut[r], cut[r + 1]);
                std::sort(k.begin() + cut[r], k.begin() + cut[r + 1], lt);
            });
            for (int w = 1; w < kRuns; w *= 2)  // the keys are distinct (job index last): a strict order
                par(kRuns / (2 * w), [&, w](int i) {
                    const int r = 2 * w * i;
                    std::inplace_merge(k.begin() + cut[r], k.begin() + cut[r + w],
                                       k.begin() + cut[std::min(r + 2 * w, kRuns)], lt);
                });
        }
        for (size_t i = 0; i < v.size(); ++i) v[i] = k[i].j;
    }
    bool queue_less(int l, int r) const {  // session_plugins.go:270-295, proportion.go:144-157
        if (l == r) return false;  // copies of one queue (one heap entry per job) are equal
        const HQueue &L = S.queues[l], &R = S.queues[r];
        if (queue_prop && L.share != R.share) return L.share < R.share;
        if (L.ts == R.ts) return L.rank < R.rank;
        return L.ts < R.ts;
    }
    bool task_less(int l, int r) const {  // session_plugins.go:297-329, priority.go:39-55
        const HPod &L = S.pods[l], &R = S.pods[r];
        if (task_prio && L.priority != R.priority) return L.priority > R.priority;
        if (L.ts == R.ts) return L.uid_rank < R.uid_rank;
        return L.ts < R.ts;
    }
    void drf_update(HJob& j) {  // drf.go:156-170
        double res = 0;
        for (int k = 0; k < 3; ++k) { double x = share(j.drf_alloc.get(k), S.total.get(k)); if (x > res) res = x; }
        j.drf_share = res;
    }
    void prop_update(HQueue& q) {  // proportion.go:229-241
        double res = 0;
        for (int k = 0; k < 3; ++k) { double x = share(q.allocated.get(k), q.deserved.get(k)); if (x > res) res = x; }
        q.share = res;
    }
    void open_plugins() {
        if (S.plugins_opened) return;
        S.plugins_opened = true;
        if (S.drf_on) {  // drf.go:65-82 (each job's sum over its own tasks, in order: job ranges in parallel)
            const int J = (int)S.jobs.size();
            const int nth = J < (1 << 14) ? 1 : host_threads();
            auto drf = [&](int t) {
                for (int jb = (int)((int64_t)J * t / nth); jb < (int)((int64_t)J * (t + 1) / nth); ++jb) {
                    HJob& j = S.jobs[jb];
                    for (int k : j.tasks) if (allocated_status(S.pods[k].status)) j.drf_alloc.add(S.pods[k].req);
                    drf_update(j);
                }
            };
            vector<std::thread> th;
            for (int t = 1; t < nth; ++t) th.emplace_back(drf, t);
            drf(0);
            for (auto& x : th) x.join();
        }
        if (S.prop_on) {  // proportion.go:65-142
            // each queue's sums in job and task order (floating point: the order is kept), queues
            // split over the threads — or, when prop_sums_exact finds every addend and every
            // total a non-negative integer below 2^53, job ranges in parallel
            const int NQ = (int)S.queues.size();
            const int nth = S.pods.size() < (1u << 16) ? 1 : std::min(NQ, host_threads());
            auto prop = [&](int t) {
                for (auto& j : S.jobs) {
                    if (j.queue % nth != t) continue;
                    HQueue& q = S.queues[j.queue];
                    q.has_attr = true;
                    for (int k : j.tasks) {
                        const HPod& p = S.pods[k];
                        if (allocated_status(p.status)) { q.allocated.add(p.req); q.request.add(p.req); }
                        else if (p.status == Pending) q.request.add(p.req);
                    }
                }
            };
            if (!(S.pods.size() >= (1u << 16) && prop_sums_exact())) {
                vector<std::thread> th;
                for (int t = 1; t < nth; ++t) th.emplace_back(prop, t);
                if (nth > 0) prop(0);
                for (auto& x : th) x.join();
            }
            vector<int> order;
            for (size_t i = 0; i < S.queues.size(); ++i) if (S.queues[i].has_attr) order.push_back((int)i);
            F3 remaining = S.total;
            vector<char> meet(S.queues.size(), 0);
            for (;;) {
                int32_t tw = 0;
                for (int q : order) if (!meet[q]) tw += S.queues[q].weight;
                if (tw == 0) break;
                F3 deserved;
                for (int qi : order) {
                    if (meet[qi]) continue;
                    HQueue& q = S.queues[qi];
                    const double ratio = (double)q.weight / (double)tw;
                    F3 r = remaining;
                    r.c *= ratio; r.m *= ratio; r.g *= ratio;
                    q.deserved.addf(r);
                    if (!q.deserved.less_equal(q.request)) {  // helpers.Min
                        q.deserved.c = std::fmin(q.deserved.c, q.request.c);
                        q.deserved.g = std::fmin(q.deserved.g, q.request.g);
                        q.deserved.m = std::fmin(q.deserved.m, q.request.m);
                        meet[qi] = 1;
                    }
                    prop_update(q);
                    deserved.addf(q.deserved);
                }
                remaining.subf(deserved);
                if (remaining.empty()) break;
            }
        }
    }
    // proportion's queue sums (proportion.go:88-103) over job ranges in parallel. A float64 sum
    // of non-negative integers whose total stays below 2^53 is exact in any order (every
    // partial sum is an integer no larger than the total), so it equals the in-order sum; the
    // queues are written only when every addend, start value and total meets that.
    bool prop_sums_exact() {
        constexpr int64_t kLim = int64_t(1) << 53;
        const int NQ = (int)S.queues.size(), J = (int)S.jobs.size();
        const int nth = std::max(1, std::min(host_threads(), J / 256));
        vector<vector<int64_t>> acc(nth, vector<int64_t>(6 * (size_t)NQ, 0));
        vector<vector<uint8_t>> has(nth, vector<uint8_t>(NQ, 0));
        vector<uint8_t> ok(nth, 1);
        run_ranges(nth, [&](int t) {
            int64_t* a = acc[t].data();
            auto put = [&](int64_t* s, const R3& r) {
                if ((uint64_t)r.c >= (uint64_t)kLim || (uint64_t)r.m >= (uint64_t)kLim ||
                    (uint64_t)r.g >= (uint64_t)kLim)
                    return false;  // negative or too large
                s[0] += r.c; s[1] += r.m; s[2] += r.g;
                return s[0] < kLim && s[1] < kLim && s[2] < kLim;
            };
            for (int jb = (int)((int64_t)J * t / nth); jb < (int)((int64_t)J * (t + 1) / nth); ++jb) {
                const HJob& j = S.jobs[jb];
                has[t][j.queue] = 1;
                int64_t* qa = a + 6 * (size_t)j.queue;
                for (int k : j.tasks) {
                    const HPod& p = S.pods[k];
                    bool good = true;
                    if (allocated_status(p.status)) good = put(qa, p.req) && put(qa + 3, p.req);
                    else if (p.status == Pending) good = put(qa + 3, p.req);
                    if (!good) { ok[t] = 0; return; }
                }
            }
        });
        for (int t = 0; t < nth; ++t) if (!ok[t]) return false;
        vector<double> out(6 * (size_t)NQ);
        for (int q = 0; q < NQ; ++q) {
            const HQueue& Q = S.queues[q];
            const double x0[6] = {Q.allocated.c, Q.allocated.m, Q.allocated.g, Q.request.c, Q.request.m, Q.request.g};
            for (int k = 0; k < 6; ++k) {
                if (!(x0[k] >= 0 && x0[k] < (double)kLim && x0[k] == std::floor(x0[k]))) return false;
                int64_t s = (int64_t)x0[k];
                for (int t = 0; t < nth; ++t) s += acc[t][6 * (size_t)q + k];  // each < 2^53: no overflow
                if (s >= kLim) return false;
                out[6 * (size_t)q + k] = (double)s;
            }
        }
        for (int q = 0; q < NQ; ++q) {
            HQueue& Q = S.queues[q];
            const double* o = &out[6 * (size_t)q];
            Q.allocated.c = o[0]; Q.allocated.m = o[1]; Q.allocated.g = o[2];
            Q.request.c = o[3]; Q.request.m = o[4]; Q.request.g = o[5];
            for (int t = 0; t < nth; ++t) if (has[t][q]) Q.has_attr = true;
        }
        return true;
    }
    bool overused(int qi) const {  // proportion.go:186-197
        if (!S.prop_on) return false;
        return S.queues[qi].deserved.less_equal(S.queues[qi].allocated);
    }
    void on_allocate(int pi) {  // event handlers drf.go:134-143, proportion.go:200-210
        const HPod& p = S.pods[pi];
        HJob& j = S.jobs[p.job];
        if (S.drf_on) { j.drf_alloc.add(p.req); drf_update(j); }
        if (S.prop_on) { HQueue& q = S.queues[j.queue]; q.allocated.add(p.req); prop_update(q); }
    }

    void run() {  // allocate.go:41-201
        auto t0 = std::chrono::steady_clock::now();
        // KBHIP_OPEN_PROFILE=1: the setup's phases on stderr (diagnostic)
        static const bool prof = std::getenv("KBHIP_OPEN_PROFILE") != nullptr;
        auto tp = t0;
        auto mark = [&](const char* what) {
            if (!prof) return;
            auto now = std::chrono::steady_clock::now();
            std::fprintf(stderr, "[alloc] %-10s %8.2f ms\n", what, std::chrono::duration<double>(now - tp).count() * 1e3);
            tp = now;
        };
        compile_orders();
        open_plugins();
        mark("plugins");
        auto ql = [this](int a, int b) { return queue_less(a, b); };
        auto jl = [this](int a, int b) { return job_less(a, b); };
        GoHeap<decltype(ql)> queues(ql);
        std::map<int, JobQueue<decltype(jl)>> jobs_map;
        // allocate.go:91-104: a job has work if it holds a pending task that is not BestEffort
        // (its task lists scanned over job ranges in parallel; the pushes below stay in order)
        const int NJ = (int)S.jobs.size();
        vector<uint8_t> has_work(NJ, 0);
        const int nth_w = NJ < (1 << 14) ? 1 : host_threads();
        run_ranges(nth_w, [&, NJ, nth_w](int r) {
            const int nth = nth_w;
            for (int j = (int)((int64_t)NJ * r / nth); j < (int)((int64_t)NJ * (r + 1) / nth); ++j) {
                const HJob& job = S.jobs[j];
                bool work = false;
                if (job.pending_built) work = job.cursor < job.pending.size();
                else if (job.maybe_pending)
                    for (int t : job.tasks) {
                        const HPod& p = S.pods[t];
                        if (p.status == Pending && !(p.req.c < kMinCPU && p.req.m < kMinMem && p.req.g < kMinGPU)) {
                            work = true;
                            break;
                        }
                    }
                has_work[j] = work;
            }
        });
        for (size_t j = 0; j < S.jobs.size(); ++j) {
            const HJob& job = S.jobs[j];
            int q = job.queue;
            // one queue copy per job, as allocate.go pushes them: a queue's share changes while
            // its other copies sit in the heap, so the Go heap's layout — which the copies of
            // jobs without pending tasks shape too — decides later pops (exactness needs them)
            queues.push(q);
            auto it = jobs_map.find(q);
            if (it == jobs_map.end()) it = jobs_map.emplace(q, JobQueue<decltype(jl)>(jl)).first;
            if (has_work[j]) {
                it->second.push((int)j);
            } else {
                it->second.idle.push_back((int)j);
                S.jobs[j].pending_built = true;  // what build_pending would find: nothing
            }
        }
        mark("heaps");
        for (auto& kv : jobs_map) sort_jobs(kv.second.idle);
        mark("idle");
        vector<int32_t> ids, onode;
        vector<uint8_t> okind;
        const int gm = S.gang_ready ? 1 : 0;
        if (!S.ev_run[0]) { HIPCHK(hipEventCreate(&S.ev_run[0])); HIPCHK(hipEventCreate(&S.ev_run[1])); }
        ov_quiesce(S);
        mark("quiesce");
        S.stats.alloc_setup_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        HIPCHK(hipEventRecord(S.ev_run[0], S.stream));
        auto build_pending = [&](HJob& job) {  // allocate.go:91-104; TaskOrderFn is a strict total order
            if (job.pending_built) return;
            for (int t : job.tasks) {
                const HPod& p = S.pods[t];
                if (p.status != Pending) continue;
                if (p.req.c < kMinCPU && p.req.m < kMinMem && p.req.g < kMinGPU) continue;  // BestEffort
                job.pending.push_back(t);
            }
            std::sort(job.pending.begin(), job.pending.end(), [this](int a, int b) { return task_less(a, b); });
            job.pending_built = true;
        };

        // Speculation: while a batched pop runs, the host
        // predicts the next pops — assuming each places its tasks as Allocated
        // up to the gang stop — by running the loop below on its own state with
        // every change undone afterwards (heap operations through a journal,
        // job / queue fields saved), and queues those pops' launches behind the
        // running one.  The next real pop uses the oldest queued launch only if
        // it is exactly that pop (job, first task, ready count, class, chunk),
        // in which case the launch ran on exactly the device state the real pop
        // sees; otherwise every queued launch is retracted (k_undo_pop) before
        // anything else runs.
        struct Spec {
            BatchLaunch L;
            int jb = -1;
            size_t cursor = 0;
            int ready = 0;
        };
        std::deque<Spec> specs;  // launched predictions, oldest first
        HeapJournal journal;
        queues.jr = &journal;
        for (auto& kv : jobs_map) kv.second.set_journal(&journal);
        struct JobSave {
            int jb, cnt;
            size_t cur;
            F3 drf;
            double share;
        };
        struct QueueSave {
            int q;
            F3 alloc;
            double share;
        };
        vector<JobSave> job_saves;
        vector<QueueSave> queue_saves;
        auto discard_all = [&]() {
            if (specs.empty()) return;
            vector<int32_t> node(specs.size() * kMaxChunk), kind(specs.size() * kMaxChunk);
            vector<int> nd(specs.size());
            for (size_t i = 0; i < specs.size(); ++i) {
                int st = 0;
                collect_batched(S, specs[i].L, &nd[i], &st, node.data() + i * kMaxChunk, kind.data() + i * kMaxChunk);
            }
            ov_quiesce(S);
            for (size_t i = 0; i < specs.size(); ++i) {  // inverse updates commute
                HIPCHK(launch_undo_pop(S.nc, S.tab, specs[i].L.cls, nd[i], node.data() + i * kMaxChunk,
                                       kind.data() + i * kMaxChunk, S.stream));
                S.stats.spec_missed++;
            }
            if (S.overlap > 0) HIPCHK(hipStreamSynchronize(S.stream));  // overlapped pops are not ordered after it
            specs.clear();
        };
        // The predicted outcome of pop (q, jb) whose first chunk of m of its n
        // remaining tasks runs: k tasks Allocated, then the stop; -1 if the pop
        // would continue past this chunk.  Saves what it changes.
        auto apply_outcome = [&](int q, int jb, int m, int n) -> int {
            HJob& job = S.jobs[jb];
            int k, pstop;
            if (S.gang_ready) {  // gang.go:63-66: stop once #AllocatedStatuses >= MinAvailable
                const int need = job.min_avail - job.cnt_alloc;
                k = need <= 1 ? 1 : need;
                if (k <= m) pstop = KBHIP_STOP_READY;
                else if (m == n) { k = m; pstop = KBHIP_STOP_ALL; }
                else return -1;
            } else {
                k = 1;  // no JobReadyFn: always ready, one task per pop
                pstop = KBHIP_STOP_READY;
            }
            HQueue& Q = S.queues[q];
            job_saves.push_back({jb, job.cnt_alloc, job.cursor, job.drf_alloc, job.drf_share});
            queue_saves.push_back({q, Q.allocated, Q.share});
            for (int i = 0; i < k; ++i) {
                const HPod& p = S.pods[job.pending[job.cursor + i]];
                if (S.drf_on) job.drf_alloc.add(p.req);
                if (S.prop_on) Q.allocated.add(p.req);
            }
            job.cnt_alloc += k;
            job.cursor += k;
            if (S.drf_on) drf_update(job);
            if (S.prop_on) prop_update(Q);
            return pstop;
        };
        constexpr int kPredictSkip = 64;
        struct Pred {
            int q = -1, jb = -1, cls = -1, m = 0, n = 0, ready = 0;
            size_t cur = 0;
        };
        // The loop's next pop after pop (q, jb) stopped with pstop (heaps
        // changed through the journal); false when it is not a batched pop.
        // The loop's steps that place nothing (an overused queue or one without
        // jobs is dropped, a job without pending tasks is dropped and its queue
        // pushed back) are followed, up to kPredictSkip of them.
        auto next_pop = [&](int q, int jb, int pstop, Pred* P) -> bool {
            if (pstop == KBHIP_STOP_READY) jobs_map.at(q).push(jb);
            queues.push(q);
            for (int skip = 0; skip <= kPredictSkip && !queues.empty(); ++skip) {
                const int q2 = queues.pop();
                if (overused(q2)) continue;
                auto jit2 = jobs_map.find(q2);
                if (jit2 == jobs_map.end() || jit2->second.empty()) continue;
                const int jb2 = jit2->second.pop();
                HJob& j2 = S.jobs[jb2];
                build_pending(j2);
                const size_t cur2 = j2.cursor;
                if (cur2 >= j2.pending.size()) {  // an empty pop
                    queues.push(q2);
                    continue;
                }
                const int cls2 = S.pods[j2.pending[cur2]].cls;
                const size_t rem = j2.pending.size() - cur2;
                int m2 = 0;
                while ((size_t)m2 < rem && m2 < kMaxChunk && S.pods[j2.pending[cur2 + m2]].cls == cls2) ++m2;
                if (!batchable(S, cls2)) return false;
                *P = Pred{q2, jb2, cls2, m2, (int)rem, j2.cnt_alloc, cur2};
                return true;
            }
            return false;
        };
        auto launch_pred = [&](const Pred& p) {
            Spec sp;
            sp.L = launch_batched(S, p.cls, p.m, gm, S.jobs[p.jb].min_avail, p.ready);
            sp.jb = p.jb;
            sp.cursor = p.cur;
            sp.ready = p.ready;
            specs.push_back(sp);
        };
        // Keep up to S.speculate predicted pops queued behind pop (q, jb).
        auto speculate = [&](int q, int jb, int m, int n) {
            Pred p[kMaxSpeculate];
            int got = 0;
            journal.on = true;
            for (int cq = q, cjb = jb, cm = m, cn = n; got < S.speculate && got < kMaxSpeculate;) {
                const int ps = apply_outcome(cq, cjb, cm, cn);
                if (ps < 0 || !next_pop(cq, cjb, ps, &p[got])) break;
                cq = p[got].q;
                cjb = p[got].jb;
                cm = p[got].m;
                cn = p[got].n;
                ++got;
            }
            journal.on = false;
            journal.rollback();
            for (auto it = job_saves.rbegin(); it != job_saves.rend(); ++it) {
                HJob& j = S.jobs[it->jb];
                j.cnt_alloc = it->cnt;
                j.cursor = it->cur;
                j.drf_alloc = it->drf;
                j.drf_share = it->share;
            }
            for (auto it = queue_saves.rbegin(); it != queue_saves.rend(); ++it) {
                HQueue& Q = S.queues[it->q];
                Q.allocated = it->alloc;
                Q.share = it->share;
            }
            job_saves.clear();
            queue_saves.clear();
            // queued predictions are the oldest ones: chain only behind agreeing ones
            for (size_t i = 0; i < specs.size(); ++i) {
                if ((int)i >= got) return;
                const Spec& s0 = specs[i];
                if (s0.jb != p[i].jb || s0.cursor != p[i].cur || s0.ready != p[i].ready || s0.L.cls != p[i].cls ||
                    s0.L.m != p[i].m)
                    return;
            }
            for (int i = (int)specs.size(); i < got; ++i) launch_pred(p[i]);
        };
        // The walk FitDelta histogram of a pop's last task when the kernels did
        // not report it (a pop that placed every pending task and left its job
        // not Ready): recomputed on the device state that task saw — queued
        // predictions retracted, its own commit undone and redone around the
        // recount (k_fit_key / k_fit_delta), the fallback node as it was before
        // that commit, and for a class with inter-pod priority terms the
        // score's min / max prepass on that state.  Shards: the chosen node's
        // walk key (its owner computes it) and the counts are all-reduced.
        auto fit_sync = [&](int cls, int node, int kind, HJob& job) {
            S.stats.fit_syncs++;
            discard_all();
            ov_quiesce(S);
            const int32_t nd[1] = {node}, kd[1] = {kind};
            if (node >= 0) {
                HIPCHK(launch_undo_pop(S.nc, S.tab, cls, 1, nd, kd, S.stream));
                sess_placed(S, node, -1);  // the fallback node the task saw
            }
            ctrl_setup(S, 1, &cls, 0, 0, 0, 0, -1, 0);
            if (node >= 0) sess_placed(S, node, +1);
            if (S.classes[cls].ipa_n > 0) {
                HIPCHK(launch_ipa_minmax(S.nc, S.tab, S.d_ctrl, 0, S.stream));
                exchange(S, &S.d_ctrl->ipa_lo[0], KBHIP_RED_MIN_I64);
                exchange(S, &S.d_ctrl->ipa_hi[0], KBHIP_RED_MAX_I64);
            }
            if (node >= 0) {
                HIPCHK(launch_fit_key(S.conf, S.nc, S.tab, S.d_ctrl, node, S.stream));
                exchange(S, &S.d_ctrl->slot[0], KBHIP_RED_MAX_U64);
            }
            HIPCHK(hipMemsetAsync(S.d_fit4, 0, 4 * sizeof(int32_t), S.stream));
            HIPCHK(launch_fit_count(S.conf, S.nc, S.tab, S.d_ctrl, node, kind, S.d_fit4, S.stream));
            if (node >= 0) HIPCHK(launch_redo_pop(S.nc, S.tab, cls, 1, nd, kd, S.stream));
            HIPCHK(hipMemcpyAsync(job.fit, S.d_fit4, 4 * sizeof(int32_t), hipMemcpyDeviceToHost, S.stream));
            HIPCHK(hipStreamSynchronize(S.stream));
            fit_allreduce(S, job.fit);
        };
        // One job pop through the device: the first chunk batched (possibly
        // already queued by speculation), the rest through place_job.
        auto exec_pop = [&](int q, int jb, int n, int32_t* n_done, int32_t* stop) {
            HJob& job = S.jobs[jb];
            const int cls0 = S.pods[ids[0]].cls;
            int m = 1;
            while (m < n && m < kMaxChunk && S.pods[ids[m]].cls == cls0) ++m;
            bool batch = batchable(S, cls0);
            if (batch && S.any_bf && cls0 < (int)S.bf_backoff.size() && S.bf_backoff[cls0] > 0) {
                S.bf_backoff[cls0]--;  // placement 6 missed for this class recently (place_job)
                batch = false;
            }
            bool have = false;
            BatchLaunch L;
            if (!specs.empty()) {
                const Spec& s0 = specs.front();
                if (batch && s0.jb == jb && s0.cursor == job.cursor && s0.ready == job.cnt_alloc && s0.L.cls == cls0 &&
                    s0.L.m == m) {
                    L = s0.L;
                    have = true;
                    specs.pop_front();
                    S.stats.spec_hits++;
                } else {
                    discard_all();
                }
            }
            if (!batch) {
                place_job(S, ids.data(), n, gm, job.min_avail, job.cnt_alloc, onode.data(), okind.data(), n_done, stop);
                return;
            }
            if (!have) L = launch_batched(S, cls0, m, gm, job.min_avail, job.cnt_alloc);
            if (S.speculate > 0 && !S.any_bf) speculate(q, jb, m, n);  // the undo of a pop has no visit rule
            int nd = 0, st = 0;
            collect_batched(S, L, &nd, &st, S.res_node_buf, S.res_kind_buf);
            if (st < 0) throw Error(KBHIP_EDEVICE, "device pop did not complete");
            if (nd == 0 && L.bf) {  // placed nothing: the rest of this pop and the class's next pops take
                if (S.bf_backoff.size() < S.classes.size()) S.bf_backoff.resize(S.classes.size(), 0);
                S.bf_backoff[cls0] = kBfBackoff + 1;  // the general path (place_job below consumes one)
            }
            int alloc = 0;
            for (int j = 0; j < nd; ++j) alloc += S.res_kind_buf[j] == 1;
            apply_results(S, ids.data(), nd, S.res_node_buf, S.res_kind_buf, onode.data(), okind.data());
            if (st == KBHIP_STOP_ALL && nd < n) {  // more chunks: the prediction assumed the pop ended here
                discard_all();
                int32_t nd2 = 0, st2 = 0;
                place_job(S, ids.data() + nd, n - nd, gm, job.min_avail, job.cnt_alloc + alloc, onode.data() + nd,
                          okind.data() + nd, &nd2, &st2);
                nd += nd2;
                st = st2;
            }
            *n_done = nd;
            *stop = st;
        };

        while (!queues.empty()) {
            int q = queues.pop();
            if (overused(q)) continue;
            auto jit = jobs_map.find(q);
            if (jit == jobs_map.end() || jit->second.empty()) continue;
            int jb = jit->second.pop();
            HJob& job = S.jobs[jb];
            S.stats.pops++;
            build_pending(job);
            if (job.cursor < job.pending.size()) {
                int n = (int)(job.pending.size() - job.cursor);
                ids.assign(job.pending.begin() + job.cursor, job.pending.end());
                onode.assign(n, -1);
                okind.assign(n, 0);
                int32_t n_done = 0, stop = 0;
                exec_pop(q, jb, n, &n_done, &stop);
                S.stats.tasks += n_done;
                for (int i = 0; i < n_done; ++i) {
                    const int pi = ids[i];
                    if (onode[i] < 0) continue;
                    HPod& p = S.pods[pi];
                    p.node = onode[i];
                    if (okind[i] == KBHIP_ALLOCATED) { p.status = Allocated; job.cnt_alloc++; }
                    else p.status = Pipelined;
                    job.priority = p.priority;  // UpdateTaskStatus -> AddTaskInfo (job_info.go:242)
                    on_allocate(pi);
                    S.log.emplace_back(pi, onode[i], okind[i]);
                    S.stats.placed++;
                    if (p.status == Allocated && job_ready(job))  // dispatch: Allocated -> Binding (session.go:286-294)
                        for (int t : job.tasks)
                            if (S.pods[t].status == Allocated) { S.pods[t].status = Binding; job.priority = S.pods[t].priority; }
                }
                job.cursor += n_done;
                // NodesFitDelta (allocate.go:124-126, 164-167): what the job keeps is the walk of
                // the task that ended its last pop; only a job left not Ready reports it
                if (stop == KBHIP_STOP_UNASSIGNED && S.last_fit_ok) {
                    for (int q = 0; q < 4; ++q) job.fit[q] = S.last_fit[q];
                } else if (S.gang_close && n_done >= 1 &&
                           (stop == KBHIP_STOP_UNASSIGNED || (stop == KBHIP_STOP_ALL && !job_ready(job)))) {
                    const int last = n_done - 1;
                    fit_sync(S.pods[ids[last]].cls, stop == KBHIP_STOP_UNASSIGNED ? -1 : onode[last], okind[last], job);
                }
                if (stop == KBHIP_STOP_READY) jit->second.push(jb);
                if (stop == KBHIP_STOP_UNASSIGNED) S.stats.unassigned_pops++;
            }
            queues.push(q);
        }
        discard_all();  // predicted pops that never came
        ov_quiesce(S);
        ev_harvest_all(S);
        HIPCHK(hipEventRecord(S.ev_run[1], S.stream));
        HIPCHK(hipStreamSynchronize(S.stream));
        float dms = 0;
        HIPCHK(hipEventElapsedTime(&dms, S.ev_run[0], S.ev_run[1]));
        S.alloc_device_s += dms * 1e-3;
        S.stats.allocate_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    }

    // -----------------------------------------------------------------------
    // reclaim / preempt (actions/reclaim/reclaim.go:41-196,
    // actions/preempt/preempt.go:43-353, framework/statement.go).  The walk
    // order of a preemptor's nodes comes from the device (kbhip_evict.hip);
    // victims are chosen per node on the host model, in the pinned order of
    // NodeInfo.Tasks (pod index).  Evictions / pipelines update the device rows
    // (Releasing, pod count, nonzero requests, ports) before the next sweep.
    // -----------------------------------------------------------------------
    static bool le_tol(const R3& a, const R3& b) {  // Resource.LessEqual on exact integers (Appendix A.2)
        return a.c - b.c < kMinCPU && a.m - b.m < kMinMem && a.g - b.g < kMinGPU;
    }
    static bool less_strict(const R3& a, const R3& b) { return a.c < b.c && a.m < b.m && a.g < b.g; }
    // Node-sharded sessions: the host model — victims, statements, records — is
    // replicated on every rank; each rank ranks its own node range and the sorted lists are
    // all-gathered and merged (the keys carry the global node index, so the merge is the
    // one-GPU order); evictions and pipelines change the device rows of the owning shard only,
    // the pod-affinity count tables on every shard.
    void check_evict_supported() {
        if (S.world != 1 && !S.xgfn && !S.comm)
            throw Error(KBHIP_EINVAL, "reclaim / preempt on a node-sharded session need an all-gather "
                                      "(kbhip_shard_connect_host with a gather, or kbhip_shard_connect_rccl)");
    }
    int local_node(int g) const {  // this shard's row of global node g, or -1
        const int l = g - S.nc.base;
        return l >= 0 && l < S.nc.n ? l : -1;
    }
    void on_deallocate(int pi) {  // event handlers drf.go:144-151, proportion.go:211-219
        const HPod& p = S.pods[pi];
        HJob& j = S.jobs[p.job];
        if (S.drf_on) { j.drf_alloc.sub(p.req); drf_update(j); }
        if (S.prop_on) { HQueue& q = S.queues[j.queue]; q.allocated.sub(p.req); prop_update(q); }
    }
    // JobInfo.UpdateTaskStatus (job_info.go:251-264): the status index, and
    // AddTaskInfo's "job priority = this task's priority" (:242)
    static bool gang_ready_status(int st) { return allocated_status(st) || st == Succeeded || st == Pipelined; }
    void set_status(int pi, int st) {
        HPod& p = S.pods[pi];
        HJob& j = S.jobs[p.job];
        if (p.job < (int)ready_ok.size() && ready_ok[p.job])  // keep the cached readyTaskNum exact
            ready_val[p.job] += (int)gang_ready_status(st) - (int)gang_ready_status(p.status);
        if (pi < (int)run_copy.size()) run_copy[pi] = (st == Running && !p.node_rel) ? 1 : 0;
        if (allocated_status(p.status)) j.cnt_alloc--;
        if (p.status == AOB) j.cnt_aob--;
        p.status = st;
        if (allocated_status(st)) j.cnt_alloc++;
        if (st == AOB) j.cnt_aob++;
        j.priority = p.priority;
    }
    void build_node_tasks() {  // NodeInfo.Tasks of every node from the host model
        // two passes over the pod records (≈ 110 MB at C5) by pod ranges in parallel: each
        // pod's running-copy byte and per range the tasks per node; then each node's list
        // sized and the ranges' pods written at their offsets (pod order within a node kept)
        const int N = S.n_total, P = (int)S.pods.size();  // (every node: the host model is global on shards)
        const int nth = P < (1 << 16) ? 1 : host_threads();
        vector<vector<int32_t>> cnt(nth, vector<int32_t>(N, 0));
        run_copy.assign(P, 0);
        auto range = [&](int r, int& b, int& e) { b = (int)((int64_t)P * r / nth); e = (int)((int64_t)P * (r + 1) / nth); };
        run_ranges(nth, [&](int r) {
            int b, e;
            range(r, b, e);
            int32_t* c = cnt[r].data();
            for (int i = b; i < e; ++i) {
                const HPod& p = S.pods[i];
                run_copy[i] = (p.status == Running && !p.node_rel) ? 1 : 0;
                if (on_node_of(p) && p.status != Pending) c[p.node]++;
            }
        });
        S.node_tasks.resize(N);
        for (int n = 0; n < N; ++n) {
            int32_t base = 0;
            for (int r = 0; r < nth; ++r) { const int32_t k = cnt[r][n]; cnt[r][n] = base; base += k; }
            S.node_tasks[n].resize(base);
        }
        run_ranges(nth, [&](int r) {
            int b, e;
            range(r, b, e);
            int32_t* c = cnt[r].data();
            for (int i = b; i < e; ++i) {
                const HPod& p = S.pods[i];
                if (on_node_of(p) && p.status != Pending) S.node_tasks[p.node][c[p.node]++] = i;
            }
        });
    }
    // fn(0..nth-1), fn(0) on this thread
    template <typename Fn>
    static void run_ranges(int nth, Fn fn) {
        vector<std::thread> th;
        for (int r = 1; r < nth; ++r) th.emplace_back(fn, r);
        fn(0);
        for (auto& x : th) x.join();
    }
    // The eviction actions' job scan (reclaim.go:60-90 / preempt.go:58-85 build their
    // preemptor lists from every job's Pending tasks): per job its Pending tasks in
    // TaskOrderFn order, and gang's readyTaskNum (gang.go:212-222) of every job, kept exact
    // from here on by set_status; job ranges in parallel
    void scan_jobs(vector<vector<int>>& pend) {
        const int J = (int)S.jobs.size();
        pend.assign(J, {});
        reset_ready_cache();
        const int nth = S.pods.size() < (1u << 16) ? 1 : host_threads();
        run_ranges(nth, [&](int r) {
            for (int jb = (int)((int64_t)J * r / nth); jb < (int)((int64_t)J * (r + 1) / nth); ++jb) {
                int c = 0;
                for (int t : S.jobs[jb].tasks) {
                    const int st = S.pods[t].status;
                    c += gang_ready_status(st);
                    if (st == Pending) pend[jb].push_back(t);
                }
                ready_val[jb] = c;
                ready_ok[jb] = 1;
                if (pend[jb].size() > 1)
                    std::sort(pend[jb].begin(), pend[jb].end(), [this](int a, int b) { return task_less(a, b); });
            }
        });
    }
    bool node_copy_running(int pi) const { return S.pods[pi].status == Running && !S.pods[pi].node_rel; }
    // node_copy_running per pod as a byte (the candidate filters read it for every task of every
    // node visited): built with pod_queue, kept exact by set_status and unevict
    vector<uint8_t> run_copy;
    // The walk order of the task of class cls: preempt (by_score) = SelectBestNode order of
    // the nodes passing PredicateFn with a NodeOrderFn score; reclaim = passing nodes in order.
    void rank_nodes(int cls, bool by_score, vector<int>& out) {
        const auto tr0 = std::chrono::steady_clock::now();
        rank_nodes_inner(cls, by_score, out);
        S.stats.evict_rank_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - tr0).count();
    }
    void rank_nodes_inner(int cls, bool by_score, vector<int>& out) {
        const int N = S.nc.n;
        rank_buffers(S);
        flush_tables(S);  // evictions / unevicts so far change pod-affinity predicates
        ctrl_setup(S, 1, &cls, 0, 0, 0, 0, -1, 0);
        HIPCHK(hipMemsetAsync(S.b_rank_cnt.p, 0, 2 * sizeof(uint32_t), S.stream));
        auto sr = S.class_srange[cls];
        if (by_score && S.classes[cls].ipa_n > 0) {  // inter-pod priority: normalisation prepass, wider range
            HIPCHK(launch_ipa_minmax(S.nc, S.tab, S.d_ctrl, 0, S.stream));
            exchange(S, &S.d_ctrl->ipa_lo[0], KBHIP_RED_MIN_I64);  // (shards: over every node)
            exchange(S, &S.d_ctrl->ipa_hi[0], KBHIP_RED_MAX_I64);
            const int64_t w = 10 * (int64_t)S.conf.w_pa * S.conf.score_mult;
            sr.first += std::min<int64_t>(0, w);
            sr.second += std::max<int64_t>(0, w);
        }
        const bool counting = !S.force_radix && sr.second - sr.first < 256 && sr.first >= INT32_MIN &&
                              sr.second <= INT32_MAX;
        if (counting && S.rank_group && S.world == 1) {  // one launch with the concurrent what-if sessions' rankings
            StepBatcher::Req r;
            r.kind = StepBatcher::kRank;
            HIPCHK(fill_rank_desc(&r.rank, S.conf, S.nc, S.tab, S.classes[cls], S.d_ctrl, by_score ? 1 : 0, (int)sr.first,
                                  (int)sr.second, (uint64_t*)S.b_rank_keys.p, (uint32_t*)S.b_rank_tmp.p,
                                  (uint64_t*)S.b_rank_sorted.p, (uint32_t*)S.b_rank_cnt.p));
            r.st = S.stream;
            r.device = S.device;
            HIPCHK(hipStreamSynchronize(S.stream));  // this request's control block and counters are in place
            StepBatcher::get().submit(r);
            HIPCHK(hipSetDevice(S.device));
            HIPCHK(r.err);
            S.stats.rank_requests++;
            S.stats.rank_batch_sum += r.batch;
        } else if (counting) {  // hand-written stable counting sort over the score
            HIPCHK(launch_rank_sorted(S.conf, S.nc, S.tab, S.classes[cls], S.d_ctrl, by_score ? 1 : 0, (int)sr.first,
                                      (int)sr.second,
                                      (uint64_t*)S.b_rank_keys.p, (uint32_t*)S.b_rank_tmp.p,
                                      (uint64_t*)S.b_rank_sorted.p, (uint32_t*)S.b_rank_cnt.p, S.stream));
        } else {  // wide score ranges (large nodeorder weights): 8-bit LSD radix passes over the score
            HIPCHK(launch_rank_nodes(S.conf, S.nc, S.tab, S.d_ctrl, by_score ? 1 : 0, (uint64_t*)S.b_rank_keys.p,
                                     (uint32_t*)S.b_rank_cnt.p, S.stream));
            HIPCHK(launch_rank_radix((const uint64_t*)S.b_rank_keys.p, N, (const uint32_t*)S.b_rank_cnt.p,
                                     (uint32_t*)S.b_rank_tmp.p, (uint64_t*)S.b_rank_radix.p,
                                     (uint64_t*)S.b_rank_sorted.p, S.stream));
        }
        const int first = std::min(N, S.rank_first);
        HIPCHK(hipMemcpyAsync(S.h_rank, S.b_rank_cnt.p, 2 * sizeof(uint32_t), hipMemcpyDeviceToHost, S.stream));
        HIPCHK(hipMemcpyAsync(S.h_rank + 1, S.b_rank_sorted.p, first * sizeof(uint64_t), hipMemcpyDeviceToHost,
                              S.stream));
        HIPCHK(hipStreamSynchronize(S.stream));
        const int cnt = (int)(uint32_t)S.h_rank[0];
        if (S.h_rank[0] >> 32) throw Error(KBHIP_EDEVICE, "rank_nodes: node score outside the class score range");
        if (cnt > first) {
            HIPCHK(hipMemcpyAsync(S.h_rank + 1 + first, (const uint64_t*)S.b_rank_sorted.p + first,
                                  (size_t)(cnt - first) * sizeof(uint64_t), hipMemcpyDeviceToHost, S.stream));
            HIPCHK(hipStreamSynchronize(S.stream));
        }
        if (S.world > 1) {
            merge_shard_ranks(cnt, out);
        } else {
            out.resize(cnt);
            for (int i = 0; i < cnt; ++i) out[i] = key_idx(S.h_rank[1 + i]);
        }
        S.stats.sweeps++;
        S.stats.tasks++;
    }
    // Node-sharded ranking: every shard's sorted passing keys (descending; global node index
    // inside) all-gathered as fixed-size records [count, keys...], merged into the order one
    // GPU's sort of every node gives (the keys are distinct).
    void merge_shard_ranks(int cnt, vector<int>& out) {
        const size_t rec = (size_t)(S.n_total + S.world - 1) / S.world + 1;  // >= every shard's rows + 1
        vector<uint64_t> send(rec, 0), recv(rec * S.world);
        send[0] = (uint64_t)cnt;
        std::memcpy(send.data() + 1, S.h_rank + 1, (size_t)cnt * sizeof(uint64_t));
        gather_host(S, send.data(), recv.data(), rec * sizeof(uint64_t));
        vector<size_t> at(S.world), end(S.world);
        size_t total = 0;
        for (int r = 0; r < S.world; ++r) {
            const uint64_t c = recv[rec * r];
            if (c >= rec) throw Error(KBHIP_EDEVICE, "shard ranking: a rank's count exceeds its record");
            at[r] = rec * r + 1;
            end[r] = at[r] + c;
            total += c;
        }
        out.resize(total);
        for (size_t i = 0; i < total; ++i) {
            int best = -1;
            for (int r = 0; r < S.world; ++r)
                if (at[r] < end[r] && (best < 0 || recv[at[r]] > recv[at[best]])) best = r;
            out[i] = key_idx(recv[at[best]++]);
        }
    }
    void dev_op(int op, int pi) {  // the row on the owning shard, the count tables on every shard
        const HPod& p = S.pods[pi];
        HIPCHK(launch_node_op(S.nc, S.tab, op, local_node(p.node), p.node, p.cls, p.req.c, p.req.m, p.req.g,
                              S.stream));
    }
    // the session half of an eviction (session.go:331-356 / statement.go:35-67)
    void evict_in_session(int v) {
        if (allocated_status(S.pods[v].status)) queue_target(S, v, -1);  // no longer a predicate target
        set_status(v, Releasing);
        // node.UpdateTask: Releasing += Resreq.  No node ranking reads Releasing, so
        // evictions are summed per node and applied in one launch (flush_evictions)
        const HPod& p = S.pods[v];
        if (S.rel_delta.empty()) { S.rel_delta.assign(S.n_total, R3{}); S.rel_flag.assign(S.n_total, 0); }
        if (!S.rel_flag[p.node]) { S.rel_flag[p.node] = 1; S.rel_touched.push_back(p.node); }
        R3& d = S.rel_delta[p.node];
        d.c += p.req.c; d.m += p.req.m; d.g += p.req.g;
        on_deallocate(v);
    }
    void flush_evictions() {
        const int nt = (int)S.rel_touched.size();
        if (!nt) return;
        vector<int32_t> nodes;
        vector<int64_t> d;
        nodes.reserve(nt);
        d.reserve(3 * (size_t)nt);
        for (int i = 0; i < nt; ++i) {
            const int v = S.rel_touched[i];
            const int l = local_node(v);  // (shards: the owning rank's rows only)
            if (l >= 0) {
                nodes.push_back(l);
                d.push_back(S.rel_delta[v].c); d.push_back(S.rel_delta[v].m); d.push_back(S.rel_delta[v].g);
            }
            S.rel_delta[v] = R3{};
            S.rel_flag[v] = 0;
        }
        S.rel_touched.clear();
        const int n = (int)nodes.size();
        if (!n) { flush_tables(S); return; }
        int32_t* dn = S.b_rel_nodes.alloc<int32_t>(n);
        int64_t* dd = S.b_rel_d.alloc<int64_t>(3 * (size_t)n);
        HIPCHK(hipMemcpyAsync(dn, nodes.data(), n * sizeof(int32_t), hipMemcpyHostToDevice, S.stream));
        HIPCHK(hipMemcpyAsync(dd, d.data(), d.size() * sizeof(int64_t), hipMemcpyHostToDevice, S.stream));
        HIPCHK(launch_rel_add(S.nc, dn, dd, n, S.stream));
        HIPCHK(hipStreamSynchronize(S.stream));  // the pageable sources must outlive the copies
        flush_tables(S);
    }
    void unevict(int v) {  // statement.go:81-105: node.AddTask fails, the node keeps its Releasing copy
        set_status(v, Running);
        queue_target(S, v, +1);  // a predicate target again (the lister reads the job's status index)
        S.pods[v].node_rel = true;
        if (v < (int)run_copy.size()) run_copy[v] = 0;
        on_allocate(v);
    }
    void pipeline(int t, int n) {  // statement.go:96-136 / session.go:199-235
        HPod& p = S.pods[t];
        set_status(t, Pipelined);
        p.node = n;
        auto& nt = S.node_tasks[n];
        nt.insert(std::lower_bound(nt.begin(), nt.end(), t), t);
        dev_op(1, t);
        S.used[n].c += p.req.c; S.used[n].m += p.req.m; S.used[n].g += p.req.g;
        sess_placed(S, n, +1);
        if (S.classes[p.cls].backfill) S.any_bf = 1;
        on_allocate(t);
    }
    void unpipeline(int t) {  // statement.go:141-172 (task.NodeName stays set)
        HPod& p = S.pods[t];
        set_status(t, Pending);
        auto& nt = S.node_tasks[p.node];
        nt.erase(std::lower_bound(nt.begin(), nt.end(), t));
        dev_op(2, t);
        S.used[p.node].c -= p.req.c; S.used[p.node].m -= p.req.m; S.used[p.node].g -= p.req.g;
        sess_placed(S, p.node, -1);
        on_deallocate(t);
    }
    struct Stmt {  // framework.Statement: (0 evict | 1 pipeline, pod)
        vector<std::pair<int, int>> ops;
    };
    void commit(Stmt& st) {  // statement.go:188-198: evictions reach the cache (recorded), pipelines bind nothing
        for (auto& op : st.ops)
            S.log.emplace_back(op.second, S.pods[op.second].node, op.first == 0 ? KBHIP_EVICTED : KBHIP_PIPELINED);
        st.ops.clear();
    }
    void discard(Stmt& st) {  // statement.go:174-186
        for (auto it = st.ops.rbegin(); it != st.ops.rend(); ++it) {
            if (it->first == 0) unevict(it->second);
            else unpipeline(it->second);
        }
        st.ops.clear();
    }
    // Session.Preemptable / Reclaimable (session_plugins.go:67-148): per tier the
    // intersection of the enabled plugins' victims; the first non-empty tier decides,
    // and once a plugin has answered later tiers only intersect further.
    // readyTaskNum per job (gang.go:212-222), computed on first use in an
    // eviction action and kept exact by set_status (every status change of the
    // action goes through it); reset at the start of each action
    vector<uint8_t> ready_ok;
    vector<int> ready_val;
    // per-call scratch keyed by job / queue slot, valid where stamp == the call's epoch
    vector<uint32_t> alloc_stamp;
    vector<F3> alloc_val;
    uint32_t epoch = 0;
    vector<int> cand, inter;
    vector<uint32_t> mark;  // pod -> epoch: membership in the plugin's answer (the tier intersection)
    // per action: the victim functions in tier order as codes (1 gang, 2 conformance, 3 drf,
    // 4 proportion; the tiers' plugin names compared once, not per node visited), and per pod
    // its job's queue and MinAvailable (read for every candidate of every visit)
    vector<vector<int>> vic_tiers;
    int vic_mode = -1;  // the action vic_tiers was compiled for (1 preempt, 0 reclaim)
    void reset_ready_cache() {
        ready_ok.assign(S.jobs.size(), 0);
        ready_val.assign(S.jobs.size(), 0);
    }
    void compile_victims(bool preempt) {
        vic_mode = preempt ? 1 : 0;
        vic_tiers.clear();
        for (auto& tier : S.tiers) {
            vector<int> codes;
            for (auto& pl : tier) {
                if (pl.flags & (preempt ? KBS_DIS_PREEMPTABLE : KBS_DIS_RECLAIMABLE)) continue;
                if (pl.name == "gang") codes.push_back(1);
                else if (pl.name == "conformance") codes.push_back(2);
                else if (preempt && pl.name == "drf" && S.drf_on) codes.push_back(3);
                else if (!preempt && pl.name == "proportion" && S.prop_on) codes.push_back(4);
            }
            vic_tiers.push_back(std::move(codes));
        }
        const int P = (int)S.pods.size();
        if ((int)run_copy.size() != P) {  // (build_node_tasks fills it in its pass over the pods)
            run_copy.assign(P, 0);
            for (int i = 0; i < P; ++i) run_copy[i] = node_copy_running(i) ? 1 : 0;
        }
        if ((int)S.pod_queue.size() != P || S.pod_queue_gen != S.model_gen) {  // once per session model
            S.pod_queue.assign(P, -1);
            S.pod_min.assign(P, 0);
            for (const HJob& J : S.jobs)  // job-major: a job's tasks are neighbouring pods
                for (int t : J.tasks) { S.pod_queue[t] = J.queue; S.pod_min[t] = J.min_avail; }
            S.pod_queue_gen = S.model_gen;
        }
    }
    void victims_of(bool preempt, int evictor, const vector<int>& evictees, vector<int>& victims) {
        victims.clear();
        S.stats.evict_visits++;
        S.stats.evict_cands += (int64_t)evictees.size();
        if (evictees.empty()) return;  // every plugin returns nil for no candidates
        bool init = false;
        if (alloc_stamp.empty()) {
            const size_t J = S.jobs.size(), Q = S.queues.size();
            alloc_stamp.assign(std::max(J, Q), 0); alloc_val.assign(std::max(J, Q), F3{});
            mark.assign(S.pods.size(), 0);
        }
        if (ready_ok.size() != S.jobs.size()) reset_ready_cache();
        if (vic_mode != (preempt ? 1 : 0) || S.pod_queue.size() != S.pods.size()) compile_victims(preempt);
        for (auto& tier : vic_tiers) {
            for (int code : tier) {
                cand.clear();
                if (code == 1) {  // gang.go:107-129
                    for (int e : evictees) {
                        const int jb = S.pods[e].job;
                        if (!ready_ok[jb]) {  // readyTaskNum (gang.go:212-222)
                            int c = 0;
                            for (int t : S.jobs[jb].tasks) c += gang_ready_status(S.pods[t].status);
                            ready_ok[jb] = 1;
                            ready_val[jb] = c;
                        }
                        const int mn = S.pod_min[e];
                        if (mn <= ready_val[jb] - 1 || mn == 1) cand.push_back(e);
                    }
                } else if (code == 2) {  // conformance.go:37-56
                    for (int e : evictees) if (!S.pods[e].critical) cand.push_back(e);
                } else if (code == 3) {  // drf.go:84-109
                    const HPod& pr = S.pods[evictor];
                    F3 la = S.jobs[pr.job].drf_alloc;
                    la.add(pr.req);
                    const double ls = drf_share_of(la);
                    const uint32_t ea = ++epoch;
                    for (int e : evictees) {
                        const int jb = S.pods[e].job;
                        if (alloc_stamp[jb] != ea) { alloc_stamp[jb] = ea; alloc_val[jb] = S.jobs[jb].drf_alloc; }
                        alloc_val[jb].sub(S.pods[e].req);
                        const double rs = drf_share_of(alloc_val[jb]);
                        if (ls < rs || std::fabs(ls - rs) <= 0.000001) cand.push_back(e);  // shareDelta (drf.go:29)
                    }
                } else if (code == 4) {  // proportion.go:159-183
                    const uint32_t ea = ++epoch;
                    for (int e : evictees) {
                        const int qi = S.pod_queue[e];
                        const HQueue& q = S.queues[qi];
                        if (alloc_stamp[qi] != ea) { alloc_stamp[qi] = ea; alloc_val[qi] = q.allocated; }
                        F3 rq;
                        rq.add(S.pods[e].req);
                        if (alloc_val[qi].less(rq)) continue;
                        alloc_val[qi].sub(S.pods[e].req);
                        if (q.deserved.less_equal(alloc_val[qi])) cand.push_back(e);
                    }
                }
                if (!init) {
                    victims = cand;
                    init = true;
                } else {  // victims in their order, kept where the plugin also answered them
                    const uint32_t em = ++epoch;
                    for (int c : cand) mark[c] = em;
                    inter.clear();
                    for (int v : victims)
                        if (mark[v] == em) inter.push_back(v);
                    victims.swap(inter);
                }
            }
            if (!victims.empty()) return;
        }
    }
    double drf_share_of(const F3& a) const {  // drf.go:160-170
        double res = 0;
        for (int k = 0; k < 3; ++k) { double x = share(a.get(k), S.total.get(k)); if (x > res) res = x; }
        return res;
    }
    // preempt() (preempt.go:259-353); filter over the node's task copies
    template <typename Filter>
    bool preempt_one(Stmt& st, int pi, Filter keep) {
        const HPod& pr = S.pods[pi];
        if (pr.cls < 0) throw Error(KBHIP_EUNSUPPORTED, "preemptor without a task class");
        vector<int> order, cands, victims;
        rank_nodes(pr.cls, true, order);
        const int no = (int)order.size();
        for (int i = 0; i < std::min(no, kPrefetchAhead); ++i) prefetch_pods(order[i]);
        for (int oi = 0; oi < no; ++oi) {
            const int n = order[oi];
            if (oi + kPrefetchAhead < no) prefetch_pods(order[oi + kPrefetchAhead]);
            if (oi + 1 < no) prefetch_jobs(order[oi + 1]);
            cands.clear();
            for (int t : S.node_tasks[n]) if (keep(t)) cands.push_back(t);
            victims_of(true, pi, cands, victims);
            if (victims.empty()) continue;  // validateVictims (:355-370)
            R3 all, resreq = pr.ireq, got;
            for (int v : victims) { all.c += S.pods[v].req.c; all.m += S.pods[v].req.m; all.g += S.pods[v].req.g; }
            if (less_strict(all, resreq)) continue;
            for (int v : victims) {
                const R3 vr = S.pods[v].req;
                evict_in_session(v);
                st.ops.emplace_back(0, v);
                got.c += vr.c; got.m += vr.m; got.g += vr.g;
                if (le_tol(resreq, vr)) break;
                resreq.c -= vr.c; resreq.m -= vr.m; resreq.g -= vr.g;
            }
            if (le_tol(pr.ireq, got)) {
                pipeline(pi, n);
                st.ops.emplace_back(1, pi);
                return true;
            }
        }
        return false;
    }
    // The walks read the records of every task on each visited node (run copy, queue,
    // MinAvailable, job, request) and evict most candidates (C5: ≈ 2.4 M candidates and
    // ≈ 720 k evictions per reclaim, pods scattered over 160 MB of records): the next
    // nodes' records are prefetched while one node is visited (the order is known), their
    // jobs one visit ahead (the job index is in the pod record fetched before).
    static constexpr int kPrefetchAhead = 3;
    void prefetch_pods(int n) {
        for (int t : S.node_tasks[n]) {
            const char* pp = reinterpret_cast<const char*>(&S.pods[t]);
            for (size_t o = 0; o < sizeof(HPod); o += 64) __builtin_prefetch(pp + o);
            __builtin_prefetch(pp + sizeof(HPod) - 1);
            __builtin_prefetch(&run_copy[t]);
            __builtin_prefetch(&S.pod_queue[t]);
            __builtin_prefetch(&S.pod_min[t]);
        }
    }
    void prefetch_jobs(int n) {
        for (int t : S.node_tasks[n]) {
            const int jb = S.pods[t].job;
            if (jb < 0) continue;
            const char* jp = reinterpret_cast<const char*>(&S.jobs[jb]);
            for (size_t o = 0; o < sizeof(HJob); o += 64) __builtin_prefetch(jp + o);
            __builtin_prefetch(jp + sizeof(HJob) - 1);
            __builtin_prefetch(&ready_val[jb]);
        }
    }
#ifdef KBHIP_WALK_PROF  // diagnostic build: reclaim walk split (gather / victims / evictions), stderr
    uint64_t wp_acc[3] = {0, 0, 0}, wp_last = 0;
    int wp_ph = -1;
    void wp_mark(int ph) {
        const uint64_t t = __builtin_ia32_rdtsc();
        if (wp_ph >= 0) wp_acc[wp_ph] += t - wp_last;
        wp_last = t;
        wp_ph = ph;
    }
#define WP_MARK(ph) wp_mark(ph)
#define WP_REPORT(name) (fprintf(stderr, "walkprof %s gather %.3g victims %.3g evict %.3g Gcycles\n", name, \
                                 wp_acc[0] * 1e-9, wp_acc[1] * 1e-9, wp_acc[2] * 1e-9), wp_ph = -1)
#else
#define WP_MARK(ph) ((void)0)
#define WP_REPORT(name) ((void)0)
#endif
    // host wall time of an eviction action minus its node rankings (stats.evict_walk_s)
    struct WalkTimer {
        Session& S;
        std::chrono::steady_clock::time_point t0;
        double rank0;
        explicit WalkTimer(Session& s) : S(s), t0(std::chrono::steady_clock::now()), rank0(s.stats.evict_rank_s) {}
        void setup_done() {
            S.stats.evict_setup_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        }
        ~WalkTimer() {
            S.stats.evict_walk_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() -
                                    (S.stats.evict_rank_s - rank0);
        }
    };
    void preempt_action() {  // preempt.go:43-255
        WalkTimer wt(S);
        reset_ready_cache();
        compile_orders();
        open_plugins();
        check_evict_supported();
        build_node_tasks();
        compile_victims(true);
        auto jl = [this](int a, int b) { return job_less(a, b); };
        std::map<int, GoHeap<decltype(jl)>> preemptors;
        std::unordered_map<int, std::pair<vector<int>, size_t>> ptasks;  // job -> (tasks, cursor)
        vector<int> under;
        vector<char> seen(S.queues.size(), 0);
        vector<vector<int>> pends;
        scan_jobs(pends);
        for (int jb = 0; jb < (int)S.jobs.size(); ++jb) {
            HJob& j = S.jobs[jb];
            seen[j.queue] = 1;
            vector<int>& pend = pends[jb];
            if (pend.empty()) continue;
            auto it = preemptors.find(j.queue);
            if (it == preemptors.end()) it = preemptors.emplace(j.queue, GoHeap<decltype(jl)>(jl)).first;
            it->second.push(jb);
            under.push_back(jb);
            ptasks[jb] = {std::move(pend), 0};
        }
        wt.setup_done();
        Stmt st;
        for (int qi = 0; qi < (int)S.queues.size(); ++qi) {  // map `queues`, pinned to queue order
            if (!seen[qi]) continue;
            for (;;) {  // between jobs of the queue (:87-149)
                auto pit = preemptors.find(qi);
                if (pit == preemptors.end() || pit->second.empty()) break;
                const int pj = pit->second.pop();
                bool assigned = false;
                auto& tq = ptasks[pj];
                for (;;) {
                    if (tq.second >= tq.first.size()) break;
                    const int pt = tq.first[tq.second++];
                    const int pq = S.jobs[pj].queue, ptj = S.pods[pt].job;
                    if (preempt_one(st, pt, [&](int t) {
                            const HPod& p = S.pods[t];
                            return run_copy[t] && p.job >= 0 && S.pod_queue[t] == pq && ptj != p.job;
                        }))
                        assigned = true;
                    if (job_ready(S.jobs[pj])) {
                        commit(st);
                        break;
                    }
                }
                if (!job_ready(S.jobs[pj])) {
                    discard(st);
                    continue;
                }
                st.ops.clear();  // neither committed nor discarded: the session keeps the operations
                if (assigned) pit->second.push(pj);
            }
            for (int jb : under) {  // between tasks of a job (:151-181)
                auto& tq = ptasks[jb];
                for (;;) {
                    if (tq.second >= tq.first.size()) break;
                    const int pt = tq.first[tq.second++];
                    Stmt s2;
                    const int ptj = S.pods[pt].job;
                    const bool assigned = preempt_one(s2, pt, [&](int t) {
                        return run_copy[t] && ptj == S.pods[t].job;
                    });
                    commit(s2);
                    if (!assigned) break;
                }
            }
        }
        flush_evictions();
    }
    void reclaim_action() {  // reclaim.go:41-196
        WalkTimer wt(S);
        reset_ready_cache();
        compile_orders();
        open_plugins();
        check_evict_supported();
        build_node_tasks();
        compile_victims(false);
        auto ql = [this](int a, int b) { return queue_less(a, b); };
        auto jl = [this](int a, int b) { return job_less(a, b); };
        GoHeap<decltype(ql)> queues(ql);
        vector<char> qseen(S.queues.size(), 0);
        std::map<int, GoHeap<decltype(jl)>> preemptors;
        std::unordered_map<int, std::pair<vector<int>, size_t>> ptasks;
        vector<vector<int>> pends;
        scan_jobs(pends);
        for (int jb = 0; jb < (int)S.jobs.size(); ++jb) {
            HJob& j = S.jobs[jb];
            if (!qseen[j.queue]) { qseen[j.queue] = 1; queues.push(j.queue); }
            vector<int>& pend = pends[jb];
            if (pend.empty()) continue;
            auto it = preemptors.find(j.queue);
            if (it == preemptors.end()) it = preemptors.emplace(j.queue, GoHeap<decltype(jl)>(jl)).first;
            it->second.push(jb);
            ptasks[jb] = {std::move(pend), 0};
        }
        wt.setup_done();
        vector<int> order, cands, victims;
        while (!queues.empty()) {
            const int qi = queues.pop();
            if (overused(qi)) continue;
            auto pit = preemptors.find(qi);
            if (pit == preemptors.end() || pit->second.empty()) continue;
            const int jb = pit->second.pop();
            auto& tq = ptasks[jb];
            if (tq.second >= tq.first.size()) continue;
            const int pt = tq.first[tq.second++];
            const HPod& pr = S.pods[pt];
            if (pr.cls < 0) throw Error(KBHIP_EUNSUPPORTED, "reclaimer without a task class");
            const int jq = S.jobs[jb].queue;
            bool assigned = false;
            rank_nodes(pr.cls, false, order);
            const int no = (int)order.size();
            for (int i = 0; i < std::min(no, kPrefetchAhead); ++i) prefetch_pods(order[i]);
            for (int oi = 0; oi < no; ++oi) {
                const int n = order[oi];
                WP_MARK(0);
                if (oi + kPrefetchAhead < no) prefetch_pods(order[oi + kPrefetchAhead]);
                if (oi + 1 < no) prefetch_jobs(order[oi + 1]);
                cands.clear();
                for (int t : S.node_tasks[n])
                    if (run_copy[t] && S.pod_queue[t] >= 0 && S.pod_queue[t] != jq) cands.push_back(t);
                WP_MARK(1);
                victims_of(false, pt, cands, victims);
                WP_MARK(2);
                if (victims.empty()) continue;
                R3 all, resreq = pr.ireq, got;
                for (int v : victims) { all.c += S.pods[v].req.c; all.m += S.pods[v].req.m; all.g += S.pods[v].req.g; }
                if (less_strict(all, resreq)) continue;
                for (int v : victims) {
                    const R3 vr = S.pods[v].req;
                    S.log.emplace_back(v, S.pods[v].node, KBHIP_EVICTED);  // ssn.Evict: cache.Evict first
                    evict_in_session(v);
                    got.c += vr.c; got.m += vr.m; got.g += vr.g;
                    if (le_tol(resreq, vr)) break;
                    resreq.c -= vr.c; resreq.m -= vr.m; resreq.g -= vr.g;
                }
                if (le_tol(pr.ireq, got)) {
                    pipeline(pt, n);
                    S.log.emplace_back(pt, n, KBHIP_PIPELINED);
                    S.stats.placed++;
                    assigned = true;
                    break;
                }
            }
            if (assigned) queues.push(qi);
        }
        WP_MARK(0);
        WP_REPORT("reclaim");
        flush_evictions();
        HIPCHK(hipStreamSynchronize(S.stream));
    }
};


// The actions other files run (05_actions.cpp, 06_carry.cpp): the allocate
// action, reclaim / preempt, and the first-fit node loop of given tasks.
void allocate_run(Session& S) {
    Allocator a(S);
    a.run();
}
void evict_run(Session& S, bool preempt) {
    Allocator a(S);
    if (preempt) a.preempt_action();
    else a.reclaim_action();
}

// ---------------------------------------------------------------------------
// backfill action (actions/backfill/backfill.go:40-70): every Pending task of
// every job whose InitResreq is empty is allocated on the first node (lowest
// index) passing the predicates.  Pinned order:
// jobs by UID, tasks by UID, nodes by index.  Per-task first-fit sweeps of the
// general kernel (mode 1), 64 tasks per control-block round trip.
// ---------------------------------------------------------------------------
// first_fit: the inner loop of backfill.go:51-65 for the given tasks, in
// order: each goes to the lowest-index node passing PredicateFn and is
// committed with Session.Allocate (session.go:237-297); out_node[i] = that
// node or -1.  Tasks must be Pending tasks of the session (task class >= 0).
void first_fit(Session& S, const int32_t* ids, int n, int32_t* out_node) {
    vector<int> cand(ids, ids + n);
    for (int t : cand)
        if (t < 0 || t >= (int)S.pods.size() || S.pods[t].cls < 0 || S.pods[t].status != Pending)
            throw Error(KBHIP_EINVAL, "task id is not a pending task of the session");
    std::fill(out_node, out_node + n, -1);
    ov_quiesce(S);
    Allocator A(S);
    A.compile_orders();
    A.open_plugins();
    for (size_t off = 0; off < cand.size(); off += kMaxChunk) {
        const int m = (int)std::min<size_t>(kMaxChunk, cand.size() - off);
        int cls[kMaxChunk];
        for (int i = 0; i < m; ++i) cls[i] = S.pods[cand[off + i]].cls;
        uint32_t epoch = 0;
        const int slot = take_slot(S, &epoch);
        ctrl_setup(S, m, cls, 0, 0, 0, 1, slot, epoch);
        sweep_chunk(S, m, cls, false);
        int n_done = 0, stop = -1;
        collect_tasks(S, slot, epoch, m, &n_done, &stop, S.res_node_buf, S.res_kind_buf, nullptr);
        S.stats.sweeps += m;
        S.stats.tasks += m;
        if (n_done != m || stop != 0) throw Error(KBHIP_EDEVICE, "backfill chunk did not complete");
        for (int i = 0; i < m; ++i) {
            const int node = S.res_node_buf[i];
            out_node[off + i] = node;
            if (node < 0) continue;
            const int pi = cand[off + i];
            HPod& p = S.pods[pi];
            HJob& job = S.jobs[p.job];
            p.status = Allocated;  // Session.Allocate(task, node, false) (session.go:237-297)
            p.node = node;
            job.cnt_alloc++;
            job.priority = p.priority;  // UpdateTaskStatus -> AddTaskInfo (job_info.go:242)
            S.used[node].c += p.req.c; S.used[node].m += p.req.m; S.used[node].g += p.req.g;
            sess_placed(S, node, +1);
            A.on_allocate(pi);  // drf / proportion AllocateFunc
            S.stats.placed++;
            S.log.emplace_back(pi, node, KBHIP_ALLOCATED);
            if (A.job_ready(job))  // dispatch: Allocated -> Binding (session.go:286-321)
                for (int t : job.tasks)
                    if (S.pods[t].status == Allocated) { S.pods[t].status = Binding; job.priority = S.pods[t].priority; }
            if (S.classes[cls[i]].backfill) S.any_bf = 1;  // IsBackfill commit (commit_task)
        }
    }
}

}  // namespace kbhip
