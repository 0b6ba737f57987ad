// kbhost — the host side a Go shim keeps when it binds libkbhip's per-pop ABI
// (INTEGRATION.md): allocateAction.Execute's loop
// (pkg/scheduler/actions/allocate/allocate.go:41-201) with the ordering
// plugins of the tiers (priority.go:38-79, gang.go:63-66, drf.go:52-170,
// proportion.go:57-241) and Go's container/heap (container/heap/heap.go),
// written in C++ because this image has no Go toolchain.  Each job pop — the
// job's remaining pending tasks in TaskOrderFn order — goes to the engine;
// its decisions come back and are applied to the host model, as ssn.Allocate /
// ssn.Pipeline would.
//
// Two ways to drive the engine:
//   sync   one kbhip_place_job call per pop (a round trip per pop);
//   async  kbhip_place_job_submit / _wait / _cancel: while pop e runs the
//          host predicts the next `depth` pops (assuming each places its tasks
//          as Allocated up to the gang stop) on its own model — every change
//          journaled and undone — and submits them; a wrong prediction is
//          withdrawn with kbhip_place_job_cancel.
// A third run, kbhip_allocate (the engine's own C++ mirror of the loop), gives
// the reference log and time.  The three placement logs must be identical.
//
// usage: kbhost SNAPSHOT.kbs [--reps R] [--depth D] [--device K] [--modes allocate,sync,async]
// prints one JSON line: per-mode median ms, pops, placements, digests, equal.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <stdexcept>
#include <string>
#include <vector>

#include "kbhip.h"
#include "kbsnap.h"

namespace {

using std::string;
using std::vector;

constexpr double kMin[3] = {10.0, 10.0 * 1024 * 1024, 10.0};  // resource_info.go minMilliCPU / minMemory / minGPU
enum Status { PENDING, ALLOCATED, PIPELINED, BOUND, RUNNING, RELEASING, OTHER };

double share(double l, double r) { return r == 0 ? (l == 0 ? 0.0 : 1.0) : l / r; }  // helpers.go:35-48
bool less_equal(const double* a, const double* b) {  // Resource.LessEqual (resource_info.go:164-168)
    for (int k = 0; k < 3; ++k)
        if (!(a[k] < b[k] || std::fabs(b[k] - a[k]) < kMin[k])) return false;
    return true;
}

void check(int rc, const char* what) {
    if (rc < 0) throw std::runtime_error(string(what) + ": " + kbhip_last_error());
}

// Undo log of the speculative steps: ints / doubles at an address, elements
// and sizes of heap vectors (by index: vectors may reallocate).
struct Journal {
    bool on = false;
    struct E {
        int kind;  // 0 int, 1 double, 2 vector size, 3 vector element
        void* p;
        int64_t i;
        double d;
    };
    vector<E> e;
    void set(int& x, int v) {
        if (on) e.push_back({0, &x, x, 0});
        x = v;
    }
    void set(double& x, double v) {
        if (on) e.push_back({1, &x, 0, x});
        x = v;
    }
    void rollback() {
        for (auto it = e.rbegin(); it != e.rend(); ++it) {
            switch (it->kind) {
                case 0: *(int*)it->p = (int)it->i; break;
                case 1: *(double*)it->p = it->d; break;
                case 2: ((vector<int>*)it->p)->resize((size_t)it->i); break;
                default: {
                    auto* v = (vector<int>*)it->p;
                    (*v)[(size_t)(it->i >> 32)] = (int)(uint32_t)it->i;
                }
            }
        }
        e.clear();
        on = false;
    }
};

// Go container/heap (heap.go up / down) over item ids with a less callback.
template <typename L>
struct GoHeap {
    vector<int> it;
    L less;
    Journal* jr;
    GoHeap(L l, Journal* j) : less(l), jr(j) {}
    void put(int pos, int v) {
        if (jr->on) jr->e.push_back({3, &it, ((int64_t)pos << 32) | (uint32_t)it[pos], 0});
        it[pos] = v;
    }
    void swap_at(int i, int j) {
        const int a = it[i], b = it[j];
        put(i, b);
        put(j, a);
    }
    bool Less(int i, int j) { return less(it[i], it[j]); }
    void push(int x) {
        if (jr->on) jr->e.push_back({2, &it, (int64_t)it.size(), 0});
        it.push_back(x);
        for (int j = (int)it.size() - 1;;) {  // up
            const int i = (j - 1) / 2;
            if (i == j || !Less(j, i)) break;
            swap_at(i, j);
            j = i;
        }
    }
    int pop() {
        const int n = (int)it.size() - 1;
        swap_at(0, n);
        for (int i = 0;;) {  // down(0, n)
            const int j1 = 2 * i + 1;
            if (j1 >= n || j1 < 0) break;
            int j = j1;
            if (j1 + 1 < n && Less(j1 + 1, j1)) j = j1 + 1;
            if (!Less(j, i)) break;
            swap_at(i, j);
            i = j;
        }
        const int x = it[n];
        if (jr->on) {
            jr->e.push_back({3, &it, ((int64_t)n << 32) | (uint32_t)x, 0});
            jr->e.push_back({2, &it, (int64_t)it.size(), 0});
        }
        it.pop_back();
        return x;
    }
    bool empty() const { return it.empty(); }
};

struct Pod {
    int prio;
    int64_t ts;
    double req[3];
    Status st;
    int job;  // -1: none
};
struct Job {
    string uid;
    int queue, min;
    int64_t ts;
    vector<int> tasks;
    int prio = 0, alloc_n = 0, cursor = 0;
    double drf_alloc[3] = {0, 0, 0}, drf = 0;
    bool built = false;
    vector<int32_t> pending;
};
struct Queue {
    string name;
    int weight;
    int64_t ts;
    double share = 0, deserved[3] = {0, 0, 0}, allocated[3] = {0, 0, 0}, request[3] = {0, 0, 0};
    bool attr = false;
};
struct Pop {
    int q = -1, k = -1, cursor = 0, ready = 0;
    bool operator==(const Pop& o) const { return q == o.q && k == o.k && cursor == o.cursor && ready == o.ready; }
};
struct Rec {
    int32_t pod, node, kind;  // kind 4 Allocated, 8 Pipelined (the oracle's log)
};

struct Host {
    vector<Pod> pods;
    vector<Job> jobs;
    vector<Queue> queues;
    double total[3] = {0, 0, 0};
    vector<int> job_order;  // 0 priority, 1 gang, 2 drf
    bool queue_prop = false, task_prio = false, gang_ready = false, drf_on = false, prop_on = false;
    Journal jr;

    explicit Host(const kbs::Snapshot& S) {
        // tiers: plugin names with their *Disabled flags (conf/scheduler_conf.go:20-54)
        auto pn = S.vec<int32_t>("conf_plugin_name");
        auto pt = S.vec<int32_t>("conf_plugin_tier");
        auto pf = S.vec<int32_t>("conf_plugin_flags");
        vector<size_t> order(pn.size());
        for (size_t i = 0; i < order.size(); ++i) order[i] = i;
        std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) { return pt[a] < pt[b]; });
        for (size_t i : order) {
            const string n = S.s(pn[i]);
            const int fl = pf[i];
            if ((n == "priority" || n == "gang" || n == "drf") && !(fl & KBS_DIS_JOBORDER))
                job_order.push_back(n == "priority" ? 0 : n == "gang" ? 1 : 2);
            if (n == "proportion" && !(fl & KBS_DIS_QUEUEORDER)) queue_prop = true;
            if (n == "priority" && !(fl & KBS_DIS_TASKORDER)) task_prio = true;
            if (n == "gang" && !(fl & KBS_DIS_JOBREADY)) gang_ready = true;
            drf_on = drf_on || n == "drf";
            prop_on = prop_on || n == "proportion";
        }
        auto qn = S.vec<int32_t>("q_name");
        auto qw = S.vec<int32_t>("q_weight");
        auto qt = S.vec<int64_t>("q_ts");
        for (size_t i = 0; i < qn.size(); ++i) queues.push_back(Queue{S.s(qn[i]), qw[i], qt[i]});
        auto qidx = [&](const string& n) {
            for (size_t i = 0; i < queues.size(); ++i)
                if (queues[i].name == n) return (int)i;
            return -1;
        };
        const char* ac[3] = {"n_alloc_cpu", "n_alloc_mem", "n_alloc_gpu"};
        for (int r = 0; r < 3; ++r)
            for (int64_t v : S.span<int64_t>(ac[r])) total[r] += (double)v;
        // jobs whose queue exists (cache.go:556-560) + shadow jobs of group-less pods
        auto jns = S.vec<int32_t>("j_ns");
        auto jnm = S.vec<int32_t>("j_name");
        auto jq = S.vec<int32_t>("j_queue");
        auto jmin = S.vec<int32_t>("j_min");
        auto jts = S.vec<int64_t>("j_ts");
        const int def_q = qidx("default");
        vector<int> job_of_row(jns.size(), -1);
        vector<Job> js;
        for (size_t k = 0; k < jns.size(); ++k) {
            const int q = qidx(S.s(jq[k]));
            if (q < 0) continue;
            job_of_row[k] = (int)js.size();
            Job j;
            j.uid = S.s(jns[k]) + "/" + S.s(jnm[k]);
            j.queue = q;
            j.min = jmin[k];
            j.ts = jts[k];
            js.push_back(std::move(j));
        }
        auto puid = S.span<int32_t>("p_uid");
        auto pjob = S.span<int32_t>("p_job");
        auto pnode = S.span<int32_t>("p_node");
        auto pph = S.span<uint8_t>("p_phase");
        auto pdel = S.span<uint8_t>("p_deleting");
        auto ppr = S.span<int32_t>("p_priority");
        auto pts = S.span<int64_t>("p_ts");
        auto coff = S.offs("p_ctr_off", puid.size());
        auto ccpu = S.span<int64_t>("c_cpu");
        auto cmem = S.span<int64_t>("c_mem");
        auto cgpu = S.span<int64_t>("c_gpu");
        const size_t P = puid.size();
        pods.resize(P);
        for (size_t i = 0; i < P; ++i) {
            Pod& p = pods[i];
            p.prio = ppr[i];
            p.ts = pts[i];
            p.req[0] = p.req[1] = p.req[2] = 0;
            int64_t r[3] = {0, 0, 0};
            for (int c = coff[i]; c < coff[i + 1]; ++c) { r[0] += ccpu[c]; r[1] += cmem[c]; r[2] += cgpu[c]; }
            for (int k = 0; k < 3; ++k) p.req[k] = (double)r[k];
            const bool del = !pdel.empty() && pdel[i];
            switch (pph[i]) {  // api/helpers.go:35-61
                case KBS_RUNNING: p.st = del ? RELEASING : RUNNING; break;
                case KBS_PENDING: p.st = del ? RELEASING : (pnode[i] >= 0 ? BOUND : PENDING); break;
                default: p.st = OTHER;
            }
            p.job = pjob[i] >= 0 ? job_of_row[pjob[i]] : -1;
            if (pjob[i] < 0 && def_q >= 0) {  // shadow PodGroup (job uid = pod uid, queue "default", min 1)
                Job j;
                j.uid = S.s(puid[i]);
                j.queue = def_q;
                j.min = 1;
                j.ts = 0;
                p.job = (int)js.size();
                js.push_back(std::move(j));
            }
        }
        // UID order (Go map iteration pinned to ascending UID: SURVEY Appendix B)
        vector<int> perm(js.size());
        for (size_t i = 0; i < perm.size(); ++i) perm[i] = (int)i;
        std::sort(perm.begin(), perm.end(), [&](int a, int b) { return js[a].uid < js[b].uid; });
        vector<int> inv(js.size());
        for (size_t i = 0; i < perm.size(); ++i) inv[perm[i]] = (int)i;
        jobs.resize(js.size());
        for (size_t i = 0; i < perm.size(); ++i) jobs[i] = std::move(js[perm[i]]);
        for (size_t i = 0; i < P; ++i)
            if (pods[i].job >= 0) {
                pods[i].job = inv[pods[i].job];
                jobs[pods[i].job].tasks.push_back((int)i);
            }
        for (Job& j : jobs) {
            j.prio = j.tasks.empty() ? 0 : pods[j.tasks.back()].prio;  // job_info.go:242 (last task added)
            for (int t : j.tasks)
                if (allocated_status(pods[t].st)) j.alloc_n++;
        }
        open_plugins();
    }

    static bool allocated_status(Status s) { return s == BOUND || s == RUNNING || s == ALLOCATED; }

    void open_plugins() {
        for (Job& j : jobs) {  // drf.go:65-82
            for (int t : j.tasks)
                if (allocated_status(pods[t].st))
                    for (int k = 0; k < 3; ++k) j.drf_alloc[k] += pods[t].req[k];
            j.drf = drf_share(j);
        }
        if (!prop_on) return;
        for (Job& j : jobs) {  // proportion.go:65-101
            Queue& q = queues[j.queue];
            q.attr = true;
            for (int t : j.tasks) {
                const Pod& p = pods[t];
                if (allocated_status(p.st)) {
                    for (int k = 0; k < 3; ++k) { q.allocated[k] += p.req[k]; q.request[k] += p.req[k]; }
                } else if (p.st == PENDING) {
                    for (int k = 0; k < 3; ++k) q.request[k] += p.req[k];
                }
            }
        }
        double remaining[3] = {total[0], total[1], total[2]};
        vector<bool> meet(queues.size(), false);
        for (;;) {  // proportion.go:104-136
            double tw = 0;
            for (size_t i = 0; i < queues.size(); ++i)
                if (queues[i].attr && !meet[i]) tw += queues[i].weight;
            if (tw == 0) break;
            double deserved[3] = {0, 0, 0};
            for (size_t i = 0; i < queues.size(); ++i) {
                Queue& q = queues[i];
                if (!q.attr || meet[i]) continue;
                const double ratio = q.weight / tw;
                for (int k = 0; k < 3; ++k) q.deserved[k] += remaining[k] * ratio;
                if (!less_equal(q.deserved, q.request)) {
                    for (int k = 0; k < 3; ++k) q.deserved[k] = std::min(q.deserved[k], q.request[k]);
                    meet[i] = true;
                }
                q.share = prop_share(q);
                for (int k = 0; k < 3; ++k) deserved[k] += q.deserved[k];
            }
            bool small = true;
            for (int k = 0; k < 3; ++k) {
                remaining[k] -= deserved[k];
                small = small && remaining[k] < kMin[k];
            }
            if (small) break;
        }
    }
    double drf_share(const Job& j) const {
        double s = 0;
        for (int k = 0; k < 3; ++k) s = std::max(s, share(j.drf_alloc[k], total[k]));
        return s;
    }
    static double prop_share(const Queue& q) {  // proportion.go:229-241
        double s = 0;
        for (int k = 0; k < 3; ++k) s = std::max(s, share(q.allocated[k], q.deserved[k]));
        return s;
    }

    // ---- order functions (framework/session_plugins.go:244-329) ----
    bool job_less(int l, int r) const {
        const Job& L = jobs[l];
        const Job& R = jobs[r];
        for (int p : job_order) {
            int c = 0;
            if (p == 0) {
                c = L.prio > R.prio ? -1 : L.prio < R.prio ? 1 : 0;
            } else if (p == 1) {
                const bool lr = L.alloc_n >= L.min, rr = R.alloc_n >= R.min;
                c = lr && rr ? 0 : lr ? 1 : rr ? -1 : 0;
            } else {
                c = L.drf == R.drf ? 0 : L.drf < R.drf ? -1 : 1;
            }
            if (c) return c < 0;
        }
        if (L.ts == R.ts) return l < r;  // UID order
        return L.ts < R.ts;
    }
    bool queue_less(int l, int r) const {
        const Queue& L = queues[l];
        const Queue& R = queues[r];
        if (queue_prop && L.share != R.share) return L.share < R.share;
        if (L.ts == R.ts) return l < r;  // name order
        return L.ts < R.ts;
    }
    bool overused(int q) const { return prop_on && less_equal(queues[q].deserved, queues[q].allocated); }

    void on_allocate(int t) {  // drf.go:134-143, proportion.go:200-210
        const Pod& p = pods[t];
        Job& j = jobs[p.job];
        if (drf_on) {
            for (int k = 0; k < 3; ++k) jr.set(j.drf_alloc[k], j.drf_alloc[k] + p.req[k]);
            jr.set(j.drf, drf_share(j));
        }
        if (prop_on) {
            Queue& q = queues[j.queue];
            for (int k = 0; k < 3; ++k) jr.set(q.allocated[k], q.allocated[k] + p.req[k]);
            jr.set(q.share, prop_share(q));
        }
    }

    // ---- the loop ----
    struct JL {
        const Host* h;
        bool operator()(int a, int b) const { return h->job_less(a, b); }
    };
    struct QL {
        const Host* h;
        bool operator()(int a, int b) const { return h->queue_less(a, b); }
    };
    GoHeap<QL>* qh = nullptr;
    vector<GoHeap<JL>> jh;
    vector<Rec> log;
    int64_t pops = 0;

    void build_pending(Job& j) {  // allocate.go:91-104 (BestEffort tasks skipped), TaskOrderFn order
        if (j.built) return;
        j.built = true;
        for (int t : j.tasks) {
            const Pod& p = pods[t];
            const bool best_effort = p.req[0] < kMin[0] && p.req[1] < kMin[1] && p.req[2] < kMin[2];
            if (p.st == PENDING && !best_effort) j.pending.push_back(t);
        }
        std::stable_sort(j.pending.begin(), j.pending.end(), [&](int a, int b) {
            const int pa = task_prio ? -pods[a].prio : 0, pb = task_prio ? -pods[b].prio : 0;
            if (pa != pb) return pa < pb;
            if (pods[a].ts != pods[b].ts) return pods[a].ts < pods[b].ts;
            return a < b;
        });
    }
    bool next_pop(Pop* out) {
        while (!qh->empty()) {
            const int q = qh->pop();
            if (overused(q)) continue;
            if (jh[q].empty()) continue;
            const int k = jh[q].pop();
            Job& j = jobs[k];
            build_pending(j);
            if (j.cursor >= (int)j.pending.size()) {
                qh->push(q);
                continue;
            }
            *out = Pop{q, k, j.cursor, j.alloc_n};
            return true;
        }
        return false;
    }
    // The decisions of pop p applied to the model (ssn.Allocate / ssn.Pipeline effects on the host).
    void apply(const Pop& p, int n_done, const int32_t* node, const uint8_t* kind, int stop, bool real) {
        Job& j = jobs[p.k];
        for (int i = 0; i < n_done; ++i) {
            if (node[i] < 0) continue;
            const int t = j.pending[p.cursor + i];
            if (real) {
                pods[t].st = kind[i] == KBHIP_ALLOCATED ? ALLOCATED : PIPELINED;
                log.push_back(Rec{t, node[i], kind[i] == KBHIP_ALLOCATED ? 4 : 8});
            }
            if (kind[i] == KBHIP_ALLOCATED) jr.set(j.alloc_n, j.alloc_n + 1);
            jr.set(j.prio, pods[t].prio);  // UpdateTaskStatus -> AddTaskInfo (job_info.go:242)
            on_allocate(t);
        }
        jr.set(j.cursor, p.cursor + n_done);
        if (stop == KBHIP_STOP_READY) jh[p.q].push(p.k);  // allocate.go:191-195
        qh->push(p.q);
    }
    // The predicted outcome: Allocated up to the gang stop (gang.go:63-66).
    void apply_predicted(const Pop& p) {
        const Job& j = jobs[p.k];
        const int n = (int)j.pending.size() - p.cursor;
        int k = 1, stop = KBHIP_STOP_READY;
        if (gang_ready) {
            const int need = j.min - p.ready;
            k = need <= 1 ? 1 : need;
            if (k > n) { k = n; stop = KBHIP_STOP_ALL; }
        }
        static thread_local vector<int32_t> node;
        static thread_local vector<uint8_t> kind;
        node.assign(k, 0);
        kind.assign(k, KBHIP_ALLOCATED);
        apply(p, k, node.data(), kind.data(), stop, false);
    }

    void start() {
        qh = new GoHeap<QL>(QL{this}, &jr);
        jh.assign(queues.size(), GoHeap<JL>(JL{this}, &jr));
        for (size_t k = 0; k < jobs.size(); ++k) {  // allocate.go:48-63
            qh->push(jobs[k].queue);
            jh[jobs[k].queue].push((int)k);
        }
    }
    ~Host() { delete qh; }

    const int32_t* ids(const Pop& p) const { return jobs[p.k].pending.data() + p.cursor; }
    int n_ids(const Pop& p) const { return (int)jobs[p.k].pending.size() - p.cursor; }

    void run_sync(kb_session* s) {
        start();
        vector<int32_t> node;
        vector<uint8_t> kind;
        Pop p;
        while (next_pop(&p)) {
            ++pops;
            const int n = n_ids(p);
            node.assign(n, -1);
            kind.assign(n, 0);
            int32_t nd = 0, stop = 0;
            check(kbhip_place_job(s, ids(p), n, gang_ready, jobs[p.k].min, p.ready, node.data(), kind.data(), &nd,
                                  &stop),
                  "kbhip_place_job");
            apply(p, nd, node.data(), kind.data(), stop, true);
        }
    }

    int64_t misses = 0;
    void run_async(kb_session* s, int depth) {
        start();
        auto submit = [&](const Pop& p) {
            const int64_t t = kbhip_place_job_submit(s, ids(p), n_ids(p), gang_ready, jobs[p.k].min, p.ready);
            check((int)std::max<int64_t>(t, -100), "kbhip_place_job_submit");
            return t;
        };
        std::deque<std::pair<int64_t, Pop>> q;  // outstanding tickets, oldest (the running pop) first
        Pop p;
        if (next_pop(&p)) q.push_back({submit(p), p});
        vector<int32_t> node;
        vector<uint8_t> kind;
        // predictions pay off only if the engine launches them ahead (it runs a pop it cannot
        // launch at submit — e.g. in a session with Backfilled nodes — inside its wait): after
        // 16 pops without a launch ahead, the loop stops predicting (same records either way)
        int64_t waited = 0;
        while (!q.empty()) {
            if (depth > 0 && waited == 16) {
                kbhip_stats st{};
                check(kbhip_get_stats(s, &st), "kbhip_get_stats");
                if (st.async_launched == 0) depth = 0;
            }
            // predictions behind the running pop, replayed on the journaled model, topped up to `depth`
            jr.on = true;
            Pop pc = q.front().second;
            size_t i = 1;
            for (; i < q.size(); ++i) {
                apply_predicted(pc);
                Pop np;
                if (!next_pop(&np) || !(np == q[i].second)) break;
                pc = np;
            }
            if (i < q.size()) {  // cannot happen for a deterministic model; withdraw what no longer follows
                check(kbhip_place_job_cancel(s, q[i].first), "kbhip_place_job_cancel");
                q.erase(q.begin() + i, q.end());
            } else {
                while ((int)q.size() <= depth) {
                    apply_predicted(pc);
                    Pop np;
                    if (!next_pop(&np)) break;
                    q.push_back({submit(np), np});
                    pc = np;
                }
            }
            jr.rollback();
            // the running pop's real results
            const auto cur = q.front();
            q.pop_front();
            const int n = n_ids(cur.second);
            node.assign(n, -1);
            kind.assign(n, 0);
            int32_t nd = 0, stop = 0;
            check(kbhip_place_job_wait(s, cur.first, node.data(), kind.data(), &nd, &stop), "kbhip_place_job_wait");
            ++pops;
            ++waited;
            apply(cur.second, nd, node.data(), kind.data(), stop, true);
            Pop nx;
            const bool has = next_pop(&nx);
            if (!q.empty() && has && nx == q.front().second) continue;
            if (!q.empty()) {
                check(kbhip_place_job_cancel(s, q.front().first), "kbhip_place_job_cancel");
                q.clear();
                ++misses;
            }
            if (has) q.push_back({submit(nx), nx});
        }
    }
};

uint64_t digest(const vector<Rec>& log) {  // FNV-1a over (pod, node, kind)
    uint64_t h = 1469598103934665603ull;
    for (const Rec& r : log)
        for (int32_t v : {r.pod, r.node, r.kind})
            for (int b = 0; b < 4; ++b) {
                h ^= (uint8_t)(v >> (8 * b));
                h *= 1099511628211ull;
            }
    return h;
}

double median(vector<double> v) {
    std::sort(v.begin(), v.end());
    return v.empty() ? 0 : v[v.size() / 2];
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s SNAPSHOT.kbs [--reps R] [--depth D] [--device K] [--modes m1,m2]\n", argv[0]);
        return 2;
    }
    const string path = argv[1];
    int reps = 3, depth = 2, device = 0;
    string modes = "allocate,sync,async", log_out;
    for (int i = 2; i + 1 < argc; i += 2) {
        const string a = argv[i];
        if (a == "--reps") reps = std::atoi(argv[i + 1]);
        else if (a == "--depth") depth = std::atoi(argv[i + 1]);
        else if (a == "--device") device = std::atoi(argv[i + 1]);
        else if (a == "--modes") modes = argv[i + 1];
        else if (a == "--log-out") log_out = argv[i + 1];
        else { std::fprintf(stderr, "unknown option %s\n", a.c_str()); return 2; }
    }
    try {
        kbs::Snapshot snap(path);
        string json = "{";
        bool equal = true;
        uint64_t ref = 0;
        bool have_ref = false;
        size_t pos = 0;
        while (pos <= modes.size()) {
            size_t e = modes.find(',', pos);
            if (e == string::npos) e = modes.size();
            const string m = modes.substr(pos, e - pos);
            pos = e + 1;
            if (m.empty()) continue;
            vector<double> ms;
            vector<Rec> log;
            int64_t pops = 0, misses = 0;
            kbhip_stats st{};
            for (int r = 0; r < reps; ++r) {
                kb_session* s = nullptr;
                check(kbhip_session_open_file(path.c_str(), device, &s), "kbhip_session_open_file");
                log.clear();
                double t_ms = 0;
                if (m == "allocate") {
                    const int64_t cap = (int64_t)snap.rows("p_uid") + 1;
                    vector<int32_t> pod(cap), node(cap);
                    vector<uint8_t> kind(cap);
                    const auto t0 = std::chrono::steady_clock::now();
                    const int n = kbhip_allocate(s, pod.data(), node.data(), kind.data(), cap);
                    t_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
                    check(n, "kbhip_allocate");
                    for (int i = 0; i < n; ++i) log.push_back(Rec{pod[i], node[i], kind[i] == KBHIP_ALLOCATED ? 4 : 8});
                } else if (m == "sync" || m == "async") {
                    Host h(snap);
                    const auto t0 = std::chrono::steady_clock::now();
                    if (m == "sync") h.run_sync(s);
                    else h.run_async(s, depth);
                    t_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
                    log.swap(h.log);
                    pops = h.pops;
                    misses = h.misses;
                } else {
                    throw std::runtime_error("unknown mode " + m);
                }
                check(kbhip_get_stats(s, &st), "kbhip_get_stats");
                check(kbhip_session_close(s), "kbhip_session_close");
                ms.push_back(t_ms);
            }
            const uint64_t d = digest(log);
            if (!have_ref) { ref = d; have_ref = true; }
            equal = equal && d == ref;
            if (!log_out.empty()) {
                FILE* f = std::fopen((log_out + "." + m + ".bin").c_str(), "wb");
                if (!f) throw std::runtime_error("cannot write " + log_out);
                std::fwrite(log.data(), sizeof(Rec), log.size(), f);
                std::fclose(f);
            }
            char buf[512];
            std::snprintf(buf, sizeof buf,
                          "%s\"%s\": {\"ms\": %.3f, \"ms_all\": [", json.size() > 1 ? ", " : "", m.c_str(), median(ms));
            json += buf;
            for (size_t i = 0; i < ms.size(); ++i) {
                std::snprintf(buf, sizeof buf, "%s%.3f", i ? ", " : "", ms[i]);
                json += buf;
            }
            std::snprintf(buf, sizeof buf,
                          "], \"placements\": %zu, \"digest\": \"%016llx\", \"pops\": %lld, \"batched_pops\": %lld, "
                          "\"sweeps\": %lld, \"async_launched\": %lld, \"async_retracted\": %lld, "
                          "\"async_cancelled\": %lld, \"host_misses\": %lld, \"spec_hits\": %lld}",
                          log.size(), (unsigned long long)d, (long long)(m == "allocate" ? st.pops : pops),
                          (long long)st.batched_pops, (long long)st.sweeps, (long long)st.async_launched,
                          (long long)st.async_retracted, (long long)st.async_cancelled, (long long)misses,
                          (long long)st.spec_hits);
            json += buf;
        }
        char tail[128];
        std::snprintf(tail, sizeof tail, ", \"depth\": %d, \"reps\": %d, \"equal\": %s}", depth, reps,
                      equal ? "true" : "false");
        json += tail;
        std::printf("%s\n", json.c_str());
        return equal ? 0 : 1;
    } catch (std::exception& e) {
        std::fprintf(stderr, "kbhost: %s\n", e.what());
        return 1;
    }
}
