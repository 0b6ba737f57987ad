// session.h — the host side of libkbhip.so, shared header of its parts
// (session/*.cpp, each its own translation unit): the host model and device
// buffers of a session (Session), the pools, the what-if batcher, the C-ABI
// handle, and the functions the parts call across files.
//
// The parts: 02_open (session open: KBS1 decode, dictionary encoding, task
// classes, upload of the node SoA to HBM), 03_pop (the per-pop device driver:
// batched pops, the persistent engine, tickets), 04_allocate (a C++ mirror of
// the Go framework's ordering plugins running the allocate / reclaim /
// preempt actions), 05_actions (backfill, the standalone sweeps, the actions'
// C-ABI entry points), 06_carry (session carry-over), 07_abi (the remaining
// C-ABI entry points).
//
// Reference map (pkg/scheduler unless noted):
//   session open      cache/cache.go:515-583 (Snapshot), framework/session.go:66-122,
//                     api/node_info.go:62-145 (NodeInfo.AddTask), api/job_info.go:239-326
//   ordering          util/priority_queue.go + Go container/heap, framework/session_plugins.go:
//                     244-329 (Job/Queue/TaskOrderFn), plugins/{priority,gang,drf,proportion}
//   allocate loop     actions/allocate/allocate.go:41-201
//   placement         the HIP kernels (kbhip_kernels.hip)
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <exception>
#include <map>
#include <memory>
#include <condition_variable>
#include <mutex>
#include <random>
#include <tuple>
#include <set>
#include <stdexcept>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#include <unistd.h>

#include "../../../include/kbhip.h"
#include "../../../include/kbsnap.h"
#include "../kbhip_affinity.h"
#include "../kbhip_engine.h"
#include "../kbhip_eval.h"
#include "../kbhip_internal.h"

using std::string;
using std::vector;

namespace kbhip {

inline thread_local string g_err;

struct Error : std::runtime_error {
    int code;
    Error(int c, const string& m) : std::runtime_error(m), code(c) {}
};

#define HIPCHK(x)                                                                            \
    do {                                                                                     \
        hipError_t e_ = (x);                                                                 \
        if (e_ != hipSuccess) throw Error(KBHIP_EDEVICE, string(#x) + ": " + hipGetErrorString(e_)); \
    } while (0)

enum St { Pending = 1, AOB = 2, Allocated = 4, Pipelined = 8, Binding = 16, Bound = 32, Running = 64,
          Releasing = 128, Succeeded = 256, Failed = 512, Unknown = 1024,
          Gone = 2048 };  // Gone: deleted from the cache between sessions (kbhip_session_carry_events)
inline bool allocated_status(int s) { return s == Bound || s == Binding || s == Running || s == Allocated; }

struct Dict {
    std::unordered_map<string, int> ids;
    vector<string> strs;
    int get(const string& s) {
        auto it = ids.find(s);
        if (it != ids.end()) return it->second;
        ids.emplace(s, (int)strs.size());
        strs.push_back(s);
        return (int)strs.size() - 1;
    }
};

inline bool parse_int64(const string& s, int64_t* out) {  // strconv.ParseInt(s, 10, 64)
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

struct R3 { int64_t c = 0, m = 0, g = 0; };
struct F3 {  // float64 Resource of the ordering plugins
    double c = 0, m = 0, g = 0;
    void add(const R3& r) { c += (double)r.c; m += (double)r.m; g += (double)r.g; }
    void addf(const F3& r) { c += r.c; m += r.m; g += r.g; }
    void subf(const F3& r) { c -= r.c; m -= r.m; g -= r.g; }
    void sub(const R3& r) { c -= (double)r.c; m -= (double)r.m; g -= (double)r.g; }
    bool less(const F3& rr) const { return c < rr.c && m < rr.m && g < rr.g; }  // Resource.Less (resource_info.go:156-158)
    double get(int k) const { return k == 0 ? c : k == 1 ? m : g; }
    bool less_equal(const F3& rr) const {  // resource_info.go:164-168
        return (c < rr.c || std::fabs(rr.c - c) < (double)kMinCPU) &&
               (m < rr.m || std::fabs(rr.m - m) < (double)kMinMem) &&
               (g < rr.g || std::fabs(rr.g - g) < (double)kMinGPU);
    }
    bool empty() const { return c < (double)kMinCPU && m < (double)kMinMem && g < (double)kMinGPU; }
};
inline double share(double l, double r) { return r == 0 ? (l == 0 ? 0 : 1) : l / r; }  // helpers.go:35-48

// Host worker threads for the session's parallel passes over pods / jobs: a
// process-wide budget — the machine's hardware threads, at most 16
// (KBHIP_HOST_THREADS overrides, 1..64) — shared by the sessions alive in the
// process (what-if sessions run 16 at a time from their own host threads: 16
// passes of 16 threads each oversubscribed the box's cores).
inline std::atomic<int> g_live_sessions{0};
inline int host_threads() {
    static const int budget = [] {
        if (const char* e = std::getenv("KBHIP_HOST_THREADS")) {
            const int v = std::atoi(e);
            if (v >= 1 && v <= 64) return v;
        }
        const int hw = (int)std::thread::hardware_concurrency();
        return std::max(1, std::min(16, hw));
    }();
    return std::max(1, budget / std::max(1, g_live_sessions.load(std::memory_order_relaxed)));
}
// The hardware queues HIP gives this process per device (GPU_MAX_HW_QUEUES, the
// runtime's default 4).  Streams beyond them share queues.
inline int hw_queues() {
    const char* e = std::getenv("GPU_MAX_HW_QUEUES");
    const int v = e ? std::atoi(e) : 0;
    return v > 0 ? v : 4;
}
// Peer mailboxes of shard ranks that are threads of one process on one device
// (kbhip_shard_connect_mailbox): a rank's placement kernel spins on the other
// ranks' flags, so two ranks' chained kernels queued in ONE hardware queue
// wait on each other for ever (the r04 rank-thread rehearsal aborted so).
// Each session creates 1 + kMaxDep streams; unless all k ranks' streams fit
// in the queues with room for two more (the null stream of the runtime's own
// copies, a StepBatcher or pooled stream), refuse (one process per GPU, k = 1,
// always fits).  Returns the reason, or "" when the group is safe.
inline std::string mailbox_queue_check(int k, int queues) {
    const int per = 1 + kMaxDep;
    if (k <= 1 || k * per + 2 <= queues) return "";
    return "kbhip_shard_connect_mailbox: " + std::to_string(k) + " shard ranks of this process share one device; their " +
           std::to_string(k * per) + " streams exceed the process's " + std::to_string(queues) +
           " hardware queues (GPU_MAX_HW_QUEUES) with room for the runtime's own, so two ranks' mailbox kernels could "
           "wait on each other inside one queue: run one process per GPU, or set GPU_MAX_HW_QUEUES >= " +
           std::to_string(k * per + 2) +
           " before the process starts";
}
// A token of this process, unique across hosts and containers (process ids and
// device ordinals repeat between containers): the mailbox records tell ranks
// of this process from others by it.
inline uint64_t process_token() {
    static const uint64_t tok = [] {
        std::random_device rd;
        uint64_t v = ((uint64_t)rd() << 32) ^ rd();
        v ^= (uint64_t)std::chrono::steady_clock::now().time_since_epoch().count() * 0x9e3779b97f4a7c15ull;
        return v ^ ((uint64_t)getpid() << 17);
    }();
    return tok;
}
struct HPod {
    int32_t uid_rank = 0;  // rank of the pod UID (pods are written sorted by UID: normally the index)
    int ns = -1;
    int status = Pending;
    int32_t priority = 0;
    int64_t ts = 0;
    bool backfill = false;
    bool critical = false;  // kube-system namespace or a system-*-critical priority class (conformance.go:40-45)
    bool node_rel = false;  // the node's copy stays Releasing after an unevict (statement.go:81-105)
    bool groupless = false; // no PodGroup: a shadow job of its own (cache/util.go:42-60)
    bool detached = false;  // the cache deleted this group-less pod: it keeps its shadow job, status and
                            // NodeName but is off the node (deletePod, event_handlers.go:119-165; kbsnap.h p_detached)
    R3 req, ireq;
    int64_t nzc = 0, nzm = 0;  // GetNonzeroRequests (kbhip_session_carry recomputes node rows from them)
    int job = -1;   // session job slot
    int cls = -1;   // device task class (pending tasks)
    int node = -1;  // current node
};
// The pod is in its node's task list (NodeInfo.Tasks): bound, not terminated
// (cache addTask, event_handlers.go:63-79), not taken off by a deletePod.
inline bool on_node_of(const HPod& p) {
    return p.node >= 0 && !p.detached && p.status != Succeeded && p.status != Failed;
}
// Placement 7's per-domain candidates (kbhip_batch.h place_aff): the sweep may
// keep only the best node of each domain of topology space S when every
// count the class's predicates read is indexed by S-domain (its EA pairs and
// PAA on space S) and an Allocated placement adds to one of those counts in
// its own domain (a self-matching anti-affinity term): a node beaten by one
// of its domain fails exactly when that one does, or ranks below it.  -1:
// the class keeps plain candidates.  space_ndom: domains per space.
inline int32_t dedup_space(const AffProgram& pg, const vector<int>& space_ndom) {
    if (pg.pa_space >= 0 || !pg.ipa.empty() || pg.pred_err) return -1;
    int32_t sp = pg.paa_space;
    vector<int32_t> offs;
    if (pg.paa_space >= 0) offs.push_back(pg.paa_cnt);
    for (size_t k = 0; k + 1 < pg.ea.size(); k += 2) {
        if (sp < 0) sp = pg.ea[k];
        if (pg.ea[k] != sp) return -1;
        offs.push_back(pg.ea[k + 1]);
    }
    if (sp < 0 || sp >= (int32_t)space_ndom.size() || space_ndom[sp] > kDedupMax) return -1;
    for (size_t k = 0; k + 2 < pg.upd.size(); k += 3)
        if (pg.upd[k] == UPD_CNT_ALLOC && pg.upd[k + 1] == sp &&
            std::find(offs.begin(), offs.end(), pg.upd[k + 2]) != offs.end())
            return sp;
    return -1;
}

struct HJob {  // session jobs are numbered in UID order
    int queue = -1;
    int32_t min_avail = 0, priority = 0;
    int32_t pg_priority = 0;  // the PodGroup's priority before any task's (JobInfo.SetPodGroup)
    bool shadow = false;      // shadow PodGroup of a group-less pod (cache/util.go:42-60)
    int64_t ts = 0;
    vector<int> tasks;
    vector<int> pending;  // pending non-BestEffort tasks in TaskOrderFn order (built at first pop)
    size_t cursor = 0;
    bool pending_built = false;
    bool maybe_pending = false;  // had a Pending non-BestEffort task at open (a superset of "has one now")
    int cnt_alloc = 0, cnt_aob = 0;
    int32_t fit[4] = {0, 0, 0, 0};  // NodesFitDelta of its last task that ended a pop unplaced / not ready:
                                    // walk nodes, negative cpu / memory / GPU deltas (JobInfo.FitError)
    F3 drf_alloc;
    double drf_share = 0;
};
struct HQueue {
    string name;
    int32_t rank = 0;  // rank of name among the session's queue names (QueueOrderFn's final string compare)
    int32_t weight = 1;
    int64_t ts = 0;
    bool has_attr = false;
    F3 deserved, allocated, request;
    double share = 0;
};
// Process-wide RCCL communicators kept across sessions: a scheduler (or the
// bench) opens a node-sharded session per scheduling cycle, and
// ncclCommInitRank (a bootstrap over sockets, a collective over every rank)
// costs more than a whole session.  A later session connecting with the same
// unique id, rank, world and device takes the communicator its predecessor
// left (one session uses a communicator at a time); kept until process exit.
struct CommPool {
    struct Entry {
        string id;
        int rank, world, device;
        ncclComm_t comm;
        bool busy;
    };
    std::mutex mu;
    vector<Entry> v;
    std::set<string> aborted;  // unique ids whose communicator was aborted: a new init with one would hang
    static CommPool& get() {
        static CommPool p;
        return p;
    }
};
inline ncclComm_t comm_acquire(const string& id, int rank, int world, int device) {
    CommPool& P = CommPool::get();
    std::lock_guard<std::mutex> lk(P.mu);
    for (size_t i = 0; i < P.v.size(); ++i) {
        auto& e = P.v[i];
        if (e.busy || e.id != id || e.rank != rank || e.world != world || e.device != device) continue;
        ncclResult_t ae = ncclSuccess;
        if (ncclCommGetAsyncError(e.comm, &ae) != ncclSuccess || ae != ncclSuccess) {  // broken: never reused
            (void)ncclCommAbort(e.comm);
            P.aborted.insert(e.id);
            P.v.erase(P.v.begin() + (long)i);
            return nullptr;
        }
        e.busy = true;
        return e.comm;
    }
    return nullptr;
}
inline void comm_add(const string& id, int rank, int world, int device, ncclComm_t c) {
    CommPool& P = CommPool::get();
    std::lock_guard<std::mutex> lk(P.mu);
    P.v.push_back({id, rank, world, device, c, true});
}
inline void comm_release(ncclComm_t c) {
    CommPool& P = CommPool::get();
    std::lock_guard<std::mutex> lk(P.mu);
    for (auto& e : P.v)
        if (e.comm == c) e.busy = false;
}
// A communicator whose session failed part-way (an ABI call returned an error
// while it was connected: the ranks' collective sequences may no longer
// match) or that reports an asynchronous error is aborted and leaves the pool.
inline void comm_drop(ncclComm_t c) {
    {
        CommPool& P = CommPool::get();
        std::lock_guard<std::mutex> lk(P.mu);
        for (size_t i = 0; i < P.v.size(); ++i)
            if (P.v[i].comm == c) {
                P.aborted.insert(P.v[i].id);
                P.v.erase(P.v.begin() + (long)i);
                break;
            }
    }
    (void)ncclCommAbort(c);
}
// A unique id serves one ncclCommInitRank bootstrap (its root listens once):
// after its communicator was aborted, the ranks connect with a new id.
inline bool comm_id_aborted(const string& id) {
    CommPool& P = CommPool::get();
    std::lock_guard<std::mutex> lk(P.mu);
    return P.aborted.count(id) != 0;
}

// Peer mailboxes (kbhip_shard_connect_mailbox): a process keeps its mailbox
// allocations (one per device, reused by the next session: its IPC handle,
// and so the peers' mappings of it, stay valid) and every peer mailbox it
// opened (hipIpcOpenMemHandle, keyed by the handle's bytes) for its lifetime —
// a mailbox is never freed while another process may still map it.
struct MboxPool {
    std::mutex mu;
    std::multimap<int, std::pair<Mailbox*, int>> free_own;  // device -> (mailbox, allocation kind)
    std::map<string, void*> opened;                         // peer handle bytes -> mapping
    static MboxPool& get() {
        static MboxPool p;
        return p;
    }
};

struct Plugin {
    string name;
    int flags = 0;
    std::map<string, string> args;
};

// Process-wide cache of device and pinned host allocations: a closed
// session's buffers serve the next session's (hipMalloc / hipHostMalloc cost
// up to milliseconds, hipFree synchronises the device).  A block is reused for
// a request of at least half its size; at most kCap bytes stay cached.
// KBHIP_NO_POOL=1 frees instead (diagnostic).
class MemPool {
  public:
    enum Kind { kDevice = 0, kPinned = 1, kPinnedMapped = 2 };
    static MemPool& get() {
        static MemPool pool;
        return pool;
    }
    // Returns a block of at least `bytes` on the current device; *cap_out = its size.
    void* take(Kind kind, size_t bytes, size_t* cap_out) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (!off_) {
            std::lock_guard<std::mutex> lk(mu_);
            auto it = free_.lower_bound(std::make_tuple(dev, (int)kind, bytes));
            if (it != free_.end() && std::get<0>(it->first) == dev && std::get<1>(it->first) == (int)kind &&
                std::get<2>(it->first) <= 2 * bytes) {
                void* p = it->second;
                *cap_out = std::get<2>(it->first);
                cached_ -= *cap_out;
                free_.erase(it);
                return p;
            }
        }
        void* p = nullptr;
        hipError_t e = kind == kDevice ? hipMalloc(&p, bytes)
                                       : hipHostMalloc(&p, bytes, kind == kPinned ? hipHostMallocDefault
                                                                                   : hipHostMallocMapped |
                                                                                         hipHostMallocCoherent);
        if (e != hipSuccess) {  // drop the cache and retry once
            trim();
            e = kind == kDevice ? hipMalloc(&p, bytes)
                                : hipHostMalloc(&p, bytes, kind == kPinned ? hipHostMallocDefault
                                                                           : hipHostMallocMapped | hipHostMallocCoherent);
            if (e != hipSuccess) throw Error(KBHIP_EDEVICE, kind == kDevice ? "hipMalloc failed" : "hipHostMalloc failed");
        }
        *cap_out = bytes;
        return p;
    }
    void give(Kind kind, void* p, size_t cap, int dev) {
        if (!p) return;
        {
            std::lock_guard<std::mutex> lk(mu_);
            if (!off_ && cached_ + cap <= kCap) {
                free_.emplace(std::make_tuple(dev, (int)kind, cap), p);
                cached_ += cap;
                return;
            }
        }
        release(kind, p);
    }
    // Non-blocking streams, reused likewise (hipStreamDestroy costs milliseconds).
    hipStream_t take_stream() {
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (!off_) {
            std::lock_guard<std::mutex> lk(mu_);
            auto it = streams_.find(dev);
            if (it != streams_.end()) {
                hipStream_t st = it->second;
                streams_.erase(it);
                return st;
            }
        }
        hipStream_t st = nullptr;
        if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess)
            throw Error(KBHIP_ENODEV, "hipStreamCreate failed");
        return st;
    }
    void give_stream(hipStream_t st, int dev) {  // st must be idle
        if (!st) return;
        if (off_) {
            (void)hipStreamDestroy(st);
            return;
        }
        std::lock_guard<std::mutex> lk(mu_);
        streams_.emplace(dev, st);
    }
    void trim() {
        std::lock_guard<std::mutex> lk(mu_);
        for (auto& kv : free_) release((Kind)std::get<1>(kv.first), kv.second);
        free_.clear();
        cached_ = 0;
    }

  private:
    MemPool() : off_(std::getenv("KBHIP_NO_POOL") != nullptr) {}
    static void release(Kind kind, void* p) {
        if (kind == kDevice) (void)hipFree(p);
        else (void)hipHostFree(p);
    }
    static constexpr size_t kCap = size_t(8) << 30;
    std::mutex mu_;
    std::multimap<std::tuple<int, int, size_t>, void*> free_;
    std::multimap<int, hipStream_t> streams_;
    size_t cached_ = 0;
    const bool off_;
};

// The one host array above glibc's mmap threshold (1M pods x 96 B): handed
// from a closed session to the next, so its pages stay mapped (no page faults
// at open, no munmap at close).
template <typename T>
struct SpareVec {
    std::mutex mu;
    vector<T> v;
    void take(vector<T>& out) {
        std::lock_guard<std::mutex> lk(mu);
        out.swap(v);
        v.clear();
        out.clear();
    }
    void take_keep(vector<T>& out) {  // the elements stay (the caller resets the ones it uses)
        std::lock_guard<std::mutex> lk(mu);
        out.swap(v);
        v.clear();
    }
    void give(vector<T>& in) {
        std::lock_guard<std::mutex> lk(mu);
        if (in.capacity() > v.capacity()) in.swap(v);
    }
};

struct DevBuf {  // device memory (pooled), or host memory for encode-only sessions
    void* p = nullptr;
    bool host = false;
    size_t cap = 0;
    int dev = 0;
    ~DevBuf() { release(); }
    void release() {
        if (p) { if (host) std::free(p); else MemPool::get().give(MemPool::kDevice, p, cap, dev); }
        p = nullptr;
    }
    template <typename T>
    T* alloc(size_t n, bool on_host = false) {
        release();
        host = on_host;
        size_t bytes = std::max<size_t>(n * sizeof(T), 16);
        if (host) {
            p = std::calloc(1, bytes);
            if (!p) throw Error(KBHIP_EINVAL, "out of host memory");
        } else {
            (void)hipGetDevice(&dev);
            p = MemPool::get().take(MemPool::kDevice, bytes, &cap);
        }
        return (T*)p;
    }
};

inline SpareVec<HPod>& spare_pods() {
    static SpareVec<HPod> sp;
    return sp;
}
// The job records and job UIDs likewise: their elements own heap buffers (a
// job's task list, a UID string — ≈ 400 k of them at C5, whose frees were
// most of a session's close); a session reuses its predecessor's elements and
// their capacity.  (The node task lists of the eviction actions are not
// reused: reclaim's walk over reused, scattered lists measured slower.)
inline SpareVec<HJob>& spare_jobs() {
    static SpareVec<HJob> sp;
    return sp;
}
inline SpareVec<string>& spare_uids() {
    static SpareVec<string> sp;
    return sp;
}

// ---------------------------------------------------------------------------
// batched pop launches: one k_pop_batch per job-pop chunk of one class.  Two
// result slots, so that the predicted next pop can be queued on the stream
// behind a running one (Allocator::speculate) and its results told apart.
// ---------------------------------------------------------------------------
struct BatchLaunch {
    int slot = 0;
    uint32_t epoch = 0;
    int cls = -1, m = 0;
    bool timed = false;
    hipStream_t st = nullptr;
    bool fit = false;  // placement 2: the kernel reports the FitDelta histogram of a task that found no node
    bool bf = false;   // placement 6 (Backfilled nodes): may end before its first task (n_done 0)
    bool aff = false;  // placement 7 (pod-affinity class): may end before its first task (n_done 0)
    bool engine = false;  // served by the persistent pop engine (no launch of its own)
};

// A job pop submitted through the asynchronous per-pop ABI
// (kbhip_place_job_submit): launched at submit time when it is one batched
// chunk and nothing deferred is ahead of it, else run at its wait.
// What kbhip_session_carry_snapshot's fast path keeps from the open: the
// dictionaries and class table a new pod's class is compiled against, and
// digests of the snapshot parts it does not re-derive (conf, node labels and
// taints).  Filled at the end of open_session.
struct CarryKeep {
    bool ok = false;                                     // a one-GPU session without pod affinity
    std::unordered_map<string, int> class_ids;           // class signature -> class
    vector<uint64_t> masks;                              // host copy of DevTables::masks
    vector<std::tuple<string, string, string>> taint_defs;  // taint ids (key, value, effect)
    Dict nss;                                            // namespace ids
    uint64_t conf_digest = 0, node_spec_digest = 0;
};

struct PopTicket {
    int64_t id = 0;
    bool launched = false;
    bool collected = false;  // place_job_wait: results read back (c_nd / c_st; rows in res_*_buf)
    int c_nd = 0, c_st = 0;
    BatchLaunch L;
    vector<int32_t> ids;
    int gang = 0, min_avail = 0, ready = 0;
};

struct Session {
    int device = 0;
    hipStream_t stream = nullptr;
    // host model
    vector<HPod> pods;
    vector<HJob> jobs;
    vector<HQueue> queues;
    vector<vector<Plugin>> tiers;
    bool drf_on = false, prop_on = false, gang_ready = false;
    F3 total;
    vector<R3> used;  // NodeInfo.Used mirror (for kbhip_read_nodes)
    vector<R3> h_alloc;                       // Allocatable (cpu, mem, gpu) per node (kbhip_session_carry)
    vector<int32_t> pod_port_off, pod_port_ids;  // host-port ids per pod, CSR (kbhip_session_carry)
    int64_t carry_bytes = 0;                     // bytes the last kbhip_session_carry uploaded
    int any_bf = 0;
    // placement 6 backoff per class: a batched pop of the class that placed nothing (the
    // fitting node lies below the list of walked nodes, or there is none) sends the class's
    // next pops to the general path directly (same records either way)
    vector<uint8_t> bf_backoff;
    // reclaim / preempt: each pod's job queue and MinAvailable (Allocator::compile_victims), valid
    // while pod_queue_gen == model_gen (every carry-over bumps model_gen)
    vector<int32_t> pod_queue, pod_min;
    uint64_t model_gen = 0, pod_queue_gen = ~0ull;
    bool plugins_opened = false;  // OnSessionOpen state of drf / proportion (once per session, every action sees it)
    // reclaim / preempt (kbhip_evict.hip): per-node order keys, their sorted copy, sort scratch, passing count
    DevBuf b_rank_keys, b_rank_sorted, b_rank_tmp, b_rank_cnt, b_rank_radix;
    DevBuf b_tab_idx;  // count-table deltas (flush_tables)
    DevBuf b_sweep_cnt;  // kbhip_sweep_scores' passing counts (8 counters, one 128-B line each)
    size_t rank_tmp_bytes = 0;
    uint64_t* h_rank = nullptr;  // pinned: [0] = count, then sorted keys
    size_t h_rank_cap = 0;
    int rank_first = 2048;  // sorted keys read back with the count (option "rank_first"); the rest on demand
    bool force_radix = false;  // option "rank_radix": the wide-range radix passes for every class (tests)
    bool bf_batch = true;      // option "bf_batch": batched pops (placement 6) in sessions with Backfilled nodes
    bool aff_batch = true;     // option "aff_batch": batched pops (placement 7) of anti-affinity classes
    bool aff_fence = true;     // option "aff_fence": placement-7 pops ordered behind overlapped ones on the
                               // device (ov_fence) instead of a host drain
    bool rank_group = false;   // option "rank_group": a what-if session batched with others (StepBatcher)
    hipEvent_t ev_pop = nullptr;  // this session's stream before a StepBatcher pop request
    vector<vector<int>> node_tasks;  // NodeInfo.Tasks (pod indices, pinned order), rebuilt per evicting action
    vector<R3> rel_delta;            // evictions not yet applied on the device: Releasing += per node
    vector<int32_t> rel_touched;     // nodes with a rel_delta entry, in first-touch order
    vector<uint8_t> rel_flag;        // node is in rel_touched
    DevBuf b_rel_nodes, b_rel_d;
    int32_t fallback = -1;  // lowest node index holding a session-placed pod (nodeorder.go:78-93)
    vector<int32_t> sess_cnt;  // per node: session-placed pods on it (fallback after an unpipeline)
    std::unique_ptr<AffinityModel> aff;       // pod (anti-)affinity model (kept for evictions / carry)
    CarryKeep keep;                           // kbhip_session_carry_snapshot's fast path
    std::map<int64_t, int32_t> tab_delta;     // pending count-table changes: idx >= 0 cnt, < 0 scalar (-1 - idx)
    // device
    Conf conf{};
    NodeCols nc{};
    DevTables tab{};
    vector<TaskClass> classes;
    vector<KeyFormat> class_kf;  // batched-path selection-key format per class
    vector<std::pair<int64_t, int64_t>> class_srange;  // score range [lo, hi] per class (no inter-pod term)
    bool keys32 = true;          // option "keys32": 32-bit keys where they fit
    int sweeps_cold = 0;         // option "time_sweeps_cold": kbhip_time_sweeps evicts the caches before each
                                 // launch (1: a 512 MB write, 2: a 512 MB read — no dirty lines left behind)
    DevBuf b_cols[20], b_labels, b_taints, b_ports, b_classes, b_terms, b_reqs, b_vals, b_valint, b_valok, b_masks,
        b_ctrl, b_walk, b_dom, b_aff_items, b_aff_cnt, b_aff_scalar, b_dd_max;
    PopCtrl* d_ctrl = nullptr;
    size_t h_out_cap = 0;
    DevBuf b_cand2, b_arrive;
    uint64_t* d_cand2 = nullptr;  // per-block candidate lists of the v2 batched kernel
    uint32_t* d_arrive = nullptr; // its block-arrival counter (reset by the last block)
    // option "overlap" = k (placement 2): batched pops rotate over k + 1
    // streams, up to k of them beside each other, chained on the device
    // (k_pop_batch_ov, PopLink); 0 = one stream, one pop kernel at a time
#ifdef KBHIP_STAMPS
    int overlap = 0;            // stamps are written by k_pop_batch only
#else
    int overlap = 1;            // deeper rotations measured slower at C4 (the sweep of pop e waits
#endif                          // for pop e-1's candidates, so k > 1 adds merge latency to the chain)
    hipStream_t ov_streams[kMaxDep + 1] = {};  // [0] is `stream`
    DevBuf b_cand_ov[kMaxDep + 1], b_arrive_ov[kMaxDep + 1], b_link;
    uint64_t* d_cand_ov[kMaxDep + 1] = {};
    uint32_t* d_arrive_ov[kMaxDep + 1] = {};
    PopLink* d_link = nullptr;
    uint32_t ov_seq = 0;        // sequence number of the last overlapped pop launched
    uint32_t msg_from = 1;      // PopLink row messages of pops from this one on are current (none drained since)
    // persistent pop engine (option "engine", kbhip_engine.hip): the batched pops of
    // eligible classes go to one resident kernel on `stream` through a pinned descriptor ring
#ifdef KBHIP_STAMPS
    bool engine = false;        // stamps are written by k_pop_batch only
#else
    bool engine = true;
#endif
    bool eng_running = false;   // its kernel was launched and has not been seen to end
    bool eng_claimed = false;   // this session holds its device's engine claim (eng_claim)
    // restart hysteresis (eng_eligible): a run stopped after few pops (C3: affinity pops between
    // short runs of engine-eligible ones) raises eng_backoff, the eligible pops in a row the
    // launched path takes before the engine starts again; a long run clears it
    int eng_backoff = 0, eng_streak = 0;
    bool eng_stop_cls = false;  // the pending eng_stop is for an engine-ineligible batched pop
    int64_t eng_run_pops0 = 0;  // stats.engine_pops when the current run started
    uint32_t eng_seq = 0;       // the last descriptor written (pop or exit)
    uint32_t eng_first = 1;     // the first pop of the next launch
    int eng_nw = 0, eng_npb = 0, eng_ng = 0;  // worker blocks (0: not sized yet, -1: the engine cannot run here)
    int eng_nw_opt = 0;         // option "engine_workers" (0: as many as stay resident)
    int eng_ng_opt = -1;        // option "engine_groups": merger blocks (0: the final merger reads the worker lists; -1: auto)
    bool eng_quick = true;      // option "engine_quick" = 0 (test mode): place_decide_wave without its fast path
    bool eng_lists = false;     // option "engine_lists": list mode when every eligible class fits (DESIGN.md §4.11;
                                // measured no faster than sweep mode at C4, so off by default)
    int eng_nown = 0;           // list mode: class-owner blocks (0: sweep mode)
    int eng_kshift = 0, eng_kidxmax = 0;  // ... and the 32-bit key format they write
    size_t eng_ncls = 0;        // classes when the engine was sized (a carry may add classes)
    vector<int32_t> eng_own_of; // class -> owner block (-1: none)
    DevBuf b_eng_own;           // owners' classes, key bases and FitDelta bits
    DevBuf b_eng;               // EngCtl + the worker and group lists
    EngCtl* d_eng_ctl = nullptr;
    EngPkg* d_eng_pkg = nullptr;
    uint64_t* d_eng_bl = nullptr;
    uint64_t* d_eng_gl = nullptr;
    uint64_t* h_eng = nullptr;  // pinned, mapped: [kEngHostRing][kEngDescWords] descriptor words, then the exit word
    uint64_t* dv_eng = nullptr; // ... as the device sees it
    size_t h_eng_cap = 0;
    DevBuf b_eng_tl;            // option "engine_timeline": the engine's event stamps (kEngTlSlots pops)
    uint64_t* d_eng_tl = nullptr;
    int32_t last_fit[4] = {0, 0, 0, 0};  // FitDelta histogram of the last pop's failing task
    bool last_fit_ok = false;            // ... computed in-kernel (else: fit_sync)
    DevBuf b_fit4;
    int32_t* d_fit4 = nullptr;
    vector<string> job_uid;              // by job slot (UID order)
    bool gang_close = false;             // the gang plugin is in the tiers (its OnSessionClose reports)
    uint8_t fit_set[kMaxDep + 2] = {};   // FitDelta counter set of the next launch, per stream (last: k_pop_batch)
    bool ov_pending = false;    // an overlapped pop may still run on either stream
    PopOutHost* h_out = nullptr;  // pinned, mapped: written by the device; 2 result slots
    void* d_out = nullptr;
    static constexpr int kSlots = 8;  // result slots: up to 1 + speculate batched pops in flight
    static_assert(1 + kMaxSpeculate < kSlots, "a result slot per batched pop in flight");
    uint32_t slot_epoch[kSlots] = {};  // granule tags per result slot
    int next_slot = 0;                // slot of the next batched launch (round robin)
    // HIP-event pairs around batched pop launches (option "time_every"): a ring, each
    // pair read back when it comes round again (long complete by then) or at the end
    static constexpr int kEvRing = 256;
    hipEvent_t ev_ring[kEvRing][2] = {};
    bool ev_used[kEvRing] = {};
    int ev_next = 0;
    hipEvent_t ev_run[2] = {};        // device span of kbhip_allocate
    double alloc_device_s = 0;
#ifdef KBHIP_STAMPS
    int speculate = 0;                // stamps are read per launch: no overlapped launches
#else
    int speculate = 4;                // predicted pops queued ahead of the running one (0..kMaxSpeculate)
#endif
    int32_t res_node_buf[kMaxChunk], res_kind_buf[kMaxChunk];
    std::deque<PopTicket> tickets;    // asynchronous per-pop ABI: outstanding pops, oldest first
    int64_t next_ticket = 0;
#ifdef KBHIP_STAMPS
    DevBuf b_stamps;
    uint64_t* d_stamps = nullptr;
    double phase[20] = {0};  // accumulated phase durations (us)
    int64_t phase_n = 0;
#endif
    uint64_t* d_walk = nullptr;
    // kbhip_set_option("debug_keys"): every per-task sweep's keys, for tests
    bool debug_keys = false;
    DevBuf b_dbg;
    uint64_t* d_dbg = nullptr;
    vector<uint64_t> dbg_keys;  // rows of 2 npad + 4: keys, raw ipa counts, ipa lo, ipa hi, fallback, max key
    vector<int32_t> dbg_pods;
    bool batched = true;
    int64_t time_every = 0;       // time every k-th sweep launch with HIP events (0 = off)
    int64_t sweep_launches = 0;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    hipEvent_t ev_nonov = nullptr;  // after a non-overlapped batched pop: the next overlapped one waits for it
    hipEvent_t ev_fence[kMaxDep + 1] = {};  // ov_fence: the overlap streams' ends, waited on by the session stream
    bool nonov_pending = false;
    double timed_ms = 0;          // summed duration of the timed sweep launches
    hipEvent_t ev_sweep[2] = {nullptr, nullptr};  // kbhip_sweep_scores' standalone sweep (time_every > 0)
    double host_launch_s = 0, host_wait_s = 0;
    int64_t timed_n = 0;
    kbhip_stats stats{};
    vector<std::tuple<int, int, int>> log;
    // node-array sharding: this session holds nodes [nc.base, nc.base + nc.n)
    int rank = 0, world = 1, n_total = 0;
    ncclComm_t comm = nullptr;                 // RCCL exchange (one GPU per rank)
    bool comm_pooled = false;                  // comm belongs to the process-wide CommPool
    bool comm_bad = false;                     // an ABI call failed while comm was connected (not reused)
    kbhip_allreduce_fn xfn = nullptr;          // or a host-side exchange callback
    void* xctx = nullptr;
    kbhip_allgather_fn xgfn = nullptr;         // host all-gather (batched pops of a shard session)
    void* xgctx = nullptr;
    DevBuf b_shard_send, b_shard_recv;         // this shard's ShardMsg / all of them (rank order)
    DevBuf b_gather;                           // gather_host's staging (RCCL)
    DevBuf b_ipa;                              // the per-task path's raw inter-pod counts (k_ipa_minmax -> sweep)
    int64_t* d_ipa = nullptr;
    ShardMsg* d_shard_send = nullptr;
    ShardMsg* d_shard_recv = nullptr;
    Mailbox* mbox_own = nullptr;               // peer mailboxes (kbhip_shard_connect_mailbox): this rank's,
    int mbox_kind = 0;                         // its allocation (0 uncached, 1 fine-grained, 2 default)
    Mailbox* mbox_peer[kMaxWorld] = {};        // and every rank's as mapped here (own included)
    uint32_t mbox_seq = 0;                     // sequence number of the last batched pop sent
    uint32_t sh_chained_seq = 0;               // the last overlapped shard pop (k_shard_sweep_ov), 0: none
    bool cu_masked = false;  // option "cu_split": the streams run on a share of the CUs (rehearsals)
    bool shard_overlap = false;                // option "shard_overlap": overlapped shard pops (with "overlap" > 0;
                                               // off: measured slower in the one-chip rehearsal)
    bool chain_fence = false;                  // device work ran on the session stream after the last drain
    vector<uint8_t> h_shard;                   // host staging of the host all-gather
    // encode-only sessions (kbhip_debug_encode): host copies of the compiled tables
    bool encode_only = false;
    string broken;  // non-empty: a carry failed part way; every call but close fails with this message
    vector<int32_t> h_dom, h_aff_cnt, h_aff_scalar, h_aff_items;
    int n_spaces = 0;
    size_t n_aff_cnt = 0, n_aff_scalar = 0;  // table sizes (device sessions read them back for tests)

    // Device side of the teardown: drain the streams, then hand streams, pinned
    // and device buffers back to the pool.  Idempotent.
    void release_device() {
        if (eng_running && h_eng) {  // the engine's exit descriptor, then the stream drains below
            const uint32_t sq = ++eng_seq;
            for (int i = 0; i < kEngDescWords; ++i)
                __atomic_store_n(&h_eng[(sq % kEngHostRing) * kEngDescWords + i],
                                 ((uint64_t)sq << 32) | (i == kDwFlags ? (uint64_t)kEngOpExit << 12 : 0),
                                 __ATOMIC_RELEASE);
            eng_running = false;
        }
        for (int k = 1; k <= kMaxDep; ++k)
            if (ov_streams[k]) (void)hipStreamSynchronize(ov_streams[k]);
        if (stream) (void)hipStreamSynchronize(stream);
        eng_unclaim();
        if (mbox_own) {  // back to the process's pool (peers may keep their mapping of it)
            MboxPool& P = MboxPool::get();
            std::lock_guard<std::mutex> lk(P.mu);
            P.free_own.emplace(device, std::make_pair(mbox_own, mbox_kind));
        }
        mbox_own = nullptr;
        for (auto& m : mbox_peer) m = nullptr;
        if (comm) {
            ncclResult_t ae = ncclSuccess;
            const bool async_err = ncclCommGetAsyncError(comm, &ae) != ncclSuccess || ae != ncclSuccess;
            if (comm_bad || async_err) comm_drop(comm);
            else if (comm_pooled) comm_release(comm);
            else (void)ncclCommDestroy(comm);
        }
        comm = nullptr;
        comm_pooled = false;
        comm_bad = false;
        for (hipEvent_t* e : {&ev0, &ev1, &ev_run[0], &ev_run[1], &ev_nonov, &ev_pop, &ev_sweep[0], &ev_sweep[1]})
            if (*e) { (void)hipEventDestroy(*e); *e = nullptr; }
        for (auto& e : ev_fence)
            if (e) { (void)hipEventDestroy(e); e = nullptr; }
        for (auto& pr : ev_ring)
            for (auto& e : pr)
                if (e) { (void)hipEventDestroy(e); e = nullptr; }
        if (h_out) MemPool::get().give(MemPool::kPinnedMapped, h_out, h_out_cap, device);
        if (h_eng) MemPool::get().give(MemPool::kPinnedMapped, h_eng, h_eng_cap, device);
        h_eng = nullptr;
        dv_eng = nullptr;
        b_eng.release();
        b_eng_own.release();
        b_eng_tl.release();
        d_eng_tl = nullptr;
        eng_nw = 0;
        if (h_rank) MemPool::get().give(MemPool::kPinned, h_rank, h_rank_cap, device);
        h_rank = nullptr;
        h_out = nullptr;
        if (cu_masked) {  // streams of option "cu_split" are this session's own
            for (int k = 1; k <= kMaxDep; ++k)
                if (ov_streams[k]) (void)hipStreamDestroy(ov_streams[k]);
            if (stream) (void)hipStreamDestroy(stream);
        } else {
            for (int k = 1; k <= kMaxDep; ++k) MemPool::get().give_stream(ov_streams[k], device);
            MemPool::get().give_stream(stream, device);
        }
        for (auto& st : ov_streams) st = nullptr;
        stream = nullptr;
        for (auto& b : b_cols) b.release();
        for (DevBuf* b : {&b_labels, &b_taints, &b_ports, &b_classes, &b_terms, &b_reqs, &b_vals, &b_valint, &b_valok,
                          &b_masks, &b_ctrl, &b_walk, &b_dom, &b_aff_items, &b_aff_cnt, &b_aff_scalar, &b_cand2,
                          &b_arrive, &b_link, &b_dbg, &b_fit4, &b_rank_keys, &b_rank_sorted, &b_rank_tmp, &b_rank_cnt,
                          &b_rank_radix,
                          &b_shard_send, &b_shard_recv, &b_tab_idx, &b_sweep_cnt, &b_dd_max})
            b->release();
        for (auto& b : b_cand_ov) b.release();
        for (auto& b : b_arrive_ov) b.release();
#ifdef KBHIP_STAMPS
        b_stamps.release();
#endif
    }
    ~Session();
    void eng_unclaim();  // (03_pop.cpp: the engine arbiter)
};

inline Session::~Session() {
    release_device();
    spare_pods().give(pods);
    spare_jobs().give(jobs);
    spare_uids().give(job_uid);
}

// Table upload: HBM on the session stream, or a host copy for encode-only
// sessions (kbhip_debug_encode / kbhip_debug_replay).
template <typename T>
inline T* upload(Session& S, DevBuf& b, const vector<T>& v) {
    T* d = b.alloc<T>(v.size(), S.encode_only);
    if (v.empty()) return d;
    if (S.encode_only) std::memcpy(d, v.data(), v.size() * sizeof(T));
    else HIPCHK(hipMemcpyAsync(d, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, S.stream));
    return d;
}

// ---------------------------------------------------------------------------
// What-if sessions batched per launch:
// sessions opened with option "rank_group", each driven by its own host
// thread, send their device requests — the allocate pops of sessions with
// Backfilled nodes or of pod-affinity classes (placements 6 / 7: one pop in
// flight per session), per-task chunks, and the reclaim / preempt node
// rankings — to this batcher, which serves every request pending in a lane as
// ONE multi-session launch per kind and device (k_pop_batch_multi, task k of
// every chunk in k_sweep_argmax_multi, the k_rank_*_multi sorts; blockIdx.y =
// session).  Pops are ordered by events after each session's earlier device
// work and before its later work; their results are the sessions' own
// granules.  Rankings complete before their requesters resume.  Combining:
// a request is issued at once with whatever else is pending in its lane;
// while a step is being launched new requests collect, and the first of
// their requesters to find the lane free issues them all — no session waits
// for another's host work.  (r03-r05 issued lockstep steps, once every member
// inside an action of the kind had a request in: 7.0-7.4 sessions/s at 16 in
// flight against 9.5-11.3 ungrouped and 9.6 combining, profiles/r06c_*;
// removed.)
// ---------------------------------------------------------------------------
struct StepBatcher {
    static StepBatcher& get() {
        static StepBatcher b;
        return b;
    }
    // kSweep requests (per-task chunks) go in the pop lane: the same sessions
    // (sessions inside allocate or backfill) send either
    enum Kind { kPop = 0, kRank = 1, kSweep = 2 };
    static int lane_of(int kind) { return kind == kRank ? 1 : 0; }
    struct Req {
        int kind = kPop;
        int device = 0;
        PopReq pop{};
        SweepReq sweep{};
        hipEvent_t before = nullptr;  // pop: recorded on the requester's stream (its earlier work)
        hipEvent_t after = nullptr;   // pop: recorded after the launch that served it
        RankDesc rank{};
        hipStream_t st = nullptr;     // rank: the requester's stream
        std::atomic<bool> done{false};
        hipError_t err = hipSuccess;
        int batch = 0;                // requests of its kind in the launch that served it
        std::chrono::steady_clock::time_point t0;  // when it was submitted (linger)
    };
    std::mutex mu;
    std::condition_variable cv;  // a step is out: requests done, the lane free
    // One lane per request lane kind: pops and chunks in one, rankings in the
    // other (a ranking waits for its launch; pops and chunks do not).
    struct Lane {
        vector<Req*> pending;
        bool busy = false;
    };
    Lane lane[2];
    int64_t steps = 0;
    // Test knob (option "group_linger_us", process-wide; 0 = off): a lane waits
    // until every grouped session has a request in it, or its oldest request
    // is that old, so that concurrent sessions' requests meet deterministically.
    std::atomic<int64_t> linger_us{0};
    std::atomic<int> sessions{0};  // live sessions with rank_group set
    static constexpr int kStreams = 4;
    struct Dev {
        hipStream_t sts[kStreams] = {};  // pop / chunk steps, round robin (a session has one request in
        int rr = 0;                      // flight, so consecutive steps need no order between them)
        hipStream_t st = nullptr;        // this step's
        vector<hipEvent_t> ring;
        size_t next = 0;
        RankDesc* h_desc = nullptr;  // pinned: the step's ranking descriptors, copied to d_desc
        RankDesc* d_desc = nullptr;  // device memory (kernels reading descriptors from mapped host memory
                                     // measured 1.6x slower at 64 sessions: profiles/r06m_c5_multi.jsonl)
        size_t cap_bytes = 0, n_cap = 0;
    };
    std::map<int, Dev> dev;

    // The requester issues at once if the lane is free, else it sleeps until
    // the current step is out and then one of the waiting requesters issues
    // what has collected.  (Spinning requesters — r03-r05 — took the host
    // cores the other sessions' host work needed: 16 sessions in flight are
    // host-bound.)
    void submit(Req& r) {
        const int l = lane_of(r.kind);
        r.t0 = std::chrono::steady_clock::now();
        std::unique_lock<std::mutex> lk(mu);
        lane[l].pending.push_back(&r);
        while (!r.done.load(std::memory_order_acquire)) {
            if (ready(l)) {
                issue(lk, l);
                continue;
            }
            if (linger_us.load(std::memory_order_relaxed) > 0) cv.wait_for(lk, std::chrono::microseconds(100));
            else cv.wait(lk);
        }
    }

  private:
    bool ready(int l) const {
        const Lane& L = lane[l];
        if (L.busy || L.pending.empty()) return false;
        const int64_t lg = linger_us.load(std::memory_order_relaxed);
        if (lg <= 0 || (int)L.pending.size() >= sessions.load(std::memory_order_relaxed)) return true;
        return std::chrono::steady_clock::now() - L.pending.front()->t0 >= std::chrono::microseconds(lg);
    }
    // One step of one lane: every pending request of that lane (the lock is
    // released while launching).
    void issue(std::unique_lock<std::mutex>& lk, int l) {
        Lane& L = lane[l];
        L.busy = true;
        vector<Req*> batch;
        batch.swap(L.pending);
        ++steps;
        // each device's streams and events, created under the lock (both lanes may issue at once)
        hipError_t e0 = hipSuccess;
        for (Req* q : batch)
            if (e0 == hipSuccess && (e0 = hipSetDevice(q->device)) == hipSuccess) (void)device(q->device, &e0);
        lk.unlock();
        std::map<int, vector<Req*>> by;  // device -> requests
        for (Req* q : batch) by[q->device].push_back(q);
        for (auto& kv : by) {
            if (e0 != hipSuccess) {
                for (Req* q : kv.second) q->err = e0;
                continue;
            }
            if (l == 1) {
                const hipError_t e = launch_ranks(kv.first, kv.second);
                for (Req* q : kv.second) { q->err = e; q->batch = (int)kv.second.size(); }
                continue;
            }
            vector<Req*> pops, sweeps;
            for (Req* q : kv.second) (q->kind == kSweep ? sweeps : pops).push_back(q);
            int pl = 0, sl = 0, sw_tasks = 0;
            hipError_t e = hipSetDevice(kv.first);
            if (e == hipSuccess) {
                Dev& D = device(kv.first, &e);
                if (e == hipSuccess) D.st = D.sts[D.rr++ % kStreams];  // this step's stream
            }
            if (e == hipSuccess && !pops.empty()) e = launch_pops(kv.first, pops, &pl);
            if (e == hipSuccess && !sweeps.empty()) e = launch_sweeps(kv.first, sweeps, &sl, &sw_tasks);
            if (e == hipSuccess) e = record_after(kv.first, kv.second);
            for (Req* q : pops) q->batch = (int)((pops.size() + std::max(pl, 1) - 1) / std::max(pl, 1));
            for (Req* q : sweeps) q->batch = (int)((sw_tasks + std::max(sl, 1) - 1) / std::max(sl, 1));
            for (Req* q : kv.second) q->err = e;
        }
        lk.lock();
        L.busy = false;
        // q may go away after this; requests that came in meanwhile are issued by their requesters
        for (Req* q : batch) q->done.store(true, std::memory_order_release);
        cv.notify_all();
    }
    Dev& device(int d, hipError_t* e) {
        Dev& D = dev[d];
        *e = hipSuccess;
        if (!D.st) {
            for (auto& s : D.sts)
                if ((*e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking)) != hipSuccess) return D;
            D.st = D.sts[0];
            D.ring.assign(64, nullptr);
            for (auto& ev : D.ring)
                if ((*e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) return D;
        }
        return D;
    }
    hipError_t launch_pops(int d, const vector<Req*>& b, int* launches) {
        hipError_t e = hipSetDevice(d);
        if (e != hipSuccess) return e;
        Dev& D = device(d, &e);
        if (e != hipSuccess) return e;
        vector<PopReq> qs;
        for (Req* q : b) {
            if ((e = hipStreamWaitEvent(D.st, q->before, 0)) != hipSuccess) return e;
            qs.push_back(q->pop);
        }
        int nl = 0;
        if ((e = launch_pop_batch_multi(qs.data(), (int)qs.size(), D.st, &nl)) != hipSuccess) return e;
        *launches = std::max(nl, 1);
        return hipSuccess;
    }
    // Task k of every chunk for k = 0, 1, ...: each session's tasks in order on
    // the one stream, the sessions side by side (*tasks: session-tasks swept).
    hipError_t launch_sweeps(int d, const vector<Req*>& b, int* launches, int* tasks) {
        hipError_t e = hipSetDevice(d);
        if (e != hipSuccess) return e;
        Dev& D = device(d, &e);
        if (e != hipSuccess) return e;
        vector<SweepReq> qs;
        int max_m = 0;
        for (Req* q : b) {
            if ((e = hipStreamWaitEvent(D.st, q->before, 0)) != hipSuccess) return e;
            qs.push_back(q->sweep);
            max_m = std::max(max_m, q->sweep.m);
            *tasks += q->sweep.m;
        }
        for (int k = 0; k < max_m; ++k)
            if ((e = launch_sweep_multi(qs.data(), (int)qs.size(), k, D.st, launches)) != hipSuccess) return e;
        return hipSuccess;
    }
    // Every request of the step follows its launches on the requester's stream.
    hipError_t record_after(int d, const vector<Req*>& b) {
        hipError_t e = hipSetDevice(d);
        if (e != hipSuccess) return e;
        Dev& D = device(d, &e);
        if (e != hipSuccess) return e;
        hipEvent_t ev = D.ring[D.next++ % D.ring.size()];
        if ((e = hipEventRecord(ev, D.st)) != hipSuccess) return e;
        for (Req* q : b) q->after = ev;
        return hipSuccess;
    }
    hipError_t launch_ranks(int d, const vector<Req*>& b) {
        hipError_t e = hipSetDevice(d);
        if (e != hipSuccess) return e;
        Dev& D = device(d, &e);
        if (e != hipSuccess) return e;
        if (b.size() > D.n_cap) {
            if (D.h_desc) MemPool::get().give(MemPool::kPinned, D.h_desc, D.cap_bytes, d);
            if (D.d_desc && (e = hipFree(D.d_desc)) != hipSuccess) return e;
            D.h_desc = nullptr;
            D.d_desc = nullptr;
            D.n_cap = std::max<size_t>(64, b.size());
            D.h_desc = (RankDesc*)MemPool::get().take(MemPool::kPinned, D.n_cap * sizeof(RankDesc), &D.cap_bytes);
            if ((e = hipMalloc((void**)&D.d_desc, D.n_cap * sizeof(RankDesc))) != hipSuccess) return e;
        }
        int max_nblk = 1;
        for (size_t i = 0; i < b.size(); ++i) {
            D.h_desc[i] = b[i]->rank;
            max_nblk = std::max(max_nblk, b[i]->rank.nblk);
        }
        hipStream_t st = b[0]->st;  // a stream of this device; every requester's inputs are in place
        if ((e = hipMemcpyAsync(D.d_desc, D.h_desc, b.size() * sizeof(RankDesc), hipMemcpyHostToDevice, st)) !=
            hipSuccess)
            return e;
        if ((e = launch_rank_sorted_multi(D.d_desc, (int)b.size(), max_nblk, st)) != hipSuccess) return e;
        return hipStreamSynchronize(st);  // (h_desc is reused by the next step)
    }
};

constexpr uint8_t kBfBackoff = 4;  // pops of a class sent to the general path after a placement-6 miss

// ---------------------------------------------------------------------------
// Functions defined in one part and called from others
// ---------------------------------------------------------------------------
void cu_split(Session& S, int part, int parts);
void class_key_format(const Session& S, const TaskClass& c, const vector<Term>& terms, int N, KeyFormat* kf_out,
                             std::pair<int64_t, int64_t>* range_out);
uint64_t conf_digest(const kbs::Snapshot& s);
uint64_t node_spec_digest(const kbs::Snapshot& s);
void open_session(Session& S, const kbs::Snapshot& s, int device, bool encode_only = false, int rank = 0,
                         int world = 1);
void fail_unsupported(const string& m);
void apply_results(Session& S, const int32_t* ids, int n, const int32_t* res_node, const int32_t* res_kind,
                          int32_t* out_node, uint8_t* out_kind);
bool batchable(const Session& S, int cls);
void collect_batched(Session& S, const BatchLaunch& L, int* n_done_out, int* stop_out, int32_t* res_node,
                            int32_t* res_kind);
void collect_tasks(Session& S, int slot, uint32_t epoch, int m, int* n_done, int* stop, int32_t* node,
                          int32_t* kind, int32_t* fit4);
void ctrl_setup(Session& S, int m, const int* cls, int ready, int min_avail, int gang, int mode, int slot,
                       uint32_t epoch);
void ev_harvest_all(Session& S);
void exchange(Session& S, void* dev, int op, int n = 1);
void gather_host(Session& S, const void* send, void* recv, size_t bytes);
void fit_allreduce(Session& S, int32_t* fit4);
void flush_tables(Session& S);
BatchLaunch launch_batched(Session& S, int cls, int m, int gang_mode, int min_avail, int ready_count);
void ov_quiesce(Session& S);
void ov_fence(Session& S);
int place_job(Session& S, const int32_t* ids, int n, int gang_mode, int min_avail, int ready_count,
                     int32_t* out_node, uint8_t* out_kind, int32_t* out_n_done, int32_t* out_stop);
int place_job_cancel(Session& S, int64_t ticket);
int64_t place_job_submit(Session& S, const int32_t* ids, int n, int gang_mode, int min_avail,
                                int ready_count);
int place_job_wait(Session& S, int64_t ticket, int32_t* out_node, uint8_t* out_kind, int32_t* out_n_done,
                          int32_t* out_stop);
void queue_target(Session& S, int pi, int sign);
void require_no_tickets(const Session& S);
void sess_placed(Session& S, int n, int d);
void sweep_chunk(Session& S, int m, const int* cls, bool defer, bool per_task = false);
int take_slot(Session& S, uint32_t* epoch);
void sweep_task(Session& S, int i, int cls, bool defer_visits = false);
void rank_buffers(Session& S);
void backfill_run(Session& S);
int sweep_scores(Session& S, int pod, uint64_t* out_keys);
double time_sweeps(Session& S, const int32_t* ids, int n);
double time_rank_multi(Session* const* ss, int n, const int32_t* ids, int reps, int evict, int mapped);
string fit_error(const HJob& j);
string gang_close_text(const Session& S);
int device_count();
void session_carry(Session& S, const int32_t* ev_pod = nullptr, const uint8_t* ev = nullptr, int64_t n_ev = 0);
void carry_snapshot(kb_session* ks, const kbs::Snapshot& s, const int32_t* old_pod, const int32_t* old_node);
int evict_action(kb_session* s, bool preempt, int32_t* out_pod, int32_t* out_node, uint8_t* out_kind,
                        int64_t cap);
void reopen_in_place(kb_session* ks, const kbs::Snapshot& s);
void allocate_run(Session& S);
void evict_run(Session& S, bool preempt);
void first_fit(Session& S, const int32_t* ids, int n, int32_t* out_node);

}  // namespace kbhip

struct kb_session {
    kb_session() { kbhip::g_live_sessions.fetch_add(1, std::memory_order_relaxed); }
    ~kb_session() {
        kbhip::g_live_sessions.fetch_sub(1, std::memory_order_relaxed);
        set_grouped(false);
    }
    void set_grouped(bool g) {  // the StepBatcher's count of live grouped sessions
        if (g != grouped) kbhip::StepBatcher::get().sessions.fetch_add(g ? 1 : -1, std::memory_order_relaxed);
        grouped = g;
    }
    bool grouped = false;
    kb_session(const kb_session&) = delete;
    kb_session& operator=(const kb_session&) = delete;
    kbhip::Session s;
};
inline void taint_comm(kb_session* s) {
    if (s && s->s.comm) s->s.comm_bad = true;
}
inline void check_usable(kb_session* s) {
    if (s && !s->s.broken.empty()) throw kbhip::Error(KBHIP_EINVAL, s->s.broken);
}

inline void check_log_args(kb_session* s, const int32_t* out_pod, const int32_t* out_node, const uint8_t* out_kind,
                           int64_t cap) {
    if (!s) throw kbhip::Error(KBHIP_EINVAL, "null session");
    if (s->s.encode_only) throw kbhip::Error(KBHIP_EINVAL, "encode-only session has no device state");
    if (cap < 0 || (cap > 0 && (!out_pod || !out_node || !out_kind)))
        throw kbhip::Error(KBHIP_EINVAL, "null output array with cap > 0");
}

#define ABI_GUARD(...)                                       \
    try {                                                    \
        __VA_ARGS__                                          \
    } catch (kbhip::Error & e) {                             \
        kbhip::g_err = e.what();                             \
        return e.code;                                       \
    } catch (std::exception & e) {                           \
        kbhip::g_err = e.what();                             \
        return KBHIP_EINVAL;                                 \
    } catch (...) {                                          \
        kbhip::g_err = "unknown error";                      \
        return KBHIP_EINVAL;                                 \
    }
// The same for calls on a session: a failure while the session's RCCL
// communicator is connected taints it (aborted at close, never pooled).
#define ABI_GUARD_S(sp, ...)                                 \
    try {                                                    \
        check_usable(sp);                                    \
        __VA_ARGS__                                          \
    } catch (kbhip::Error & e) {                             \
        kbhip::g_err = e.what();                             \
        taint_comm(sp);                                      \
        return e.code;                                       \
    } catch (std::exception & e) {                           \
        kbhip::g_err = e.what();                             \
        taint_comm(sp);                                      \
        return KBHIP_EINVAL;                                 \
    } catch (...) {                                          \
        kbhip::g_err = "unknown error";                      \
        taint_comm(sp);                                      \
        return KBHIP_EINVAL;                                 \
    }

