// kbhip_session.cpp — host side of libkbhip.so: session open (KBS1 decode,
// dictionary encoding, upload of the node SoA to HBM), the per-pop device
// driver (kbhip_place_job) and a C++ mirror of the Go framework's ordering
// plugins that runs the whole allocate action (kbhip_allocate).
//
// Reference map (pkg/scheduler unless noted):
//   session open      cache/cache.go:515-583 (Snapshot), framework/session.go:66-122,
//                     api/node_info.go:62-145 (NodeInfo.AddTask), api/job_info.go:239-326
//   ordering          util/priority_queue.go + Go container/heap, framework/session_plugins.go:
//                     244-329 (Job/Queue/TaskOrderFn), plugins/{priority,gang,drf,proportion}
//   allocate loop     actions/allocate/allocate.go:41-201
//   placement         the HIP kernels (kbhip_kernels.hip)
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
#include <tuple>
#include <set>
#include <stdexcept>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#include <unistd.h>

#include "../../include/kbhip.h"
#include "../../include/kbsnap.h"
#include "kbhip_affinity.h"
#include "kbhip_engine.h"
#include "kbhip_eval.h"
#include "kbhip_internal.h"

using std::string;
using std::vector;

namespace kbhip {

static thread_local string g_err;

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
static inline bool allocated_status(int s) { return s == Bound || s == Binding || s == Running || s == Allocated; }

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

static bool parse_int64(const string& s, int64_t* out) {  // strconv.ParseInt(s, 10, 64)
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
static double share(double l, double r) { return r == 0 ? (l == 0 ? 0 : 1) : l / r; }  // helpers.go:35-48

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
static inline bool on_node_of(const HPod& p) {
    return p.node >= 0 && !p.detached && p.status != Succeeded && p.status != Failed;
}
// Placement 7's per-domain candidates (kbhip_batch.h place_aff): the sweep may
// keep only the best node of each domain of topology space S when every
// count the class's predicates read is indexed by S-domain (its EA pairs and
// PAA on space S) and an Allocated placement adds to one of those counts in
// its own domain (a self-matching anti-affinity term): a node beaten by one
// of its domain fails exactly when that one does, or ranks below it.  -1:
// the class keeps plain candidates.  space_ndom: domains per space.
static int32_t dedup_space(const AffProgram& pg, const vector<int>& space_ndom) {
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
static ncclComm_t comm_acquire(const string& id, int rank, int world, int device) {
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
static void comm_add(const string& id, int rank, int world, int device, ncclComm_t c) {
    CommPool& P = CommPool::get();
    std::lock_guard<std::mutex> lk(P.mu);
    P.v.push_back({id, rank, world, device, c, true});
}
static void comm_release(ncclComm_t c) {
    CommPool& P = CommPool::get();
    std::lock_guard<std::mutex> lk(P.mu);
    for (auto& e : P.v)
        if (e.comm == c) e.busy = false;
}
// A communicator whose session failed part-way (an ABI call returned an error
// while it was connected: the ranks' collective sequences may no longer
// match) or that reports an asynchronous error is aborted and leaves the pool.
static void comm_drop(ncclComm_t c) {
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
static bool comm_id_aborted(const string& id) {
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
    bool rank_group = false;   // option "rank_group": a what-if session of the lockstep group (StepBatcher)
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
    uint32_t eng_seq = 0;       // the last descriptor written (pop or exit)
    uint32_t eng_first = 1;     // the first pop of the next launch
    int eng_nw = 0, eng_npb = 0, eng_ng = 0;  // worker blocks (0: not sized yet, -1: the engine cannot run here)
    int eng_nw_opt = 0;         // option "engine_workers" (0: as many as stay resident)
    int eng_ng_opt = -1;        // option "engine_groups": merger blocks (0: the final merger reads the worker lists; -1: auto)
    bool eng_quick = true;      // option "engine_quick" = 0 (test mode): place_decide_wave without its fast path
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
    ShardMsg* d_shard_send = nullptr;
    ShardMsg* d_shard_recv = nullptr;
    Mailbox* mbox_own = nullptr;               // peer mailboxes (kbhip_shard_connect_mailbox): this rank's,
    int mbox_kind = 0;                         // its allocation (0 uncached, 1 fine-grained, 2 default)
    Mailbox* mbox_peer[kMaxWorld] = {};        // and every rank's as mapped here (own included)
    uint32_t mbox_seq = 0;                     // sequence number of the last batched pop sent
    uint32_t sh_chained_seq = 0;               // the last overlapped shard pop (k_shard_sweep_ov), 0: none
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
        b_eng_tl.release();
        d_eng_tl = nullptr;
        eng_nw = 0;
        if (h_rank) MemPool::get().give(MemPool::kPinned, h_rank, h_rank_cap, device);
        h_rank = nullptr;
        h_out = nullptr;
        for (int k = 1; k <= kMaxDep; ++k) MemPool::get().give_stream(ov_streams[k], device);
        MemPool::get().give_stream(stream, device);
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
};

Session::~Session() {
    release_device();
    spare_pods().give(pods);
}

// Table upload: HBM on the session stream, or a host copy for encode-only
// sessions (kbhip_debug_encode / kbhip_debug_replay).
template <typename T>
static T* upload(Session& S, DevBuf& b, const vector<T>& v) {
    T* d = b.alloc<T>(v.size(), S.encode_only);
    if (v.empty()) return d;
    if (S.encode_only) std::memcpy(d, v.data(), v.size() * sizeof(T));
    else HIPCHK(hipMemcpyAsync(d, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, S.stream));
    return d;
}

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

static void fail_unsupported(const string& m) { throw Error(KBHIP_EUNSUPPORTED, m); }

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
static void class_key_format(const Session& S, const TaskClass& c, const vector<Term>& terms, int N, KeyFormat* kf_out,
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
static uint64_t conf_digest(const kbs::Snapshot& s) {
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
static uint64_t node_spec_digest(const kbs::Snapshot& s) {
    uint64_t h = 1469598103934665603ULL;
    const size_t N = s.rows("n_name");
    auto loff = s.offs("n_label_off", N), toff = s.offs("n_taint_off", N);
    auto lk = s.span<int32_t>("nl_key"), lv = s.span<int32_t>("nl_val");
    auto tk = s.span<int32_t>("nt_key"), tv = s.span<int32_t>("nt_val"), te = s.span<int32_t>("nt_effect");
    for (size_t i = 0; i < N; ++i) {
        for (int k = loff[i]; k < loff[i + 1]; ++k) { h = fnv_str(h, s.str(lk[k])); h = fnv_str(h, s.str(lv[k])); }
        h = fnv(h, "|", 1);
        for (int k = toff[i]; k < toff[i + 1]; ++k) {
            h = fnv_str(h, s.str(tk[k]));
            h = fnv_str(h, s.str(tv[k]));
            h = fnv_str(h, s.str(te[k]));
        }
        h = fnv(h, "#", 1);
    }
    return h;
}

static void open_session(Session& S, const kbs::Snapshot& s, int device, bool encode_only = false, int rank = 0,
                         int world = 1) {
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
        constexpr int kThreads = 8;
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
        constexpr int kThreads = 8;
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
    const int jth = srcs.size() < (1u << 14) ? 1 : 8;
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
            slot = (int)S.jobs.size();
            S.jobs.push_back(j);
            uid_src.push_back((int32_t)si);
        }
        if (src.row >= 0) row_slot[src.row] = slot;
        else shadow_slot[src.pod] = slot;
    }
    {
        const size_t nj = uid_src.size();
        S.job_uid.resize(nj);
        par_j([&](int t) {
            for (size_t k = nj * t / jth; k < nj * (t + 1) / jth; ++k) {
                const Src& src = srcs[uid_src[k]];
                S.job_uid[k] = src.b ? string(src.a) + "/" + src.b : string(src.a);
            }
        });
    }
    mark("jobs:slots");
    // Pass B (pod order): namespace and host-port dictionaries, node accumulation,
    // job slots (a job's tasks are its pods in pod order).
    vector<int32_t> ntask(S.jobs.size(), 0), slot_of(P);
    vector<AffPod> ap(P);  // the pod (anti-)affinity model's view of each pod
    std::unordered_map<int32_t, int> ns_by_off;  // strtab offset -> namespace id
    int32_t last_ns_off = -1, last_ns = -1;       // consecutive pods (one job) share a namespace
    for (int i = 0; i < P; ++i) {
        HPod& p = S.pods[i];
        if (pns[i] != last_ns_off) {
            auto it = ns_by_off.find(pns[i]);
            if (it == ns_by_off.end()) it = ns_by_off.emplace(pns[i], E.nss.get(s.s(pns[i]))).first;
            last_ns_off = pns[i];
            last_ns = it->second;
        }
        p.ns = last_ns;
        {
            const int slot = pjob[i] >= 0 ? row_slot[pjob[i]] : shadow_slot[i];
            p.job = slot;
            slot_of[i] = slot;
            if (slot >= 0) {
                ntask[slot]++;
                HJob& j = S.jobs[slot];
                j.priority = p.priority;  // JobInfo.AddTaskInfo: the last task's priority (job_info.go:242)
                if (allocated_status(p.status)) j.cnt_alloc++;
                if (p.status == AOB) j.cnt_aob++;
            }
            AffPod& a = ap[i];
            a.ns = p.ns;
            a.status = p.status;
            a.session_job = slot >= 0;
            const bool on_node = on_node_of(p);
            a.node = on_node ? p.node : -1;
            a.target = a.session_job && allocated_status(p.status) && on_node;
            a.pending = a.session_job && p.status == Pending;
        }
        S.pod_port_off[i] = (int32_t)S.pod_port_ids.size();
        for (int k = pco[i]; k < pco[i + 1]; ++k) {
            for (int q = cpo[k]; q < cpo[k + 1]; ++q) {
                if (ptpo[q] <= 0) continue;  // HostPortInfo.Add ignores port <= 0
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
        if (on_node_of(p)) {  // cache addTask -> NodeInfo.AddTask
            int n = p.node;
            if (p.backfill) { bf[n].c += p.req.c; bf[n].m += p.req.m; bf[n].g += p.req.g; }
            if (p.status == Releasing) {
                rel[n].c += p.req.c; rel[n].m += p.req.m; rel[n].g += p.req.g;
                idle[n].c -= p.req.c; idle[n].m -= p.req.m; idle[n].g -= p.req.g;
            } else {
                idle[n].c -= p.req.c; idle[n].m -= p.req.m; idle[n].g -= p.req.g;
            }
            S.used[n].c += p.req.c; S.used[n].m += p.req.m; S.used[n].g += p.req.g;
            podcnt[n]++;
            nzc[n] += p.nzc;
            nzm[n] += p.nzm;
            for (size_t k = (size_t)S.pod_port_off[i]; k < S.pod_port_ids.size(); ++k)  // pod i's run (still open)
                node_ports[n].push_back(S.pod_port_ids[k]);
        }
    }
    S.pod_port_off[P] = (int32_t)S.pod_port_ids.size();
    for (int i = 0; i < N; ++i) if (bf[i].c || bf[i].m || bf[i].g) S.any_bf = 1;
    S.h_alloc.resize(N);
    for (int i = 0; i < N; ++i) S.h_alloc[i] = R3{acpu[i], amem[i], agpu[i]};

    mark("pods:B");
    {
        for (size_t j = 0; j < S.jobs.size(); ++j) S.jobs[j].tasks.reserve(ntask[j]);
        for (int i = 0; i < P; ++i)
            if (slot_of[i] >= 0) {
                HJob& j = S.jobs[slot_of[i]];
                j.tasks.push_back(i);
                const HPod& p = S.pods[i];
                if (p.status == Pending && !(p.req.c < kMinCPU && p.req.m < kMinMem && p.req.g < kMinGPU))
                    j.maybe_pending = true;
            }
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
    int prev_pending = -1;
    for (int i = 0; i < P; ++i) {
        HPod& p = S.pods[i];
        if (p.status != Pending || p.job < 0) continue;
        if (prev_pending >= 0 && same_class_inputs(prev_pending, i)) {
            p.cls = S.pods[prev_pending].cls;
            prev_pending = i;
            continue;
        }
        prev_pending = i;
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
        E.tw = ((int)E.taint_defs.size() + 63) / 64;
        vector<uint64_t> tol(E.tw, 0);
        for (size_t t = 0; t < E.taint_defs.size(); ++t) {
            bool ok = false;
            for (int k = pto[i]; k < pto[i + 1] && !ok; ++k) {
                string key = s.s(tlk[k]), op = s.s(tlo[k]), val = s.s(tlv[k]), eff = s.s(tle[k]);
                if (!eff.empty() && eff != std::get<2>(E.taint_defs[t])) continue;
                if (!key.empty() && key != std::get<0>(E.taint_defs[t])) continue;
                if (op.empty() || op == "Equal") ok = val == std::get<1>(E.taint_defs[t]);
                else if (op == "Exists") ok = true;
            }
            if (ok) tol[t / 64] |= 1ULL << (t % 64);
        }
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
        if (it != class_ids.end()) { p.cls = it->second; continue; }
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
        S.classes.push_back(c);
        cls_pod.push_back(i);  // classes are created in pod order: i is the class's first pod
    }
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
    S.stats.nodes = N;
    S.stats.open_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

// ---------------------------------------------------------------------------
// cross-shard exchange of n 8-byte values in device memory:
// RCCL all-reduce on the session stream, or a host round trip through the
// caller's callback (tests: several ranks sharing one GPU over gloo).
// ---------------------------------------------------------------------------
// KBHIP_TRACE_SHARD=1: every collective of a shard session on stderr (diagnostic)
static const bool g_trace_shard = std::getenv("KBHIP_TRACE_SHARD") != nullptr;
static void exchange(Session& S, void* dev, int op, int n = 1) {
    if (S.world == 1) return;
    S.stats.collectives++;
    if (g_trace_shard)
        std::fprintf(stderr, "[shard %d] #%lld all-reduce op %d n %d\n", S.rank, (long long)S.stats.collectives, op, n);
    if (S.comm) {
        const ncclDataType_t dt = op == KBHIP_RED_MAX_U64 ? ncclUint64 : ncclInt64;
        const ncclRedOp_t ro = op == KBHIP_RED_MIN_I64 ? ncclMin : op == KBHIP_RED_SUM_I64 ? ncclSum : ncclMax;
        const ncclResult_t r = ncclAllReduce(dev, dev, n, dt, ro, S.comm, S.stream);
        if (r != ncclSuccess) throw Error(KBHIP_EDEVICE, string("ncclAllReduce: ") + ncclGetErrorString(r));
        return;
    }
    if (!S.xfn) throw Error(KBHIP_EINVAL, "sharded session is not connected (kbhip_shard_connect_*)");
    uint64_t v[8];
    if (n < 1 || n > 8) throw Error(KBHIP_EINVAL, "exchange of more than 8 values");
    HIPCHK(hipMemcpyAsync(v, dev, 8 * (size_t)n, hipMemcpyDeviceToHost, S.stream));
    HIPCHK(hipStreamSynchronize(S.stream));
    if (S.xfn(S.xctx, v, n, op) != 0) throw Error(KBHIP_EDEVICE, "shard exchange callback failed");
    HIPCHK(hipMemcpyAsync(dev, v, 8 * (size_t)n, hipMemcpyHostToDevice, S.stream));
    HIPCHK(hipStreamSynchronize(S.stream));
}

// The FitDelta counts of one task summed over the shards (in place; one GPU: nothing).
static void fit_allreduce(Session& S, int32_t* fit4) {
    if (S.world == 1) return;
    int64_t* d = (int64_t*)S.d_fit4 + 2;  // after the device counters (int32[4])
    int64_t h[4] = {fit4[0], fit4[1], fit4[2], fit4[3]};
    HIPCHK(hipMemcpyAsync(d, h, sizeof h, hipMemcpyHostToDevice, S.stream));
    exchange(S, d, KBHIP_RED_SUM_I64, 4);
    HIPCHK(hipMemcpyAsync(h, d, sizeof h, hipMemcpyDeviceToHost, S.stream));
    HIPCHK(hipStreamSynchronize(S.stream));
    for (int q = 0; q < 4; ++q) fit4[q] = (int32_t)h[q];
}

// The all-gather of a batched pop on a node-array shard: every rank's
// ShardMsg into d_shard_recv in rank order.  RCCL on the session stream (no
// host synchronisation), or the host callback around two copies.
static void shard_gather(Session& S) {
    const size_t bytes = sizeof(ShardMsg);
    S.stats.collectives++;
    if (g_trace_shard)
        std::fprintf(stderr, "[shard %d] #%lld all-gather (pop %lld)\n", S.rank, (long long)S.stats.collectives,
                     (long long)S.stats.pops);
    if (S.comm) {
        const ncclResult_t r = ncclAllGather(S.d_shard_send, S.d_shard_recv, bytes, ncclUint8, S.comm, S.stream);
        if (r != ncclSuccess) throw Error(KBHIP_EDEVICE, string("ncclAllGather: ") + ncclGetErrorString(r));
        return;
    }
    if (!S.xgfn) throw Error(KBHIP_EINVAL, "sharded session has no all-gather (kbhip_shard_connect_*)");
    S.h_shard.resize(bytes * (S.world + 1));
    uint8_t* send = S.h_shard.data() + bytes * S.world;
    HIPCHK(hipMemcpyAsync(send, S.d_shard_send, bytes, hipMemcpyDeviceToHost, S.stream));
    HIPCHK(hipStreamSynchronize(S.stream));
    if (S.xgfn(S.xgctx, send, S.h_shard.data(), (int64_t)bytes) != 0)
        throw Error(KBHIP_EDEVICE, "shard all-gather callback failed");
    HIPCHK(hipMemcpyAsync(S.d_shard_recv, S.h_shard.data(), bytes * S.world, hipMemcpyHostToDevice, S.stream));
    HIPCHK(hipStreamSynchronize(S.stream));  // the staging buffer is reused by the next pop
}

// One task of the per-task path: [IPA min/max prepass + exchange], sweep,
// [cross-shard max of the key + commit].
// defer_visits: the walk's GetAccessibleResource mutation as a grid-wide second
// kernel (worth it whenever some node may carry Backfilled resources).
static void sweep_task(Session& S, int i, int cls, bool defer_visits = false) {
    if (S.classes[cls].ipa_n > 0) {
        HIPCHK(launch_ipa_minmax(S.nc, S.tab, S.d_ctrl, i, S.stream));
        exchange(S, &S.d_ctrl->ipa_lo[i], KBHIP_RED_MIN_I64);
        exchange(S, &S.d_ctrl->ipa_hi[i], KBHIP_RED_MAX_I64);
    }
    HIPCHK(launch_sweep_argmax(S.conf, S.nc, S.tab, S.d_ctrl, i, S.d_walk, S.stream, S.world == 1, S.d_dbg,
                               defer_visits && S.world == 1));
    if (S.world > 1) {
        exchange(S, &S.d_ctrl->slot[i], KBHIP_RED_MAX_U64);
        HIPCHK(launch_commit_task(S.nc, S.tab, S.d_ctrl, i, S.d_walk, S.stream));
    }
}

// ---------------------------------------------------------------------------
// What-if sessions batched per launch:
// sessions opened with option "rank_group" = 1, each driven by its own host
// thread, join a process-wide lockstep group while they run an action.  Their
// device requests — the allocate pops of sessions with Backfilled nodes or of
// pod-affinity classes (placements 6 / 7: one pop in flight per session) and
// the reclaim / preempt node rankings — go to this batcher, which issues a
// STEP of a kind once every member inside an action of that kind (allocate for
// pops; reclaim / preempt for rankings) has a request in (a member doing other
// work in its action — a per-task sweep, host bookkeeping — is waited for; one
// that leaves its action leaves that lane): one multi-session launch per kind and device
// (k_pop_batch_multi / the k_rank_*_multi sorts, blockIdx.y = session), up to
// kPopMulti pops per launch.  Pops are ordered by events after each session's
// earlier device work and before its later work; their results are the
// sessions' own granules.  Rankings complete before their requesters resume.
// No timeouts: the sessions step together.
// ---------------------------------------------------------------------------
struct StepBatcher {
    static StepBatcher& get() {
        static StepBatcher b;
        return b;
    }
    // kSweep requests (per-task chunks) step in the pop lane: the same members
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
    };
    std::mutex mu;
    // One lockstep lane per request kind: the members inside allocate step
    // their pops together, the members inside reclaim / preempt their rankings;
    // a session busy in another action's host work never holds a lane up.
    struct Lane {
        vector<Req*> pending;
        int members = 0;  // grouped sessions inside an action of this kind
        bool busy = false;
    };
    Lane lane[2];
    int64_t steps = 0;
    struct Dev {
        hipStream_t st = nullptr;  // pop launches
        vector<hipEvent_t> ring;
        size_t next = 0;
        RankDesc* h_desc = nullptr;  // pinned, mapped: the ranking kernels read the descriptors in place
        void* d_desc = nullptr;
        size_t cap_bytes = 0, n_cap = 0;
    };
    std::map<int, Dev> dev;

    void join(int kind) {
        std::lock_guard<std::mutex> lk(mu);
        ++lane[lane_of(kind)].members;
    }
    void leave(int kind) {
        std::unique_lock<std::mutex> lk(mu);
        const int l = lane_of(kind);
        --lane[l].members;
        if (ready(l)) issue(lk, l);
    }
    // The member whose request (or departure) completes the step issues it;
    // the others spin on their own request (a step is microseconds of host
    // work: a sleeping wait would cost every member a wake-up per step).
    void submit(Req& r) {
        {
            std::unique_lock<std::mutex> lk(mu);
            const int l = lane_of(r.kind);
            lane[l].pending.push_back(&r);
            if (ready(l)) issue(lk, l);
        }
        for (long spin = 0; !r.done.load(std::memory_order_acquire); ++spin) {
            if ((spin & 1023) == 1023) std::this_thread::yield();
            else __builtin_ia32_pause();
        }
    }

  private:
    bool ready(int l) const {
        const Lane& L = lane[l];
        return !L.busy && !L.pending.empty() && (int)L.pending.size() >= L.members;
    }
    // One step of one lane: every pending request of that lane (the lock is
    // released while launching).
    void issue(std::unique_lock<std::mutex>& lk, int l) {
        Lane& L = lane[l];
        L.busy = true;
        vector<Req*> batch;
        batch.swap(L.pending);
        ++steps;
        lk.unlock();
        std::map<int, vector<Req*>> by;  // device -> requests
        for (Req* q : batch) by[q->device].push_back(q);
        for (auto& kv : by) {
            if (l == 1) {
                const hipError_t e = launch_ranks(kv.first, kv.second);
                for (Req* q : kv.second) { q->err = e; q->batch = (int)kv.second.size(); }
                continue;
            }
            vector<Req*> pops, sweeps;
            for (Req* q : kv.second) (q->kind == kSweep ? sweeps : pops).push_back(q);
            int pl = 0, sl = 0, sw_tasks = 0;
            hipError_t e = pops.empty() ? hipSuccess : launch_pops(kv.first, pops, &pl);
            if (e == hipSuccess && !sweeps.empty()) e = launch_sweeps(kv.first, sweeps, &sl, &sw_tasks);
            if (e == hipSuccess) e = record_after(kv.first, kv.second);
            for (Req* q : pops) q->batch = (int)((pops.size() + std::max(pl, 1) - 1) / std::max(pl, 1));
            for (Req* q : sweeps) q->batch = (int)((sw_tasks + std::max(sl, 1) - 1) / std::max(sl, 1));
            for (Req* q : kv.second) q->err = e;
        }
        lk.lock();
        L.busy = false;
        for (Req* q : batch) q->done.store(true, std::memory_order_release);  // q may go away after this
        if (ready(l)) issue(lk, l);  // requests that came in while this step was being launched
    }
    Dev& device(int d, hipError_t* e) {
        Dev& D = dev[d];
        *e = hipSuccess;
        if (!D.st) {
            if ((*e = hipStreamCreateWithFlags(&D.st, hipStreamNonBlocking)) != hipSuccess) return D;
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
            if (D.h_desc) MemPool::get().give(MemPool::kPinnedMapped, D.h_desc, D.cap_bytes, d);
            D.n_cap = std::max<size_t>(64, b.size());
            D.h_desc = (RankDesc*)MemPool::get().take(MemPool::kPinnedMapped, D.n_cap * sizeof(RankDesc), &D.cap_bytes);
            if ((e = hipHostGetDevicePointer(&D.d_desc, D.h_desc, 0)) != hipSuccess) return e;
        }
        int max_nblk = 1;
        for (size_t i = 0; i < b.size(); ++i) {
            D.h_desc[i] = b[i]->rank;
            max_nblk = std::max(max_nblk, b[i]->rank.nblk);
        }
        hipStream_t st = b[0]->st;  // a stream of this device; every requester's inputs are in place
        if ((e = launch_rank_sorted_multi((const RankDesc*)D.d_desc, (int)b.size(), max_nblk, st)) != hipSuccess)
            return e;
        return hipStreamSynchronize(st);
    }
};

// A grouped session inside an action (StepBatcher member).
struct GroupScope {
    bool on;
    int kind;
    GroupScope(bool o, int k) : on(o), kind(k) {
        if (on) StepBatcher::get().join(kind);
    }
    ~GroupScope() {
        if (on) StepBatcher::get().leave(kind);
    }
};

// The sweeps of a per-task chunk (tasks 0 .. m-1 of the control block): one
// k_sweep_argmax launch per task, or, for a what-if session of the lockstep
// group, one request that the StepBatcher serves together with the group's
// other chunks (k_sweep_argmax_multi: task k of every chunk in one launch).
// Classes with inter-pod priority terms (their k_ipa_minmax prepass) and
// debug-key sessions keep the per-task launches.
static void sweep_chunk(Session& S, int m, const int* cls, bool defer, bool per_task = false) {
    S.stats.pertask_sweeps += m;
    bool group = S.rank_group && S.world == 1 && !S.d_dbg && !per_task;
    for (int i = 0; i < m && group; ++i) group = S.classes[cls[i]].ipa_n == 0;
    if (!group) {
        for (int i = 0; i < m; ++i) sweep_task(S, i, cls[i], defer);
        return;
    }
    StepBatcher::Req r;
    r.kind = StepBatcher::kSweep;
    r.sweep = SweepReq{S.conf, S.nc, S.tab, S.d_ctrl, S.d_walk, m, defer ? 1 : 0};
    r.device = S.device;
    if (!S.ev_pop) HIPCHK(hipEventCreateWithFlags(&S.ev_pop, hipEventDisableTiming));
    HIPCHK(hipEventRecord(S.ev_pop, S.stream));  // the control block's setup is in
    r.before = S.ev_pop;
    StepBatcher::get().submit(r);
    HIPCHK(hipSetDevice(S.device));
    HIPCHK(r.err);
    HIPCHK(hipStreamWaitEvent(S.stream, r.after, 0));  // this session's later work follows the launches
    S.stats.sweep_requests++;
    S.stats.sweep_batch_sum += r.batch;
}

// ---------------------------------------------------------------------------
// persistent pop engine (kbhip_engine.hip).  Eligible batched
// pops are written as descriptors into a pinned ring; one resident kernel on
// the session stream serves them in order and reports through the usual
// result slots.  It runs until an exit descriptor (eng_stop: before any other
// device work, from ov_drain) or until it has been idle for a second (then
// eng_poll restarts it for descriptors written meanwhile).
// ---------------------------------------------------------------------------
static void eng_size(Session& S) {
    S.eng_nw = -1;
    const int N = S.nc.n;
    if (S.encode_only || S.world != 1 || N < 1) return;
    int cus = 0, bpc = 0;
    HIPCHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, S.device));
    HIPCHK(engine_occupancy(&bpc));
    const int resident = cus * bpc;  // every block of the grid must be resident at once
    int nw = std::min(kEngWorkersMax, resident - kEngMaxGroups - 3);  // + final merger, placer, dispatcher
    if (S.eng_nw_opt > 0) nw = std::min(nw, S.eng_nw_opt);
    nw = std::min(nw, std::max(1, (N + 63) / 64));  // at least 64 nodes per worker
    if (nw < 1) return;
    const int npb = (N + nw - 1) / nw;
    if (npb > kEngMaxNpb) return;
    const int ng = S.eng_ng_opt >= 0 ? std::min(S.eng_ng_opt, nw) : std::min(kEngMaxGroups, nw);
    const size_t lists = (size_t)kEngSlots * (nw + ng) * kEngListWords;
    static_assert(sizeof(EngCtl) % 256 == 0 && sizeof(EngPkg) % 256 == 0, "engine buffers stay line-aligned");
    const size_t words = (sizeof(EngCtl) + kEngSlots * sizeof(EngPkg)) / 8 + lists;
    char* d = (char*)S.b_eng.alloc<uint64_t>(words);
    S.d_eng_ctl = (EngCtl*)d;
    S.d_eng_pkg = (EngPkg*)(d + sizeof(EngCtl));
    S.d_eng_bl = (uint64_t*)(d + sizeof(EngCtl) + kEngSlots * sizeof(EngPkg));
    S.d_eng_gl = S.d_eng_bl + (size_t)kEngSlots * nw * kEngListWords;
    HIPCHK(hipMemsetAsync(d, 0, words * 8, S.stream));  // every tag 0: no pop has that sequence number
    if (!S.h_eng) {
        S.h_eng = (uint64_t*)MemPool::get().take(MemPool::kPinnedMapped, (kEngHostRing * kEngDescWords + 8) * sizeof(uint64_t),
                                                 &S.h_eng_cap);
        std::memset(S.h_eng, 0, (kEngHostRing * kEngDescWords + 8) * sizeof(uint64_t));
        void* dv = nullptr;
        HIPCHK(hipHostGetDevicePointer(&dv, S.h_eng, 0));
        S.dv_eng = (uint64_t*)dv;
        S.eng_seq = 0;
        S.eng_first = 1;
    }
    S.eng_nw = nw;
    S.eng_npb = npb;
    S.eng_ng = ng;
    S.stats.engine_workers = nw;
}

// A batched pop the engine can serve: one GPU, no Backfilled nodes, a class
// without pod affinity, host ports or the backfill annotation, 32-bit keys
// and placement entries (the engine's single placement instantiation).
static bool eng_eligible(Session& S, int cls, const KeyFormat& kf) {
    if (!S.engine || S.world != 1 || S.any_bf || S.rank_group || S.encode_only) return false;
    const TaskClass& c = S.classes[cls];
    if (c.aff || c.has_ports || c.backfill || !kf.use32 || !kf.ent32) return false;
    if (S.eng_nw == 0) eng_size(S);
    return S.eng_nw > 0;
}

static uint64_t* eng_exit_word(Session& S) { return S.h_eng + kEngHostRing * kEngDescWords; }

static void eng_write(Session& S, uint32_t seq, const uint32_t* w) {
    uint64_t* slot = S.h_eng + (size_t)(seq % kEngHostRing) * kEngDescWords;
    for (int i = 0; i < kEngDescWords; ++i) __atomic_store_n(&slot[i], ((uint64_t)seq << 32) | w[i], __ATOMIC_RELEASE);
}

static void eng_start(Session& S) {
    HIPCHK(hipMemsetAsync(S.d_eng_ctl, 0, sizeof(EngCtl), S.stream));  // done 0, no error, ring tags 0
    __atomic_store_n(eng_exit_word(S), (uint64_t)0, __ATOMIC_RELEASE);
    EngArgs A{};
    A.ctl = S.d_eng_ctl;
    A.blists = S.d_eng_bl;
    A.glists = S.d_eng_gl;
    A.pkg = S.d_eng_pkg;
    A.hring = S.dv_eng;
    A.hexit = S.dv_eng + kEngHostRing * kEngDescWords;
    A.out = S.d_out;
    A.first = S.eng_first;
    A.nw = S.eng_nw;
    A.npb = S.eng_npb;
    A.ng = S.eng_ng;
    A.tl = S.d_eng_tl;
    A.quick = S.eng_quick ? 1 : 0;
    HIPCHK(launch_engine(S.conf, S.nc, S.tab, A, S.stream));
    S.eng_running = true;
    S.stats.engine_launches++;
}

// The engine's kernel ended (its exit word, after a stream sync): check its
// error word; the next launch starts at the first pop it did not serve.
static void eng_ended(Session& S) {
    HIPCHK(hipStreamSynchronize(S.stream));
    S.eng_running = false;
    uint32_t err = 0;
    HIPCHK(hipMemcpy(&err, &S.d_eng_ctl->err, sizeof(err), hipMemcpyDeviceToHost));
    const uint64_t x = __atomic_load_n(eng_exit_word(S), __ATOMIC_ACQUIRE);
    if (err || !(x & (1ull << 41))) throw Error(KBHIP_EDEVICE, "the pop engine stopped on a fault (error " +
                                                                    std::to_string(err) + ")");
    S.eng_first = (uint32_t)(x & 0xffffffffu);
    const bool idle = (x >> 40) & 1;
    if (!idle) S.eng_first += 1;  // an exit descriptor took that sequence number
    S.msg_from = S.ov_seq + 1;    // the overlapped path's row messages are stale now
    S.chain_fence = true;
}

// While waiting for an engine pop: a kernel that ended idle before it read
// descriptors written meanwhile is restarted.  true: it was.
static bool eng_poll(Session& S) {
    if (!S.eng_running) return false;
    const uint64_t x = __atomic_load_n(eng_exit_word(S), __ATOMIC_ACQUIRE);
    if (!(x & (1ull << 41))) return false;
    eng_ended(S);
    if ((int32_t)(S.eng_seq - S.eng_first) >= 0) eng_start(S);  // descriptors it never served
    return true;
}

static void eng_submit(Session& S, BatchLaunch& L, int cls, int m, int gang_mode, int min_avail, int ready_count,
                       const KeyFormat& kf) {
    if (S.eng_running) eng_poll(S);
    uint32_t w[kEngDescWords] = {};
    static_assert(kEngDescClass + sizeof(TaskClass) / 4 <= kEngDescWords, "the descriptor carries the class");
    std::memcpy(w + kEngDescClass, &S.classes[cls], sizeof(TaskClass));
    w[kDwCls] = (uint32_t)cls;
    w[kDwFlags] = (uint32_t)m | ((uint32_t)(gang_mode ? 1 : 0) << 8) | (1u << 9) | (kEngOpPop << 12);
    w[kDwMinAvail] = (uint32_t)min_avail;
    w[kDwReady] = (uint32_t)ready_count;
    w[kDwEpochSlot] = (L.epoch & 0xffff) | ((uint32_t)L.slot << 16);
    w[kDwKbase] = (uint32_t)kf.base;
    w[kDwKshift] = (uint32_t)kf.shift;
    w[kDwKidxmax] = (uint32_t)kf.idxmax;
    eng_write(S, ++S.eng_seq, w);
    if (!S.eng_running) {
        if (S.ov_pending) {  // overlapped pops of the launched path may still run on the other stream
            for (int k = 1; k <= kMaxDep; ++k) HIPCHK(hipStreamSynchronize(S.ov_streams[k]));
            S.ov_pending = false;
        }
        eng_start(S);
    }
    S.stats.engine_pops++;
    L.engine = true;
    L.st = S.stream;
}

// Stop the engine: an exit descriptor behind every pop written, then the
// kernel's end.  The pops ahead of it complete first (their results stay in
// the result slots for collect_batched).
static void eng_stop(Session& S) {
    if (!S.eng_running) return;
    const uint32_t sq = ++S.eng_seq;
    uint32_t w[kEngDescWords] = {};
    w[kDwFlags] = kEngOpExit << 12;
    eng_write(S, sq, w);
    for (;;) {
        eng_ended(S);
        if ((int32_t)(S.eng_first - sq) > 0) return;  // it reached the exit descriptor
        eng_start(S);  // it ended idle before that: serve the rest
    }
}

// Wait until no overlapped pop can still run.
static void ov_drain(Session& S) {
    eng_stop(S);
    S.msg_from = S.ov_seq + 1;  // device work outside the chain may follow: earlier row messages go stale
    S.chain_fence = true;       // ... on the session stream: the next chained pop is ordered after it
    if (!S.ov_pending) return;
    for (int k = 1; k <= kMaxDep; ++k) HIPCHK(hipStreamSynchronize(S.ov_streams[k]));
    HIPCHK(hipStreamSynchronize(S.stream));
    S.ov_pending = false;
}

// Wait until no batched pop can still run (before device work that is not a
// batched pop, which the overlap chain does not order).
static void ov_quiesce(Session& S) { ov_drain(S); }

// The device-side form of ov_quiesce for a non-overlapped batched pop on the
// session stream (placement 7): that stream waits for the end of every
// overlap stream's work, without the host waiting.  Row messages of earlier
// pops go stale as after a drain (the pop writes rows outside their
// candidate lists); the overlapped pops after it wait for it (ev_nonov).
static void ov_fence(Session& S) {
    S.msg_from = S.ov_seq + 1;
    if (!S.ov_pending) return;
    for (int k = 1; k <= S.overlap; ++k) {
        if (!S.ev_fence[k]) HIPCHK(hipEventCreateWithFlags(&S.ev_fence[k], hipEventDisableTiming));
        HIPCHK(hipEventRecord(S.ev_fence[k], S.ov_streams[k]));
        HIPCHK(hipStreamWaitEvent(S.stream, S.ev_fence[k], 0));
    }
}

// Nothing but the winner's row can change between the chunk's tasks: the
// condition under which one sweep serves a whole chunk (kbhip_kernels.hip).
// Duration of the timed launch in event pair k (waits for it if needed).
static void ev_harvest(Session& S, int k) {
    hipEvent_t* ev = S.ev_ring[k];
    if (!S.ev_used[k]) return;
    HIPCHK(hipEventSynchronize(ev[1]));
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, ev[0], ev[1]));
    S.timed_ms += ms;
    S.timed_n++;
    S.ev_used[k] = false;
}
static void ev_harvest_all(Session& S) {
    for (int k = 0; k < Session::kEvRing; ++k) ev_harvest(S, k);
}

static bool batchable(const Session& S, int cls) {
    const TaskClass& c = S.classes[cls];
    // Backfilled nodes (some Idle grows on each walk visit): placement 6, one GPU only
    const bool bf_ok = !S.any_bf || (S.world == 1 && S.bf_batch);
    // pod-affinity classes: placement 7 (anti-affinity predicates only), one GPU, no Backfilled nodes
    const bool aff_ok = !c.aff || (S.aff_batch && S.world == 1 && !S.any_bf && aff_batchable(c));
    return S.batched && (S.world == 1 || S.comm || S.xgfn || S.mbox_own) && bf_ok && !c.backfill && aff_ok &&
           S.n_total < (1 << 25);
}

// The next result slot (pinned, mapped PopOutHost) and its granules' tag.
static int take_slot(Session& S, uint32_t* epoch) {
    const int slot = S.next_slot;
    S.next_slot = (S.next_slot + 1) % Session::kSlots;
    uint32_t& ep = S.slot_epoch[slot];
    if (((ep + 1) & 0xffff) == 0) {  // tag wrap: clear this (idle) slot's stale granules, skip tag 0
        std::memset(S.h_out + slot, 0, sizeof(PopOutHost));
        ++ep;
    }
    *epoch = (++ep) & 0xffff;
    return slot;
}

// The per-task path's chunk: control block set up on the device (k_ctrl_init,
// no copy), results as tagged granules in result slot `slot`.
static void ctrl_setup(Session& S, int m, const int* cls, int ready, int min_avail, int gang, int mode, int slot,
                       uint32_t epoch) {
    CtrlInit ci{};
    ci.ready_count = ready;
    ci.min_avail = min_avail;
    ci.gang_mode = gang;
    ci.n_tasks = m;
    ci.any_bf = S.any_bf;
    ci.fallback = S.fallback;
    ci.mode = mode;
    ci.epoch = slot >= 0 ? epoch : 0;
    ci.out = slot >= 0 ? (uint64_t*)((char*)S.d_out + (size_t)slot * sizeof(PopOutHost)) : nullptr;
    for (int i = 0; i < m; ++i) ci.cls[i] = cls[i];
    HIPCHK(launch_ctrl_init(S.d_ctrl, ci, S.stream));
}

// Poll the per-task granules of a chunk (written by commit_task): results up
// to the task whose granule carries the chunk's stop; fit4 (optional) gets
// that task's walk FitDelta counts when it found no node.
static void collect_tasks(Session& S, int slot, uint32_t epoch, int m, int* n_done, int* stop, int32_t* node,
                          int32_t* kind, int32_t* fit4) {
    const PopOutHost& o = S.h_out[slot];
    auto tag = [](uint64_t g) { return (uint32_t)(g >> 48); };
    auto tw0 = std::chrono::steady_clock::now();
    int j = 0, st = -1;
    for (long spin = 0; j < m && st < 0; ++spin) {
        const uint64_t g = __atomic_load_n(&o.g[j], __ATOMIC_ACQUIRE);
        if (tag(g) == epoch) {
            node[j] = (int32_t)(g & 0xffffffffu) - 1;
            kind[j] = (int32_t)((g >> 34) & 3);
            st = (int)((g >> 44) & 0xf) - 1;
            ++j;
            spin = 0;
            continue;
        }
        if (spin == (1L << 22)) HIPCHK(hipStreamSynchronize(S.stream));  // long waits: runtime (errors)
        if (spin > (1L << 22) + 1000) throw Error(KBHIP_EDEVICE, "per-task sweeps produced no result");
        __builtin_ia32_pause();
    }
    S.host_wait_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - tw0).count();
    *n_done = j;
    *stop = st;
    if (fit4 && st == KBHIP_STOP_UNASSIGNED) {
        uint64_t f0 = 0, f1 = 0;
        for (long spin = 0;; ++spin) {
            f0 = __atomic_load_n(&o.fit[0], __ATOMIC_ACQUIRE);
            f1 = __atomic_load_n(&o.fit[1], __ATOMIC_ACQUIRE);
            if (tag(f0) == epoch && tag(f1) == epoch) break;
            if (spin > (1L << 24)) throw Error(KBHIP_EDEVICE, "per-task sweep produced no FitDelta histogram");
            __builtin_ia32_pause();
        }
        fit4[0] = (int32_t)(f0 & 0xffffff); fit4[1] = (int32_t)((f0 >> 24) & 0xffffff);
        fit4[2] = (int32_t)(f1 & 0xffffff); fit4[3] = (int32_t)((f1 >> 24) & 0xffffff);
    }
}

static BatchLaunch launch_batched(Session& S, int cls, int m, int gang_mode, int min_avail, int ready_count) {
    BatchLaunch L;
    L.slot = take_slot(S, &L.epoch);
    L.cls = cls;
    L.m = m;
    const KeyFormat kf = S.keys32 ? S.class_kf[cls] : KeyFormat{};
    if (eng_eligible(S, cls, kf)) {  // the persistent engine: a descriptor, no launch
        auto te0 = std::chrono::steady_clock::now();
        eng_submit(S, L, cls, m, gang_mode, min_avail, ready_count, kf);
        L.fit = true;
        S.sweep_launches++;
        S.host_launch_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - te0).count();
        return L;
    }
    eng_stop(S);  // any other device work is ordered behind the engine's exit
    L.timed = S.time_every > 0 && (S.sweep_launches % S.time_every) == 0;
    S.sweep_launches++;
    hipEvent_t* ev = nullptr;
    if (L.timed) {
        const int k = S.ev_next;
        S.ev_next = (S.ev_next + 1) % Session::kEvRing;
        ev = S.ev_ring[k];
        if (S.ev_used[k]) ev_harvest(S, k);
        if (!ev[0]) { HIPCHK(hipEventCreate(&ev[0])); HIPCHK(hipEventCreate(&ev[1])); }
        S.ev_used[k] = true;
    }
    L.bf = S.any_bf != 0;
    // A session of the what-if lockstep group takes every batched pop through the group (a grouped
    // session running an overlapped pop would hold the group's pop lane up until it left allocate):
    // a pop without Backfilled nodes uses placement 7, which is exact for any class — with no
    // pod-affinity program it is the plain greedy over the list, ending where a node outside it could win.
    const bool grouped = S.rank_group && S.world == 1;
    L.aff = !L.bf && (S.classes[cls].aff || grouped);
    const bool ov = S.overlap > 0 && S.world == 1 && !L.bf && !L.aff;
    // node-array shard over peer mailboxes: pop e's sweep beside pop e-1's placement (k_shard_sweep_ov)
    const bool shov = S.overlap > 0 && S.world > 1 && S.mbox_own && S.shard_overlap && !L.bf && !L.aff;
    // a placement-7 pop between overlapped ones is ordered on the device (ov_fence), so the
    // host can keep predicted pops queued behind it; the other non-overlapped pops drain
    if (!ov && !shov) {
        if (L.aff && S.world == 1 && !grouped && S.overlap > 0 && S.aff_fence) ov_fence(S);
        else ov_quiesce(S);
    }

    const uint32_t seq = ov ? S.ov_seq + 1 : 0;
    const int si = ov ? (int)(seq % (uint32_t)(S.overlap + 1)) : 0;  // pop seq-overlap-1 ran on it before
    L.st = S.ov_streams[si];
    // an overlapped pop chains on the device only behind overlapped pops (its
    // sweep runs beside the previous pop, ordered after the pop before that by
    // its stream): after a non-overlapped batched pop (stream 0), every
    // overlap stream waits for that pop's end before its next launch
    if ((ov || shov) && S.chain_fence && !S.nonov_pending) {  // work issued after a drain (the per-task path)
        if (!S.ev_nonov) HIPCHK(hipEventCreateWithFlags(&S.ev_nonov, hipEventDisableTiming));
        HIPCHK(hipEventRecord(S.ev_nonov, S.stream));
        S.nonov_pending = true;
    }
    if ((ov || shov) && S.nonov_pending) {
        for (int k = 0; k <= std::max(S.overlap, 1); ++k) HIPCHK(hipStreamWaitEvent(S.ov_streams[k], S.ev_nonov, 0));
        S.nonov_pending = false;
    }
    if (ov || shov) S.chain_fence = false;
    L.fit = !L.bf && !L.aff;
    auto tl0 = std::chrono::steady_clock::now();
    if (L.timed) HIPCHK(hipEventRecord(ev[0], L.st));
    void* out = (char*)S.d_out + L.slot * sizeof(PopOutHost);
    if (shov) {  // overlapped shard pops: both kernels on stream seq % 2, chained to pop seq-1 on the device
        MboxArgs mb{};
        for (int p = 0; p < S.world; ++p) mb.dst[p] = S.mbox_peer[p];
        mb.rank = S.rank;
        mb.world = S.world;
        mb.seq = ++S.mbox_seq;
        S.stats.collectives++;
        const int si = (int)(mb.seq & 1u);
        L.st = S.ov_streams[si];
        if (L.timed) HIPCHK(hipEventRecord(ev[0], L.st));
        const int prev_chained = S.sh_chained_seq != 0 && S.sh_chained_seq == mb.seq - 1;
        HIPCHK(launch_shard_sweep_ov(S.conf, S.nc, S.tab, cls, S.classes[cls], m, gang_mode, min_avail, ready_count,
                                     L.epoch, S.d_cand_ov[si], S.d_arrive_ov[si], kf, S.fit_set[si], S.d_link,
                                     prev_chained, mb, L.st));
        if (L.timed) HIPCHK(hipEventRecord(ev[1], L.st));  // timed: the shard's sweep kernel
        S.fit_set[si] ^= 1;
        const int slot = (int)(mb.seq & (kMboxSlots - 1));
        HIPCHK(launch_shard_place(S.conf, S.nc, S.tab, cls, m, gang_mode, min_avail, ready_count, L.epoch, kf,
                                  &S.mbox_own->msg[slot][0], S.world, out, L.st, &S.mbox_own->flag[slot][0][0],
                                  mb.seq, S.d_link));
        S.sh_chained_seq = mb.seq;
        S.ov_pending = true;
    } else if (S.world > 1 && S.mbox_own) {  // node-array shard, peer mailboxes: no host step between the two kernels
        MboxArgs mb{};
        for (int p = 0; p < S.world; ++p) mb.dst[p] = S.mbox_peer[p];
        mb.rank = S.rank;
        mb.world = S.world;
        mb.seq = ++S.mbox_seq;
        S.stats.collectives++;
        HIPCHK(launch_pop_batch(S.conf, S.nc, S.tab, cls, m, gang_mode, min_avail, ready_count, L.epoch, S.d_cand2,
                                S.d_arrive, out, S.stream, 3, kf, S.fit_set[kMaxDep + 1], nullptr, &mb));
        if (L.timed) HIPCHK(hipEventRecord(ev[1], L.st));  // timed: the shard's sweep kernel
        S.fit_set[kMaxDep + 1] ^= 1;
        const int slot = (int)(mb.seq & (kMboxSlots - 1));
        HIPCHK(launch_shard_place(S.conf, S.nc, S.tab, cls, m, gang_mode, min_avail, ready_count, L.epoch, kf,
                                  &S.mbox_own->msg[slot][0], S.world, out, S.stream, &S.mbox_own->flag[slot][0][0],
                                  mb.seq));
    } else if (S.world > 1) {  // node-array shard: sweep -> all-gather of the shards' lists -> identical placement
        HIPCHK(launch_pop_batch(S.conf, S.nc, S.tab, cls, m, gang_mode, min_avail, ready_count, L.epoch, S.d_cand2,
                                S.d_arrive, out, S.stream, 3, kf, S.fit_set[kMaxDep + 1], S.d_shard_send));
        if (L.timed) HIPCHK(hipEventRecord(ev[1], L.st));  // timed: the shard's sweep kernel
        S.fit_set[kMaxDep + 1] ^= 1;
        shard_gather(S);
        HIPCHK(launch_shard_place(S.conf, S.nc, S.tab, cls, m, gang_mode, min_avail, ready_count, L.epoch, kf,
                                  S.d_shard_recv, S.world, out, S.stream));
    } else if (ov) {
        HIPCHK(launch_pop_batch_ov(S.conf, S.nc, S.tab, cls, S.classes[cls], m, gang_mode, min_avail, ready_count, L.epoch,
                                   S.d_cand_ov[si], S.d_arrive_ov[si], out, L.st, kf, S.d_link, seq, S.fit_set[si],
                                   S.overlap, S.msg_from));
        S.fit_set[si] ^= 1;
        S.ov_seq = seq;
        S.ov_pending = true;
    } else if (S.rank_group && S.world == 1) {  // what-if sessions: pops batched across sessions (StepBatcher)
        StepBatcher::Req r;
        r.kind = StepBatcher::kPop;
        r.pop = PopReq{S.conf, S.nc, S.tab, cls, m, gang_mode, min_avail, ready_count, L.epoch, kf, S.d_cand2,
                       S.d_arrive, out, L.bf ? 6 : 7, S.fit_set[kMaxDep + 1]};
        S.fit_set[kMaxDep + 1] ^= 1;
        r.device = S.device;
        if (!S.ev_pop) HIPCHK(hipEventCreateWithFlags(&S.ev_pop, hipEventDisableTiming));
        HIPCHK(hipEventRecord(S.ev_pop, S.stream));
        r.before = S.ev_pop;
        StepBatcher::get().submit(r);
        HIPCHK(hipSetDevice(S.device));
        HIPCHK(r.err);
        HIPCHK(hipStreamWaitEvent(S.stream, r.after, 0));  // this session's later work follows the launch
        S.stats.pop_requests++;
        S.stats.pop_batch_sum += r.batch;
    } else {
        HIPCHK(launch_pop_batch(S.conf, S.nc, S.tab, cls, m, gang_mode, min_avail, ready_count, L.epoch, S.d_cand2,
                                S.d_arrive, out, S.stream, L.bf ? 6 : L.aff ? 7 : 2, kf,
                                S.fit_set[kMaxDep + 1]));
        S.fit_set[kMaxDep + 1] ^= 1;
        if (S.overlap > 0) {
            if (!S.ev_nonov) HIPCHK(hipEventCreateWithFlags(&S.ev_nonov, hipEventDisableTiming));
            HIPCHK(hipEventRecord(S.ev_nonov, S.stream));
            S.nonov_pending = true;
        }
    }
    if (L.timed && S.world == 1) HIPCHK(hipEventRecord(ev[1], L.st));
    S.host_launch_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - tl0).count();
    return L;
}

// Wait for a batched launch's self-tagged result granules (each one 8-byte
// store on the device) and decode them.
static void collect_batched(Session& S, const BatchLaunch& L, int* n_done_out, int* stop_out, int32_t* res_node,
                            int32_t* res_kind) {
    const PopOutHost& o = S.h_out[L.slot];
    auto tag = [](uint64_t g) { return (uint32_t)(g >> 48); };
    auto load = [&](int j) { return __atomic_load_n(&o.g[j], __ATOMIC_ACQUIRE); };
    auto tw0 = std::chrono::steady_clock::now();
    int got = 0, n_done = -1;
    for (long spin = 0;; ++spin) {
        if (n_done < 0) {
            const uint64_t g0 = load(0);
            if (tag(g0) == L.epoch) n_done = (int)((g0 >> 36) & 0xff);
        }
        if (n_done >= 0) {
            while (got < n_done && tag(load(got)) == L.epoch) ++got;
            if (got == n_done) break;
        }
        if (L.engine && (spin & 0x3fff) == 0x3fff && eng_poll(S)) spin = 0;  // restarted after an idle end
        if (spin == (1L << 22)) {  // long waits: the runtime (errors), or the engine's end
            if (L.engine) {
                if (S.eng_running) eng_stop(S);
            } else {
                HIPCHK(hipStreamSynchronize(L.st));
            }
        }
        if (spin > (1L << 22) + 1000) throw Error(KBHIP_EDEVICE, "batched pop produced no result");
        __builtin_ia32_pause();
    }
    S.host_wait_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - tw0).count();
    S.stats.sweeps += 1;
    S.stats.batched_pops += 1;
    if (n_done < (L.bf || L.aff ? 0 : 1) || n_done > L.m) throw Error(KBHIP_EDEVICE, "batched pop returned a bad task count");
    for (int j = 0; j < n_done; ++j) {
        const uint64_t g = load(j);
        res_node[j] = (int32_t)(g & 0xffffffffu) - 1;
        res_kind[j] = (int32_t)((g >> 34) & 3);
    }
    *n_done_out = n_done;
    *stop_out = (int)((load(0) >> 44) & 0xf) - 1;
    if (L.aff || L.bf) {  // the sequential placements: how often a launch ends before its chunk does
        S.stats.seq_launches++;
        if (n_done == 0) S.stats.seq_none++;
        else if (*stop_out == KBHIP_STOP_ALL && n_done < L.m) S.stats.seq_cut++;
    }
    S.last_fit_ok = false;
    if (*stop_out == KBHIP_STOP_UNASSIGNED && L.fit) {
        uint64_t f0 = 0, f1 = 0;
        for (long spin = 0;; ++spin) {
            f0 = __atomic_load_n(&o.fit[0], __ATOMIC_ACQUIRE);
            f1 = __atomic_load_n(&o.fit[1], __ATOMIC_ACQUIRE);
            if (tag(f0) == L.epoch && tag(f1) == L.epoch) break;
            if (spin > (1L << 24)) throw Error(KBHIP_EDEVICE, "batched pop produced no FitDelta histogram");
            __builtin_ia32_pause();
        }
        S.last_fit[0] = (int32_t)(f0 & 0xffffff); S.last_fit[1] = (int32_t)((f0 >> 24) & 0xffffff);
        S.last_fit[2] = (int32_t)(f1 & 0xffffff); S.last_fit[3] = (int32_t)((f1 >> 24) & 0xffffff);
        S.last_fit_ok = true;
    }
#ifdef KBHIP_STAMPS
    {
        int R2;
        const int nb2 = pop_blocks(S.nc.n, &R2);
        vector<uint64_t> st((size_t)nb2 * 4 + 16);
        HIPCHK(hipMemcpy(st.data(), S.d_stamps, st.size() * 8, hipMemcpyDeviceToHost));
        uint64_t t0 = UINT64_MAX, tbm = 0;
        double sw = 0, bm = 0;
        for (int b = 0; b < nb2; ++b) {
            t0 = std::min(t0, st[b * 4]);
            tbm = std::max(tbm, st[b * 4 + 2]);
            sw += (st[b * 4 + 1] - st[b * 4]) * 0.01;
            bm += (st[b * 4 + 2] - st[b * 4 + 1]) * 0.01;
        }
        const uint64_t* P = st.data() + nb2 * 4;
        S.phase[0] += sw / nb2;                    // per-block sweep + wave sort
        S.phase[1] += bm / nb2;                    // per-block merge + store
        S.phase[2] += (tbm - t0) * 0.01;           // first block start -> every block list stored
        S.phase[3] += ((double)P[4] - (double)tbm) * 0.01;  // -> final merger starts
        S.phase[4] += (P[0] - P[4]) * 0.01;        // final merge
        if (P[11] && P[12]) {
            S.phase[17] += (P[11] - P[1]) * 0.01;  // placement: rows from cache / memory
            S.phase[18] += (P[12] - P[11]) * 0.01; // placement: LDS init + barrier
        }
        if (P[10]) {                               // overlapped kernel: wait for the previous pop, patch
            S.phase[15] += (P[10] - P[0]) * 0.01;
            S.phase[16] += (P[1] - P[10]) * 0.01;
        }
        S.phase[5] += (P[1] - P[0]) * 0.01;        // chain precompute (overlapped: wait + patch)
        S.phase[6] += (P[2] - P[1]) * 0.01;        // placement loop
        S.phase[7] += (P[3] - P[2]) * 0.01;        // write back
        S.phase[8] += (P[3] - t0) * 0.01;          // total in-kernel span
        S.phase[9] += L.m;
        if (P[5] && P[6] && P[7]) {  // parallel-levels sub-phases
            S.phase[10] += (P[5] - P[1]) * 0.01;   // candidate rows loaded
            S.phase[11] += (P[6] - P[5]) * 0.01;   // round-0 depth evaluation
            S.phase[12] += (P[7] - P[6]) * 0.01;   // round-0 sort + merge
            if (P[8] && P[9]) {
                S.phase[13] += (P[8] - P[2]) * 0.01;   // write back: ranks, kinds, stop rule
                S.phase[14] += (P[9] - P[8]) * 0.01;   // write back: LDS counts
            }
        }
        S.phase_n++;
    }
#endif
}

// A session-placed pod (its Spec.NodeName is still "") arrives on / leaves
// node n: the inter-pod priority's fallback node is the lowest such node
// (nodeorder.go:78-93).
static void sess_placed(Session& S, int n, int d) {
    if (S.sess_cnt.empty()) S.sess_cnt.assign(S.n_total, 0);  // global node indices (shards too)
    S.sess_cnt[n] += d;
    if (d > 0 && (S.fallback < 0 || n < S.fallback)) S.fallback = n;
    if (d < 0 && S.sess_cnt[n] == 0 && n == S.fallback) {
        S.fallback = -1;
        for (int k = n + 1; k < S.n_total; ++k)
            if (S.sess_cnt[k] > 0) { S.fallback = k; break; }
    }
}

// Count-table changes of a predicate target leaving / re-entering the target
// set (eviction / unevict, AffinityModel::target_updates), queued on the host
// and applied before the next device read of the tables (flush_tables).
static void queue_target(Session& S, int pi, int sign) {
    if (!S.aff || !S.aff->active) return;
    const HPod& p = S.pods[pi];
    if (p.node < 0) return;
    static thread_local vector<int32_t> upd;
    S.aff->target_updates(pi, upd);
    const int npad = S.aff->npad();
    for (size_t k = 0; k + 2 < upd.size(); k += 3) {
        if (upd[k] == UPD_CNT_ALLOC) {
            const int d = S.aff->dom[(size_t)upd[k + 1] * npad + p.node];
            if (d >= 0) S.tab_delta[(int64_t)upd[k + 2] + d] += sign;
        } else if (upd[k] == UPD_SCALAR_ALLOC) {
            S.tab_delta[-1 - (int64_t)upd[k + 2]] += sign;
        }
    }
}
static void flush_tables(Session& S) {
    if (S.tab_delta.empty()) return;
    vector<int32_t> idx, val;
    for (auto& kv : S.tab_delta)
        if (kv.second) { idx.push_back((int32_t)kv.first); val.push_back(kv.second); }
    S.tab_delta.clear();
    if (idx.empty()) return;
    const int n = (int)idx.size();
    int32_t* di = S.b_tab_idx.alloc<int32_t>(2 * (size_t)n);
    idx.insert(idx.end(), val.begin(), val.end());
    HIPCHK(hipMemcpyAsync(di, idx.data(), idx.size() * sizeof(int32_t), hipMemcpyHostToDevice, S.stream));
    HIPCHK(launch_tab_add(S.tab, di, di + n, n, S.stream));
    HIPCHK(hipStreamSynchronize(S.stream));  // the pageable source must outlive the copy
}

// Host mirror of the device commits of consumed tasks (NodeInfo.Used, the
// fallback node of nodeorder.go:78-93) + the caller's output arrays.
static void apply_results(Session& S, const int32_t* ids, int n, const int32_t* res_node, const int32_t* res_kind,
                          int32_t* out_node, uint8_t* out_kind) {
    for (int i = 0; i < n; ++i) {
        out_node[i] = res_node[i];
        out_kind[i] = (uint8_t)res_kind[i];
        const int node = res_node[i];
        if (node >= 0) {
            const HPod& p = S.pods[ids[i]];
            S.used[node].c += p.req.c; S.used[node].m += p.req.m; S.used[node].g += p.req.g;
            sess_placed(S, node, +1);
        }
    }
}

// ---------------------------------------------------------------------------
// device driver for one job pop
// ---------------------------------------------------------------------------
static void check_task_ids(const Session& S, const int32_t* ids, int n) {
    for (int i = 0; i < n; ++i)
        if (ids[i] < 0 || ids[i] >= (int)S.pods.size() || S.pods[ids[i]].cls < 0)
            throw Error(KBHIP_EINVAL, "task id is not a pending task of the session");
}

constexpr uint8_t kBfBackoff = 4;  // pops of a class sent to the general path after a placement-6 miss
static int place_job(Session& S, const int32_t* ids, int n, int gang_mode, int min_avail, int ready_count,
                     int32_t* out_node, uint8_t* out_kind, int32_t* out_n_done, int32_t* out_stop) {
    int done = 0, stop = KBHIP_STOP_ALL;
    check_task_ids(S, ids, n);
    while (done < n) {
        const int cls0 = S.pods[ids[done]].cls;
        int m = 1;
        while (done + m < n && m < kMaxChunk && S.pods[ids[done + m]].cls == cls0) ++m;
        bool batch = batchable(S, cls0);
        if (batch && S.any_bf && cls0 < (int)S.bf_backoff.size() && S.bf_backoff[cls0] > 0) {
            S.bf_backoff[cls0]--;
            batch = false;
        }
        int n_done, stop_c, ready_c, any_bf_c = S.any_bf;
        const int32_t* res_node;
        const int32_t* res_kind;
        if (batch) {
            // one launch: sweep + per-block top-64 + merge + placement of the chunk
            const BatchLaunch L = launch_batched(S, cls0, m, gang_mode, min_avail, ready_count);
            collect_batched(S, L, &n_done, &stop_c, S.res_node_buf, S.res_kind_buf);
            if (n_done == 0) {  // placement 6 / 7 could not place the first task exactly: general path for it
                batch = false;
                m = 1;
                if (L.bf) {
                    if (S.bf_backoff.size() < S.classes.size()) S.bf_backoff.resize(S.classes.size(), 0);
                    S.bf_backoff[cls0] = kBfBackoff;
                }
            }
        } else {  // general path: up to a chunk of mixed classes, no longer than the pop can run
            m = std::min(n - done, kMaxChunk);  // (it stops once Ready: after `need` more Allocated tasks)
            const int need = gang_mode ? min_avail - ready_count : 1;
            m = std::min(m, std::max(need, 1));
        }
        // sampled HIP-event timing of a general-path launch (kbhip_set_option "time_every")
        const bool timed = !batch && S.time_every > 0 && (S.sweep_launches % S.time_every) == 0;
        if (timed && !S.ev0) { HIPCHK(hipEventCreate(&S.ev0)); HIPCHK(hipEventCreate(&S.ev1)); }
        if (!batch) S.sweep_launches++;
        if (batch) {
            int alloc = 0;
            for (int j = 0; j < n_done; ++j) alloc += S.res_kind_buf[j] == 1;
            ready_c = ready_count + alloc;
            res_node = S.res_node_buf;
            res_kind = S.res_kind_buf;
        } else {
            ov_quiesce(S);
            int cls[kMaxChunk];
            for (int i = 0; i < m; ++i) cls[i] = S.pods[ids[done + i]].cls;
            uint32_t epoch = 0;
            const int slot = take_slot(S, &epoch);
            ctrl_setup(S, m, cls, ready_count, min_avail, gang_mode, 0, slot, epoch);
            bool defer = S.any_bf != 0;  // a backfill-annotated task may set any_bf on the device mid-chunk
            for (int i = 0; i < m; ++i) defer = defer || S.classes[cls[i]].backfill;
            if (timed) {
                for (int i = 0; i < m; ++i) {
                    if (i == 0) HIPCHK(hipEventRecord(S.ev0, S.stream));
                    sweep_task(S, i, cls[i], defer);
                    if (i == 0) HIPCHK(hipEventRecord(S.ev1, S.stream));
                }
            } else {
                sweep_chunk(S, m, cls, defer);
            }
            S.stats.sweeps += m;
            int32_t fit4[4] = {0, 0, 0, 0};
            collect_tasks(S, slot, epoch, m, &n_done, &stop_c, S.res_node_buf, S.res_kind_buf, fit4);
            if (S.d_dbg) {
                HIPCHK(hipStreamSynchronize(S.stream));
                const size_t row = 2 * (size_t)S.nc.npad + 4;
                const size_t off = S.dbg_keys.size();
                S.dbg_keys.resize(off + row * n_done);
                HIPCHK(hipMemcpy(S.dbg_keys.data() + off, S.d_dbg, row * n_done * 8, hipMemcpyDeviceToHost));
                for (int i = 0; i < n_done; ++i) S.dbg_pods.push_back(ids[done + i]);
            }
            S.last_fit_ok = stop_c == KBHIP_STOP_UNASSIGNED && n_done >= 1;
            if (S.last_fit_ok) {  // this shard's counts of the walk of the task that found no node
                for (int q = 0; q < 4; ++q) S.last_fit[q] = fit4[q];
                fit_allreduce(S, S.last_fit);
            }
            int alloc = 0;
            for (int j = 0; j < n_done; ++j) {
                alloc += S.res_kind_buf[j] == 1;
                if (S.res_node_buf[j] >= 0 && S.classes[cls[j]].backfill) any_bf_c = 1;  // IsBackfill commit
            }
            ready_c = ready_count + alloc;
            res_node = S.res_node_buf;
            res_kind = S.res_kind_buf;
        }
        if (timed) {
            float ms = 0;
            HIPCHK(hipEventElapsedTime(&ms, S.ev0, S.ev1));
            S.timed_ms += ms;
            S.timed_n++;
        }
        if (stop_c < 0 || n_done < 1 || n_done > m) throw Error(KBHIP_EDEVICE, "device pop did not complete");
        apply_results(S, ids + done, n_done, res_node, res_kind, out_node + done, out_kind + done);
        S.any_bf = any_bf_c;
        ready_count = ready_c;
        done += n_done;
        stop = stop_c;
        if (stop != KBHIP_STOP_ALL) break;
    }
    *out_n_done = done;
    *out_stop = stop;
    return 0;
}

// ---------------------------------------------------------------------------
// asynchronous per-pop ABI (kbhip_place_job_submit / _wait / _cancel): the
// pipelining of kbhip_allocate's speculation (Allocator::speculate), offered
// to a host that keeps allocate.go's loop itself.  A submitted pop runs on the
// device state its predecessors leave; launched tickets form a prefix of the
// queue (a deferred one, run at its wait, holds back the ones behind it).
// ---------------------------------------------------------------------------
static constexpr int kMaxLaunchedTickets = 4;  // < Session::kSlots result slots in flight
static constexpr size_t kMaxTickets = 64;

static void require_no_tickets(const Session& S) {
    if (!S.tickets.empty())
        throw Error(KBHIP_EINVAL, "submitted job pops are outstanding (kbhip_place_job_wait / _cancel them first)");
}

// One batched chunk of one class, no Backfilled nodes (the undo of a pop has no visit rule).
static bool ticket_launchable(Session& S, const PopTicket& t) {
    const int n = (int)t.ids.size();
    if (n < 1 || n > kMaxChunk || S.any_bf) return false;
    const int cls0 = S.pods[t.ids[0]].cls;
    for (int i = 1; i < n; ++i)
        if (S.pods[t.ids[i]].cls != cls0) return false;
    return batchable(S, cls0);
}

// Launch deferred tickets in queue order while they can run as one batched launch.
static void promote_tickets(Session& S) {
    int launched = 0;
    for (PopTicket& t : S.tickets) {
        if (t.launched) { ++launched; continue; }
        if (launched >= kMaxLaunchedTickets || !ticket_launchable(S, t)) return;
        t.L = launch_batched(S, S.pods[t.ids[0]].cls, (int)t.ids.size(), t.gang, t.min_avail, t.ready);
        t.launched = true;
        S.stats.async_launched++;
        ++launched;
    }
}

// Withdraw the launches of tickets [from, end): collect, then undo their node
// updates on the device (inverse updates commute); the tickets become deferred.
static void retract_tickets(Session& S, size_t from) {
    int32_t fit_save[4];
    std::memcpy(fit_save, S.last_fit, sizeof fit_save);
    const bool fit_ok = S.last_fit_ok;
    struct Got { int cls, n; int32_t node[kMaxChunk], kind[kMaxChunk]; };
    vector<Got> got;
    for (size_t i = from; i < S.tickets.size(); ++i) {
        PopTicket& t = S.tickets[i];
        if (!t.launched) continue;
        Got g;
        int st = 0;
        g.cls = t.L.cls;
        collect_batched(S, t.L, &g.n, &st, g.node, g.kind);
        got.push_back(g);
        t.launched = false;
    }
    std::memcpy(S.last_fit, fit_save, sizeof fit_save);
    S.last_fit_ok = fit_ok;
    if (got.empty()) return;
    ov_quiesce(S);
    for (const Got& g : got) {
        HIPCHK(launch_undo_pop(S.nc, S.tab, g.cls, g.n, g.node, g.kind, S.stream));
        S.stats.async_retracted++;
    }
    if (S.overlap > 0) HIPCHK(hipStreamSynchronize(S.stream));  // overlapped pops are not ordered after it
}

static int64_t place_job_submit(Session& S, const int32_t* ids, int n, int gang_mode, int min_avail,
                                int ready_count) {
    check_task_ids(S, ids, n);
    if (S.tickets.size() >= kMaxTickets) throw Error(KBHIP_EINVAL, "too many outstanding job pops");
    PopTicket t;
    t.id = S.next_ticket++;
    t.ids.assign(ids, ids + n);
    t.gang = gang_mode;
    t.min_avail = min_avail;
    t.ready = ready_count;
    const int64_t id = t.id;
    S.tickets.push_back(std::move(t));
    try {
        promote_tickets(S);
    } catch (...) {
        // the caller gets an error and no ticket id: the new ticket must not stay queued
        // (a launch that failed left it deferred; earlier tickets keep their state)
        if (!S.tickets.empty() && S.tickets.back().id == id && !S.tickets.back().launched) S.tickets.pop_back();
        throw;
    }
    return id;
}

static int place_job_wait(Session& S, int64_t ticket, int32_t* out_node, uint8_t* out_kind, int32_t* out_n_done,
                          int32_t* out_stop) {
    if (S.tickets.empty() || S.tickets.front().id != ticket)
        throw Error(KBHIP_EINVAL, "kbhip_place_job_wait must name the oldest outstanding ticket");
    if (S.tickets.front().launched) {
        // collected before the ticket leaves the queue: if the collection fails, the launched pop stays
        // outstanding (its device updates can still be collected by a retried wait or undone by a cancel)
        PopTicket& f = S.tickets.front();
        int nd = 0, st = 0;
        collect_batched(S, f.L, &nd, &st, S.res_node_buf, S.res_kind_buf);
        f.launched = false;
        f.collected = true;
        f.c_nd = nd;
        f.c_st = st;
    }
    PopTicket t = std::move(S.tickets.front());
    S.tickets.pop_front();
    const int n = (int)t.ids.size();
    bool sync = !t.collected;
    if (t.collected) {
        const int nd = t.c_nd, st = t.c_st;
        if (nd == 0) {  // placement 7 could not place the first task exactly: the pop runs synchronously,
            retract_tickets(S, 0);  // and the launches behind it ran on a state it is about to change
            sync = true;
        } else {
            if (st < 0 || nd > n) throw Error(KBHIP_EDEVICE, "device pop did not complete");
            int alloc = 0;
            for (int j = 0; j < nd; ++j) alloc += S.res_kind_buf[j] == 1;
            apply_results(S, t.ids.data(), nd, S.res_node_buf, S.res_kind_buf, out_node, out_kind);
            *out_n_done = nd;
            *out_stop = st;
            if (st == KBHIP_STOP_ALL && nd < n) {
                // the launch ended before its chunk did (a sequential placement whose list ran out): the
                // pop goes on with its remaining tasks (allocate.go:110-196), synchronously; the launches
                // behind it ran on a state it is about to change
                retract_tickets(S, 0);
                int32_t nd2 = 0, st2 = 0;
                place_job(S, t.ids.data() + nd, n - nd, t.gang, t.min_avail, t.ready + alloc, out_node + nd,
                          out_kind + nd, &nd2, &st2);
                *out_n_done = nd + nd2;
                *out_stop = st2;
            }
        }
    }
    if (sync) place_job(S, t.ids.data(), n, t.gang, t.min_avail, t.ready, out_node, out_kind, out_n_done, out_stop);
    promote_tickets(S);
    return 0;
}

static int place_job_cancel(Session& S, int64_t ticket) {
    size_t from = 0;
    while (from < S.tickets.size() && S.tickets[from].id < ticket) ++from;
    if (from == S.tickets.size() || S.tickets[from].id != ticket)
        throw Error(KBHIP_EINVAL, "kbhip_place_job_cancel names no outstanding ticket");
    retract_tickets(S, from);
    const int k = (int)(S.tickets.size() - from);
    S.tickets.erase(S.tickets.begin() + from, S.tickets.end());
    S.stats.async_cancelled += k;
    return k;
}

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
        for (size_t i = 0; i < v.size(); ++i) {
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
        auto lt = [nd](const K& a, const K& b) {
            for (int c = 0; c < nd; ++c)
                if (a.d[c] != b.d[c]) return a.d[c] < b.d[c];
            if (a.ts != b.ts) return a.ts < b.ts;
            return a.j < b.j;
        };
        const size_t n = k.size();
        if (n < (1u << 15)) {
            std::sort(k.begin(), k.end(), lt);
        } else {  // C5: ~180 k running jobs without pending tasks: 8 sorted runs in parallel, merged
            constexpr int kRuns = 8;
            vector<size_t> cut(kRuns + 1);
            for (int r = 0; r <= kRuns; ++r) cut[r] = n * r / kRuns;
            vector<std::thread> th;
            for (int r = 1; r < kRuns; ++r)
                th.emplace_back([&, r]() { std::sort(k.begin() + cut[r], k.begin() + cut[r + 1], lt); });
            std::sort(k.begin(), k.begin() + cut[1], lt);
            for (auto& x : th) x.join();
            for (int w = 1; w < kRuns; w *= 2)  // the keys are distinct (job index last): a strict order
                for (int r = 0; r + w < kRuns; r += 2 * w)
                    std::inplace_merge(k.begin() + cut[r], k.begin() + cut[r + w],
                                       k.begin() + cut[std::min(r + 2 * w, kRuns)], lt);
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
            const int nth = J < (1 << 14) ? 1 : 8;
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
            for (auto& j : S.jobs) {
                HQueue& q = S.queues[j.queue];
                q.has_attr = true;
                for (int t : j.tasks) {
                    const HPod& p = S.pods[t];
                    if (allocated_status(p.status)) { q.allocated.add(p.req); q.request.add(p.req); }
                    else if (p.status == Pending) q.request.add(p.req);
                }
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
        GroupScope group(S.rank_group && S.world == 1, StepBatcher::kPop);  // what-if sessions: pops step with the group
        auto t0 = std::chrono::steady_clock::now();
        compile_orders();
        open_plugins();
        auto ql = [this](int a, int b) { return queue_less(a, b); };
        auto jl = [this](int a, int b) { return job_less(a, b); };
        GoHeap<decltype(ql)> queues(ql);
        std::map<int, JobQueue<decltype(jl)>> jobs_map;
        for (size_t j = 0; j < S.jobs.size(); ++j) {
            const HJob& job = S.jobs[j];
            int q = job.queue;
            // one queue copy per job, as allocate.go pushes them: a queue's share changes while
            // its other copies sit in the heap, so the Go heap's layout — which the copies of
            // jobs without pending tasks shape too — decides later pops (exactness needs them)
            queues.push(q);
            auto it = jobs_map.find(q);
            if (it == jobs_map.end()) it = jobs_map.emplace(q, JobQueue<decltype(jl)>(jl)).first;
            bool work = false;  // allocate.go:91-104: a pending task that is not BestEffort
            if (job.pending_built) work = job.cursor < job.pending.size();
            else if (job.maybe_pending)
                for (int t : job.tasks) {
                    const HPod& p = S.pods[t];
                    if (p.status == Pending && !(p.req.c < kMinCPU && p.req.m < kMinMem && p.req.g < kMinGPU)) {
                        work = true;
                        break;
                    }
                }
            if (work) {
                it->second.push((int)j);
            } else {
                it->second.idle.push_back((int)j);
                S.jobs[j].pending_built = true;  // what build_pending would find: nothing
            }
        }
        for (auto& kv : jobs_map) sort_jobs(kv.second.idle);
        vector<int32_t> ids, onode;
        vector<uint8_t> okind;
        const int gm = S.gang_ready ? 1 : 0;
        if (!S.ev_run[0]) { HIPCHK(hipEventCreate(&S.ev_run[0])); HIPCHK(hipEventCreate(&S.ev_run[1])); }
        ov_quiesce(S);
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
    void check_evict_supported() {
        if (S.world != 1) throw Error(KBHIP_EUNSUPPORTED, "reclaim / preempt on a node-sharded session");
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
        const int N = S.nc.n, P = (int)S.pods.size();
        const int nth = P < (1 << 16) ? 1 : 8;
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
        const int nth = S.pods.size() < (1u << 16) ? 1 : 8;
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
        if (!S.b_rank_sorted.p) {
            S.b_rank_keys.alloc<uint64_t>(N);
            S.b_rank_sorted.alloc<uint64_t>(N);
            S.b_rank_cnt.alloc<uint32_t>(4);
            S.rank_tmp_bytes = std::max<size_t>((size_t)16, rank_hist_words(N) * sizeof(uint32_t));
            S.b_rank_tmp.alloc<uint8_t>(S.rank_tmp_bytes);
            S.b_rank_radix.alloc<uint64_t>(std::max(N, 1));
            S.h_rank = (uint64_t*)MemPool::get().take(MemPool::kPinned, (size_t)(N + 1) * sizeof(uint64_t),
                                                      &S.h_rank_cap);
        }
        flush_tables(S);  // evictions / unevicts so far change pod-affinity predicates
        ctrl_setup(S, 1, &cls, 0, 0, 0, 0, -1, 0);
        HIPCHK(hipMemsetAsync(S.b_rank_cnt.p, 0, 2 * sizeof(uint32_t), S.stream));
        auto sr = S.class_srange[cls];
        if (by_score && S.classes[cls].ipa_n > 0) {  // inter-pod priority: normalisation prepass, wider range
            HIPCHK(launch_ipa_minmax(S.nc, S.tab, S.d_ctrl, 0, S.stream));
            const int64_t w = 10 * (int64_t)S.conf.w_pa * S.conf.score_mult;
            sr.first += std::min<int64_t>(0, w);
            sr.second += std::max<int64_t>(0, w);
        }
        const bool counting = !S.force_radix && sr.second - sr.first < 256 && sr.first >= INT32_MIN &&
                              sr.second <= INT32_MAX;
        if (counting && S.rank_group) {  // one launch with the concurrent what-if sessions' rankings
            StepBatcher::Req r;
            r.kind = StepBatcher::kRank;
            HIPCHK(fill_rank_desc(&r.rank, S.conf, S.nc, S.tab, S.d_ctrl, by_score ? 1 : 0, (int)sr.first,
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
            HIPCHK(launch_rank_sorted(S.conf, S.nc, S.tab, S.d_ctrl, by_score ? 1 : 0, (int)sr.first, (int)sr.second,
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
        out.resize(cnt);
        for (int i = 0; i < cnt; ++i) out[i] = key_idx(S.h_rank[1 + i]);
        S.stats.sweeps++;
        S.stats.tasks++;
    }
    void dev_op(int op, int pi) {
        const HPod& p = S.pods[pi];
        HIPCHK(launch_node_op(S.nc, S.tab, op, p.node, p.cls, p.req.c, p.req.m, p.req.g, S.stream));
    }
    // the session half of an eviction (session.go:331-356 / statement.go:35-67)
    void evict_in_session(int v) {
        if (allocated_status(S.pods[v].status)) queue_target(S, v, -1);  // no longer a predicate target
        set_status(v, Releasing);
        // node.UpdateTask: Releasing += Resreq.  No node ranking reads Releasing, so
        // evictions are summed per node and applied in one launch (flush_evictions)
        const HPod& p = S.pods[v];
        if (S.rel_delta.empty()) { S.rel_delta.assign(S.nc.n, R3{}); S.rel_flag.assign(S.nc.n, 0); }
        if (!S.rel_flag[p.node]) { S.rel_flag[p.node] = 1; S.rel_touched.push_back(p.node); }
        R3& d = S.rel_delta[p.node];
        d.c += p.req.c; d.m += p.req.m; d.g += p.req.g;
        on_deallocate(v);
    }
    void flush_evictions() {
        const int n = (int)S.rel_touched.size();
        if (!n) return;
        vector<int32_t> nodes(n);
        vector<int64_t> d(3 * (size_t)n);
        for (int i = 0; i < n; ++i) {
            const int v = S.rel_touched[i];
            nodes[i] = v;
            d[3 * i] = S.rel_delta[v].c; d[3 * i + 1] = S.rel_delta[v].m; d[3 * i + 2] = S.rel_delta[v].g;
            S.rel_delta[v] = R3{};
            S.rel_flag[v] = 0;
        }
        S.rel_touched.clear();
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
        GroupScope group(S.rank_group, StepBatcher::kRank);
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
        GroupScope group(S.rank_group, StepBatcher::kRank);
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
static void first_fit(Session& S, const int32_t* ids, int n, int32_t* out_node) {
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

static void backfill_run(Session& S) {
    GroupScope group(S.rank_group && S.world == 1, StepBatcher::kPop);  // what-if sessions: first-fits step with the group
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
static int sweep_scores(Session& S, int pod, uint64_t* out_keys) {
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
// (no copies in between), one HIP-event pair around the whole sequence: the
// device time per sweep launch, boundaries between launches included.
static double time_sweeps(Session& S, const int32_t* ids, int n) {
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

// JobInfo.FitError (job_info.go:343-372) from the histogram of the job's last walk.
static string fit_error(const HJob& j) {
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
static string gang_close_text(const Session& S) {
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

static int device_count() {
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

}  // namespace kbhip

using namespace kbhip;

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

extern "C" {

struct kb_session {
    kbhip::Session s;
};
static void taint_comm(kb_session* s) {
    if (s && s->s.comm) s->s.comm_bad = true;
}
static void check_usable(kb_session* s) {
    if (s && !s->s.broken.empty()) throw kbhip::Error(KBHIP_EINVAL, s->s.broken);
}

const char* kbhip_last_error(void) { return kbhip::g_err.c_str(); }

int kbhip_device_count(void) { ABI_GUARD(return kbhip::device_count();) }

// Arguments of the actions that return a record log: a device session and,
// when cap > 0, three output arrays of at least cap entries.
static void check_log_args(kb_session* s, const int32_t* out_pod, const int32_t* out_node, const uint8_t* out_kind,
                           int64_t cap) {
    if (!s) throw kbhip::Error(KBHIP_EINVAL, "null session");
    if (s->s.encode_only) throw kbhip::Error(KBHIP_EINVAL, "encode-only session has no device state");
    if (cap < 0 || (cap > 0 && (!out_pod || !out_node || !out_kind)))
        throw kbhip::Error(KBHIP_EINVAL, "null output array with cap > 0");
}

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
        kbhip::Allocator a(s->s);
        a.run();
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

int kbhip_sweep_scores(kb_session* s, int32_t task_id, uint64_t* out_keys) {
    ABI_GUARD_S(s, {
        if (!s) throw kbhip::Error(KBHIP_EINVAL, "null session");
        if (s->s.encode_only) throw kbhip::Error(KBHIP_EINVAL, "encode-only session has no device state");
        kbhip::require_no_tickets(s->s);
        HIPCHK(hipSetDevice(s->s.device));
        return kbhip::sweep_scores(s->s, task_id, out_keys);
    })
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
static void session_carry(Session& S, const int32_t* ev_pod = nullptr, const uint8_t* ev = nullptr, int64_t n_ev = 0) {
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
};
static SavedOptions save_options(const Session& S) {
    return SavedOptions{S.batched, S.keys32, S.bf_batch, S.aff_batch, S.aff_fence, S.shard_overlap, S.rank_group,
                        S.force_radix,
                        S.debug_keys,
                        S.time_every, S.speculate, S.overlap, S.rank_first};
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

static void reopen_in_place(kb_session* ks, const kbs::Snapshot& s) {
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

static void carry_snapshot(kb_session* ks, const kbs::Snapshot& s, const int32_t* old_pod, const int32_t* old_node) {
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
            const int nth = P < (1 << 16) ? 1 : 8;
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
        constexpr int kThreads = 8;
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
    const int jth = JN < (1 << 13) ? 1 : 8;
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
    const int jth_p = P < (1 << 15) ? 1 : 8;
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
        const int nth = P < (1 << 15) ? 1 : 8;
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
        constexpr int kThreads = 8;
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

static int evict_action(kb_session* s, bool preempt, int32_t* out_pod, int32_t* out_node, uint8_t* out_kind,
                        int64_t cap) {
    ABI_GUARD_S(s, {
        check_log_args(s, out_pod, out_node, out_kind, cap);
        kbhip::require_no_tickets(s->s);
        HIPCHK(hipSetDevice(s->s.device));
        kbhip::ov_quiesce(s->s);
        s->s.log.clear();
        kbhip::Allocator a(s->s);
        if (preempt) a.preempt_action();
        else a.reclaim_action();
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
int kbhip_session_carry(kb_session* s, int64_t* out_uploaded_bytes) {
    ABI_GUARD_S(s, {
        if (!s) throw kbhip::Error(KBHIP_EINVAL, "null session");
        if (s->s.encode_only) throw kbhip::Error(KBHIP_EINVAL, "encode-only session has no device state");
        kbhip::require_no_tickets(s->s);
        HIPCHK(hipSetDevice(s->s.device));
        session_carry(s->s);
        if (out_uploaded_bytes) *out_uploaded_bytes = s->s.carry_bytes;
        return 0;
    })
}
int kbhip_session_carry_events(kb_session* s, const int32_t* pods, const uint8_t* events, int64_t n,
                               int64_t* out_uploaded_bytes) {
    ABI_GUARD_S(s, {
        if (!s) throw kbhip::Error(KBHIP_EINVAL, "null session");
        if (n < 0 || (n > 0 && (!pods || !events))) throw kbhip::Error(KBHIP_EINVAL, "null argument");
        if (s->s.encode_only) throw kbhip::Error(KBHIP_EINVAL, "encode-only session has no device state");
        kbhip::require_no_tickets(s->s);
        HIPCHK(hipSetDevice(s->s.device));
        session_carry(s->s, pods, events, n);
        if (out_uploaded_bytes) *out_uploaded_bytes = s->s.carry_bytes;
        return 0;
    })
}
int kbhip_reclaim(kb_session* s, int32_t* out_pod, int32_t* out_node, uint8_t* out_kind, int64_t cap) {
    return evict_action(s, false, out_pod, out_node, out_kind, cap);
}
int kbhip_preempt(kb_session* s, int32_t* out_pod, int32_t* out_node, uint8_t* out_kind, int64_t cap) {
    return evict_action(s, true, out_pod, out_node, out_kind, cap);
}
int kbhip_session_carry_snapshot(kb_session* s, const void* kbs_bytes, size_t len, const int32_t* old_pod,
                                 const int32_t* old_node, int64_t* out_uploaded_bytes) {
    ABI_GUARD_S(s, {
        if (!s || !kbs_bytes) throw kbhip::Error(KBHIP_EINVAL, "null argument");
        if (s->s.encode_only) throw kbhip::Error(KBHIP_EINVAL, "encode-only session has no device state");
        kbs::Snapshot snap;
        snap.view_bytes(kbs_bytes, len);
        const size_t P = snap.rows("p_uid"), N = snap.rows("n_name");
        if ((P && !old_pod) || (N && !old_node)) throw kbhip::Error(KBHIP_EINVAL, "null index map");
        HIPCHK(hipSetDevice(s->s.device));
        auto t0 = std::chrono::steady_clock::now();
        carry_snapshot(s, snap, old_pod, old_node);
        s->s.stats.open_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (out_uploaded_bytes) *out_uploaded_bytes = s->s.carry_bytes;
        return KBHIP_OK;
    })
}

int kbhip_read_nodes(kb_session* s, int64_t* out, int64_t n_nodes) {
    ABI_GUARD_S(s, {
        if (!s || !out) throw kbhip::Error(KBHIP_EINVAL, "null argument");
        if (s->s.encode_only) throw kbhip::Error(KBHIP_EINVAL, "encode-only session has no device state");
        kbhip::Session& S = s->s;
        kbhip::require_no_tickets(S);
        const int N = S.nc.n;
        if (n_nodes < N) throw kbhip::Error(KBHIP_EINVAL, "output too small");
        HIPCHK(hipSetDevice(S.device));
        kbhip::ov_quiesce(S);
        vector<int64_t> buf[9];
        int64_t* src[9] = {S.nc.idle_cpu, S.nc.idle_mem, S.nc.idle_gpu, S.nc.rel_cpu, S.nc.rel_mem,
                           S.nc.rel_gpu, S.nc.bf_cpu, S.nc.bf_mem, S.nc.bf_gpu};
        for (int k = 0; k < 9; ++k) {
            buf[k].resize(N);
            if (N) HIPCHK(hipMemcpy(buf[k].data(), src[k], N * sizeof(int64_t), hipMemcpyDeviceToHost));
        }
        for (int i = 0; i < N; ++i) {
            int64_t* o = out + (int64_t)i * 12;
            o[0] = buf[0][i]; o[1] = buf[1][i]; o[2] = buf[2][i];
            const R3& u = S.used[i + S.nc.base];
            o[3] = u.c; o[4] = u.m; o[5] = u.g;
            o[6] = buf[3][i]; o[7] = buf[4][i]; o[8] = buf[5][i];
            o[9] = buf[6][i]; o[10] = buf[7][i]; o[11] = buf[8][i];
        }
        return N;
    })
}

int kbhip_get_stats(kb_session* s, kbhip_stats* out) {
    ABI_GUARD({
        if (!s || !out) throw kbhip::Error(KBHIP_EINVAL, "null argument");
        if (!s->s.encode_only) {
            HIPCHK(hipSetDevice(s->s.device));
            kbhip::ev_harvest_all(s->s);
        }
        *out = s->s.stats;
        out->device_s = s->s.timed_ms * 1e-3;
        out->timed_launches = s->s.timed_n;
        out->host_launch_s = s->s.host_launch_s;
        out->host_wait_s = s->s.host_wait_s;
        out->alloc_device_s = s->s.alloc_device_s;
        return KBHIP_OK;
    })
}

int kbhip_set_option(kb_session* s, const char* key, int64_t value) {
    ABI_GUARD({
        if (!s || !key) throw kbhip::Error(KBHIP_EINVAL, "null argument");
        kbhip::require_no_tickets(s->s);  // options change how queued pops would run
        if (std::strcmp(key, "batched") == 0) s->s.batched = value != 0;
        else if (std::strcmp(key, "time_every") == 0) s->s.time_every = value;
        else if (std::strcmp(key, "sweep_variant") == 0) {  // kbhip_sweep_scores' kernel shape (tuning)
            if (value < 0 || value > 3) throw kbhip::Error(KBHIP_EINVAL, "sweep_variant must be 0..3");
            kbhip::set_sweep_variant((int)value);
        }
        else if (std::strcmp(key, "speculate") == 0) {
            if (value < 0 || value > kbhip::kMaxSpeculate) throw kbhip::Error(KBHIP_EINVAL, "speculate must be 0..6");
            s->s.speculate = (int)value;
        }
        else if (std::strcmp(key, "keys32") == 0) s->s.keys32 = value != 0;
        else if (std::strcmp(key, "engine") == 0 || std::strcmp(key, "engine_workers") == 0 ||
                 std::strcmp(key, "engine_timeline") == 0 || std::strcmp(key, "engine_quick") == 0 ||
                 std::strcmp(key, "engine_groups") == 0) {
            kbhip::Session& S = s->s;
            if (!S.encode_only) {
                HIPCHK(hipSetDevice(S.device));
                kbhip::ov_quiesce(S);  // the running engine (if any) ends first
            }
            if (key[6] == 0) {
                S.engine = value != 0;
            } else if (std::strcmp(key, "engine_groups") == 0) {
                if (value < -1 || value > kbhip::kEngMaxGroups) throw kbhip::Error(KBHIP_EINVAL, "engine_groups out of range");
                S.eng_ng_opt = (int)value;
                S.eng_nw = 0;  // sized again at the next engine pop
            } else if (std::strcmp(key, "engine_quick") == 0) {  // 0 (test mode): no fast path, every candidate in the levels
                S.eng_quick = value != 0;
            } else if (std::strcmp(key, "engine_timeline") == 0) {  // diagnostic: the engine's event stamps
                const size_t words = (size_t)kbhip::kEngTlSlots * kbhip::kEngTlEvents;
                if (value && !S.d_eng_tl && !S.encode_only) {
                    S.d_eng_tl = S.b_eng_tl.alloc<uint64_t>(words);
                    HIPCHK(hipMemset(S.d_eng_tl, 0, words * 8));
                }
            } else {
                if (value < 0 || value > kbhip::kEngWorkersMax) throw kbhip::Error(KBHIP_EINVAL, "engine_workers out of range");
                S.eng_nw_opt = (int)value;
                S.eng_nw = 0;  // sized again at the next engine pop
            }
        }
        else if (std::strcmp(key, "overlap") == 0) {
            if (value < 0 || value > kbhip::kMaxDep) throw kbhip::Error(KBHIP_EINVAL, "overlap must be 0, 1 or 2");
            if (!s->s.encode_only) {
                HIPCHK(hipSetDevice(s->s.device));
                kbhip::ov_quiesce(s->s);  // the stream rotation changes
            }
            s->s.overlap = (int)value;
        }
        else if (std::strcmp(key, "rank_radix") == 0) s->s.force_radix = value != 0;
        else if (std::strcmp(key, "bf_batch") == 0) s->s.bf_batch = value != 0;
        else if (std::strcmp(key, "aff_batch") == 0) s->s.aff_batch = value != 0;
        else if (std::strcmp(key, "aff_fence") == 0) s->s.aff_fence = value != 0;
        else if (std::strcmp(key, "shard_overlap") == 0) {
            if (!s->s.encode_only) {
                HIPCHK(hipSetDevice(s->s.device));
                kbhip::ov_quiesce(s->s);
            }
            s->s.shard_overlap = value != 0;
        }
        else if (std::strcmp(key, "rank_group") == 0) s->s.rank_group = value != 0;
        else if (std::strcmp(key, "rank_first") == 0) {  // reclaim / preempt: keys read back with the count
            if (value < 1) throw kbhip::Error(KBHIP_EINVAL, "rank_first must be >= 1");
            s->s.rank_first = (int)std::min<int64_t>(value, 1 << 20);
        } else if (std::strcmp(key, "debug_keys") == 0) {  // record per-task sweep keys (tests only)
            kbhip::Session& S = s->s;
            S.debug_keys = value != 0;
            if (S.debug_keys && !S.d_dbg && !S.encode_only) {
                HIPCHK(hipSetDevice(S.device));
                S.d_dbg = S.b_dbg.alloc<uint64_t>((size_t)kbhip::kMaxChunk * (2 * S.nc.npad + 4));
            }
        }
        else throw kbhip::Error(KBHIP_EINVAL, string("unknown option ") + key);
        return KBHIP_OK;
    })
}

#ifdef KBHIP_STAMPS
int kbhip_debug_phases(kb_session* s, double* out, int n) {
    ABI_GUARD({
        for (int i = 0; i < n && i < 20; ++i) out[i] = s->s.phase_n ? s->s.phase[i] / s->s.phase_n : 0;
        return (int)s->s.phase_n;
    })
}
#endif

#ifdef KBHIP_TIMELINE
// Diagnostic build only (libkbhip_tl.so): the overlapped pops' event timeline
// (kbhip_batch.h TL / TLB events).
// reset != 0 zeroes the buffer (allocating it once); otherwise copies it out.
int64_t kbhip_debug_timeline(kb_session* s, uint64_t* out, int64_t cap_words, int reset) {
    ABI_GUARD({
        static uint64_t* d_tl = nullptr;
        const size_t words = (size_t)32768 * 32 + (size_t)512 * 256 * 8;  // TL + TLB areas
        HIPCHK(hipSetDevice(s->s.device));
        if (!d_tl) {
            HIPCHK(hipMalloc(&d_tl, words * 8));
            HIPCHK(kbhip::set_timeline_buffer(d_tl));
        }
        HIPCHK(hipDeviceSynchronize());
        if (reset) HIPCHK(hipMemset(d_tl, 0, words * 8));
        else if (out && cap_words >= (int64_t)words) HIPCHK(hipMemcpy(out, d_tl, words * 8, hipMemcpyDeviceToHost));
        HIPCHK(hipDeviceSynchronize());
        return (int64_t)words;
    })
}
#endif

int kbhip_session_open_shard(const void* bytes, size_t len, int device, int32_t rank, int32_t world,
                             kb_session** out) {
    ABI_GUARD({
        if (!bytes || !out) throw kbhip::Error(KBHIP_EINVAL, "null argument");
        int nd = kbhip::device_count();
        if (nd <= 0) throw kbhip::Error(KBHIP_ENODEV, "no gfx950 HIP device available");
        if (device < 0 || device >= nd) throw kbhip::Error(KBHIP_EINVAL, "device index out of range");
        kbs::Snapshot snap;
        snap.load_bytes(bytes, len);
        std::unique_ptr<kb_session> s(new kb_session());
        kbhip::open_session(s->s, snap, device, false, rank, world);
        *out = s.release();
        return KBHIP_OK;
    })
}
int kbhip_shard_info(kb_session* s, int32_t* out4) {
    ABI_GUARD({
        if (!s || !out4) throw kbhip::Error(KBHIP_EINVAL, "null argument");
        out4[0] = s->s.rank;
        out4[1] = s->s.world;
        out4[2] = s->s.nc.base;
        out4[3] = s->s.nc.base + s->s.nc.n;
        return KBHIP_OK;
    })
}
int kbhip_rccl_unique_id(void* out, int64_t cap) {
    ABI_GUARD({
        ncclUniqueId id;
        if ((int64_t)sizeof(id) > cap || !out) throw kbhip::Error(KBHIP_EINVAL, "unique id buffer too small");
        const ncclResult_t r = ncclGetUniqueId(&id);
        if (r != ncclSuccess) throw kbhip::Error(KBHIP_EDEVICE, string("ncclGetUniqueId: ") + ncclGetErrorString(r));
        std::memcpy(out, &id, sizeof(id));
        return (int)sizeof(id);
    })
}
int kbhip_shard_connect_rccl(kb_session* s, const void* unique_id, int64_t len) {
    ABI_GUARD({
        if (!s || !unique_id) throw kbhip::Error(KBHIP_EINVAL, "null argument");
        ncclUniqueId id;
        if (len != (int64_t)sizeof(id)) throw kbhip::Error(KBHIP_EINVAL, "bad unique id length");
        std::memcpy(&id, unique_id, sizeof(id));
        if (s->s.comm) throw kbhip::Error(KBHIP_EINVAL, "session already connected");
        kbhip::require_no_tickets(s->s);
        HIPCHK(hipSetDevice(s->s.device));
        const string key((const char*)unique_id, sizeof(id));
        if (ncclComm_t c = kbhip::comm_acquire(key, s->s.rank, s->s.world, s->s.device)) {
            s->s.comm = c;  // a previous session's communicator (same id, rank, world, device)
            s->s.comm_pooled = true;
            s->s.stats.comm_reused = 1;
            return KBHIP_OK;
        }
        if (kbhip::comm_id_aborted(key))
            throw kbhip::Error(KBHIP_EINVAL, "the communicator of this unique id was aborted after a failed session; "
                                             "connect with a new kbhip_rccl_unique_id");
        ncclComm_t c = nullptr;
        const ncclResult_t r = ncclCommInitRank(&c, s->s.world, id, s->s.rank);
        if (r != ncclSuccess) throw kbhip::Error(KBHIP_EDEVICE, string("ncclCommInitRank: ") + ncclGetErrorString(r));
        kbhip::comm_add(key, s->s.rank, s->s.world, s->s.device, c);
        s->s.comm = c;
        s->s.comm_pooled = true;
        return KBHIP_OK;
    })
}
int kbhip_shard_connect_mailbox(kb_session* s, kbhip_allgather_fn fn, void* ctx) {
    ABI_GUARD_S(s, {
        if (!s || !fn) throw kbhip::Error(KBHIP_EINVAL, "null argument");
        kbhip::Session& S = s->s;
        if (S.encode_only) throw kbhip::Error(KBHIP_EINVAL, "encode-only session has no device state");
        if (S.mbox_own) throw kbhip::Error(KBHIP_EINVAL, "session already has a mailbox");
        kbhip::require_no_tickets(S);  // a new mailbox restarts its sequence under launched pops
        HIPCHK(hipSetDevice(S.device));
        using kbhip::Mailbox;
        {  // this rank's mailbox: the pooled one of this device, else a new allocation (uncached memory,
           // else fine-grained, else default) that can be exported
            kbhip::MboxPool& P = kbhip::MboxPool::get();
            std::lock_guard<std::mutex> lk(P.mu);
            auto it = P.free_own.find(S.device);
            if (it != P.free_own.end()) {
                S.mbox_own = it->second.first;
                S.mbox_kind = it->second.second;
                P.free_own.erase(it);
            }
        }
        hipIpcMemHandle_t h;
        if (!S.mbox_own) {
            const unsigned kinds[3] = {hipDeviceMallocUncached, hipDeviceMallocFinegrained, hipDeviceMallocDefault};
            for (int k = 0; k < 3 && !S.mbox_own; ++k) {
                void* p = nullptr;
                if (hipExtMallocWithFlags(&p, sizeof(Mailbox), kinds[k]) != hipSuccess) { (void)hipGetLastError(); continue; }
                if (hipIpcGetMemHandle(&h, p) != hipSuccess) {
                    (void)hipGetLastError();
                    (void)hipFree(p);
                    continue;
                }
                S.mbox_own = (Mailbox*)p;
                S.mbox_kind = k;
            }
            if (!S.mbox_own) throw kbhip::Error(KBHIP_EDEVICE, "no exportable device memory for the shard mailbox");
        }
        HIPCHK(hipIpcGetMemHandle(&h, S.mbox_own));
        HIPCHK(hipMemsetAsync(S.mbox_own, 0, sizeof(Mailbox), S.stream));  // flags 0: no pop yet
        HIPCHK(hipStreamSynchronize(S.stream));
        // every rank's record: its handle, process id and pointer (ranks of one process — threads
        // driving several shard sessions — use each other's pointers directly); the gather also
        // orders every rank's zeroing before any pop
        struct Rec {
            hipIpcMemHandle_t h;
            int64_t pid;
            uint64_t ptr;
        } mine{h, (int64_t)getpid(), (uint64_t)(uintptr_t)S.mbox_own};
        vector<Rec> recv((size_t)S.world);
        if (fn(ctx, &mine, recv.data(), (int64_t)sizeof(Rec)) != 0)
            throw kbhip::Error(KBHIP_EDEVICE, "mailbox handle all-gather callback failed");
        for (int p = 0; p < S.world; ++p) {
            if (p == S.rank) { S.mbox_peer[p] = S.mbox_own; continue; }
            if (recv[p].pid == (int64_t)getpid()) { S.mbox_peer[p] = (Mailbox*)(uintptr_t)recv[p].ptr; continue; }
            const string key((const char*)&recv[p].h, sizeof(h));
            kbhip::MboxPool& P = kbhip::MboxPool::get();
            std::lock_guard<std::mutex> lk(P.mu);
            auto it = P.opened.find(key);
            if (it == P.opened.end()) {
                hipIpcMemHandle_t ph;
                std::memcpy(&ph, key.data(), sizeof(ph));
                void* ptr = nullptr;
                HIPCHK(hipIpcOpenMemHandle(&ptr, ph, hipIpcMemLazyEnablePeerAccess));
                it = P.opened.emplace(key, ptr).first;
            }
            S.mbox_peer[p] = (Mailbox*)it->second;
        }
        S.mbox_seq = 0;
        return KBHIP_OK;
    })
}
int kbhip_shard_connect_host(kb_session* s, kbhip_allreduce_fn fn, void* ctx) {
    ABI_GUARD({
        if (!s || !fn) throw kbhip::Error(KBHIP_EINVAL, "null argument");
        kbhip::require_no_tickets(s->s);
        s->s.xfn = fn;
        s->s.xctx = ctx;
        return KBHIP_OK;
    })
}
int kbhip_shard_connect_host_gather(kb_session* s, kbhip_allgather_fn fn, void* ctx) {
    ABI_GUARD({
        if (!s || !fn) throw kbhip::Error(KBHIP_EINVAL, "null argument");
        kbhip::require_no_tickets(s->s);
        s->s.xgfn = fn;
        s->s.xgctx = ctx;
        return KBHIP_OK;
    })
}
int kbhip_debug_encode(const void* bytes, size_t len, kb_session** out) {
    ABI_GUARD({
        if (!bytes || !out) throw kbhip::Error(KBHIP_EINVAL, "null argument");
        kbs::Snapshot snap;
        snap.view_bytes(bytes, len);
        std::unique_ptr<kb_session> s(new kb_session());
        kbhip::open_session(s->s, snap, -1, true);
        *out = s.release();
        return KBHIP_OK;
    })
}
int64_t kbhip_debug_table(kb_session* s, const char* name, void* out, int64_t cap_bytes) {
    ABI_GUARD({
        if (!s || !name) throw kbhip::Error(KBHIP_EINVAL, "null argument");
        const kbhip::Session& S = s->s;
        vector<int32_t> v;
        const string n = name;
        if (n == "pod_class") {
            for (auto& p : S.pods) v.push_back(p.cls);
        } else if (n == "class_aff") {  // per class: 16 int32 fields (kbhip.h)
            for (auto& c : S.classes) {
                const int32_t f[16] = {c.aff, c.pred_err, c.ea_off, c.ea_n, c.pa_space, c.pa_cnt, c.pa_total,
                                       c.pa_self, c.paa_space, c.paa_cnt, c.ipa_off, c.ipa_n, c.upd_off, c.upd_n,
                                       c.score_err, 0};
                v.insert(v.end(), f, f + 16);
            }
        } else if (n == "aff_dom") {
            if (!S.encode_only) throw kbhip::Error(KBHIP_EINVAL, "tables are kept by encode-only sessions");
            v = S.h_dom;
        } else if (n == "aff_cnt" || n == "aff_scalar") {  // device sessions: the current device table
            if (S.encode_only) {
                v = n == "aff_cnt" ? S.h_aff_cnt : S.h_aff_scalar;
            } else {
                v.resize(n == "aff_cnt" ? S.n_aff_cnt : S.n_aff_scalar);
                HIPCHK(hipSetDevice(S.device));
                kbhip::ov_quiesce(s->s);
                HIPCHK(hipStreamSynchronize(S.stream));
                HIPCHK(hipMemcpy(v.data(), n == "aff_cnt" ? S.tab.aff_cnt : S.tab.aff_scalar, v.size() * 4,
                                 hipMemcpyDeviceToHost));
            }
        } else if (n == "aff_items") {
            v = S.h_aff_items;
        } else if (n == "dbg_keys") {  // u64 words, rows of 2 npad + 4 (kbhip_set_option "debug_keys")
            const int64_t bytes = (int64_t)(S.dbg_keys.size() * 8);
            if (out && cap_bytes >= bytes && bytes) std::memcpy(out, S.dbg_keys.data(), (size_t)bytes);
            return bytes;
        } else if (n == "dbg_pods") {
            v = S.dbg_pods;
        } else if (n == "engine_tl") {  // u64 words: kEngTlSlots x kEngTlEvents (option "engine_timeline")
            if (!S.d_eng_tl) throw kbhip::Error(KBHIP_EINVAL, "set option engine_timeline first");
            const int64_t bytes = (int64_t)kbhip::kEngTlSlots * kbhip::kEngTlEvents * 8;
            HIPCHK(hipSetDevice(S.device));
            kbhip::ov_quiesce(s->s);
            if (out && cap_bytes >= bytes) HIPCHK(hipMemcpy(out, S.d_eng_tl, (size_t)bytes, hipMemcpyDeviceToHost));
            return bytes;
        } else if (n == "pod_status" || n == "pod_node") {  // the host model: TaskStatus code / node per pod
            v.resize(S.pods.size());
            for (size_t i = 0; i < S.pods.size(); ++i) v[i] = n == "pod_status" ? S.pods[i].status : S.pods[i].node;
        } else if (n == "dims") {  // n_nodes, npad, n_spaces, n_classes
            v = {S.nc.n, S.nc.npad, S.n_spaces, (int32_t)S.classes.size()};
        } else {
            throw kbhip::Error(KBHIP_EINVAL, "unknown table " + n);
        }
        const int64_t bytes = (int64_t)(v.size() * sizeof(int32_t));
        if (out && cap_bytes >= bytes && bytes) std::memcpy(out, v.data(), (size_t)bytes);
        return bytes;
    })
}
int kbhip_debug_replay(kb_session* s, int32_t n_steps, const int32_t* pods, const int32_t* modes,
                       const int32_t* nodes, const uint8_t* kinds, uint64_t* out_keys) {
    ABI_GUARD({
        if (!s || (n_steps && (!pods || !modes || !nodes || !kinds || !out_keys)))
            throw kbhip::Error(KBHIP_EINVAL, "null argument");
        kbhip::Session& S = s->s;
        if (!S.encode_only) throw kbhip::Error(KBHIP_EINVAL, "replay needs an encode-only session");
        using namespace kbhip;
        const NodeCols& nc = S.nc;
        const DevTables& t = S.tab;
        const int N = nc.n;
        int F = -1, any_bf = S.any_bf;
        vector<uint64_t> walk(N);
        for (int i = 0; i < n_steps; ++i) {
            if (pods[i] < 0 || pods[i] >= (int)S.pods.size() || S.pods[pods[i]].cls < 0)
                throw Error(KBHIP_EINVAL, "replay step is not a pending task");
            const TaskClass& c = S.classes[S.pods[pods[i]].cls];
            uint64_t* keys = out_keys + (int64_t)i * N;
            const bool first_fit = modes[i] == 1;
            const bool track = !first_fit && any_bf;
            // the sweep: k_ipa_minmax + k_sweep_argmax, node by node
            int64_t lo = 0, hi = 0;
            if (!first_fit && c.ipa_n > 0)
                for (int n = 0; n < N; ++n) {
                    const int64_t v = ipa_count(c, t, nc, n, F);
                    lo = std::min(lo, v);
                    hi = std::max(hi, v);
                }
            for (int n = 0; n < N; ++n) {
                int32_t sc = 0;
                bool passed = false;
                keys[n] = first_fit ? eval_first_fit(S.conf, c, t, nc, n)
                                    : eval_node_aff(S.conf, c, t, nc, n, lo, hi, F, &sc, &passed);
                walk[n] = passed ? pack_key(sc, n + nc.base, 0) : 0;
            }
            // the commit of the given decision: commit_task's arithmetic
            const int w = nodes[i];
            if (w >= N) throw Error(KBHIP_EINVAL, "replay node out of range");
            const uint64_t k = w >= 0 ? keys[w] : 0;
            if (w >= 0 && !k) throw Error(KBHIP_EINVAL, "replay decision on a node with key 0");
            if (w >= 0) {
                const int kind = first_fit ? 1 : kinds[i];
                if (track) {
                    nc.idle_cpu[w] += nc.bf_cpu[w]; nc.idle_mem[w] += nc.bf_mem[w]; nc.idle_gpu[w] += nc.bf_gpu[w];
                }
                commit_node(c, t, nc, w, kind);
                if (c.aff) commit_aff(c, t, nc, w, kind);
                if (F < 0 || w < F) F = w;
                if (c.backfill) any_bf = 1;
            }
            if (track) {
                const uint64_t wk = k ? pack_key(key_score(k), key_idx(k), 0) : 0;
                for (int n = 0; n < N; ++n) {
                    if (!walk[n] || n == w) continue;
                    if (k && walk[n] < wk) continue;
                    nc.idle_cpu[n] += nc.bf_cpu[n]; nc.idle_mem[n] += nc.bf_mem[n]; nc.idle_gpu[n] += nc.bf_gpu[n];
                }
            }
        }
        return KBHIP_OK;
    })
}
int64_t kbhip_gang_unschedulable(kb_session* s, char* out, int64_t cap) {
    ABI_GUARD({
        if (!s) throw kbhip::Error(KBHIP_EINVAL, "null session");
        const std::string t = kbhip::gang_close_text(s->s);
        if (out && cap > (int64_t)t.size()) std::memcpy(out, t.c_str(), t.size() + 1);
        return (int64_t)t.size();
    })
}

int kbhip_session_close(kb_session* s) {
    ABI_GUARD({
        static const bool prof = std::getenv("KBHIP_OPEN_PROFILE") != nullptr;
        auto t0 = std::chrono::steady_clock::now();
        if (s && !s->s.encode_only) {
            (void)hipSetDevice(s->s.device);
            s->s.release_device();
        }
        delete s;  // the host model: freeing it on another thread measured slower (contention with the next open)
        if (prof)
            std::fprintf(stderr, "[close] total      %8.2f ms\n",
                         std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() * 1e3);
        return KBHIP_OK;
    })
}

}  // extern "C"
