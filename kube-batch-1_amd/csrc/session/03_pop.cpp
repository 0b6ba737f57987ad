// kbhip session, part 03: the per-pop device driver (batched pops, the persistent engine, tickets)
#include "session.h"

namespace kbhip {

// ---------------------------------------------------------------------------
// cross-shard exchange of n 8-byte values in device memory:
// RCCL all-reduce on the session stream, or a host round trip through the
// caller's callback (tests: several ranks sharing one GPU over gloo).
// ---------------------------------------------------------------------------
// KBHIP_TRACE_SHARD=1: every collective of a shard session on stderr (diagnostic)
static const bool g_trace_shard = std::getenv("KBHIP_TRACE_SHARD") != nullptr;
void exchange(Session& S, void* dev, int op, int n) {
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
void fit_allreduce(Session& S, int32_t* fit4) {
    if (S.world == 1) return;
    int64_t* d = (int64_t*)S.d_fit4 + 2;  // after the device counters (int32[4])
    int64_t h[4] = {fit4[0], fit4[1], fit4[2], fit4[3]};
    HIPCHK(hipMemcpyAsync(d, h, sizeof h, hipMemcpyHostToDevice, S.stream));
    exchange(S, d, KBHIP_RED_SUM_I64, 4);
    HIPCHK(hipMemcpyAsync(h, d, sizeof h, hipMemcpyDeviceToHost, S.stream));
    HIPCHK(hipStreamSynchronize(S.stream));
    for (int q = 0; q < 4; ++q) fit4[q] = (int32_t)h[q];
}

// All-gather of `bytes` host bytes per rank into recv, in rank order (the
// eviction actions' node rankings on shards): the host callback, or RCCL
// through a device staging buffer on the session stream.
void gather_host(Session& S, const void* send, void* recv, size_t bytes) {
    S.stats.collectives++;
    if (g_trace_shard)
        std::fprintf(stderr, "[shard %d] #%lld all-gather %zu bytes\n", S.rank, (long long)S.stats.collectives, bytes);
    if (S.xgfn) {
        if (S.xgfn(S.xgctx, send, recv, (int64_t)bytes) != 0) throw Error(KBHIP_EDEVICE, "shard all-gather callback failed");
        return;
    }
    if (!S.comm) throw Error(KBHIP_EINVAL, "sharded session has no all-gather (kbhip_shard_connect_*)");
    uint8_t* d = S.b_gather.alloc<uint8_t>(bytes * (S.world + 1));
    HIPCHK(hipMemcpyAsync(d + bytes * S.world, send, bytes, hipMemcpyHostToDevice, S.stream));
    const ncclResult_t r = ncclAllGather(d + bytes * S.world, d, bytes, ncclUint8, S.comm, S.stream);
    if (r != ncclSuccess) throw Error(KBHIP_EDEVICE, string("ncclAllGather: ") + ncclGetErrorString(r));
    HIPCHK(hipMemcpyAsync(recv, d, bytes * S.world, hipMemcpyDeviceToHost, S.stream));
    HIPCHK(hipStreamSynchronize(S.stream));
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
void sweep_task(Session& S, int i, int cls, bool defer_visits) {
    int64_t* ipa = nullptr;
    if (S.classes[cls].ipa_n > 0) {
        if (!S.d_ipa) S.d_ipa = S.b_ipa.alloc<int64_t>((size_t)S.nc.npad);
        ipa = S.d_ipa;
        HIPCHK(launch_ipa_minmax(S.nc, S.tab, S.d_ctrl, i, S.stream, ipa));
        exchange(S, &S.d_ctrl->ipa_lo[i], KBHIP_RED_MIN_I64);
        exchange(S, &S.d_ctrl->ipa_hi[i], KBHIP_RED_MAX_I64);
    }
    HIPCHK(launch_sweep_argmax(S.conf, S.nc, S.tab, S.d_ctrl, i, S.d_walk, S.stream, S.world == 1, S.d_dbg,
                               defer_visits && S.world == 1, ipa));
    if (S.world > 1) {
        exchange(S, &S.d_ctrl->slot[i], KBHIP_RED_MAX_U64);
        HIPCHK(launch_commit_task(S.nc, S.tab, S.d_ctrl, i, S.d_walk, S.stream));
    }
}


// The sweeps of a per-task chunk (tasks 0 .. m-1 of the control block): one
// k_sweep_argmax launch per task, or, for a what-if session of the batched
// group, one request that the StepBatcher serves together with the other
// sessions' pending chunks (k_sweep_argmax_multi: task k of every chunk in one launch).
// Classes with inter-pod priority terms (their k_ipa_minmax prepass) and
// debug-key sessions keep the per-task launches.
void sweep_chunk(Session& S, int m, const int* cls, bool defer, bool per_task) {
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
// Restart hysteresis (eng_eligible / eng_stop): a run that an engine-ineligible
// pop ended after fewer than kEngShortRun pops sets the backoff to 8 or doubles
// it (at most kEngBackoffMax); a run of 4 * kEngShortRun pops or more clears it.
static constexpr int kEngShortRun = 16;
static constexpr int kEngBackoffMax = 64;

// A class the engine can serve (with a session that can run it, eng_eligible):
// no pod affinity, host ports or backfill annotation, 32-bit keys and entries.
static bool eng_class_ok(const Session& S, int cls, const KeyFormat& kf) {
    const TaskClass& c = S.classes[cls];
    return !(c.aff || c.has_ports || c.backfill || !kf.use32 || !kf.ent32);
}

// List mode: one owner block per eligible class, when every
// eligible class's score range fits an owner's key byte, the node array fits
// its LDS, and the owners plus the placer and the dispatcher stay resident.
// Fills S.eng_own_of; returns the owners' classes (empty: sweep mode).
static vector<int32_t> eng_owners(Session& S, int resident) {
    vector<int32_t> own;
    S.eng_own_of.assign(S.classes.size(), -1);
    if (!S.eng_lists || !S.keys32 || S.nc.base != 0 || S.nc.n > kOwnMaxN) return own;
    for (size_t ci = 0; ci < S.classes.size(); ++ci) {
        const KeyFormat& kf = S.class_kf[ci];
        if (!eng_class_ok(S, (int)ci, kf)) continue;
        const int64_t levels = S.class_srange[ci].second - S.class_srange[ci].first + 1;
        if (levels < 1 || levels > kOwnLv - 1 || kf.base != S.class_srange[ci].first) return {};
        own.push_back((int32_t)ci);
    }
    if (own.empty() || (int)own.size() + 2 > std::min(resident, kEngOwnMax)) return {};
    for (size_t o = 0; o < own.size(); ++o) S.eng_own_of[own[o]] = (int32_t)o;
    return own;
}

static void eng_size(Session& S) {
    S.eng_nw = -1;
    S.eng_nown = 0;
    S.eng_ncls = S.classes.size();
    const int N = S.nc.n;
    if (S.encode_only || S.world != 1 || N < 1) return;
    int cus = 0, bpc = 0, bpc_l = 0;
    HIPCHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, S.device));
    HIPCHK(engine_occupancy(&bpc));
    HIPCHK(engine_occupancy(&bpc_l, true));
    const vector<int32_t> own = eng_owners(S, cus * bpc_l);
    int nw = 0, ng = 0, npb = 0;
    if (!own.empty()) {  // list mode: the placer reads one owner's count words (a "worker list" slot)
        nw = 1;
        npb = N;
    } else {
        const int resident = cus * bpc;  // every block of the grid must be resident at once
        nw = std::min(kEngWorkersMax, resident - kEngMaxGroups - 3);  // + final merger, placer, dispatcher
        if (S.eng_nw_opt > 0) nw = std::min(nw, S.eng_nw_opt);
        nw = std::min(nw, std::max(1, (N + 63) / 64));  // at least 64 nodes per worker
        if (nw < 1) return;
        npb = (N + nw - 1) / nw;
        if (npb > kEngMaxNpb) return;
        ng = S.eng_ng_opt >= 0 ? std::min(S.eng_ng_opt, nw) : std::min(kEngMaxGroups, nw);
    }
    const size_t lists = (size_t)kEngSlots * (nw + ng) * kEngListWords;
    static_assert(sizeof(EngCtl) % 256 == 0 && sizeof(EngPkg) % 256 == 0, "engine buffers stay line-aligned");
    const size_t words = (sizeof(EngCtl) + kEngSlots * sizeof(EngPkg)) / 8 + lists;
    char* d = (char*)S.b_eng.alloc<uint64_t>(words);
    S.d_eng_ctl = (EngCtl*)d;
    S.d_eng_pkg = (EngPkg*)(d + sizeof(EngCtl));
    S.d_eng_bl = (uint64_t*)(d + sizeof(EngCtl) + kEngSlots * sizeof(EngPkg));
    S.d_eng_gl = S.d_eng_bl + (size_t)kEngSlots * nw * kEngListWords;
    HIPCHK(hipMemsetAsync(d, 0, words * 8, S.stream));  // every tag 0: no pop has that sequence number
    if (!own.empty()) {  // owners' classes and key bases, then their FitDelta bits ([nown][npad] bytes)
        const size_t no = own.size();
        vector<int32_t> h(2 * no);
        for (size_t o = 0; o < no; ++o) {
            h[o] = own[o];
            h[no + o] = S.class_kf[own[o]].base;
        }
        const size_t bytes = 2 * no * sizeof(int32_t) + no * (size_t)S.nc.npad;
        char* b = (char*)S.b_eng_own.alloc<uint64_t>((bytes + 7) / 8);
        HIPCHK(hipMemcpyAsync(b, h.data(), h.size() * sizeof(int32_t), hipMemcpyHostToDevice, S.stream));
        HIPCHK(hipStreamSynchronize(S.stream));  // (h is a local)
        S.eng_nown = (int)no;
        S.eng_kshift = S.class_kf[own[0]].shift;  // (every class: the node count's index bits)
        S.eng_kidxmax = S.class_kf[own[0]].idxmax;
    }
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
    S.stats.engine_workers = S.eng_nown ? 0 : nw;
    S.stats.engine_owners = S.eng_nown;
}

static void eng_stop(Session& S);
static bool eng_claim(Session& S);

// A batched pop the engine can serve: one GPU, no Backfilled nodes, an
// eligible class (eng_class_ok) — in list mode one with an owner.  A stopped
// engine starts again after more than S.eng_backoff such pops in a row (the
// ones before take the launched path: same results, no launch + exit of the
// persistent grid for a run of a few pops).
static bool eng_eligible(Session& S, int cls, const KeyFormat& kf) {
    if (!S.engine || S.world != 1 || S.any_bf || S.rank_group || S.encode_only) return false;
    if (!eng_class_ok(S, cls, kf)) {
        S.eng_streak = 0;
        S.eng_stop_cls = S.eng_running;  // the stop that follows (launch_batched) ends the run for this pop
        return false;
    }
    if (S.eng_nw != 0 && S.eng_ncls != S.classes.size()) {  // a carry added classes: size again (owners)
        eng_stop(S);
        S.eng_nw = 0;
    }
    if (S.eng_nw == 0) eng_size(S);
    if (!(S.eng_nw > 0 && (S.eng_nown == 0 || S.eng_own_of[cls] >= 0))) return false;
    if (S.eng_running) return true;
    if (++S.eng_streak <= S.eng_backoff) return false;
    return eng_claim(S);  // another session's engine on this device: the launched path
}

static uint64_t* eng_exit_word(Session& S) { return S.h_eng + kEngHostRing * kEngDescWords; }

static void eng_write(Session& S, uint32_t seq, const uint32_t* w) {
    uint64_t* slot = S.h_eng + (size_t)(seq % kEngHostRing) * kEngDescWords;
    for (int i = 0; i < kEngDescWords; ++i) __atomic_store_n(&slot[i], ((uint64_t)seq << 32) | w[i], __ATOMIC_RELEASE);
}

// One engine per device in this process (its grid must be resident whole; a
// second one would wait for CUs the first holds): a session claims the device
// before its first engine pop and keeps the claim until its engine has served
// every descriptor written (eng_release); other sessions' pops take the
// launched path meanwhile.  Across processes the grid's arrival check guards
// (eng_arrive: a grid that cannot become resident ends, and is started again).
struct EngArbiter {
    std::mutex mu;
    std::map<int, const Session*> holder;  // device -> the session whose engine may run there
    static EngArbiter& get() {
        static EngArbiter a;
        return a;
    }
};
static bool eng_claim(Session& S) {
    if (S.eng_claimed) return true;
    EngArbiter& A = EngArbiter::get();
    std::lock_guard<std::mutex> lk(A.mu);
    const Session*& h = A.holder[S.device];
    if (h && h != &S) return false;
    h = &S;
    S.eng_claimed = true;
    return true;
}
static void eng_release(Session& S) {
    if (!S.eng_claimed || S.eng_running) return;
    EngArbiter& A = EngArbiter::get();
    std::lock_guard<std::mutex> lk(A.mu);
    auto it = A.holder.find(S.device);
    if (it != A.holder.end() && it->second == &S) A.holder.erase(it);
    S.eng_claimed = false;
}

void Session::eng_unclaim() {
    eng_running = false;  // (release_device: the exit descriptor is written, the stream drained)
    eng_release(*this);
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
    A.idle_ticks = kEngIdleTicks;
    A.nown = S.eng_nown;
    if (S.eng_nown) {
        char* b = (char*)S.b_eng_own.p;
        A.own_cls = (const int32_t*)b;
        A.own_kbase = (const int32_t*)b + S.eng_nown;
        A.own_fb = (uint8_t*)(b + 2 * (size_t)S.eng_nown * sizeof(int32_t));
        A.kshift = S.eng_kshift;
        A.kidxmax = S.eng_kidxmax;
    }
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
    S.msg_from = S.ov_seq + 1;    // the overlapped path's row messages are stale now
    S.chain_fence = true;
    if (err == kEngErrResident && (x & (1ull << 41)) && (x & (1ull << 42))) {
        // the grid could not become resident (other kernels held CUs): it served nothing;
        // the caller starts it again (after a short pause, so that those kernels can end)
        S.stats.engine_not_resident++;
        std::this_thread::sleep_for(std::chrono::microseconds(500));
        return;
    }
    if (err || !(x & (1ull << 41))) throw Error(KBHIP_EDEVICE, "the pop engine stopped on a fault (error " +
                                                                    std::to_string(err) + ")");
    S.eng_first = (uint32_t)(x & 0xffffffffu);
    const bool idle = (x >> 40) & 1;
    if (!idle) S.eng_first += 1;  // an exit descriptor took that sequence number
}

// While waiting for an engine pop: a kernel that ended idle before it read
// descriptors written meanwhile is restarted.  true: it was.
static bool eng_poll(Session& S) {
    if (!S.eng_running) return false;
    const uint64_t x = __atomic_load_n(eng_exit_word(S), __ATOMIC_ACQUIRE);
    if (!(x & (1ull << 41))) return false;
    eng_ended(S);
    if ((int32_t)(S.eng_seq - S.eng_first) >= 0) eng_start(S);  // descriptors it never served
    else eng_release(S);
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
        S.eng_run_pops0 = S.stats.engine_pops;
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
        if ((int32_t)(S.eng_first - sq) > 0) {  // it reached the exit descriptor
            eng_release(S);
            // the restart hysteresis: runs ended by an engine-ineligible pop (other stops leave it)
            const int64_t served = S.stats.engine_pops - S.eng_run_pops0;
            if (S.eng_stop_cls && served < kEngShortRun)
                S.eng_backoff = std::min(kEngBackoffMax, std::max(8, 2 * S.eng_backoff));
            else if (served >= 4 * kEngShortRun)
                S.eng_backoff = 0;
            S.eng_stop_cls = false;
            S.eng_streak = 0;
            return;
        }
        eng_start(S);  // it ended idle (or was not resident) before that: serve the rest
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
void ov_quiesce(Session& S) { ov_drain(S); }

// The device-side form of ov_quiesce for a non-overlapped batched pop on the
// session stream (placement 7): that stream waits for the end of every
// overlap stream's work, without the host waiting.  Row messages of earlier
// pops go stale as after a drain (the pop writes rows outside their
// candidate lists); the overlapped pops after it wait for it (ev_nonov).
void ov_fence(Session& S) {
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
void ev_harvest_all(Session& S) {
    for (int k = 0; k < Session::kEvRing; ++k) ev_harvest(S, k);
}

bool batchable(const Session& S, int cls) {
    const TaskClass& c = S.classes[cls];
    // Backfilled nodes (some Idle grows on each walk visit): placement 6, one GPU only
    const bool bf_ok = !S.any_bf || (S.world == 1 && S.bf_batch);
    // pod-affinity classes: placement 7 (anti-affinity predicates only), one GPU, no Backfilled nodes
    const bool aff_ok = !c.aff || (S.aff_batch && S.world == 1 && !S.any_bf && aff_batchable(c));
    return S.batched && (S.world == 1 || S.comm || S.xgfn || S.mbox_own) && bf_ok && !c.backfill && aff_ok &&
           S.n_total < (1 << 25);
}

// The next result slot (pinned, mapped PopOutHost) and its granules' tag.
int take_slot(Session& S, uint32_t* epoch) {
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
void ctrl_setup(Session& S, int m, const int* cls, int ready, int min_avail, int gang, int mode, int slot,
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
void collect_tasks(Session& S, int slot, uint32_t epoch, int m, int* n_done, int* stop, int32_t* node,
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

BatchLaunch launch_batched(Session& S, int cls, int m, int gang_mode, int min_avail, int ready_count) {
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
    // A session of the what-if group sends every batched pop to the group (one pop in flight per
    // session, so the other sessions' pops can share its launch): a pop without Backfilled nodes uses placement 7, which is exact for any class — with no
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
void collect_batched(Session& S, const BatchLaunch& L, int* n_done_out, int* stop_out, int32_t* res_node,
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
void sess_placed(Session& S, int n, int d) {
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
void queue_target(Session& S, int pi, int sign) {
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
void flush_tables(Session& S) {
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
void apply_results(Session& S, const int32_t* ids, int n, const int32_t* res_node, const int32_t* res_kind,
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

int place_job(Session& S, const int32_t* ids, int n, int gang_mode, int min_avail, int ready_count,
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

void require_no_tickets(const Session& S) {
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

int64_t place_job_submit(Session& S, const int32_t* ids, int n, int gang_mode, int min_avail,
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

int place_job_wait(Session& S, int64_t ticket, int32_t* out_node, uint8_t* out_kind, int32_t* out_n_done,
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

int place_job_cancel(Session& S, int64_t ticket) {
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

}  // namespace kbhip
