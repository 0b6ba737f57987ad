// kbhip session, part 07: the remaining C-ABI entry points (carry, options, shards, debug, close)
#include "session.h"

using namespace kbhip;

extern "C" {
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
        else if (std::strcmp(key, "cu_split") == 0) {  // value = part * 256 + parts (rehearsals)
            kbhip::require_no_tickets(s->s);
            HIPCHK(hipSetDevice(s->s.device));
            kbhip::cu_split(s->s, (int)(value >> 8), (int)(value & 0xff));
        }
        else if (std::strcmp(key, "sweep_variant") == 0) {  // kbhip_sweep_scores' kernel shape (tuning)
            if (value < 0 || value > 6) throw kbhip::Error(KBHIP_EINVAL, "sweep_variant must be 0..6");
            kbhip::set_sweep_variant((int)value);
        }
        else if (std::strcmp(key, "speculate") == 0) {
            if (value < 0 || value > kbhip::kMaxSpeculate) throw kbhip::Error(KBHIP_EINVAL, "speculate must be 0..6");
            s->s.speculate = (int)value;
        }
        else if (std::strcmp(key, "keys32") == 0) s->s.keys32 = value != 0;
        else if (std::strcmp(key, "time_sweeps_cold") == 0) {
            if (value < 0 || value > 2) throw kbhip::Error(KBHIP_EINVAL, "time_sweeps_cold must be 0..2");
            s->s.sweeps_cold = (int)value;
        }
        else if (std::strcmp(key, "engine") == 0 || std::strcmp(key, "engine_workers") == 0 ||
                 std::strcmp(key, "engine_timeline") == 0 || std::strcmp(key, "engine_quick") == 0 ||
                 std::strcmp(key, "engine_groups") == 0 || std::strcmp(key, "engine_lists") == 0) {
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
            } else if (std::strcmp(key, "engine_lists") == 0) {  // list mode (class owners) when it fits; 0: sweep mode
                S.eng_lists = value != 0;
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
        else if (std::strcmp(key, "rank_group") == 0) {
            s->s.rank_group = value != 0;
            s->set_grouped(value != 0);
        } else if (std::strcmp(key, "group_linger_us") == 0) {  // test knob, process-wide
            if (value < 0 || value > 1000000) throw kbhip::Error(KBHIP_EINVAL, "group_linger_us must be 0..1e6");
            kbhip::StepBatcher::get().linger_us.store(value);
        }
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
        // a failure after this point hands the mailbox back and leaves the session unconnected
        // (so that a later connect, or kbhip_shard_connect_host_gather, starts clean)
        struct Rollback {
            kbhip::Session& S;
            bool done = false;
            ~Rollback() {
                if (done) return;
                if (S.mbox_own) {
                    kbhip::MboxPool& P = kbhip::MboxPool::get();
                    std::lock_guard<std::mutex> lk(P.mu);
                    P.free_own.emplace(S.device, std::make_pair(S.mbox_own, S.mbox_kind));
                }
                S.mbox_own = nullptr;
                for (auto& m : S.mbox_peer) m = nullptr;
            }
        } rollback{S};
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
            uint64_t proc;  // process_token(): unique across hosts and containers
            uint64_t ptr;
            int64_t device;
        } mine{h, kbhip::process_token(), (uint64_t)(uintptr_t)S.mbox_own, (int64_t)S.device};
        vector<Rec> recv((size_t)S.world);
        if (fn(ctx, &mine, recv.data(), (int64_t)sizeof(Rec)) != 0)
            throw kbhip::Error(KBHIP_EDEVICE, "mailbox handle all-gather callback failed");
        {  // ranks of this process on this device: their streams must not share a hardware queue
            int k = 0;
            for (const Rec& r : recv) k += r.proc == kbhip::process_token() && r.device == (int64_t)S.device;
            const std::string why = kbhip::mailbox_queue_check(k, kbhip::hw_queues());
            if (!why.empty()) throw kbhip::Error(KBHIP_EUNSUPPORTED, why);
        }
        for (int p = 0; p < S.world; ++p) {
            if (p == S.rank) { S.mbox_peer[p] = S.mbox_own; continue; }
            if (recv[p].proc == kbhip::process_token()) { S.mbox_peer[p] = (Mailbox*)(uintptr_t)recv[p].ptr; continue; }
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
        rollback.done = true;
        return KBHIP_OK;
    })
}
int kbhip_shard_mailbox_fits(int32_t ranks_on_device, int32_t hw_queues) {
    return kbhip::mailbox_queue_check(ranks_on_device, hw_queues > 0 ? hw_queues : kbhip::hw_queues()).empty() ? 1 : 0;
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
        const auto t1 = std::chrono::steady_clock::now();
        delete s;  // the host model: freeing it on another thread measured slower (contention with the next open)
        if (prof)
            std::fprintf(stderr, "[close] total      %8.2f ms (device %.2f ms)\n",
                         std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() * 1e3,
                         std::chrono::duration<double>(t1 - t0).count() * 1e3);
        return KBHIP_OK;
    })
}

}  // extern "C"
