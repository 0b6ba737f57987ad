// kbhip_kernels.hip — gfx950 kernels of the placement engine.
//
// One sweep evaluates, for one task class and every node, the predicates
// plugin (pkg/scheduler/plugins/predicates/predicates.go:123-203), the
// nodeorder score (plugins/nodeorder/nodeorder.go:252-317) and the fit test
// of the allocate walk (actions/allocate/allocate.go:149-185), and reduces to
// the packed key (score, -index): the argmax of that key over feasible nodes
// IS the node util.SelectBestNode + the walk would pick.
//
// Two ways to use a sweep:
//  * per-task (general): k_sweep_argmax — one launch per task, 64-lane
//    wave reduction -> LDS block reduction -> one 64-bit atomicMax per block;
//    the last block to arrive commits the winner (Session.Allocate/Pipeline
//    node update) and decides whether the job pop stops.
//  * batched: when every task of a pop chunk has the same class and nothing
//    but the winner's row can change between tasks, ONE launch serves the
//    whole chunk: k_pop_batch sweeps, keeps the global top-64 keys and places
//    the chunk's tasks in sequence against that sorted candidate list,
//    re-evaluating only rows it changed.  Placements are identical to
//    per-task sweeps (tests/test_gpu_parity.py).
//  * pod (anti-)affinity classes always take the per-task path: their
//    predicate and inter-pod score read count tables every commit may change
//    (kbhip_affinity.h); k_ipa_minmax is the score's normalisation prepass.
#include <hip/hip_runtime.h>
#include <cstdlib>
#include <vector>

#include "kbhip_batch.h"
#include "kbhip_internal.h"

// Built as three translation units (Makefile: KBHIP_PART 1, 2, 3) so that the
// template instantiations compile in parallel; KBHIP_PART 0 = all of it.
#ifndef KBHIP_PART
#define KBHIP_PART 0
#endif

namespace kbhip {


#if KBHIP_PART <= 1  // everything but the batched-pop launchers of parts 2 / 3
__global__ __launch_bounds__(kBlock) void k_ipa_minmax(NodeCols nc, DevTables t, PopCtrl* ctrl, int task_i,
                                                       int64_t* counts) {
    __shared__ int64_t rlo[kBlock / 64], rhi[kBlock / 64];
    if (ctrl->stop >= 0) return;
    const int cls = __builtin_amdgcn_readfirstlane(ctrl->cls[task_i]);
    const TaskClass c = t.classes[cls];
    const int F = ctrl->fallback;
    int64_t lo = 0, hi = 0;  // maxCount / minCount start at 0 (interpod_affinity.go:214-226)
    for (int n = blockIdx.x * kBlock + threadIdx.x; n < nc.n; n += gridDim.x * kBlock) {
        const int64_t v = ipa_count(c, t, nc, n, F);
        if (counts) counts[n] = v;  // (the sweep that follows reads them instead of counting again)
        lo = v < lo ? v : lo;
        hi = v > hi ? v : hi;
    }
    for (int o = 32; o > 0; o >>= 1) {
        const int64_t a = __shfl_xor(lo, o, 64), b = __shfl_xor(hi, o, 64);
        lo = a < lo ? a : lo;
        hi = b > hi ? b : hi;
    }
    if ((threadIdx.x & 63) == 0) { rlo[threadIdx.x >> 6] = lo; rhi[threadIdx.x >> 6] = hi; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kBlock / 64; ++w) { lo = rlo[w] < lo ? rlo[w] : lo; hi = rhi[w] > hi ? rhi[w] : hi; }
        lo = rlo[0] < lo ? rlo[0] : lo;
        hi = rhi[0] > hi ? rhi[0] : hi;
        if (lo < 0) atomicMin((long long*)&ctrl->ipa_lo[task_i], (long long)lo);
        if (hi > 0) atomicMax((long long*)&ctrl->ipa_hi[task_i], (long long)hi);
    }
}


// ---------------------------------------------------------------------------
// per-task path
// ---------------------------------------------------------------------------
// The chunk's control block: the request fields from the kernel argument,
// every per-task counter and result cleared.
__global__ __launch_bounds__(kBlock) void k_ctrl_init(PopCtrl* ctrl, CtrlInit ci) {
    const int i = threadIdx.x;
    if (i == 0) {
        ctrl->stop = -1;
        ctrl->n_done = 0;
        ctrl->ready_count = ci.ready_count;
        ctrl->min_avail = ci.min_avail;
        ctrl->gang_mode = ci.gang_mode;
        ctrl->n_tasks = ci.n_tasks;
        ctrl->any_bf = ci.any_bf;
        ctrl->fallback = ci.fallback;
        ctrl->mode = ci.mode;
        ctrl->pad = 0;
        ctrl->epoch = ci.epoch;
        ctrl->out = ci.out;
    }
    if (i < kMaxChunk) {
        ctrl->cls[i] = ci.cls[i];
        ctrl->res_node[i] = -1;
        ctrl->res_kind[i] = 0;
        ctrl->arrive[i] = 0;
        ctrl->slot[i] = 0;
        ctrl->ipa_lo[i] = 0;
        ctrl->ipa_hi[i] = 0;
        for (int q = 0; q < 4; ++q) ctrl->fit[i][q] = 0;
    }
}
hipError_t launch_ctrl_init(PopCtrl* ctrl, const CtrlInit& ci, hipStream_t st) {
    hipLaunchKernelGGL(k_ctrl_init, dim3(1), dim3(kBlock), 0, st, ctrl, ci);
    return hipGetLastError();
}

// The result of task task_i as a self-tagged granule in pinned host memory
// (the batched path's PopOut format; the host polls instead of copying the
// control block back): stop after this task, tasks consumed, kind, node; a
// task that found no node also sends this shard's walk FitDelta counts.
__device__ void task_granule(PopCtrl* ctrl, int task_i, int kind, int node) {
    PopOut* out = (PopOut*)ctrl->out;
    if (!out) return;
    if (ctrl->stop == 1) {
        int32_t f[4];
        for (int q = 0; q < 4; ++q)
            f[q] = __hip_atomic_load(&ctrl->fit[task_i][q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&out->fit[0], make_fit_granule(ctrl->epoch, f[0], f[1]), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&out->fit[1], make_fit_granule(ctrl->epoch, f[2], f[3]), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    }
    __hip_atomic_store(&out->g[task_i], make_granule(ctrl->epoch, ctrl->stop, ctrl->n_done, kind, node),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// Commit of task task_i once ctrl->slot[task_i] holds the winner key over ALL
// nodes (all shards): result, gang stop, node row (owner only), pod-affinity
// tables and fallback node (every shard, identically), and the
// GetAccessibleResource mutation of the visited nodes of this shard.  Run by
// one block: the last sweep block (one GPU) or k_commit_task (sharded).
__device__ void commit_task(const NodeCols& nc, const DevTables& t, PopCtrl* ctrl, int task_i, const TaskClass& c,
                            bool first_fit, bool track, const uint64_t* walk, bool defer_visits = false) {
    __shared__ uint64_t win;
    __shared__ int s_aff_g, s_aff_kind;  // the pod-affinity count tables' commit (global node, kind; -1: none)
    if (threadIdx.x == 0) {
        s_aff_g = -1;
        const uint64_t k = __hip_atomic_load(&ctrl->slot[task_i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        win = k;
        const int g = k ? key_idx(k) : -1;            // global node index
        const int n = g - nc.base;                    // local row
        const bool own = k && n >= 0 && n < nc.n;
        if (first_fit) {  // backfill: Session.Allocate on the first passing node; no stop rule
            ctrl->res_node[task_i] = g;
            ctrl->res_kind[task_i] = k ? 1 : 0;
            if (k) {
                if (own) commit_node(c, t, nc, n, 1);
                s_aff_g = g;
                s_aff_kind = 1;
                if (ctrl->fallback < 0 || g < ctrl->fallback) ctrl->fallback = g;
                if (c.backfill) ctrl->any_bf = 1;
            }
            ctrl->n_done = task_i + 1;
            if (task_i + 1 == ctrl->n_tasks) ctrl->stop = 0;
            task_granule(ctrl, task_i, k ? 1 : 0, g);
        } else if (k == 0) {
            ctrl->res_node[task_i] = -1;
            ctrl->res_kind[task_i] = 0;
            ctrl->n_done = task_i + 1;
            ctrl->stop = 1;
            task_granule(ctrl, task_i, 0, -1);
        } else {
            const int kind = key_kind(k);
            ctrl->res_node[task_i] = g;
            ctrl->res_kind[task_i] = kind;
            if (own) {
                if (track) {  // the winner is visited too: Idle += Backfilled first (node_info.go:209-211)
                    nc.idle_cpu[n] += nc.bf_cpu[n]; nc.idle_mem[n] += nc.bf_mem[n]; nc.idle_gpu[n] += nc.bf_gpu[n];
                }
                commit_node(c, t, nc, n, kind);
            }
            s_aff_g = g;
            s_aff_kind = kind;
            if (ctrl->fallback < 0 || g < ctrl->fallback) ctrl->fallback = g;
            if (c.backfill) ctrl->any_bf = 1;
            after_assign(ctrl, task_i, kind);
            task_granule(ctrl, task_i, kind, g);
        }
    }
    __syncthreads();
    // commit_aff with one update per lane (was one lane looping over the class's updates, each a
    // dependent chain of loads and a read-modify-write); atomic: two updates may share an entry
    if (c.aff && s_aff_g >= 0 && (int)threadIdx.x < c.upd_n) {
        const int32_t* it = t.aff_items + c.upd_off + 3 * threadIdx.x;
        const bool to_cnt = it[0] == 0;
        const int d = to_cnt ? dom_g(nc, it[1], s_aff_g) : 0;
        const bool apply = (it[0] == 2 || s_aff_kind == 1) && d >= 0;
        int32_t* tab = to_cnt ? t.aff_cnt : t.aff_scalar;
        __hip_atomic_fetch_add(tab + it[2] + (d >= 0 ? d : 0), apply ? 1 : 0, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
    if (defer_visits) {  // k_visit_mutate does the loop below over the whole grid
        if (threadIdx.x == 0) ctrl->pad = track ? 1 : 0;
        return;
    }
    if (!track) return;
    // GetAccessibleResource mutation for every other visited node of this shard.
    const uint64_t k = win;
    const uint64_t wk = k ? pack_key(key_score(k), key_idx(k), 0) : 0;
    const int wn = k ? key_idx(k) : -1;
    for (int n = threadIdx.x; n < nc.n; n += kBlock) {
        const uint64_t v = walk[n];
        if (!v || n + nc.base == wn) continue;
        if (k && v < wk) continue;
        nc.idle_cpu[n] += nc.bf_cpu[n]; nc.idle_mem[n] += nc.bf_mem[n]; nc.idle_gpu[n] += nc.bf_gpu[n];
    }
}

// Sweep of task task_i over this shard's nodes -> max key in ctrl->slot.
// commit_here: the last block commits (one GPU); otherwise the slot is
// reduced across shards first and k_commit_task commits.
// (bx, nbx: this block's index among the session's nbx blocks — blockIdx.x /
// gridDim.x, or one session's blocks of a multi-session grid)
__device__ __forceinline__ void sweep_body(const Conf& cf, const NodeCols& nc, const DevTables& t, PopCtrl* ctrl,
                                           int task_i, uint64_t* walk, int commit_here, uint64_t* dbg, int bx,
                                           int nbx, const int64_t* ipa_pre = nullptr) {
    __shared__ uint64_t red[kBlock / 64];
    __shared__ int last;
    __shared__ int32_t s_fit[4];
    if (ctrl->stop >= 0) return;  // the pop already stopped (uniform)
    if (threadIdx.x < 4) s_fit[threadIdx.x] = 0;
    const int cls = __builtin_amdgcn_readfirstlane(ctrl->cls[task_i]);
    const TaskClass c = t.classes[cls];
    const bool first_fit = ctrl->mode == 1;
    const bool track = !first_fit && ctrl->any_bf != 0;  // backfill never calls GetAccessibleResource
    const int64_t ilo = ctrl->ipa_lo[task_i], ihi = ctrl->ipa_hi[task_i];
    const int F = ctrl->fallback;
    uint64_t best = 0;
    int32_t fc[4] = {0, 0, 0, 0};  // this task's FitDelta histogram, should it find no node
    for (int n = bx * kBlock + threadIdx.x; n < nc.n; n += nbx * kBlock) {
        int32_t s = 0;
        bool passed = false;
        uint32_t fb = 0;
        const uint64_t k = first_fit ? eval_first_fit(cf, c, t, nc, n)
                                     : eval_node_aff(cf, c, t, nc, n, ilo, ihi, F, &s, &passed, &fb, ipa_pre);
        for (int b = 0; b < 4; ++b) fc[b] += (fb >> b) & 1;
        if (track) walk[n] = passed ? pack_key(s, n + nc.base, 0) : 0;
        if (dbg) {  // kbhip_set_option("debug_keys")
            dbg[(int64_t)task_i * (2 * nc.npad + 4) + n] = k;
            dbg[(int64_t)task_i * (2 * nc.npad + 4) + nc.npad + n] = (uint64_t)(c.ipa_n ? ipa_count(c, t, nc, n, F) : 0);
        }
        best = k > best ? k : best;
    }
    best = wave_max_u64(best);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = best;
    if (track) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // walk[] stores drained before the release
    __syncthreads();  // s_fit zeroed
    for (int b = 0; b < 4; ++b)
        if (fc[b]) atomicAdd(&s_fit[b], fc[b]);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t b = red[0];
        for (int w = 1; w < kBlock / 64; ++w) b = red[w] > b ? red[w] : b;
        if (b) atomicMax((unsigned long long*)&ctrl->slot[task_i], (unsigned long long)b);
        for (int q = 0; q < 4; ++q)
            if (s_fit[q]) atomicAdd(&ctrl->fit[task_i][q], s_fit[q]);
        __threadfence();
        const unsigned prev = atomicAdd(&ctrl->arrive[task_i], 1u);
        last = prev == (unsigned)nbx - 1;
        __threadfence();
    }
    __syncthreads();
    if (!last) return;
    if (dbg && threadIdx.x == 0) {
        uint64_t* d = dbg + (int64_t)task_i * (2 * nc.npad + 4) + 2 * nc.npad;
        d[0] = (uint64_t)ilo; d[1] = (uint64_t)ihi; d[2] = (uint64_t)(int64_t)F;
        d[3] = __hip_atomic_load(&ctrl->slot[task_i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (!(commit_here & 1)) return;
    commit_task(nc, t, ctrl, task_i, c, first_fit, track, walk, (commit_here & 2) != 0);
}
__global__ __launch_bounds__(kBlock) void k_sweep_argmax(Conf cf, NodeCols nc, DevTables t, PopCtrl* ctrl,
                                                         int task_i, uint64_t* walk, int commit_here, uint64_t* dbg,
                                                         const int64_t* ipa_pre) {
    sweep_body(cf, nc, t, ctrl, task_i, walk, commit_here, dbg, blockIdx.x, gridDim.x, ipa_pre);
}

// The GetAccessibleResource mutation of task task_i's walk (node_info.go:209-211,
// SURVEY Appendix A.1) over the whole grid, after k_sweep_argmax committed it
// with the mutation deferred (one block looping over every node is a chain of
// N / kBlock dependent memory round trips).  Runs only if task_i was swept
// (n_done == task_i + 1) and its sweep tracked the walk (pad, set by commit_task).
__device__ __forceinline__ void visit_body(const NodeCols& nc, const PopCtrl* ctrl, int task_i, const uint64_t* walk,
                                           int bx, int nbx) {
    if (ctrl->n_done != task_i + 1 || !ctrl->pad) return;  // uniform
    const uint64_t k = ctrl->slot[task_i];
    const uint64_t wk = k ? pack_key(key_score(k), key_idx(k), 0) : 0;
    const int wn = k ? key_idx(k) : -1;
    for (int n = bx * kBlock + threadIdx.x; n < nc.n; n += nbx * kBlock) {
        const uint64_t v = walk[n];
        if (!v || n + nc.base == wn) continue;
        if (k && v < wk) continue;
        nc.idle_cpu[n] += nc.bf_cpu[n]; nc.idle_mem[n] += nc.bf_mem[n]; nc.idle_gpu[n] += nc.bf_gpu[n];
    }
}
__global__ __launch_bounds__(kBlock) void k_visit_mutate(NodeCols nc, const PopCtrl* ctrl, int task_i,
                                                         const uint64_t* walk) {
    visit_body(nc, ctrl, task_i, walk, blockIdx.x, gridDim.x);
}

// What-if sessions stepping together (StepBatcher, option rank_group): task
// k of the per-task chunks of up to kPopMulti sessions in one launch,
// blockIdx.y = session, each session's blocks sweeping its own node columns
// and committing into its own control block exactly as k_sweep_argmax does.
struct SweepDesc {
    Conf cf;
    NodeCols nc;
    DevTables t;
    PopCtrl* ctrl;
    uint64_t* walk;
    int task_i, mode, nb;
};
struct SweepDescs {
    SweepDesc d[kPopMulti];
};
static_assert(sizeof(SweepDescs) <= 4000, "multi-session sweep descriptors exceed the kernel argument space");
__global__ __launch_bounds__(kBlock) void k_sweep_argmax_multi(SweepDescs d) {
    const SweepDesc& q = d.d[blockIdx.y];
    if ((int)blockIdx.x >= q.nb) return;
    sweep_body(q.cf, q.nc, q.t, q.ctrl, q.task_i, q.walk, q.mode, nullptr, blockIdx.x, q.nb);
}
__global__ __launch_bounds__(kBlock) void k_visit_mutate_multi(SweepDescs d) {
    const SweepDesc& q = d.d[blockIdx.y];
    if ((int)blockIdx.x >= q.nb || (q.mode & 2) == 0) return;
    visit_body(q.nc, q.ctrl, q.task_i, q.walk, blockIdx.x, q.nb);
}

// Sharded sessions: the commit after the cross-shard max of ctrl->slot[task_i].
__global__ __launch_bounds__(kBlock) void k_commit_task(NodeCols nc, DevTables t, PopCtrl* ctrl, int task_i,
                                                        const uint64_t* walk) {
    if (ctrl->stop >= 0) return;
    const int cls = __builtin_amdgcn_readfirstlane(ctrl->cls[task_i]);
    const TaskClass c = t.classes[cls];
    const bool first_fit = ctrl->mode == 1;
    commit_task(nc, t, ctrl, task_i, c, first_fit, !first_fit && ctrl->any_bf != 0, walk);
}

#endif
// ---------------------------------------------------------------------------
// batched path
// PL: the placement compiled into this instantiation — 2 parallel levels,
// 6 sessions with Backfilled nodes (walk keys, sequential placement), 7
// pod-affinity classes (affinity predicates in the sweep, sequential
// placement with count-table slots), 3 the node-array shard's sweep only (no
// placement: the exchange follows) — so that a kernel's registers (and the
// occupancy of its sweep blocks) are those of one placement path: compiling
// several placements into one kernel raised it from 101 to 194 VGPRs and
// halved the sweep's occupancy.
// One session's batched pop in a multi-session launch (k_pop_batch_multi):
// the kernel arguments carry kPopMulti descriptors (4 KB kernarg limit).
struct PopDesc {
    Conf cf;
    NodeCols nc;
    DevTables t;
    PopArgs a;
    uint64_t* cand;
    uint32_t* arrive;
    void* out;
    int nb;
};
struct PopDescs {
    PopDesc d[kPopMulti];
};
static_assert(sizeof(PopDescs) <= 4000, "multi-session pop descriptors exceed the kernel argument space");

// Placement 7 with per-domain candidates (TaskClass::dd_space, session/session.h
// dedup_space): of the block's nodes of one domain of the space only the one
// with the largest key can win (keys are unique: they carry the node index).
// Every block adds its domain maxima to the session's dd_max table, from which
// the final merger takes the best node of every domain (dedup_final), and
// sends only its nodes without the topology key through the merge tree.  So
// the pop's 64 candidates reach across up to 64 domains instead of stopping at
// the first few domains' best nodes.
template <typename KT, int R>
__device__ __forceinline__ void dedup_domains(const NodeCols& nc, const DevTables& t, int space, int ndom, int bid,
                                              KT (&keys)[R]) {
    __shared__ KT dmax[kDedupMax];
    for (int i = threadIdx.x; i < ndom; i += kPopThreads) dmax[i] = 0;
    __syncthreads();
    int d[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int n = (bid * R + r) * kPopThreads + threadIdx.x;
        d[r] = (keys[r] != 0 && n < nc.n) ? dom_of(nc, space, n) : -1;
        if (d[r] >= 0) {
            if constexpr (sizeof(KT) == 8) atomicMax((unsigned long long*)&dmax[d[r]], (unsigned long long)keys[r]);
            else atomicMax((unsigned int*)&dmax[d[r]], (unsigned int)keys[r]);
        }
    }
    __syncthreads();
    // Every node with the topology key leaves the block's list: dd_max holds the
    // exact best key of each domain over all blocks, so the merge tree carries
    // only nodes without the key and yields their exact top 64 (a keyed node
    // kept here could push keyless ones out of a merged list and the final
    // merger would then miss them).
#pragma unroll
    for (int r = 0; r < R; ++r)
        if (d[r] >= 0) keys[r] = 0;
    for (int i = threadIdx.x; i < ndom; i += kPopThreads) {  // (drained before the block arrives)
        const KT v = dmax[i];
        if (v) atomicMax((unsigned long long*)&t.dd_max[i], (unsigned long long)v);
    }
}

// The final merger of a placement-7 pop with per-domain candidates (wave 0):
// the merged list is the exact top 64 of the nodes without the topology key
// (dedup_domains left the others out); every domain contributes its best node
// from dd_max (all blocks added theirs before they arrived), which is reset
// for the next launch.  The top 64 of those: at most one node per domain.
template <typename KT>
__device__ __forceinline__ KT dedup_final(const NodeCols& nc, const DevTables& t, const TaskClass& c, const PopArgs& a,
                                          KT k) {
    const int lane = threadIdx.x & 63;
    const int nd = k ? key_node(k, a) : -1;
    const bool keep = nd >= 0 && dom_g(nc, c.dd_space, nd) < 0;
    KT acc = wave_sort_desc(keep ? k : (KT)0);
    for (int j0 = 0; j0 < c.dd_ndom; j0 += 64) {
        const int j = j0 + lane;
        uint64_t v = 0;
        if (j < c.dd_ndom) {
            v = ld_sc1(&t.dd_max[j]);
            if (v) st_sc1(&t.dd_max[j], (uint64_t)0);
        }
        acc = wave_merge_desc(acc, wave_sort_desc((KT)v));
    }
    return acc;
}

// The batched pop's body: block `bid` of `nb_` (k_pop_batch: the grid's own;
// k_pop_batch_multi: one session's blocks within a multi-session grid).
template <int R, typename KT, int PL>
__device__ __forceinline__ void pop_batch_body(const Conf& cf, const NodeCols& nc, const DevTables& t, const PopArgs& a,
                                               uint64_t* cand64, uint32_t* arrive, PopOut* out, ShardMsg* smsg,
                                               const MboxArgs& mb,
                                               const int bid, const int nb_) {
    __shared__ KT wlk[kPopThreads / 64][64];  // sweep / merge lists in the key type
    __shared__ uint64_t wl64[sizeof(KT) == 8 ? 1 : kPopThreads / 64][64];
    uint64_t (*wl)[64] = nullptr;             // placement lists (64-bit keys / entries)
    if constexpr (sizeof(KT) == 8) wl = (uint64_t (*)[64])wlk;
    else wl = wl64;
    KT* cand = (KT*)cand64;
    __shared__ int role;
    __shared__ uint32_t s_fitb[4];
    __shared__ int32_t s_fitin[4];
    uint32_t* fitc = fit_counters(arrive, a.fit_set);
    fit_zero_other(arrive, a.fit_set);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    STAMP(bid * 4 + 0);
    const TaskClass c = t.classes[a.cls];
    if (threadIdx.x < 4) s_fitb[threadIdx.x] = 0;
    // 1. evaluate R nodes per lane, wave top-64, block top-64
    KT best = 0;
    uint32_t fbs[R];
    KT keys[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int n = (bid * R + r) * kPopThreads + threadIdx.x;
        KT k = 0;
        fbs[r] = 0;
        if (n < nc.n) {
            int32_t s;
            bool passed;
            if constexpr (PL == 6) k = sweep_key<KT>(eval_node_walk(cf, c, t, nc, n, &fbs[r]), a);
            else if constexpr (PL == 7) k = sweep_key<KT>(eval_node_aff(cf, c, t, nc, n, 0, 0, -1, &s, &passed, &fbs[r]), a);
            else k = sweep_key<KT>(eval_node(cf, c, t, nc, n, &s, &passed, &fbs[r]), a);
        }
        keys[r] = k;
    }
    if constexpr (PL == 7) {
        if (c.dd_space >= 0) dedup_domains<KT, R>(nc, t, c.dd_space, c.dd_ndom, bid, keys);  // uniform: the pop's class
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const KT k = wave_sort_desc(keys[r]);
        best = r == 0 ? k : wave_merge_desc(best, k);
    }
    wlk[wave][lane] = best;
    __syncthreads();
#pragma unroll
    for (int r = 0; r < R; ++r) fit_block_add(s_fitb, fbs[r]);
    STAMP(bid * 4 + 1);
    block_tree_merge(wlk, wave, lane);
    const int nb = nb_;
    const int g = bid % kGroups;
    const int g_count = (nb - g + kGroups - 1) / kGroups;   // blocks in my group
    const int n_groups = nb < kGroups ? nb : kGroups;
    KT* gcand = cand + (int64_t)nb * 64;                     // group lists after the block lists
    if (wave == 0) {
        if (lane < 4 && s_fitb[lane])
            __hip_atomic_fetch_add(&fitc[g * kCtrStride + lane], s_fitb[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        put_list(cand + (int64_t)bid * 64, wlk[0][lane]);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if constexpr (PL == 7) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave's dd_max atomics
    __syncthreads();
    STAMP(bid * 4 + 2);
    if (threadIdx.x == 0) role = atomicAdd(&arrive[g * kCtrStride], 1u) == (unsigned)(g_count - 1);
    __syncthreads();
    if (!role) return;
    // 2a. last block of group g: merge the group's block lists (strided over
    // waves; each wave issues its lists' loads together, then merges)
    {
        KT acc = 0;
        constexpr int kPf = 4;
        for (int i0 = wave; i0 < g_count; i0 += kPf * (kPopThreads / 64)) {
            KT v[kPf];
#pragma unroll
            for (int q = 0; q < kPf; ++q) {
                const int i = i0 + q * (kPopThreads / 64);
                v[q] = i < g_count ? get_list(cand + (int64_t)(g + i * kGroups) * 64) : (KT)0;
            }
#pragma unroll
            for (int q = 0; q < kPf; ++q) acc = wave_merge_desc(acc, v[q]);
        }
        wlk[wave][lane] = acc;
        __syncthreads();
        block_tree_merge(wlk, wave, lane);
        if (wave == 0) {
            put_list(gcand + (int64_t)g * 64, wlk[0][lane]);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
        if (threadIdx.x == 0) role = atomicAdd(&arrive[kGroups * kCtrStride], 1u) == (unsigned)(n_groups - 1);
        __syncthreads();
        if (!role) return;
    }
    STAMP(nb_ * 4 + 4);
    // 2b. last group merger: merge the group lists; reset the counters for the next launch
    {
        KT acc = 0;
        for (int gi = wave; gi < n_groups; gi += kPopThreads / 64) acc = wave_merge_desc(acc, get_list(gcand + (int64_t)gi * 64));
        wlk[wave][lane] = acc;
    }
    __syncthreads();
    block_tree_merge(wlk, wave, lane);
    STAMP(nb_ * 4 + 0);
    if constexpr (PL == 7) {
        if (c.dd_space >= 0) {  // (uniform)
            if (wave == 0) wlk[0][lane] = dedup_final<KT>(nc, t, c, a, wlk[0][lane]);
            __syncthreads();
        }
    }
    if constexpr (sizeof(KT) != 8) {  // placement works on 64-bit keys
        const uint64_t k64 = key64_of(wlk[0][lane], a);
        __syncthreads();
        if (wave == 0) wl[0][lane] = k64;
        __syncthreads();
    }
    if (wave == 0 && lane <= kGroups)
        __hip_atomic_store(&arrive[lane * kCtrStride], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // the sweep's FitDelta counts (every block added before it arrived), left in flight
    const uint32_t fit_raw = wave == 0 ? fit_load(fitc, n_groups) : 0u;
    if (wave == 0 && lane < 4) s_fitin[lane] = 0;  // + the counts of nodes the sweep left out
    __syncthreads();
    if constexpr (PL == 3) {  // node-array shard: emit the shard's list, the placement runs after the exchange
        shard_emit(cf, nc, t, c, wl[0][lane], fit_raw, smsg, mb);
        return;
    } else if constexpr (PL == 6) {  // Backfilled nodes in the session
        if (wave != 0) return;
        STAMP(nb_ * 4 + 1);
        place_bf(cf, nc, t, c, a, out, wl[0][lane]);
        STAMP(nb_ * 4 + 3);
        return;
    } else if constexpr (PL == 7) {  // pod-affinity class (aff_batchable)
        if (wave != 0) return;
        STAMP(nb_ * 4 + 1);
        place_aff(cf, nc, t, c, a, out, wl[0][lane]);
        STAMP(nb_ * 4 + 2);
        STAMP(nb_ * 4 + 3);
        return;
    } else {  // PL == 2: parallel levels, every wave takes part
        static_assert(PL == 2, "batched placements: 2, 3, 6, 7");
        STAMP(nb_ * 4 + 1);
        if (a.ent32) place_parallel<uint32_t>(cf, nc, t, c, a, out, wl, nullptr, 0, (const RowCache*)nullptr, s_fitin, fit_raw);
        else place_parallel<uint64_t>(cf, nc, t, c, a, out, wl, nullptr, 0, (const RowCache*)nullptr, s_fitin, fit_raw);
    }
}

template <int R, typename KT, int PL>
__global__ __launch_bounds__(kPopThreads) void k_pop_batch(Conf cf, NodeCols nc, DevTables t, PopArgs a,
                                                           uint64_t* cand64, uint32_t* arrive, PopOut* out,
                                                           ShardMsg* smsg, MboxArgs mb) {
    pop_batch_body<R, KT, PL>(cf, nc, t, a, cand64, arrive, out, smsg, mb, blockIdx.x, gridDim.x);
}

// What-if sessions batched per launch: one launch
// serves the batched pops of up to kPopMulti concurrent sessions, session
// blockIdx.y with its own node columns, tables, candidates, counters and
// result slot (descriptors in the kernel arguments).
template <int R, typename KT, int PL>
__global__ __launch_bounds__(kPopThreads) void k_pop_batch_multi(PopDescs d) {
    const PopDesc& q = d.d[blockIdx.y];
    if ((int)blockIdx.x >= q.nb) return;
    const MboxArgs none{};
    pop_batch_body<R, KT, PL>(q.cf, q.nc, q.t, q.a, q.cand, q.arrive, (PopOut*)q.out, nullptr, none, blockIdx.x, q.nb);
}

// ---------------------------------------------------------------------------
// Overlapped batched pops (option "overlap").  Pop e runs while pop e-1
// (launched on the other stream) may still be placing.  Every row a
// placement writes belongs to one of its 64 candidates, which pop e-1
// publishes (PopLink::touched) as soon as its candidate list is final —
// normally long before pop e's blocks finish evaluating.  Pop e's sweep ranks
// every other node exactly (their rows are final) and leaves pop e-1's
// candidates out; its final merger waits for pop e-1's write-back (done),
// evaluates those candidates on their final rows and merges them in: the
// top-64 of all nodes, as the non-overlapped kernel sees it.
// Hand-offs: candidates as self-tagged 8-byte granules {seq, node} (one sc1
// store each, no flag); rows as sc1 stores drained before the sc1 done flag,
// read with sc1 loads (MI355X_MICROARCH.md valid forms, R2 and row 1).
// ---------------------------------------------------------------------------

constexpr long kLinkSpin = 1L << 21;  // poll bound (~1 s): a broken chain ends the pop with an error

// Relaxed sc1 poll of a sequence word until it reaches `want`, with two
// loads in flight (a store that lands just after one load was issued is
// seen by the next, about half a round trip later).  false: timed out.
__device__ __forceinline__ bool poll_done(const uint32_t* p, uint32_t want) {
    uint32_t a = (uint32_t)__builtin_amdgcn_readfirstlane((int)ld_sc1(p));
    uint32_t b = (uint32_t)__builtin_amdgcn_readfirstlane((int)ld_sc1(p));
    for (long spin = 0; spin < kLinkSpin; ++spin) {
        if ((int32_t)(a - want) >= 0) return true;
        a = (uint32_t)__builtin_amdgcn_readfirstlane((int)ld_sc1(p));
        if ((int32_t)(b - want) >= 0) return true;
        b = (uint32_t)__builtin_amdgcn_readfirstlane((int)ld_sc1(p));
    }
    return false;
}

// The pop's task class comes by value in the kernel arguments (cl = the
// session's classes[a.cls]): the sweep's row loads wait for no dependent load
// of the class record.
template <int R, typename KT>
__global__ __launch_bounds__(kPopThreads) void k_pop_batch_ov(Conf cf, NodeCols nc, DevTables t, PopArgs a,
                                                              TaskClass cl, uint64_t* cand64, uint32_t* arrive,
                                                              PopOut* out, PopLink* link, uint32_t seq, int dep,
                                                              uint32_t msg_from) {
    __shared__ KT wlk[kPopThreads / 64][64];               // sweep / merge lists in the key type
    __shared__ uint64_t wl[kPopThreads / 64][64];          // placement lists (64-bit keys / entries)
    __shared__ uint32_t s_skip[R * kPopThreads / 32];      // this block's nodes among pop seq-1's (and seq-2's) candidates
    __shared__ int role, s_ok, s_bad, s_list_ready, s_pdone[2], s_prow[2];
    __shared__ uint32_t s_fitb[4];
    __shared__ int32_t s_fitin[4];
    uint32_t* fitc = fit_counters(arrive, a.fit_set);
    fit_zero_other(arrive, a.fit_set);
    KT* cand = (KT*)cand64;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (threadIdx.x == 0) { s_bad = 0; s_list_ready = 0; s_pdone[0] = s_pdone[1] = 0; s_prow[0] = s_prow[1] = 0; }  // (before the first barrier)
    __shared__ RowCache rc;  // the final merger's (block 0 in the tagged path)
    if (blockIdx.x == 0)
        for (int h = threadIdx.x; h < kRcHash; h += kPopThreads) rc.hkey[h] = -1;
    // one node per lane, 32-bit keys: the blocks' and groups' lists travel as
    // self-tagged granules to fixed mergers (else: counters, last arriver merges)
    constexpr bool kTagged = R == 1 && sizeof(KT) == 4;
    STAMP(blockIdx.x * 4 + 0);
    if (blockIdx.x == 0 && threadIdx.x == 0) TL(seq, 0);
    if (threadIdx.x == 0) TLB(seq, 0);
    const TaskClass& c = cl;
    const int base = blockIdx.x * R * kPopThreads;
    // pop seq-1 (and with dep 2 pop seq-2) may still be writing rows: their
    // candidates, in flight while the rows below load
    uint64_t tv = 0, tv2 = 0;
    if (wave == 0 && seq > 1) tv = ld_sc1(&link->touched[(seq - 1) % kLinkSlots][lane]);
    const bool dep2 = dep > 1 && seq > 2;
    if (wave == 0 && dep2) tv2 = ld_sc1(&link->touched[(seq - 2) % kLinkSlots][lane]);
    // wave 0: wait for the candidates of pop `want`, mark this block's among them (0: timed out)
    auto wait_touched = [&](uint64_t& v, uint32_t want, int* node) -> bool {
        // two re-reads of every granule in flight: a granule that lands just
        // after one was issued is seen by the next, half a round trip later
        const uint64_t* src = &link->touched[want % kLinkSlots][lane];
        uint64_t w = ld_sc1(src);
        long spin = 0;
        for (;;) {
            if (__ballot((uint32_t)(v >> 32) != want) == 0) break;
            v = ld_sc1(src);
            if (__ballot((uint32_t)(w >> 32) != want) == 0) { v = w; break; }
            w = ld_sc1(src);
            if (++spin >= kLinkSpin) { *node = -1; return false; }
        }
        *node = (int)(uint32_t)v;
        if (*node >= base && *node < base + R * kPopThreads)
            atomicOr(&s_skip[(*node - base) >> 5], 1u << ((*node - base) & 31));
        return true;
    };
    for (int i = threadIdx.x; i < R * kPopThreads / 32; i += kPopThreads) s_skip[i] = 0;
    if (threadIdx.x < 4) s_fitb[threadIdx.x] = 0;
    // 1. evaluate R nodes per lane, then leave pop seq-1's candidates out
    KT keys[R];
    uint32_t fbs[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int n = base + r * kPopThreads + threadIdx.x;
        keys[r] = 0;
        fbs[r] = 0;
        if (n < nc.n) {
            int32_t s;
            bool passed;
            keys[r] = sweep_key<KT>(eval_node(cf, c, t, nc, n, &s, &passed, &fbs[r]), a);
        }
    }
    int tn = -1, tn2 = -1;  // wave 0: candidate `lane` of pop seq-1 / seq-2 (-1: none)
    bool ok2 = true;
    __shared__ int32_t s_tn[64], s_tn2[64];  // pop seq-1's / seq-2's candidates (the final merger's other waves)
    if (dep2) {  // pop seq-2's candidates (published about one period before this kernel began) leave the sweep
        __syncthreads();  // s_skip zeroed
        if (wave == 0) {
            ok2 = wait_touched(tv2, seq - 2, &tn2);
            s_tn2[lane] = tn2;
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int o = r * kPopThreads + threadIdx.x;
            if ((s_skip[o >> 5] >> (o & 31)) & 1u) { keys[r] = 0; fbs[r] = 0; }  // counted by the patch
        }
    }
    if constexpr (R == 1) {
        // The block's top 128 over all its nodes, sorted and merged before pop
        // seq-1's candidates are known (they arrive at the end of its patch);
        // then those of them in this block (at most 64) leave the list and
        // the counts, and the first 64 left are the block's exact top 64.
        __shared__ KT wlk2[kPopThreads / 64][64];  // ranks 64..127 of the block merge
        __shared__ uint8_t s_fb[kPopThreads];      // FitDelta bits per node (0: left out already)
        s_fb[threadIdx.x] = (uint8_t)fbs[0];
        fit_block_add(s_fitb, fbs[0]);
        wlk[wave][lane] = wave_sort_desc(keys[0]);
        __syncthreads();  // s_skip, s_fitb zeroed; wave lists and s_fb written
        STAMP(blockIdx.x * 4 + 1);
        block_tree_merge128(wlk, wlk2, wave, lane);
        if (threadIdx.x == 0) TLB(seq, 1);
        if (wave == 0) {
            bool ok = ok2;
            if (seq > 1 && !wait_touched(tv, seq - 1, &tn)) ok = false;
            s_tn[lane] = tn;
            if (lane == 0) { s_ok = ok; TLB(seq, 2); }
            const bool mine = tn >= base && tn < base + kPopThreads;  // rows in flight: counted by the patch
            const uint32_t fb = mine ? s_fb[tn - base] : 0u;  // 0 for a node of pop seq-2's too
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int cnt = __popcll(__ballot((fb >> b) & 1u));
                if (lane == b && cnt) atomicSub(&s_fitb[b], (uint32_t)cnt);  // group mergers' waves add concurrently
            }
            const KT k0 = wlk[0][lane], k1 = wlk2[0][lane];
            __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's s_skip bits and list reads
            __builtin_amdgcn_wave_barrier();
            auto kept = [&](KT k) {
                if (!k) return false;
                const int o = key_node(k, a) - base;
                return ((s_skip[o >> 5] >> (o & 31)) & 1u) == 0;
            };
            const bool c0 = kept(k0), c1 = kept(k1);
            const uint64_t m0 = __ballot(c0), m1 = __ballot(c1);
            const int q0 = __builtin_amdgcn_mbcnt_hi((uint32_t)(m0 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m0, 0));
            const int q1 = __popcll(m0) +
                           __builtin_amdgcn_mbcnt_hi((uint32_t)(m1 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m1, 0));
            wlk[0][lane] = 0;  // LDS operations of one wave complete in order
            if (c0) wlk[0][q0] = k0;  // q0 < 64
            if (c1 && q1 < 64) wlk[0][q1] = k1;
            __builtin_amdgcn_s_waitcnt(0xc07f);
            __builtin_amdgcn_wave_barrier();
        }
    } else {
        __syncthreads();  // s_skip zeroed
        if (wave == 0) {
            bool ok = ok2;
            if (seq > 1 && !wait_touched(tv, seq - 1, &tn)) ok = false;
            s_tn[lane] = tn;
            if (lane == 0) { s_ok = ok; TLB(seq, 2); }
        }
        __syncthreads();
        KT best = 0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int o = r * kPopThreads + threadIdx.x;
            const bool skip = (s_skip[o >> 5] >> (o & 31)) & 1u;  // rows in flight: counted by the patch
            fit_block_add(s_fitb, skip ? 0u : fbs[r]);
            const KT k = wave_sort_desc(skip ? (KT)0 : keys[r]);
            best = r == 0 ? k : wave_merge_desc(best, k);
        }
        wlk[wave][lane] = best;
        __syncthreads();
        STAMP(blockIdx.x * 4 + 1);
        block_tree_merge(wlk, wave, lane);
    }
    const int nb = gridDim.x;
    const int g = blockIdx.x % kGroups;
    const int g_count = (nb - g + kGroups - 1) / kGroups;
    const int n_groups = nb < kGroups ? nb : kGroups;
    uint32_t fit_raw = 0;  // wave 0 of the final merger: the sweep's FitDelta counts (fit_sum layout)
    if constexpr (kTagged) {
        // Merge tree by self-tagged granules {seq, key} (MI355X_MICROARCH.md
        // handoff-1to1: no drain, no counter): block b of group g = b % 8
        // stores its list and counts; fixed mergers — block g merges group g,
        // block 0 then merges the groups — poll them.
        uint64_t* G = cand64;
        if ((int)blockIdx.x >= n_groups) {
            if (wave == 0) {
                uint64_t* dst = G + (int64_t)blockIdx.x * kCandStride;
                st_sc1(&dst[lane], ((uint64_t)seq << 32) | (uint32_t)wlk[0][lane]);
                if (lane < 4) st_sc1(&dst[64 + lane], ((uint64_t)seq << 32) | s_fitb[lane]);
            }
            if (threadIdx.x == 0) TLB(seq, 3);
            return;
        }
        // poll the granules of `cnt` lists at src[0], src[stride], ...; merge
        // their keys into acc and add their counts to s_fitb (0: timed out)
        auto gather = [&](const uint64_t* src, int cnt, int64_t stride, KT& acc) -> bool {
            constexpr int kQ = 8;  // all of a wave's lists in one round trip (group: <= 4 per wave; final: 7)
            for (int q0 = 0; q0 < cnt; q0 += kQ) {
                uint64_t v[kQ], f[kQ];
#pragma unroll
                for (int q = 0; q < kQ; ++q) {
                    const uint64_t* p = src + (int64_t)(q0 + q) * stride;
                    const bool in = q0 + q < cnt;
                    v[q] = in ? ld_sc1(&p[lane]) : ((uint64_t)seq << 32);
                    f[q] = (in && lane < 4) ? ld_sc1(&p[64 + lane]) : ((uint64_t)seq << 32);
                }
                long spin = 0;
                for (;;) {
                    bool miss = false;
#pragma unroll
                    for (int q = 0; q < kQ; ++q) {
                        if (__ballot((uint32_t)(v[q] >> 32) != seq || (uint32_t)(f[q] >> 32) != seq) == 0) continue;
                        miss = true;
                        const uint64_t* p = src + (int64_t)(q0 + q) * stride;
                        v[q] = ld_sc1(&p[lane]);
                        if (lane < 4) f[q] = ld_sc1(&p[64 + lane]);
                    }
                    if (!miss) break;
                    if (++spin >= kLinkSpin) return false;
                    __builtin_amdgcn_s_sleep(1);
                }
#pragma unroll
                for (int q = 0; q < kQ; ++q) {
                    acc = wave_merge_desc(acc, (KT)(uint32_t)v[q]);
                    if (lane < 4 && (uint32_t)f[q]) atomicAdd(&s_fitb[lane], (uint32_t)f[q]);
                }
            }
            return true;
        };
        // 2a. group g: this block's list (wave 0) and the lists of blocks g + 8i, i >= 1, over the waves
        KT acc = wave == 0 ? wlk[0][lane] : (KT)0;
        {
            const int per = (g_count - 1 + kPopThreads / 64 - 1) / (kPopThreads / 64);  // lists per wave
            const int i0 = 1 + wave * per;
            const int cnt = i0 < g_count ? (g_count - i0 < per ? g_count - i0 : per) : 0;
            if (cnt > 0 && !gather(G + (int64_t)(g + i0 * kGroups) * kCandStride, cnt, (int64_t)kGroups * kCandStride, acc))
                s_bad = 1;
        }
        __syncthreads();  // wlk[0] read by wave 0 above; every wave's counts added
        wlk[wave][lane] = acc;
        __syncthreads();
        block_tree_merge(wlk, wave, lane);
        if (g != 0) {  // publish group g (a timed-out merger publishes nothing: the final merger times out too)
            if (wave == 0 && !s_bad) {
                uint64_t* dst = G + (int64_t)(nb + g) * kCandStride;
                st_sc1(&dst[lane], ((uint64_t)seq << 32) | (uint32_t)wlk[0][lane]);
                if (lane < 4) st_sc1(&dst[64 + lane], ((uint64_t)seq << 32) | s_fitb[lane]);
            }
            if (threadIdx.x == 0) TLB(seq, 4);
            return;
        }
        // 2b. block 0, the final merger.  Wave 0 alone merges group 0's list
        // with groups 1 .. n_groups-1 (no block-wide barrier: waves 6 / 7
        // are meanwhile patching with the previous pops' candidates, §3) and
        // flags the final list in LDS for wave 1.
        if (wave == 0) {
            KT fin = wlk[0][lane];
            if (n_groups > 1 && !gather(G + (int64_t)(nb + 1) * kCandStride, n_groups - 1, kCandStride, fin))
                s_bad = 1;
            wlk[0][lane] = fin;
            fit_raw = lane < 4 ? s_fitb[lane] : 0u;  // every block's counts: this wave added the groups'
            __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the list is in LDS before the flag
            if (lane == 0) __hip_atomic_store(&s_list_ready, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            STAMP(gridDim.x * 4 + 0);
            if (lane == 0) TL(seq, 4);
        }
    } else {
    KT* gcand = cand + (int64_t)nb * 64;
    if (wave == 0) {
        if (lane < 4 && s_fitb[lane])
            __hip_atomic_fetch_add(&fitc[g * kCtrStride + lane], s_fitb[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        put_list(cand + (int64_t)blockIdx.x * 64, wlk[0][lane]);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    STAMP(blockIdx.x * 4 + 2);
    if (threadIdx.x == 0) { TLB(seq, 3); role = atomicAdd(&arrive[g * kCtrStride], 1u) == (unsigned)(g_count - 1); }
    __syncthreads();
    if (!role) return;
    // 2a. last block of group g merges the group's lists
    {
        KT acc = 0;
        constexpr int kPf = 4;
        for (int i0 = wave; i0 < g_count; i0 += kPf * (kPopThreads / 64)) {
            KT v[kPf];
#pragma unroll
            for (int q = 0; q < kPf; ++q) {
                const int i = i0 + q * (kPopThreads / 64);
                v[q] = i < g_count ? get_list(cand + (int64_t)(g + i * kGroups) * 64) : (KT)0;
            }
#pragma unroll
            for (int q = 0; q < kPf; ++q) acc = wave_merge_desc(acc, v[q]);
        }
        wlk[wave][lane] = acc;
        __syncthreads();
        block_tree_merge(wlk, wave, lane);
        if (wave == 0) {
            put_list(gcand + (int64_t)g * 64, wlk[0][lane]);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
        if (threadIdx.x == 0) { TLB(seq, 4); role = atomicAdd(&arrive[kGroups * kCtrStride], 1u) == (unsigned)(n_groups - 1); }
        __syncthreads();
        if (!role) return;
    }
    // 2b. last group merger: the top-64 of every node but the previous pop's candidates
    STAMP(gridDim.x * 4 + 4);
    {
        KT acc = 0;
        for (int gi = wave; gi < n_groups; gi += kPopThreads / 64) acc = wave_merge_desc(acc, get_list(gcand + (int64_t)gi * 64));
        wlk[wave][lane] = acc;
        for (int h = threadIdx.x; h < kRcHash; h += kPopThreads) rc.hkey[h] = -1;  // before either wave inserts
    }
    __syncthreads();
    block_tree_merge(wlk, wave, lane);
    STAMP(gridDim.x * 4 + 0);
    if (threadIdx.x == 0) TL(seq, 4);
    if (wave == 0 && lane <= kGroups)
        __hip_atomic_store(&arrive[lane * kCtrStride], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // the sweep's FitDelta counts (every block added before it arrived), left in flight
    if (wave == 0) fit_raw = fit_load(fitc, n_groups);
    }
    if (wave == 0 && lane < 4) s_fitin[lane] = 0;  // + the counts of nodes the sweep left out
    // 3. Waves of the final merger, side by side:
    //   wave 1: the rows of the final list's nodes (final: no pop in flight
    //     touches them) into the row cache (tagged: once wave 0 flags the list);
    //   wave kP1 (tagged 6, else 0): pop seq-1's candidates — static parts,
    //     then pop seq-1's done (relaxed sc1 poll), then their final rows
    //     (sc1 loads) into the cache and their keys into s_e0;
    //   wave kP2 (tagged 7, else 2; depth 2): the same for pop seq-2's
    //     candidates not among seq-1's (final too once seq-1's done is seen:
    //     seq-1 waited for seq-2's).
    // Then wave 0 merges the keys into the list and publishes the candidates.
    constexpr int kP1 = kTagged ? 6 : 0, kP2 = kTagged ? 7 : 2;
    __shared__ KT s_e[2][64];
    __shared__ uint8_t s_fbp[2][64];
    __shared__ uint8_t s_pst[2][64];  // tagged: 1 = the candidate's row is in the cache, 2 = its static predicates pass
    auto patch = [&](int q, int node, bool skip) {
        bool okp = true;
        bool pst = false;
        int32_t pna = 0;
        const bool use = node >= 0 && !skip;
        if (use) {
            pst = static_pred(cf, c, t, nc, node);
            pna = (pst && cf.score_mult) ? na_weight(c, t, nc, node) : 0;
        }
        // the rows of pop `src`'s candidates as it left them: its row message
        // (written after its write-back drained), self-tagged
        const uint32_t src = seq - 1 - q;
        const uint64_t (*m)[64] = link->rows[src % kLinkSlots];
        uint32_t w[kRowWords];
        const bool via_msg = src >= msg_from;  // else: device work outside the chain ran since (the node columns)
        if (!via_msg) {
            okp = poll_done(&link->done, seq - 1);
        } else {
            // poll the message itself: every read brings the data with its
            // tags, so the round trip that sees them complete is the last
            long spin = 0;
            for (;;) {
                bool bad = false;
#pragma unroll
                for (int f = 0; f < kRowWords; ++f) {
                    const uint64_t x = ld_sc1(&m[f][lane]);
                    bad |= (uint32_t)(x >> 32) != src;
                    w[f] = (uint32_t)x;
                }
                if (__ballot(bad) == 0) break;
                if (++spin >= kLinkSpin) { okp = false; break; }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        if (q == 0 && lane == 0) TL(seq, 5);
        KT e = 0;
        uint32_t fb = 0;
        const int slot = 64 * (q + 1) + lane;
        Row r{};
        uint64_t pw[4] = {0, 0, 0, 0};  // (port words: the node columns, written before the message)
        if (okp && use) {
            r = via_msg ? words_row(w) : load_row_sc1(nc, node);
            if (c.has_ports)
                for (int w = 0; w < 4; ++w) if (w < port_win(c, nc)) pw[w] = load_port_t<true>(nc, c.pw_lo + w, node);
            rc.row[slot] = r;
            for (int w = 0; w < 4; ++w) rc.pw[slot][w] = pw[w];
            rc.na[slot] = pna;
            rc_insert(&rc, node, slot);
        }
        if constexpr (kTagged) {  // the rows are in the cache: a helper wave takes the depth-1 scores
            s_pst[q][lane] = (okp && use) ? (uint8_t)(1 | (pst ? 2 : 0)) : (uint8_t)0;
            __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
            if (lane == 0) __hip_atomic_store(&s_prow[q], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        if (okp && use) {
            int32_t sc;
            bool passed;
            const uint64_t k0 = dyn_key(cf, c, t, nc, r, pw, node, pst, pna, &sc, &passed);
            e = sweep_key<KT>(k0, a);
            fb = fit_bits(c, r, passed);
            if constexpr (!kTagged) rc.s1[slot] = k0 ? depth1_score(cf, nc, t, c, r, pw, node, pna, k0) : INT32_MIN;
        }
        if (q == 0) TL(seq, 13);
        s_e[q][lane] = e;
        s_fbp[q][lane] = (uint8_t)fb;
        if (!okp && lane == 0) s_bad = 1;
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the keys and the cache are in LDS before the flag
        if (lane == 0) __hip_atomic_store(&s_pdone[q], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    if (wave == 1) {
        if constexpr (kTagged) {
            while (__hip_atomic_load(&s_list_ready, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0)
                __builtin_amdgcn_s_sleep(1);
        }
        const KT lk = wlk[0][lane];
        const int ln = lk ? key_node(lk, a) : -1;
        if (ln >= 0) {
            rc.row[lane] = load_row(nc, ln);
            for (int w = 0; w < 4; ++w) rc.pw[lane][w] = (c.has_ports && w < port_win(c, nc)) ? load_port_t<false>(nc, c.pw_lo + w, ln) : 0;
            rc.na[lane] = cf.score_mult ? na_weight(c, t, nc, ln) : 0;
            rc.s1[lane] = depth1_score(cf, nc, t, c, rc.row[lane], rc.pw[lane], ln, rc.na[lane], key64_of(lk, a));
            rc_insert(&rc, ln, lane);
        }
        if (lane == 0) TL(seq, 12);
    }
    if constexpr (kTagged) {
        // waves 3 / 5: the depth-1 scores of pop seq-1's / seq-2's candidates
        // (read by the placement only), off the path to the candidates'
        // publication, on SIMDs other than the patching waves' (wave w runs on
        // SIMD w % 4: 0 merges, 6 and 7 patch, 1 gathers rows)
        if (wave == 3 || (wave == 5 && dep2)) {
            const int q = wave == 3 ? 0 : 1;
            while (__hip_atomic_load(&s_prow[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0)
                __builtin_amdgcn_s_sleep(1);
            const uint32_t st = s_pst[q][lane];
            if (st & 1u) {
                const int slot = 64 * (q + 1) + lane;
                const int node = q == 0 ? s_tn[lane] : s_tn2[lane];
                const Row r = rc.row[slot];
                uint64_t pw[4];
                for (int w = 0; w < 4; ++w) pw[w] = rc.pw[slot][w];
                const int32_t pna = rc.na[slot];
                int32_t sc;
                bool passed;
                const uint64_t k0 = dyn_key(cf, c, t, nc, r, pw, node, (st & 2u) != 0, pna, &sc, &passed);
                rc.s1[slot] = k0 ? depth1_score(cf, nc, t, c, r, pw, node, pna, k0) : INT32_MIN;
            }
        }
    }
    if (wave == kP1) patch(0, s_tn[lane], false);
    if (wave == kP2 && dep2) {
        const int n2 = s_tn2[lane];
        bool dup = false;
        for (int i = 0; i < 64; ++i) dup = dup || s_tn[i] == n2;
        patch(1, n2, dup);
    }
    if (wave == 0) {  // the patch keys (LDS flags: the list rows are needed only by the placement)
        while ((kP1 != 0 && __hip_atomic_load(&s_pdone[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0) ||
               (dep2 && __hip_atomic_load(&s_pdone[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0))
            __builtin_amdgcn_s_sleep(1);
        const bool ok = s_ok && !s_bad;
        KT top = wave_merge_desc(wlk[0][lane], wave_sort_desc(s_e[0][lane]));  // all 64 lanes: cross-lane networks
        uint32_t fb_prev = s_fbp[0][lane];  // FitDelta bits of the candidates the sweep left out
        if (dep2) {
            top = wave_merge_desc(top, wave_sort_desc(s_e[1][lane]));
            fb_prev |= (uint32_t)s_fbp[1][lane] << 4;
        }
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const int cnt = __popcll(__ballot((fb_prev >> b) & 1u)) + __popcll(__ballot((fb_prev >> (b + 4)) & 1u));
            if (lane == b) s_fitin[b] += cnt;
        }
        // this pop's candidates, one self-tagged granule each
        const int tnode = (ok && top) ? key_node(top, a) : -1;
        st_sc1(&link->touched[seq % kLinkSlots][lane], ((uint64_t)seq << 32) | (uint32_t)tnode);
        if (lane == 0) TL(seq, 6);
        wl[0][lane] = ok ? key64_of(top, a) : 0;
        if (lane == 0) s_ok = ok;
    }
    __syncthreads();
    STAMP(gridDim.x * 4 + 1);
    if (threadIdx.x == 0) TL(seq, 11);
    if (s_ok) {
        uint64_t (*msg)[64] = link->rows[seq % kLinkSlots];
        if (a.ent32)
            place_parallel<uint32_t, true>(cf, nc, t, c, a, out, wl, &link->done, seq, &rc, s_fitin, fit_raw, 0,
                                           0x7fffffff, 0, msg);
        else
            place_parallel<uint64_t, true>(cf, nc, t, c, a, out, wl, &link->done, seq, &rc, s_fitin, fit_raw, 0,
                                           0x7fffffff, 0, msg);
    } else if (wave == 0 && lane == 0) {  // broken chain: keep the chain going, n_done = 0 tells the host
        st_sc1(&link->done, seq);
        __hip_atomic_store(&out->g[0], make_granule(a.epoch, 0, 0, 0, -1), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

#if KBHIP_PART <= 1
// ---------------------------------------------------------------------------
// launchers (host)
// ---------------------------------------------------------------------------
hipError_t launch_sweep_argmax(const Conf& cf, const NodeCols& nc, const DevTables& t, PopCtrl* ctrl, int task_i,
                               uint64_t* walk, hipStream_t st, bool commit_here, uint64_t* dbg, bool defer_visits,
                               const int64_t* ipa_pre) {
    int grid = (nc.n + kBlock - 1) / kBlock;
    if (grid > 2048) grid = 2048;
    if (grid < 1) grid = 1;
    const int mode = commit_here ? (defer_visits ? 3 : 1) : 0;
    hipLaunchKernelGGL(k_sweep_argmax, dim3(grid), dim3(kBlock), 0, st, cf, nc, t, ctrl, task_i, walk, mode, dbg,
                       ipa_pre);
    if (commit_here && defer_visits)
        hipLaunchKernelGGL(k_visit_mutate, dim3(grid), dim3(kBlock), 0, st, nc, (const PopCtrl*)ctrl, task_i,
                           (const uint64_t*)walk);
    return hipGetLastError();
}

// Task k of every request whose chunk has more than k tasks, kPopMulti
// sessions per launch (requests in order: each session's tasks run in order
// on the one stream).
hipError_t launch_sweep_multi(const SweepReq* reqs, int n, int k, hipStream_t st, int* launches) {
    SweepDescs d{};
    int cnt = 0, max_nb = 1, any_defer = 0;
    auto flush = [&]() {
        if (!cnt) return;
        hipLaunchKernelGGL(k_sweep_argmax_multi, dim3(max_nb, cnt), dim3(kBlock), 0, st, d);
        if (any_defer) hipLaunchKernelGGL(k_visit_mutate_multi, dim3(max_nb, cnt), dim3(kBlock), 0, st, d);
        ++*launches;
        d = SweepDescs{};
        cnt = 0;
        max_nb = 1;
        any_defer = 0;
    };
    for (int i = 0; i < n; ++i) {
        const SweepReq& r = reqs[i];
        if (k >= r.m) continue;
        int nb = (r.nc.n + kBlock - 1) / kBlock;
        nb = nb > 2048 ? 2048 : nb < 1 ? 1 : nb;
        d.d[cnt] = SweepDesc{r.cf, r.nc, r.t, r.ctrl, r.walk, k, r.defer ? 3 : 1, nb};
        max_nb = nb > max_nb ? nb : max_nb;
        any_defer |= r.defer;
        if (++cnt == kPopMulti) flush();
    }
    flush();
    return hipGetLastError();
}

// Retraction of a batched pop whose prediction failed (Allocator::speculate):
// the inverse node updates of its placements, in one lane (a node may appear
// several times).
struct UndoArgs {
    int32_t cls, n;
    int32_t node[kMaxChunk];
    int32_t kind[kMaxChunk];
};
// One lane per task, every update an atomic add: the inverse updates commute
// (a node may appear several times), so the pop's tasks are retracted side by
// side instead of as one lane's chain of dependent read-modify-writes.
template <typename T>
__device__ __forceinline__ void atomic_add_dev(T* p, T v) {
    __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__global__ __launch_bounds__(64) void k_undo_pop(NodeCols nc, DevTables t, UndoArgs u) {
    const int i = threadIdx.x;
    if (i >= u.n) return;
    const TaskClass c = t.classes[u.cls];
    const int g = u.node[i], kind = u.kind[i];
    const int n = g - nc.base;
    if (g >= 0 && n >= 0 && n < nc.n) {  // this shard's rows only: uncommit_node, atomically
        if (c.backfill) {
            atomic_add_dev(&nc.bf_cpu[n], -c.req_cpu); atomic_add_dev(&nc.bf_mem[n], -c.req_mem);
            atomic_add_dev(&nc.bf_gpu[n], -c.req_gpu);
        }
        if (kind == 1) {
            atomic_add_dev(&nc.idle_cpu[n], c.req_cpu); atomic_add_dev(&nc.idle_mem[n], c.req_mem);
            atomic_add_dev(&nc.idle_gpu[n], c.req_gpu);
        } else {
            atomic_add_dev(&nc.rel_cpu[n], c.req_cpu); atomic_add_dev(&nc.rel_mem[n], c.req_mem);
            atomic_add_dev(&nc.rel_gpu[n], c.req_gpu);
        }
        atomic_add_dev(&nc.pods[n], -1);
        atomic_add_dev(&nc.nzc[n], -c.nz_cpu);
        atomic_add_dev(&nc.nzm[n], -c.nz_mem);
        if (c.has_ports)
            for (int w = 0; w < 4; ++w)
                if (w < port_win(c, nc))
                    __hip_atomic_fetch_and(&nc.ports[port_at(c, nc, w, n)], ~t.masks[c.pown_off + w], __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
    }
    if (c.aff && g >= 0) {  // replicated tables: uncommit_aff, atomically
        for (int q = 0; q < c.upd_n; ++q) {
            const int32_t* it = t.aff_items + c.upd_off + 3 * q;
            const bool to_cnt = it[0] == 0;
            const int d = to_cnt ? dom_g(nc, it[1], g) : 0;
            const bool apply = (it[0] == 2 || kind == 1) && d >= 0;
            int32_t* tab = to_cnt ? t.aff_cnt : t.aff_scalar;
            atomic_add_dev(tab + it[2] + (d >= 0 ? d : 0), apply ? -1 : 0);
        }
    }
}

hipError_t launch_undo_pop(const NodeCols& nc, const DevTables& t, int cls, int n, const int32_t* node,
                           const int32_t* kind, hipStream_t st) {
    UndoArgs u{};
    u.cls = cls;
    u.n = n < kMaxChunk ? n : kMaxChunk;
    for (int i = 0; i < u.n; ++i) { u.node[i] = node[i]; u.kind[i] = kind[i]; }
    hipLaunchKernelGGL(k_undo_pop, dim3(1), dim3(64), 0, st, nc, t, u);
    return hipGetLastError();
}

__global__ __launch_bounds__(64) void k_redo_pop(NodeCols nc, DevTables t, UndoArgs u) {
    if (threadIdx.x != 0) return;
    const TaskClass c = t.classes[u.cls];
    for (int i = 0; i < u.n; ++i) {
        if (u.node[i] - nc.base >= 0 && u.node[i] - nc.base < nc.n)
            commit_node(c, t, nc, u.node[i] - nc.base, u.kind[i]);
        if (c.aff && u.node[i] >= 0) commit_aff(c, t, nc, u.node[i], u.kind[i]);
    }
}

hipError_t launch_redo_pop(const NodeCols& nc, const DevTables& t, int cls, int n, const int32_t* node,
                           const int32_t* kind, hipStream_t st) {
    UndoArgs u{};
    u.cls = cls;
    u.n = n < kMaxChunk ? n : kMaxChunk;
    for (int i = 0; i < u.n; ++i) { u.node[i] = node[i]; u.kind[i] = kind[i]; }
    hipLaunchKernelGGL(k_redo_pop, dim3(1), dim3(64), 0, st, nc, t, u);
    return hipGetLastError();
}

// The walk's FitDelta histogram (allocate.go:164-167) of one task recomputed
// on the current node state, which must be the state the task saw (the
// walk's GetAccessibleResource visits already applied; the host undoes the
// task's own commit around it).  The task's class, the inter-pod affinity
// normalisation (ctrl->ipa_lo / ipa_hi[0], from k_ipa_minmax on that state)
// and the fallback node are ctrl's task 0.  chosen < 0: the task found no
// node, every walk node counts; else the walk stopped at node `chosen` with
// kind chosen_kind: the walk nodes before it count (walk order = key order
// without the fit bit, ctrl->slot[0] = the chosen node's walk key from
// k_fit_key, all-reduced over shards), and `chosen` itself when Pipelined.
// out4 (zeroed by the caller) gets this shard's counts.
__device__ __forceinline__ uint64_t fit_walk_key(const Conf& cf, const NodeCols& nc, const DevTables& t,
                                                 const PopCtrl* ctrl, const TaskClass& c, int n) {
    int32_t s = 0;
    bool passed = false;
    (void)eval_node_aff(cf, c, t, nc, n, ctrl->ipa_lo[0], ctrl->ipa_hi[0], ctrl->fallback, &s, &passed);
    return passed ? pack_key(s, n + nc.base, 0) : 0;
}
__global__ __launch_bounds__(64) void k_fit_key(Conf cf, NodeCols nc, DevTables t, PopCtrl* ctrl, int chosen) {
    if (threadIdx.x != 0) return;
    const TaskClass c = t.classes[ctrl->cls[0]];
    const int n = chosen - nc.base;
    ctrl->slot[0] = (n >= 0 && n < nc.n) ? fit_walk_key(cf, nc, t, ctrl, c, n) : 0;
}
__global__ __launch_bounds__(kBlock) void k_fit_delta(Conf cf, NodeCols nc, DevTables t, const PopCtrl* ctrl,
                                                      int chosen, int chosen_kind, int32_t* out4) {
    __shared__ int32_t s_fit[4];
    if (threadIdx.x < 4) s_fit[threadIdx.x] = 0;
    __syncthreads();
    const TaskClass c = t.classes[ctrl->cls[0]];
    const uint64_t wk = ctrl->slot[0];  // walk-order key of the chosen node
    for (int n = blockIdx.x * kBlock + threadIdx.x; n < nc.n; n += gridDim.x * kBlock) {
        const uint64_t k = fit_walk_key(cf, nc, t, ctrl, c, n);
        Row r = load_row(nc, n);
        r.bf_cpu = r.bf_mem = r.bf_gpu = 0;  // Idle as the walk left it
        const bool in = k && (chosen < 0 || k > wk || (n + nc.base == chosen && chosen_kind == 2));
        const uint32_t fb = in ? fit_bits(c, r, true) : 0u;
        for (int b = 0; b < 4; ++b)
            if ((fb >> b) & 1u) atomicAdd(&s_fit[b], 1);
    }
    __syncthreads();
    if (threadIdx.x < 4 && s_fit[threadIdx.x]) atomicAdd(&out4[threadIdx.x], s_fit[threadIdx.x]);
}

hipError_t launch_fit_key(const Conf& cf, const NodeCols& nc, const DevTables& t, PopCtrl* ctrl, int chosen,
                          hipStream_t st) {
    hipLaunchKernelGGL(k_fit_key, dim3(1), dim3(64), 0, st, cf, nc, t, ctrl, chosen);
    return hipGetLastError();
}
hipError_t launch_fit_count(const Conf& cf, const NodeCols& nc, const DevTables& t, PopCtrl* ctrl, int chosen,
                            int chosen_kind, int32_t* out4, hipStream_t st) {
    const int grid = (nc.n + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(k_fit_delta, dim3(grid > 0 ? grid : 1), dim3(kBlock), 0, st, cf, nc, t, (const PopCtrl*)ctrl,
                       chosen, chosen_kind, out4);
    return hipGetLastError();
}

hipError_t launch_commit_task(const NodeCols& nc, const DevTables& t, PopCtrl* ctrl, int task_i, const uint64_t* walk,
                              hipStream_t st) {
    hipLaunchKernelGGL(k_commit_task, dim3(1), dim3(kBlock), 0, st, nc, t, ctrl, task_i, walk);
    return hipGetLastError();
}

hipError_t launch_ipa_minmax(const NodeCols& nc, const DevTables& t, PopCtrl* ctrl, int task_i, hipStream_t st,
                             int64_t* counts) {
    int grid = (nc.n + kBlock - 1) / kBlock;
    if (grid > 2048) grid = 2048;
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL(k_ipa_minmax, dim3(grid), dim3(kBlock), 0, st, nc, t, ctrl, task_i, counts);
    return hipGetLastError();
}

// Grid of the batched pop kernels: nodes per lane R (a power of two, 1 up
// to 262k nodes) so that the block lists stay few enough for the merge tree.
int pop_blocks(int n_nodes, int* R_out) {
    int R = 1;
    while ((int64_t)kPopThreads * R * 512 < n_nodes && R < 16) R <<= 1;
    *R_out = R;
    return (n_nodes + kPopThreads * R - 1) / (kPopThreads * R);
}

#endif
#if KBHIP_PART == 0 || KBHIP_PART == 2  // k_pop_batch (placements 2, 3, 6, 7)
template <typename KT>
static void launch_pop_batch_t(int R, int nb, const Conf& cf, const NodeCols& nc, const DevTables& t, const PopArgs& a,
                               uint64_t* cand, uint32_t* arrive, PopOut* o, ShardMsg* m, const MboxArgs& mb,
                               hipStream_t st) {
#define KBHIP_PB1(RR, PP) \
    hipLaunchKernelGGL((k_pop_batch<RR, KT, PP>), dim3(nb), dim3(kPopThreads), 0, st, cf, nc, t, a, cand, arrive, o, m, mb)
#define KBHIP_PB(RR)                                                   \
    do {                                                               \
        switch (a.placement) {                                         \
            case 3: KBHIP_PB1(RR, 3); break;                           \
            case 6: KBHIP_PB1(RR, 6); break;                           \
            case 7: KBHIP_PB1(RR, 7); break;                           \
            default: KBHIP_PB1(RR, 2); break;                          \
        }                                                              \
    } while (0)
    switch (R) {
        case 1: KBHIP_PB(1); break;
        case 2: KBHIP_PB(2); break;
        case 4: KBHIP_PB(4); break;
        case 8: KBHIP_PB(8); break;
        default: KBHIP_PB(16); break;
    }
#undef KBHIP_PB
#undef KBHIP_PB1
}

#endif
#if KBHIP_PART == 0 || KBHIP_PART == 3  // k_pop_batch_multi
// Multi-session launches: requests grouped by (nodes per lane, key type,
// placement), up to kPopMulti per launch.
template <int R, typename KT, int PL>
static void launch_multi_t(const PopDescs& d, int n, int max_nb, hipStream_t st) {
    hipLaunchKernelGGL((k_pop_batch_multi<R, KT, PL>), dim3(max_nb, n), dim3(kPopThreads), 0, st, d);
}
template <typename KT, int PL>
static void launch_multi_r(int R, const PopDescs& d, int n, int max_nb, hipStream_t st) {
    switch (R) {
        case 1: launch_multi_t<1, KT, PL>(d, n, max_nb, st); break;
        case 2: launch_multi_t<2, KT, PL>(d, n, max_nb, st); break;
        case 4: launch_multi_t<4, KT, PL>(d, n, max_nb, st); break;
        case 8: launch_multi_t<8, KT, PL>(d, n, max_nb, st); break;
        default: launch_multi_t<16, KT, PL>(d, n, max_nb, st); break;
    }
}
hipError_t launch_pop_batch_multi(const PopReq* reqs, int n, hipStream_t st, int* launches) {
    std::vector<char> used(n, 0);
    int nl = 0;
    for (int i = 0; i < n; ++i) {
        if (used[i]) continue;
        int Ri;
        (void)pop_blocks(reqs[i].nc.n, &Ri);
        const bool k32 = reqs[i].kf.use32;
        const int pl = reqs[i].placement;
        if (pl != 6 && pl != 7) return hipErrorInvalidValue;  // the sequential placements only
        PopDescs d{};
        int m = 0, max_nb = 1;
        for (int j = i; j < n && m < kPopMulti; ++j) {
            int Rj;
            const int nbj = pop_blocks(reqs[j].nc.n, &Rj);
            if (used[j] || Rj != Ri || reqs[j].kf.use32 != k32 || reqs[j].placement != pl) continue;
            used[j] = 1;
            const PopReq& q = reqs[j];
            PopDesc& e = d.d[m++];
            e.cf = q.cf;
            e.nc = q.nc;
            e.t = q.t;
            e.a = PopArgs{q.cls, q.n_tasks, q.gang_mode, q.min_avail, q.ready_count, q.epoch, pl, q.kf.base, q.kf.shift,
                          q.kf.idxmax, q.kf.use32 && q.kf.ent32 ? 1 : 0, q.fit_set};
            e.cand = q.cand;
            e.arrive = q.arrive;
            e.out = q.out;
            e.nb = nbj;
            max_nb = nbj > max_nb ? nbj : max_nb;
        }
        if (k32) {
            if (pl == 6) launch_multi_r<uint32_t, 6>(Ri, d, m, max_nb, st);
            else launch_multi_r<uint32_t, 7>(Ri, d, m, max_nb, st);
        } else {
            if (pl == 6) launch_multi_r<uint64_t, 6>(Ri, d, m, max_nb, st);
            else launch_multi_r<uint64_t, 7>(Ri, d, m, max_nb, st);
        }
        ++nl;
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    if (launches) *launches = nl;
    return hipSuccess;
}

#endif
#if KBHIP_PART == 0 || KBHIP_PART == 2
hipError_t launch_pop_batch(const Conf& cf, const NodeCols& nc, const DevTables& t, int cls, int n_tasks,
                            int gang_mode, int min_avail, int ready_count, uint32_t epoch, uint64_t* cand,
                            uint32_t* arrive, void* out_dev, hipStream_t st, int placement, const KeyFormat& kf,
                            int fit_set, ShardMsg* shard_out, const MboxArgs* mbox) {
    if (placement == 3 && !shard_out && !mbox) return hipErrorInvalidValue;
    const MboxArgs mb = mbox ? *mbox : MboxArgs{};
    int R;
    const int nb = pop_blocks(nc.n, &R);
    PopArgs a{cls, n_tasks, gang_mode, min_avail, ready_count, epoch, placement, kf.base, kf.shift, kf.idxmax,
              kf.use32 && kf.ent32 ? 1 : 0, fit_set};
    PopOut* o = (PopOut*)out_dev;
    if (kf.use32) launch_pop_batch_t<uint32_t>(R, nb, cf, nc, t, a, cand, arrive, o, shard_out, mb, st);
    else launch_pop_batch_t<uint64_t>(R, nb, cf, nc, t, a, cand, arrive, o, shard_out, mb, st);
    return hipGetLastError();
}

#endif
#include "kernels/shard.inc"  // node-array shard kernels, launchers (KBHIP_PART <= 1)
}  // namespace kbhip
