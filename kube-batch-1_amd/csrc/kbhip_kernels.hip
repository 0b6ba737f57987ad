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

#include "kbhip_eval.h"
#include "kbhip_internal.h"

namespace kbhip {

#ifdef KBHIP_STAMPS
// Diagnostic build only: phase stamps (s_memrealtime, 100 MHz) of k_pop_batch.
// Layout: [block][0..3] = start, after sweep+wave sort, after block merge, after arrival;
// [nb*4 + 0..7] = last block: merged, chain precomputed, placement done, end.
__device__ uint64_t* g_stamps;
#define STAMP(slot)                                                       \
    do {                                                                  \
        if (threadIdx.x == 0) g_stamps[(slot)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define STAMP(slot) do {} while (0)
#endif

__global__ __launch_bounds__(kBlock) void k_ipa_minmax(NodeCols nc, DevTables t, PopCtrl* ctrl, int task_i) {
    __shared__ int64_t rlo[kBlock / 64], rhi[kBlock / 64];
    if (ctrl->stop >= 0) return;
    const int cls = __builtin_amdgcn_readfirstlane(ctrl->cls[task_i]);
    const TaskClass c = t.classes[cls];
    const int F = ctrl->fallback;
    int64_t lo = 0, hi = 0;  // maxCount / minCount start at 0 (interpod_affinity.go:214-226)
    for (int n = blockIdx.x * kBlock + threadIdx.x; n < nc.n; n += gridDim.x * kBlock) {
        const int64_t v = ipa_count(c, t, nc, n, F);
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
// wave-level exchange: lane i <-> lane i ^ J without the LDS crossbar.
// J = 1, 2: DPP quad_perm; 4: DPP row_shl:4 / row_shr:4 + select; 8: DPP
// row_ror:8; 16 / 32: gfx950 v_permlane16_swap / v_permlane32_swap.
// (ds_bpermute, what __shfl_xor lowers to, costs an LDS round trip per
// 32-bit half; these are VALU ops.)  Checked against __shfl_xor on the GPU.
// ---------------------------------------------------------------------------
template <int J>
__device__ __forceinline__ uint32_t xor_lane32(uint32_t v) {
    const int lane = threadIdx.x & 63;
    if constexpr (J == 1) {
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xf, 0xf, false);  // quad_perm [1,0,3,2]
    } else if constexpr (J == 2) {
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xf, 0xf, false);  // quad_perm [2,3,0,1]
    } else if constexpr (J == 4) {
        const uint32_t up = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x104, 0xf, 0xf, false);  // row_shl:4
        const uint32_t dn = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
        return (lane & 4) ? dn : up;
    } else if constexpr (J == 8) {
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xf, 0xf, false);  // row_ror:8
    } else if constexpr (J == 16) {
        const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
        return (lane & 16) ? r[0] : r[1];
    } else {
        static_assert(J == 32, "xor distance");
        const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        return (lane & 32) ? r[0] : r[1];
    }
}
template <int J>
__device__ __forceinline__ uint64_t xor_lane64(uint64_t v) {
    return ((uint64_t)xor_lane32<J>((uint32_t)(v >> 32)) << 32) | xor_lane32<J>((uint32_t)v);
}
template <int J, typename T>
__device__ __forceinline__ T xor_lane(T v) {
    if constexpr (sizeof(T) == 8) return xor_lane64<J>(v);
    else return xor_lane32<J>(v);
}
template <typename T>
__device__ __forceinline__ T reverse_lanes(T v) {  // lane i <- lane 63 - i (= i ^ 63)
    if constexpr (sizeof(T) == 8) {
        const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, 0x140, 0xf, 0xf, false);  // row_mirror
        const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v >> 32), 0x140, 0xf, 0xf, false);
        return xor_lane64<32>(xor_lane64<16>(((uint64_t)hi << 32) | lo));
    } else {
        const uint32_t m = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xf, 0xf, false);
        return xor_lane32<32>(xor_lane32<16>(m));
    }
}

// ---------------------------------------------------------------------------
// wave / block reductions
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
    uint64_t u;
    u = xor_lane64<32>(v); v = u > v ? u : v;
    u = xor_lane64<16>(v); v = u > v ? u : v;
    u = xor_lane64<8>(v); v = u > v ? u : v;
    u = xor_lane64<4>(v); v = u > v ? u : v;
    u = xor_lane64<2>(v); v = u > v ? u : v;
    u = xor_lane64<1>(v); v = u > v ? u : v;
    return v;
}

// ---------------------------------------------------------------------------
// per-task path
// ---------------------------------------------------------------------------
// Commit of task task_i once ctrl->slot[task_i] holds the winner key over ALL
// nodes (all shards): result, gang stop, node row (owner only), pod-affinity
// tables and fallback node (every shard, identically), and the
// GetAccessibleResource mutation of the visited nodes of this shard.  Run by
// one block: the last sweep block (one GPU) or k_commit_task (sharded).
__device__ void commit_task(const NodeCols& nc, const DevTables& t, PopCtrl* ctrl, int task_i, const TaskClass& c,
                            bool first_fit, bool track, const uint64_t* walk, bool defer_visits = false) {
    __shared__ uint64_t win;
    if (threadIdx.x == 0) {
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
                if (c.aff) commit_aff(c, t, nc, g, 1);
                if (ctrl->fallback < 0 || g < ctrl->fallback) ctrl->fallback = g;
                if (c.backfill) ctrl->any_bf = 1;
            }
            ctrl->n_done = task_i + 1;
            if (task_i + 1 == ctrl->n_tasks) ctrl->stop = 0;
        } else if (k == 0) {
            ctrl->res_node[task_i] = -1;
            ctrl->res_kind[task_i] = 0;
            ctrl->n_done = task_i + 1;
            ctrl->stop = 1;
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
            if (c.aff) commit_aff(c, t, nc, g, kind);
            if (ctrl->fallback < 0 || g < ctrl->fallback) ctrl->fallback = g;
            if (c.backfill) ctrl->any_bf = 1;
            after_assign(ctrl, task_i, kind);
        }
    }
    __syncthreads();
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
__global__ __launch_bounds__(kBlock) void k_sweep_argmax(Conf cf, NodeCols nc, DevTables t, PopCtrl* ctrl,
                                                         int task_i, uint64_t* walk, int commit_here, uint64_t* dbg) {
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
    for (int n = blockIdx.x * kBlock + threadIdx.x; n < nc.n; n += gridDim.x * kBlock) {
        int32_t s = 0;
        bool passed = false;
        uint32_t fb = 0;
        const uint64_t k = first_fit ? eval_first_fit(cf, c, t, nc, n)
                                     : eval_node_aff(cf, c, t, nc, n, ilo, ihi, F, &s, &passed, &fb);
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
        last = prev == gridDim.x - 1;
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

// The GetAccessibleResource mutation of task task_i's walk (node_info.go:209-211,
// SURVEY Appendix A.1) over the whole grid, after k_sweep_argmax committed it
// with the mutation deferred (one block looping over every node is a chain of
// N / kBlock dependent memory round trips).  Runs only if task_i was swept
// (n_done == task_i + 1) and its sweep tracked the walk (pad, set by commit_task).
__global__ __launch_bounds__(kBlock) void k_visit_mutate(NodeCols nc, const PopCtrl* ctrl, int task_i,
                                                         const uint64_t* walk) {
    if (ctrl->n_done != task_i + 1 || !ctrl->pad) return;  // uniform
    const uint64_t k = ctrl->slot[task_i];
    const uint64_t wk = k ? pack_key(key_score(k), key_idx(k), 0) : 0;
    const int wn = k ? key_idx(k) : -1;
    for (int n = blockIdx.x * kBlock + threadIdx.x; n < nc.n; n += gridDim.x * kBlock) {
        const uint64_t v = walk[n];
        if (!v || n + nc.base == wn) continue;
        if (k && v < wk) continue;
        nc.idle_cpu[n] += nc.bf_cpu[n]; nc.idle_mem[n] += nc.bf_mem[n]; nc.idle_gpu[n] += nc.bf_gpu[n];
    }
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

// ---------------------------------------------------------------------------
// batched path
// ---------------------------------------------------------------------------
// ---------------------------------------------------------------------------
// batched path v2: one launch per pop chunk
// ---------------------------------------------------------------------------
// Wave-level sorting on registers: lane i holds one key (u32 or u64);
// descending order.  Bitonic network, every exchange a DPP / permlane op.
template <int K, int J, typename T>
__device__ __forceinline__ T bitonic_step(T v) {
    const int lane = threadIdx.x & 63;
    const T o = xor_lane<J>(v);
    const bool keep_max = ((lane & J) == 0) == ((lane & K) == 0);
    return keep_max ? (o > v ? o : v) : (o < v ? o : v);
}
template <int K, typename T>
__device__ __forceinline__ T bitonic_stage(T v) {
    if constexpr (K >= 64) v = bitonic_step<K, 32>(v);
    if constexpr (K >= 32) v = bitonic_step<K, 16>(v);
    if constexpr (K >= 16) v = bitonic_step<K, 8>(v);
    if constexpr (K >= 8) v = bitonic_step<K, 4>(v);
    if constexpr (K >= 4) v = bitonic_step<K, 2>(v);
    return bitonic_step<K, 1>(v);
}
template <typename T>
__device__ __forceinline__ T wave_sort_desc(T v) {
    v = bitonic_stage<2>(v);
    v = bitonic_stage<4>(v);
    v = bitonic_stage<8>(v);
    v = bitonic_stage<16>(v);
    v = bitonic_stage<32>(v);
    return bitonic_stage<64>(v);
}
// Top-64 of two descending lists (lane i holds a[i], b[i]); result descending.
template <int J, typename T>
__device__ __forceinline__ T half_clean_desc(T v) {
    const int lane = threadIdx.x & 63;
    const T o = xor_lane<J>(v);
    return ((lane & J) == 0) ? (o > v ? o : v) : (o < v ? o : v);
}
template <typename T>
__device__ __forceinline__ T wave_merge_desc(T a, T b) {
    const T br = reverse_lanes(b);
    T v = a > br ? a : br;  // bitonic, holds the top 64 of a U b
    v = half_clean_desc<32>(v);
    v = half_clean_desc<16>(v);
    v = half_clean_desc<8>(v);
    v = half_clean_desc<4>(v);
    v = half_clean_desc<2>(v);
    return half_clean_desc<1>(v);
}

// Results land in pinned host memory as self-tagged 8-byte granules, one per
// consumed task, each written by ONE 8-byte store (no fence needed: the host
// polls the tags).  granule = epoch<<48 | (stop+1)<<44 | n_done<<36 | kind<<34 | (node+1)
struct PopOut {
    uint64_t g[kMaxChunk];
    uint64_t fit[2];  // FitDelta histogram of a task that found no node: walk nodes, cpu | memory, GPU
};
__host__ __device__ inline uint64_t make_fit_granule(uint32_t epoch, uint32_t a, uint32_t b) {
    return ((uint64_t)(epoch & 0xffff) << 48) | ((uint64_t)(b & 0xffffffu) << 24) | (uint64_t)(a & 0xffffffu);
}
// Per-group FitDelta counters of the batched sweep, after the arrival counters:
// two sets; a launch adds to one and zeroes the other (its stream's previous
// launch read that one and the next one adds to it).
__device__ __forceinline__ uint32_t* fit_counters(uint32_t* arrive, int set) {
    return arrive + (kMaxGroups + 1) * 32 + set * kMaxGroups * 32;
}
// Block: add this lane's fit bits to the block's LDS counters (every lane of every wave).
__device__ __forceinline__ void fit_block_add(uint32_t* s_fitb, uint32_t fb) {
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const int cnt = __popcll(__ballot((fb >> b) & 1u));
        if ((threadIdx.x & 63) == 0 && cnt) atomicAdd(&s_fitb[b], (uint32_t)cnt);
    }
}
__host__ __device__ inline uint64_t make_granule(uint32_t epoch, int stop, int n_done, int kind, int node) {
    return ((uint64_t)(epoch & 0xffff) << 48) | ((uint64_t)(stop + 1) << 44) | ((uint64_t)n_done << 36) |
           ((uint64_t)kind << 34) | (uint64_t)(uint32_t)(node + 1);
}

struct PopArgs {
    int32_t cls, n_tasks, gang_mode, min_avail, ready_count;
    uint32_t epoch;
    int32_t placement;  // 0: sequential loop over precomputed chains, 1: running-min levels, 2: parallel levels
    // 32-bit selection keys (when the class's score range and the node count
    // fit): key = (score - kbase + 1) << kshift | (kidxmax - idx) << 1 | pipelined,
    // ordered exactly as pack_key; halves the sort / merge network work.
    int32_t kbase, kshift, kidxmax;
    int32_t ent32;  // placement entries in 32 bits: (rm - kbase + 1) fits in 32 - kshift - 5 bits
    int32_t fit_set;  // FitDelta counter set of this launch (alternates per stream; the other one is zeroed)
};

// Selection key of the batched sweep in type T (see PopArgs).
template <typename T>
__device__ __forceinline__ T sweep_key(uint64_t k64, const PopArgs& a) {
    if constexpr (sizeof(T) == 8) {
        return k64;
    } else {
        if (!k64) return 0;
        return ((uint32_t)(key_score(k64) - a.kbase + 1) << a.kshift) |
               ((uint32_t)(a.kidxmax - key_idx(k64)) << 1) | (uint32_t)(k64 & 1);
    }
}
template <typename T>
__device__ __forceinline__ uint64_t key64_of(T k, const PopArgs& a) {
    if constexpr (sizeof(T) == 8) {
        return k;
    } else {
        if (!k) return 0;
        return pack_key((int32_t)(k >> a.kshift) - 1 + a.kbase, a.kidxmax - (int32_t)((k >> 1) & (uint32_t)a.kidxmax),
                        (int32_t)(k & 1));
    }
}

constexpr int kPopThreads = 512;  // 8 waves
constexpr int kDepth = 3;         // post-commit keys precomputed per candidate

__device__ __forceinline__ Row apply_commits(Row r, const TaskClass& c, int na, int np) {
    r.idle_cpu -= na * c.req_cpu; r.idle_mem -= na * c.req_mem; r.idle_gpu -= na * c.req_gpu;
    r.rel_cpu -= np * c.req_cpu; r.rel_mem -= np * c.req_mem; r.rel_gpu -= np * c.req_gpu;
    const int n = na + np;
    r.pods += n;
    r.nzc += n * c.nz_cpu;
    r.nzm += n * c.nz_mem;
    return r;
}

// 64-lane max of a u32 with DPP row shifts + row broadcasts (GFX9 family),
// broadcast to every lane.
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
    uint32_t t;
    t = (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x111, 0xf, 0xf, false); v = t > v ? t : v;  // row_shr:1
    t = (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x112, 0xf, 0xf, false); v = t > v ? t : v;  // row_shr:2
    t = (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x114, 0xf, 0xf, false); v = t > v ? t : v;  // row_shr:4
    t = (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x118, 0xf, 0xf, false); v = t > v ? t : v;  // row_shr:8
    t = (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x142, 0xa, 0xf, false); v = t > v ? t : v;  // row_bcast:15
    t = (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x143, 0xc, 0xf, false); v = t > v ? t : v;  // row_bcast:31
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
__device__ __forceinline__ uint64_t wave_max_key(uint64_t v) {
    const uint32_t hi = wave_max_u32((uint32_t)(v >> 32));
    const uint32_t lo = wave_max_u32((uint32_t)(v >> 32) == hi ? (uint32_t)v : 0u);
    return ((uint64_t)hi << 32) | lo;
}

// ---------------------------------------------------------------------------
// Placement by levels (option "placement" = 1).  The greedy of a chunk picks,
// task after task, the node with the largest current key; only the winner's
// key changes.  Give candidate j the entries e(j, d) for its d-th extra
// commit: (running minimum of its scores over levels 0..d, index, d, real
// kind).  The greedy's choice sequence equals the entries sorted descending:
// a node whose key RISES after a commit is picked again at once (every other
// current key is below its previous one), which the running minimum keeps in
// place; between nodes, equal scores go to the lower index as in pack_key.
// Entries are generated level by level (one re-evaluation per lane), merged
// into a sorted top-64, and generation stops when no lane's newest entry
// reaches the current m-th entry (deeper entries of a node are smaller).
// ---------------------------------------------------------------------------
constexpr int kEntryIdxMax = (1 << 25) - 1;  // batched path: < 2^25 nodes

// Node rows handed from one overlapped pop to the next (k_pop_batch_ov):
// written with sc1 (write-through) stores, read with sc1 loads (L1 bypass),
// the storing wave drained before the flag (MI355X_MICROARCH.md valid forms,
// row 1) — no release / acquire fences on the pop-to-pop critical path.
template <typename T>
__device__ __forceinline__ T ld_sc1(const T* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ void st_sc1(T* p, T v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// load_row with the columns a batched placement writes read through sc1
// (Backfilled, allocatable and MaxTaskNum never change on the batched path).
__device__ __forceinline__ Row load_row_sc1(const NodeCols& nc, int n) {
    Row r;
    r.idle_cpu = ld_sc1(&nc.idle_cpu[n]); r.idle_mem = ld_sc1(&nc.idle_mem[n]); r.idle_gpu = ld_sc1(&nc.idle_gpu[n]);
    r.rel_cpu = ld_sc1(&nc.rel_cpu[n]); r.rel_mem = ld_sc1(&nc.rel_mem[n]); r.rel_gpu = ld_sc1(&nc.rel_gpu[n]);
    r.bf_cpu = nc.bf_cpu[n]; r.bf_mem = nc.bf_mem[n]; r.bf_gpu = nc.bf_gpu[n];
    r.acpu = nc.acpu[n]; r.amem = nc.amem[n]; r.nzc = ld_sc1(&nc.nzc[n]); r.nzm = ld_sc1(&nc.nzm[n]);
    r.pods = ld_sc1(&nc.pods[n]); r.maxtasks = nc.maxtasks[n];
    return r;
}
template <bool SC1>
__device__ __forceinline__ Row load_row_t(const NodeCols& nc, int n) {
    if constexpr (SC1) return load_row_sc1(nc, n);
    else return load_row(nc, n);
}
template <bool SC1>
__device__ __forceinline__ uint64_t load_port_t(const NodeCols& nc, int w, int n) {
    const uint64_t* p = nc.ports + (int64_t)w * nc.npad + n;
    if constexpr (SC1) return ld_sc1(p);
    else return *p;
}
// eval_node with the rows read through sc1.
__device__ __forceinline__ uint64_t eval_node_sc1(const Conf& cf, const TaskClass& c, const DevTables& t,
                                                  const NodeCols& nc, int n, uint32_t* fit = nullptr) {
    const bool st = static_pred(cf, c, t, nc, n);
    const int32_t na = (st && cf.score_mult) ? na_weight(c, t, nc, n) : 0;
    const Row r = load_row_sc1(nc, n);
    uint64_t pw[4] = {0, 0, 0, 0};
    if (c.has_ports)
        for (int w = 0; w < nc.port_words && w < 4; ++w) pw[w] = load_port_t<true>(nc, w, n);
    int32_t s;
    bool passed;
    const uint64_t k = dyn_key(cf, c, t, nc, r, pw, n, st, na, &s, &passed);
    if (fit) *fit = fit_bits(c, r, passed);
    return k;
}

__device__ __forceinline__ uint64_t level_entry(int32_t rm, int n, int d, uint64_t key) {
    return ((uint64_t)((uint32_t)rm ^ 0x80000000u) << 32) | ((uint64_t)(kEntryIdxMax - n) << 7) |
           ((uint64_t)(63 - d) << 1) | (key & 1);
}
__device__ __forceinline__ int entry_idx(uint64_t e) { return kEntryIdxMax - (int)((e >> 7) & kEntryIdxMax); }
__device__ __forceinline__ int entry_kind(uint64_t e) { return (e & 1) ? 2 : 1; }
__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
    return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(v >> 32), l) << 32 |
           (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}

// Hand-off of 64-key lists between workgroups: write-through (sc1) 8-byte
// stores drained before an agent-scope counter add, sc1 loads on the consumer
// after its add returned (MI355X_MICROARCH.md, valid forms, table row 1).
template <typename T>
__device__ __forceinline__ void put_list(T* dst, T v) {
    __hip_atomic_store(dst + (threadIdx.x & 63), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ T get_list(const T* src) {
    return __hip_atomic_load(src + (threadIdx.x & 63), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

#ifndef KBHIP_GROUPS
#define KBHIP_GROUPS 8
#endif
constexpr int kGroups = KBHIP_GROUPS;  // second-level merge groups (blockIdx % kGroups)
static_assert(kGroups >= 1 && kGroups <= 32, "group lists and counters");
constexpr int kCtrStride = 32;    // one counter per 128-byte line

// Tree merge of the 8 per-wave lists in wl[] into wl[0] (all waves call).
template <typename T>
__device__ __forceinline__ void block_tree_merge(T (*wl)[64], int wave, int lane) {
#pragma unroll
    for (int s = kPopThreads / 128; s >= 1; s >>= 1) {
        if (wave < s) wl[wave][lane] = wave_merge_desc(wl[wave][lane], wl[wave + s][lane]);
        __syncthreads();
    }
}

// Wave 0 of the final merger: K = lane's candidate key (sorted top-64).
__device__ void place_levels(const Conf& cf, const NodeCols& nc, const DevTables& t, const TaskClass& c,
                             const PopArgs& a, uint64_t K, PopOut* out) {
    const int lane = threadIdx.x & 63;
    const int n = K ? key_idx(K) : -1;
    Row base{};
    uint64_t pw[4] = {0, 0, 0, 0};
    int32_t na_n = 0;
    if (n >= 0) {
        base = load_row(nc, n);
        if (c.has_ports)
            for (int w = 0; w < nc.port_words && w < 4; ++w) pw[w] = nc.ports[(int64_t)w * nc.npad + n];
        if (cf.score_mult) na_n = na_weight(c, t, nc, n);
    }
    uint64_t pwc[4];  // ports after one or more commits of this class
    for (int w = 0; w < 4; ++w) pwc[w] = pw[w] | ((c.has_ports && w < nc.port_words) ? t.masks[c.pown_off + w] : 0);
    const int m = a.n_tasks;
    uint64_t key = K;                                  // real key of the node after `ca + cp` commits
    int32_t rm = K ? key_score(K) : 0;                 // running minimum of its scores
    uint64_t cur = K ? level_entry(rm, n, 0, K) : 0;   // this lane's newest entry
    uint64_t L = cur;                                  // sorted top-64 entries: lane p holds entry p
    int ca = 0, cp = 0;
    for (int d = 1; d < 64; ++d) {
        const uint64_t T = readlane64(L, m - 1);       // m-th entry: deeper entries below it never place
        if (!__ballot(cur != 0 && cur >= T)) break;
        uint64_t e = 0;
        if (key) {
            if (key & 1) ++cp; else ++ca;              // the commit of the previous level (Pipeline / Allocate)
            const Row r = apply_commits(base, c, ca, cp);
            int32_t s;
            bool passed;
            key = dyn_key(cf, c, t, nc, r, pwc, n, true, na_n, &s, &passed);
            if (key) {
                rm = key_score(key) < rm ? key_score(key) : rm;
                e = level_entry(rm, n, d, key);
            }
        }
        cur = e;
        L = wave_merge_desc(L, wave_sort_desc(e >= T ? e : 0));  // entries below T cannot reach the top m
    }
    STAMP(gridDim.x * 4 + 2);
    // stop rule over the placement order (allocate.go:187-195, gang.go:63-66)
    const bool valid = lane < m && L != 0;
    const uint64_t amask = __ballot(valid && entry_kind(L) == 1);  // Pipelined is not an AllocatedStatus
    const uint64_t upto = lane == 63 ? ~0ull : ((2ull << lane) - 1);
    const int ready_p = a.ready_count + __popcll(amask & upto);
    const uint64_t smask = __ballot(lane < m && (!valid || !a.gang_mode || ready_p >= a.min_avail));
    int done, stop;
    if (smask) {
        const int p = __ffsll((unsigned long long)smask) - 1;
        done = p + 1;
        stop = __builtin_amdgcn_readlane((int)valid, p) ? 2 : 1;
    } else {
        done = m;
        stop = 0;
    }
    // commits of this lane's node among the placed entries; write the row back
    int na = 0, np = 0;
    for (int p = 0; p < done; ++p) {
        const uint64_t e = readlane64(L, p);
        if (e && entry_idx(e) == n) { if (entry_kind(e) == 1) ++na; else ++np; }
    }
    if (n >= 0 && na + np > 0) {
        const Row r = apply_commits(base, c, na, np);
        nc.idle_cpu[n] = r.idle_cpu; nc.idle_mem[n] = r.idle_mem; nc.idle_gpu[n] = r.idle_gpu;
        nc.rel_cpu[n] = r.rel_cpu; nc.rel_mem[n] = r.rel_mem; nc.rel_gpu[n] = r.rel_gpu;
        nc.pods[n] = r.pods;
        nc.nzc[n] = r.nzc;
        nc.nzm[n] = r.nzm;
        if (c.has_ports)
            for (int w = 0; w < nc.port_words && w < 4; ++w) nc.ports[(int64_t)w * nc.npad + n] = pwc[w];
    }
    if (lane < done)
        __hip_atomic_store(&out->g[lane],
                           make_granule(a.epoch, stop, done, L ? entry_kind(L) : 0, L ? entry_idx(L) : -1),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    STAMP(gridDim.x * 4 + 3);
}

// ---------------------------------------------------------------------------
// Placement by parallel levels (option "placement" = 2): the same entries as
// place_levels, but a round computes 8 depths at once — wave w evaluates
// candidate j after d = 8r + w commits of this class — then one sort + tree
// merge of the round's 512 entries.  Commit kinds along a chain are
// Allocate^a Pipeline^p (once Idle + Backfilled cannot fit, later commits
// only touch Releasing), so a first pass assumes Allocate everywhere and the
// depths behind a lane's first Pipeline are recomputed.  An entry is
// (running min, index, depth) — a position's depth is the number of commits
// its node already took — and a small LDS hash from node index to candidate
// lane finds the candidate's commit kinds and counts.  Another round runs
// only while some candidate's deepest entry still reaches the m-th entry.
// ---------------------------------------------------------------------------
// 64-bit: (rm biased) << 32 | (kEntryIdxMax - n) << 7 | (63 - d) << 1 | 1.
// 32-bit (PopArgs::ent32): (rm - kbase + 1) << (kshift + 5) | (kidxmax - n) << 6 | (63 - d).
template <typename ET>
__device__ __forceinline__ ET depth_entry(int32_t rm, int n, int d, const PopArgs& a) {
    if constexpr (sizeof(ET) == 8)
        return ((uint64_t)((uint32_t)rm ^ 0x80000000u) << 32) | ((uint64_t)(kEntryIdxMax - n) << 7) |
               ((uint64_t)(63 - d) << 1) | 1ull;
    else
        return ((uint32_t)(rm - a.kbase + 1) << (a.kshift + 5)) | ((uint32_t)(a.kidxmax - n) << 6) |
               (uint32_t)(63 - d);
}
template <typename ET>
__device__ __forceinline__ int entry_depth(ET e) {
    if constexpr (sizeof(ET) == 8) return 63 - (int)((e >> 1) & 63);
    else return 63 - (int)(e & 63);
}
template <typename ET>
__device__ __forceinline__ int entry_node(ET e, const PopArgs& a) {
    if constexpr (sizeof(ET) == 8) return entry_idx(e);
    else return a.kidxmax - (int)((e >> 6) & (uint32_t)a.kidxmax);
}
template <typename T>
__device__ __forceinline__ T readlane_t(T v, int l) {
    if constexpr (sizeof(T) == 8) return readlane64(v, l);
    else return (T)__builtin_amdgcn_readlane((int)v, l);
}
constexpr int kHash = 256;  // node index -> candidate lane (64 keys, open addressing)
__device__ __forceinline__ int hash_slot(int n) { return (int)(((uint32_t)n * 2654435761u) >> 24); }

// Rows of the nodes a placement may use, gathered before it starts (LDS):
// the overlapped pop loads them while it waits for the previous pop, so the
// placement reads no node row from memory.  Slot lookup by node index.
constexpr int kRcSlots = 128;
struct RowCache {
    Row row[kRcSlots];
    uint64_t pw[kRcSlots][4];
    int32_t na[kRcSlots];
    int32_t hkey[kHash];
    int32_t hslot[kHash];
};
__device__ __forceinline__ void rc_insert(RowCache* rc, int n, int slot) {  // n distinct
    int h = hash_slot(n);
    while (atomicCAS(&rc->hkey[h], -1, n) != -1) h = (h + 1) & (kHash - 1);
    rc->hslot[h] = slot;
}
__device__ __forceinline__ int rc_find(const RowCache* rc, int n) {
    int h = hash_slot(n);
    for (int i = 0; i < kHash; ++i, h = (h + 1) & (kHash - 1)) {
        const int k = rc->hkey[h];
        if (k == n) return rc->hslot[h];
        if (k == -1) return -1;
    }
    return -1;
}

__device__ __forceinline__ void fit_zero_other(uint32_t* arrive, int set) {
    if (blockIdx.x == 0 && threadIdx.x < kGroups * 4)
        fit_counters(arrive, 1 - set)[(threadIdx.x >> 2) * 32 + (threadIdx.x & 3)] = 0;
}
// Wave 0 of the final merger: lane 4g + b loads group g's count b (one round
// trip, consumed only if a task finds no node: fit_sum).
__device__ __forceinline__ uint32_t fit_load(const uint32_t* fitc, int n_groups) {
    const int lane = threadIdx.x & 63;
    uint32_t v = 0;
    for (int gi = lane >> 2; gi < n_groups; gi += 16) v += ld_sc1(&fitc[gi * 32 + (lane & 3)]);
    return v;
}
__device__ __forceinline__ uint32_t fit_sum(uint32_t v) {  // count b in lanes b, b+4, ...
    v += __shfl_xor(v, 4, 64);
    v += __shfl_xor(v, 8, 64);
    v += __shfl_xor(v, 16, 64);
    return v + __shfl_xor(v, 32, 64);
}

// SC1: rows read and written through sc1 (overlapped pops); the write-back is
// then published as done = seq before the result stores.
// L sorted descending over the lanes, e not in L: L with e inserted (the last
// entry drops off).  A ballot gives the position, a DPP wave_shr:1 moves the tail.
template <typename T>
__device__ __forceinline__ T wave_shr1(T v) {  // lane i <- lane i - 1 (lane 0 <- 0)
    if constexpr (sizeof(T) == 8) {
        const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, 0x138, 0xf, 0xf, false);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v >> 32), 0x138, 0xf, 0xf, false);
        return ((uint64_t)hi << 32) | lo;
    } else {
        return (T)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xf, 0xf, false);
    }
}
template <typename T>
__device__ __forceinline__ T wave_insert_sorted(T L, T e) {
    const int lane = threadIdx.x & 63;
    const int pos = __popcll(__ballot(L > e));
    const T sh = wave_shr1(L);
    return lane < pos ? L : (lane == pos ? e : sh);
}

// INS: the round's entries join the running list by insertion (only those
// above the m-th entry; usually a few) instead of a sort + merge tree.
template <typename ET, bool SC1 = false, bool INS = false>
__device__ void place_parallel(const Conf& cf, const NodeCols& nc, const DevTables& t, const TaskClass& c,
                               const PopArgs& a, PopOut* out, uint64_t (*wl64)[64], uint32_t* done_flag = nullptr,
                               uint32_t seq = 0, const RowCache* rc = nullptr, const int32_t* fit_in = nullptr,
                               uint32_t fit_raw = 0, int wb_base = 0, int wb_n = 0x7fffffff) {
    // wb_base / wb_n: node rows [wb_base, wb_base + wb_n) are this device's
    // (a node-array shard writes back only its own; one GPU: all of them).
    // Node indices in keys and entries are global.
    constexpr int kW = kPopThreads / 64;  // depths per round
    __shared__ int32_t s_sc[kW][64];      // this round's scores, by depth slot
    __shared__ uint8_t s_kind[64][64];    // [depth][candidate]: 1 Allocate, 2 Pipeline, 0 infeasible
    __shared__ int32_t s_rm[2][64];       // running min through the previous round's deepest depth
    __shared__ int32_t s_apos[64];        // first Pipeline depth (64: none yet)
    __shared__ ET s_last[64];             // entry at the round's deepest depth
    __shared__ int32_t s_cnt[64];
    __shared__ int32_t s_hkey[kHash];
    __shared__ int32_t s_hlane[kHash];
    __shared__ int s_more;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t K = wl64[0][lane];
    ET (*wl)[64] = (ET (*)[64])wl64;      // sort / merge lists of entries (same LDS)
    const int n = K ? key_idx(K) : -1;
    Row base{};
    uint64_t pw[4] = {0, 0, 0, 0};
    int32_t na_n = 0;
    const int rslot = (rc && n >= 0) ? rc_find(rc, n) : -1;
    if (rslot >= 0) {
        base = rc->row[rslot];
        for (int w = 0; w < 4; ++w) pw[w] = rc->pw[rslot][w];
        na_n = rc->na[rslot];
    } else if (n >= 0) {
        base = load_row_t<SC1>(nc, n);
        if (c.has_ports)
            for (int w = 0; w < nc.port_words && w < 4; ++w) pw[w] = load_port_t<SC1>(nc, w, n);
        if (cf.score_mult) na_n = na_weight(c, t, nc, n);
    }
    STAMP(gridDim.x * 4 + 11);
    uint64_t pwc[4];
    for (int w = 0; w < 4; ++w) pwc[w] = pw[w] | ((c.has_ports && w < nc.port_words) ? t.masks[c.pown_off + w] : 0);
    const int m = a.n_tasks;
    if (wave == 0) { s_apos[lane] = 64; s_cnt[lane] = 0; }
    if (threadIdx.x < kHash) s_hkey[threadIdx.x] = -1;
    __syncthreads();  // K read by every wave; wl free
    STAMP(gridDim.x * 4 + 12);
    if (wave == 0 && n >= 0) {  // candidate nodes are distinct
        int h = hash_slot(n);
        while (atomicCAS(&s_hkey[h], -1, n) != -1) h = (h + 1) & (kHash - 1);
        s_hlane[h] = lane;
    }
    STAMP(gridDim.x * 4 + 5);
    auto eval_at = [&](int d, int ap, int32_t* sc) -> int {  // kind of commit d+1's key (0: infeasible)
        if (d == 0) { *sc = key_score(K); return key_kind(K); }
        const int na = d < ap ? d : ap;
        const Row r = apply_commits(base, c, na, d - na);
        int32_t s;
        bool passed;
        const uint64_t k = dyn_key(cf, c, t, nc, r, pwc, n, true, na_n, &s, &passed);
        *sc = k ? key_score(k) : 0;
        return k ? key_kind(k) : 0;
    };
    ET L = 0;            // wave 0: merged top-64 entries so far (lane p = entry p)
    bool alive = n >= 0; // candidate still relevant (uniform over waves)
    for (int r = 0; r < 64 / kW; ++r) {
        const int d = r * kW + wave;
        int ap = s_apos[lane];
        int32_t sc = 0;
        int kind = alive ? eval_at(d, ap, &sc) : 0;
        s_kind[d][lane] = (uint8_t)kind;
        __syncthreads();
        if (ap == 64) {  // first Pipeline within this round: recompute the depths behind it
            // (no barrier before the rewrites below: they only touch depths
            // after the first Pipeline, which every scan stops at)
            for (int w2 = 0; w2 < kW; ++w2)
                if (s_kind[r * kW + w2][lane] == 2) { ap = r * kW + w2; break; }
            if (alive && ap < d) {
                kind = eval_at(d, ap, &sc);
                s_kind[d][lane] = (uint8_t)kind;
            }
        }
        s_sc[wave][lane] = sc;
        if (wave == 0) s_apos[lane] = ap;
        __syncthreads();
        // running minimum through depth d; the chain ends at the first infeasible depth
        bool ok = alive;
        int32_t rm = r == 0 ? INT32_MAX : s_rm[r & 1][lane];
#pragma unroll
        for (int w2 = 0; w2 < kW; ++w2) {
            if (w2 > wave) break;
            ok = ok && s_kind[r * kW + w2][lane] != 0;
            const int32_t x = s_sc[w2][lane];
            rm = x < rm ? x : rm;
        }
        const ET e = ok ? depth_entry<ET>(rm, n, d, a) : (ET)0;
        if (r == 0) STAMP(gridDim.x * 4 + 6);
        if (wave == kW - 1) { s_last[lane] = e; s_rm[(r + 1) & 1][lane] = rm; }
        if constexpr (INS) {
            wl[wave][lane] = e;
            __syncthreads();
            if (wave == 0) {
                // depth 0 (round 0, wave 0): the candidate list itself, already sorted
                int w0 = 0;
                if (r == 0) { L = e; w0 = 1; }
                ET T = readlane_t(L, m - 1);
                for (int w2 = w0; w2 < kW; ++w2) {
                    const ET x = wl[w2][lane];
                    for (uint64_t q = __ballot(x > T); q; q &= q - 1) {
                        const ET y = readlane_t(x, __ffsll((unsigned long long)q) - 1);
                        if (y > T) {
                            L = wave_insert_sorted(L, y);
                            T = readlane_t(L, m - 1);
                        }
                    }
                }
            }
        } else {
            wl[wave][lane] = wave_sort_desc(e);
            __syncthreads();
            block_tree_merge(wl, wave, lane);
            if (wave == 0) L = r == 0 ? wl[0][lane] : wave_merge_desc(L, wl[0][lane]);
        }
        if (wave == 0) {
            if (r == 0) STAMP(gridDim.x * 4 + 7);
            const ET T = readlane_t(L, m - 1);  // m-th entry: deeper entries below it never place
            const ET le = s_last[lane];
            const bool more = le != 0 && le >= T;
            const bool any = __ballot(more) != 0;  // all 64 lanes active
            if (lane == 0) s_more = any;
            s_last[lane] = more;  // reused as the alive flag of the next round
        }
        __syncthreads();
        if (!s_more) break;
        alive = s_last[lane] != 0;  // rewritten by wave kW-1 only after the next round's first barrier
    }
    if (wave != 0) return;
    STAMP(gridDim.x * 4 + 2);
    // commit kind of each position: its node's candidate lane, the entry's depth
    const bool inm = lane < m && L != 0;
    int lf = 0;
    if (inm) {
        const int ni = entry_node(L, a);
        int h = hash_slot(ni);
        while (s_hkey[h] != ni) h = (h + 1) & (kHash - 1);
        lf = s_hlane[h];
    }
    const int kind = inm ? s_kind[entry_depth(L)][lf] : 0;
    // stop rule over the placement order (allocate.go:187-195, gang.go:63-66)
    const uint64_t amask = __ballot(inm && kind == 1);  // Pipelined is not an AllocatedStatus
    const uint64_t upto = lane == 63 ? ~0ull : ((2ull << lane) - 1);
    const int ready_p = a.ready_count + __popcll(amask & upto);
    const uint64_t smask = __ballot(lane < m && (!inm || !a.gang_mode || ready_p >= a.min_avail));
    int done, stop;
    if (smask) {
        const int p = __ffsll((unsigned long long)smask) - 1;
        done = p + 1;
        stop = __builtin_amdgcn_readlane((int)inm, p) ? 2 : 1;
    } else {
        done = m;
        stop = 0;
    }
    STAMP(gridDim.x * 4 + 8);
    if (lane < done && inm) atomicAdd(&s_cnt[lf], 1);
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the LDS adds of this wave
    __builtin_amdgcn_wave_barrier();
    const int cc = s_cnt[lane];
    STAMP(gridDim.x * 4 + 9);
    if (fit_in && stop == 1) {  // a task found no node: the walk's FitDelta histogram at that task
        // fit_in: every node at the state this pop started from; the candidates
        // then carry the commits made before the failing task
        uint32_t fb_base = 0, fb_post = 0;
        if (n >= 0) {
            fb_base = fit_bits(c, base, true);  // candidates had a key: in the walk
            const int ap = s_apos[lane];
            const int na = cc < ap ? cc : ap;
            const Row r = apply_commits(base, c, na, cc - na);
            int32_t sc;
            bool passed;
            (void)dyn_key(cf, c, t, nc, r, cc > 0 ? pwc : pw, n, true, na_n, &sc, &passed);
            fb_post = fit_bits(c, r, passed);
        }
        const uint32_t sweep = fit_sum(fit_raw);
        int32_t tot[4];
#pragma unroll
        for (int b = 0; b < 4; ++b)
            tot[b] = (int32_t)__builtin_amdgcn_readlane((int)sweep, b) + fit_in[b] +
                     __popcll(__ballot((fb_post >> b) & 1u)) - __popcll(__ballot((fb_base >> b) & 1u));
        if (lane == 0) {
            __hip_atomic_store(&out->fit[0], make_fit_granule(a.epoch, tot[0], tot[1]), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&out->fit[1], make_fit_granule(a.epoch, tot[2], tot[3]), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    const int ln = n - wb_base;  // local row of the written-back node
    if (n >= 0 && cc > 0 && ln >= 0 && ln < wb_n) {  // Allocate^a Pipeline^p: a = min(cc, first Pipeline depth)
        const int ap = s_apos[lane];
        const int na = cc < ap ? cc : ap;
        const Row r = apply_commits(base, c, na, cc - na);
        if constexpr (SC1) {
            st_sc1(&nc.idle_cpu[ln], r.idle_cpu); st_sc1(&nc.idle_mem[ln], r.idle_mem); st_sc1(&nc.idle_gpu[ln], r.idle_gpu);
            st_sc1(&nc.rel_cpu[ln], r.rel_cpu); st_sc1(&nc.rel_mem[ln], r.rel_mem); st_sc1(&nc.rel_gpu[ln], r.rel_gpu);
            st_sc1(&nc.pods[ln], r.pods);
            st_sc1(&nc.nzc[ln], r.nzc);
            st_sc1(&nc.nzm[ln], r.nzm);
            if (c.has_ports)
                for (int w = 0; w < nc.port_words && w < 4; ++w) st_sc1(&nc.ports[(int64_t)w * nc.npad + ln], pwc[w]);
        } else {
            nc.idle_cpu[ln] = r.idle_cpu; nc.idle_mem[ln] = r.idle_mem; nc.idle_gpu[ln] = r.idle_gpu;
            nc.rel_cpu[ln] = r.rel_cpu; nc.rel_mem[ln] = r.rel_mem; nc.rel_gpu[ln] = r.rel_gpu;
            nc.pods[ln] = r.pods;
            nc.nzc[ln] = r.nzc;
            nc.nzm[ln] = r.nzm;
            if (c.has_ports)
                for (int w = 0; w < nc.port_words && w < 4; ++w) nc.ports[(int64_t)w * nc.npad + ln] = pwc[w];
        }
    }
    if constexpr (SC1) {  // the only storing wave drained, then the flag (sc1)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) st_sc1(done_flag, seq);
    }
    if (lane < done)
        __hip_atomic_store(&out->g[lane], make_granule(a.epoch, stop, done, kind, inm ? entry_node(L, a) : -1),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    STAMP(gridDim.x * 4 + 3);
}


// ---------------------------------------------------------------------------
// Placement by insertion (option "placement" = 4): one wave, no sort
// networks.  The greedy order is the descending order of the entries
// e(j, d) = (running min of node j's scores over depths 0..d, index, depth)
// (see place_levels).  The depth-0 entries are the sorted candidate list
// itself; a node's entries decrease with depth, so the top-m entries hold a
// prefix of each node's sequence.  Rounds: every lane whose newest entry is
// still among the top m evaluates its next depth (its own row, its own
// Allocate^a Pipeline^p chain, no fix-ups); new entries above the m-th are
// inserted into the sorted list one at a time (a ballot gives the position,
// a DPP wave shift moves the tail).  A round that inserts nothing ends it —
// typically after one or two rounds, as a commit lowers a node's score.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t wave_shr1_64(uint64_t v) {  // lane i <- lane i - 1 (lane 0 <- 0)
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, 0x138, 0xf, 0xf, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v >> 32), 0x138, 0xf, 0xf, false);
    return ((uint64_t)hi << 32) | lo;
}
// L sorted descending over the lanes, e not in L: L with e inserted (the last entry drops off).
__device__ __forceinline__ uint64_t wave_insert_desc(uint64_t L, uint64_t e) {
    const int lane = threadIdx.x & 63;
    const int pos = __popcll(__ballot(L > e));
    const uint64_t sh = wave_shr1_64(L);
    return lane < pos ? L : (lane == pos ? e : sh);
}

template <bool SC1 = false>
__device__ void place_insert(const Conf& cf, const NodeCols& nc, const DevTables& t, const TaskClass& c,
                             const PopArgs& a, PopOut* out, uint64_t K, uint32_t* done_flag = nullptr,
                             uint32_t seq = 0, const RowCache* rc = nullptr, const int32_t* fit_in = nullptr,
                             uint32_t fit_raw = 0, int wb_base = 0, int wb_n = 0x7fffffff) {
    const int lane = threadIdx.x & 63;
    const int n = K ? key_idx(K) : -1;  // global node index (keys are global)
    Row base{};
    uint64_t pw[4] = {0, 0, 0, 0};
    int32_t na_n = 0;
    const int rslot = (rc && n >= 0) ? rc_find(rc, n) : -1;
    if (rslot >= 0) {
        base = rc->row[rslot];
        for (int w = 0; w < 4; ++w) pw[w] = rc->pw[rslot][w];
        na_n = rc->na[rslot];
    } else if (n >= 0) {
        base = load_row_t<SC1>(nc, n);
        if (c.has_ports)
            for (int w = 0; w < nc.port_words && w < 4; ++w) pw[w] = load_port_t<SC1>(nc, w, n);
        if (cf.score_mult) na_n = na_weight(c, t, nc, n);
    }
    uint64_t pwc[4];  // ports after one or more commits of this class
    for (int w = 0; w < 4; ++w) pwc[w] = pw[w] | ((c.has_ports && w < nc.port_words) ? t.masks[c.pown_off + w] : 0);
    const int m = a.n_tasks;
    // this lane's chain: depth d of its newest entry, commits by kind behind it, first Pipeline depth
    int d = 0, ca = 0, cp = 0, apos = 64;
    uint64_t key = K;  // key at depth d (its kind is the kind of commit d + 1)
    int32_t rm = K ? key_score(K) : 0;
    uint64_t last = K ? level_entry(rm, n, 0, K) : 0;  // newest entry
    uint64_t L = last;  // lane p: entry p of the sorted top entries (depth-0 entries are the sorted list)
    uint64_t T = readlane64(L, m - 1);
    for (int round = 1; round < 64; ++round) {
        const bool act = last != 0 && last >= T;  // its newest entry is among the top m
        if (!__ballot(act)) break;
        uint64_t e = 0;
        if (act) {
            if (key & 1) { ++cp; if (apos == 64) apos = d; } else ++ca;  // commit d + 1 takes the depth-d kind
            ++d;
            const Row r = apply_commits(base, c, ca, cp);
            int32_t s;
            bool passed;
            key = dyn_key(cf, c, t, nc, r, pwc, n, true, na_n, &s, &passed);
            if (key) {
                rm = key_score(key) < rm ? key_score(key) : rm;
                e = level_entry(rm, n, d, key);
            }
            last = e;
        }
        // insert the new entries that beat the m-th (T only rises: one below it never enters)
        for (uint64_t q = __ballot(e != 0 && e > T); q; q &= q - 1) {
            const uint64_t x = readlane64(e, __ffsll((unsigned long long)q) - 1);
            if (x > T) {
                L = wave_insert_desc(L, x);
                T = readlane64(L, m - 1);
            }
        }
    }
    // stop rule over the placement order (allocate.go:187-195, gang.go:63-66)
    const bool inm = lane < m && L != 0;
    const int kind = inm ? entry_kind(L) : 0;
    const uint64_t amask = __ballot(inm && kind == 1);  // Pipelined is not an AllocatedStatus
    const uint64_t upto = lane == 63 ? ~0ull : ((2ull << lane) - 1);
    const int ready_p = a.ready_count + __popcll(amask & upto);
    const uint64_t smask = __ballot(lane < m && (!inm || !a.gang_mode || ready_p >= a.min_avail));
    int done, stop;
    if (smask) {
        const int p = __ffsll((unsigned long long)smask) - 1;
        done = p + 1;
        stop = __builtin_amdgcn_readlane((int)inm, p) ? 2 : 1;
    } else {
        done = m;
        stop = 0;
    }
    // commits of this lane's node among the placed entries
    int cc = 0;
    for (int p = 0; p < done; ++p) {
        const uint64_t x = readlane64(L, p);
        cc += (x != 0 && entry_idx(x) == n) ? 1 : 0;
    }
    const int nal = cc < apos ? cc : apos;  // Allocate^a Pipeline^p: a = min(cc, first Pipeline depth)
    if (fit_in && stop == 1) {  // a task found no node: the walk's FitDelta histogram at that task
        uint32_t fb_base = 0, fb_post = 0;
        if (n >= 0) {
            fb_base = fit_bits(c, base, true);  // candidates had a key: in the walk
            const Row r = apply_commits(base, c, nal, cc - nal);
            int32_t sc;
            bool passed;
            (void)dyn_key(cf, c, t, nc, r, cc > 0 ? pwc : pw, n, true, na_n, &sc, &passed);
            fb_post = fit_bits(c, r, passed);
        }
        const uint32_t sweep = fit_sum(fit_raw);
        int32_t tot[4];
#pragma unroll
        for (int b = 0; b < 4; ++b)
            tot[b] = (int32_t)__builtin_amdgcn_readlane((int)sweep, b) + fit_in[b] +
                     __popcll(__ballot((fb_post >> b) & 1u)) - __popcll(__ballot((fb_base >> b) & 1u));
        if (lane == 0) {
            __hip_atomic_store(&out->fit[0], make_fit_granule(a.epoch, tot[0], tot[1]), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&out->fit[1], make_fit_granule(a.epoch, tot[2], tot[3]), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    const int ln = n - wb_base;
    if (n >= 0 && cc > 0 && ln >= 0 && ln < wb_n) {
        const Row r = apply_commits(base, c, nal, cc - nal);
        if constexpr (SC1) {
            st_sc1(&nc.idle_cpu[ln], r.idle_cpu); st_sc1(&nc.idle_mem[ln], r.idle_mem); st_sc1(&nc.idle_gpu[ln], r.idle_gpu);
            st_sc1(&nc.rel_cpu[ln], r.rel_cpu); st_sc1(&nc.rel_mem[ln], r.rel_mem); st_sc1(&nc.rel_gpu[ln], r.rel_gpu);
            st_sc1(&nc.pods[ln], r.pods);
            st_sc1(&nc.nzc[ln], r.nzc);
            st_sc1(&nc.nzm[ln], r.nzm);
            if (c.has_ports)
                for (int w = 0; w < nc.port_words && w < 4; ++w) st_sc1(&nc.ports[(int64_t)w * nc.npad + ln], pwc[w]);
        } else {
            nc.idle_cpu[ln] = r.idle_cpu; nc.idle_mem[ln] = r.idle_mem; nc.idle_gpu[ln] = r.idle_gpu;
            nc.rel_cpu[ln] = r.rel_cpu; nc.rel_mem[ln] = r.rel_mem; nc.rel_gpu[ln] = r.rel_gpu;
            nc.pods[ln] = r.pods;
            nc.nzc[ln] = r.nzc;
            nc.nzm[ln] = r.nzm;
            if (c.has_ports)
                for (int w = 0; w < nc.port_words && w < 4; ++w) nc.ports[(int64_t)w * nc.npad + ln] = pwc[w];
        }
    }
    if constexpr (SC1) {  // the only storing wave drained, then the flag (sc1)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) st_sc1(done_flag, seq);
    }
    if (lane < done)
        __hip_atomic_store(&out->g[lane], make_granule(a.epoch, stop, done, kind, inm ? entry_idx(L) : -1),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ---------------------------------------------------------------------------
// Placement of a session with Backfilled nodes (placement 6; one wave, task
// after task).  Visiting a node in a walk adds its Backfilled to its Idle
// (GetAccessibleResource, node_info.go:209-211; allocate.go:150-180): every
// node ahead of the winner in the walk order, and the winner itself, before
// its commit.  So nodes other than the winner change between the pop's tasks,
// and the entry order of the other placements does not hold.  Lane j holds
// candidate j of the sweep's list — the top 64 of the walk keys of nodes that
// fit or carry Backfilled (eval_node_walk) — with its row; per task:
//   winner  = the largest current key (fitting nodes: walk key + kind);
//   visited = lanes whose walk key is above the winner's (only nodes with
//             Backfilled change);
// exact while the winner's walk key is at least the list's last one (every
// node above it that could be visited or win is in the list; nodes outside
// do not change).  Otherwise the launch ends before that task (done < m,
// stop 0; done = 0 asks the host for the general path for one task), and a
// task that finds no node is left to the general path too (its walk covers
// every node and reports the FitDelta histogram).
// ---------------------------------------------------------------------------
__device__ void place_bf(const Conf& cf, const NodeCols& nc, const DevTables& t, const TaskClass& c,
                         const PopArgs& a, PopOut* out, uint64_t K) {
    const int lane = threadIdx.x & 63;
    const int n = K ? key_idx(K) : -1;
    Row r{};
    uint64_t pw[4] = {0, 0, 0, 0};
    int32_t na_n = 0;
    if (n >= 0) {
        r = load_row(nc, n);
        if (c.has_ports)
            for (int w = 0; w < nc.port_words && w < 4; ++w) pw[w] = nc.ports[(int64_t)w * nc.npad + n];
        if (cf.score_mult) na_n = na_weight(c, t, nc, n);
    }
    const bool has_bf = (r.bf_cpu | r.bf_mem | r.bf_gpu) != 0;
    const uint64_t t0w = readlane64(K, 63) >> 1;  // walk key of the list's last entry (0: the list holds all)
    int32_t s = 0;
    bool passed = false;
    uint64_t key = n >= 0 ? dyn_key(cf, c, t, nc, r, pw, n, true, na_n, &s, &passed) : 0;
    uint64_t wk = (n >= 0 && passed) ? pack_key(s, n, 0) >> 1 : 0;  // walk key (0: not in the walk)
    bool changed = false;
    int ready = a.ready_count, done = 0, stop = 0;
    uint64_t mine = 0;  // lane i: winner key of task i
    for (int i = 0; i < a.n_tasks; ++i) {
        const uint64_t w = wave_max_key(key);
        if (!w || (w >> 1) < t0w) break;  // no node, or one outside the list may come first: the host goes on
        if (lane == i) mine = w;
        const bool win = n >= 0 && key == w;
        const bool visit = has_bf && (win || wk > (w >> 1));
        if (visit) { r.idle_cpu += r.bf_cpu; r.idle_mem += r.bf_mem; r.idle_gpu += r.bf_gpu; }
        const int kind = key_kind(w);
        if (win) {
            r = apply_commits(r, c, kind == 1 ? 1 : 0, kind == 1 ? 0 : 1);
            if (c.has_ports)
                for (int q = 0; q < 4; ++q) pw[q] |= (q < nc.port_words) ? t.masks[c.pown_off + q] : 0;
        }
        if (visit || win) {
            changed = true;
            key = dyn_key(cf, c, t, nc, r, pw, n, true, na_n, &s, &passed);
            wk = passed ? pack_key(s, n, 0) >> 1 : 0;
        }
        done = i + 1;
        if (kind == 1) ++ready;  // Pipelined is not an AllocatedStatus (types.go:82-84)
        if (!a.gang_mode || ready >= a.min_avail) { stop = 2; break; }  // allocate.go:191-195
    }
    if (changed) {
        nc.idle_cpu[n] = r.idle_cpu; nc.idle_mem[n] = r.idle_mem; nc.idle_gpu[n] = r.idle_gpu;
        nc.rel_cpu[n] = r.rel_cpu; nc.rel_mem[n] = r.rel_mem; nc.rel_gpu[n] = r.rel_gpu;
        nc.pods[n] = r.pods;
        nc.nzc[n] = r.nzc;
        nc.nzm[n] = r.nzm;
        if (c.has_ports)
            for (int w = 0; w < nc.port_words && w < 4; ++w) nc.ports[(int64_t)w * nc.npad + n] = pw[w];
    }
    if (lane < done || (done == 0 && lane == 0))
        __hip_atomic_store(&out->g[lane],
                           make_granule(a.epoch, stop, done, mine ? key_kind(mine) : 0, mine ? key_idx(mine) : -1),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The shard epilogue of k_pop_batch (placement 3): wave 0 of the final merger
// writes this shard's top-64 with their rows and the sweep's FitDelta counts.
__device__ void shard_emit(const Conf& cf, const NodeCols& nc, const DevTables& t, const TaskClass& c, uint64_t K,
                           uint32_t fit_raw, ShardMsg* msg) {
    const int lane = threadIdx.x & 63;
    ShardCand e{};
    e.node = -1;
    if (K) {
        const int g = key_idx(K);
        const int n = g - nc.base;
        e.key = K;
        e.node = g;
        e.row = load_row(nc, n);
        if (c.has_ports)
            for (int w = 0; w < nc.port_words && w < 4; ++w) e.pw[w] = nc.ports[(int64_t)w * nc.npad + n];
        e.na = cf.score_mult ? na_weight(c, t, nc, n) : 0;
    }
    msg->c[lane] = e;
    const uint32_t sweep = fit_sum(fit_raw);
    if (lane < 4) msg->fit[lane] = sweep;
}

// PL: the placement compiled into this instantiation — 2 parallel levels,
// 5 parallel levels merged by insertion, 6 sessions with Backfilled nodes
// (walk keys, sequential placement), 3 the node-array shard's sweep only
// (no placement: the exchange follows), -1 the test-only modes 0 / 1 / 4 —
// so that a kernel's registers (and the occupancy of its sweep blocks) are
// those of one placement path.
template <int R, typename KT, int PL>
__global__ __launch_bounds__(kPopThreads) void k_pop_batch(Conf cf, NodeCols nc, DevTables t, PopArgs a,
                                                           uint64_t* cand64, uint32_t* arrive, PopOut* out,
                                                           ShardMsg* smsg) {
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
    STAMP(blockIdx.x * 4 + 0);
    const TaskClass c = t.classes[a.cls];
    if (threadIdx.x < 4) s_fitb[threadIdx.x] = 0;
    // 1. evaluate R nodes per lane, wave top-64, block top-64
    KT best = 0;
    uint32_t fbs[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int n = (blockIdx.x * R + r) * kPopThreads + threadIdx.x;
        KT k = 0;
        fbs[r] = 0;
        if (n < nc.n) {
            int32_t s;
            bool passed;
            if constexpr (PL == 6) k = sweep_key<KT>(eval_node_walk(cf, c, t, nc, n, &fbs[r]), a);
            else k = sweep_key<KT>(eval_node(cf, c, t, nc, n, &s, &passed, &fbs[r]), a);
        }
        k = wave_sort_desc(k);
        best = r == 0 ? k : wave_merge_desc(best, k);
    }
    wlk[wave][lane] = best;
    __syncthreads();
#pragma unroll
    for (int r = 0; r < R; ++r) fit_block_add(s_fitb, fbs[r]);
    STAMP(blockIdx.x * 4 + 1);
    block_tree_merge(wlk, wave, lane);
    const int nb = gridDim.x;
    const int g = blockIdx.x % kGroups;
    const int g_count = (nb - g + kGroups - 1) / kGroups;   // blocks in my group
    const int n_groups = nb < kGroups ? nb : kGroups;
    KT* gcand = cand + (int64_t)nb * 64;                     // group lists after the block lists
    if (wave == 0) {
        if (lane < 4 && s_fitb[lane])
            __hip_atomic_fetch_add(&fitc[g * kCtrStride + lane], s_fitb[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        put_list(cand + (int64_t)blockIdx.x * 64, wlk[0][lane]);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    STAMP(blockIdx.x * 4 + 2);
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
    STAMP(gridDim.x * 4 + 4);
    // 2b. last group merger: merge the group lists; reset the counters for the next launch
    {
        KT acc = 0;
        for (int gi = wave; gi < n_groups; gi += kPopThreads / 64) acc = wave_merge_desc(acc, get_list(gcand + (int64_t)gi * 64));
        wlk[wave][lane] = acc;
    }
    __syncthreads();
    block_tree_merge(wlk, wave, lane);
    STAMP(gridDim.x * 4 + 0);
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
        if (wave == 0) shard_emit(cf, nc, t, c, wl[0][lane], fit_raw, smsg);
        return;
    } else if constexpr (PL == 6) {  // Backfilled nodes in the session
        if (wave != 0) return;
        STAMP(gridDim.x * 4 + 1);
        place_bf(cf, nc, t, c, a, out, wl[0][lane]);
        STAMP(gridDim.x * 4 + 3);
        return;
    } else {
    if constexpr (PL == 2 || PL == 5) {  // every wave takes part
        STAMP(gridDim.x * 4 + 1);
        if (a.ent32) place_parallel<uint32_t, false, PL == 5>(cf, nc, t, c, a, out, wl, nullptr, 0, nullptr, s_fitin, fit_raw);
        else place_parallel<uint64_t, false, PL == 5>(cf, nc, t, c, a, out, wl, nullptr, 0, nullptr, s_fitin, fit_raw);
        return;
    } else {
    if (a.placement == 1) {  // uniform
        if (wave != 0) return;
        STAMP(gridDim.x * 4 + 1);
        place_levels(cf, nc, t, c, a, wl[0][lane], out);
        return;
    }
    if (a.placement == 4) {  // uniform
        if (wave != 0) return;
        STAMP(gridDim.x * 4 + 1);
        place_insert<false>(cf, nc, t, c, a, out, wl[0][lane], nullptr, 0, nullptr, s_fitin, fit_raw);
        STAMP(gridDim.x * 4 + 3);
        return;
    }
    // 3. placement.  Lane j owns candidate j of the sorted global top-64: node
    // n, sweep key K.  The post-commit keys of each candidate (after 1..kDepth
    // more tasks of this class, assuming every commit is an Allocate) are
    // computed by waves 0..kDepth-1 in parallel.
    __shared__ uint64_t chainbuf[kDepth][64];
    const uint64_t K = wl[0][lane];
    const int n = K ? key_idx(K) : -1;
    Row base{};
    uint64_t pw[4] = {0, 0, 0, 0};
    int32_t na_n = 0;  // static node-affinity weight of this lane's node
    if (n >= 0 && wave <= kDepth) {
        base = load_row(nc, n);
        if (c.has_ports)
            for (int w = 0; w < nc.port_words && w < 4; ++w) pw[w] = nc.ports[(int64_t)w * nc.npad + n];
        if (cf.score_mult) na_n = na_weight(c, t, nc, n);
    }
    uint64_t pwc[4];  // ports after one or more commits of this class
    for (int w = 0; w < 4; ++w) pwc[w] = pw[w] | ((c.has_ports && w < nc.port_words) ? t.masks[c.pown_off + w] : 0);
    if (wave < kDepth) {
        uint64_t v = 0;
        if (n >= 0) {
            const Row r = apply_commits(base, c, wave + 1, 0);
            int32_t s;
            bool passed;
            v = dyn_key(cf, c, t, nc, r, pwc, n, true, na_n, &s, &passed);
        }
        chainbuf[wave][lane] = v;
    }
    __syncthreads();
    if (wave != 0) return;
    STAMP(gridDim.x * 4 + 1);
    uint64_t chain[kDepth];
#pragma unroll
    for (int d = 0; d < kDepth; ++d) chain[d] = chainbuf[d][lane];
    // Winner of each task = max(first unchanged list entry, best changed entry).
    // Changed entries are always a prefix [0, first) of the list.  The hot
    // loop only reads precomputed post-commit keys; a lane whose chain is
    // exhausted (or that was pipelined) leaves the loop for a recompute.
    uint64_t val = K;       // current key of this lane's candidate
    int na = 0, np = 0;     // commits on this lane's node by kind
    int first = 0;          // uniform
    uint64_t bc_val = 0;    // uniform: best key among changed entries
    int bc_lane = -1;       // uniform
    int ready = a.ready_count, stop = -1, done = 0;
    uint64_t mine = 0;      // lane i: winner key of task i
    int i = 0;
    while (i < a.n_tasks && stop < 0) {
        int slow_lane = -1;
        for (; i < a.n_tasks; ++i) {
            const uint64_t cu = first < 64 ? ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(K >> 32), first) << 32 |
                                              (uint32_t)__builtin_amdgcn_readlane((int)K, first))
                                           : 0;
            uint64_t w;
            int wl;
            if (cu > bc_val) { w = cu; wl = first; ++first; }
            else { w = bc_val; wl = bc_lane; }
            done = i + 1;
            if (!w) { stop = 1; break; }
            if (lane == i) mine = w;
            const int kind = key_kind(w);
            bool fast = true;
            if (lane == wl) {
                if (kind == 1) ++na; else ++np;
                const int cc = na + np;
                fast = np == 0 && cc <= kDepth;
                uint64_t x = chain[0];
#pragma unroll
                for (int d = 1; d < kDepth; ++d) if (cc == d + 1) x = chain[d];
                if (fast) val = x;
            }
            if (kind == 1) ++ready;  // Pipelined is not an AllocatedStatus (types.go:82-84)
            if (!a.gang_mode || ready >= a.min_avail) stop = 2;  // allocate.go:191-195
            else if (i + 1 == a.n_tasks) stop = 0;
            if (!__builtin_amdgcn_readlane((int)fast, wl)) { slow_lane = wl; ++i; break; }
            const uint64_t nv = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(val >> 32), wl) << 32 |
                                (uint32_t)__builtin_amdgcn_readlane((int)val, wl);
            if (wl == bc_lane) {  // the best changed node changed again: rescan the changed prefix
                bc_val = wave_max_key(lane < first ? val : 0);
                const uint64_t m = __ballot(lane < first && val == bc_val && bc_val != 0);
                bc_lane = m ? __ffsll((unsigned long long)m) - 1 : -1;
            } else if (nv > bc_val) {
                bc_val = nv;
                bc_lane = wl;
            }
            if (stop >= 0) { ++i; break; }
        }
        if (slow_lane < 0) break;
        // rare: re-evaluate the winner's node after its latest commit
        if (lane == slow_lane) {
            const Row r = apply_commits(base, c, na, np);
            int32_t s;
            bool passed;
            val = dyn_key(cf, c, t, nc, r, pwc, n, true, na_n, &s, &passed);
        }
        const uint64_t nv = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(val >> 32), slow_lane) << 32 |
                            (uint32_t)__builtin_amdgcn_readlane((int)val, slow_lane);
        if (slow_lane == bc_lane) {
            bc_val = wave_max_key(lane < first ? val : 0);
            const uint64_t m = __ballot(lane < first && val == bc_val && bc_val != 0);
            bc_lane = m ? __ffsll((unsigned long long)m) - 1 : -1;
        } else if (nv > bc_val) {
            bc_val = nv;
            bc_lane = slow_lane;
        }
    }
    STAMP(gridDim.x * 4 + 2);
    // 4. write back committed rows and the results
    if (na + np > 0) {
        const Row r = apply_commits(base, c, na, np);
        nc.idle_cpu[n] = r.idle_cpu; nc.idle_mem[n] = r.idle_mem; nc.idle_gpu[n] = r.idle_gpu;
        nc.rel_cpu[n] = r.rel_cpu; nc.rel_mem[n] = r.rel_mem; nc.rel_gpu[n] = r.rel_gpu;
        nc.pods[n] = r.pods;
        nc.nzc[n] = r.nzc;
        nc.nzm[n] = r.nzm;
        if (c.has_ports)
            for (int w = 0; w < nc.port_words && w < 4; ++w) nc.ports[(int64_t)w * nc.npad + n] = pwc[w];
    }
    if (lane < done)
        __hip_atomic_store(&out->g[lane],
                           make_granule(a.epoch, stop, done, mine ? key_kind(mine) : 0, mine ? key_idx(mine) : -1),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    STAMP(gridDim.x * 4 + 3);
    }  // placement 0
    }  // PL != 3
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
template <typename KT>
__device__ __forceinline__ int key_node(KT k, const PopArgs& a) {
    if constexpr (sizeof(KT) == 8) return key_idx(k);
    else return a.kidxmax - (int)((k >> 1) & (uint32_t)a.kidxmax);
}

constexpr long kLinkSpin = 1L << 21;  // poll bound (~1 s): a broken chain ends the pop with an error

// INS: the placement merges each round by insertion (placement 5) instead of
// sort + merge trees (placement 2); one placement per instantiation keeps the
// kernel's registers (and so the occupancy of its sweep blocks) at one path's.
template <int R, typename KT, bool INS>
__global__ __launch_bounds__(kPopThreads) void k_pop_batch_ov(Conf cf, NodeCols nc, DevTables t, PopArgs a,
                                                              uint64_t* cand64, uint32_t* arrive, PopOut* out,
                                                              PopLink* link, uint32_t seq, int ndep) {
    __shared__ KT wlk[kPopThreads / 64][64];               // sweep / merge lists in the key type
    __shared__ uint64_t wl[kPopThreads / 64][64];          // placement lists (64-bit keys / entries)
    __shared__ uint32_t s_skip[R * kPopThreads / 32];      // this block's nodes among pop seq-1's candidates
    __shared__ int role, s_ok;
    __shared__ uint32_t s_fitb[4];
    __shared__ int32_t s_fitin[4];
    uint32_t* fitc = fit_counters(arrive, a.fit_set);
    fit_zero_other(arrive, a.fit_set);
    KT* cand = (KT*)cand64;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    STAMP(blockIdx.x * 4 + 0);
    const TaskClass c = t.classes[a.cls];
    const int base = blockIdx.x * R * kPopThreads;
    // the ndep pops before this one may still be writing rows: seq-1 .. seq-ndep
    uint64_t tv[kMaxDep] = {};
#pragma unroll
    for (int k = 0; k < kMaxDep; ++k)  // in flight while the rows below load
        if (wave == 0 && k < ndep && seq > (uint32_t)(k + 1))
            tv[k] = ld_sc1(&link->touched[(seq - 1 - k) % kLinkSlots][lane]);
    for (int i = threadIdx.x; i < R * kPopThreads / 32; i += kPopThreads) s_skip[i] = 0;
    if (threadIdx.x < 4) s_fitb[threadIdx.x] = 0;
    // 1. evaluate R nodes per lane, then leave pop seq-1's candidates out
    KT keys[R];
    uint32_t fbs[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int n = (blockIdx.x * R + r) * kPopThreads + threadIdx.x;
        keys[r] = 0;
        fbs[r] = 0;
        if (n < nc.n) {
            int32_t s;
            bool passed;
            keys[r] = sweep_key<KT>(eval_node(cf, c, t, nc, n, &s, &passed, &fbs[r]), a);
        }
    }
    __syncthreads();  // s_skip zeroed
    int tn[kMaxDep];  // wave 0: candidate `lane` of pop seq-1-k (-1: none)
    if (wave == 0) {
        bool ok = true;
#pragma unroll
        for (int k = 0; k < kMaxDep; ++k) {
            tn[k] = -1;
            if (k >= ndep || seq <= (uint32_t)(k + 1)) continue;
            const uint32_t want = seq - 1 - k;
            long spin = 0;
            while (ok && __ballot((uint32_t)(tv[k] >> 32) != want) != 0) {  // re-read every granule
                if (++spin >= kLinkSpin) ok = false;
                __builtin_amdgcn_s_sleep(2);
                tv[k] = ld_sc1(&link->touched[want % kLinkSlots][lane]);
            }
            const int x = ok ? (int)(uint32_t)tv[k] : -1;
            tn[k] = x;
            if (x >= base && x < base + R * kPopThreads) atomicOr(&s_skip[(x - base) >> 5], 1u << ((x - base) & 31));
        }
        if (lane == 0) s_ok = ok;
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
    const int nb = gridDim.x;
    const int g = blockIdx.x % kGroups;
    const int g_count = (nb - g + kGroups - 1) / kGroups;
    const int n_groups = nb < kGroups ? nb : kGroups;
    KT* gcand = cand + (int64_t)nb * 64;
    if (wave == 0) {
        if (lane < 4 && s_fitb[lane])
            __hip_atomic_fetch_add(&fitc[g * kCtrStride + lane], s_fitb[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        put_list(cand + (int64_t)blockIdx.x * 64, wlk[0][lane]);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    STAMP(blockIdx.x * 4 + 2);
    if (threadIdx.x == 0) role = atomicAdd(&arrive[g * kCtrStride], 1u) == (unsigned)(g_count - 1);
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
        if (threadIdx.x == 0) role = atomicAdd(&arrive[kGroups * kCtrStride], 1u) == (unsigned)(n_groups - 1);
        __syncthreads();
        if (!role) return;
    }
    // 2b. last group merger: the top-64 of every node but the previous pops' candidates
    STAMP(gridDim.x * 4 + 4);
    {
        KT acc = 0;
        for (int gi = wave; gi < n_groups; gi += kPopThreads / 64) acc = wave_merge_desc(acc, get_list(gcand + (int64_t)gi * 64));
        wlk[wave][lane] = acc;
    }
    __syncthreads();
    block_tree_merge(wlk, wave, lane);
    STAMP(gridDim.x * 4 + 0);
    if (wave == 0 && lane <= kGroups)
        __hip_atomic_store(&arrive[lane * kCtrStride], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // the sweep's FitDelta counts (every block added before it arrived), left in flight
    const uint32_t fit_raw = wave == 0 ? fit_load(fitc, n_groups) : 0u;
    if (wave == 0 && lane < 4) s_fitin[lane] = 0;  // + the counts of nodes the sweep left out
    // 3. while pop seq-1 may still write back: the rows of this list's nodes
    // (final: no pop in flight touches them) and the static parts of pop
    // seq-1's candidates, into the row cache
    __shared__ RowCache rc;
    int32_t pna = 0;  // wave 0: pop seq-1's candidate `lane`: node-affinity weight, static predicates
    bool pst = false;
    if (wave == 0) {
        for (int h = lane; h < kHash; h += 64) rc.hkey[h] = -1;
        const KT lk = wlk[0][lane];
        const int ln = lk ? key_node(lk, a) : -1;
        if (ln >= 0) {
            rc.row[lane] = load_row(nc, ln);
            for (int w = 0; w < 4; ++w) rc.pw[lane][w] = (c.has_ports && w < nc.port_words) ? load_port_t<false>(nc, w, ln) : 0;
            rc.na[lane] = cf.score_mult ? na_weight(c, t, nc, ln) : 0;
        }
        if (tn[0] >= 0) {
            pst = static_pred(cf, c, t, nc, tn[0]);
            pna = (pst && cf.score_mult) ? na_weight(c, t, nc, tn[0]) : 0;
        }
        __builtin_amdgcn_wave_barrier();
        if (ln >= 0) rc_insert(&rc, ln, lane);
    }
    // pop seq-1's write-back, which follows seq-2's ... (relaxed sc1 poll;
    // every load of their rows below is sc1); their candidates on final rows
    if (threadIdx.x == 0) {
        bool ok = s_ok;
        long spin = 0;
        while (ok && (int32_t)(ld_sc1(&link->done) - (seq - 1)) < 0) {
            if (++spin >= kLinkSpin) ok = false;
            __builtin_amdgcn_s_sleep(2);
        }
        s_ok = ok;
    }
    __syncthreads();
    STAMP(gridDim.x * 4 + 10);
    const bool ok = s_ok;
    if (wave == 0) {
        KT e0 = 0;
        uint32_t fb_prev = 0;  // FitDelta bits of the previous pops' candidates (left out of the sweep)
        if (ok && tn[0] >= 0) {  // pop seq-1's candidates: rows into the cache, keys
            const Row r = load_row_sc1(nc, tn[0]);
            uint64_t pw[4] = {0, 0, 0, 0};
            if (c.has_ports)
                for (int w = 0; w < nc.port_words && w < 4; ++w) pw[w] = load_port_t<true>(nc, w, tn[0]);
            rc.row[64 + lane] = r;
            for (int w = 0; w < 4; ++w) rc.pw[64 + lane][w] = pw[w];
            rc.na[64 + lane] = pna;
            rc_insert(&rc, tn[0], 64 + lane);
            int32_t sc;
            bool passed;
            e0 = sweep_key<KT>(dyn_key(cf, c, t, nc, r, pw, tn[0], pst, pna, &sc, &passed), a);
            fb_prev = fit_bits(c, r, passed);
        }
        KT top = wave_merge_desc(wlk[0][lane], wave_sort_desc(e0));  // all 64 lanes: cross-lane networks
#pragma unroll
        for (int k = 1; k < kMaxDep; ++k) {  // older pops (overlap > 1): not cached
            if (k >= ndep) break;
            bool dup = false;  // a node among several pops' candidates counts once
#pragma unroll
            for (int j = 0; j < k; ++j)
                for (uint64_t mm = __ballot(tn[j] >= 0); mm; mm &= mm - 1)
                    dup = dup || tn[k] == __builtin_amdgcn_readlane(tn[j], __ffsll((unsigned long long)mm) - 1);
            uint32_t fbk = 0;
            const KT e = (ok && tn[k] >= 0 && !dup) ? sweep_key<KT>(eval_node_sc1(cf, c, t, nc, tn[k], &fbk), a)
                                                     : (KT)0;
            top = wave_merge_desc(top, wave_sort_desc(e));
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int cnt = __popcll(__ballot((fbk >> b) & 1u));
                if (lane == b) s_fitin[b] += cnt;
            }
        }
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const int cnt = __popcll(__ballot((fb_prev >> b) & 1u));
            if (lane == b) s_fitin[b] += cnt;
        }
        // this pop's candidates, one self-tagged granule each
        st_sc1(&link->touched[seq % kLinkSlots][lane],
               ((uint64_t)seq << 32) | (uint32_t)((ok && top) ? key_node(top, a) : -1));
        wl[0][lane] = ok ? key64_of(top, a) : 0;
    }
    __syncthreads();
    STAMP(gridDim.x * 4 + 1);
    if (ok) {
        if (a.ent32) place_parallel<uint32_t, true, INS>(cf, nc, t, c, a, out, wl, &link->done, seq, &rc, s_fitin, fit_raw);
        else place_parallel<uint64_t, true, INS>(cf, nc, t, c, a, out, wl, &link->done, seq, &rc, s_fitin, fit_raw);
    } else if (wave == 0 && lane == 0) {  // broken chain: keep the chain going, n_done = 0 tells the host
        st_sc1(&link->done, seq);
        __hip_atomic_store(&out->g[0], make_granule(a.epoch, 0, 0, 0, -1), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// ---------------------------------------------------------------------------
// launchers (host)
// ---------------------------------------------------------------------------
hipError_t launch_sweep_argmax(const Conf& cf, const NodeCols& nc, const DevTables& t, PopCtrl* ctrl, int task_i,
                               uint64_t* walk, hipStream_t st, bool commit_here, uint64_t* dbg, bool defer_visits) {
    int grid = (nc.n + kBlock - 1) / kBlock;
    if (grid > 2048) grid = 2048;
    if (grid < 1) grid = 1;
    const int mode = commit_here ? (defer_visits ? 3 : 1) : 0;
    hipLaunchKernelGGL(k_sweep_argmax, dim3(grid), dim3(kBlock), 0, st, cf, nc, t, ctrl, task_i, walk, mode, dbg);
    if (commit_here && defer_visits)
        hipLaunchKernelGGL(k_visit_mutate, dim3(grid), dim3(kBlock), 0, st, nc, (const PopCtrl*)ctrl, task_i,
                           (const uint64_t*)walk);
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
__global__ __launch_bounds__(64) void k_undo_pop(NodeCols nc, DevTables t, UndoArgs u) {
    if (threadIdx.x != 0) return;
    const TaskClass c = t.classes[u.cls];
    for (int i = 0; i < u.n; ++i)
        if (u.node[i] - nc.base >= 0 && u.node[i] - nc.base < nc.n)  // this shard's rows only
            uncommit_node(c, t, nc, u.node[i] - nc.base, u.kind[i]);
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
    for (int i = 0; i < u.n; ++i)
        if (u.node[i] - nc.base >= 0 && u.node[i] - nc.base < nc.n)
            commit_node(c, t, nc, u.node[i] - nc.base, u.kind[i]);
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
// walk's GetAccessibleResource visits already applied): chosen < 0 — the task
// found no node, every walk node counts; else the walk stopped at node
// `chosen` with kind chosen_kind: the walk nodes before it count (walk order
// = key order without the fit bit), and `chosen` itself when Pipelined.
// Classes without pod-affinity terms.  out4 is zeroed by the caller.
__global__ __launch_bounds__(kBlock) void k_fit_delta(Conf cf, NodeCols nc, DevTables t, int cls, int chosen,
                                                      int chosen_kind, int32_t* out4) {
    __shared__ int32_t s_fit[4];
    if (threadIdx.x < 4) s_fit[threadIdx.x] = 0;
    __syncthreads();
    const TaskClass c = t.classes[cls];
    uint64_t wk = 0;  // walk-order key of the chosen node
    if (chosen >= 0) {
        int32_t s = 0;
        bool passed = false;
        (void)eval_node(cf, c, t, nc, chosen - nc.base, &s, &passed);
        wk = pack_key(s, chosen, 0);
    }
    for (int n = blockIdx.x * kBlock + threadIdx.x; n < nc.n; n += gridDim.x * kBlock) {
        int32_t s = 0;
        bool passed = false;
        (void)eval_node(cf, c, t, nc, n, &s, &passed);
        Row r = load_row(nc, n);
        r.bf_cpu = r.bf_mem = r.bf_gpu = 0;  // Idle as the walk left it
        const bool in = passed && (chosen < 0 || pack_key(s, n + nc.base, 0) > wk ||
                                   (n + nc.base == chosen && chosen_kind == 2));
        const uint32_t fb = in ? fit_bits(c, r, true) : 0u;
        for (int b = 0; b < 4; ++b)
            if ((fb >> b) & 1u) atomicAdd(&s_fit[b], 1);
    }
    __syncthreads();
    if (threadIdx.x < 4 && s_fit[threadIdx.x]) atomicAdd(&out4[threadIdx.x], s_fit[threadIdx.x]);
}

hipError_t launch_fit_delta(const Conf& cf, const NodeCols& nc, const DevTables& t, int cls, int chosen,
                            int chosen_kind, int32_t* out4, hipStream_t st) {
    const int grid = (nc.n + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(k_fit_delta, dim3(grid > 0 ? grid : 1), dim3(kBlock), 0, st, cf, nc, t, cls, chosen,
                       chosen_kind, out4);
    return hipGetLastError();
}

hipError_t launch_commit_task(const NodeCols& nc, const DevTables& t, PopCtrl* ctrl, int task_i, const uint64_t* walk,
                              hipStream_t st) {
    hipLaunchKernelGGL(k_commit_task, dim3(1), dim3(kBlock), 0, st, nc, t, ctrl, task_i, walk);
    return hipGetLastError();
}

hipError_t launch_ipa_minmax(const NodeCols& nc, const DevTables& t, PopCtrl* ctrl, int task_i, hipStream_t st) {
    int grid = (nc.n + kBlock - 1) / kBlock;
    if (grid > 2048) grid = 2048;
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL(k_ipa_minmax, dim3(grid), dim3(kBlock), 0, st, nc, t, ctrl, task_i);
    return hipGetLastError();
}

int pop_blocks(int n_nodes, int* R_out) {
    static const int forced = [] {  // KBHIP_POP_R: nodes per lane (tuning experiments only)
        const char* e = std::getenv("KBHIP_POP_R");
        return e ? std::atoi(e) : 0;
    }();
    int R = 1;
    while ((int64_t)kPopThreads * R * 512 < n_nodes && R < 16) R <<= 1;
    if (forced == 1 || forced == 2 || forced == 4 || forced == 8 || forced == 16) R = forced;
    *R_out = R;
    return (n_nodes + kPopThreads * R - 1) / (kPopThreads * R);
}

template <typename KT>
static void launch_pop_batch_t(int R, int nb, const Conf& cf, const NodeCols& nc, const DevTables& t, const PopArgs& a,
                               uint64_t* cand, uint32_t* arrive, PopOut* o, ShardMsg* m, hipStream_t st) {
#define KBHIP_PB1(RR, PP) \
    hipLaunchKernelGGL((k_pop_batch<RR, KT, PP>), dim3(nb), dim3(kPopThreads), 0, st, cf, nc, t, a, cand, arrive, o, m)
#define KBHIP_PB(RR)                                                   \
    do {                                                               \
        switch (a.placement) {                                         \
            case 2: KBHIP_PB1(RR, 2); break;                           \
            case 3: KBHIP_PB1(RR, 3); break;                           \
            case 5: KBHIP_PB1(RR, 5); break;                           \
            case 6: KBHIP_PB1(RR, 6); break;                           \
            default: KBHIP_PB1(RR, -1); break;                         \
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

hipError_t launch_pop_batch(const Conf& cf, const NodeCols& nc, const DevTables& t, int cls, int n_tasks,
                            int gang_mode, int min_avail, int ready_count, uint32_t epoch, uint64_t* cand,
                            uint32_t* arrive, void* out_dev, hipStream_t st, int placement, const KeyFormat& kf,
                            int fit_set, ShardMsg* shard_out) {
    if (placement == 3 && !shard_out) return hipErrorInvalidValue;
    int R;
    const int nb = pop_blocks(nc.n, &R);
    PopArgs a{cls, n_tasks, gang_mode, min_avail, ready_count, epoch, placement, kf.base, kf.shift, kf.idxmax,
              kf.use32 && kf.ent32 ? 1 : 0, fit_set};
    PopOut* o = (PopOut*)out_dev;
    if (kf.use32) launch_pop_batch_t<uint32_t>(R, nb, cf, nc, t, a, cand, arrive, o, shard_out, st);
    else launch_pop_batch_t<uint64_t>(R, nb, cf, nc, t, a, cand, arrive, o, shard_out, st);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Node-array shards, batched pops: after the all-gather of
// every shard's ShardMsg, each shard runs this identical placement on the
// merged list — the global top-64, since every shard's list holds its own
// top-64 — and writes back the rows it owns.  One workgroup.
// ---------------------------------------------------------------------------
constexpr int kShardHash = 2048;  // node -> (rank, slot) of the gathered candidates (<= 16 ranks x 64)
__global__ __launch_bounds__(kPopThreads) void k_shard_place(Conf cf, NodeCols nc, DevTables t, PopArgs a,
                                                             const ShardMsg* msgs, int world, PopOut* out) {
    __shared__ uint64_t wl[kPopThreads / 64][64];
    __shared__ RowCache rc;
    __shared__ int32_t s_hk[kShardHash];
    __shared__ int16_t s_hv[kShardHash];
    __shared__ int32_t s_fitin[4];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const TaskClass c = t.classes[a.cls];
    for (int i = threadIdx.x; i < kShardHash; i += kPopThreads) s_hk[i] = -1;
    for (int i = threadIdx.x; i < kHash; i += kPopThreads) rc.hkey[i] = -1;
    if (threadIdx.x < 4) {
        uint32_t f = 0;
        for (int r = 0; r < world; ++r) f += msgs[r].fit[threadIdx.x];
        s_fitin[threadIdx.x] = (int32_t)f;
    }
    __syncthreads();
    // every gathered candidate into the node -> entry table; lists merged by waves
    uint64_t acc = 0;
    for (int r = wave; r < world; r += kPopThreads / 64) {
        const ShardCand& e = msgs[r].c[lane];
        if (e.node >= 0) {
            int h = (int)(((uint32_t)e.node * 2654435761u) >> 21);
            while (atomicCAS(&s_hk[h], -1, e.node) != -1) h = (h + 1) & (kShardHash - 1);
            s_hv[h] = (int16_t)(r * 64 + lane);
        }
        acc = wave_merge_desc(acc, e.key);
    }
    wl[wave][lane] = acc;
    __syncthreads();
    block_tree_merge(wl, wave, lane);  // wl[0]: the global top-64 keys
    if (wave == 0) {  // their rows into the row cache (slot = lane)
        const uint64_t K = wl[0][lane];
        if (K) {
            const int g = key_idx(K);
            int h = (int)(((uint32_t)g * 2654435761u) >> 21);
            while (s_hk[h] != g) h = (h + 1) & (kShardHash - 1);
            const int src = s_hv[h];
            const ShardCand& e = msgs[src >> 6].c[src & 63];
            rc.row[lane] = e.row;
            for (int w = 0; w < 4; ++w) rc.pw[lane][w] = e.pw[w];
            rc.na[lane] = e.na;
            rc_insert(&rc, g, lane);
        }
    }
    __syncthreads();
    NodeCols ncg = nc;  // keys / entries carry global node indices
    ncg.base = 0;
    if (a.placement == 4) {
        if (wave == 0) place_insert<false>(cf, ncg, t, c, a, out, wl[0][lane], nullptr, 0, &rc, s_fitin, 0u, nc.base, nc.n);
    } else if (a.placement == 5) {
        if (a.ent32) place_parallel<uint32_t, false, true>(cf, ncg, t, c, a, out, wl, nullptr, 0, &rc, s_fitin, 0u, nc.base, nc.n);
        else place_parallel<uint64_t, false, true>(cf, ncg, t, c, a, out, wl, nullptr, 0, &rc, s_fitin, 0u, nc.base, nc.n);
    } else if (a.ent32) place_parallel<uint32_t>(cf, ncg, t, c, a, out, wl, nullptr, 0, &rc, s_fitin, 0u, nc.base, nc.n);
    else place_parallel<uint64_t>(cf, ncg, t, c, a, out, wl, nullptr, 0, &rc, s_fitin, 0u, nc.base, nc.n);
}

hipError_t launch_shard_place(const Conf& cf, const NodeCols& nc, const DevTables& t, int cls, int n_tasks,
                              int gang_mode, int min_avail, int ready_count, uint32_t epoch, const KeyFormat& kf,
                              const ShardMsg* msgs, int world, void* out_dev, hipStream_t st, int placement) {
    if (world < 1 || world * 64 > kShardHash / 2) return hipErrorInvalidValue;
    PopArgs a{cls, n_tasks, gang_mode, min_avail, ready_count, epoch, (placement == 4 || placement == 5) ? placement : 2,
              kf.base, kf.shift, kf.idxmax,
              kf.use32 && kf.ent32 ? 1 : 0, 0};
    hipLaunchKernelGGL(k_shard_place, dim3(1), dim3(kPopThreads), 0, st, cf, nc, t, a, msgs, world, (PopOut*)out_dev);
    return hipGetLastError();
}

template <typename KT, bool INS>
static void launch_pop_batch_ov_t(int R, int nb, const Conf& cf, const NodeCols& nc, const DevTables& t,
                                  const PopArgs& a, uint64_t* cand, uint32_t* arrive, PopOut* o, PopLink* link,
                                  uint32_t seq, int ndep, hipStream_t st) {
#define KBHIP_OV(RR)                                                                                              \
    hipLaunchKernelGGL((k_pop_batch_ov<RR, KT, INS>), dim3(nb), dim3(kPopThreads), 0, st, cf, nc, t, a, cand, arrive, \
                       o, link, seq, ndep)
    switch (R) {
        case 1: KBHIP_OV(1); break;
        case 2: KBHIP_OV(2); break;
        case 4: KBHIP_OV(4); break;
        case 8: KBHIP_OV(8); break;
        default: KBHIP_OV(16); break;
    }
#undef KBHIP_OV
}

hipError_t launch_pop_batch_ov(const Conf& cf, const NodeCols& nc, const DevTables& t, int cls, int n_tasks,
                               int gang_mode, int min_avail, int ready_count, uint32_t epoch, uint64_t* cand,
                               uint32_t* arrive, void* out_dev, hipStream_t st, const KeyFormat& kf, PopLink* link,
                               uint32_t seq, int ndep, int fit_set, int placement) {
    if (ndep < 1 || ndep > kMaxDep) return hipErrorInvalidValue;
    int R;
    const int nb = pop_blocks(nc.n, &R);
    const bool ins = placement == 5;
    PopArgs a{cls, n_tasks, gang_mode, min_avail, ready_count, epoch, ins ? 5 : 2, kf.base, kf.shift, kf.idxmax,
              kf.use32 && kf.ent32 ? 1 : 0, fit_set};
    PopOut* o = (PopOut*)out_dev;
    if (kf.use32) {
        if (ins) launch_pop_batch_ov_t<uint32_t, true>(R, nb, cf, nc, t, a, cand, arrive, o, link, seq, ndep, st);
        else launch_pop_batch_ov_t<uint32_t, false>(R, nb, cf, nc, t, a, cand, arrive, o, link, seq, ndep, st);
    } else {
        if (ins) launch_pop_batch_ov_t<uint64_t, true>(R, nb, cf, nc, t, a, cand, arrive, o, link, seq, ndep, st);
        else launch_pop_batch_ov_t<uint64_t, false>(R, nb, cf, nc, t, a, cand, arrive, o, link, seq, ndep, st);
    }
    return hipGetLastError();
}

size_t pop_out_bytes() { return sizeof(PopOut); }

#ifdef KBHIP_STAMPS
hipError_t set_stamp_buffer(uint64_t* p) { return hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &p, sizeof(p)); }
#endif

}  // namespace kbhip
