// Reclaim / preempt node ranking on gfx950.
//
// Both actions walk the nodes for one preemptor task in a fixed order and stop
// at the first node whose victims cover the request:
//   preempt  (actions/preempt/preempt.go:270-288): nodes passing PredicateFn
//            with a NodeOrderFn score, in util.SelectBestNode order (score
//            descending, then the pinned node order);
//   reclaim  (actions/reclaim/reclaim.go:115-119): nodes passing PredicateFn,
//            in the pinned node order.
// The victim choice itself (tier-intersected Preemptable / Reclaimable over the
// node's tasks) is per-node host logic on the host model.  The device produces
// the order: one HBM sweep writes a key per node — pack_key(score, idx) for
// preempt (descending = SelectBestNode order), pack_key(0, idx) for reclaim —
// zero for a node that fails; a stable counting sort over the class's small
// score range orders them (launch_rank_sorted; classes whose score range
// exceeds 256 values: four stable 8-bit counting passes over the score,
// launch_rank_radix), and the host reads the passing prefix back.  Traffic per task: the columns
// PredicateFn + NodeOrderFn read — 41 B per node (flags, acpu / amem / nzc / nzm, pods, maxtasks;
// no Idle / Releasing / Backfilled column: the compiler drops the fit loads, whose result the
// sweep does not use) + 8 B written per node + the sort's passes over 8 B keys.
#include <hip/hip_runtime.h>

#include "kbhip_eval.h"
#include "kbhip_internal.h"

namespace kbhip {

__global__ __launch_bounds__(kBlock) void k_rank_nodes(Conf cf, NodeCols nc, DevTables t, const PopCtrl* ctrl,
                                                       int by_score, uint64_t* keys, uint32_t* count) {
    __shared__ uint32_t s_cnt;
    if (threadIdx.x == 0) s_cnt = 0;
    __syncthreads();
    const int cls = __builtin_amdgcn_readfirstlane(ctrl->cls[0]);
    const TaskClass c = t.classes[cls];
    const int64_t ilo = ctrl->ipa_lo[0], ihi = ctrl->ipa_hi[0];
    const int F = ctrl->fallback;
    uint32_t cnt = 0;
    for (int n = blockIdx.x * kBlock + threadIdx.x; n < nc.n; n += gridDim.x * kBlock) {
        uint64_t k;
        if (by_score) {
            int32_t s = 0;
            bool passed = false;
            (void)eval_node_aff(cf, c, t, nc, n, ilo, ihi, F, &s, &passed);
            k = passed ? pack_key(s, n + nc.base, 0) : 0;
        } else {
            k = eval_first_fit(cf, c, t, nc, n);
        }
        keys[n] = k;
        cnt += k != 0;
    }
    // wave sum, then one LDS atomic per wave and one global atomic per block
    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
    if ((threadIdx.x & 63) == 0 && cnt) atomicAdd(&s_cnt, cnt);
    __syncthreads();
    if (threadIdx.x == 0 && s_cnt) atomicAdd(count, s_cnt);
}

// The standalone predicate + score sweep of one task (kbhip_sweep_scores:
// preempt.go:270-287's PredicateFn + NodeOrderFn over every node): per node
// pack_key(score, index) when it passes, 0 otherwise; the passing count in
// kGroups counters on separate lines, block b adding to counter b % kGroups
// (one device-scope counter taking an add from every block serialises the
// tail of the launch: MI355X_MICROARCH.md fanin).  PLAIN: a class without pod
// (anti-)affinity or inter-pod terms (eval_node: the row loads are issued
// before the predicates' early exits); otherwise eval_node_aff.
constexpr int kSweepGroups = 8;
// TB threads per block, NPT nodes per thread (node = block base + r * TB + thread:
// every load instruction of a wave stays coalesced); all of a thread's row loads
// are issued before its first evaluation.
template <bool PLAIN, int TB, int NPT>
__global__ __launch_bounds__(TB) void k_score_sweep(Conf cf, NodeCols nc, DevTables t, TaskClass c,
                                                    const PopCtrl* ctrl, uint64_t* keys, uint32_t* counts) {
    __shared__ uint32_t s_cnt;
    if (threadIdx.x == 0) s_cnt = 0;
    const int n0 = blockIdx.x * TB * NPT + threadIdx.x;
    uint32_t cnt = 0;
    if constexpr (PLAIN && NPT > 1) {
        Row r[NPT];
        uint8_t fl[NPT];
#pragma unroll
        for (int q = 0; q < NPT; ++q) {
            const int n = n0 + q * TB;
            if (n < nc.n) { fl[q] = nc.flags[n]; r[q] = load_row(nc, n); }
        }
#pragma unroll
        for (int q = 0; q < NPT; ++q) {
            const int n = n0 + q * TB;
            bool passed = false;
            if (n < nc.n) {
                uint64_t pw[4] = {0, 0, 0, 0};
                if (c.has_ports)
                    for (int w = 0; w < 4; ++w) if (w < port_win(c, nc)) pw[w] = nc.ports[port_at(c, nc, w, n)];
                const bool st = static_pred_f(cf, c, t, nc, n, fl[q]);
                const int32_t na = (st && cf.score_mult) ? na_weight(c, t, nc, n) : 0;
                int32_t s = 0;
                (void)dyn_key(cf, c, t, nc, r[q], pw, n, st, na, &s, &passed);
                keys[n] = passed ? pack_key(s, n + nc.base, 0) : 0;
            }
            cnt += (uint32_t)__popcll(__ballot(passed));
        }
    } else {
#pragma unroll
        for (int q = 0; q < NPT; ++q) {
            const int n = n0 + q * TB;
            bool passed = false;
            if (n < nc.n) {
                int32_t s = 0;
                if constexpr (PLAIN) (void)eval_node(cf, c, t, nc, n, &s, &passed);
                else (void)eval_node_aff(cf, c, t, nc, n, ctrl->ipa_lo[0], ctrl->ipa_hi[0], ctrl->fallback, &s, &passed);
                keys[n] = passed ? pack_key(s, n + nc.base, 0) : 0;
            }
            cnt += (uint32_t)__popcll(__ballot(passed));
        }
    }
    __syncthreads();  // s_cnt zeroed
    if ((threadIdx.x & 63) == 0 && cnt) atomicAdd(&s_cnt, cnt);
    __syncthreads();
    if (threadIdx.x == 0 && s_cnt) atomicAdd(&counts[(blockIdx.x % kSweepGroups) * 32], s_cnt);
}

// The same sweep for a plain class over a grid of a few blocks per CU: each
// thread walks nodes n, n + stride, ... and loads the next node's columns
// before it evaluates the current one, so a wave's loads overlap its own
// arithmetic (the one-node-per-thread grid issues every wave's loads, then
// every wave's evaluation).  Only the columns the keys depend on are read:
// flags, acpu / amem / nzc / nzm, pods, maxtasks (41 B per node; the fit
// columns are not part of PredicateFn + NodeOrderFn) plus the class's port
// words when it has host ports.
struct SweepIn {
    int64_t acpu, amem, nzc, nzm;
    int32_t pods, maxtasks;
    uint8_t fl;
};
__device__ __forceinline__ SweepIn sweep_in(const NodeCols& nc, int n) {
    SweepIn v;
    v.acpu = nc.acpu[n]; v.amem = nc.amem[n]; v.nzc = nc.nzc[n]; v.nzm = nc.nzm[n];
    v.pods = nc.pods[n]; v.maxtasks = nc.maxtasks[n]; v.fl = nc.flags[n];
    return v;
}
template <int TB>
__global__ __launch_bounds__(TB) void k_score_sweep_gs(Conf cf, NodeCols nc, DevTables t, TaskClass c,
                                                       uint64_t* keys, uint32_t* counts) {
    __shared__ uint32_t s_cnt;
    if (threadIdx.x == 0) s_cnt = 0;
    const int stride = gridDim.x * TB;
    int n = blockIdx.x * TB + threadIdx.x;
    uint32_t cnt = 0;
    SweepIn cur{};
    if (n < nc.n) cur = sweep_in(nc, n);
    for (; n < nc.n; n += stride) {
        SweepIn nxt{};
        if (n + stride < nc.n) nxt = sweep_in(nc, n + stride);
        uint64_t pw[4] = {0, 0, 0, 0};
        if (c.has_ports)
            for (int w = 0; w < 4; ++w) if (w < port_win(c, nc)) pw[w] = nc.ports[port_at(c, nc, w, n)];
        Row r{};
        r.acpu = cur.acpu; r.amem = cur.amem; r.nzc = cur.nzc; r.nzm = cur.nzm;
        r.pods = cur.pods; r.maxtasks = cur.maxtasks;
        const bool st = static_pred_f(cf, c, t, nc, n, cur.fl);
        const int32_t na = (st && cf.score_mult) ? na_weight(c, t, nc, n) : 0;
        int32_t s = 0;
        bool passed = false;
        (void)dyn_key(cf, c, t, nc, r, pw, n, st, na, &s, &passed);  // passed and s read no fit column
        keys[n] = passed ? pack_key(s, n + nc.base, 0) : 0;
        cnt += passed;
        cur = nxt;
    }
    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
    __syncthreads();  // s_cnt zeroed
    if ((threadIdx.x & 63) == 0 && cnt) atomicAdd(&s_cnt, cnt);
    __syncthreads();
    if (threadIdx.x == 0 && s_cnt) atomicAdd(&counts[(blockIdx.x % kSweepGroups) * 32], s_cnt);
}

static int cu_count() {
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
    }
    return cus;
}

// Cache eviction by reading (kbhip_time_sweeps, option time_sweeps_cold = 2):
// every 16-byte word of the buffer loaded, one word written only if the xor
// hits a value it never takes (the loads stay live).
__global__ __launch_bounds__(256) void k_evict_read(const uint4* p, size_t n16, uint32_t* sink) {
    uint32_t x = 0;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) {
        const uint4 v = p[i];
        x ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (x == 0x9e3779b9u && sink) sink[0] = x;
}
hipError_t launch_evict_read(const void* buf, size_t bytes, hipStream_t st) {
    hipLaunchKernelGGL(k_evict_read, dim3(cu_count() * 8), dim3(256), 0, st, (const uint4*)buf, bytes / 16,
                       (uint32_t*)nullptr);
    return hipGetLastError();
}

// variant (option "sweep_variant", a tuning knob): 0 = 256 threads x 1 node,
// 1 = 512 x 1, 2 = 256 x 2, 3 = 256 x 4; 4 / 5 / 6 = the prefetching grid
// (k_score_sweep_gs) with 8 / 4 / 16 blocks of 256 per CU
static int g_sweep_variant = 0;
void set_sweep_variant(int v) { g_sweep_variant = v; }
template <int TB, int NPT>
static void launch_sweep_t(const Conf& cf, const NodeCols& nc, const DevTables& t, const TaskClass& c,
                           const PopCtrl* ctrl, uint64_t* keys, uint32_t* counts, hipStream_t st) {
    const int per = TB * NPT;
    const int grid = nc.n > 0 ? (nc.n + per - 1) / per : 1;
    if (!c.aff && c.ipa_n == 0)
        hipLaunchKernelGGL((k_score_sweep<true, TB, NPT>), dim3(grid), dim3(TB), 0, st, cf, nc, t, c, ctrl, keys, counts);
    else
        hipLaunchKernelGGL((k_score_sweep<false, TB, NPT>), dim3(grid), dim3(TB), 0, st, cf, nc, t, c, ctrl, keys,
                           counts);
}
hipError_t launch_score_sweep(const Conf& cf, const NodeCols& nc, const DevTables& t, const TaskClass& c,
                              const PopCtrl* ctrl, uint64_t* keys, uint32_t* counts, hipStream_t st) {
    if (g_sweep_variant >= 4 && g_sweep_variant <= 6 && !c.aff && c.ipa_n == 0) {
        const int per_cu = g_sweep_variant == 4 ? 8 : g_sweep_variant == 5 ? 4 : 16;
        const int need = nc.n > 0 ? (nc.n + 255) / 256 : 1;
        const int grid = need < cu_count() * per_cu ? need : cu_count() * per_cu;
        hipLaunchKernelGGL((k_score_sweep_gs<256>), dim3(grid), dim3(256), 0, st, cf, nc, t, c, keys, counts);
        return hipGetLastError();
    }
    switch (g_sweep_variant) {
        case 1: launch_sweep_t<512, 1>(cf, nc, t, c, ctrl, keys, counts, st); break;
        case 2: launch_sweep_t<256, 2>(cf, nc, t, c, ctrl, keys, counts, st); break;
        case 3: launch_sweep_t<256, 4>(cf, nc, t, c, ctrl, keys, counts, st); break;
        default: launch_sweep_t<256, 1>(cf, nc, t, c, ctrl, keys, counts, st); break;
    }
    return hipGetLastError();
}

// One node-row update of a reclaim / preempt operation, in one lane:
//   op 0 evict       NodeInfo.UpdateTask Running -> Releasing: Releasing += Resreq
//                    (node_info.go:147-185; Idle / Used / Backfilled net unchanged)
//   op 1 pipeline    NodeInfo.AddTask Pipelined (commit_node, kind 2)
//   op 2 unpipeline  NodeInfo.RemoveTask of the Pipelined copy (uncommit_node, kind 2)
// n: this shard's row of global node g, or -1 (another shard's node: the
// replicated count tables only).
__global__ __launch_bounds__(64) void k_node_op(NodeCols nc, DevTables t, int op, int n, int g, int cls, int64_t rc,
                                                int64_t rm, int64_t rg) {
    if (threadIdx.x != 0) return;
    if (op == 0) {
        if (n >= 0) { nc.rel_cpu[n] += rc; nc.rel_mem[n] += rm; nc.rel_gpu[n] += rg; }
    } else if (op == 1) {
        const TaskClass c = t.classes[cls];
        if (n >= 0) commit_node(c, t, nc, n, 2);
        if (c.aff) commit_aff(c, t, nc, g, 2);  // a session-placed pod (inter-pod priority)
    } else {
        const TaskClass c = t.classes[cls];
        if (n >= 0) uncommit_node(c, t, nc, n, 2);
        if (c.aff) uncommit_aff(c, t, nc, g, 2);
    }
}

// Count-table changes queued on the host (evictions / unevicts of predicate
// targets, session/03_pop.cpp flush_tables): idx >= 0 -> aff_cnt[idx],
// idx < 0 -> aff_scalar[-1 - idx]; the indices are distinct.
__global__ __launch_bounds__(kBlock) void k_tab_add(DevTables t, const int32_t* idx, const int32_t* delta, int n) {
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const int32_t x = idx[i];
    if (x >= 0) t.aff_cnt[x] += delta[i];
    else t.aff_scalar[-1 - x] += delta[i];
}

hipError_t launch_tab_add(const DevTables& t, const int32_t* idx, const int32_t* delta, int n, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_tab_add, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, st, t, idx, delta, n);
    return hipGetLastError();
}

// Accumulated evictions (op 0 of k_node_op, summed per node on the host):
// Releasing += d[3 i .. 3 i + 2] on node[i]; the nodes are distinct.
__global__ __launch_bounds__(kBlock) void k_rel_add(NodeCols nc, const int32_t* node, const int64_t* d, int n) {
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const int v = node[i];
    nc.rel_cpu[v] += d[3 * i]; nc.rel_mem[v] += d[3 * i + 1]; nc.rel_gpu[v] += d[3 * i + 2];
}

hipError_t launch_rel_add(const NodeCols& nc, const int32_t* node, const int64_t* d, int n, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_rel_add, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, st, nc, node, d, n);
    return hipGetLastError();
}

// Carry-over's node rows (kbhip_session_carry_snapshot): every element that differs
// from the read-back device rows, packed on the host, written in one launch
// (instead of one copy per run of differing rows).
__global__ __launch_bounds__(kBlock) void k_row_patch(const RowPatch* e, int n) {
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const RowPatch p = e[i];
    if (p.size == 8) *reinterpret_cast<uint64_t*>(p.addr) = p.val;
    else if (p.size == 4) *reinterpret_cast<uint32_t*>(p.addr) = (uint32_t)p.val;
    else *reinterpret_cast<uint8_t*>(p.addr) = (uint8_t)p.val;
}

hipError_t launch_row_patch(const RowPatch* e, int n, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_row_patch, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, st, e, n);
    return hipGetLastError();
}

hipError_t launch_rank_nodes(const Conf& cf, const NodeCols& nc, const DevTables& t, const PopCtrl* ctrl,
                             int by_score, uint64_t* keys, uint32_t* count, hipStream_t st) {
    int grid = (nc.n + kBlock - 1) / kBlock;
    if (grid > 2048) grid = 2048;
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL(k_rank_nodes, dim3(grid), dim3(kBlock), 0, st, cf, nc, t, ctrl, by_score, keys, count);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Wide score ranges: an LSD radix sort of the passing nodes' keys by their
// score, 8 bits per pass from the lowest, digits taken descending; every
// pass is a stable counting sort (per-block digit counts, one scan, a
// scatter that keeps the order within a block by wave ballots), so ties in
// score keep the node order of the first pass's input (index ascending): the
// result is the descending key order, as util.SelectBestNode walks it.
// Pass 0 reads k_rank_nodes' keys (0 = failing node, dropped), later passes
// the previous pass's output (count[0] entries).
// ---------------------------------------------------------------------------
__device__ __forceinline__ int radix_digit(uint64_t k, int shift) {  // 0 = best (highest score digit)
    return 255 - (int)(((uint32_t)(k >> 32) >> shift) & 255u);
}
__global__ __launch_bounds__(kBlock) void k_radix_bucket(const uint64_t* in, int n_in, const uint32_t* count,
                                                         int shift, uint32_t* hist, int nblk) {
    __shared__ uint32_t s_h[256];
    for (int i = threadIdx.x; i < 256; i += kBlock) s_h[i] = 0;
    __syncthreads();
    const int n = count ? (int)count[0] : n_in;
    const int i = blockIdx.x * kBlock + threadIdx.x;
    const uint64_t k = i < n ? in[i] : 0;
    if (k) atomicAdd(&s_h[radix_digit(k, shift)], 1u);
    __syncthreads();
    for (int b = threadIdx.x; b < 256; b += kBlock) hist[(size_t)b * nblk + blockIdx.x] = s_h[b];
}
__global__ __launch_bounds__(kBlock) void k_radix_scatter(const uint64_t* in, int n_in, const uint32_t* count,
                                                          int shift, const uint32_t* offs, int nblk, uint64_t* out) {
    __shared__ uint32_t s_cnt[kBlock / 64][256];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int i = lane; i < 256; i += 64) s_cnt[wave][i] = 0;
    const int n = count ? (int)count[0] : n_in;
    const int i = blockIdx.x * kBlock + threadIdx.x;
    const uint64_t k = i < n ? in[i] : 0;
    const int b = k ? radix_digit(k, shift) : -1;
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    uint32_t rank = 0;
    __builtin_amdgcn_wave_barrier();
    for (uint64_t todo = __ballot(b >= 0); todo;) {
        const int bv = __builtin_amdgcn_readlane(b, __ffsll((unsigned long long)todo) - 1);
        const uint64_t m = __ballot(b == bv);
        if (b == bv) rank = __popcll(m & lt);
        if (lane == 0) s_cnt[wave][bv] = __popcll(m);
        todo &= ~m;
    }
    __syncthreads();
    if (b >= 0) {
        uint32_t base = offs[(size_t)b * nblk + blockIdx.x];
        for (int w = 0; w < wave; ++w) base += s_cnt[w][b];
        out[base + rank] = k;
    }
}
__global__ __launch_bounds__(1024) void k_rank_scan(uint32_t* v, int n);

hipError_t launch_rank_radix(const uint64_t* keys, int n, const uint32_t* count, uint32_t* hist, uint64_t* tmp,
                             uint64_t* sorted, hipStream_t st) {
    const int nblk = (n + kBlock - 1) / kBlock;
    if (nblk < 1) return hipSuccess;
    // pass 0: keys -> sorted, 1: sorted -> tmp, 2: tmp -> sorted, 3: sorted -> tmp ... ending in sorted
    const uint64_t* in = keys;
    uint64_t* bufs[2] = {tmp, sorted};
    for (int p = 0; p < 4; ++p) {
        uint64_t* out = bufs[(p + 1) & 1];
        const uint32_t* cnt = p == 0 ? nullptr : count;  // pass 0 drops the failing nodes' zero keys
        hipLaunchKernelGGL(k_radix_bucket, dim3(nblk), dim3(kBlock), 0, st, in, n, cnt, 8 * p, hist, nblk);
        hipLaunchKernelGGL(k_rank_scan, dim3(1), dim3(1024), 0, st, hist, 256 * nblk);
        hipLaunchKernelGGL(k_radix_scatter, dim3(nblk), dim3(kBlock), 0, st, in, n, cnt, 8 * p, (const uint32_t*)hist,
                           nblk, out);
        in = out;
    }
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// The walk order by a stable counting sort over the score (hand-written; the
// score range of a class is small: <= kRankBuckets values).  Order wanted:
// score descending, then node index ascending (= the descending key order).
//   k_rank_bucket   one node per thread, blocks over contiguous node ranges:
//                   key, bucket = shi - score (0 = best), per-block bucket
//                   counts -> hist[bucket * nblk + block], passing count
//   k_rank_scan     exclusive scan of hist in (bucket, block) order -> offsets
//   k_rank_scatter  position = offset + rank among the same bucket before it in
//                   the block (wave ballots, then earlier waves' counts)
// ---------------------------------------------------------------------------
constexpr int kRankBuckets = 256;
// blk / nblk: this block's node range and the number of blocks of the ranking
__device__ __forceinline__ void rank_bucket(const Conf& cf, const NodeCols& nc, const DevTables& t, const TaskClass& c,
                                            const PopCtrl* ctrl, int by_score, int shi, int nb, uint64_t* keys,
                                            uint32_t* hist, uint32_t* count, int blk, int nblk) {
    __shared__ uint32_t s_h[kRankBuckets];
    const int n = blk * kBlock + threadIdx.x;
    // a plain class's columns (SweepIn) are loaded first: their latency runs
    // under the histogram's zeroing and the predicates' table reads
    const bool plain = by_score && !c.aff && c.ipa_n == 0;
    SweepIn pre{};
    if (plain && n < nc.n) pre = sweep_in(nc, n);
    for (int i = threadIdx.x; i < nb; i += kBlock) s_h[i] = 0;
    uint64_t k = 0;
    if (n < nc.n) {
        if (plain) {
            uint64_t pw[4] = {0, 0, 0, 0};
            if (c.has_ports)
                for (int w = 0; w < 4; ++w) if (w < port_win(c, nc)) pw[w] = nc.ports[port_at(c, nc, w, n)];
            Row r{};
            r.acpu = pre.acpu; r.amem = pre.amem; r.nzc = pre.nzc; r.nzm = pre.nzm;
            r.pods = pre.pods; r.maxtasks = pre.maxtasks;
            const bool st = static_pred_f(cf, c, t, nc, n, pre.fl);
            const int32_t na = (st && cf.score_mult) ? na_weight(c, t, nc, n) : 0;
            int32_t s = 0;
            bool passed = false;
            (void)dyn_key(cf, c, t, nc, r, pw, n, st, na, &s, &passed);  // passed and s read no fit column
            k = passed ? pack_key(s, n + nc.base, 0) : 0;
        } else if (by_score) {
            int32_t s = 0;
            bool passed = false;
            (void)eval_node_aff(cf, c, t, nc, n, ctrl->ipa_lo[0], ctrl->ipa_hi[0], ctrl->fallback, &s, &passed);
            k = passed ? pack_key(s, n + nc.base, 0) : 0;
        } else {
            k = eval_first_fit(cf, c, t, nc, n);
        }
        const int b = k ? (by_score ? shi - key_score(k) : 0) : -1;
        if (b >= nb) {  // outside the class's score range: never sorted; the host fails loudly on count[1]
            atomicAdd(&count[1], 1u);
            k = 0;
        }
        keys[n] = k;
    }
    __syncthreads();  // s_h zeroed
    // the histogram: one LDS add per distinct bucket of the wave (a class's
    // nodes fall into few score buckets: one add per node serialised up to
    // 64 adds on one LDS word)
    {
        const int bb = k ? (by_score ? shi - key_score(k) : 0) : -1;
        for (uint64_t todo = __ballot(bb >= 0); todo;) {
            const int bv = __builtin_amdgcn_readlane(bb, __ffsll((unsigned long long)todo) - 1);
            const uint64_t m = __ballot(bb == bv);
            if ((threadIdx.x & 63) == 0) atomicAdd(&s_h[bv], (uint32_t)__popcll(m));
            todo &= ~m;
        }
    }
    __syncthreads();
    uint32_t tot = 0;
    for (int i = threadIdx.x; i < nb; i += kBlock) {
        hist[(size_t)i * nblk + blk] = s_h[i];
        tot += s_h[i];
    }
    for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o, 64);
    if ((threadIdx.x & 63) == 0 && tot) atomicAdd(count, tot);
}

__device__ __forceinline__ void rank_scan(uint32_t* v, int n) {  // in-place exclusive scan, one 1024-thread block
    __shared__ uint32_t s_sum[1024];
    const int per = (n + 1023) / 1024, lo = threadIdx.x * per, hi = lo + per < n ? lo + per : n;
    uint32_t acc = 0;
    for (int i = lo; i < hi; ++i) acc += v[i];
    s_sum[threadIdx.x] = acc;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {  // Hillis-Steele inclusive scan of the chunk sums
        const uint32_t x = threadIdx.x >= (unsigned)o ? s_sum[threadIdx.x - o] : 0u;
        __syncthreads();
        s_sum[threadIdx.x] += x;
        __syncthreads();
    }
    uint32_t run = threadIdx.x ? s_sum[threadIdx.x - 1] : 0u;
    for (int i = lo; i < hi; ++i) {
        const uint32_t x = v[i];
        v[i] = run;
        run += x;
    }
}

__device__ __forceinline__ void rank_scatter(const NodeCols& nc, const uint64_t* keys, const uint32_t* offs,
                                             int by_score, int shi, uint64_t* sorted, int blk, int nblk) {
    __shared__ uint32_t s_cnt[kBlock / 64][kRankBuckets];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int i = lane; i < kRankBuckets; i += 64) s_cnt[wave][i] = 0;
    const int n = blk * kBlock + threadIdx.x;
    const uint64_t k = n < nc.n ? keys[n] : 0;
    const int b = k ? (by_score ? shi - key_score(k) : 0) : -1;  // rank_bucket zeroed keys outside [0, nb)
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;  // lanes below this one
    uint32_t rank = 0;
    __builtin_amdgcn_wave_barrier();
    for (uint64_t todo = __ballot(b >= 0); todo;) {  // each bucket present in the wave
        const int bv = __builtin_amdgcn_readlane(b, __ffsll((unsigned long long)todo) - 1);
        const uint64_t m = __ballot(b == bv);
        if (b == bv) rank = __popcll(m & lt);
        if (lane == 0) s_cnt[wave][bv] = __popcll(m);
        todo &= ~m;
    }
    __syncthreads();
    if (b >= 0) {
        uint32_t base = offs[(size_t)b * nblk + blk];
        for (int w = 0; w < wave; ++w) base += s_cnt[w][b];
        sorted[base + rank] = k;
    }
}

__global__ __launch_bounds__(kBlock) void k_rank_bucket(Conf cf, NodeCols nc, DevTables t, TaskClass c,
                                                        const PopCtrl* ctrl, int by_score, int shi, int nb,
                                                        uint64_t* keys, uint32_t* hist, uint32_t* count) {
    rank_bucket(cf, nc, t, c, ctrl, by_score, shi, nb, keys, hist, count, blockIdx.x, gridDim.x);
}
__global__ __launch_bounds__(1024) void k_rank_scan(uint32_t* v, int n) { rank_scan(v, n); }
__global__ __launch_bounds__(kBlock) void k_rank_scatter(const NodeCols nc, const uint64_t* keys, const uint32_t* offs,
                                                         int by_score, int shi, int nb, uint64_t* sorted) {
    (void)nb;
    rank_scatter(nc, keys, offs, by_score, shi, sorted, blockIdx.x, gridDim.x);
}

hipError_t launch_rank_sorted(const Conf& cf, const NodeCols& nc, const DevTables& t, const TaskClass& c,
                              const PopCtrl* ctrl, int by_score, int slo, int shi, uint64_t* keys, uint32_t* hist,
                              uint64_t* sorted, uint32_t* count, hipStream_t st) {
    const int nb = by_score ? shi - slo + 1 : 1;
    if (nb < 1 || nb > kRankBuckets) return hipErrorInvalidValue;
    const int nblk = (nc.n + kBlock - 1) / kBlock;
    if (nblk < 1) return hipSuccess;
    hipLaunchKernelGGL(k_rank_bucket, dim3(nblk), dim3(kBlock), 0, st, cf, nc, t, c, ctrl, by_score, shi, nb, keys,
                       hist, count);
    hipLaunchKernelGGL(k_rank_scan, dim3(1), dim3(1024), 0, st, hist, nb * nblk);
    hipLaunchKernelGGL(k_rank_scatter, dim3(nblk), dim3(kBlock), 0, st, nc, (const uint64_t*)keys,
                       (const uint32_t*)hist, by_score, shi, nb, sorted);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// The same for a batch of what-if sessions:
// one launch of each kernel ranks the nodes of every session in the batch —
// blockIdx.y is the session, its descriptor (RankDesc) says where its node
// rows, tables, request and outputs are.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_rank_bucket_multi(const RankDesc* d) {
    const RankDesc& q = d[blockIdx.y];
    if ((int)blockIdx.x >= q.nblk) return;  // uniform
    rank_bucket(q.cf, q.nc, q.t, q.c, q.ctrl, q.by_score, q.shi, q.nb, q.keys, q.hist, q.count, blockIdx.x, q.nblk);
}
__global__ __launch_bounds__(1024) void k_rank_scan_multi(const RankDesc* d) {
    const RankDesc& q = d[blockIdx.x];
    rank_scan(q.hist, q.nb * q.nblk);
}
__global__ __launch_bounds__(kBlock) void k_rank_scatter_multi(const RankDesc* d) {
    const RankDesc& q = d[blockIdx.y];
    if ((int)blockIdx.x >= q.nblk) return;
    rank_scatter(q.nc, q.keys, q.hist, q.by_score, q.shi, q.sorted, blockIdx.x, q.nblk);
}

hipError_t fill_rank_desc(RankDesc* q, const Conf& cf, const NodeCols& nc, const DevTables& t, const TaskClass& c,
                          const PopCtrl* ctrl, int by_score, int slo, int shi, uint64_t* keys, uint32_t* hist,
                          uint64_t* sorted, uint32_t* count) {
    const int nb = by_score ? shi - slo + 1 : 1;
    if (nb < 1 || nb > kRankBuckets) return hipErrorInvalidValue;
    *q = RankDesc{cf, nc, t, c, ctrl, by_score ? 1 : 0, shi, nb, (nc.n + kBlock - 1) / kBlock, keys, hist, sorted,
                  count};
    return hipSuccess;
}

hipError_t launch_rank_sorted_multi(const RankDesc* d_desc, int n_desc, int max_nblk, hipStream_t st) {
    if (n_desc < 1 || max_nblk < 1) return hipSuccess;
    hipLaunchKernelGGL(k_rank_bucket_multi, dim3(max_nblk, n_desc), dim3(kBlock), 0, st, d_desc);
    hipLaunchKernelGGL(k_rank_scan_multi, dim3(n_desc), dim3(1024), 0, st, d_desc);
    hipLaunchKernelGGL(k_rank_scatter_multi, dim3(max_nblk, n_desc), dim3(kBlock), 0, st, d_desc);
    return hipGetLastError();
}
size_t rank_hist_words(int n_nodes) { return (size_t)kRankBuckets * ((n_nodes + kBlock - 1) / kBlock + 1); }

hipError_t launch_node_op(const NodeCols& nc, const DevTables& t, int op, int n, int g, int cls, int64_t rc,
                          int64_t rm, int64_t rg, hipStream_t st) {
    if (n >= nc.n || g < 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_node_op, dim3(1), dim3(64), 0, st, nc, t, op, n, g, cls, rc, rm, rg);
    return hipGetLastError();
}

}  // namespace kbhip
