// kbhip_batch.h — device building blocks of the batched placement path
// (kbhip_kernels.hip): wave exchange / sort / merge networks, selection keys,
// the placements (parallel levels, Backfilled nodes, pod-affinity classes,
// node-array shards), the result granules and the row cache.
#pragma once
#include <hip/hip_runtime.h>

#include "kbhip_eval.h"
#include "kbhip_internal.h"

namespace kbhip {

#if defined(KBHIP_STAMPS) && !defined(KBHIP_STAMPS_OFF)
// Diagnostic build only: phase stamps (s_memrealtime, 100 MHz) of k_pop_batch.
// Layout: [block][0..3] = start, after sweep+wave sort, after block merge, after arrival;
// [nb*4 + 0..7] = last block: merged, chain precomputed, placement done, end.
static __device__ uint64_t* g_stamps;
#define STAMP(slot)                                                       \
    do {                                                                  \
        if (threadIdx.x == 0) g_stamps[(slot)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define STAMP(slot) do {} while (0)
#endif

#ifdef KBHIP_TIMELINE
// Diagnostic build only: steady-state timeline of the overlapped pops at full
// speed (s_memrealtime, 100 MHz).  TL: one writer per event, kTlSlots pops x
// kTlEvents words by sequence number.  TLB: per-block events of every 64th
// pop (kTlbSamples x kTlbBlocks x 8 words after the TL area) — plain stores
// to a block's own slots, no atomics on shared words (those perturbed the
// timing they measured).
constexpr int kTlSlots = 32768, kTlEvents = 32;
constexpr int kTlbSamples = 512, kTlbBlocks = 256;
static __constant__ uint64_t* g_tl;  // scalar-loaded: no vector-memory wait per event
#define TL(seq, ev)                                                                             \
    do {                                                                                        \
        if (g_tl) g_tl[((seq) % kTlSlots) * kTlEvents + (ev)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#define TL_VAL(seq, ev, v) do { if (g_tl) g_tl[((seq) % kTlSlots) * kTlEvents + (ev)] = (v); } while (0)
#define TLB(seq, ev)                                                                            \
    do {                                                                                        \
        if (g_tl && ((seq) & 63) == 0 && blockIdx.x < kTlbBlocks)                               \
            g_tl[(size_t)kTlSlots * kTlEvents +                                                 \
                 ((size_t)(((seq) >> 6) % kTlbSamples) * kTlbBlocks + blockIdx.x) * 8 + (ev)] =  \
                __builtin_amdgcn_s_memrealtime();                                               \
    } while (0)
#else
#define TL(seq, ev) do {} while (0)
#define TL_VAL(seq, ev, v) do {} while (0)
#define TLB(seq, ev) do {} while (0)
#endif

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
// A bitonic 64-sequence sorted descending (half-cleaners at 32 .. 1).
template <typename T>
__device__ __forceinline__ T bitonic_clean_desc(T v) {
    v = half_clean_desc<32>(v);
    v = half_clean_desc<16>(v);
    v = half_clean_desc<8>(v);
    v = half_clean_desc<4>(v);
    v = half_clean_desc<2>(v);
    return half_clean_desc<1>(v);
}
template <typename T>
__device__ __forceinline__ T wave_merge_desc(T a, T b) {
    const T br = reverse_lanes(b);
    return bitonic_clean_desc(a > br ? a : br);  // bitonic, holds the top 64 of a U b
}
// Top 128 of two descending 128-lists held as (ranks 0..63, ranks 64..127):
// c[i] = max(a[i], b[127 - i]) is bitonic and holds them; one exchange at
// distance 64, then each half is cleaned.
template <typename T>
__device__ __forceinline__ void wave_merge128_desc(T& a0, T& a1, T b0, T b1) {
    const T r1 = reverse_lanes(b1), r0 = reverse_lanes(b0);
    const T c0 = a0 > r1 ? a0 : r1, c1 = a1 > r0 ? a1 : r0;
    a0 = bitonic_clean_desc(c0 > c1 ? c0 : c1);
    a1 = bitonic_clean_desc(c0 > c1 ? c1 : c0);
}
// Top 256 of two descending 256-lists (a[k] holds ranks 64k .. 64k + 63):
// c[i] = max(a[i], b[255 - i]) is bitonic; half-cleaners at distances 128
// and 64 (between registers), then each register is cleaned.
template <typename T>
__device__ __forceinline__ void wave_merge256_desc(T* a, const T* b) {
    T c[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const T r = reverse_lanes(b[3 - k]);
        c[k] = a[k] > r ? a[k] : r;
    }
    const T x0 = c[0] > c[2] ? c[0] : c[2], x2 = c[0] > c[2] ? c[2] : c[0];
    const T x1 = c[1] > c[3] ? c[1] : c[3], x3 = c[1] > c[3] ? c[3] : c[1];
    a[0] = bitonic_clean_desc(x0 > x1 ? x0 : x1);
    a[1] = bitonic_clean_desc(x0 > x1 ? x1 : x0);
    a[2] = bitonic_clean_desc(x2 > x3 ? x2 : x3);
    a[3] = bitonic_clean_desc(x2 > x3 ? x3 : x2);
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
    int32_t placement;  // 2 parallel levels, 3 node-array shard sweep, 6 Backfilled nodes, 7 pod-affinity class
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
// The node index of a selection key.
template <typename KT>
__device__ __forceinline__ int key_node(KT k, const PopArgs& a) {
    if constexpr (sizeof(KT) == 8) return key_idx(k);
    else return a.kidxmax - (int)((k >> 1) & (uint32_t)a.kidxmax);
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
        for (int w = 0; w < 4; ++w) if (w < port_win(c, nc)) pw[w] = load_port_t<true>(nc, c.pw_lo + w, n);
    int32_t s;
    bool passed;
    const uint64_t k = dyn_key(cf, c, t, nc, r, pw, n, st, na, &s, &passed);
    if (fit) *fit = fit_bits(c, r, passed);
    return k;
}

// A candidate's row as kRowWords self-tagged 32-bit halves (PopLink::rows):
// idle, releasing (cpu, mem, gpu), allocatable cpu / mem, nonzero requests
// cpu / mem (two halves each), pod count, MaxTaskNum.  Backfilled is 0 in
// every session whose pops overlap.
__device__ __forceinline__ void row_words(const Row& r, uint32_t* w) {
    const int64_t v[10] = {r.idle_cpu, r.idle_mem, r.idle_gpu, r.rel_cpu, r.rel_mem, r.rel_gpu,
                           r.acpu, r.amem, r.nzc, r.nzm};
#pragma unroll
    for (int i = 0; i < 10; ++i) { w[2 * i] = (uint32_t)v[i]; w[2 * i + 1] = (uint32_t)((uint64_t)v[i] >> 32); }
    w[20] = (uint32_t)r.pods;
    w[21] = (uint32_t)r.maxtasks;
}
__device__ __forceinline__ Row words_row(const uint32_t* w) {
    auto v = [&](int i) { return (int64_t)(((uint64_t)w[2 * i + 1] << 32) | w[2 * i]); };
    Row r;
    r.idle_cpu = v(0); r.idle_mem = v(1); r.idle_gpu = v(2);
    r.rel_cpu = v(3); r.rel_mem = v(4); r.rel_gpu = v(5);
    r.bf_cpu = r.bf_mem = r.bf_gpu = 0;
    r.acpu = v(6); r.amem = v(7); r.nzc = v(8); r.nzm = v(9);
    r.pods = (int32_t)w[20];
    r.maxtasks = (int32_t)w[21];
    return r;
}

__device__ __forceinline__ int entry_idx(uint64_t e) { return kEntryIdxMax - (int)((e >> 7) & kEntryIdxMax); }
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

// Tree merge of the 8 per-wave sorted lists in wl[] into the block's sorted
// top 128: ranks 0..63 in wl[0], 64..127 in wl2[0] (all waves call).
template <typename T>
__device__ __forceinline__ void block_tree_merge128(T (*wl)[64], T (*wl2)[64], int wave, int lane) {
    if (wave < kPopThreads / 128) {  // two 64-lists -> one sorted 128-list
        const T a = wl[wave][lane], b = reverse_lanes(wl[wave + kPopThreads / 128][lane]);
        wl[wave][lane] = bitonic_clean_desc(a > b ? a : b);
        wl2[wave][lane] = bitonic_clean_desc(a > b ? b : a);
    }
    __syncthreads();
#pragma unroll
    for (int s = kPopThreads / 256; s >= 1; s >>= 1) {
        if (wave < s) {
            T a0 = wl[wave][lane], a1 = wl2[wave][lane];
            wave_merge128_desc(a0, a1, wl[wave + s][lane], wl2[wave + s][lane]);
            wl[wave][lane] = a0;
            wl2[wave][lane] = a1;
        }
        __syncthreads();
    }
}

// Tree merge of the 8 per-wave lists in wl[] into wl[0] (all waves call).
template <typename T>
__device__ __forceinline__ void block_tree_merge(T (*wl)[64], int wave, int lane) {
#pragma unroll
    for (int s = kPopThreads / 128; s >= 1; s >>= 1) {
        if (wave < s) wl[wave][lane] = wave_merge_desc(wl[wave][lane], wl[wave + s][lane]);
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// Placement by parallel levels.  The greedy of a chunk picks, task after
// task, the node with the largest current key; only the winner's key changes.
// Give candidate j the entries e(j, d) for its d-th extra commit: (running
// minimum of its scores over depths 0..d, index, d, real kind).  The greedy's
// choice sequence equals the entries sorted descending: a node whose key
// RISES after a commit is picked again at once (every other current key is
// below its previous one), which the running minimum keeps in place; between
// nodes, equal scores go to the lower index as in pack_key
// (tests/test_gpu_placement_levels.py checks the argument exhaustively on
// CPU).  A round computes 8 depths at once — wave w evaluates candidate j
// after d = 8r + w commits of this class — then one sort + tree merge of the
// round's 512 entries.  Commit kinds along a chain are
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
// Running-minimum score of a placement entry.
template <typename ET>
__device__ __forceinline__ int32_t entry_rm(ET e, const PopArgs& a) {
    if constexpr (sizeof(ET) == 8) return (int32_t)((uint32_t)(e >> 32) ^ 0x80000000u);
    else return (int32_t)(e >> (a.kshift + 5)) - 1 + a.kbase;
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
// RowCache (k_pop_batch_ov, k_shard_place): slots 0..63 the sweep's list,
// 64..127 pop seq-1's candidates, 128..191 pop seq-2's (overlap depth 2).
// The persistent engine (kbhip_engine.hip) keeps four pops' candidates.
template <int S, int HB>  // S slots, 2^HB hash entries
struct RowCacheT {
    static constexpr int kSlots = S, kHashN = 1 << HB;
    Row row[S];
    uint64_t pw[S][4];
    int32_t na[S];
    int32_t s1[S];  // score after one more commit (depth-1 key; INT32_MIN: infeasible)
    int32_t hkey[1 << HB];
    int32_t hslot[1 << HB];
};
constexpr int kRcSlots = 192, kRcHash = 512;
using RowCache = RowCacheT<kRcSlots, 9>;
template <typename RC>
__device__ __forceinline__ int rc_slot(int n) {
    constexpr int hb = RC::kHashN == 512 ? 9 : RC::kHashN == 1024 ? 10 : RC::kHashN == 2048 ? 11 : 8;
    static_assert((1 << hb) == RC::kHashN, "row-cache hash size");
    return (int)(((uint32_t)n * 2654435761u) >> (32 - hb));
}
// Score of candidate n after one more commit of class c (Allocate unless its
// key is a Pipeline), INT32_MIN when that key is infeasible: the placement's
// fast-path test (place_parallel), computed where the row is loaded.
__device__ __forceinline__ int32_t depth1_score(const Conf& cf, const NodeCols& nc, const DevTables& t,
                                                const TaskClass& c, const Row& r, const uint64_t* pw, int n,
                                                int32_t na_n, uint64_t k0) {
    const int na = key_kind(k0) == 2 ? 0 : 1;
    const Row r1 = apply_commits(r, c, na, 1 - na);
    uint64_t pwc[4];
    for (int w = 0; w < 4; ++w) pwc[w] = pw[w] | ((c.has_ports && w < port_win(c, nc)) ? t.masks[c.pown_off + w] : 0);
    int32_t s1;
    bool passed1;
    const uint64_t k1 = dyn_key(cf, c, t, nc, r1, pwc, n, true, na_n, &s1, &passed1);
    return k1 ? key_score(k1) : INT32_MIN;
}
template <typename RC>
__device__ __forceinline__ void rc_insert(RC* rc, int n, int slot) {  // n distinct
    int h = rc_slot<RC>(n);
    while (atomicCAS(&rc->hkey[h], -1, n) != -1) h = (h + 1) & (RC::kHashN - 1);
    rc->hslot[h] = slot;
}
template <typename RC>
__device__ __forceinline__ int rc_find(const RC* rc, int n) {
    int h = rc_slot<RC>(n);
    for (int i = 0; i < RC::kHashN; ++i, h = (h + 1) & (RC::kHashN - 1)) {
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

// What a parallel-levels placement decided, per lane of wave 0: lane j holds
// candidate j (its node, row before the chunk, port words and node-affinity
// weight) and position j of the placement order (entry L, its candidate lane
// lf and commit kind); cc = commits of candidate j, ap_l = its first Pipeline
// depth; done / stop for the chunk.
template <typename ET>
struct PlaceDec {
    int n;
    Row base;
    uint64_t pw[4], pwc[4];
    int32_t na_n;
    ET L;
    bool inm;
    int lf, kind, cc, ap_l;
    int done, stop;
};
// Candidate j's row after the chunk's commits (Allocate^a Pipeline^p, a = min(cc, first Pipeline depth)).
template <typename ET>
__device__ __forceinline__ Row place_row(const TaskClass& c, const PlaceDec<ET>& D) {
    if (D.cc <= 0) return D.base;
    const int na = D.cc < D.ap_l ? D.cc : D.ap_l;
    return apply_commits(D.base, c, na, D.cc - na);
}

// The end of a placement decision (wave 0): the stop rule over the placement
// order (allocate.go:187-195, gang.go:63-66), the commits per candidate, the
// decision into D.  Position p holds entry L of candidate lane lf with commit
// kind `kind`; fast: position p is candidate p (else cnt[64], zeroed, counts).
template <typename ET, bool SC1>
__device__ __forceinline__ bool place_tail(const PopArgs& a, uint64_t t0, bool fast, ET L, bool inm, int lf, int kind,
                                           int ap_l, int32_t* cnt, const Row& base, const uint64_t* pw,
                                           const uint64_t* pwc, int32_t na_n, int n, uint32_t seq, PlaceDec<ET>& D) {
    const int lane = threadIdx.x & 63;
    const int m = a.n_tasks;
    const uint64_t amask = __ballot(inm && kind == 1);  // Pipelined is not an AllocatedStatus
    const uint64_t upto = lane == 63 ? ~0ull : ((2ull << lane) - 1);
    const int ready_p = a.ready_count + __popcll(amask & upto);
    const uint64_t smask = __ballot(lane < m && (!inm || !a.gang_mode || ready_p >= a.min_avail));
    int cap = m;  // positions decided exactly (a prefix: the entries are sorted)
    if (t0) {
        const int32_t s0 = key_score(t0);
        const int i0 = key_idx(t0);
        const int32_t rm = inm ? entry_rm<ET>(L, a) : 0;
        const bool ex = inm && (rm > s0 || (rm == s0 && entry_node(L, a) <= i0));
        cap = __popcll(__ballot(ex && lane < m));
    }
    int done, stop;
    const int p0 = smask ? __ffsll((unsigned long long)smask) - 1 : 64;
    if (p0 < cap) {
        done = p0 + 1;
        stop = __builtin_amdgcn_readlane((int)inm, p0) ? 2 : 1;
    } else {
        done = cap;  // cap == m: every task placed, the pop goes on (stop 0)
        stop = 0;
    }
    STAMP(gridDim.x * 4 + 8);
    int cc;
    if (fast) {  // position p is candidate p, once
        cc = lane < done ? 1 : 0;
    } else {
        if (lane < done && inm) atomicAdd(&cnt[lf], 1);
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the LDS adds of this wave
        __builtin_amdgcn_wave_barrier();
        cc = cnt[lane];
    }
    STAMP(gridDim.x * 4 + 9);
    if constexpr (SC1) {
        if (lane == 0) { TL(seq, 7); TL_VAL(seq, 9, fast ? 1 : 2); TL_VAL(seq, 10, (uint64_t)done); }
    }
    D.n = n;
    D.base = base;
    for (int w = 0; w < 4; ++w) { D.pw[w] = pw[w]; D.pwc[w] = pwc[w]; }
    D.na_n = na_n;
    D.L = L;
    D.inm = inm;
    D.lf = lf;
    D.kind = kind;
    D.cc = cc;
    D.ap_l = ap_l;
    D.done = done;
    D.stop = stop;
    return true;
}

// The parallel-levels decision (every wave calls; true on wave 0, which holds
// the result — the other waves return false after their last barrier).
// t0 (a cut): the candidates are exact down to the selection key t0 only
// — a node outside them may beat an entry below it — so the launch places
// the entries at or above it and leaves the rest of the chunk to the host
// (stop 0 with done < m; done 0 when none).
// Node indices in keys and entries are global.
// rc_slots (LDS, optional): candidate j's row is in row-cache slot rc_slots[j] (no lookup).
// CACHED (the persistent engine): every candidate's row is in the cache and
// read from there where it is used (not held in registers); no host ports.
template <typename ET, bool SC1, typename RC, bool CACHED = false>
__device__ __forceinline__ bool place_decide(const Conf& cf, const NodeCols& nc, const DevTables& t, const TaskClass& c,
                                             const PopArgs& a, uint64_t (*wl64)[64], uint32_t seq, const RC* rc,
                                             uint64_t t0, PlaceDec<ET>& D, const int32_t* rc_slots = nullptr) {
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
    D.n = n;
    Row base{};
    uint64_t pw[4] = {0, 0, 0, 0};
    int32_t na_n = 0;
    const int rslot = (rc && n >= 0) ? (rc_slots ? rc_slots[lane] : rc_find(rc, n)) : -1;
    if constexpr (CACHED) {
        if (rslot >= 0) na_n = rc->na[rslot];
    } else if (rslot >= 0) {
        base = rc->row[rslot];
        for (int w = 0; w < 4; ++w) pw[w] = rc->pw[rslot][w];
        na_n = rc->na[rslot];
    } else if (n >= 0) {
        base = load_row_t<SC1>(nc, n);
        if (c.has_ports)
            for (int w = 0; w < 4; ++w) if (w < port_win(c, nc)) pw[w] = load_port_t<SC1>(nc, c.pw_lo + w, n);
        if (cf.score_mult) na_n = na_weight(c, t, nc, n);
    }
    auto base_row = [&]() -> Row {
        if constexpr (CACHED) return rslot >= 0 ? rc->row[rslot] : Row{};
        else return base;
    };
    STAMP(gridDim.x * 4 + 11);
    uint64_t pwc[4];
    for (int w = 0; w < 4; ++w)
        pwc[w] = CACHED ? 0 : pw[w] | ((c.has_ports && w < port_win(c, nc)) ? t.masks[c.pown_off + w] : 0);
    const int m = a.n_tasks;
    // Fast path (no second commit reaches the chunk): T0 = the m-th depth-0
    // entry.  A second entry of any candidate is its running minimum after one
    // commit at depth 1, and deeper entries are below it; if none of the first
    // m candidates' depth-1 entries reaches T0, the chunk's top m entries are
    // the first m candidates once each, in list order.  Wave 0 decides; the
    // other waves learn it at the barrier the levels need anyway.
    __shared__ int s_fast;
    if constexpr (SC1) {
        if (threadIdx.x == 0) TL(seq, 14);
    }
    if (wave == 0) {
        bool fast0 = false;
        const uint64_t Km = m >= 1 && m <= 64 ? readlane64(K, m - 1) : 0;
        if (Km) {  // the first m candidates are all feasible
            const int ap0 = key_kind(K) == 2 ? 0 : 64;
            bool reach = false;
            if (lane < m) {
                int32_t s1d;  // the row cache holds it (computed beside the row load), else computed here
                if (rslot >= 0) {
                    s1d = rc->s1[rslot];
                } else {
                    const int na = ap0 == 0 ? 0 : 1;
                    const Row r1 = apply_commits(base_row(), c, na, 1 - na);
                    int32_t s1;
                    bool passed1;
                    const uint64_t k1 = dyn_key(cf, c, t, nc, r1, pwc, n, true, na_n, &s1, &passed1);
                    s1d = k1 ? key_score(k1) : INT32_MIN;
                }
                if (s1d != INT32_MIN) {
                    const int32_t s0 = key_score(K), sm = key_score(Km);
                    const int32_t rm = s1d < s0 ? s1d : s0;
                    // (rm, n, depth 1) vs (sm, node of Km, depth 0): higher score, lower index, lower depth
                    reach = rm > sm || (rm == sm && n < key_idx(Km));
                }
            }
            fast0 = __ballot(reach) == 0;
        }
        if (lane == 0) s_fast = fast0;
        if (!fast0) { s_apos[lane] = 64; s_cnt[lane] = 0; }
    }
    if (threadIdx.x < kHash) s_hkey[threadIdx.x] = -1;
    __syncthreads();  // the decision; K read by every wave; wl free
    const bool fast = s_fast != 0;
    if constexpr (SC1) {
        if (threadIdx.x == 0) TL(seq, 15);
    }
    ET L = 0;            // wave 0: merged top-64 entries so far (lane p = entry p)
    int lf = 0, kind = 0, ap_l = 64;
    bool inm = false;
    if (fast) {
        if (wave != 0) return false;
        STAMP(gridDim.x * 4 + 13);
        inm = lane < m;
        L = inm ? depth_entry<ET>(key_score(K), n, 0, a) : (ET)0;
        lf = lane;
        kind = inm ? key_kind(K) : 0;
        ap_l = key_kind(K) == 2 ? 0 : 64;
    } else {
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
        const Row r = apply_commits(base_row(), c, na, d - na);
        int32_t s;
        bool passed;
        const uint64_t k = dyn_key(cf, c, t, nc, r, pwc, n, true, na_n, &s, &passed);
        *sc = k ? key_score(k) : 0;
        return k ? key_kind(k) : 0;
    };
    bool alive = n >= 0; // candidate still relevant (uniform over waves)
    for (int r = 0; r < 64 / kW; ++r) {
        const int d = r * kW + wave;
        int ap = s_apos[lane];
        int32_t sc = 0;
        int kd = alive ? eval_at(d, ap, &sc) : 0;
        s_kind[d][lane] = (uint8_t)kd;
        __syncthreads();
        if (ap == 64) {  // first Pipeline within this round: recompute the depths behind it
            // (no barrier before the rewrites below: they only touch depths
            // after the first Pipeline, which every scan stops at)
            for (int w2 = 0; w2 < kW; ++w2)
                if (s_kind[r * kW + w2][lane] == 2) { ap = r * kW + w2; break; }
            if (alive && ap < d) {
                kd = eval_at(d, ap, &sc);
                s_kind[d][lane] = (uint8_t)kd;
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
        if (r == 0) { STAMP(gridDim.x * 4 + 6); }
        if (wave == kW - 1) { s_last[lane] = e; s_rm[(r + 1) & 1][lane] = rm; }
        wl[wave][lane] = wave_sort_desc(e);
        __syncthreads();
        block_tree_merge(wl, wave, lane);
        if (wave == 0) L = r == 0 ? wl[0][lane] : wave_merge_desc(L, wl[0][lane]);
        if (wave == 0) {
            if (r == 0) { STAMP(gridDim.x * 4 + 7); }
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
    if (wave != 0) return false;
    STAMP(gridDim.x * 4 + 2);
    // commit kind of each position: its node's candidate lane, the entry's depth
    inm = lane < m && L != 0;
    if (inm) {
        const int ni = entry_node(L, a);
        int h = hash_slot(ni);
        while (s_hkey[h] != ni) h = (h + 1) & (kHash - 1);
        lf = s_hlane[h];
    }
    kind = inm ? s_kind[entry_depth(L)][lf] : 0;
    ap_l = s_apos[lane];
    }  // slow path
    return place_tail<ET, SC1>(a, t0, fast, L, inm, lf, kind, ap_l, s_cnt, base_row(), pw, pwc, na_n, n, seq, D);
}

// The decision on wave 0 alone, with no block barrier (the other waves go on
// with other work): the fast path, or the levels on one wave.  Only the
// candidates whose second entry reaches the chunk (set R, see the fast path
// in place_decide) can place more than once; their deeper entries are
// computed in rounds, lane = (member r, one of Dd = 64 / |members| depths,
// rounded to powers of two, following the member's deepest so far), merged
// into the placement order L; a member stays for the next round while its
// deepest entry still reaches the m-th position.  The same entries, commit
// kinds and order as the levels over all waves.  every_member (a test mode):
// every feasible candidate in R, no fast path.  Every candidate's row is in
// the row cache (slot rc_slots[j]); no cut (t0 = 0); no host ports (false:
// nothing decided).
template <typename ET, bool SC1, typename RC>
__device__ __forceinline__ bool place_decide_wave(const Conf& cf, const NodeCols& nc, const DevTables& t,
                                                  const TaskClass& c, const PopArgs& a, const uint64_t* K0,
                                                  uint32_t seq, const RC* rc, const int32_t* rc_slots,
                                                  bool every_member, PlaceDec<ET>& D) {
    __shared__ uint8_t q_kind[64][64];  // [depth][candidate]: 1 Allocate, 2 Pipeline, 0 infeasible
    __shared__ int32_t q_rl[64];        // this round's members, in list order
    __shared__ int32_t q_cnt[64], q_apos[64], q_rm[64], q_dl[64];
    __shared__ uint8_t q_alive[64];
    __shared__ int32_t q_hkey[kHash], q_hlane[kHash];
    const int lane = threadIdx.x & 63;
    if (c.has_ports) return false;  // (host-port words: the levels over all waves)
    const uint64_t K = K0[lane];
    const int n = K ? key_idx(K) : -1;
    const int rslot = n >= 0 ? rc_slots[lane] : -1;
    const int32_t s1d = rslot >= 0 ? rc->s1[rslot] : INT32_MIN;
    const uint64_t pw[4] = {0, 0, 0, 0};
    auto tail = [&](bool fast, ET L, bool inm, int lf, int kind, int ap_l) {
        Row base{};  // (loaded here: not live across the evaluation)
        int32_t na_n = 0;
        if (rslot >= 0) {
            base = rc->row[rslot];
            na_n = rc->na[rslot];
        }
        return place_tail<ET, SC1>(a, 0, fast, L, inm, lf, kind, ap_l, q_cnt, base, pw, pw, na_n, n, seq, D);
    };
    const int m = a.n_tasks;
    const uint64_t Km = m >= 1 && m <= 64 ? readlane64(K, m - 1) : 0;
    bool reach = false;  // (with fewer than m feasible candidates every second entry counts)
    if (K && (lane < m || !Km || every_member) && s1d != INT32_MIN) {
        if (!Km || every_member) {
            reach = true;
        } else {
            const int32_t s0 = key_score(K), sm = key_score(Km);
            const int32_t rm = s1d < s0 ? s1d : s0;
            reach = rm > sm || (rm == sm && n < key_idx(Km));
        }
    }
    uint64_t alive = __ballot(reach);
    const int ap_own = K && key_kind(K) == 2 ? 0 : 64;
    if (Km && !alive && !every_member) {  // the first m candidates once each, in list order
        const bool inm = lane < m;
        const ET L = inm ? depth_entry<ET>(key_score(K), n, 0, a) : (ET)0;
        return tail(true, L, inm, lane, inm ? key_kind(K) : 0, ap_own);
    }
    q_cnt[lane] = 0;
    q_apos[lane] = ap_own;
    q_rm[lane] = K ? key_score(K) : 0;
    q_dl[lane] = 0;
    q_kind[0][lane] = K ? (uint8_t)key_kind(K) : (uint8_t)0;
    for (int h = lane; h < kHash; h += 64) q_hkey[h] = -1;
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    if (n >= 0) {  // node -> candidate lane (candidate nodes are distinct)
        int h = hash_slot(n);
        while (atomicCAS(&q_hkey[h], -1, n) != -1) h = (h + 1) & (kHash - 1);
        q_hlane[h] = lane;
    }
    ET L = K ? depth_entry<ET>(key_score(K), n, 0, a) : (ET)0;  // the depth-0 entries (list order)
    while (alive) {
        const int k = __popcll(alive);
        const int lk = k <= 1 ? 0 : k <= 2 ? 1 : k <= 4 ? 2 : k <= 8 ? 3 : k <= 16 ? 4 : k <= 32 ? 5 : 6;
        const int Dd = 64 >> lk;  // depths per member this round
        if ((alive >> lane) & 1)
            q_rl[__builtin_amdgcn_mbcnt_hi((uint32_t)(alive >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)alive, 0))] = lane;
        q_alive[lane] = 0;
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
        const int seg = lane >> (6 - lk), off = lane & (Dd - 1);
        int j = seg < k ? q_rl[seg] : -1;
        const int dl = j >= 0 ? q_dl[j] : 0;
        const int d = dl + 1 + off;
        const int lastoff = (Dd < 63 - dl ? Dd : 63 - dl) - 1;  // the member's deepest lane (depth 63 at most)
        if (off > lastoff) j = -1;
        Row bj{};
        int32_t naj = 0, rm0 = 0;
        int nj = -1, apj = 64;
        if (j >= 0) {
            const int sl = rc_slots[j];
            nj = key_idx(K0[j]);
            bj = rc->row[sl];
            naj = rc->na[sl];
            rm0 = q_rm[j];
            apj = q_apos[j];
        }
        auto eval_at = [&](int dd, int ap, int32_t* sc) -> int {  // kind of commit dd+1's key (0: infeasible)
            const int na = dd < ap ? dd : ap;
            const Row r = apply_commits(bj, c, na, dd - na);
            int32_t s = 0;
            bool passed;
            const uint64_t kk = dyn_key(cf, c, t, nc, r, pw, nj, true, naj, &s, &passed);
            *sc = kk ? key_score(kk) : 0;
            return kk ? key_kind(kk) : 0;
        };
        int32_t sc = 0;
        int kd = j >= 0 ? eval_at(d, apj, &sc) : 0;
        // the member's first Pipeline depth; the depths behind it, assumed Allocates: again
        int ap = (j >= 0 && kd == 2) ? d : 64;
        for (int o = 1; o < Dd; o <<= 1) {
            const int x = __shfl_xor(ap, o, 64);
            ap = x < ap ? x : ap;
        }
        ap = apj < ap ? apj : ap;
        const bool redo = j >= 0 && apj == 64 && d > ap;
        if (__ballot(redo) != 0 && redo) kd = eval_at(d, ap, &sc);
        // entries: running minimum through depth d; the chain ends at the first infeasible depth
        bool ok = j >= 0 && kd != 0;
        int32_t rm = sc;
        for (int o = 1; o < Dd; o <<= 1) {
            const int32_t x = __shfl_up(rm, o, 64);
            const int y = __shfl_up((int)ok, o, 64);
            if (off >= o) {
                rm = x < rm ? x : rm;
                ok = ok && y;
            }
        }
        rm = rm0 < rm ? rm0 : rm;
        const ET e = ok ? depth_entry<ET>(rm, nj, d, a) : (ET)0;
        if (j >= 0) q_kind[d][j] = (uint8_t)kd;
        L = wave_merge_desc(L, wave_sort_desc(e));
        const ET T = readlane_t(L, m - 1);  // the m-th entry (0: fewer entries than tasks)
        if (j >= 0 && off == lastoff) {
            q_rm[j] = rm;
            q_dl[j] = d;
            q_apos[j] = ap;
            q_alive[j] = (e != 0 && e >= T && d < 63) ? 1 : 0;
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
        alive = __ballot(q_alive[lane] != 0);
    }
    const bool inm = lane < m && L != 0;
    int lf = 0;
    if (inm) {
        const int ni = entry_node(L, a);
        int h = hash_slot(ni);
        while (q_hkey[h] != ni) h = (h + 1) & (kHash - 1);
        lf = q_hlane[h];
    }
    const int kind = inm ? q_kind[entry_depth(L)][lf] : 0;
    return tail(false, L, inm, lf, kind, q_apos[lane]);
}

// The walk FitDelta histogram of a task that found no node (D.stop == 1):
// fit_in = the counts of the candidates the sweep left out (at the state the
// pop started from), fit_raw = the sweep's counts (fit_sum layout); the
// candidates then carry the commits made before the failing task.  Two
// granules beside the placements (wave 0).
template <typename ET>
__device__ __forceinline__ void place_fit_vals(const Conf& cf, const NodeCols& nc, const DevTables& t,
                                               const TaskClass& c, const PopArgs& a, const PlaceDec<ET>& D,
                                               const int32_t* fit_in, uint32_t fit_raw, uint64_t* g0, uint64_t* g1) {
    uint32_t fb_base = 0, fb_post = 0;
    if (D.n >= 0) {
        fb_base = fit_bits(c, D.base, true);  // candidates had a key: in the walk
        const Row r = place_row(c, D);
        int32_t sc;
        bool passed;
        (void)dyn_key(cf, c, t, nc, r, D.cc > 0 ? D.pwc : D.pw, D.n, true, D.na_n, &sc, &passed);
        fb_post = fit_bits(c, r, passed);
    }
    const uint32_t sweep = fit_sum(fit_raw);
    int32_t tot[4];
#pragma unroll
    for (int b = 0; b < 4; ++b)
        tot[b] = (int32_t)__builtin_amdgcn_readlane((int)sweep, b) + fit_in[b] +
                 __popcll(__ballot((fb_post >> b) & 1u)) - __popcll(__ballot((fb_base >> b) & 1u));
    *g0 = make_fit_granule(a.epoch, tot[0], tot[1]);
    *g1 = make_fit_granule(a.epoch, tot[2], tot[3]);
}
template <typename ET>
__device__ __forceinline__ void place_fit(const Conf& cf, const NodeCols& nc, const DevTables& t, const TaskClass& c,
                                          const PopArgs& a, PopOut* out, const PlaceDec<ET>& D, const int32_t* fit_in,
                                          uint32_t fit_raw) {
    uint64_t g0, g1;
    place_fit_vals(cf, nc, t, c, a, D, fit_in, fit_raw, &g0, &g1);
    if ((threadIdx.x & 63) == 0) {
        __hip_atomic_store(&out->fit[0], g0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&out->fit[1], g1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// The result granule of position `lane` (0: none to write).
template <typename ET>
__device__ __forceinline__ uint64_t place_granule_val(const PopArgs& a, const PlaceDec<ET>& D) {
    const int lane = threadIdx.x & 63;
    if (!(lane < D.done || (D.done == 0 && lane == 0))) return 0;
    return make_granule(a.epoch, D.stop, D.done, lane < D.done ? D.kind : 0,
                        (lane < D.done && D.inm) ? entry_node(D.L, a) : -1);
}
// The result granules of the chunk (wave 0; pinned host memory, one 8-byte store each).
template <typename ET>
__device__ __forceinline__ void place_granules(const PopArgs& a, PopOut* out, const PlaceDec<ET>& D) {
    const uint64_t g = place_granule_val(a, D);
    if (g) __hip_atomic_store(&out->g[threadIdx.x & 63], g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <typename ET, bool SC1 = false, typename RC = RowCache>
__device__ __forceinline__ void place_parallel(const Conf& cf, const NodeCols& nc, const DevTables& t, const TaskClass& c,
                               const PopArgs& a, PopOut* out, uint64_t (*wl64)[64], uint32_t* done_flag = nullptr,
                               uint32_t seq = 0, const RC* rc = nullptr, const int32_t* fit_in = nullptr,
                               uint32_t fit_raw = 0, int wb_base = 0, int wb_n = 0x7fffffff, uint64_t t0 = 0,
                               uint64_t (*row_msg)[64] = nullptr) {
    // wb_base / wb_n: node rows [wb_base, wb_base + wb_n) are this device's
    // (a node-array shard writes back only its own; one GPU: all of them).
    PlaceDec<ET> D;
    if (!place_decide<ET, SC1>(cf, nc, t, c, a, wl64, seq, rc, t0, D)) return;
    const int lane = threadIdx.x & 63;
    if (fit_in && D.stop == 1) place_fit(cf, nc, t, c, a, out, D, fit_in, fit_raw);
    const int n = D.n, cc = D.cc;
    const int ln = n - wb_base;  // local row of the written-back node
    if (n >= 0 && cc > 0 && ln >= 0 && ln < wb_n) {
        const Row r = place_row(c, D);
        if constexpr (SC1) {
            st_sc1(&nc.idle_cpu[ln], r.idle_cpu); st_sc1(&nc.idle_mem[ln], r.idle_mem); st_sc1(&nc.idle_gpu[ln], r.idle_gpu);
            st_sc1(&nc.rel_cpu[ln], r.rel_cpu); st_sc1(&nc.rel_mem[ln], r.rel_mem); st_sc1(&nc.rel_gpu[ln], r.rel_gpu);
            st_sc1(&nc.pods[ln], r.pods);
            st_sc1(&nc.nzc[ln], r.nzc);
            st_sc1(&nc.nzm[ln], r.nzm);
            if (c.has_ports)
                for (int w = 0; w < 4; ++w) if (w < port_win(c, nc)) st_sc1(&nc.ports[port_at(c, nc, w, ln)], D.pwc[w]);
        } else {
            nc.idle_cpu[ln] = r.idle_cpu; nc.idle_mem[ln] = r.idle_mem; nc.idle_gpu[ln] = r.idle_gpu;
            nc.rel_cpu[ln] = r.rel_cpu; nc.rel_mem[ln] = r.rel_mem; nc.rel_gpu[ln] = r.rel_gpu;
            nc.pods[ln] = r.pods;
            nc.nzc[ln] = r.nzc;
            nc.nzm[ln] = r.nzm;
            if (c.has_ports)
                for (int w = 0; w < 4; ++w) if (w < port_win(c, nc)) nc.ports[port_at(c, nc, w, ln)] = D.pwc[w];
        }
    }
    if constexpr (SC1) {  // the only storing wave drained, then the row message, then the flag (sc1)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (row_msg) {  // every candidate's row after this pop (self-tagged halves, PopLink::rows)
            const Row rw = place_row(c, D);
            uint32_t w[kRowWords];
            row_words(rw, w);
#pragma unroll
            for (int f = 0; f < kRowWords; ++f) st_sc1(&row_msg[f][lane], ((uint64_t)seq << 32) | w[f]);
        }
        if (lane == 0) { st_sc1(done_flag, seq); TL(seq, 8); }
    }
    place_granules(a, out, D);
    STAMP(gridDim.x * 4 + 3);
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
            for (int w = 0; w < 4; ++w) if (w < port_win(c, nc)) pw[w] = nc.ports[port_at(c, nc, w, n)];
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
                for (int q = 0; q < 4; ++q) pw[q] |= (q < port_win(c, nc)) ? t.masks[c.pown_off + q] : 0;
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
            for (int w = 0; w < 4; ++w) if (w < port_win(c, nc)) nc.ports[port_at(c, nc, w, n)] = pw[w];
    }
    if (lane < done || (done == 0 && lane == 0))
        __hip_atomic_store(&out->g[lane],
                           make_granule(a.epoch, stop, done, mine ? key_kind(mine) : 0, mine ? key_idx(mine) : -1),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ---------------------------------------------------------------------------
// Placement of a pod-affinity class (placement 7; one wave, task after task;
// classes with aff_batchable, kbhip_eval.h).  A placement adds the pod to
// count tables (commit_aff), which can only turn nodes of the placed pod's
// topology domains infeasible for the class's later tasks (a required
// anti-affinity target now exists there, predicates.go:1293-1458); no node's
// key rises.  Lane j holds candidate j of the sweep's list (keys with the
// affinity predicates, eval_node_aff) with its row and the count-table slots
// its predicates read (slot = table offset + the node's domain, -1 without
// the key) and their counts.  Per task: winner = the largest current key;
// the winner's count-table updates are broadcast as slots and every lane
// whose predicate reads one of them adds to its count; a lane whose
// predicate now fails drops out; the winner's row is committed and its key
// re-evaluated.  Nodes outside the list had keys below the list's last one
// and can only fall, so the choice is exact while the winner's key is at
// least the list's last key; otherwise (or when no node is left) the launch
// ends before that task and the host goes on (n_done 0: the general path for
// one task, which also reports a no-node task's FitDelta histogram).
// ---------------------------------------------------------------------------
__device__ void place_aff(const Conf& cf, const NodeCols& nc, const DevTables& t, const TaskClass& c,
                          const PopArgs& a, PopOut* out, uint64_t K) {
    const int lane = threadIdx.x & 63;
    const int n = K ? key_idx(K) : -1;  // one GPU: global index = row
    Row r{};
    uint64_t pw[4] = {0, 0, 0, 0};
    int32_t na_n = 0;
    int32_t slot[kAffItems], cnt[kAffItems];
    const int n_ea = c.ea_n;
    const int n_items = n_ea + (c.paa_space >= 0 ? 1 : 0);
#pragma unroll
    for (int k = 0; k < kAffItems; ++k) {
        slot[k] = -1;
        cnt[k] = 0;
        if (k < n_items && n >= 0) {
            const int space = k < n_ea ? t.aff_items[c.ea_off + 2 * k] : c.paa_space;
            const int tab = k < n_ea ? t.aff_items[c.ea_off + 2 * k + 1] : c.paa_cnt;
            const int d = dom_of(nc, space, n);
            if (d >= 0) {
                slot[k] = tab + d;
                cnt[k] = t.aff_cnt[tab + d];
            }
        }
    }
    // the class's commit updates as this lane's node would apply them (commit_aff): table slot
    // (offset + the node's domain; -1: the node lacks the key) — loaded once, off the task loop
    int32_t uslot[kAffUpd];
    const int n_upd = c.upd_n;
#pragma unroll
    for (int u = 0; u < kAffUpd; ++u) {
        uslot[u] = -1;
        if (u < n_upd && n >= 0) {
            const int32_t* it = t.aff_items + c.upd_off + 3 * u;
            const int d = it[0] == 0 ? dom_g(nc, it[1], n) : 0;
            if (d >= 0) uslot[u] = it[2] + d;
        }
    }
    int32_t utype[kAffUpd];  // uniform: the class's items
#pragma unroll
    for (int u = 0; u < kAffUpd; ++u) utype[u] = u < n_upd ? t.aff_items[c.upd_off + 3 * u] : -1;
    if (n >= 0) {
        r = load_row(nc, n);
        if (c.has_ports)
            for (int w = 0; w < 4; ++w) if (w < port_win(c, nc)) pw[w] = nc.ports[port_at(c, nc, w, n)];
        if (cf.score_mult) na_n = na_weight(c, t, nc, n);
    }
    int wins_alloc = 0, wins_pipe = 0;  // this lane's node: placements (the device tables after the loop)
    // uniform loop bounds in scalar registers: the task loop is one wave's serial chain, so
    // every item it skips with a scalar branch instead of a masked vector step counts
    const int nit = __builtin_amdgcn_readfirstlane(n_items);
    uint32_t m0bits = 0;  // the UPD_CNT_ALLOC items
#pragma unroll
    for (int u = 0; u < kAffUpd; ++u) m0bits |= (u < n_upd && utype[u] == 0) ? (1u << u) : 0u;
    const uint32_t m0mask = (uint32_t)__builtin_amdgcn_readfirstlane((int)m0bits);
    const uint64_t t0 = readlane64(K, 63);  // the list's last key (0: the list holds every feasible node)
    uint64_t key = K;
    bool changed = false;
    int ready = a.ready_count, done = 0, stop = 0;
    uint64_t mine = 0;  // lane i: winner key of task i
    // Per-domain candidates (dd_space): the list holds at most one node per domain, and an
    // Allocated placement closes its winner's domain and nothing else the class reads, so
    // while the winners are Allocated nodes that carry the key, task i takes list entry i:
    // the whole run at once (ballots and a scalar walk for the stops) instead of the task
    // loop.  A node without the key at the head of the list takes the loop.
    bool fast = false;
    if (c.dd_space >= 0 && nit > 0) {  // (uniform)
        const bool keyed = n >= 0 && slot[0] >= 0;
        const uint64_t V = __ballot(K != 0 && keyed);
        const uint64_t Z = __ballot(K != 0);
        if ((V & 1ull) || !(Z & 1ull)) {
            fast = true;
            const uint64_t P2 = __ballot(K != 0 && key_kind(K) == 2);
            const int len = V == ~0ull ? 64 : __builtin_ctzll(~V);
            const int m = len < a.n_tasks ? len : a.n_tasks;
            int r_s = a.ready_count, d_s = 0, st_s = 0;
            for (int i = 0; i < m; ++i) {  // scalar: the loop's stop rules over list order
                const bool pipe = (P2 >> i) & 1ull;
                d_s = i + 1;
                if (!pipe) ++r_s;
                if (!a.gang_mode || r_s >= a.min_avail) { st_s = 2; break; }
                if (pipe) break;  // a Pipelined winner does not close its domain
            }
            done = d_s;
            stop = st_s;
            ready = r_s;
            if (lane < done) {
                mine = K;
                const int kind = key_kind(K);
                if (kind == 1) ++wins_alloc;
                else ++wins_pipe;
                r = apply_commits(r, c, kind == 1 ? 1 : 0, kind == 1 ? 0 : 1);
                if (c.has_ports)
                    for (int q = 0; q < 4; ++q) pw[q] |= (q < port_win(c, nc)) ? t.masks[c.pown_off + q] : 0;
                changed = true;
            }
        }
    }
    for (int i = 0; i < a.n_tasks && !fast; ++i) {
        const uint64_t w = wave_max_key(key);
        if (!w || w < t0) break;  // no node, or one outside the list may come first: the host goes on
        if (lane == i) mine = w;
        const bool win = n >= 0 && key == w;
        const int wl = __ffsll((unsigned long long)__ballot(win)) - 1;
        const int kind = key_kind(w);
        // the winner's count-table updates (UPD_CNT_ALLOC: Allocated only), as slots
        if (kind == 1) {
#pragma unroll
            for (int u = 0; u < kAffUpd; ++u) {
                if (!((m0mask >> u) & 1u)) continue;  // (scalar)
                const int us = __builtin_amdgcn_readlane(uslot[u], wl);
                if (us >= 0) {  // (scalar)
#pragma unroll
                    for (int k = 0; k < kAffItems; ++k)
                        if (k < nit) cnt[k] += (slot[k] == us) ? 1 : 0;
                }
            }
        }
        bool aff_ok = true;
#pragma unroll
        for (int k = 0; k < kAffItems; ++k)
            if (k < nit) aff_ok = aff_ok && !(slot[k] >= 0 && cnt[k] > 0);
        // the winner's next key: only if its own predicates still pass (a self-anti-affine
        // winner's domain is closed): a scalar branch around the key evaluation
        const bool alive = __builtin_amdgcn_readlane((int)aff_ok, wl) != 0;
        if (win) {
            if (kind == 1) ++wins_alloc;
            else ++wins_pipe;
            r = apply_commits(r, c, kind == 1 ? 1 : 0, kind == 1 ? 0 : 1);
            if (c.has_ports)
                for (int q = 0; q < 4; ++q) pw[q] |= (q < port_win(c, nc)) ? t.masks[c.pown_off + q] : 0;
            changed = true;
        }
        if (alive) {
            if (win) {
                int32_t s = 0;
                bool passed = false;
                key = dyn_key(cf, c, t, nc, r, pw, n, true, na_n, &s, &passed);
            }
        } else if (win) {
            key = 0;
        }
        if (!win && !aff_ok) key = 0;
        done = i + 1;
        if (kind == 1) ++ready;  // Pipelined is not an AllocatedStatus (types.go:82-84)
        if (!a.gang_mode || ready >= a.min_avail) { stop = 2; break; }  // allocate.go:191-195
        // per-domain candidates: only an Allocated placement closes its domain; after a
        // Pipelined one a node of the winner's domain left out by the sweep may come next
        if (c.dd_space >= 0 && kind != 1) break;
    }
    if (changed) {
        nc.idle_cpu[n] = r.idle_cpu; nc.idle_mem[n] = r.idle_mem; nc.idle_gpu[n] = r.idle_gpu;
        nc.rel_cpu[n] = r.rel_cpu; nc.rel_mem[n] = r.rel_mem; nc.rel_gpu[n] = r.rel_gpu;
        nc.pods[n] = r.pods;
        nc.nzc[n] = r.nzc;
        nc.nzm[n] = r.nzm;
        if (c.has_ports)
            for (int w = 0; w < 4; ++w) if (w < port_win(c, nc)) nc.ports[port_at(c, nc, w, n)] = pw[w];
        // the device tables (later launches read them; commit_aff per placement): every winning
        // lane adds its placements at once — atomics, since lanes may share entries
#pragma unroll
        for (int u = 0; u < kAffUpd; ++u) {
            const int add = utype[u] == 2 ? wins_alloc + wins_pipe : wins_alloc;
            if (uslot[u] >= 0 && add > 0)
                __hip_atomic_fetch_add((utype[u] == 0 ? t.aff_cnt : t.aff_scalar) + uslot[u], add, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    if (lane < done || (done == 0 && lane == 0))
        __hip_atomic_store(&out->g[lane],
                           make_granule(a.epoch, stop, done, mine ? key_kind(mine) : 0, mine ? key_idx(mine) : -1),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// System-scope (sc0 sc1) 8-byte accesses: what crosses between ranks' devices
// through the mailboxes (and what a placement reads of them).
__device__ __forceinline__ void st_sys(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint64_t ld_sys(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
template <typename T>
__device__ __forceinline__ void store_words_sys(T* dst, const T& v) {
    uint64_t w[sizeof(T) / 8];
    __builtin_memcpy(w, &v, sizeof(T));
#pragma unroll
    for (int i = 0; i < (int)(sizeof(T) / 8); ++i) st_sys((uint64_t*)dst + i, w[i]);
}
template <typename T>
__device__ __forceinline__ T load_words_sys(const T* src) {
    uint64_t w[sizeof(T) / 8];
#pragma unroll
    for (int i = 0; i < (int)(sizeof(T) / 8); ++i) w[i] = ld_sys((const uint64_t*)src + i);
    T v;
    __builtin_memcpy(&v, w, sizeof(T));
    return v;
}

// 16-byte system-scope store (sc0 sc1, a vector store): mailbox payload.
typedef unsigned int kb_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st_sys16(void* p, kb_u32x4 v) {
    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" : : "v"(p), "v"(v) : "memory");
}

// The shard epilogue of k_pop_batch (placement 3), run by every thread of
// the final merger: this shard's top-64 (wave 0 lane j: candidate j) with
// their rows and the sweep's FitDelta counts go to its own exchange buffer
// (msg, for the all-gather), or straight into every rank's mailbox (mb.world
// > 0): the candidates are staged in LDS, every thread of the block stores
// its share of (destination, candidate, 16-byte chunk) — a class without
// host ports leaves the port words out — each wave drains its stores, the
// block meets, and lane p of wave 0 raises rank p's flag.  k_shard_place
// reads them with system-scope loads.
// SC1: the rows are read through sc1 (an overlapped shard sweep: some of its
// candidates were just written back by the previous pop's placement on this
// device, from another XCD).  bad: the chain broke; the message says so
// (count word 0xffffffff) and k_shard_place reports a lost exchange.
template <bool SC1 = false>
__device__ void shard_emit(const Conf& cf, const NodeCols& nc, const DevTables& t, const TaskClass& c, uint64_t K,
                           uint32_t fit_raw, ShardMsg* msg, const MboxArgs& mb, bool bad = false) {
    __shared__ ShardCand s_c[kTopK];
    __shared__ uint64_t s_fit[2];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (wave == 0) {
        ShardCand e{};
        e.node = -1;
        if (K) {
            const int g = key_idx(K);
            const int n = g - nc.base;
            e.key = K;
            e.node = g;
            e.row = load_row_t<SC1>(nc, n);
            if (c.has_ports)
                for (int w = 0; w < 4; ++w) if (w < port_win(c, nc)) e.pw[w] = load_port_t<SC1>(nc, c.pw_lo + w, n);
            e.na = cf.score_mult ? na_weight(c, t, nc, n) : 0;
        }
        uint32_t sweep = fit_sum(fit_raw);  // count b in lane b
        if (bad && lane == 0) sweep = 0xffffffffu;
        if (mb.world == 0) {
            msg->c[lane] = e;
            if (lane < 4) msg->fit[lane] = sweep;
            return;
        }
        s_c[lane] = e;
        if (lane == 0) {
            s_fit[0] = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)sweep, 0) |
                       (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)sweep, 1) << 32;
            s_fit[1] = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)sweep, 2) |
                       (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)sweep, 3) << 32;
        }
    }
    if (mb.world == 0) return;  // (uniform)
    __syncthreads();
    const int slot = (int)(mb.seq & (kMboxSlots - 1));
    constexpr int kChunks = (int)(sizeof(ShardCand) / 16);
    constexpr int kPortChunks = (int)(sizeof(((ShardCand*)nullptr)->pw) / 16);  // the last chunks
    const int chunks = c.has_ports ? kChunks : kChunks - kPortChunks;
    const int items = mb.world * kTopK * chunks;
    for (int i = threadIdx.x; i < items; i += kPopThreads) {
        const int p = i / (kTopK * chunks), rem = i - p * (kTopK * chunks);
        const int j = rem / chunks, q = rem - j * chunks;
        ShardMsg* m = &mb.dst[p]->msg[slot][mb.rank];
        st_sys16((char*)&m->c[j] + 16 * q, *(const kb_u32x4*)((const char*)&s_c[j] + 16 * q));
    }
    if (threadIdx.x < mb.world) {
        ShardMsg* m = &mb.dst[threadIdx.x]->msg[slot][mb.rank];
        st_sys((uint64_t*)m->fit, s_fit[0]);
        st_sys((uint64_t*)m->fit + 1, s_fit[1]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's mailbox stores completed
    __syncthreads();                                   // ... and every other wave's
    if (threadIdx.x < mb.world) st_sys(&mb.dst[threadIdx.x]->flag[slot][mb.rank][0], (uint64_t)mb.seq);
}
}  // namespace kbhip
