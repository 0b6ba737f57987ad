// kbhip_pp.hip — pipelined batched pops with a persistent placer (option "pp").
//
// The overlapped pop kernel (k_pop_batch_ov) chains pops through memory: pop
// e's placement waits for pop e-1's rows to be written back, re-reads them
// and re-evaluates pop e-1's candidates before it can place — a serial chain
// of write-back, flag, re-read and placement per pop.  Here that chain lives
// in ONE workgroup that stays resident for a run of pops (the placer) and
// keeps the rows it committed in LDS; the sweeps run ahead of it:
//
//   k_pp_sweep (one launch per pop e, many workgroups, any stream): every
//     node's selection key for pop e's class on the rows in memory — which
//     may miss the placer's latest commits — reduced to the top-128 keys, with
//     the rows, static node-affinity weight and the FitDelta bits the sweep
//     counted (one nibble per node), and W = the placer's progress every
//     block saw before it read rows (commands <= W are in memory).  Published
//     in ring slot e % kPPSlots behind a sequence flag.
//   k_pp_placer (one workgroup, persistent): for command e — the nodes the
//     placer committed to in pops W+1 .. e-1 (its LDS history) are the only
//     rows the sweep may have read stale; their keys are recomputed from the
//     history rows, the other list keys are exact, and every node outside the
//     list has a key below the list's 128th (t0).  The top-64 of the exact
//     keys place the chunk (place_parallel) exactly down to t0; a chunk that
//     reaches below t0 stops there and the host goes on with the rest (a new
//     sweep).  Rows are written back write-through, then the progress flag.
//
// Hand-offs (MI355X_MICROARCH.md, valid forms, row 1): producers store sc1,
// drain (s_waitcnt vmcnt(0)) and then store one sc1 flag / add one agent
// counter; consumers poll sc1 and load every handed-off byte sc1.  The
// placer leaves after kPPIdle of no command (the host relaunches it), so no
// launch of this file waits without bound.
#define KBHIP_STAMPS_OFF
#include <hip/hip_runtime.h>
#include <cstdint>
namespace kbhip {
__shared__ uint64_t pp_ts[16];  // placement phase sums of the placer launch (thread 0), [15] = last mark
}
#define PSTAMP(k)                                                         \
    do {                                                                  \
        if (threadIdx.x == 0) {                                           \
            const uint64_t x_ = __builtin_amdgcn_s_memrealtime();         \
            pp_ts[(k)] += x_ - pp_ts[15];                                 \
            pp_ts[15] = x_;                                               \
        }                                                                 \
    } while (0)
#include "kbhip_batch.h"

namespace kbhip {

constexpr int kPPK = 128;                   // sweep list length
constexpr int kPPSlots = 8;                 // command ring
constexpr int kPPHist = 4;                  // pops whose committed rows the placer keeps
constexpr int kPPDHash = 1024;              // dirty node hash (kPPHist * 64 keys)
constexpr uint64_t kPPIdle = 2000000;       // placer idle exit: 20 ms of s_memrealtime (100 MHz)
enum : uint32_t { PP_PLACE = 1, PP_STOP = 2 };

struct PPSlot {
    uint32_t seq, type;
    uint32_t Wn;  // ~min over the sweep's blocks of the progress they read (0 = none yet)
    uint32_t out_slot;
    PopArgs a;
    uint32_t fit[4];  // the sweep's FitDelta counts over every node
    uint64_t key[kPPK];
    Row row[kPPK];
    uint64_t pw[kPPK][4];
    int32_t na[kPPK];
};
struct PPCtrl {
    uint32_t written;  // commands <= written are applied and their rows are in memory
    uint32_t pad[15];
    uint64_t prof[8];  // placer phase sums (s_memrealtime ticks): wait, list+dirty, keys+merge, rows, place, tail; count
    uint64_t pprof[16];  // place_parallel's phases (PSTAMP 1..9)
};
struct PPHost {  // pinned host memory
    uint32_t consumed;  // the command the placer waits for / stopped at
    uint32_t exited;    // 1 once the placer left (idle or STOP)
    uint32_t pad[14];
};

// 128-lists: lane i holds entries i (a) and 64 + i (b), descending.
template <typename T>
struct List2 {
    T a, b;
};
template <typename T>
__device__ __forceinline__ T bitonic_clean64(T v) {
    v = half_clean_desc<32>(v);
    v = half_clean_desc<16>(v);
    v = half_clean_desc<8>(v);
    v = half_clean_desc<4>(v);
    v = half_clean_desc<2>(v);
    return half_clean_desc<1>(v);
}
// top-128 of x U y: the first half-cleaner of the 256-entry bitonic network
// (x followed by y reversed), then the bitonic sort of that half.
template <typename T>
__device__ __forceinline__ List2<T> merge128(List2<T> x, List2<T> y) {
    const T ra = reverse_lanes(y.a), rb = reverse_lanes(y.b);
    const T za = x.a > rb ? x.a : rb, zb = x.b > ra ? x.b : ra;
    List2<T> r;
    r.a = bitonic_clean64(za > zb ? za : zb);
    r.b = bitonic_clean64(za > zb ? zb : za);
    return r;
}
template <typename T>
__device__ __forceinline__ void tree_merge128(T (*wl)[2][64], int wave, int lane) {
#pragma unroll
    for (int s = kPopThreads / 128; s >= 1; s >>= 1) {
        if (wave < s) {
            const List2<T> x{wl[wave][0][lane], wl[wave][1][lane]}, y{wl[wave + s][0][lane], wl[wave + s][1][lane]};
            const List2<T> z = merge128(x, y);
            wl[wave][0][lane] = z.a;
            wl[wave][1][lane] = z.b;
        }
        __syncthreads();
    }
}
__device__ __forceinline__ void st_row_sc1(Row* d, const Row& r) {
    st_sc1(&d->idle_cpu, r.idle_cpu); st_sc1(&d->idle_mem, r.idle_mem); st_sc1(&d->idle_gpu, r.idle_gpu);
    st_sc1(&d->rel_cpu, r.rel_cpu); st_sc1(&d->rel_mem, r.rel_mem); st_sc1(&d->rel_gpu, r.rel_gpu);
    st_sc1(&d->bf_cpu, r.bf_cpu); st_sc1(&d->bf_mem, r.bf_mem); st_sc1(&d->bf_gpu, r.bf_gpu);
    st_sc1(&d->acpu, r.acpu); st_sc1(&d->amem, r.amem); st_sc1(&d->nzc, r.nzc); st_sc1(&d->nzm, r.nzm);
    st_sc1(&d->pods, r.pods); st_sc1(&d->maxtasks, r.maxtasks);
}
__device__ __forceinline__ Row ld_row_sc1(const Row* s) {
    Row r;
    r.idle_cpu = ld_sc1(&s->idle_cpu); r.idle_mem = ld_sc1(&s->idle_mem); r.idle_gpu = ld_sc1(&s->idle_gpu);
    r.rel_cpu = ld_sc1(&s->rel_cpu); r.rel_mem = ld_sc1(&s->rel_mem); r.rel_gpu = ld_sc1(&s->rel_gpu);
    r.bf_cpu = ld_sc1(&s->bf_cpu); r.bf_mem = ld_sc1(&s->bf_mem); r.bf_gpu = ld_sc1(&s->bf_gpu);
    r.acpu = ld_sc1(&s->acpu); r.amem = ld_sc1(&s->amem); r.nzc = ld_sc1(&s->nzc); r.nzm = ld_sc1(&s->nzm);
    r.pods = ld_sc1(&s->pods); r.maxtasks = ld_sc1(&s->maxtasks);
    return r;
}

// ---------------------------------------------------------------------------
// the sweep of command `seq` (a PLACE): lists is this slot's (blocks + groups)
// x 128 keys, arrive its counters (group arrivals, then the final one, then the
// per-group FitDelta counters), fitw its nibble array (8 nodes per word).
// ---------------------------------------------------------------------------
template <int R, typename KT>
__global__ __launch_bounds__(kPopThreads) void k_pp_sweep(Conf cf, NodeCols nc, DevTables t, PopArgs a, PPSlot* slot,
                                                          KT* lists, uint32_t* arrive, uint32_t* fitw,
                                                          const PPCtrl* ctrl, uint32_t seq, uint32_t out_slot) {
    __shared__ KT wl[kPopThreads / 64][2][64];
    __shared__ int role;
    __shared__ uint32_t s_W;
    __shared__ uint32_t s_fitb[4];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const TaskClass c = t.classes[a.cls];
    uint32_t* fitc = arrive + (kMaxGroups + 1) * kCtrStride;
    if (threadIdx.x == 0) s_W = ld_sc1(&ctrl->written);  // before any row load; every row load below is sc1
    if (threadIdx.x < 4) s_fitb[threadIdx.x] = 0;
    __syncthreads();
    // 1. keys of R nodes per lane (rows through sc1), FitDelta nibbles, block top-128
    List2<KT> best{0, 0};
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int n = (blockIdx.x * R + r) * kPopThreads + threadIdx.x;
        KT k = 0;
        uint32_t fb = 0;
        if (n < nc.n) k = sweep_key<KT>(eval_node_sc1(cf, c, t, nc, n, &fb), a);
        uint32_t w = fb << ((lane & 7) * 4);
        w |= (uint32_t)__shfl_xor((int)w, 1, 64);
        w |= (uint32_t)__shfl_xor((int)w, 2, 64);
        w |= (uint32_t)__shfl_xor((int)w, 4, 64);
        if ((lane & 7) == 0 && n < nc.n) st_sc1(&fitw[n >> 3], w);
        fit_block_add(s_fitb, fb);
        const List2<KT> cur{wave_sort_desc(k), (KT)0};
        best = r == 0 ? cur : merge128(best, cur);
    }
    wl[wave][0][lane] = best.a;
    wl[wave][1][lane] = best.b;
    __syncthreads();
    tree_merge128(wl, wave, lane);
    const int nb = gridDim.x;
    const int g = blockIdx.x % kGroups;
    const int g_count = (nb - g + kGroups - 1) / kGroups;
    const int n_groups = nb < kGroups ? nb : kGroups;
    KT* glist = lists + (int64_t)nb * kPPK;
    if (wave == 0) {
        if (lane < 4 && s_fitb[lane])
            __hip_atomic_fetch_add(&fitc[g * kCtrStride + lane], s_fitb[lane], __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        if (lane == 0) __hip_atomic_fetch_max(&slot->Wn, ~s_W, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        put_list(lists + (int64_t)blockIdx.x * kPPK, wl[0][0][lane]);
        put_list(lists + (int64_t)blockIdx.x * kPPK + 64, wl[0][1][lane]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave's nibble / list stores and atomics
    __syncthreads();
    if (threadIdx.x == 0) role = atomicAdd(&arrive[g * kCtrStride], 1u) == (unsigned)(g_count - 1);
    __syncthreads();
    if (!role) return;
    // 2a. last block of group g: merge the group's block lists (4 loads in flight per wave)
    {
        List2<KT> acc{0, 0};
        constexpr int kPf = 4;
        for (int i0 = wave; i0 < g_count; i0 += kPf * (kPopThreads / 64)) {
            List2<KT> v[kPf];
#pragma unroll
            for (int q = 0; q < kPf; ++q) {
                const int i = i0 + q * (kPopThreads / 64);
                const KT* src = lists + (int64_t)(g + i * kGroups) * kPPK;
                v[q].a = i < g_count ? get_list(src) : (KT)0;
                v[q].b = i < g_count ? get_list(src + 64) : (KT)0;
            }
#pragma unroll
            for (int q = 0; q < kPf; ++q) acc = merge128(acc, v[q]);
        }
        wl[wave][0][lane] = acc.a;
        wl[wave][1][lane] = acc.b;
        __syncthreads();
        tree_merge128(wl, wave, lane);
        if (wave == 0) {
            put_list(glist + (int64_t)g * kPPK, wl[0][0][lane]);
            put_list(glist + (int64_t)g * kPPK + 64, wl[0][1][lane]);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) role = atomicAdd(&arrive[kGroups * kCtrStride], 1u) == (unsigned)(n_groups - 1);
        __syncthreads();
        if (!role) return;
    }
    // 2b. last group merger: the top-128, their rows, the FitDelta totals; publish
    {
        List2<KT> acc{0, 0};
        for (int gi = wave; gi < n_groups; gi += kPopThreads / 64) {
            const KT* src = glist + (int64_t)gi * kPPK;
            const List2<KT> v{get_list(src), get_list(src + 64)};
            acc = merge128(acc, v);
        }
        wl[wave][0][lane] = acc.a;
        wl[wave][1][lane] = acc.b;
    }
    __syncthreads();
    tree_merge128(wl, wave, lane);
    if (wave < 2) {  // wave w: entries 64 w + lane
        const uint64_t k = key64_of(wl[0][wave][lane], a);
        const int j = wave * 64 + lane;
        st_sc1(&slot->key[j], k);
        if (k) {
            const int n = key_idx(k);
            st_row_sc1(&slot->row[j], load_row_sc1(nc, n));
            for (int w = 0; w < 4; ++w)
                // the node's port words whatever this class asks: the placer keeps the row for later pops
                st_sc1(&slot->pw[j][w], (uint64_t)(w < port_win(c, nc) ? load_port_t<true>(nc, c.pw_lo + w, n) : 0ull));
            st_sc1(&slot->na[j], cf.score_mult ? na_weight(c, t, nc, n) : 0);
        }
    } else if (wave == 2) {
        if (lane < 4) {
            uint32_t f = 0;
            for (int gi = 0; gi < n_groups; ++gi) {
                f += ld_sc1(&fitc[gi * kCtrStride + lane]);
                st_sc1(&fitc[gi * kCtrStride + lane], 0u);
            }
            st_sc1(&slot->fit[lane], f);
        }
        if (lane <= kGroups) st_sc1(&arrive[lane * kCtrStride], 0u);
        const uint32_t* src = (const uint32_t*)&a;
        for (int i = lane; i < (int)(sizeof(PopArgs) / 4); i += 64) st_sc1(&((uint32_t*)&slot->a)[i], src[i]);
        if (lane == 0) {
            st_sc1(&slot->out_slot, out_slot);
            st_sc1(&slot->type, (uint32_t)PP_PLACE);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) st_sc1(&slot->seq, seq);
}

// A STOP command (host: end of a run of pops, before other device work).
__global__ void k_pp_post_stop(PPSlot* slot, uint32_t seq) {
    if (threadIdx.x == 0) {
        st_sc1(&slot->type, (uint32_t)PP_STOP);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        st_sc1(&slot->seq, seq);
    }
}

// ---------------------------------------------------------------------------
// the placer
// ---------------------------------------------------------------------------
struct PPHistEntry {
    uint32_t seq;
    PPHistOut o;
};

__global__ __launch_bounds__(kPopThreads) void k_pp_placer(Conf cf, NodeCols nc, DevTables t, PPSlot* ring,
                                                           PPCtrl* ctrl, char* outs, const uint32_t* fitw_base,
                                                           int64_t fitw_words, PPHost* host, uint32_t seq0) {
    __shared__ PPHistEntry hist[kPPHist];
    __shared__ RowCache rc;
    __shared__ uint64_t wl[kPopThreads / 64][64];
    __shared__ int32_t s_dk[kPPDHash];   // dirty node -> latest history position (entry * 64 + index)
    __shared__ int32_t s_dv[kPPDHash];
    __shared__ int32_t s_dn[kPPHist * 64];
    __shared__ int32_t s_nd;
    __shared__ uint32_t s_cmd[4];
    __shared__ int32_t s_fitin[4];
    __shared__ PopArgs s_a;
    __shared__ uint64_t s_t0;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (threadIdx.x < kPPHist) hist[threadIdx.x].seq = 0;
    if (threadIdx.x < 16) pp_ts[threadIdx.x] = 0;
    uint64_t tp[7] = {};  // thread 0: phase sums of this launch (added to ctrl->prof when it leaves)
    uint64_t tm = __builtin_amdgcn_s_memrealtime();
    auto mark = [&](int k) {
        if (threadIdx.x == 0) {
            const uint64_t x = __builtin_amdgcn_s_memrealtime();
            tp[k] += x - tm;
            tm = x;
        }
    };
    for (uint32_t e = seq0;; ++e) {
        PPSlot* sl = ring + (e % kPPSlots);
        // 1. wait for command e (thread 0 polls; the other waves load after the barrier)
        if (threadIdx.x == 0) {
            const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
            uint32_t st = 0;
            for (;;) {
                if (ld_sc1(&sl->seq) == e) { st = 1; break; }
                if (__builtin_amdgcn_s_memrealtime() - t_start > kPPIdle) { st = 2; break; }
                __builtin_amdgcn_s_sleep(1);
            }
            s_cmd[0] = st;
            if (st == 1) {
                s_cmd[1] = ld_sc1(&sl->type);
                s_cmd[2] = ~ld_sc1(&sl->Wn);
                s_cmd[3] = ld_sc1(&sl->out_slot);
            }
        }
        for (int i = threadIdx.x; i < kPPDHash; i += kPopThreads) { s_dk[i] = -1; s_dv[i] = -1; }
        for (int i = threadIdx.x; i < kHash; i += kPopThreads) rc.hkey[i] = -1;
        if (threadIdx.x == 0) s_nd = 0;
        if (threadIdx.x < 4) s_fitin[threadIdx.x] = 0;
        __syncthreads();
        mark(0);
        if (s_cmd[0] != 1 || s_cmd[1] != PP_PLACE) {  // idle or STOP: leave; `consumed` says where
            if (threadIdx.x == 0) {
                for (int k = 0; k < 7; ++k) ctrl->prof[k] += tp[k];
                for (int k = 0; k < 15; ++k) ctrl->pprof[k] += pp_ts[k];
                if (s_cmd[0] == 1) st_sc1(&ctrl->written, e);  // a STOP is applied by leaving
                __hip_atomic_store(&host->consumed, s_cmd[0] == 1 ? e + 1 : e, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store(&host->exited, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            return;
        }
        const uint32_t W = s_cmd[2];
        PopOut* out = (PopOut*)(outs + (size_t)s_cmd[3] * sizeof(PopOut));
        // 2. the list, its rows and the arguments (in flight while the dirty set is built)
        uint64_t lk = 0;  // waves 0, 1: list entry 64 wave + lane
        Row lrow{};
        uint64_t lpw[4] = {0, 0, 0, 0};
        int32_t lna = 0;
        if (wave < 2) {
            const int j = wave * 64 + lane;
            lk = ld_sc1(&sl->key[j]);
            lrow = ld_row_sc1(&sl->row[j]);
            for (int w = 0; w < 4; ++w) lpw[w] = ld_sc1(&sl->pw[j][w]);
            lna = ld_sc1(&sl->na[j]);
        } else if (wave == 2) {
            for (int i = lane; i < (int)(sizeof(PopArgs) / 4); i += 64)
                ((uint32_t*)&s_a)[i] = ld_sc1(&((const uint32_t*)&sl->a)[i]);
            if (lane < 4) s_fitin[lane] = 0;
            if (lane == 4) s_t0 = ld_sc1(&sl->key[kPPK - 1]);
        }
        // 3. the dirty set: nodes committed by pops W+1 .. e-1 (latest row wins)
        bool broken = W >= e || (e - 1) - W > (uint32_t)kPPHist;  // W <= e - 1; at most kPPHist pops behind
        if (!broken)
            for (uint32_t p = W + 1; p < e; ++p) broken = broken || hist[p % kPPHist].seq != p;
        if (!broken && threadIdx.x < kPPHist * 64) {
            const int hi = threadIdx.x >> 6, q = threadIdx.x & 63;
            const uint32_t ps = hist[hi].seq;
            if (ps > W && ps + 1 <= e && q < hist[hi].o.n) {
                const int n = hist[hi].o.node[q];
                const int val = (int)((ps - W) << 12) | (hi << 6) | q;  // later pops win
                int h = (int)(((uint32_t)n * 2654435761u) >> 22);
                for (;;) {
                    const int prev = atomicCAS(&s_dk[h], -1, n);
                    if (prev == -1) {
                        s_dn[atomicAdd(&s_nd, 1)] = n;
                        atomicMax(&s_dv[h], val);
                        break;
                    }
                    if (prev == n) { atomicMax(&s_dv[h], val); break; }
                    h = (h + 1) & (kPPDHash - 1);
                }
            }
        }
        __syncthreads();
        const PopArgs a = s_a;
        const TaskClass c = t.classes[a.cls];
        const uint64_t t0 = s_t0;
        auto dirty_slot = [&](int n) -> int {  // history position of dirty node n, -1 if clean
            int h = (int)(((uint32_t)n * 2654435761u) >> 22);
            for (int i = 0; i < kPPDHash; ++i, h = (h + 1) & (kPPDHash - 1)) {
                const int k = s_dk[h];
                if (k == n) return s_dv[h] & 0xfff;
                if (k == -1) return -1;
            }
            return -1;
        };
        // 4. candidate keys: the list's clean entries (waves 0, 1), the dirty nodes re-evaluated (waves 2..5)
        uint64_t ck = 0;
        if (!broken) {
            if (wave < 2) {
                const int n = lk ? key_idx(lk) : -1;
                if (n >= 0 && dirty_slot(n) < 0) ck = lk;
            } else if (wave < 2 + kPPHist) {
                const int i = (wave - 2) * 64 + lane;
                if (i < s_nd) {
                    const int n = s_dn[i];
                    const int hp = dirty_slot(n);
                    const Row& r = hist[hp >> 6].o.row[hp & 63];
                    const uint64_t* pw = hist[hp >> 6].o.pw[hp & 63];
                    const bool stp = static_pred(cf, c, t, nc, n);
                    const int32_t na = (stp && cf.score_mult) ? na_weight(c, t, nc, n) : 0;
                    int32_t sc;
                    bool passed;
                    ck = dyn_key(cf, c, t, nc, r, pw, n, stp, na, &sc, &passed);
                }
            }
        }
        mark(1);
        // sorted per wave, merged: wl[0] = top-64 candidate keys
        wl[wave][lane] = wave_sort_desc(ck);
        __syncthreads();
        block_tree_merge(wl, wave, lane);
        mark(2);
        // 5. rows of the candidates into the row cache (slot = candidate position):
        // dirty ones from the history, clean ones from the list (registers of waves 0, 1)
        if (wave == 0) {
            const uint64_t k = wl[0][lane];
            const int n = k ? key_idx(k) : -1;
            if (n >= 0) {
                const int hp = dirty_slot(n);
                if (hp >= 0) {
                    rc.row[lane] = hist[hp >> 6].o.row[hp & 63];
                    for (int w = 0; w < 4; ++w) rc.pw[lane][w] = hist[hp >> 6].o.pw[hp & 63][w];
                    rc.na[lane] = cf.score_mult && static_pred(cf, c, t, nc, n) ? na_weight(c, t, nc, n) : 0;
                }
                rc_insert(&rc, n, lane);
            }
        }
        __syncthreads();
        if (wave < 2 && lk) {  // clean list nodes that are candidates: their rows from the list
            const int n = key_idx(lk);
            const int slot_c = rc_find(&rc, n);
            if (slot_c >= 0 && dirty_slot(n) < 0) {
                rc.row[slot_c] = lrow;
                for (int w = 0; w < 4; ++w) rc.pw[slot_c][w] = lpw[w];
                rc.na[slot_c] = lna;
            }
        }
        __syncthreads();
        // 6. FitDelta corrections for the dirty nodes (used only if a task finds no node)
        if (!broken && wave >= 2 && wave < 2 + kPPHist) {
            const int i = (wave - 2) * 64 + lane;
            if (i < s_nd) {
                const int n = s_dn[i];
                const int hp = dirty_slot(n);
                const Row& r = hist[hp >> 6].o.row[hp & 63];
                const uint32_t sw = (n >> 3) < fitw_words
                    ? (ld_sc1(&fitw_base[(int64_t)(e % kPPSlots) * fitw_words + (n >> 3)]) >> ((n & 7) * 4)) & 15u
                    : 0u;
                uint32_t now;
                if (rc_find(&rc, n) >= 0) {
                    now = fit_bits(c, r, true);  // a candidate: place_parallel counts it from here
                } else {
                    const bool stp = static_pred(cf, c, t, nc, n);
                    const int32_t na = (stp && cf.score_mult) ? na_weight(c, t, nc, n) : 0;
                    int32_t sc;
                    bool passed;
                    (void)dyn_key(cf, c, t, nc, r, hist[hp >> 6].o.pw[hp & 63], n, stp, na, &sc, &passed);
                    now = fit_bits(c, r, passed);
                }
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    const int d = (int)((now >> b) & 1u) - (int)((sw >> b) & 1u);
                    if (d) atomicAdd(&s_fitin[b], d);
                }
            }
        }
        uint32_t fit_raw = 0;
        if (wave == 0 && lane < 4) fit_raw = ld_sc1(&sl->fit[lane]);
        __syncthreads();
        mark(3);
        if (threadIdx.x == 0) pp_ts[15] = __builtin_amdgcn_s_memrealtime();
        // 7. place; rows written back sc1, then written = e; history entry e
        PPHistEntry& he = hist[e % kPPHist];
        if (broken) {  // the sweep saw rows older than the history: the host sweeps this pop again
            if (wave == 0) {
                if (lane == 0) {
                    he.o.n = 0;
                    st_sc1(&ctrl->written, e);
                    __hip_atomic_store(&out->g[0], make_granule(a.epoch, 0, 0, 0, -1), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_SYSTEM);
                }
            }
        } else if (a.ent32) {  // the entry width follows the class's key format
            place_parallel<uint32_t, true, true>(cf, nc, t, c, a, out, wl, &ctrl->written, e, &rc, s_fitin, fit_raw,
                                                 0, 0x7fffffff, t0, &he.o);
        } else {
            place_parallel<uint64_t, true, true>(cf, nc, t, c, a, out, wl, &ctrl->written, e, &rc, s_fitin, fit_raw,
                                                 0, 0x7fffffff, t0, &he.o);
        }
        __syncthreads();
        mark(4);
        if (threadIdx.x == 0) {
            tp[6] += 1;
            he.seq = e;
            st_sc1(&sl->Wn, 0u);  // the slot's next sweep starts its minimum afresh
            __hip_atomic_store(&host->consumed, e + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        __syncthreads();
        mark(5);
    }
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
size_t pp_slot_bytes() { return sizeof(PPSlot); }
size_t pp_ctrl_bytes() { return sizeof(PPCtrl); }
size_t pp_host_bytes() { return sizeof(PPHost); }
int pp_slots() { return kPPSlots; }
size_t pp_list_keys(int n_nodes) {
    int R;
    const int nb = pop_blocks(n_nodes, &R);
    return (size_t)(nb + kMaxGroups) * kPPK;
}
size_t pp_arrive_words() { return (size_t)(2 * kMaxGroups + 1) * kCtrStride; }

hipError_t launch_pp_sweep(const Conf& cf, const NodeCols& nc, const DevTables& t, int cls, int n_tasks,
                           int gang_mode, int min_avail, int ready_count, uint32_t epoch, const KeyFormat& kf,
                           void* ring, void* lists, uint32_t* arrive, uint32_t* fitw, const void* ctrl, uint32_t seq,
                           uint32_t out_slot, hipStream_t st) {
    int R;
    const int nb = pop_blocks(nc.n, &R);
    PopArgs a{cls, n_tasks, gang_mode, min_avail, ready_count, epoch, 5, kf.base, kf.shift, kf.idxmax,
              kf.use32 && kf.ent32 ? 1 : 0, 0};
    PPSlot* slot = (PPSlot*)ring + (seq % kPPSlots);
    const PPCtrl* c = (const PPCtrl*)ctrl;
#define KBHIP_PPS(RR, KT) \
    hipLaunchKernelGGL((k_pp_sweep<RR, KT>), dim3(nb), dim3(kPopThreads), 0, st, cf, nc, t, a, slot, (KT*)lists, arrive, fitw, c, seq, out_slot)
#define KBHIP_PPR(KT)                       \
    switch (R) {                            \
        case 1: KBHIP_PPS(1, KT); break;    \
        case 2: KBHIP_PPS(2, KT); break;    \
        case 4: KBHIP_PPS(4, KT); break;    \
        case 8: KBHIP_PPS(8, KT); break;    \
        default: KBHIP_PPS(16, KT); break;  \
    }
    if (kf.use32) { KBHIP_PPR(uint32_t); }
    else { KBHIP_PPR(uint64_t); }
#undef KBHIP_PPR
#undef KBHIP_PPS
    return hipGetLastError();
}

hipError_t launch_pp_placer(const Conf& cf, const NodeCols& nc, const DevTables& t, void* ring, void* ctrl, void* outs,
                            const uint32_t* fitw, int64_t fitw_words, void* host, uint32_t seq0, hipStream_t st) {
    hipLaunchKernelGGL(k_pp_placer, dim3(1), dim3(kPopThreads), 0, st, cf, nc, t, (PPSlot*)ring, (PPCtrl*)ctrl,
                       (char*)outs, fitw, fitw_words, (PPHost*)host, seq0);
    return hipGetLastError();
}

hipError_t launch_pp_stop(void* ring, uint32_t seq, hipStream_t st) {
    hipLaunchKernelGGL(k_pp_post_stop, dim3(1), dim3(64), 0, st, (PPSlot*)ring + (seq % kPPSlots), seq);
    return hipGetLastError();
}

}  // namespace kbhip
