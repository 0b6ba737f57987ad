// engine_placer.h — the placer (decision, write-back, the next pop's front)
// and the dispatcher, shared by both engine kernels.
#pragma once
#include <hip/hip_runtime.h>

#define KBHIP_STAMPS_OFF  // phase stamps belong to k_pop_batch (kbhip_kernels.hip)
#include "../kbhip_batch.h"
#include "../kbhip_engine.h"
#include "engine_dev.h"

namespace kbhip {

// ---------------------------------------------------------------------------
// placer
// ---------------------------------------------------------------------------
static_assert(sizeof(Row) == 4 * (kPkFlags - kPkRow), "the package carries a Row as 28 32-bit words");
static_assert(kEngDescClass + sizeof(TaskClass) / 4 <= kEngDescWords, "a descriptor carries its class");

// Candidate j's row after the chunk's commits (place_row) from its row before
// (`base`: the placer's row cache — the decision does not keep its copy live).
template <typename ET>
__device__ __forceinline__ Row eng_row_after(const TaskClass& c, const PlaceDec<ET>& D, const Row& base) {
    // branch-free (no commits: zero of each): a Row chosen between two branches is copied
    // through the stack, and its reload waits for every store in flight
    const int cc = D.cc > 0 ? D.cc : 0;
    const int na = cc < D.ap_l ? cc : D.ap_l;
    return apply_commits(base, c, na, cc - na);
}
// place_fit_vals for engine classes (no host ports), the row before from the cache.
template <typename ET>
__device__ __forceinline__ void eng_fit_vals(const Conf& cf, const NodeCols& nc, const DevTables& t,
                                             const TaskClass& c, const PopArgs& a, const PlaceDec<ET>& D,
                                             const Row& base, const int32_t* fit_in, uint32_t fit_raw, uint64_t* g0,
                                             uint64_t* g1) {
    uint32_t fb_base = 0, fb_post = 0;
    if (D.n >= 0) {
        fb_base = fit_bits(c, base, true);  // candidates had a key: in the walk
        const Row r = eng_row_after(c, D, base);
        const uint64_t pw[4] = {0, 0, 0, 0};
        int32_t sc;
        bool passed;
        (void)dyn_key(cf, c, t, nc, r, pw, D.n, true, D.na_n, &sc, &passed);
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

// The placer's wave 0 after the decision: the FitDelta histogram of a task
// that found no node (the sweep's counts from the group count words), the
// result granules into LDS for wave 5 (which stores them to the host: the
// system-scope stores' completion never holds up a wait of this wave), the
// chunk's rows into the cache (ring r0) and, write-through, into the node
// columns.  The row stores are left in flight: the next pop drains them
// before it publishes its candidates, and only then raises `done` for this
// pop (*pend).
template <bool LIST, typename ET>
__device__ __forceinline__ void eng_finish(const Conf& cf, const NodeCols& nc, const DevTables& t, const TaskClass& c,
                                           const PopArgs& a, const EngArgs& A, EngPlacerLds& L, uint32_t p, int r0,
                                           const PlaceDec<ET>& D, uint32_t* pend) {
    const int lane = threadIdx.x & 63;
    EngCtl* ctl = A.ctl;
    uint64_t g0 = 0, g1 = 0;
    if (D.stop == 1) {
        uint32_t fr = 0;  // group g's count b in lane 4g + b (fit_sum layout)
        const int g = lane >> 2;
        if constexpr (LIST) {  // list mode: the class owner's four count words (count b in lane b)
            const uint64_t* s = A.blists + (size_t)(p % kEngSlots) * kEngListWords + 128 + (lane & 3);
            uint64_t x = lane < 4 ? ld_sc1(s) : ((uint64_t)p << 32);
            EngWait wt(ctl, kEngWaitTicks);
            while (__ballot((uint32_t)(x >> 32) != p) != 0) {
                if (!wt.tick()) break;
                if (lane < 4) x = ld_sc1(s);
            }
            fr = lane < 4 ? (uint32_t)x : 0u;
        } else if (A.ng == 0) {  // the worker count words: two 16-bit counts each, count b in lane b
            uint32_t t0 = 0, t1 = 0, t2 = 0, t3 = 0;
            for (int i0 = 0; i0 < A.nw; i0 += 64) {
                const int i = i0 + lane;
                const uint64_t* s =
                    i < A.nw ? A.blists + ((size_t)(p % kEngSlots) * A.nw + i) * kEngListWords + 128 : nullptr;
                uint64_t x0 = s ? ld_sc1(&s[0]) : ((uint64_t)p << 32), x1 = s ? ld_sc1(&s[1]) : ((uint64_t)p << 32);
                EngWait wt(ctl, kEngWaitTicks);
                while (__ballot((uint32_t)(x0 >> 32) != p || (uint32_t)(x1 >> 32) != p) != 0) {
                    if (!wt.tick()) break;
                    if (s) { x0 = ld_sc1(&s[0]); x1 = ld_sc1(&s[1]); }
                }
                const uint32_t y0 = (uint32_t)x0, y1 = (uint32_t)x1;
                t0 += wave_sum_u32(y0 & 0xffff);
                t1 += wave_sum_u32(y0 >> 16);
                t2 += wave_sum_u32(y1 & 0xffff);
                t3 += wave_sum_u32(y1 >> 16);
            }
            fr = lane == 0 ? t0 : lane == 1 ? t1 : lane == 2 ? t2 : lane == 3 ? t3 : 0u;
        } else if (g < A.ng) {
            const uint64_t* s = A.glists + ((size_t)(p % kEngSlots) * A.ng + g) * kEngListWords + 128 + (lane & 3);
            uint64_t x = ld_sc1(s);
            EngWait wt(ctl, kEngWaitTicks);
            while (__ballot((uint32_t)(x >> 32) != p) != 0) {
                if (!wt.tick()) break;
                x = ld_sc1(s);
            }
            fr = (uint32_t)x;
        }
        eng_fit_vals(cf, nc, t, c, a, D, L.rc.row[L.srcslot[lane]], L.fitin, fr, &g0, &g1);
    }
    ETL(A, p, 47);
    L.gran[lane] = place_granule_val(a, D);
    if (lane == 0) { L.gfit[0] = g0; L.gfit[1] = g1; }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the granules are in LDS before the flag
    if (lane == 0) __hip_atomic_store(&L.gran_seq, (int)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    const int n = D.n;
    {
        const int cc = D.cc > 0 ? D.cc : 0;
        const int na = cc < D.ap_l ? cc : D.ap_l;
        L.ccm[lane] = n >= 0 ? (na | ((cc - na) << 8)) : 0;
    }
    if (n >= 0) {  // every candidate's row after the chunk into ring r0 (the next three pops re-evaluate them;
                   // from its row before in the cache, not the decision's copy)
        const int src = L.srcslot[lane];
        L.rc.row[64 * r0 + lane] = eng_row_after(c, D, L.rc.row[src]);
        L.flags[64 * r0 + lane] = L.flags[src];
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the rows are in LDS before the flag (the front reads them)
    if (lane == 0) __hip_atomic_store(&L.rows_seq, (int)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    ETL(A, p, 27);
    if (n >= 0 && D.cc > 0) {
        const Row r = L.rc.row[64 * r0 + lane];
        st_sc1(&nc.idle_cpu[n], r.idle_cpu); st_sc1(&nc.idle_mem[n], r.idle_mem); st_sc1(&nc.idle_gpu[n], r.idle_gpu);
        st_sc1(&nc.rel_cpu[n], r.rel_cpu); st_sc1(&nc.rel_mem[n], r.rel_mem); st_sc1(&nc.rel_gpu[n], r.rel_gpu);
        st_sc1(&nc.pods[n], r.pods);
        st_sc1(&nc.nzc[n], r.nzc);
        st_sc1(&nc.nzm[n], r.nzm);
    }
    ETL(A, p, 7);
    *pend = p;
}

// Wave 0: drain this wave's stores (the write-back of pop *pend), then raise `done`.
__device__ __forceinline__ void eng_publish_done(EngCtl* ctl, uint32_t* pend) {
    if (!*pend) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if ((threadIdx.x & 63) == 0) st_sc1(&ctl->done, *pend);
    *pend = 0;
}

// Wave 0 (list mode): until every owner has applied pop `want` (L.apmin: the
// owners' minimum as last read).  false: the wait gave up.
__device__ __forceinline__ bool eng_own_apmin(const EngArgs& A, EngPlacerLds& L, uint32_t want) {
    const int lane = threadIdx.x & 63;
    EngWait wt(A.ctl, kEngWaitTicks);
    for (;;) {
        uint32_t m = 0xffffffffu;  // the minimum of (ap - want) as signed distances, biased
        for (int o = lane; o < A.nown; o += 64) {
            const uint32_t d = ld_sc1(&A.ctl->own_ap[o]) - want + 0x80000000u;
            m = d < m ? d : m;
        }
#pragma unroll
        for (int dd = 1; dd < 64; dd <<= 1) {
            const uint32_t u = (uint32_t)__shfl_xor((int)m, dd, 64);
            m = u < m ? u : m;
        }
        const uint32_t mn = m - 0x80000000u + want;  // the owners' minimum
        if (lane == 0) L.apmin = mn;
        if ((int32_t)(mn - want) >= 0) return true;
        if (!wt.tick()) return false;
    }
}

// Wave 5: pop p's result granules (from LDS, eng_finish) to the host's pinned slot.
__device__ __forceinline__ void eng_host_out(const EngArgs& A, EngPlacerLds& L, uint32_t p, uint32_t slot) {
    const int lane = threadIdx.x & 63;
    while (__hip_atomic_load(&L.gran_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != (int)p) {
        if (!__hip_atomic_load(&L.ok, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) return;
        __builtin_amdgcn_s_sleep(1);
    }
    PopOut* out = (PopOut*)((char*)A.out + (size_t)slot * sizeof(PopOut));
    const uint64_t g = L.gran[lane];
    if (lane < 2 && L.gfit[lane])
        __hip_atomic_store(&out->fit[lane], L.gfit[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (g) __hip_atomic_store(&out->g[lane], g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    ETL(A, p, 8);
}

// One wave: pop q's package keys without pop q-1's candidates (stale: the
// workers evaluated them before pop q-1 placed; at most 64 of 128, so the
// first 64 left are exact) into L.s64, the kept entries' rows hashed into the
// row cache.  Needs the front's hash of pops q-1..q-3's candidates.
__device__ __forceinline__ void eng_drop_stale(EngPlacerLds& L, const PopArgs& a, uint32_t q) {
    const int lane = threadIdx.x & 63;
    EngRowCache& rc = L.rc;
    const int r1 = (int)((q + 3) % 4);
    const int stage = kEngStage + kEngPkgN * (int)(q % 2);
    L.s64[lane] = 0;
    const uint32_t k0 = L.pkey[q % 2][lane], k1 = L.pkey[q % 2][64 + lane];
    auto kept = [&](uint32_t k) {
        if (!k) return false;
        const int sl = rc_find(&rc, key_node(k, a));
        return !(sl >= 64 * r1 && sl < 64 * r1 + 64);
    };
    const bool c0 = kept(k0), c1 = kept(k1);
    const uint64_t m0 = __ballot(c0), m1 = __ballot(c1);
    const int q0 = __builtin_amdgcn_mbcnt_hi((uint32_t)(m0 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m0, 0));
    const int q1 = __popcll(m0) +
                   __builtin_amdgcn_mbcnt_hi((uint32_t)(m1 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m1, 0));
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    if (c0) L.s64[q0] = k0;
    if (c1 && q1 < 64) L.s64[q1] = k1;
    // the kept nodes' rows: their package entries
    if (c0) rc_insert(&rc, key_node(k0, a), stage + lane);
    if (c1 && q1 < 64) rc_insert(&rc, key_node(k1, a), stage + 64 + lane);
}

// Role 0 of one candidate on row r: its key, FitDelta bits, key kind, node-affinity
// weight, and (kind 2) the depth-1 score after a Pipeline.
struct FrontKey {
    uint32_t e, fb, kind;
    int32_t na, s1p;
};
__device__ __forceinline__ FrontKey front_key(const Conf& cf, const NodeCols& nc, const DevTables& t,
                                              const TaskClass& c, const PopArgs& a, int node, const Row& r,
                                              uint8_t fl) {
    FrontKey k{0u, 0u, 0u, 0, INT32_MIN};
    const uint64_t pw[4] = {0, 0, 0, 0};
    int32_t sc;
    bool passed;
    const bool st = static_pred_f(cf, c, t, nc, node, fl);
    k.na = (st && cf.score_mult) ? na_weight(c, t, nc, node) : 0;
    const uint64_t k0 = dyn_key(cf, c, t, nc, r, pw, node, st, k.na, &sc, &passed);
    k.e = sweep_key<uint32_t>(k0, a);
    k.fb = fit_bits(c, r, passed);
    k.kind = k0 ? key_kind(k0) : 0;
    if (__ballot(k.kind == 2) != 0 && k.kind == 2) {  // (rare)
        const uint64_t k1 = dyn_key(cf, c, t, nc, apply_commits(r, c, 0, 1), pw, node, true, k.na, &sc, &passed);
        k.s1p = k1 ? key_score(k1) : INT32_MIN;
    }
    return k;
}
// Role 1: the depth-1 score after an Allocate on row r.
__device__ __forceinline__ int32_t front_s1a(const Conf& cf, const NodeCols& nc, const DevTables& t,
                                             const TaskClass& c, int node, const Row& r) {
    const uint64_t pw[4] = {0, 0, 0, 0};
    int32_t sc;
    bool passed;
    const int32_t na = cf.score_mult ? na_weight(c, t, nc, node) : 0;
    const uint64_t k1 = dyn_key(cf, c, t, nc, apply_commits(r, c, 1, 0), pw, node, true, na, &sc, &passed);
    return k1 ? key_score(k1) : INT32_MIN;
}
__device__ __forceinline__ bool front_wait(const EngPlacerLds& L, const int* seq, int want) {
    while (__hip_atomic_load(seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != want) {
        if (!__hip_atomic_load(&L.ok, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) return false;
        __builtin_amdgcn_s_sleep(1);
    }
    return true;
}

// Pop q's previous candidates, evaluated during pop q-1's placement by waves
// it leaves idle: set s = pop q-1-s's candidates (ring (q + 3 - s) % 4); role 0
// the key (static predicates, node-affinity weight, FitDelta bits, kind), 1 the
// depth-1 score after an Allocate (after a Pipeline: with role 0, for the rare
// keys of that kind).  Into the front arrays (fe, ...): pop q-1's placement
// still reads the row cache's na / s1 of the older slots; pop q's P2 moves the
// ones that count there.  Set 0's rows are pop q-1's results: its candidates are
// evaluated ahead of that decision on their rows before it (variant 0, here)
// and after one Allocate of its class (variant 1, eng_front_v1, another wave);
// once the decision is in (L.rows_seq) each lane takes the variant of its
// commits (L.ccm), or evaluates its final row (two or more commits, a Pipeline).
template <bool LIST>
__device__ __forceinline__ void eng_front_eval(const Conf& cf, const NodeCols& nc, const DevTables& t,
                                               const EngArgs& A, EngPlacerLds& L, uint32_t q, uint32_t dw, int set,
                                               int role) {
    const int lane = eng_lane();
    uint32_t w[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = (uint32_t)__builtin_amdgcn_readlane((int)dw, i);
    const EngDesc d = eng_decode(w);
    const PopArgs a = eng_args(d);
    const TaskClass c = eng_class_x(dw);
    const int ring = (int)((q + 3 - set) % 4);
    const int sl = 64 * ring + lane;
    if (!LIST && set == 0) {  // sweep mode: pop q-1's candidates on their final rows (its decision)
        if (!front_wait(L, &L.rows_seq, (int)(q - 1))) return;
        const int node = L.xn[ring][lane];
        if (role == 0) {
            ETL(A, q - 1, 32);
            FrontKey k{0u, 0u, 0u, 0, INT32_MIN};
            if (node >= 0) k = front_key(cf, nc, t, c, a, node, L.rc.row[sl], L.flags[sl]);
            ETL(A, q - 1, 33);
            L.fe[0][lane] = k.e;
            L.ffb[0][lane] = (uint8_t)k.fb;
            L.fkind[0][lane] = (uint8_t)k.kind;
            L.fna[0][lane] = k.na;
            if (k.kind == 2) L.fs1p[0][lane] = k.s1p;
            ETL(A, q - 1, 34);
            L.e[0][lane] = wave_sort_desc(node >= 0 ? k.e : 0u);
            L.fbp[0][lane] = node >= 0 ? (uint8_t)k.fb : (uint8_t)0;
            __builtin_amdgcn_s_waitcnt(0xc07f);
            if (lane == 0) __hip_atomic_store(&L.sort_seq[0], (int)q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            ETL(A, q - 1, 35);
        } else if (node >= 0) {
            L.fs1a[0][lane] = front_s1a(cf, nc, t, c, node, L.rc.row[sl]);
        }
        return;
    }
    if (set == 0) {  // list mode: pop q-1's candidates (its P3): their rows before it, both variants
        if (!front_wait(L, &L.xn_seq, (int)(q - 1))) return;
        const int node = L.xn[ring][lane];
        const int src = node >= 0 ? L.srcslot[lane] : 0;
        // (a row P3 had to load into this pop's own ring is overwritten by the decision: final row only)
        const bool own_ring = src >= 64 * ring && src < 64 * ring + 64;
        if (role == 0) {
            FrontKey k{0u, 0u, 0u, 0, INT32_MIN};
            if (node >= 0) k = front_key(cf, nc, t, c, a, node, L.rc.row[src], L.flags[src]);
            if (!front_wait(L, &L.rows_seq, (int)(q - 1))) return;
            ETL(A, q - 1, 32);
            const int m = L.ccm[lane];
            if (m == 1 && node >= 0 && !own_ring) {  // one Allocate: variant 1
                if (!front_wait(L, &L.v1_seq[0], (int)q)) return;
                k.e = L.v1e[lane]; k.fb = L.v1fb[lane]; k.kind = L.v1kind[lane]; k.s1p = L.v1s1p[lane];
            }
            const bool slow = node >= 0 && (m > 1 || own_ring);  // two or more commits, or a Pipeline: the final row
            if (__ballot(slow) != 0 && slow) k = front_key(cf, nc, t, c, a, node, L.rc.row[sl], L.flags[sl]);
            ETL(A, q - 1, 33);
            L.fe[0][lane] = k.e;
            L.ffb[0][lane] = (uint8_t)k.fb;
            L.fkind[0][lane] = (uint8_t)k.kind;
            L.fna[0][lane] = k.na;
            if (k.kind == 2) L.fs1p[0][lane] = k.s1p;
            ETL(A, q - 1, 34);
            L.e[0][lane] = wave_sort_desc(node >= 0 ? k.e : 0u);
            L.fbp[0][lane] = node >= 0 ? (uint8_t)k.fb : (uint8_t)0;
            __builtin_amdgcn_s_waitcnt(0xc07f);
            if (lane == 0) __hip_atomic_store(&L.sort_seq[0], (int)q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            ETL(A, q - 1, 35);
        } else {
            int32_t s1 = INT32_MIN;
            if (node >= 0) s1 = front_s1a(cf, nc, t, c, node, L.rc.row[src]);
            if (!front_wait(L, &L.rows_seq, (int)(q - 1))) return;
            const int m = L.ccm[lane];
            if (m == 1 && node >= 0 && !own_ring) {
                if (!front_wait(L, &L.v1_seq[1], (int)q)) return;
                s1 = L.v1s1a[lane];
            }
            const bool slow = node >= 0 && (m > 1 || own_ring);
            if (__ballot(slow) != 0 && slow) s1 = front_s1a(cf, nc, t, c, node, L.rc.row[sl]);
            if (node >= 0) L.fs1a[0][lane] = s1;
        }
        return;
    }
    if (role == 0) ETL(A, q - 1, 32 + 4 * set);  // timeline (pop q-1's slot): set s's key at events 32 + 4 s ..
    const int node = L.xn[ring][lane];
    if (role == 0) {
        FrontKey k{0u, 0u, 0u, 0, INT32_MIN};
        if (node >= 0) k = front_key(cf, nc, t, c, a, node, L.rc.row[sl], L.flags[sl]);
        ETL(A, q - 1, 33 + 4 * set);
        L.fe[set][lane] = k.e;
        L.ffb[set][lane] = (uint8_t)k.fb;
        L.fkind[set][lane] = (uint8_t)k.kind;
        L.fna[set][lane] = k.na;
        if (k.kind == 2) L.fs1p[set][lane] = k.s1p;
        // the set's keys that count (not a later set's node, from wave 2's hash) sorted for
        // pop q's P3, and their FitDelta bits; else the placer's P2 does it
        bool hashed = false;
        for (int i = 0; i < 4096 && !hashed; ++i) {
            hashed = __hip_atomic_load(&L.hash_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == (int)q;
            if (!hashed) __builtin_amdgcn_s_sleep(1);
        }
        ETL(A, q - 1, 34 + 4 * set);
        if (hashed) {
            const bool use = node >= 0 && (set == 1 ? L.x2use[lane] : L.x3use[lane]);
            L.e[set][lane] = wave_sort_desc(use ? k.e : 0u);
            L.fbp[set][lane] = use ? (uint8_t)k.fb : (uint8_t)0;
            __builtin_amdgcn_s_waitcnt(0xc07f);
            if (lane == 0) __hip_atomic_store(&L.sort_seq[set], (int)q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            ETL(A, q - 1, 35 + 4 * set);
        }
    } else if (node >= 0) {
        L.fs1a[set][lane] = front_s1a(cf, nc, t, c, node, L.rc.row[sl]);
    }
}

// Variant 1 of set 0 (eng_front_eval): pop q-1's candidates after one Allocate of
// its class, role 0 (key) or 1 (depth-1 score), into L.v1*; then L.v1_seq[role] = q.
__device__ __forceinline__ void eng_front_v1(const Conf& cf, const NodeCols& nc, const DevTables& t,
                                             EngPlacerLds& L, uint32_t q, uint32_t dw, int role) {
    const int lane = eng_lane();
    uint32_t w[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = (uint32_t)__builtin_amdgcn_readlane((int)dw, i);
    const PopArgs a = eng_args(eng_decode(w));
    const TaskClass c = eng_class_x(dw);
    if (!front_wait(L, &L.xn_seq, (int)(q - 1))) return;
    const TaskClass& cp = *(const TaskClass*)&L.desc[(q - 1) % 2][kEngDescClass];  // pop q-1's class
    const int ring = (int)((q + 3) % 4);
    const int node = L.xn[ring][lane];
    if (node >= 0) {
        const int src = L.srcslot[lane];
        const Row r = apply_commits(L.rc.row[src], cp, 1, 0);
        if (role == 0) {
            const FrontKey k = front_key(cf, nc, t, c, a, node, r, L.flags[src]);
            L.v1e[lane] = k.e; L.v1fb[lane] = (uint8_t)k.fb; L.v1kind[lane] = (uint8_t)k.kind; L.v1s1p[lane] = k.s1p;
        } else {
            L.v1s1a[lane] = front_s1a(cf, nc, t, c, node, r);
        }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    if (lane == 0) __hip_atomic_store(&L.v1_seq[role], (int)q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Pop q's front, by waves: 2 the hash of pops q-1 / q-2 / q-3's candidates
// (node -> latest row slot), 1, 2, 3, 5, 6, 7 the evaluation of pops q-2 /
// q-3's candidates (eng_front_eval; wave 0's SIMD left to the placement),
// then 3, 4, 6, 7 its package — fields
// 8k .. 8k + 7 of the 128 entries each, wave 3 also the descriptor and class —
// into LDS, polled until every granule carries q (one round trip when it is
// ready).  Run for pop p + 1 by the waves pop p's placement leaves idle (and
// for the first pop up front).  An exit descriptor has no package: its
// descriptor comes from the device ring.
// Field block K of a package (8 of its 32 fields, 128 entries: 16 granules per
// lane) from registers into the placer's LDS: keys, the row words, flags,
// node-affinity weights, depth-1 scores.
template <int K>
__device__ __forceinline__ void front_pkg_store(EngPlacerLds& L, const uint64_t (&v)[16], int base, uint32_t q,
                                                int lane) {
    EngRowCache& rc = L.rc;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        constexpr int kF0 = 8 * K;
        const int f = kF0 + (i >> 1), e = lane + 64 * (i & 1), sl = base + e;
        const uint32_t x = (uint32_t)v[i];
        if (f == kPkKey) L.pkey[q % 2][e] = x;
        else if (f < kPkFlags) ((uint32_t*)&rc.row[sl])[f - kPkRow] = x;
        else if (f == kPkFlags) L.flags[sl] = (uint8_t)x;
        else if (f == kPkNa) rc.na[sl] = (int32_t)x;
        else rc.s1[sl] = (int32_t)x;
    }
}

template <bool LIST>
__device__ __forceinline__ void eng_front(const Conf& cf, const NodeCols& nc, const DevTables& t, const EngArgs& A,
                                          EngPlacerLds& L, uint32_t q, int wave) {
    const int lane = threadIdx.x & 63;
    EngCtl* ctl = A.ctl;
    EngRowCache& rc = L.rc;
    if (wave == 0) return;
    const int k = wave == 3 ? 0 : wave == 4 ? 1 : wave - 4;  // field block of a loading wave (3, 4, 6, 7)
    const EngPkg* pk = A.pkg + (q % kEngSlots);
    uint64_t v[16];
    // pop q's descriptor and class (prefetched during P2, else from the ring); wave 3
    // leaves them in L.desc.  An exit has no package.
    uint32_t dw;
    if (__hip_atomic_load(&L.ndesc_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == (int)q) {
        dw = L.ndesc[lane];
    } else {
        const uint64_t* src = &ctl->desc[q % kEngRing][lane];
        EngWait wt(ctl, kEngDescTicks);
        uint64_t x = 0;
        for (;;) {
            x = ld_sc1(src);
            if (__ballot((uint32_t)(x >> 32) != q) == 0) break;
            if (!wt.tick(kEngErrDesc)) {
                if (wave == 3 && lane == 0) L.ok = 0;
                return;
            }
        }
        dw = (uint32_t)x;
    }
    if (wave == 3) L.desc[q % 2][lane] = dw;
    if (((uint32_t)__builtin_amdgcn_readlane((int)dw, kDwFlags) >> 12 & 0xf) != kEngOpPop) return;
    if (wave == 2) {
        const int r1 = (int)((q + 3) % 4), r2 = (int)((q + 2) % 4), r3 = (int)((q + 1) % 4);
        // pop q-1's candidates (its P3); the hash is rebuilt only after that P3's look-ups
        while (__hip_atomic_load(&L.xn_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != (int)(q - 1)) {
            if (!__hip_atomic_load(&L.ok, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) return;
            __builtin_amdgcn_s_sleep(1);
        }
        for (int h = lane; h < EngRowCache::kHashN; h += 64) rc.hkey[h] = -1;
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
        const int n1 = L.xn[r1][lane];
        if (n1 >= 0) rc_insert(&rc, n1, 64 * r1 + lane);
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
        const int n2 = L.xn[r2][lane];
        // list mode: the package holds pop q-2's candidates too (with stale keys) — a node of both
        // pops is in both sets, pop q-1's row is the latest either way; the hash keeps that one
        const bool use2 = n2 >= 0 && rc_find(&rc, n2) < 0;  // a node of both: pop q-1's row is the latest
        L.x2use[lane] = use2;
        if (use2) rc_insert(&rc, n2, 64 * r2 + lane);
        if (!LIST) {  // sweep mode: pop q-3's candidates too (list mode: the owner re-keyed them)
            __builtin_amdgcn_s_waitcnt(0xc07f);
            __builtin_amdgcn_wave_barrier();
            const int n3 = L.xn[r3][lane];
            const bool use3 = n3 >= 0 && rc_find(&rc, n3) < 0;
            L.x3use[lane] = use3;
            if (use3) rc_insert(&rc, n3, 64 * r3 + lane);
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the hash is in LDS before the flag
        if (lane == 0) __hip_atomic_store(&L.hash_seq, (int)q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        ETL(A, q - 1, 63);
        eng_front_eval<LIST>(cf, nc, t, A, L, q, dw, 0, 1);
        return;
    }
    // the evaluations (set, role: 0 the key, 1 the depth-1 score after an Allocate), a few
    // per wave; waves w and w + 4 share a SIMD's issue slots.  List mode: two sets, set 0
    // (pop q-1's candidates) evaluated beside pop q-1's decision (variants 0 and 1) and only
    // chosen once it is in; sweep mode: three sets, set 0 after the decision.
    if constexpr (LIST) {
        if (wave == 1) { eng_front_eval<LIST>(cf, nc, t, A, L, q, dw, 0, 0); return; }
        if (wave == 5) { eng_front_v1(cf, nc, t, L, q, dw, 1); return; }  // (after the host results)
        if (wave == 3) eng_front_eval<LIST>(cf, nc, t, A, L, q, dw, 1, 1);
        else if (wave == 6) eng_front_eval<LIST>(cf, nc, t, A, L, q, dw, 1, 0);
        else if (wave == 7) eng_front_v1(cf, nc, t, L, q, dw, 0);  // (wave 4: wave 0's SIMD, loads only)
    } else {
        if (wave == 1) { eng_front_eval<LIST>(cf, nc, t, A, L, q, dw, 0, 0); return; }
        if (wave == 5) { eng_front_eval<LIST>(cf, nc, t, A, L, q, dw, 1, 1); return; }
        if (wave == 3) eng_front_eval<LIST>(cf, nc, t, A, L, q, dw, 2, 1);
        else if (wave == 6) eng_front_eval<LIST>(cf, nc, t, A, L, q, dw, 1, 0);
        else if (wave == 7) eng_front_eval<LIST>(cf, nc, t, A, L, q, dw, 2, 0);
    }
    ETL(A, q - 1, 56 + k);  // (timeline: the loading wave's evaluation done)
    // the package's flag (one granule: its writer drained every store before it), then
    // this wave's field block in one round trip (r05: the whole block re-read until every
    // tag matched — a fifth of the front's time at C4, profiles/r06t*_tl_sweep.json)
    bool got = false;
    if (!eng_poll_tag(ctl, &ctl->pkg_ready[q % kEngSlots][0], q, kEngWaitTicks)) {
        if (k == 0 && lane == 0) L.ok = 0;
        return;
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = ld_sc1(&pk->w[8 * k + (i >> 1)][lane + 64 * (i & 1)]);
    EngWait wt(ctl, kEngWaitTicks);
    for (;;) {  // (every tag is q after the flag; the check stays as a guard)
        bool miss = false;
#pragma unroll
        for (int i = 0; i < 16; ++i) miss |= (uint32_t)(v[i] >> 32) != q;
        if (__ballot(miss) == 0) { got = true; break; }
#pragma unroll
        for (int i = 0; i < 16; ++i)
            if ((uint32_t)(v[i] >> 32) != q) v[i] = ld_sc1(&pk->w[8 * k + (i >> 1)][lane + 64 * (i & 1)]);
        if (!wt.tick()) break;
    }
    if (got) {
        ETL(A, q - 1, 48 + k);  // (timeline: this wave's package fields in registers)
        const int base = kEngStage + kEngPkgN * (int)(q % 2);
        switch (k) {  // (the field block as a constant: every store's target resolved at compile time)
            case 0: front_pkg_store<0>(L, v, base, q, lane); break;
            case 1: front_pkg_store<1>(L, v, base, q, lane); break;
            case 2: front_pkg_store<2>(L, v, base, q, lane); break;
            default: front_pkg_store<3>(L, v, base, q, lane); break;
        }
        ETL(A, q - 1, 52 + k);  // (timeline: ... and in LDS)
        if (k == 0) {
            for (int w = 0; w < 4; ++w) { rc.pw[base + lane][w] = 0; rc.pw[base + 64 + lane][w] = 0; }
            // pop q-1's candidates out of the package (its keys, written above by this wave),
            // once wave 2 has hashed the rings; else the placer's P2 does it
            bool hashed = false;
            for (int i = 0; i < 4096 && !hashed; ++i) {
                hashed = __hip_atomic_load(&L.hash_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == (int)q;
                if (!hashed) __builtin_amdgcn_s_sleep(1);
            }
            ETL(A, q - 1, 62);
            if (hashed) {
                uint32_t w8[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) w8[i] = (uint32_t)__builtin_amdgcn_readlane((int)dw, i);
                eng_drop_stale(L, eng_args(eng_decode(w8)), q);
                __builtin_amdgcn_s_waitcnt(0xc07f);
                if (lane == 0) __hip_atomic_store(&L.drop_seq, (int)q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                ETL(A, q - 1, 60);
                // the list merged with sets 1 and 2 once they are sorted (P3 then merges set 0 only)
                bool both = false;
                for (int i = 0; i < 4096 && !both; ++i) {
                    both = __hip_atomic_load(&L.sort_seq[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == (int)q &&
                           (LIST ||
                            __hip_atomic_load(&L.sort_seq[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == (int)q);
                    if (!both) __builtin_amdgcn_s_sleep(1);
                }
                if (both) {
                    uint32_t top = wave_merge_desc(L.s64[lane], L.e[1][lane]);
                    L.pre64[lane] = LIST ? top : wave_merge_desc(top, L.e[2][lane]);
                    __builtin_amdgcn_s_waitcnt(0xc07f);
                    if (lane == 0) __hip_atomic_store(&L.pre_seq, (int)q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    ETL(A, q - 1, 61);
                }
            }
        }
    } else if (k == 0 && lane == 0) {  // a wait gave up (the error is recorded)
        L.ok = 0;
    }
}

// The placer, per pop p (its front — descriptor, class, candidate hash,
// package, pops p-1 / p-2 / p-3's candidates evaluated — was prepared during
// pop p-1's placement):
//   P2  wave 0 drops pop p-1's candidates from the package list (stale keys: at most 64
//       of 128, the first 64 left are exact); waves 1, 5, 6 move the front's results for
//       pops p-1 / p-2 / p-3's candidates that count into place; wave 4 prefetches pop
//       p+1's descriptor;
//   P3  the final top 64, pop p-1's `done` (its write-back drained), pop p's candidates
//       published, their rows into ring p % 4;
//   P4  the placement (place_decide_wave, one wave); wave 0 then the results and rows,
//       wave 5 stores the results to the host, the other waves prepare pop p+1's front.
// The workers of pop p leave out pops p-3 / p-2's candidates and may hold stale
// keys of pop p-1's: every node of the three sets is re-evaluated here.
template <bool LIST>
__device__ __forceinline__ void eng_placer(const Conf& cf, const NodeCols& nc, const DevTables& t, const EngArgs& A,
                                           EngPlacerLds& L) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    EngCtl* ctl = A.ctl;
    EngRowCache& rc = L.rc;
    for (int i = threadIdx.x; i < 4 * 64; i += kPopThreads) L.xn[i >> 6][i & 63] = -1;
    if (threadIdx.x == 0) {
        L.ok = 1; L.gran_seq = 0; L.ndesc_seq = 0; L.rows_seq = (int)A.first - 1;
        L.hash_seq = L.drop_seq = (int)A.first - 1;
        L.xn_seq = (int)A.first - 1;
        L.v1_seq[0] = L.v1_seq[1] = L.pre_seq = (int)A.first - 1;
        L.sort_seq[0] = L.sort_seq[1] = L.sort_seq[2] = (int)A.first - 1;
        L.apmin = A.first - 1;
    }
    __syncthreads();
    eng_front<LIST>(cf, nc, t, A, L, A.first, wave);
    uint32_t pend = 0;  // wave 0: the pop whose write-back is still in flight (0: none)
    for (uint32_t p = A.first;; ++p) {
        // rings of p-1, p-2, p-3, p
        const int r1 = (int)((p + 3) % 4), r2 = (int)((p + 2) % 4), r3 = (int)((p + 1) % 4), r0 = (int)(p % 4);
        __syncthreads();
        if (!L.ok) return;
        const EngDesc d = eng_decode(L.desc[p % 2]);
        if (d.op != kEngOpPop) {
            if (wave == 0) eng_publish_done(ctl, &pend);
            return;
        }
        const PopArgs a = eng_args(d);
        const TaskClass& c = *(const TaskClass*)&L.desc[p % 2][kEngDescClass];
        if (wave == 0) {
            ETL(A, p, 0);
            if (lane == 0 && A.tl) A.tl[(size_t)(p % kEngTlSlots) * kEngTlEvents + 31] = p;
        }
        // P2
        if (wave == 0) {
            if (__hip_atomic_load(&L.drop_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != (int)p)
                eng_drop_stale(L, a, p);
            ETL(A, p, 1);
        } else if (wave == 4) {  // pop p+1's descriptor, if the dispatcher has it (one attempt)
            const uint64_t x = ld_sc1(&ctl->desc[(p + 1) % kEngRing][lane]);
            if (__ballot((uint32_t)(x >> 32) != p + 1) == 0) {
                L.ndesc[lane] = (uint32_t)x;
                __builtin_amdgcn_s_waitcnt(0xc07f);
                if (lane == 0) __hip_atomic_store(&L.ndesc_seq, (int)(p + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        } else if (wave == 1 || wave == 5 || (!LIST && wave == 6)) {  // pops p-1 / p-2 (/ p-3)'s candidates that count
            // (the front's evaluation): sorted keys, FitDelta bits, node-affinity weights and
            // depth-1 scores (the one their key's kind calls for) into the row cache
            const int set = wave == 1 ? 0 : wave - 4;
            const int ring = set == 0 ? r1 : set == 1 ? r2 : r3;
            const int node = L.xn[ring][lane];
            const bool use = node >= 0 && (set == 0 || (set == 1 ? L.x2use[lane] : L.x3use[lane]));
            if (wave == 1) ETL(A, p, 2);
            if (__hip_atomic_load(&L.sort_seq[set], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != (int)p) {
                L.e[set][lane] = wave_sort_desc(use ? L.fe[set][lane] : 0u);
                L.fbp[set][lane] = use ? L.ffb[set][lane] : (uint8_t)0;
            }
            if (wave == 1) ETL(A, p, 9);
            if (use) {
                const int sl = 64 * ring + lane;
                const int kind = L.fkind[set][lane];
                rc.na[sl] = L.fna[set][lane];
                rc.s1[sl] = kind == 0 ? INT32_MIN : kind == 2 ? L.fs1p[set][lane] : L.fs1a[set][lane];
            }
        }
        __syncthreads();
        if (wave == 0) ETL(A, p, 3);
        // P3
        if (wave == 0) {
            uint32_t top;
            if (__hip_atomic_load(&L.pre_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == (int)p) {
                top = wave_merge_desc(L.pre64[lane], L.e[0][lane]);  // (the front merged sets 1 (, 2))
            } else {
                top = wave_merge_desc(L.s64[lane], L.e[0][lane]);
                top = wave_merge_desc(top, L.e[1][lane]);
                if (!LIST) top = wave_merge_desc(top, L.e[2][lane]);
            }
            // (list mode: the owner counted pop p-3's candidates)
            const uint32_t fbp = (uint32_t)L.fbp[0][lane] | ((uint32_t)L.fbp[1][lane] << 4) |
                                 (LIST ? 0u : ((uint32_t)L.fbp[2][lane] << 8));
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int k = __popcll(__ballot((fbp >> q) & 1u)) + __popcll(__ballot((fbp >> (q + 4)) & 1u)) +
                              __popcll(__ballot((fbp >> (q + 8)) & 1u));
                if (lane == q) L.fitin[q] = k;
            }
            const int n = top ? key_node(top, a) : -1;
            ETL(A, p, 44);
            eng_publish_done(ctl, &pend);  // pop p-1's write-back (every node a worker may read next)
            ETL(A, p, 45);
            if constexpr (LIST) {
                // list mode: the log entry of pop p, once every owner has applied pop p - kEngLog
                if ((int32_t)(L.apmin - (p - kEngLog)) < 0 && !eng_own_apmin(A, L, p - kEngLog)) {
                    if (lane == 0) __hip_atomic_store(&L.ok, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
                st_sc1(&ctl->tlog[p % kEngLog][lane], ((uint64_t)p << 32) | (uint32_t)n);
                if (lane == 0) st_sc1(&ctl->tcls[p % kEngLog], ((uint64_t)p << 32) | (uint32_t)a.cls);
            } else {
#pragma unroll
                for (int cp = 0; cp < kEngCandCopies; ++cp)
                    st_sc1(&ctl->cands[p % kEngSlots][cp][lane], ((uint64_t)p << 32) | (uint32_t)n);
            }
            ETL(A, p, 46);
            int src = n >= 0 ? rc_find(&rc, n) : -1;  // a previous pop's candidate, or a package entry
            if (n >= 0 && src < 0) {  // (every node of the list is one of those: kept for safety)
                src = 64 * r0 + lane;
                const Row r = load_row_sc1(nc, n);
                const int32_t na = cf.score_mult ? na_weight(c, t, nc, n) : 0;
                const uint64_t pw[4] = {0, 0, 0, 0};
                rc.row[src] = r;
                L.flags[src] = nc.flags[n];
                rc.na[src] = na;
                rc.s1[src] = depth1_score(cf, nc, t, c, r, pw, n, na, key64_of(top, a));
                for (int w = 0; w < 4; ++w) rc.pw[src][w] = 0;
            }
            L.srcslot[lane] = src;
            L.xn[r0][lane] = n;
            L.wl64[0][lane] = key64_of(top, a);
            __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the candidates are in LDS before the flag
            if (lane == 0) __hip_atomic_store(&L.xn_seq, (int)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            ETL(A, p, 4);
            ETL(A, p, 5);
        }
        // (no barrier: the other waves start pop p+1's front during P3 and take pop p's
        // candidates once L.xn_seq reads p)
        // P4 (engine pops' classes have 32-bit entries, PopArgs::ent32: the host
        // sends the others to the launched kernels).  Wave 0 decides alone
        // (place_decide_wave) and writes the results and rows, while wave 5
        // stores the results to the host and the others prepare pop p+1's front.
        if (wave == 0) {
            PlaceDec<uint32_t> D;
            if (place_decide_wave<uint32_t, true>(cf, nc, t, c, a, L.wl64[0], p, &rc, L.srcslot, !A.quick, D)) {
                ETL(A, p, 6);
                if (lane == 0 && A.tl)
                    A.tl[(size_t)(p % kEngTlSlots) * kEngTlEvents + 30] = (uint64_t)D.done | ((uint64_t)D.stop << 8);
                eng_finish<LIST>(cf, nc, t, c, a, A, L, p, r0, D, &pend);
            } else if (lane == 0) {  // (a class with host ports: never sent to the engine, eng_eligible)
                __hip_atomic_store(&ctl->err, (uint32_t)kEngErrClass, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&L.ok, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        } else {
            // (wave 5's results first: its front waits for pop p+1's descriptor, which
            // the host may send only after it has seen them)
            if (wave == 5) eng_host_out(A, L, p, d.slot);
            eng_front<LIST>(cf, nc, t, A, L, p + 1, wave);
            if (wave == 3) ETL(A, p, 15);
            if (wave == 1) ETL(A, p, 19);
            if (wave == 5) ETL(A, p, 29);
            if (wave == 7) ETL(A, p, 16);
            if (wave == 6) ETL(A, p, 17);
            if (wave == 4) ETL(A, p, 14);
            if (wave == 2) ETL(A, p, 23);
        }
    }
}

// ---------------------------------------------------------------------------
// dispatcher: host ring -> device ring (one wave)
// ---------------------------------------------------------------------------
__device__ __forceinline__ void eng_dispatch(const EngArgs& A) {
    const int lane = threadIdx.x & 63;
    EngCtl* ctl = A.ctl;
    uint32_t s = A.first;
    bool idle = false;
    for (;; ++s) {
        // the device ring slot of pop s - kEngRing is free once the placer finished pop s - 5
        if (s >= A.first + 5 && !eng_wait_done(ctl, s - 5)) break;
        const uint64_t* src = A.hring + (size_t)(s % kEngHostRing) * kEngDescWords + lane;
        uint64_t x = 0;
        uint64_t t0 = 0;
        bool got = false;
        for (uint32_t it = 0;; ++it) {
            x = __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            if (__ballot((uint32_t)(x >> 32) != s) == 0) { got = true; break; }
            if ((it & 15) == 15) {
                const uint64_t now = eng_now();
                if (!t0) t0 = now;
                if (ld_sc1(&ctl->err) != 0) break;
                if (now - t0 > (uint64_t)A.idle_ticks) { idle = true; break; }
            }
            __builtin_amdgcn_s_sleep(2);
        }
        uint32_t op = kEngOpExit;
        if (got) op = ((uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, kDwFlags) >> 12) & 0xf;
        else if (ld_sc1(&ctl->err) != 0) break;
        // forward (an idle end becomes an exit descriptor at s)
        uint64_t v = x;
        if (!got) v = lane == kDwFlags ? (((uint64_t)s << 32) | ((uint64_t)kEngOpExit << 12)) : ((uint64_t)s << 32);
        st_sc1(&ctl->desc[s % kEngRing][lane], v);
        ETL(A, s, 28);
        if (op != kEngOpPop) break;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0)
        __hip_atomic_store(A.hexit, (uint64_t)s | ((uint64_t)(idle ? 1 : 0) << 40) | (1ull << 41), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
}

// Every block at its start: wait until every block of the grid has started (its
// blocks spin on each other, so all of them must be resident at once).  One
// counter decides for all: a block that waited kEngArriveTicks closes it
// (bit 31) unless it has reached the grid size, and a closed counter never
// does — so either every block runs or none serves a pop (kEngErrResident; the
// dispatcher reports it, eng_not_resident).
__device__ __forceinline__ bool eng_arrive(const EngArgs& A, int* flag) {
    EngCtl* ctl = A.ctl;
    if (threadIdx.x == 0) {
        constexpr uint32_t kClosed = 0x80000000u;
        const uint32_t old = __hip_atomic_fetch_add(&ctl->arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        bool ok = !(old & kClosed);
        const uint64_t t0 = eng_now();
        while (ok) {
            uint32_t v = ld_sc1(&ctl->arrive);
            if (v & kClosed) { ok = false; break; }
            if (v == gridDim.x) break;
            if (eng_now() - t0 > kEngArriveTicks &&
                __hip_atomic_compare_exchange_strong(&ctl->arrive, &v, v | kClosed, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT)) {
                __hip_atomic_store(&ctl->err, (uint32_t)kEngErrResident, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ok = false;
                break;
            }
            __builtin_amdgcn_s_sleep(8);
        }
        *flag = ok;
    }
    __syncthreads();
    return *flag != 0;
}
// The dispatcher of a grid that did not become resident: the exit word (nothing served).
__device__ __forceinline__ void eng_not_resident(const EngArgs& A) {
    if (threadIdx.x == 0)
        __hip_atomic_store(A.hexit, (uint64_t)A.first | (1ull << 41) | (1ull << 42), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace kbhip
