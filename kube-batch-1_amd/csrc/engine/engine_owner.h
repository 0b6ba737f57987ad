// engine_owner.h — list mode's class owners (k_engine_lists).
#pragma once
#include <hip/hip_runtime.h>

#define KBHIP_STAMPS_OFF  // phase stamps belong to k_pop_batch (kbhip_kernels.hip)
#include "../kbhip_batch.h"
#include "../kbhip_engine.h"
#include "engine_dev.h"

namespace kbhip {

// ---------------------------------------------------------------------------
// class owner (list mode)
// ---------------------------------------------------------------------------
// A node's key for the owner's class as one byte: level << 1 | pipelined,
// level = score - kbase + 1 in [1, kOwnLv - 1] (the host admits only classes
// whose score range fits); 0 = not a candidate.  The 32-bit selection key
// (PopArgs) follows from the byte and the node index: the byte order is the
// key order among nodes of one level, and the index breaks ties.
__device__ __forceinline__ uint32_t own_val(uint64_t k64, int32_t kbase) {
    if (!k64) return 0;
    return ((uint32_t)(key_score(k64) - kbase + 1) << 1) | (uint32_t)(k64 & 1);
}
__device__ __forceinline__ uint32_t own_key(uint32_t v, int g, const EngArgs& A) {
    return ((v >> 1) << A.kshift) | ((uint32_t)(A.kidxmax - g) << 1) | (v & 1);
}
// Level counts of node n with byte v (d = 1 or ~0u: add or remove).
__device__ __forceinline__ void own_count(EngOwnerLds& L, int n, uint32_t v, uint32_t d) {
    if (!v) return;
    const uint32_t lv = v >> 1;
    atomicAdd(&L.lvl[lv], d);
    atomicAdd(&L.seg[lv >> 1][n / kOwnSeg], d << (16 * (lv & 1)));
}
__device__ __forceinline__ uint32_t own_segcnt(const EngOwnerLds& L, int lv, int sg) {
    return (L.seg[lv >> 1][sg] >> (16 * (lv & 1))) & 0xffffu;
}
// Per wave: FitDelta counts from old to new bits of the lanes with `on`.
__device__ __forceinline__ void own_fit_delta(EngOwnerLds& L, bool on, uint32_t ofb, uint32_t nfb) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const uint32_t o = (ofb >> b) & 1u, n = (nfb >> b) & 1u;
        const int up = __popcll(__ballot(on && n && !o)), dn = __popcll(__ballot(on && o && !n));
        if (lane == b && up != dn) atomicAdd(&L.fit[b], (uint32_t)(up - dn));
    }
}
// The node set (open addressing over kOwnHash slots; every user clears the
// slots it filled before the next use).
__device__ __forceinline__ int own_hslot(int n) { return (int)(((uint32_t)n * 2654435761u) >> 22); }
__device__ __forceinline__ int own_hinsert(EngOwnerLds& L, int n, bool* fresh) {
    static_assert(kOwnHash == 1024, "own_hslot takes 10 bits");
    int h = own_hslot(n);
    for (;;) {
        const int old = atomicCAS(&L.hkey[h], -1, n);
        if (old == -1 || old == n) {
            *fresh = old == -1;
            return h;
        }
        h = (h + 1) & (kOwnHash - 1);
    }
}
__device__ __forceinline__ int own_hfind(const EngOwnerLds& L, int n) {
    int h = own_hslot(n);
    for (int i = 0; i < kOwnHash; ++i, h = (h + 1) & (kOwnHash - 1)) {
        const int k = L.hkey[h];
        if (k == n) return h;
        if (k == -1) return -1;
    }
    return -1;
}

// Wave 0: pop q's logged candidate `lane` (-1: none); false: the wait gave up.
__device__ __forceinline__ bool own_log_node(EngCtl* ctl, uint32_t q, int* node) {
    const int lane = threadIdx.x & 63;
    const uint64_t* src = &ctl->tlog[q % kEngLog][lane];
    EngWait wt(ctl, kEngWaitTicks);
    for (;;) {
        const uint64_t x = ld_sc1(src);
        if (__ballot((uint32_t)(x >> 32) != q) == 0) {
            *node = (int)(uint32_t)x;
            return true;
        }
        if (!wt.tick()) return false;
    }
}

// Wave 0: from descriptor dp on, the next pop of class cls (L.next = its
// sequence number, its words in L.desc), the run's end (L.next = -2) or
// neither yet (-1); L.dp = the first descriptor not looked at.  The ring's
// slots are read together; a slot already reused by a later descriptor
// belongs to a pop that ran — its class comes from the log (it is not this
// owner's: that pop's package was this owner's to write).
__device__ __forceinline__ bool own_scan_desc(const EngArgs& A, EngOwnerLds& L, int cls, uint32_t dp) {
    const int lane = threadIdx.x & 63;
    EngCtl* ctl = A.ctl;
    uint64_t x[kEngRing];
#pragma unroll
    for (int i = 0; i < kEngRing; ++i) x[i] = ld_sc1(&ctl->desc[(dp + i) % kEngRing][lane]);
    int next = -1;
#pragma unroll
    for (int i = 0; i < kEngRing; ++i) {
        const uint32_t q = dp;
        const uint32_t tg = (uint32_t)(x[i] >> 32);
        if (__ballot(tg != q) == 0) {
            const uint32_t w = (uint32_t)x[i];
            const uint32_t flags = (uint32_t)__builtin_amdgcn_readlane((int)w, kDwFlags);
            if (((flags >> 12) & 0xf) != kEngOpPop) { next = -2; break; }
            if (__builtin_amdgcn_readlane((int)w, kDwCls) == cls) {
                L.desc[lane] = w;
                next = (int)q;
                break;
            }
            ++dp;
            continue;
        }
        if (__ballot((int32_t)(tg - q) > 0) == 0) break;  // not there yet
        // reused: pop q ran; its class from the log
        const uint64_t* src = &ctl->tcls[q % kEngLog];
        EngWait wt(ctl, kEngWaitTicks);
        uint64_t y;
        for (;;) {
            y = ld_sc1(src);
            if ((uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(y >> 32)) == q) break;
            if (!wt.tick()) return false;
        }
        if ((int)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)y) == cls) {  // cannot happen
            if (lane == 0) __hip_atomic_store(&ctl->err, (uint32_t)kEngErrDesc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return false;
        }
        ++dp;
    }
    if (lane == 0) {
        L.next = next;
        L.dp = (int)dp;
    }
    return true;
}

// Every wave: apply pops a0 .. a0 + nb - 1 (nb <= 8, each `done`): wave w
// reads pop a0 + w's candidates' rows and re-keys them; a node of several of
// these pops is applied once (every copy was read after the last one's
// `done`).  A row read while a later pop writes it is torn or newer: that node
// is a candidate of the later pop, applied again after its `done`, and left
// out of every package until then.  The candidates come from
// L.lognode (read with `done`, the log entries then published) or the log.
// The FitDelta bits are stored without a wait: every later reader of them runs
// after a barrier that the storing waves reach drained (own_drain).
__device__ __forceinline__ bool own_apply(const Conf& cf, const NodeCols& nc, const DevTables& t, const TaskClass& c,
                                          const EngArgs& A, EngOwnerLds& L, uint8_t* fbh, int32_t kbase, uint32_t a0,
                                          int nb, bool prefetched = true) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    EngCtl* ctl = A.ctl;
    int node = -1;
    bool ok = true;
    if (wave < nb) {
        node = prefetched ? L.lognode[wave][lane] : -2;
        if (__ballot(node == -2) != 0) ok = own_log_node(ctl, a0 + (uint32_t)wave, &node);
    }
    if (!ok && lane == 0) L.ok = 0;
    Row r{};
    uint8_t fl = 0;
    uint32_t ofb = 0;
    int hs = -1;
    bool fresh = false;
    if (node >= 0) {
        fl = nc.flags[node];
        r = load_row_sc1(nc, node);
        ofb = ld_sc1(&fbh[node]);
        hs = own_hinsert(L, node, &fresh);
    }
    uint32_t nfb = 0;
    const uint32_t nv = node >= 0 ? own_val(eng_eval_row(cf, c, t, nc, node, r, fl, &nfb), kbase) : 0u;
    __syncthreads();
    if (node >= 0) atomicMax(&L.hval[hs], wave);  // the latest pop's copy is applied
    __syncthreads();
    const bool win = node >= 0 && L.hval[hs] == wave;
    if (win) {
        const uint32_t ov = L.sv[node];
        L.sv[node] = (uint8_t)nv;
        own_count(L, node, ov, ~0u);
        own_count(L, node, nv, 1u);
        st_sc1(&fbh[node], (uint8_t)nfb);
    }
    own_fit_delta(L, win, ofb, nfb);
    __syncthreads();
    if (win) {  // the exact level bound of the node's block (every byte written above)
        const uint4* bw = (const uint4*)&L.sv[(node / kOwnSub) * kOwnSub];
        uint32_t mx = 0;
#pragma unroll
        for (int k = 0; k < kOwnSub / 16; ++k) {
            const uint4 q = bw[k];
#pragma unroll
            for (int b = 0; b < 4; ++b)
                mx = max(mx, max(max((q.x >> (8 * b + 1)) & 0x7fu, (q.y >> (8 * b + 1)) & 0x7fu),
                                 max((q.z >> (8 * b + 1)) & 0x7fu, (q.w >> (8 * b + 1)) & 0x7fu)));
        }
        L.smax[node / kOwnSub] = mx;
    }
    if (node >= 0) { L.hkey[hs] = -1; L.hval[hs] = -1; }
    return L.ok != 0;
}
// This wave's stores done (the FitDelta bits of an apply) before the next barrier.
__device__ __forceinline__ void own_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Every wave: pop p's package (its descriptor in L.desc) — the top 128 keys of
// the class over every node but pops p-3 and p-2's candidates, with their rows
// (the layout of eng_final) — and, once pop p-1's candidates are logged, pop
// p's FitDelta counts over every node but the three sets (the placer counts
// those on their final rows).  Everything but the last step runs before pop
// p-2's candidates are known: the top kOwnPre without pop p-3's, sorted; then
// pop p-2's leave the list (at most 64) and the first 128 left are packaged.
__device__ __forceinline__ bool own_package(const Conf& cf, const NodeCols& nc, const DevTables& t, const TaskClass& c,
                                            const EngArgs& A, EngOwnerLds& L, uint8_t* fbh, int32_t kbase, uint32_t p,
                                            uint32_t* ap) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    EngCtl* ctl = A.ctl;
    const EngDesc d = eng_decode(L.desc);
    const PopArgs a = eng_args(d);
    ETL(A, p, 10);
    // 1. pop p-3's candidates (wave 0) out of the counts and the scan
    int x3 = -1;
    bool ok = true;
    if (wave == 0) {
        if ((int32_t)(p - 3 - A.first) >= 0) ok = own_log_node(ctl, p - 3, &x3);
        if (!ok && lane == 0) L.ok = 0;
    }
    if (threadIdx.x < 4) L.xfit[threadIdx.x] = 0;
    bool xf3 = false;
    int xs3 = -1;
    if (x3 >= 0) xs3 = own_hinsert(L, x3, &xf3);
    __syncthreads();
    if (wave == 0) ETL(A, p, 21);
    uint32_t xv3 = 0;
    if (xf3) {
        xv3 = L.sv[x3];
        L.sv[x3] = 0;
        own_count(L, x3, xv3, ~0u);
    }
    __syncthreads();
    // 2. wave 0: the threshold level thr (fewer than kOwnPre nodes above it, at least kOwnPre
    // at or above; or level 1 when fewer are left) and the segments holding the entries
    if (wave == 0) {
        static_assert(kOwnLv == 128, "two levels per lane");
        const uint32_t K = (uint32_t)kOwnPre;
        const uint32_t c0 = lane ? L.lvl[2 * lane] : 0u, c1 = L.lvl[2 * lane + 1];  // levels 2 lane, 2 lane + 1
        uint32_t s = c0 + c1;  // nodes at levels >= 2 lane
#pragma unroll
        for (int dd = 1; dd < 64; dd <<= 1) {
            const uint32_t u = (uint32_t)__shfl_down((int)s, dd, 64);
            if (lane + dd < 64) s += u;
        }
        const uint32_t s1 = s - c0;  // nodes at levels >= 2 lane + 1
        const int bl = s1 >= K ? 2 * lane + 1 : (lane && s >= K) ? 2 * lane : 0;
        int thr = bl;
#pragma unroll
        for (int dd = 1; dd < 64; dd <<= 1) thr = max(thr, __shfl_xor(thr, dd, 64));
        if (thr == 0) thr = 1;  // fewer than K nodes: all of them
        const int tl = thr >> 1;
        const uint32_t s_tl = (uint32_t)__shfl((int)s, tl, 64), s1_tl = (uint32_t)__shfl((int)s1, tl, 64);
        const uint32_t c1_tl = (uint32_t)__shfl((int)c1, tl, 64);
        const uint32_t above = (thr & 1) ? s1_tl - c1_tl : s1_tl;  // nodes above thr
        const uint32_t at = (thr & 1) ? c1_tl : s_tl - s1_tl;       // nodes at thr
        const int need = (int)min(K - min(above, K), at);
        const uint64_t nz = __ballot(c0 + c1 != 0);
        const int top = nz ? 2 * (63 - __builtin_clzll(nz)) + 1 : 0;
        uint32_t hi = 0;  // (lane = segment) nodes above thr: level pairs, the words' halves
        for (int lp = (thr + 1) >> 1; lp <= (top >> 1); ++lp) {
            const uint32_t w = L.seg[lp][lane];
            hi += (2 * lp > thr ? (w & 0xffffu) : 0u) + (w >> 16);
        }
        const uint32_t eq = own_segcnt(L, thr, lane);
        uint32_t inc = eq;  // inclusive prefix over segments
#pragma unroll
        for (int dd = 1; dd < 64; dd <<= 1) {
            const uint32_t u = (uint32_t)__shfl_up((int)inc, dd, 64);
            if (lane >= dd) inc += u;
        }
        const int tk = max(0, min(need - (int)(inc - eq), (int)eq));
        const bool act = hi > 0 || tk > 0;
        const uint64_t am = __ballot(act);
        const int pos = __builtin_amdgcn_mbcnt_hi((uint32_t)(am >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)am, 0));
        if (act) {
            L.act[pos] = lane;
            L.take[pos] = tk;
            L.hic[pos] = (int)hi;
        }
        if (lane == 0) {
            L.nact = __popcll(am);
            L.thr = thr;
            L.nkeys = 0;
        }
        ETL(A, p, 24);
        if (A.tl && lane == 0) A.tl[(size_t)(p % kEngTlSlots) * kEngTlEvents + 25] = (uint64_t)__popcll(am) | ((uint64_t)thr << 8);
    }
    __syncthreads();
    // 3. the entries: wave w scans active segments w, w + 8, ... — only the blocks of
    // kOwnSub nodes whose level bound reaches thr, two per step in index order, until
    // the segment's nodes above thr and its first take[] nodes at thr are found
    {
        const int thr = L.thr, nact = L.nact;
        constexpr int nsub = kOwnSeg / kOwnSub;
        const int g = lane >> 5, w = lane & 31;  // block g of the step, word w of the block
        for (int i = wave; i < nact; i += kPopThreads / 64) {
            const int sg = L.act[i], tk = L.take[i], hs = L.hic[i];
            const int sb0 = sg * nsub;
            uint64_t cm = __ballot(lane < nsub && (int)L.smax[sb0 + min(lane, nsub - 1)] >= thr);
            int found = 0, run = 0;  // nodes above thr found, nodes at thr seen (index order)
            while (cm && (found < hs || run < tk)) {
                const int b0 = __builtin_ctzll(cm);
                const uint64_t cm1 = cm & (cm - 1);
                const int b1 = cm1 ? __builtin_ctzll(cm1) : -1;
                cm = cm1 ? (cm1 & (cm1 - 1)) : 0;
                const int sb = g == 0 ? b0 : b1;
                const uint32_t wv = sb >= 0 ? ((const uint32_t*)L.sv)[(sb0 + sb) * (kOwnSub / 4) + w] : 0u;
                const int n0 = (sb0 + sb) * kOwnSub + 4 * w;
                int below = 0, tot = 0, nh = 0;
                uint32_t mx = 0;
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    const uint32_t v = (wv >> (8 * b)) & 0xffu;
                    const uint64_t bm = __ballot(v != 0 && (int)(v >> 1) == thr);
                    below += __builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0));
                    tot += __popcll(bm);
                    nh += __popcll(__ballot((int)(v >> 1) > thr));
                    mx = max(mx, v >> 1);
                }
                // the entries of this step: positions from one LDS add per step
                bool tb[4];
                int k_in = 0;
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    const uint32_t v = (wv >> (8 * b)) & 0xffu;
                    tb[b] = false;
                    if (v && (int)(v >> 1) > thr) {
                        tb[b] = true;
                    } else if (v && (int)(v >> 1) == thr) {
                        tb[b] = run + below + k_in < tk;
                        ++k_in;
                    }
                }
                uint64_t tm[4];
                int ntot = 0;
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    tm[b] = __ballot(tb[b]);
                    ntot += __popcll(tm[b]);
                }
                uint32_t base = 0;
                if (ntot) {
                    if (lane == 0) base = atomicAdd(&L.nkeys, (uint32_t)ntot);
                    base = (uint32_t)__builtin_amdgcn_readfirstlane((int)base);
                }
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    const uint32_t at = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(tm[b] >> 32),
                                                                         __builtin_amdgcn_mbcnt_lo((uint32_t)tm[b], 0));
                    if (tb[b] && at < (uint32_t)kOwnPre)
                        L.keys[at] = own_key((wv >> (8 * b)) & 0xffu, n0 + b + nc.base, A);
                    base += (uint32_t)__popcll(tm[b]);
                }
                // the blocks read are exact now (the left-out nodes are raised back below)
#pragma unroll
                for (int dd = 1; dd < 32; dd <<= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, dd, 64));
                if (w == 0 && sb >= 0) L.smax[sb0 + sb] = mx;
                run += tot;
                found += nh;
            }
        }
    }
    __syncthreads();
    if (wave == 0) ETL(A, p, 26);
    // 4. pop p-3's nodes back; wave 0 sorts the entries (four sorted 64-lists, merged)
    if (xf3) {
        L.sv[x3] = (uint8_t)xv3;
        own_count(L, x3, xv3, 1u);
        if (xv3) atomicMax(&L.smax[x3 / kOwnSub], xv3 >> 1);
    }
    uint32_t m[4];  // (wave 0) the sorted entries, ranks 64 k .. 64 k + 63 in m[k]
    if (wave == 0) {
        static_assert(kOwnPre <= 192, "three registers and pop p-3's candidates");
        const uint32_t nk = min(L.nkeys, (uint32_t)kOwnPre);
        uint32_t r[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) r[k] = (uint32_t)(64 * k + lane) < nk ? L.keys[64 * k + lane] : 0u;
#pragma unroll
        for (int k = 0; k < 4; ++k) r[k] = wave_sort_desc(r[k]);
        uint32_t n[4];  // (r0, r1) and (r2, r3) into sorted 128-lists
        {
            const uint32_t rv = reverse_lanes(r[1]);
            m[0] = bitonic_clean_desc(r[0] > rv ? r[0] : rv);
            m[1] = bitonic_clean_desc(r[0] > rv ? rv : r[0]);
        }
        {
            const uint32_t rv = reverse_lanes(r[3]);
            n[0] = bitonic_clean_desc(r[2] > rv ? r[2] : rv);
            n[1] = bitonic_clean_desc(r[2] > rv ? rv : r[2]);
        }
        m[2] = m[3] = n[2] = n[3] = 0u;
        wave_merge256_desc(m, n);  // all of the two 128-lists, sorted (at most 192)
        ETL(A, p, 12);
    }
    __syncthreads();
    if (xs3 >= 0) { L.hkey[xs3] = -1; L.hval[xs3] = -1; }
    // 5. pop p-3's rows, once it is done: its candidates re-keyed (the apply), then merged
    // into the entries with their new keys — the package covers them, the placer re-evaluates
    // only pops p-2 and p-1's candidates (list mode)
    if ((int32_t)(p - 3 - A.first) >= 0 && (int32_t)(*ap - (p - 3)) < 0) {
        if (wave == 0) {
            EngWait wt(ctl, kEngWaitTicks);
            while ((int32_t)((uint32_t)__builtin_amdgcn_readfirstlane((int)ld_sc1(&ctl->done)) - (p - 3)) < 0)
                if (!wt.tick()) { if (lane == 0) L.ok = 0; break; }
        }
        __syncthreads();
        if (!L.ok) return false;
        if (!own_apply(cf, nc, t, c, A, L, fbh, kbase, p - 3, 1, false)) return false;
        *ap = p - 3;
        own_drain();  // (its FitDelta bits, read below)
        if (threadIdx.x == 0) st_sc1(&ctl->own_ap[blockIdx.x], *ap);
    }
    __syncthreads();
    if (wave == 0) {
        const uint32_t v = x3 >= 0 ? (uint32_t)L.sv[x3] : 0u;
        const uint32_t k3 = wave_sort_desc(v ? own_key(v, x3 + nc.base, A) : 0u);
        const uint32_t b[4] = {k3, 0u, 0u, 0u};
        wave_merge256_desc(m, b);  // the entries and pop p-3's candidates, sorted (at most 256)
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int k = 0; k < 4; ++k) L.keys[64 * k + lane] = m[k];
    }
    // 6. pop p-2's candidates (wave 1): out of the sorted entries; the first 128 left are the package
    int x2 = -1;
    if (wave == 1) {
        if ((int32_t)(p - 2 - A.first) >= 0) ok = own_log_node(ctl, p - 2, &x2);
        if (!ok && lane == 0) L.ok = 0;
        ETL(A, p, 11);
    }
    bool xf2 = false;
    int xs2 = -1;
    if (x2 >= 0) xs2 = own_hinsert(L, x2, &xf2);
    const uint32_t xfb2 = xf2 ? ld_sc1(&fbh[x2]) : 0u;
    __syncthreads();
    bool keep = false;
    uint64_t km = 0;
    if (wave < 4) {
        const uint32_t k = L.keys[64 * wave + lane];
        keep = k && own_hfind(L, key_node(k, a) - nc.base) < 0;
        km = __ballot(keep);
        if (lane == 0) L.wcnt[wave] = (uint32_t)__popcll(km);
    }
    __syncthreads();
    if (wave < 4) {
        uint32_t base = 0;
        for (int w = 0; w < wave; ++w) base += L.wcnt[w];
        const uint32_t tot = L.wcnt[0] + L.wcnt[1] + L.wcnt[2] + L.wcnt[3];
        const uint32_t pos = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(km >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)km, 0));
        if (keep && pos < (uint32_t)kEngPkgN) L.slot_entry[pos] = 64 * wave + lane;
        if (wave < 2 && (uint32_t)(64 * wave + lane) >= tot) L.slot_entry[64 * wave + lane] = -1;
    }
    __syncthreads();
    // 6. the package (waves 0, 1: slot 64 * wave + lane; eng_final's layout); then their
    // left-out nodes' FitDelta bits
    EngPkg* pk = A.pkg + (p % kEngSlots);
    const uint64_t tag = (uint64_t)p << 32;
    if (wave < 2) {
        const int e = 64 * wave + lane;
        const int src = L.slot_entry[e];
        const uint32_t k = src >= 0 ? L.keys[src] : 0u;
        const int n = k ? key_node(k, a) - nc.base : -1;
        uint32_t v[kEngPkgFields];
#pragma unroll
        for (int f = 0; f < kEngPkgFields; ++f) v[f] = 0;
        v[kPkKey] = k;
        if (n >= 0) {
            const Row r = load_row_sc1(nc, n);
            const uint8_t fl = nc.flags[n];
            const int32_t na = cf.score_mult ? na_weight(c, t, nc, n) : 0;
            const uint64_t pw[4] = {0, 0, 0, 0};
            const uint32_t* rw = (const uint32_t*)&r;
#pragma unroll
            for (int f = 0; f < (int)(sizeof(Row) / 4); ++f) v[kPkRow + f] = rw[f];
            v[kPkFlags] = fl;
            v[kPkNa] = (uint32_t)na;
            v[kPkS1] = (uint32_t)depth1_score(cf, nc, t, c, r, pw, n, na, key64_of(k, a));
        }
#pragma unroll
        for (int f = 0; f < kEngPkgFields; ++f) st_sc1(&pk->w[f][e], tag | v[f]);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // landed before the flag below
        if (wave == 0) ETL(A, p, 13);
    }
    if (wave == 1) {  // pop p-2's candidates' FitDelta bits (left out of pop p's counts)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const int kx = __popcll(__ballot(xf2 && ((xfb2 >> b) & 1u)));
            if (lane == 0 && kx) atomicAdd((uint32_t*)&L.xfit[b], (uint32_t)kx);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) st_sc1(&A.ctl->pkg_ready[p % kEngSlots][0], tag | 1u);  // the package has landed
    // 7. wave 2: pop p's FitDelta counts once pop p-1's candidates are logged
    if (wave == 2 && L.ok) {
        int n1 = -1;
        if ((int32_t)(p - 1 - A.first) >= 0) ok = own_log_node(ctl, p - 1, &n1);
        const bool in = ok && n1 >= 0 && own_hfind(L, n1) < 0;  // not a left-out node (counted there)
        const uint32_t fb1 = in ? ld_sc1(&fbh[n1]) : 0u;
        uint32_t cnt = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const uint32_t k = (uint32_t)__popcll(__ballot(in && ((fb1 >> b) & 1u)));
            if (lane == b) cnt = L.fit[b] - (uint32_t)L.xfit[b] - k;
        }
        if (ok && lane < 4) st_sc1(&A.blists[(size_t)(p % kEngSlots) * kEngListWords + 128 + lane], tag | cnt);
        if (!ok && lane == 0) L.ok = 0;
        ETL(A, p, 18);
    }
    __syncthreads();
    if (xs2 >= 0) { L.hkey[xs2] = -1; L.hval[xs2] = -1; }
    return L.ok != 0;
}

__device__ __forceinline__ void eng_owner(const Conf& cf, const NodeCols& nc, const DevTables& t, const EngArgs& A,
                                          EngOwnerLds& L, int o) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    EngCtl* ctl = A.ctl;
    const int cls = A.own_cls[o];
    const int32_t kbase = A.own_kbase[o];
    const TaskClass& c = t.classes[cls];  // (read field by field where used: scalar loads)
    uint8_t* fbh = A.own_fb + (size_t)o * nc.npad;
    const int N = nc.n;
    // every node's key for the class (rows written by pops of this run meanwhile are read
    // again when those pops are applied)
    for (int i = threadIdx.x; i < kOwnLv / 2 * kOwnSegs; i += kPopThreads) (&L.seg[0][0])[i] = 0;
    for (int i = threadIdx.x; i < kOwnHash; i += kPopThreads) { L.hkey[i] = -1; L.hval[i] = -1; }
    for (int i = threadIdx.x; i < kOwnMaxN / kOwnSub; i += kPopThreads) L.smax[i] = 0;
    for (int i = threadIdx.x; i < kOwnLv; i += kPopThreads) L.lvl[i] = 0;
    if (threadIdx.x < 4) L.fit[threadIdx.x] = 0;
    if (threadIdx.x == 0) L.ok = 1;
    __syncthreads();
    const int nend = ((N + kOwnSeg - 1) / kOwnSeg) * kOwnSeg;
    for (int n0 = 0; n0 < nend; n0 += 2 * kPopThreads) {
        uint32_t v[2] = {0, 0}, fb[2] = {0, 0};
        uint64_t k[2] = {0, 0};
#pragma unroll
        for (int u = 0; u < 2; ++u) {  // two nodes per thread in flight
            const int n = n0 + u * kPopThreads + (int)threadIdx.x;
            if (n < N) k[u] = eng_eval(cf, c, t, nc, n, &fb[u]);
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int n = n0 + u * kPopThreads + (int)threadIdx.x;
            v[u] = own_val(k[u], kbase);
            if (n < nend) L.sv[n] = (uint8_t)v[u];
            {  // the block's level bound (a wave's 64 nodes lie in one block)
                uint32_t mx = v[u] >> 1;
#pragma unroll
                for (int dd = 1; dd < 64; dd <<= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, dd, 64));
                if (lane == 0 && n < nend) atomicMax(&L.smax[n / kOwnSub], mx);
            }
            if (n < N) fbh[n] = (uint8_t)fb[u];
            fit_block_add(L.fit, fb[u]);
            // level counts, aggregated per wave (a wave's 64 nodes share a segment)
            uint64_t act = __ballot(v[u] != 0);
            while (act) {
                const int l0 = __builtin_ctzll(act);
                const uint32_t lv = (uint32_t)__shfl((int)v[u], l0, 64) >> 1;
                const uint64_t m = __ballot(v[u] != 0 && (v[u] >> 1) == lv);
                if (lane == l0) {
                    atomicAdd(&L.lvl[lv], (uint32_t)__popcll(m));
                    atomicAdd(&L.seg[lv >> 1][n / kOwnSeg], (uint32_t)__popcll(m) << (16 * (lv & 1)));
                }
                act &= ~m;
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    uint32_t ap = A.first - 1;  // the last pop whose rows are applied
    uint32_t dp = A.first;      // the next descriptor to look at
    uint64_t t0 = 0;            // wave 0: since when nothing has changed
    int seen = -1;              // wave 0 (timeline): the last own pop seen
    for (;;) {
        if (wave == 0) {
            bool ok = own_scan_desc(A, L, cls, dp);
            if (!ok && lane == 0) L.ok = 0;
        } else if (wave == 1) {  // `done`, then the log entries of the next pops (-2: not published yet)
            const uint32_t dn = ld_sc1(&ctl->done);
            uint64_t x[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) x[k] = ld_sc1(&ctl->tlog[(ap + 1 + k) % kEngLog][lane]);
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const bool got = __ballot((uint32_t)(x[k] >> 32) != ap + 1 + k) == 0;
                L.lognode[k][lane] = got ? (int)(uint32_t)x[k] : -2;
            }
            if (lane == 0) L.dn = dn;
        }
        own_drain();  // (an apply's FitDelta bits, before the barrier)
        __syncthreads();
        if (!L.ok) return;
        const int next = L.next;
        const uint32_t dn = L.dn;
        const bool moved = (uint32_t)L.dp != dp;
        if (next >= 0 && next != seen && wave == 0) {  // timeline: this owner's pop seen
            ETL(A, (uint32_t)next, 20);
            seen = next;
        }
        dp = (uint32_t)L.dp;
        if (next == -2) {  // the run's end: no package of this owner is pending
            if (threadIdx.x == 0) st_sc1(&ctl->own_ap[o], ap + (1u << 30));
            return;
        }
        // apply the pops that are done, up to pop next - 4 (or up to the last one looked at)
        const uint32_t want = next >= 0 ? (uint32_t)next - 4 : dp - 1;
        const uint32_t bound = (int32_t)(dn - want) < 0 ? dn : want;
        if ((int32_t)(bound - ap) > 0) {
            const int nb = min((int)(bound - ap), kPopThreads / 64);
            if (!own_apply(cf, nc, t, c, A, L, fbh, kbase, ap + 1, nb)) return;
            ap += (uint32_t)nb;
            if (threadIdx.x == 0) st_sc1(&ctl->own_ap[o], ap);
            t0 = 0;
            continue;
        }
        if (next >= 0 && (int32_t)(ap - ((uint32_t)next - 4)) >= 0) {
            own_drain();
            if (!own_package(cf, nc, t, c, A, L, fbh, kbase, (uint32_t)next, &ap)) return;
            dp = (uint32_t)next + 1;
            t0 = 0;
            continue;
        }
        if (wave == 0 && !moved) {  // nothing new: a bounded wait
            __builtin_amdgcn_s_sleep(2);
            const uint64_t now = eng_now();
            if (!t0) t0 = now;
            if (lane == 0 && (ld_sc1(&ctl->err) != 0 || now - t0 > kEngDescTicks)) {
                if (ld_sc1(&ctl->err) == 0)
                    __hip_atomic_store(&ctl->err, (uint32_t)kEngErrDesc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                L.ok = 0;
            }
        }
        if (moved) t0 = 0;
    }
}

}  // namespace kbhip
