// engine_sweep.h — the sweep engine's workers, mergers and final merger
// (k_engine).
#pragma once
#include <hip/hip_runtime.h>

#define KBHIP_STAMPS_OFF  // phase stamps belong to k_pop_batch (kbhip_kernels.hip)
#include "../kbhip_batch.h"
#include "../kbhip_engine.h"
#include "engine_dev.h"

namespace kbhip {

// ---------------------------------------------------------------------------
// worker
// ---------------------------------------------------------------------------
// Pop p's FitDelta counts leave out pops p-3 (not evaluated), p-2 and p-1's
// candidates (the placer counts those on their final rows): pop p-1's
// candidates are known one pop later, so pop p publishes pop p-1's counts.
// Wave 0: subtract the bits of this block's nodes among pop q's candidates
// (node, one per lane) from counts set `set` (zeroing them: a node of two
// such pops leaves the counts once).
__device__ __forceinline__ void eng_fit_drop(EngWorkerLds& L, int set, int node, int lo, int cnt) {
    const int lane = threadIdx.x & 63;
    const int o = node - lo;
    const bool own = node >= 0 && o >= 0 && o < cnt;
    uint32_t fb = 0;
    if (own) {
        fb = L.fb[set][o];
        L.fb[set][o] = 0;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int k = __popcll(__ballot((fb >> q) & 1u));
        if (lane == q && k) atomicSub(&L.fitb[set][q], (uint32_t)k);
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
}
// Wave 0: publish pop q's FitDelta counts (two 16-bit counts per word).
__device__ __forceinline__ void eng_fit_publish(const EngArgs& A, EngWorkerLds& L, uint32_t q, int b) {
    const int lane = threadIdx.x & 63;
    uint64_t* dst = A.blists + ((size_t)(q % kEngSlots) * A.nw + b) * kEngListWords;
    const int set = (int)(q % 2);
    if (lane < 2) {
        const uint32_t v = (L.fitb[set][2 * lane] & 0xffff) | (L.fitb[set][2 * lane + 1] << 16);
        st_sc1(&dst[128 + lane], ((uint64_t)q << 32) | v);
    }
}

__device__ __forceinline__ void eng_worker(const Conf& cf, const NodeCols& nc, const DevTables& t, const EngArgs& A,
                           EngWorkerLds& L, int b) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    EngCtl* ctl = A.ctl;
    const int lo = b * A.npb;
    const int cnt = nc.n - lo < A.npb ? (nc.n - lo > 0 ? nc.n - lo : 0) : A.npb;
    if (threadIdx.x == 0) L.ok = 1;
    uint32_t cpub = A.first - 1;  // wave 0: the last pop whose FitDelta counts are published
    for (uint32_t p = A.first;; ++p) {
        const int set = (int)(p % 2), pset = 1 - set;
        // 1. the pop's descriptor; the node rows as pop p-4 left them; pop p-3's candidates
        for (int i = threadIdx.x; i < (cnt + 31) / 32; i += kPopThreads) L.skip[i] = 0;
        __syncthreads();  // the previous pop done (wave 0 cleared L.ok if it failed)
        if (!L.ok) return;
        if (threadIdx.x < 4) L.fitb[set][threadIdx.x] = 0;
        const int tb = b == 0 ? 10 : -1;  // timeline: worker 0
        if (wave == 0) {
            // pop p's descriptor; meanwhile pop p-1's counts once pop p-2's candidates are
            // known (a placement whose task found no node reads them: they must not wait
            // for a descriptor the host sends only after that placement's results)
            bool ok = true;
            {
                const uint64_t* src = &ctl->desc[p % kEngRing][lane];
                EngWait wt(ctl, kEngDescTicks);
                for (;;) {
                    const uint64_t x = ld_sc1(src);
                    if (__ballot((uint32_t)(x >> 32) != p) == 0) {
                        L.desc[lane] = (uint32_t)x;
                        break;
                    }
                    if (cpub + 1 < p) {
                        int node = -1;
                        bool have = true;
                        if (p >= A.first + 2) {
                            const uint64_t cw = ld_sc1(&ctl->cands[(p - 2) % kEngSlots][b % kEngCandCopies][lane]);
                            have = __ballot((uint32_t)(cw >> 32) != p - 2) == 0;
                            node = (int)(uint32_t)cw;
                        }
                        if (have) {
                            eng_fit_drop(L, pset, node, lo, cnt);
                            eng_fit_publish(A, L, p - 1, b);
                            cpub = p - 1;
                        }
                    }
                    if (!wt.tick(kEngErrDesc)) { ok = false; break; }
                }
            }
            if (tb >= 0) ETL(A, p, tb);
            const EngDesc d0 = eng_decode(L.desc);  // (LDS written by this wave, in order)
            if (ok && d0.op == kEngOpPop) {
                if (p >= A.first + 4) ok = eng_wait_done(ctl, p - 4);
                if (tb >= 0) ETL(A, p, tb + 1);
                if (ok && p >= A.first + 3) {
                    int node = -1;
                    ok = eng_wait_cands(ctl, p - 3, &node, b);
                    const int o = node - lo;
                    if (ok && node >= 0 && o >= 0 && o < cnt) atomicOr(&L.skip[o >> 5], 1u << (o & 31));
                }
            } else if (ok && cpub + 1 < p) {  // the run ends: the last pop's counts
                int node = -1;
                if (p >= A.first + 2) ok = eng_wait_cands(ctl, p - 2, &node, b);
                if (ok) {
                    eng_fit_drop(L, pset, node, lo, cnt);
                    eng_fit_publish(A, L, p - 1, b);
                    cpub = p - 1;
                }
            }
            if (lane == 0) L.ok = ok;
        }
        __syncthreads();
        if (!L.ok) return;
        const EngDesc d = eng_decode(L.desc);
        if (d.op != kEngOpPop) return;
        const PopArgs a = eng_args(d);
        const TaskClass c = eng_class(L.desc);
        // 2. evaluate, one node per thread and chunk; each wave keeps its top 256
        uint32_t al[4] = {0, 0, 0, 0};
        for (int base = 0; base < cnt; base += kPopThreads) {
            const int o = base + (int)threadIdx.x;
            uint32_t k = 0, fb = 0;
            if (o < cnt && !((L.skip[o >> 5] >> (o & 31)) & 1u)) k = sweep_key<uint32_t>(eng_eval(cf, c, t, nc, lo + o, &fb), a);
            if (o < cnt) L.fb[set][o] = (uint8_t)fb;
            fit_block_add(L.fitb[set], fb);
            const uint32_t ks = wave_sort_desc(k);
            if (base == 0) {
                al[0] = ks;
            } else {
                const uint32_t bl[4] = {ks, 0u, 0u, 0u};
                wave_merge256_desc(al, bl);
            }
        }
        if (tb >= 0 && wave == 0) ETL(A, p, tb + 2);
        block_merge256_all(L.wl, al, wave, lane);
        // 3. pop p-2's candidates (their rows may be in flight; the placer
        // evaluates them): out of the list — the top 256 keeps at least 192
        // others, so its first 128 remaining are the top 128 without them —
        // and out of pop p's counts; publish (wave 0).  Then out of pop p-1's
        // counts, which are complete now.
        if (wave == 0) {
            bool ok = true;
            int node = -1;
            bool any_own = false;
            if (p >= A.first + 2) {
                ok = eng_wait_cands(ctl, p - 2, &node, b);
                const int o = node - lo;
                const bool own = ok && node >= 0 && o >= 0 && o < cnt;
                if (own) atomicOr(&L.skip[o >> 5], 1u << (o & 31));
                any_own = __ballot(own) != 0;
                if (ok && any_own) eng_fit_drop(L, set, node, lo, cnt);
            }
            int run = 0;
#pragma unroll
            for (int k = 0; k < (any_own ? 4 : 0); ++k) {
                const uint32_t v = L.wl[k][0][lane];
                bool keep = v != 0;
                if (keep) {
                    const int o = key_node(v, a) - lo;
                    keep = !((L.skip[o >> 5] >> (o & 31)) & 1u);
                }
                const uint64_t m = __ballot(keep);
                const int pos = run + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                                __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
                if (keep && pos < 128) L.out[pos] = v;
                run += __popcll(m);
            }
            uint32_t o0 = L.wl[0][0][lane], o1 = L.wl[1][0][lane];  // (none of them: the first 128)
            if (any_own) {
                if (lane >= run) L.out[lane] = 0;
                if (64 + lane >= run) L.out[64 + lane] = 0;
                __builtin_amdgcn_s_waitcnt(0xc07f);
                __builtin_amdgcn_wave_barrier();
                o0 = L.out[lane];
                o1 = L.out[64 + lane];
            }
            if (ok) {
                uint64_t* dst = A.blists + ((size_t)(p % kEngSlots) * A.nw + b) * kEngListWords;
                st_sc1(&dst[lane], ((uint64_t)p << 32) | o0);
                st_sc1(&dst[64 + lane], ((uint64_t)p << 32) | o1);
            }
            if (tb >= 0) ETL(A, p, tb + 3);
            if (b == A.nw - 1) ETL(A, p, 18);
            if (ok && cpub + 1 < p) {
                eng_fit_drop(L, pset, node, lo, cnt);
                eng_fit_publish(A, L, p - 1, b);
                cpub = p - 1;
            }
            if (!ok && lane == 0) L.ok = 0;  // (the error is recorded: every block gives up)
        }
    }
}

// The top 128 of pop p's worker lists g, g + stride, ... (cnt of them), in
// (a0: ranks 0..63, a1: 64..127) of each wave: wave w merges lists w, w + 8, ...
// (4 in flight); block_merge128_all then merges the waves'.  false: a wait gave up.
__device__ __forceinline__ bool eng_merge_lists(EngCtl* ctl, const uint64_t* src0, int g, int stride, int cnt,
                                                uint32_t p, uint32_t* a0, uint32_t* a1) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    bool ok = true;
    for (int i0 = wave; i0 < cnt && ok; i0 += 4 * (kPopThreads / 64)) {
        constexpr int kQ = 4;
        uint64_t v0[kQ], v1[kQ];
        const uint64_t* s[kQ];
#pragma unroll
        for (int q = 0; q < kQ; ++q) {
            const int i = i0 + q * (kPopThreads / 64);
            s[q] = i < cnt ? src0 + (size_t)(g + i * stride) * kEngListWords : nullptr;
            v0[q] = s[q] ? ld_sc1(&s[q][lane]) : ((uint64_t)p << 32);
            v1[q] = s[q] ? ld_sc1(&s[q][64 + lane]) : ((uint64_t)p << 32);
        }
        EngWait wt(ctl, kEngWaitTicks);
        for (;;) {
            bool miss = false;
#pragma unroll
            for (int q = 0; q < kQ; ++q) miss |= __ballot((uint32_t)(v0[q] >> 32) != p || (uint32_t)(v1[q] >> 32) != p) != 0;
            if (!miss) break;
            // not all there: wait on the lists' last granules (lanes 2q, 2q + 1: list q's; few
            // bytes, several loads in flight), then reload what is missing
            const int li = lane >> 1;
            const uint64_t* sl = li == 0 ? s[0] : li == 1 ? s[1] : li == 2 ? s[2] : li == 3 ? s[3] : nullptr;
            if (!eng_poll_tags(ctl, sl ? &sl[(lane & 1) ? 127 : 63] : nullptr, p, kEngWaitTicks)) { ok = false; break; }
#pragma unroll
            for (int q = 0; q < kQ; ++q) {
                if (__ballot((uint32_t)(v0[q] >> 32) != p || (uint32_t)(v1[q] >> 32) != p) == 0) continue;
                v0[q] = ld_sc1(&s[q][lane]);
                v1[q] = ld_sc1(&s[q][64 + lane]);
            }
            if (!wt.tick()) { ok = false; break; }
        }
        if (ok)
#pragma unroll
            for (int q = 0; q < kQ; ++q) wave_merge128_desc(*a0, *a1, (uint32_t)v0[q], (uint32_t)v1[q]);
    }
    return ok;
}

// ---------------------------------------------------------------------------
// merger of group g
// ---------------------------------------------------------------------------
// Wave 0 of merger g: pop q's group FitDelta counts — lane i reads worker
// g + i * ng's two count words — summed and published.  block: wait for every
// worker's words; else one attempt (false: some not there yet).
__device__ __forceinline__ bool eng_group_counts(const EngArgs& A, int g, int cg, uint32_t q, bool block, bool* ok) {
    const int lane = threadIdx.x & 63;
    EngCtl* ctl = A.ctl;
    const uint64_t* src0 = A.blists + (size_t)(q % kEngSlots) * A.nw * kEngListWords;
    uint32_t t0 = 0, t1 = 0, t2 = 0, t3 = 0;
    for (int i0 = 0; i0 < cg; i0 += 64) {
        const int i = i0 + lane;
        const uint64_t* s = i < cg ? src0 + (size_t)(g + i * A.ng) * kEngListWords + 128 : nullptr;
        uint64_t x0 = s ? ld_sc1(&s[0]) : ((uint64_t)q << 32), x1 = s ? ld_sc1(&s[1]) : ((uint64_t)q << 32);
        EngWait wt(ctl, kEngWaitTicks);
        while (__ballot((uint32_t)(x0 >> 32) != q || (uint32_t)(x1 >> 32) != q) != 0) {
            if (!block) return false;
            if (!wt.tick()) { *ok = false; return false; }
            if (s) { x0 = ld_sc1(&s[0]); x1 = ld_sc1(&s[1]); }
        }
        const uint32_t y0 = (uint32_t)x0, y1 = (uint32_t)x1;  // two 16-bit counts per word
        t0 += wave_sum_u32(y0 & 0xffff);
        t1 += wave_sum_u32(y0 >> 16);
        t2 += wave_sum_u32(y1 & 0xffff);
        t3 += wave_sum_u32(y1 >> 16);
    }
    uint64_t* dst = A.glists + ((size_t)(q % kEngSlots) * A.ng + g) * kEngListWords;
    if (lane < 4) st_sc1(&dst[128 + lane], ((uint64_t)q << 32) | (lane == 0 ? t0 : lane == 1 ? t1 : lane == 2 ? t2 : t3));
    return true;
}

// Pop p's group list; pop p-1's group counts (complete once the workers know
// pop p-2's candidates: published during the descriptor wait if they come
// first — a placement whose task found no node reads them, and the host may
// send pop p's descriptor only after its results — else after the list).
__device__ __forceinline__ void eng_merger(const EngArgs& A, EngMergerLds& L, int g) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    EngCtl* ctl = A.ctl;
    const int cg = (A.nw - g + A.ng - 1) / A.ng;  // workers of the group: g, g + ng, ...
    if (threadIdx.x == 0) L.ok = 1;
    uint32_t cpub = A.first - 1;  // wave 0: the last pop whose group counts are published
    for (uint32_t p = A.first;; ++p) {
        __syncthreads();  // the previous pop done (wave 0 cleared L.ok if it failed)
        if (!L.ok) return;
        if (wave == 0) {
            bool ok = true;
            const uint64_t* src = &ctl->desc[p % kEngRing][lane];
            EngWait wt(ctl, kEngDescTicks);
            for (;;) {
                const uint64_t x = ld_sc1(src);
                if (__ballot((uint32_t)(x >> 32) != p) == 0) {
                    L.desc[lane] = (uint32_t)x;
                    break;
                }
                if (cpub + 1 < p && eng_group_counts(A, g, cg, p - 1, false, &ok)) cpub = p - 1;
                if (!wt.tick(kEngErrDesc)) { ok = false; break; }
            }
            if (ok && eng_decode(L.desc).op != kEngOpPop && cpub + 1 < p) {  // the run ends
                eng_group_counts(A, g, cg, p - 1, true, &ok);
                cpub = p - 1;
            }
            if (lane == 0) L.ok = ok;
            if (g == 0) ETL(A, p, 24);
        }
        __syncthreads();
        if (!L.ok) return;
        if (eng_decode(L.desc).op != kEngOpPop) return;
        const uint64_t* src0 = A.blists + (size_t)(p % kEngSlots) * A.nw * kEngListWords;
        uint32_t a0 = 0, a1 = 0;
        bool ok = eng_merge_lists(ctl, src0, g, A.ng, cg, p, &a0, &a1);
        if (!ok) L.ok = 0;
        if (g == 0 && wave == 0) ETL(A, p, 25);
        block_merge128_all(L.wl, L.wl2, a0, a1, wave, lane);
        if (!L.ok) return;
        if (wave == 0) {
            uint64_t* dst = A.glists + ((size_t)(p % kEngSlots) * A.ng + g) * kEngListWords;
            st_sc1(&dst[lane], ((uint64_t)p << 32) | L.wl[0][lane]);
            st_sc1(&dst[64 + lane], ((uint64_t)p << 32) | L.wl2[0][lane]);
            if (g == 0) ETL(A, p, 26);
            if (cpub + 1 < p) {
                eng_group_counts(A, g, cg, p - 1, true, &ok);
                cpub = p - 1;
            }
            if (!ok && lane == 0) L.ok = 0;
            if (g == 0) ETL(A, p, 27);
        }
    }
}

// ---------------------------------------------------------------------------
// final merger: the group lists' top 128 with their rows -> the package
// ---------------------------------------------------------------------------
// The nodes of pop p's lists are not pop p-2's candidates (the workers left
// those out); pop p-1's may be among them with stale keys and rows (the placer
// drops them); every other node was last written by pop p-3 or earlier, whose
// write-back the workers saw drained before they evaluated pop p.
__device__ __forceinline__ void eng_final(const Conf& cf, const NodeCols& nc, const DevTables& t, const EngArgs& A,
                          EngMergerLds& L) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    EngCtl* ctl = A.ctl;
    if (threadIdx.x == 0) L.ok = 1;
    for (uint32_t p = A.first;; ++p) {
        __syncthreads();
        if (!L.ok) return;
        if (wave == 0) {
            const bool ok = eng_wait_desc(ctl, p, L.desc);
            if (lane == 0) L.ok = ok;
            ETL(A, p, 20);
        }
        __syncthreads();
        if (!L.ok) return;
        const EngDesc d = eng_decode(L.desc);
        if (d.op != kEngOpPop) return;
        const PopArgs a = eng_args(d);
        const TaskClass c = eng_class(L.desc);
        uint32_t a0 = 0, a1 = 0;
        bool ok = true;
        if (A.ng == 0) {  // no merger level: the worker lists
            ok = eng_merge_lists(ctl, A.blists + (size_t)(p % kEngSlots) * A.nw * kEngListWords, 0, 1, A.nw, p, &a0,
                                 &a1);
        } else if (wave < A.ng) {
            // group list `wave`, polled whole with kFinalDepth loads in flight (one block: a few
            // tens of GB/s), so that it is in registers about a round trip after it lands
            constexpr int kFinalDepth = 4;
            const uint64_t* s = A.glists + ((size_t)(p % kEngSlots) * A.ng + wave) * kEngListWords;
            uint64_t v0[kFinalDepth], v1[kFinalDepth];
#pragma unroll
            for (int i = 0; i < kFinalDepth; ++i) {
                v0[i] = ld_sc1(&s[lane]);
                v1[i] = ld_sc1(&s[64 + lane]);
                __builtin_amdgcn_s_sleep(2);
            }
            bool got = false;
            EngWait wt(ctl, kEngWaitTicks);
            while (!got) {
#pragma unroll
                for (int i = 0; i < kFinalDepth; ++i) {
                    if (__ballot((uint32_t)(v0[i] >> 32) != p || (uint32_t)(v1[i] >> 32) != p) == 0) {
                        a0 = (uint32_t)v0[i];
                        a1 = (uint32_t)v1[i];
                        got = true;
                        break;
                    }
                    v0[i] = ld_sc1(&s[lane]);
                    v1[i] = ld_sc1(&s[64 + lane]);
                    if (!wt.tick()) break;
                }
                if (!got && ld_sc1(&ctl->err) != 0) break;
            }
            ok = got;
        }
        if (!ok) L.ok = 0;
        block_merge128_all(L.wl, L.wl2, a0, a1, wave, lane);
        if (!L.ok) return;
        if (wave == 0) ETL(A, p, 21);
        EngPkg* pk = A.pkg + (p % kEngSlots);
        const uint64_t tag = (uint64_t)p << 32;
        if (wave < 2) {  // entry e = 64 * wave + lane: its key, row, flags, node-affinity weight, depth-1 score
            const int e = 64 * wave + lane;
            const uint32_t k = wave == 0 ? L.wl[0][lane] : L.wl2[0][lane];
            const int n = k ? key_node(k, a) : -1;
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
        }
        if (wave == 0) ETL(A, p, 22);
        __syncthreads();
        // one flag for the whole package: the placer polls it with one load instead of
        // re-reading its blocks until every granule's tag is p
        if (threadIdx.x == 0) st_sc1(&ctl->pkg_ready[p % kEngSlots][0], tag | 1u);
    }
}

}  // namespace kbhip
