// kbhip_engine.hip — the persistent pop engine: one
// resident grid places a run of batched job pops (allocate.go:110-185, one
// gang chunk of one task class per pop) with no kernel launch per pop.
// Roles by block (kbhip_engine.h):
//   [0, nw)        workers: node range [b * npb, (b + 1) * npb)
//   [nw, nw + ng)  mergers: group g = workers b with b % ng == g
//   nw + ng        final merger (the package of the group lists' top 128)
//   nw + ng + 1    placer
//   nw + ng + 2    dispatcher (one wave)
// Hand-offs are self-tagged 8-byte granules {seq << 32 | value} written with
// sc1 stores and polled with sc1 loads (MI355X_MICROARCH.md, R2), or sc1 row
// stores drained before the sc1 `done` flag (valid forms, table row 1).
// Every wait is bounded (s_memrealtime) and gives up once ctl->err is set.
#include <hip/hip_runtime.h>

#define KBHIP_STAMPS_OFF  // phase stamps belong to k_pop_batch (kbhip_kernels.hip)
#include "kbhip_batch.h"
#include "kbhip_engine.h"

namespace kbhip {

constexpr uint64_t kEngWaitTicks = 200000000ull;  // 2 s at 100 MHz: a pipeline wait that long is a fault
constexpr uint64_t kEngArriveTicks = 500000ull;  // 5 ms for every block of the grid to start (co-residency)
constexpr uint64_t kEngDescTicks = 400000000ull;  // a block waiting for its next descriptor

__device__ __forceinline__ uint64_t eng_now() { return __builtin_amdgcn_s_memrealtime(); }

// Diagnostic timeline: lane 0 of the calling wave stamps event ev of pop p
// (null buffer: nothing; the check is a scalar branch on a kernel argument).
#define ETL(A, p, ev)                                                                                    \
    do {                                                                                                 \
        if ((A).tl && (threadIdx.x & 63) == 0)                                                           \
            (A).tl[(size_t)((p) % kEngTlSlots) * kEngTlEvents + (ev)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)

// A bounded wait: call tick() once per unsuccessful poll; false = give up
// (timed out: the error is recorded; or another block recorded one).
struct EngWait {
    EngCtl* ctl;
    uint64_t limit;
    uint64_t t0 = 0;
    uint32_t it = 0;
    __device__ EngWait(EngCtl* c, uint64_t l) : ctl(c), limit(l) {}
    __device__ __forceinline__ bool tick(uint32_t code = kEngErrWait) {
        __builtin_amdgcn_s_sleep(1);
        if ((++it & 63) != 0) return true;
        const uint64_t now = eng_now();
        if (!t0) t0 = now;
        if (ld_sc1(&ctl->err) != 0) return false;
        if (now - t0 > limit) {
            __hip_atomic_store(&ctl->err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return false;
        }
        return true;
    }
};

// The lane index through an opaque move: addresses derived from it are
// computed where they are used instead of being hoisted out of the role
// loops and held (or spilled) for the kernel's lifetime.
__device__ __forceinline__ int eng_lane() {
    int l;
    asm volatile("v_and_b32 %0, 63, %1" : "=v"(l) : "v"((int)threadIdx.x));
    return l;
}

// A wave-uniform copy of v through readfirstlane (scalar registers): the
// evaluation functions read the task class field by field, from LDS one
// dependent access after another otherwise.
template <typename T>
__device__ __forceinline__ T eng_uniform(const T& v) {
    static_assert(sizeof(T) % 4 == 0, "dwords");
    T r;
    const uint32_t* s = (const uint32_t*)&v;
    uint32_t* d = (uint32_t*)&r;
#pragma unroll
    for (int i = 0; i < (int)(sizeof(T) / 4); ++i) d[i] = (uint32_t)__builtin_amdgcn_readfirstlane((int)s[i]);
    return r;
}

// A descriptor's TaskClass (words kEngDescClass.. of w, LDS; or of x, one
// descriptor word per lane) in scalar registers.
__device__ __forceinline__ TaskClass eng_class(const uint32_t* w) {
    return eng_uniform(*(const TaskClass*)(w + kEngDescClass));
}
__device__ __forceinline__ TaskClass eng_class_x(uint32_t x) {
    TaskClass c;
    uint32_t* d = (uint32_t*)&c;
#pragma unroll
    for (int i = 0; i < (int)(sizeof(TaskClass) / 4); ++i)
        d[i] = (uint32_t)__builtin_amdgcn_readlane((int)x, kEngDescClass + i);
    return c;
}

// The pop's descriptor as a block sees it (from the device ring).
struct EngDesc {
    uint32_t op, cls, m, gang, ent32, min_avail, ready, epoch, slot;
    int32_t kbase, kshift, kidxmax;
};
__device__ __forceinline__ EngDesc eng_decode(const uint32_t* w) {
    EngDesc d;
    d.cls = w[kDwCls];
    d.m = w[kDwFlags] & 0xff;
    d.gang = (w[kDwFlags] >> 8) & 1;
    d.ent32 = (w[kDwFlags] >> 9) & 1;
    d.op = (w[kDwFlags] >> 12) & 0xf;
    d.min_avail = w[kDwMinAvail];
    d.ready = w[kDwReady];
    d.epoch = w[kDwEpochSlot] & 0xffff;
    d.slot = w[kDwEpochSlot] >> 16;
    d.kbase = (int32_t)w[kDwKbase];
    d.kshift = (int32_t)w[kDwKshift];
    d.kidxmax = (int32_t)w[kDwKidxmax];
    return d;
}
__device__ __forceinline__ PopArgs eng_args(const EngDesc& d) {
    PopArgs a{};
    a.cls = (int32_t)d.cls;
    a.n_tasks = (int32_t)d.m;
    a.gang_mode = (int32_t)d.gang;
    a.min_avail = (int32_t)d.min_avail;
    a.ready_count = (int32_t)d.ready;
    a.epoch = d.epoch;
    a.placement = 2;
    a.kbase = d.kbase;
    a.kshift = d.kshift;
    a.kidxmax = d.kidxmax;
    a.ent32 = (int32_t)d.ent32;
    a.fit_set = 0;
    return a;
}

// Wave 0: wait for descriptor p in the device ring, leave its words in
// w[kEngDescWords] (LDS).
__device__ __forceinline__ bool eng_wait_desc(EngCtl* ctl, uint32_t p, uint32_t* w) {
    const int lane = threadIdx.x & 63;
    const uint64_t* src = &ctl->desc[p % kEngRing][lane];
    EngWait wt(ctl, kEngDescTicks);
    for (;;) {
        const uint64_t x = ld_sc1(src);
        if (__ballot((uint32_t)(x >> 32) != p) == 0) {
            w[lane] = (uint32_t)x;
            return true;
        }
        if (!wt.tick(kEngErrDesc)) return false;
    }
}

// Wave 0: wait until ctl->done reaches `want`.
__device__ __forceinline__ bool eng_wait_done(EngCtl* ctl, uint32_t want) {
    EngWait wt(ctl, kEngWaitTicks);
    for (;;) {
        const uint32_t v = (uint32_t)__builtin_amdgcn_readfirstlane((int)ld_sc1(&ctl->done));
        if ((int32_t)(v - want) >= 0) return true;
        if (!wt.tick()) return false;
    }
}

// Until the tag (high half) of the granule *w reads q: kPollDepth sc1 loads of
// it in flight, one issued per check, so that the wave sees the store about
// a round trip / kPollDepth after it lands rather than up to two round trips
// (every lane loads the same word: one request).  false: gave up (EngWait).
constexpr int kPollDepth = 8;
__device__ __forceinline__ bool eng_poll_tag(EngCtl* ctl, const uint64_t* w, uint32_t q, uint64_t limit) {
    uint64_t v[kPollDepth];
#pragma unroll
    for (int i = 0; i < kPollDepth; ++i) {
        v[i] = ld_sc1(w);
        __builtin_amdgcn_s_sleep(1);
    }
    EngWait wt(ctl, limit);
    for (;;) {
#pragma unroll
        for (int i = 0; i < kPollDepth; ++i) {
            if ((uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v[i] >> 32)) == q) return true;
            v[i] = ld_sc1(w);
            if (!wt.tick()) return false;
        }
    }
}

// The same for one granule per lane (w: this lane's, null: none): until every
// lane's tag has read q (tags only grow while a slot is in use).
__device__ __forceinline__ bool eng_poll_tags(EngCtl* ctl, const uint64_t* w, uint32_t q, uint64_t limit) {
    uint64_t v[kPollDepth];
#pragma unroll
    for (int i = 0; i < kPollDepth; ++i) {
        v[i] = w ? ld_sc1(w) : ((uint64_t)q << 32);
        __builtin_amdgcn_s_sleep(1);
    }
    bool seen = false;
    EngWait wt(ctl, limit);
    for (;;) {
#pragma unroll
        for (int i = 0; i < kPollDepth; ++i) {
            seen = seen || (uint32_t)(v[i] >> 32) == q;
            if (__ballot(!seen) == 0) return true;
            v[i] = (w && !seen) ? ld_sc1(w) : ((uint64_t)q << 32);
            if (!wt.tick()) return false;
        }
    }
}

// Wave 0: candidate `lane` of pop q (-1: none), waiting for the granules of
// copy `copy` (the placer stores kEngCandCopies: a few tens of pollers each).
__device__ __forceinline__ bool eng_wait_cands(EngCtl* ctl, uint32_t q, int* node, int copy) {
    const int lane = threadIdx.x & 63;
    const uint64_t* src = &ctl->cands[q % kEngSlots][copy % kEngCandCopies][lane];
    if (!eng_poll_tag(ctl, &ctl->cands[q % kEngSlots][copy % kEngCandCopies][0], q, kEngWaitTicks)) return false;
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

// Top 128 of the 8 waves' descending 128-lists (a0: ranks 0..63, a1: 64..127);
// the result in w0[0] / w1[0] (every wave calls).
template <typename T>
__device__ __forceinline__ void block_merge128_all(T (*w0)[64], T (*w1)[64], T a0, T a1, int wave, int lane) {
    w0[wave][lane] = a0;
    w1[wave][lane] = a1;
    __syncthreads();
#pragma unroll
    for (int s = kPopThreads / 128; s >= 1; s >>= 1) {
        if (wave < s) {
            T x0 = w0[wave][lane], x1 = w1[wave][lane];
            wave_merge128_desc(x0, x1, w0[wave + s][lane], w1[wave + s][lane]);
            w0[wave][lane] = x0;
            w1[wave][lane] = x1;
        }
        __syncthreads();
    }
}

// Top 256 of the 8 waves' descending 256-lists (a[k]: ranks 64k .. 64k + 63);
// the result in wl[k][0] (every wave calls).
__device__ __forceinline__ void block_merge256_all(uint32_t (*wl)[kPopThreads / 64][64], const uint32_t* a, int wave,
                                                   int lane) {
#pragma unroll
    for (int k = 0; k < 4; ++k) wl[k][wave][lane] = a[k];
    __syncthreads();
#pragma unroll
    for (int s = kPopThreads / 128; s >= 1; s >>= 1) {
        if (wave < s) {
            uint32_t x[4], y[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) { x[k] = wl[k][wave][lane]; y[k] = wl[k][wave + s][lane]; }
            wave_merge256_desc(x, y);
#pragma unroll
            for (int k = 0; k < 4; ++k) wl[k][wave][lane] = x[k];
        }
        __syncthreads();
    }
}

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t x) {
    x += __shfl_xor(x, 1, 64);
    x += __shfl_xor(x, 2, 64);
    x += __shfl_xor(x, 4, 64);
    x += __shfl_xor(x, 8, 64);
    x += __shfl_xor(x, 16, 64);
    return x + __shfl_xor(x, 32, 64);
}

// The evaluation of a worker's node: the mutable row columns through sc1
// (the placer writes them write-through from another CU), the static ones
// plain; all loads issued before the predicates' early exits (eval_node).
__device__ __forceinline__ uint64_t eng_eval_row(const Conf& cf, const TaskClass& c, const DevTables& t,
                                                 const NodeCols& nc, int n, const Row& r, uint8_t fl, uint32_t* fb) {
    const bool st = static_pred_f(cf, c, t, nc, n, fl);
    const int32_t na = (st && cf.score_mult) ? na_weight(c, t, nc, n) : 0;
    const uint64_t pw[4] = {0, 0, 0, 0};  // engine classes carry no host ports
    int32_t s;
    bool passed;
    const uint64_t k = dyn_key(cf, c, t, nc, r, pw, n, st, na, &s, &passed);
    *fb = fit_bits(c, r, passed);
    return k;
}
__device__ __forceinline__ uint64_t eng_eval(const Conf& cf, const TaskClass& c, const DevTables& t,
                                             const NodeCols& nc, int n, uint32_t* fb) {
    const uint8_t fl = nc.flags[n];
    const Row r = load_row_sc1(nc, n);
    return eng_eval_row(cf, c, t, nc, n, r, fl, fb);
}

// ---------------------------------------------------------------------------
// LDS of the roles (one union: the kernel's footprint is the largest role's)
// ---------------------------------------------------------------------------
struct EngWorkerLds {
    uint32_t wl[4][kPopThreads / 64][64];  // per-wave top-256 lists (register k of wave w in wl[k][w])
    uint32_t out[128];                     // the published top 128 (late exclusion)
    uint32_t skip[kEngMaxNpb / 32];        // pop p-3's (then also p-2's) candidates among this block's nodes
    uint8_t fb[2][kEngMaxNpb];             // FitDelta bits of pops p (p % 2) and p-1
    alignas(16) uint32_t desc[kEngDescWords];
    uint32_t fitb[2][4];                   // FitDelta counts of pops p (p % 2) and p-1
    int ok;
};
struct EngMergerLds {
    uint32_t wl[kPopThreads / 64][64], wl2[kPopThreads / 64][64];
    alignas(16) uint32_t desc[kEngDescWords];
    int ok;
};
// The placer's rows: four pops' candidates (slot 64 * (pop % 4) + lane) and
// two packages' 128 entries (pop q's in slots kEngStage + 128 * (q % 2) + e).
constexpr int kEngStage = 4 * 64, kEngRc = kEngStage + 2 * kEngPkgN;
using EngRowCache = RowCacheT<kEngRc, 10>;
struct EngPlacerLds {
    EngRowCache rc;
    uint8_t flags[kEngRc];
    int32_t xn[4][64];           // candidates of pop q in ring q % 4 (-1: none)
    uint64_t wl64[kPopThreads / 64][64];
    uint32_t pkey[2][kEngPkgN];  // pop q's package keys (q % 2)
    uint32_t s64[64];            // the merged list without pop p-1's candidates
    uint32_t e[3][64];           // re-evaluated keys of pops p-1 / p-2 / p-3's candidates (sorted)
    uint8_t fbp[3][64];          // FitDelta bits of the three sets
    // the front's evaluation of pops p-2 / p-3's candidates (set 0 / 1, by ring lane)
    uint32_t fe[3][64];
    uint8_t fkind[3][64], ffb[3][64];
    int32_t fna[3][64], fs1a[3][64], fs1p[3][64];
    int rows_seq;                // the last pop whose candidates' rows are in their ring (eng_finish)
    int xn_seq;                  // the last pop whose candidates are in their ring of L.xn (P3)
    // set 0 of the next pop evaluated ahead of the decision: on each candidate's row before this
    // pop (variant 0, in fe / ...) and after one Allocate of this pop's class (variant 1, below);
    // the decision's commits per candidate (ccm: Allocates | Pipelines << 8) select one
    int32_t ccm[64];
    uint32_t v1e[64];
    uint8_t v1fb[64], v1kind[64];
    int32_t v1s1p[64], v1s1a[64];
    int v1_seq[2];               // the pop whose variant-1 keys (0) / depth-1 scores (1) are in v1*
    uint32_t pre64[64];          // the next pop's package list merged with its sets 1 and 2 (P3 adds set 0)
    int pre_seq;
    uint8_t x2use[64], x3use[64];  // pop p-2's candidate not p-1's; pop p-3's neither
    int32_t srcslot[64];         // the final list's candidate j: its row's slot (a ring or a package entry)
    int32_t fitin[4];
    alignas(16) uint32_t desc[2][kEngDescWords];  // pop q's descriptor and class (q % 2)
    alignas(16) uint32_t ndesc[kEngDescWords];    // pop ndesc_seq's, prefetched during P2 (a front reads it)
    int ndesc_seq;
    int hash_seq;                // the pop whose front hashed its previous candidates (wave 2)
    int drop_seq;                // the pop whose package the front already cut to L.s64 (wave 3)
    int sort_seq[3];             // the pop whose front sorted set s's keys into L.e / L.fbp
    uint64_t gran[64];           // the pop's result granules (0: none), stored to the host by wave 5
    uint64_t gfit[2];            // ... and its FitDelta granules (stop 1)
    int ok;
    int gran_seq;                // the pop whose granules are in gran / gfit
    uint32_t apmin;              // list mode: every owner has applied this pop (as last read)
};
// A class owner (list mode): its class's key byte for every node, the node
// counts per level (and per segment of kOwnSeg nodes and level: the package
// scan reads only the segments that hold its entries), the FitDelta counts.
constexpr int kOwnHash = 1024;
constexpr int kOwnPre = 192;  // a package's entries before pop p-2's candidates (<= 64) leave: >= 128 stay
constexpr int kOwnSub = 128;  // the package scan's blocks: two per wave step (32 lanes x 4 nodes each)
static_assert(kOwnSeg % kOwnSub == 0 && kOwnSeg / kOwnSub <= 64, "a segment's blocks fit one wave's lanes");
struct EngOwnerLds {
    alignas(16) uint8_t sv[kOwnMaxN]; // node n: level << 1 | pipelined (0: not a candidate of the class)
    uint32_t seg[kOwnLv / 2][kOwnSegs];  // nodes per (level, segment): level l in half l & 1 of word [l / 2]
                                         // (a segment holds at most kOwnSeg < 2^16 nodes)
    uint32_t lvl[kOwnLv];             // nodes per level
    uint32_t fit[4];                  // FitDelta counts over every node (fit_bits)
    int32_t hkey[kOwnHash];           // node set (an apply batch's nodes; a package's left-out nodes)
    int32_t hval[kOwnHash];
    union {
        uint32_t keys[256];           // a package's entries: the top kOwnPre without pop p-3's candidates
        int32_t lognode[8][64];       // the next apply batch's candidates as read with `done` (-2: not yet)
    };
    int32_t slot_entry[kEngPkgN];     // package slot -> its entry (-1: none)
    uint32_t wcnt[4];                 // kept entries per wave (the package's compaction)
    uint32_t nkeys;
    uint32_t smax[kOwnMaxN / kOwnSub];  // per block of kOwnSub nodes: at least its highest level (raised by
                                        // every re-key, made exact by every package scan that reads the block)
    int32_t act[kOwnSegs];            // the segments the package scan reads ...
    int32_t take[kOwnSegs];           // ... how many level-thr nodes it takes from each ...
    int32_t hic[kOwnSegs];            // ... and how many nodes above thr each holds
    int32_t nact, thr;                // their number; the threshold level L
    int32_t xfit[4];                  // FitDelta bits of the left-out nodes
    alignas(16) uint32_t desc[kEngDescWords];
    int32_t next, dp, ok;             // wave 0's findings: own pop / exit / none, next descriptor to look at
    uint32_t dn;                      // `done` as wave 0 last read it
};
union EngLds {
    EngWorkerLds w;
    EngMergerLds m;
    EngPlacerLds p;
};
union EngLdsList {
    EngOwnerLds o;
    EngPlacerLds p;
};
static_assert(sizeof(EngLdsList) <= 160 * 1024, "one block per CU");

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
        }
        if (wave == 0) ETL(A, p, 22);
    }
}

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
template <bool LIST>
__device__ __forceinline__ void eng_front(const Conf& cf, const NodeCols& nc, const DevTables& t, const EngArgs& A,
                                          EngPlacerLds& L, uint32_t q, int wave) {
    const int lane = threadIdx.x & 63;
    EngCtl* ctl = A.ctl;
    EngRowCache& rc = L.rc;
    if (wave == 0) return;
    const bool loads = wave == 3 || wave == 4 || wave == 6 || wave == 7;
    const int k = wave == 3 ? 0 : wave == 4 ? 1 : wave - 4;  // field block of a loading wave
    const EngPkg* pk = A.pkg + (q % kEngSlots);
    // the package's loads first (in flight during the rest; reloaded below if early)
    uint64_t v[16];
    if (loads)
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = ld_sc1(&pk->w[8 * k + (i >> 1)][lane + 64 * (i & 1)]);
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
    // two generations of the package's loads in flight, checked in turn (the package is
    // read whole each time: four waves of one block, a few tens of GB/s), so that it is
    // in registers about a round trip after it lands
    uint64_t w[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) w[i] = ld_sc1(&pk->w[8 * k + (i >> 1)][lane + 64 * (i & 1)]);
    bool got = false;
    EngWait wt(ctl, kEngWaitTicks);
    for (;;) {
        bool miss = false;
#pragma unroll
        for (int i = 0; i < 16; ++i) miss |= (uint32_t)(v[i] >> 32) != q;
        if (__ballot(miss) == 0) { got = true; break; }
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = ld_sc1(&pk->w[8 * k + (i >> 1)][lane + 64 * (i & 1)]);
        miss = false;
#pragma unroll
        for (int i = 0; i < 16; ++i) miss |= (uint32_t)(w[i] >> 32) != q;
        if (__ballot(miss) == 0) {
#pragma unroll
            for (int i = 0; i < 16; ++i) v[i] = w[i];
            got = true;
            break;
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) w[i] = ld_sc1(&pk->w[8 * k + (i >> 1)][lane + 64 * (i & 1)]);
        if (!wt.tick()) break;
    }
    if (got) {
        const int base = kEngStage + kEngPkgN * (int)(q % 2);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int f = 8 * k + (i >> 1), e = lane + 64 * (i & 1), sl = base + e;
            const uint32_t x = (uint32_t)v[i];
            if (f == kPkKey) L.pkey[q % 2][e] = x;
            else if (f < kPkFlags) ((uint32_t*)&rc.row[sl])[f - kPkRow] = x;
            else if (f == kPkFlags) L.flags[sl] = (uint8_t)x;
            else if (f == kPkNa) rc.na[sl] = (int32_t)x;
            else rc.s1[sl] = (int32_t)x;
        }
        if (k == 0) {
            for (int w = 0; w < 4; ++w) { rc.pw[base + lane][w] = 0; rc.pw[base + 64 + lane][w] = 0; }
            // pop q-1's candidates out of the package (its keys, written above by this wave),
            // once wave 2 has hashed the rings; else the placer's P2 does it
            bool hashed = false;
            for (int i = 0; i < 4096 && !hashed; ++i) {
                hashed = __hip_atomic_load(&L.hash_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == (int)q;
                if (!hashed) __builtin_amdgcn_s_sleep(1);
            }
            if (hashed) {
                uint32_t w8[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) w8[i] = (uint32_t)__builtin_amdgcn_readlane((int)dw, i);
                eng_drop_stale(L, eng_args(eng_decode(w8)), q);
                __builtin_amdgcn_s_waitcnt(0xc07f);
                if (lane == 0) __hip_atomic_store(&L.drop_seq, (int)q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
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

__global__ __launch_bounds__(kPopThreads) void k_engine(Conf cf, NodeCols nc, DevTables t, EngArgs A) {
    __shared__ EngLds lds;
    __shared__ int arrived;
    const int b = blockIdx.x;
    if (!eng_arrive(A, &arrived)) {
        if (b == A.nw + A.ng + 2) eng_not_resident(A);
        return;
    }
    if (b < A.nw) {
        eng_worker(cf, nc, t, A, lds.w, b);
    } else if (b < A.nw + A.ng) {
        eng_merger(A, lds.m, b - A.nw);
    } else if (b == A.nw + A.ng) {
        eng_final(cf, nc, t, A, lds.m);
    } else if (b == A.nw + A.ng + 1) {
        eng_placer<false>(cf, nc, t, A, lds.p);
    } else if (threadIdx.x < 64) {
        eng_dispatch(A);
    }
}

// List mode: class owners, the placer, the dispatcher.  A
// kernel of its own, so that the owners' registers do not weigh on the sweep
// engine's placer.
__global__ __launch_bounds__(kPopThreads) void k_engine_lists(Conf cf, NodeCols nc, DevTables t, EngArgs A) {
    __shared__ EngLdsList lds;
    __shared__ int arrived;
    const int b = blockIdx.x;
    if (!eng_arrive(A, &arrived)) {
        if (b == A.nown + 1) eng_not_resident(A);
        return;
    }
    if (b < A.nown) eng_owner(cf, nc, t, A, lds.o, b);
    else if (b == A.nown) eng_placer<true>(cf, nc, t, A, lds.p);
    else if (threadIdx.x < 64) eng_dispatch(A);
}

int engine_grid(const EngArgs& A) { return A.nown > 0 ? A.nown + 2 : A.nw + A.ng + 3; }

hipError_t launch_engine(const Conf& cf, const NodeCols& nc, const DevTables& t, const EngArgs& A, hipStream_t st) {
    if (A.nown > 0)
        hipLaunchKernelGGL(k_engine_lists, dim3(engine_grid(A)), dim3(kPopThreads), 0, st, cf, nc, t, A);
    else
        hipLaunchKernelGGL(k_engine, dim3(engine_grid(A)), dim3(kPopThreads), 0, st, cf, nc, t, A);
    return hipGetLastError();
}

hipError_t engine_occupancy(int* blocks_per_cu, bool lists) {
    if (lists) return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, k_engine_lists, kPopThreads, 0);
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, k_engine, kPopThreads, 0);
}

}  // namespace kbhip
