// engine_dev.h — the persistent pop engine's shared device code: bounded
// waits, self-tagged granules, descriptors, block merges, the blocks' LDS
// layouts (kbhip_engine.hip, kbhip_engine_lists.hip).
#pragma once
#include <hip/hip_runtime.h>

#define KBHIP_STAMPS_OFF  // phase stamps belong to k_pop_batch (kbhip_kernels.hip)
#include "../kbhip_batch.h"
#include "../kbhip_engine.h"

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

// Polling shape (tuning builds, profiles/r06_poll.sh): sc1 loads in flight per
// granule poll, and the s_sleep between polls (64-cycle units; 0 = none).
// Measured at C4 (profiles/r06p_*, r06q_*: device period per pop): 8 loads in
// flight / sleep 1 (r05) 8.25-8.28 us, 2 / 0 8.05-8.08, 1 / 1 7.98-8.02,
// 1 / 2 8.00, 1 / 8 8.15: the pollers' own loads slowed the hand-offs they
// wait for (every poll is a request to the line's home L2 channel).
#ifndef KBHIP_POLL_DEPTH
#define KBHIP_POLL_DEPTH 1
#endif
#ifndef KBHIP_POLL_SLEEP
#define KBHIP_POLL_SLEEP 2
#endif
__device__ __forceinline__ void eng_pause() {
    if constexpr (KBHIP_POLL_SLEEP > 0) __builtin_amdgcn_s_sleep(KBHIP_POLL_SLEEP);
}

// A bounded wait: call tick() once per unsuccessful poll; false = give up
// (timed out: the error is recorded; or another block recorded one).
struct EngWait {
    EngCtl* ctl;
    uint64_t limit;
    uint64_t t0 = 0;
    uint32_t it = 0;
    __device__ EngWait(EngCtl* c, uint64_t l) : ctl(c), limit(l) {}
    __device__ __forceinline__ bool tick(uint32_t code = kEngErrWait) {
        eng_pause();
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
// it in flight, one issued per check (every lane loads the same word: one
// request).  false: gave up (EngWait).
constexpr int kPollDepth = KBHIP_POLL_DEPTH;
__device__ __forceinline__ bool eng_poll_tag(EngCtl* ctl, const uint64_t* w, uint32_t q, uint64_t limit) {
    uint64_t v[kPollDepth];
#pragma unroll
    for (int i = 0; i < kPollDepth; ++i) {
        v[i] = ld_sc1(w);
        eng_pause();
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
        eng_pause();
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
using EngRowCache = RowCacheT<kEngRc, 11>;  // (2048 hash slots for 512 rows: short probe chains)
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

}  // namespace kbhip
