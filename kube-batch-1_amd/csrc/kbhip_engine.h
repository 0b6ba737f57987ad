// kbhip_engine.h — the persistent pop engine (kbhip_engine.hip): memory
// layout shared by the host driver (session/03_pop.cpp) and the kernels.
//
// One resident grid serves a run of batched job pops (allocate.go:110-185 for
// a gang's chunk of one task class) without a kernel launch
// per pop:
//   * worker blocks own node ranges: per pop they evaluate their nodes
//     (PredicateFn + NodeOrderFn -> selection key, kbhip_eval.h) and publish
//     their top-128 keys;
//   * merger blocks (one per group of workers) merge their group's lists;
//   * the final merger merges the group lists and gathers the rows of the
//     top 128 into a package (EngPkg);
//   * the placer block loads the package, drops the previous pop's candidates,
//     re-evaluates the previous two pops' candidates from its own LDS rows,
//     places the chunk (parallel levels, kbhip_batch.h) and writes the rows back;
//   * the dispatcher block copies pop descriptors from the host's pinned ring
//     into a device ring.
// Pop p's workers read the node rows as pop p-4 left them (its write-back is
// drained before `done` reaches p-4) and leave out the candidates of pops p-3
// and p-2; pop p-1's candidates may sit in the merged top-128 with stale keys
// and the placer drops them.  Those three sets are the only rows that can have
// changed since pop p-4, and the placer holds the rows of all three (four rings
// of 64 rows) and re-evaluates them.  So the placer sees every node's exact key.
// List mode keeps the same contract: the owner of pop p's class keys every
// node on its rows as of pop p-4 or later (each applied after that pop's
// `done`), leaves out pops p-3 and p-2's candidates, and packages the top 128.
#pragma once
#include <stdint.h>

namespace kbhip {

constexpr int kEngRing = 8;       // device descriptor ring
constexpr int kEngHostRing = 16;  // host descriptor ring (pinned)
constexpr int kEngSlots = 4;      // list / candidate slots (pop % 4)
constexpr int kEngMaxGroups = 8;  // merger blocks
constexpr int kEngListWords = 136;  // a list: 128 tagged keys + 4 tagged counts (+ pad), 17 lines
constexpr int kEngMaxNpb = 8192;  // nodes per worker block
constexpr int kEngWorkersMax = 512;
#ifndef KBHIP_CAND_COPIES
#define KBHIP_CAND_COPIES 8  // (tuning builds: host and device must agree, so the whole library)
#endif
constexpr int kEngCandCopies = KBHIP_CAND_COPIES;  // the candidate granules' copies (the workers' polls spread over them)

// The final merger's package for pop p (slot p % kEngSlots): the top 128
// keys of the group lists with every entry's node row and its node-affinity
// weight and depth-1 score for the pop's class, field-major (word f of entry
// e at w[f][e]): 0 key, 1..28 the Row (kbhip_eval.h, as 32-bit words), 29
// flags, 30 na, 31 s1.  Every word is a self-tagged granule {p << 32 | value}
// (one sc1 store each): the placer takes the package once every tag reads p.
constexpr int kEngPkgN = 128, kEngPkgFields = 32;
enum : int { kPkKey = 0, kPkRow = 1, kPkFlags = 29, kPkNa = 30, kPkS1 = 31 };
struct EngPkg {
    uint64_t w[kEngPkgFields][kEngPkgN];
};

// Descriptor words (each {seq << 32 | value}, self-tagged: a reader takes a
// descriptor once all kEngDescWords tags read its sequence number): the pop's
// arguments, then the words of its TaskClass from kEngDescClass on (every
// block that reads the descriptor has the class in the same round trip).
constexpr int kEngDescWords = 64, kEngDescClass = 8;
enum : int { kDwCls = 0, kDwFlags, kDwMinAvail, kDwReady, kDwEpochSlot, kDwKbase, kDwKshift, kDwKidxmax };
// kDwFlags: m | gang << 8 | ent32 << 9 | op << 12
enum : uint32_t { kEngOpPop = 0, kEngOpExit = 1 };

// List mode: one owner block per task class keeps every
// node's selection key for its class in LDS, updated from the rows each pop
// touches; the owner of pop p's class writes pop p's package.  Owners read
// the pops' candidates and classes from a log of kEngLog pops (the placer does
// not overwrite an entry some owner has not applied yet: own_ap).
constexpr int kEngLog = 64;
constexpr int kEngOwnMax = 256;
constexpr int kOwnSeg = 1792, kOwnSegs = 64, kOwnMaxN = kOwnSeg * kOwnSegs;  // nodes per owner (LDS key bytes: 112 KiB)
static_assert(kOwnSeg % 256 == 0, "a segment is whole scan steps (64 lanes x 4 nodes)");
constexpr int kOwnLv = 128;  // key levels (score - kbase + 1) an owner's byte holds: 1 .. kOwnLv - 1

// Device control block (hipMalloc'ed, zeroed at each launch).
struct EngCtl {
    uint32_t done;  // the last pop whose node write-back is visible (sc1)
    uint32_t pad0[31];
    uint32_t err;   // first error (kEngErr*), 0: none; every wait gives up once it is set
    uint32_t pad1[31];
    uint32_t arrive;  // blocks that have started (the grid runs only once every block is resident)
    uint32_t pad2[63];
    uint64_t desc[kEngRing][kEngDescWords];  // descriptors, slot seq % kEngRing
    uint64_t cands[kEngSlots][kEngCandCopies][64];  // pop p's candidates {p << 32 | node (or 0xffffffff)}, in copies
    uint64_t pkg_ready[kEngSlots][16];  // {p << 32 | 1} once package p % kEngSlots has landed (a line each)
    uint64_t tlog[kEngLog][64];  // list mode: pop p's candidates {p << 32 | node}, slot p % kEngLog
    uint64_t tcls[kEngLog];      // ... and its class {p << 32 | cls}
    uint32_t own_ap[kEngOwnMax]; // owner o: the last pop whose rows it applied (written by owner o only)
};
enum : uint32_t { kEngErrWait = 1, kEngErrDesc = 2, kEngErrClass = 3, kEngErrResident = 4 };
// kEngErrResident: not every block of the grid became resident within kEngArriveTicks (other
// kernels hold CUs — another session's, or another process's); the grid ends at once, serving
// nothing, and the host starts it again (not a fault).  The exit word then carries bit 42.

// Kernel arguments beyond the session's tables.
struct EngArgs {
    EngCtl* ctl;
    uint64_t* blists;          // [kEngSlots][nw][kEngListWords] worker lists (+ 2 count words)
    uint64_t* glists;          // [kEngSlots][ng][kEngListWords] group lists (+ 4 count words)
    EngPkg* pkg;               // [kEngSlots] the final merger's packages
    const uint64_t* hring;     // [kEngHostRing][kEngDescWords] pinned host descriptors (device view)
    uint64_t* hexit;           // pinned host word: {exit seq | idle << 40 | 1 << 41 | not resident << 42} at the end
    uint32_t idle_ticks;       // the dispatcher ends the run after this long without a descriptor (100 MHz)
    void* out;                 // result slots (PopOut, pinned host memory, device view)
    uint32_t first;            // the first pop of this launch (earlier pops are written back)
    int nw, npb, ng;           // workers, nodes per worker, merger groups
    uint64_t* tl;              // diagnostic event timeline (option "engine_timeline"), or null
    int quick;                 // 0 (a test mode): no fast path, every feasible candidate through the levels rounds
    // list mode (nown > 0): blocks [0, nown) own a class each; then the placer and the dispatcher
    int nown;
    const int32_t* own_cls;    // [nown] owner o's class
    const int32_t* own_kbase;  // [nown] its key base (KeyFormat::base)
    uint8_t* own_fb;           // [nown][npad] each node's FitDelta bits for the owner's class (owner-private)
    int kshift, kidxmax;       // the session's 32-bit key format (KeyFormat::shift / idxmax)
};
constexpr uint32_t kEngIdleTicks = 10000000u;  // 100 ms without a descriptor: the run ends (100 MHz ticks)
// Event timeline (s_memrealtime, 100 MHz): kEngTlEvents words per pop, pop p in slot p % kEngTlSlots.
constexpr int kEngTlSlots = 32768, kEngTlEvents = 64;

}  // namespace kbhip
