// kbhip_internal.h — declarations shared by the host encoder/driver and the
// kernel translation unit (not part of the public ABI).
#pragma once
#include <hip/hip_runtime.h>

#include "kbhip_types.h"

namespace kbhip {

// Read-only per-session tables (device pointers).
struct DevTables {
    const TaskClass* classes;
    const Term* terms;
    const Req* reqs;
    const int32_t* vals;
    const int64_t* valint;  // per global value id: parsed int64 (Gt/Lt)
    const uint8_t* valok;   // per global value id: strconv.ParseInt succeeded
    const uint64_t* masks;  // tolerated-taint / port-conflict / own-port words
    // pod (anti-)affinity (kbhip_affinity.h)
    const int32_t* aff_items;  // programs: ea pairs, ipa quads, upd triples
    int32_t* aff_cnt;          // count tables, indexed cnt_off + domain
    int32_t* aff_scalar;       // PA target totals, session counters
    // placement 7 with per-domain candidates: the best key of every domain of the
    // class's dd_space over all blocks (kDedupMax entries; zero between launches)
    uint64_t* dd_max;
};

// The per-task path's control block set up on the device (CtrlInit, kbhip_types.h).
hipError_t launch_ctrl_init(PopCtrl* ctrl, const CtrlInit& ci, hipStream_t st);
// Per-task sweep; dbg (debug only): per-node keys, raw inter-pod counts,
// [lo, hi, F, max key]: rows of 2 npad + 4 words per task of the chunk; commit_here = the last block commits (one GPU).  Sharded
// sessions reduce ctrl->slot[task_i] across shards and then launch_commit_task.
hipError_t launch_sweep_argmax(const Conf& cf, const NodeCols& nc, const DevTables& t, PopCtrl* ctrl, int task_i,
                               uint64_t* walk, hipStream_t st, bool commit_here = true, uint64_t* dbg = nullptr,
                               bool defer_visits = false, const int64_t* ipa_pre = nullptr);
// defer_visits (one GPU): the GetAccessibleResource mutation of the walk runs as a
// second, grid-wide kernel (k_visit_mutate) instead of in the committing block.
hipError_t launch_commit_task(const NodeCols& nc, const DevTables& t, PopCtrl* ctrl, int task_i, const uint64_t* walk,
                              hipStream_t st);
// Inter-pod affinity priority prepass: min / max of the raw count over all
// nodes for task task_i (interpod_affinity.go:214-226) -> ctrl->ipa_lo/hi;
// counts (optional, npad entries): each node's raw count, which the sweep that
// follows on the same state then reads (launch_sweep_argmax's ipa_pre).
hipError_t launch_ipa_minmax(const NodeCols& nc, const DevTables& t, PopCtrl* ctrl, int task_i, hipStream_t st,
                             int64_t* counts = nullptr);

// Reclaim / preempt (kbhip_evict.hip): per-node order keys of the task of
// ctrl->cls[0] (by_score 1: predicates + score, preempt; 0: predicates only,
// reclaim), *count += passing nodes; one node-row update (op 0 evict, 1
// pipeline, 2 unpipeline).
// kbhip_sweep_scores' standalone sweep: keys per node, the passing count in
// 8 counters (counts[32 g], g = 0..7; the caller zeroes and sums them).
hipError_t launch_evict_read(const void* buf, size_t bytes, hipStream_t st);  // time_sweeps_cold = 2
void set_sweep_variant(int v);  // option "sweep_variant" (process-wide tuning knob)
hipError_t launch_score_sweep(const Conf& cf, const NodeCols& nc, const DevTables& t, const TaskClass& c,
                              const PopCtrl* ctrl, uint64_t* keys, uint32_t* counts, hipStream_t st);
hipError_t launch_rank_nodes(const Conf& cf, const NodeCols& nc, const DevTables& t, const PopCtrl* ctrl,
                             int by_score, uint64_t* keys, uint32_t* count, hipStream_t st);
// Wide score ranges: the passing keys of launch_rank_nodes (n keys, zeros
// dropped; *count = passing nodes) sorted descending by four stable 8-bit
// counting passes over the score (hist: rank_hist_words(n) words; tmp: n keys).
hipError_t launch_rank_radix(const uint64_t* keys, int n, const uint32_t* count, uint32_t* hist, uint64_t* tmp,
                             uint64_t* sorted, hipStream_t st);
// The walk order by a hand-written stable counting sort over the score (class
// score range [slo, shi] of at most 256 values; hipErrorInvalidValue beyond):
// keys, sorted (descending key order), *count += passing nodes; hist holds
// rank_hist_words(n) words of scratch.
hipError_t launch_rank_sorted(const Conf& cf, const NodeCols& nc, const DevTables& t, const TaskClass& c,
                              const PopCtrl* ctrl, int by_score, int slo, int shi, uint64_t* keys, uint32_t* hist,
                              uint64_t* sorted, uint32_t* count, hipStream_t st);
size_t rank_hist_words(int n_nodes);
// One session's ranking request in a batched launch (what-if sessions).
struct RankDesc {
    Conf cf;
    NodeCols nc;
    DevTables t;
    TaskClass c;  // the request's class (ctrl->cls[0]), here so a block needs no load chain to it
    const PopCtrl* ctrl;
    int by_score, shi, nb, nblk;
    uint64_t* keys;
    uint32_t* hist;
    uint64_t* sorted;
    uint32_t* count;
};
hipError_t fill_rank_desc(RankDesc* q, const Conf& cf, const NodeCols& nc, const DevTables& t, const TaskClass& c,
                          const PopCtrl* ctrl, int by_score, int slo, int shi, uint64_t* keys, uint32_t* hist,
                          uint64_t* sorted, uint32_t* count);
hipError_t launch_rank_sorted_multi(const RankDesc* d_desc, int n_desc, int max_nblk, hipStream_t st);
// Count-table deltas (pod (anti-)affinity): idx >= 0 aff_cnt, < 0 aff_scalar[-1 - idx]; distinct indices.
hipError_t launch_tab_add(const DevTables& t, const int32_t* idx, const int32_t* delta, int n, hipStream_t st);
hipError_t launch_rel_add(const NodeCols& nc, const int32_t* node, const int64_t* d, int n, hipStream_t st);
// carry's node-row patch: entry i writes the low size bytes (8, 4 or 1) of val at device address addr
struct RowPatch {
    uint64_t addr, val;
    int32_t size, pad;
};
hipError_t launch_row_patch(const RowPatch* e, int n, hipStream_t st);
// op 0 Releasing += (rc, rm, rg), 1 a pipelined pod committed, 2 uncommitted, on this shard's row n of
// global node g (n = -1: another shard's node — the replicated count tables only)
hipError_t launch_node_op(const NodeCols& nc, const DevTables& t, int op, int n, int g, int cls, int64_t rc,
                          int64_t rm, int64_t rg, hipStream_t st);

// Selection-key format of a batched launch: 32-bit keys when the class's
// score range and the node count fit (kbhip_kernels.hip, PopArgs).
struct KeyFormat {
    bool use32 = false;
    bool ent32 = false;  // parallel-levels placement entries fit 32 bits too
    int32_t base = 0, shift = 0, idxmax = 0;
};
struct ShardMsg;  // kbhip_eval.h
struct MboxArgs;  // kbhip_eval.h
// Batched path v2: one launch per pop chunk; results land in `out_dev`
// (device pointer of a pinned host PopOut, pop_out_bytes() long).
// placement 2: parallel levels; 6: sessions with Backfilled nodes; 7:
// pod-affinity classes; 3 (node-array shards): no placement — the shard's
// top-64 with rows goes to shard_out for the all-gather, then
// launch_shard_place places.
hipError_t launch_pop_batch(const Conf& cf, const NodeCols& nc, const DevTables& t, int cls, int n_tasks,
                            int gang_mode, int min_avail, int ready_count, uint32_t epoch, uint64_t* cand,
                            uint32_t* arrive, void* out_dev, hipStream_t st, int placement, const KeyFormat& kf,
                            int fit_set, ShardMsg* shard_out = nullptr, const struct MboxArgs* mbox = nullptr);
// The placement of a sharded batched pop on the gathered ShardMsgs (world of
// them, rank order): identical on every shard; each writes back its own rows.
// flags (mailbox exchange): this rank's mailbox flags of the pop's slot —
// the kernel waits until rank r's flag (flags[16 r]) reads seq.
hipError_t launch_shard_place(const Conf& cf, const NodeCols& nc, const DevTables& t, int cls, int n_tasks,
                              int gang_mode, int min_avail, int ready_count, uint32_t epoch, const KeyFormat& kf,
                              const ShardMsg* msgs, int world, void* out_dev, hipStream_t st,
                              const uint64_t* flags = nullptr, uint32_t seq = 0, struct PopLink* link = nullptr);
// Chain state of overlapped batched pops (kbhip_kernels.hip, k_pop_batch_ov):
// done = sequence number of the last pop whose node write-back is visible;
// touched[e % kLinkSlots][i] = {e << 32 | node}, candidate i of pop e (node
// -1: none).  At session open: done 0, every slot tagged 0 with no nodes.
constexpr int kMaxGroups = 32;  // >= kGroups of kbhip_kernels.hip
// Overlapped pops' lists as self-tagged granules: 64 keys + 4 FitDelta counts
// per block and per group, 80 words (5 lines) apart.
constexpr int kCandStride = 80;
constexpr int kMaxDep = 2;     // previous pops an overlapped pop runs beside (streams - 1)
constexpr int kMaxSpeculate = 6;  // predicted batched pops queued behind the running one (option "speculate")
constexpr int kLinkSlots = 4;  // > kMaxDep: a slot is rewritten only after its readers finished
// rows[e % kLinkSlots][f][i] = {e << 32 | half f of candidate i's row after
// pop e} — kRowWords 32-bit halves of Row's dynamic and static fields (not
// Backfilled: overlapped pops run only in sessions without it), written after
// pop e's write-back drained: the next pops read their previous pops'
// candidates' rows from here (contiguous, self-tagged) instead of polling
// `done` and gathering the node columns.
constexpr int kRowWords = 22;
struct PopLink {
    uint32_t done;
    uint32_t pad0[31];
    uint64_t touched[kLinkSlots][64];
    uint64_t rows[kLinkSlots][kRowWords][64];
};
// Overlapped shard pops (mailbox exchange): this shard's sweep of pop mb.seq
// beside pop mb.seq-1's k_shard_place (launch_shard_place with `link`), whose
// candidates it leaves out and then re-evaluates once that pop's write-back on
// this device is done (prev_chained: pop mb.seq-1 ran as such a pop and
// published its candidates in `link`).  Sends the shard's message like
// placement 3.
hipError_t launch_shard_sweep_ov(const Conf& cf, const NodeCols& nc, const DevTables& t, int cls, const TaskClass& cl,
                                 int n_tasks, int gang_mode, int min_avail, int ready_count, uint32_t epoch,
                                 uint64_t* cand, uint32_t* arrive, const KeyFormat& kf, int fit_set, PopLink* link,
                                 int prev_chained, const MboxArgs& mb, hipStream_t st);
// Overlapped batched pop number `seq` (>= 1) on stream st; pop seq-1 may
// still run on the other stream: it leaves that pop's candidates out of its
// sweep and re-evaluates them once pop seq-1's write-back is done.  cand
// holds (blocks + kMaxGroups) * 64 keys, arrive (3 * kMaxGroups + 1) * 32
// counters, both private to the launch's stream; fit_set alternates per
// launch on a stream (FitDelta counter sets).
hipError_t launch_pop_batch_ov(const Conf& cf, const NodeCols& nc, const DevTables& t, int cls, const TaskClass& cl,
                               int n_tasks, int gang_mode, int min_avail, int ready_count, uint32_t epoch,
                               uint64_t* cand, uint32_t* arrive, void* out_dev, hipStream_t st, const KeyFormat& kf,
                               PopLink* link, uint32_t seq, int fit_set, int dep, uint32_t msg_from);
// Node updates of given placements again (after launch_undo_pop).
hipError_t launch_redo_pop(const NodeCols& nc, const DevTables& t, int cls, int n, const int32_t* node,
                           const int32_t* kind, hipStream_t st);
// One task's walk FitDelta histogram on the current state (kbhip_kernels.hip):
// the task is ctrl's task 0 (class, fallback node, inter-pod affinity min /
// max); chosen >= 0: the node its walk stopped at (ctrl->slot[0] <- its walk
// key on this shard, 0 elsewhere: all-reduce MAX before the histogram on
// shards — launch_fit_key, then launch_fit_count).
hipError_t launch_fit_key(const Conf& cf, const NodeCols& nc, const DevTables& t, PopCtrl* ctrl, int chosen,
                          hipStream_t st);
hipError_t launch_fit_count(const Conf& cf, const NodeCols& nc, const DevTables& t, PopCtrl* ctrl, int chosen,
                            int chosen_kind, int32_t* out4, hipStream_t st);
// Inverse node updates of a batched pop's placements (a retracted prediction).
hipError_t launch_undo_pop(const NodeCols& nc, const DevTables& t, int cls, int n, const int32_t* node,
                           const int32_t* kind, hipStream_t st);
int pop_blocks(int n_nodes, int* R_out);
// A batched pop of one session in a multi-session launch (what-if sessions,
// placement 6 or 7): the arguments of launch_pop_batch.
constexpr int kPopMulti = 8;  // sessions per launch (kernel argument space)
struct PopReq {
    Conf cf;
    NodeCols nc;
    DevTables t;
    int cls, n_tasks, gang_mode, min_avail, ready_count;
    uint32_t epoch;
    KeyFormat kf;
    uint64_t* cand;
    uint32_t* arrive;
    void* out;
    int placement, fit_set;
};
// Launches every request (grouped by nodes per lane, key type and placement,
// kPopMulti per launch; *launches = launches made).
hipError_t launch_pop_batch_multi(const PopReq* reqs, int n, hipStream_t st, int* launches);
// A what-if session's per-task chunk (k_sweep_argmax_multi): m tasks of the
// control block `ctrl`, committed on the device (defer: the visited nodes'
// GetAccessibleResource mutation by k_visit_mutate_multi).
struct SweepReq {
    Conf cf;
    NodeCols nc;
    DevTables t;
    PopCtrl* ctrl;
    uint64_t* walk;
    int m;
    int defer;
};
hipError_t launch_sweep_multi(const SweepReq* reqs, int n, int k, hipStream_t st, int* launches);
size_t pop_out_bytes();
// The persistent pop engine (kbhip_engine.hip, kbhip_engine.h): one resident
// grid of engine_grid(A) blocks serving batched pops from a descriptor ring.
struct EngArgs;
hipError_t launch_engine(const Conf& cf, const NodeCols& nc, const DevTables& t, const EngArgs& A, hipStream_t st);
hipError_t engine_occupancy(int* blocks_per_cu, bool lists = false);  // lists: the list-mode kernel
int engine_grid(const EngArgs& A);
#ifdef KBHIP_STAMPS
hipError_t set_stamp_buffer(uint64_t* p);
#endif
#ifdef KBHIP_TIMELINE
hipError_t set_timeline_buffer(uint64_t* p);
#endif
struct PopOutHost {  // host view of the device PopOut: self-tagged granules
    uint64_t g[kMaxChunk];
    uint64_t fit[2];
};

}  // namespace kbhip
