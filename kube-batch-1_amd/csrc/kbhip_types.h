// kbhip_types.h — device-side data layout of the placement engine (shared by
// the host encoder and the HIP kernels).
//
// Node state lives in HBM as structure-of-arrays columns, one element per
// node, node index = position in the KBS1 snapshot (sorted by name, so the
// reference's map-order tie-break is pinned to the lowest index).  Resource
// quantities are int64: the reference keeps them as float64 that always hold
// exact integers, so integer arithmetic on device is
// exact and comparisons reduce to the LessEqual tolerance form r - rr < min.
#pragma once
#include <stdint.h>

namespace kbhip {

constexpr int kBlock = 256;      // threads per sweep block (4 wave64)
constexpr int kTopK = 64;        // candidates kept per block / tasks per batched chunk
constexpr int kMaxChunk = 64;    // tasks handed to the device per pop chunk
constexpr int64_t kMinCPU = 10, kMinGPU = 10, kMinMem = 10LL * 1024 * 1024;  // resource_info.go:54-56

// Node columns (device pointers).  Labels: one int32 column per "selector
// key" (keys referenced by any pending task's selector / node affinity),
// holding a global value id or -1 when the node lacks the key.
struct NodeCols {
    int64_t *idle_cpu, *idle_mem, *idle_gpu;   // NodeInfo.Idle
    int64_t *rel_cpu, *rel_mem, *rel_gpu;      // NodeInfo.Releasing
    int64_t *bf_cpu, *bf_mem, *bf_gpu;         // NodeInfo.Backfilled
    int64_t *acpu, *amem;                      // k8s allocatable (LR / BRA capacity)
    int64_t *nzc, *nzm;                        // k8s NodeInfo.nonzeroRequest
    int32_t *pods, *maxtasks;                  // len(node.Pods()), Allocatable.MaxTaskNum
    uint8_t *flags;                            // bit0: Spec.Unschedulable
    int32_t *labels;                           // [n_keys][npad]
    uint64_t *taints;                          // [taint_words][npad] NoSchedule/NoExecute taint ids
    uint64_t *ports;                           // [port_words][npad] used (ip, proto, port) ids
    int32_t *dom;                              // [n_spaces][dom_stride] domain ids of ALL nodes (-1: none)
    int32_t n, npad, n_keys, taint_words, port_words;
    int32_t base;        // global index of local row 0 (node-array shard; 0 on one GPU)
    int32_t dom_stride;  // row stride of dom (>= total node count)
};

// A compiled label requirement (labels.Requirement over node labels).
enum : int32_t { OP_IN = 0, OP_NOTIN = 1, OP_EXISTS = 2, OP_DNE = 3, OP_GT = 4, OP_LT = 5,
                 OP_NAME_IN = 6, OP_NAME_NOTIN = 7, OP_FALSE = 8 };
struct Req {
    int32_t key;      // label column (or unused for name ops)
    int32_t op;
    int32_t nvals;    // value ids at vals[val_off .. val_off+nvals)
    int32_t val_off;  // for OP_NAME_*: the node index (or -1: no node of that name)
    int64_t rhs;      // Gt/Lt right-hand side
};
// A conjunction of requirements (one NodeSelectorTerm, or the nodeSelector).
struct Term {
    int32_t req_off, req_n;
    int32_t weight;  // preferred terms: Weight; required terms: unused
    int32_t pad;
};

// A task class: everything the sweep needs about a pending task.  Tasks of a
// gang usually share one class, which is what lets a whole pop run from one
// node sweep (the batched path).
struct TaskClass {
    int64_t ireq_cpu, ireq_mem, ireq_gpu;  // InitResreq (fit, allocate.go:153,173)
    int64_t req_cpu, req_mem, req_gpu;     // Resreq (what Allocate/Pipeline subtract)
    int64_t nz_cpu, nz_mem;                // GetNonzeroRequests of the pod (LR / BRA)
    int32_t backfill;                      // pod carries the backfill annotation
    int32_t nsel_term;                     // -1 or term index: nodeSelector (AND)
    int32_t req_term_off, req_term_n;      // required node-affinity terms (OR); n<0: no filter
    int32_t pref_term_off, pref_term_n;    // preferred node-affinity terms (weighted)
    int32_t tol_off;                       // taint_words tolerated masks
    int32_t pconf_off;                     // port_words conflict masks
    int32_t pown_off;                      // port_words own port bits (committed on placement)
    int32_t has_ports;
    int32_t pred_err;   // predicates fail on every node (e.g. an invalid selector)
    int32_t score_err;  // NodeOrderFn errors on every node: all nodes dropped
    // pod (anti-)affinity program (kbhip_affinity.h); aff != 0 -> per-task path
    int32_t aff;
    int32_t ea_off, ea_n;                  // aff_items pairs (space, cnt_off)
    int32_t pa_space, pa_cnt, pa_total, pa_self;
    int32_t paa_space, paa_cnt;
    int32_t ipa_off, ipa_n;                // aff_items quads (space, cnt_off, sess, weight)
    int32_t upd_off, upd_n;                // aff_items triples (type, space, off)
    int32_t pw_lo;  // host-port window: the class's conflict / own masks cover port words
                    // pw_lo .. pw_lo + kPortWin - 1 (port ids sorted by protocol, port, IP)
    int32_t dd_space;  // placement 7: the topology space whose domains the batched sweep keeps one
                       // candidate of (the class kills a domain by placing into it), -1: none
    int32_t dd_ndom;   // ... its number of domains (<= kDedupMax)
};
constexpr int kDedupMax = 1024;  // domains of a dd_space (the sweep's per-block LDS table)
constexpr int kPortWin = 4;  // port words a class's masks span (its ports' 256-id window)

// Session-wide constants of the plugin configuration.
struct Conf {
    int32_t pred_on;     // predicates plugin enabled in the tiers
    int32_t score_mult;  // number of enabled nodeorder tier entries (0 = no NodeOrderFn)
    int32_t w_lr, w_bra, w_na, w_pa;  // nodeorder.go:177-249 weights
};

// Per-pop control block in device memory.
struct PopCtrl {
    int32_t stop;          // KBHIP_STOP_* once decided, -1 while running
    int32_t n_done;        // tasks consumed
    int32_t ready_count;   // AllocatedStatuses of the job
    int32_t min_avail;
    int32_t gang_mode;
    int32_t n_tasks;
    int32_t any_bf;        // some node has Backfilled != 0 (GetAccessibleResource mutates Idle)
    int32_t fallback;      // lowest node holding a session-placed pod (-1 none; nodeorder.go:78-93)
    int32_t mode;          // 0: allocate (best node, gang stop); 1: backfill (first fit, no stop)
    int32_t pad;
    uint32_t epoch;        // tag of the result granules (0: none are written)
    int32_t pad2;
    uint64_t* out;         // result granules in pinned host memory (PopOut of kbhip_batch.h) or null
    int32_t cls[kMaxChunk];        // task class of each task of the chunk
    int32_t res_node[kMaxChunk];
    int32_t res_kind[kMaxChunk];
    uint32_t arrive[kMaxChunk];    // per-task block arrival counters (general path)
    uint64_t slot[kMaxChunk];      // per-task max key (general path)
    int64_t ipa_lo[kMaxChunk];     // inter-pod affinity min / max count over nodes (0-initialised)
    int64_t ipa_hi[kMaxChunk];
    int32_t fit[kMaxChunk][4];     // per task: walk nodes, negative cpu / memory / GPU FitDelta (fit_bits)
};

// The per-task path's chunk set-up (k_ctrl_init writes it into the device
// PopCtrl: no host-to-device copy per chunk).
struct CtrlInit {
    int32_t ready_count, min_avail, gang_mode, n_tasks, any_bf, fallback, mode;
    uint32_t epoch;
    uint64_t* out;
    int32_t cls[kMaxChunk];
};

// Packed selection key: max key wins = highest score, then lowest node index.
// key = (score + 2^31) << 32 | (0x7fffffff - idx) << 1 | pipelined ; 0 = none
__host__ __device__ inline uint64_t pack_key(int32_t score, int32_t idx, int32_t pipelined) {
    return ((uint64_t)((uint32_t)score ^ 0x80000000u) << 32) | ((uint64_t)(0x7fffffff - idx) << 1) |
           (uint64_t)(pipelined & 1);
}
__host__ __device__ inline int32_t key_idx(uint64_t k) { return 0x7fffffff - (int32_t)((k >> 1) & 0x7fffffff); }
__host__ __device__ inline int32_t key_score(uint64_t k) { return (int32_t)((uint32_t)(k >> 32) ^ 0x80000000u); }
__host__ __device__ inline int32_t key_kind(uint64_t k) { return (k & 1) ? 2 : 1; }

}  // namespace kbhip
