// kbhip_eval.h — the per-node evaluation and commit arithmetic of the
// placement kernels: predicates, scores, fit, selection key, node-row and
// pod-affinity commits.  __host__ __device__ so that the same functions the
// kernels run can also be replayed on the host by the test-only entry point
// kbhip_debug_replay (checked against the CPU oracle without a GPU); the
// placement path itself runs them on the device only.
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>

#include "kbhip_internal.h"

#define KBHIP_HD __host__ __device__ __forceinline__

namespace kbhip {

// ---------------------------------------------------------------------------
// node row + evaluation
// ---------------------------------------------------------------------------
struct Row {  // the dynamic part of a node's state
    int64_t idle_cpu, idle_mem, idle_gpu, rel_cpu, rel_mem, rel_gpu, bf_cpu, bf_mem, bf_gpu;
    int64_t acpu, amem, nzc, nzm;
    int32_t pods, maxtasks;
};

// Node-array shards, batched pops: what each shard contributes
// to a pop — its top-64 keys with the rows the placement needs — exchanged by
// one all-gather; every shard then places the chunk on the merged list.
struct ShardCand {
    uint64_t key;    // 64-bit selection key (global node index), 0 = none
    int32_t node;    // global node index, -1 = none
    int32_t na;      // static node-affinity weight of the node for the class
    Row row;
    uint64_t pw[4];  // host-port words
};
struct ShardMsg {
    uint32_t fit[4];  // the shard's sweep FitDelta counts (walk nodes, cpu, memory, GPU)
    uint32_t pad[2];
    ShardCand c[kTopK];
};
static_assert(sizeof(ShardCand) % 8 == 0 && sizeof(ShardMsg) % 8 == 0, "mailbox copies move 8-byte words");

// Peer mailboxes (kbhip_shard_connect_mailbox): every rank's device holds one;
// for each batched pop every shard writes its ShardMsg straight into every
// rank's mailbox (its own included) — over xGMI when the ranks are on
// different GPUs — and then a self-tagged flag word {pop sequence number}
// per destination; the placement kernel of each rank waits for the W flags of
// its own mailbox.  Two slots (sequence parity): a shard can run at most one
// pop ahead of the slowest, whose reads of the other slot are then done.
constexpr int kMaxWorld = 16;
constexpr int kMboxSlots = 2;
struct Mailbox {
    uint64_t flag[kMboxSlots][kMaxWorld][16];  // [slot][source][0]: sequence number (a 128-B line each)
    ShardMsg msg[kMboxSlots][kMaxWorld];
};
struct MboxArgs {                 // kernel argument of a shard's sweep (world 0: no mailbox)
    Mailbox* dst[kMaxWorld];      // every rank's mailbox as mapped in this process
    int32_t rank, world;
    uint32_t seq;
    int32_t pad;
};

// Host-port words of a class: its window of the port columns (TaskClass::pw_lo).
KBHIP_HD int port_win(const TaskClass& c, const NodeCols& nc) {
    const int k = nc.port_words - c.pw_lo;
    return k < kPortWin ? k : kPortWin;
}
KBHIP_HD int64_t port_at(const TaskClass& c, const NodeCols& nc, int w, int n) {
    return (int64_t)(c.pw_lo + w) * nc.npad + n;
}

KBHIP_HD Row load_row(const NodeCols& nc, int n) {
    Row r;
    r.idle_cpu = nc.idle_cpu[n]; r.idle_mem = nc.idle_mem[n]; r.idle_gpu = nc.idle_gpu[n];
    r.rel_cpu = nc.rel_cpu[n]; r.rel_mem = nc.rel_mem[n]; r.rel_gpu = nc.rel_gpu[n];
    r.bf_cpu = nc.bf_cpu[n]; r.bf_mem = nc.bf_mem[n]; r.bf_gpu = nc.bf_gpu[n];
    r.acpu = nc.acpu[n]; r.amem = nc.amem[n]; r.nzc = nc.nzc[n]; r.nzm = nc.nzm[n];
    r.pods = nc.pods[n]; r.maxtasks = nc.maxtasks[n];
    return r;
}

KBHIP_HD bool req_match(const DevTables& t, const NodeCols& nc, const Req& r, int n) {
    // labels.Requirement.Matches (apimachinery/pkg/labels/selector.go:192-236)
    switch (r.op) {
        case OP_NAME_IN: return n + nc.base == r.val_off;      // field selector metadata.name
        case OP_NAME_NOTIN: return n + nc.base != r.val_off;
        case OP_FALSE: return false;
        default: break;
    }
    const int v = nc.labels[(int64_t)r.key * nc.npad + n];
    switch (r.op) {
        case OP_IN:
        case OP_NOTIN: {
            bool hit = false;
            for (int i = 0; i < r.nvals; ++i) hit |= t.vals[r.val_off + i] == v;
            if (r.op == OP_IN) return v >= 0 && hit;
            return v < 0 || !hit;
        }
        case OP_EXISTS: return v >= 0;
        case OP_DNE: return v < 0;
        case OP_GT: return v >= 0 && t.valok[v] && t.valint[v] > r.rhs;
        case OP_LT: return v >= 0 && t.valok[v] && t.valint[v] < r.rhs;
    }
    return false;
}

KBHIP_HD bool term_match(const DevTables& t, const NodeCols& nc, const Term& tm, int n) {
    bool ok = true;
    for (int i = 0; i < tm.req_n; ++i) ok = ok && req_match(t, nc, t.reqs[tm.req_off + i], n);
    return ok;
}

// The static part of the predicates: selector / node affinity, unschedulable,
// taints.  Does not change while a session runs.
KBHIP_HD bool static_pred_f(const Conf& cf, const TaskClass& c, const DevTables& t, const NodeCols& nc, int n,
                            uint8_t flags) {  // flags = nc.flags[n], loaded by the caller with the row
    if (!cf.pred_on) return true;
    if (c.pred_err) return false;
    if (flags & 1) return false;                                         // predicates.go:107-112
    for (int w = 0; w < nc.taint_words; ++w)                             // helper/helpers.go:425-440
        if (nc.taints[(int64_t)w * nc.npad + n] & ~t.masks[c.tol_off + w]) return false;
    if (c.nsel_term >= 0 && !term_match(t, nc, t.terms[c.nsel_term], n)) return false;  // predicates.go:809-814
    if (c.req_term_n >= 0) {                                             // predicates.go:826-846
        bool any = false;
        for (int i = 0; i < c.req_term_n; ++i) any = any || term_match(t, nc, t.terms[c.req_term_off + i], n);
        if (!any) return false;
    }
    return true;
}
KBHIP_HD bool static_pred(const Conf& cf, const TaskClass& c, const DevTables& t, const NodeCols& nc, int n) {
    return static_pred_f(cf, c, t, nc, n, cf.pred_on ? nc.flags[n] : (uint8_t)0);
}

// Static part of the node-affinity priority: the summed weights of the
// preferred terms the node matches (node_affinity.go:34-74).  Node labels do
// not change in a session, so callers compute it once per node.
KBHIP_HD int32_t na_weight(const TaskClass& c, const DevTables& t, const NodeCols& nc, int n) {
    int32_t na = 0;
    for (int i = 0; i < c.pref_term_n; ++i) {
        const Term& tm = t.terms[c.pref_term_off + i];
        if (term_match(t, nc, tm, n)) na += tm.weight;
    }
    return na;
}

// least_requested.go:44-53: ((cap - req) * 10) / cap for 0 <= req <= cap,
// cap > 0 (a quotient in [0, 10]), given f = the correctly rounded req / cap
// (BRA's fraction, computed anyway): 10 - 10 f is within 1e-14 of the exact
// quotient, so its truncation is off by at most one and the two exact
// integer steps fix it — one IEEE division per resource instead of two.
KBHIP_HD int64_t lr_score_f(int64_t req, int64_t cap, double f) {
    if (cap == 0 || req > cap) return 0;
    const int64_t num = (cap - req) * 10;
    int64_t q = (int64_t)(10.0 - 10.0 * f);
    q = q < 0 ? 0 : (q > 10 ? 10 : q);
    if (q * cap > num) --q;
    if ((q + 1) * cap <= num) ++q;
    return q;
}

// Score of a feasible node (nodeorder.go:281-313): LR and BRA from the row,
// na = na_weight(), ipa = the normalised inter-pod affinity score (0 for
// classes without inter-pod terms).
KBHIP_HD int32_t node_score(const Conf& cf, const TaskClass& c, const Row& r, int32_t na, int32_t ipa) {
    if (!cf.score_mult) return 0;
    const int64_t rc = c.nz_cpu + r.nzc, rm = c.nz_mem + r.nzm;
    // balanced_resource_allocation.go:41-77, IEEE double, no contraction
    const double cpuF = r.acpu == 0 ? 1.0 : (double)rc / (double)r.acpu;
    const double memF = r.amem == 0 ? 1.0 : (double)rm / (double)r.amem;
    const int64_t lr = (lr_score_f(rc, r.acpu, cpuF) + lr_score_f(rm, r.amem, memF)) / 2;
    int64_t bra = 0;
    if (!(cpuF >= 1.0 || memF >= 1.0)) {
        const double d = fabs(cpuF - memF);
        const double one_minus = 1.0 - d;
        bra = (int64_t)(one_minus * 10.0);
    }
    return ((int32_t)lr * cf.w_lr + (int32_t)bra * cf.w_bra + na * cf.w_na + ipa * cf.w_pa) * cf.score_mult;
}

// Dynamic predicates (pod count, host ports) + fit + key, given the row.
// passed: predicate pass and score computed (the node is in the walk).
KBHIP_HD uint64_t dyn_key(const Conf& cf, const TaskClass& c, const DevTables& t,
                                            const NodeCols& nc, const Row& r, const uint64_t* portw,
                                            int n, bool stat_ok, int32_t na, int32_t* score_out, bool* passed,
                                            int32_t ipa = 0) {
    bool ok = stat_ok;
    if (cf.pred_on) {
        if (r.maxtasks <= r.pods) ok = false;                            // predicates.go:127
        if (c.has_ports)                                                 // host_ports.go:96-125
            for (int w = 0; w < 4; ++w) if (w < port_win(c, nc))
                if (portw[w] & t.masks[c.pconf_off + w]) ok = false;
    }
    if (ok && c.score_err) ok = false;  // NodeOrderFn error drops the node (allocate.go:141-145)
    *passed = ok;
    if (!ok) return 0;
    const int32_t s = node_score(cf, c, r, na, ipa);
    *score_out = s;
    // allocate.go:153 (InitResreq <= Idle + Backfilled) and :173 (<= Releasing)
    const bool fit_acc = c.ireq_cpu - (r.idle_cpu + r.bf_cpu) < kMinCPU &&
                         c.ireq_mem - (r.idle_mem + r.bf_mem) < kMinMem &&
                         c.ireq_gpu - (r.idle_gpu + r.bf_gpu) < kMinGPU;
    const bool fit_rel = c.ireq_cpu - r.rel_cpu < kMinCPU && c.ireq_mem - r.rel_mem < kMinMem &&
                         c.ireq_gpu - r.rel_gpu < kMinGPU;
    if (!fit_acc && !fit_rel) return 0;
    return pack_key(s, n + nc.base, fit_acc ? 0 : 1);
}

// NodesFitDelta of a task that found no node (allocate.go:164-167: every node
// of the walk gets Idle.FitDelta(Resreq), resource_info.go:134-147), counted
// the way JobInfo.FitError reads it (job_info.go:343-372): bit 0 = the node is
// in the walk (predicates pass, no NodeOrderFn error), bits 1..3 = its delta
// is negative for cpu / memory / GPU.  The walk visits every such node, so
// Idle is taken after GetAccessibleResource's visit (Idle += Backfilled).
KBHIP_HD uint32_t fit_bits(const TaskClass& c, const Row& r, bool passed) {
    if (!passed) return 0;
    const int64_t ic = r.idle_cpu + r.bf_cpu, im = r.idle_mem + r.bf_mem, ig = r.idle_gpu + r.bf_gpu;
    const int64_t dc = c.req_cpu > 0 ? ic - (c.req_cpu + kMinCPU) : ic;
    const int64_t dm = c.req_mem > 0 ? im - (c.req_mem + kMinMem) : im;
    const int64_t dg = c.req_gpu > 0 ? ig - (c.req_gpu + kMinGPU) : ig;
    return 1u | (dc < 0 ? 2u : 0u) | (dm < 0 ? 4u : 0u) | (dg < 0 ? 8u : 0u);
}

KBHIP_HD uint64_t eval_node(const Conf& cf, const TaskClass& c, const DevTables& t,
                                              const NodeCols& nc, int n, int32_t* score_out, bool* passed,
                                              uint32_t* fit = nullptr) {
    // the flags, row and port words first: their loads do not depend on the
    // predicates' early exits, so they share one memory round trip instead of
    // following each other
    const uint8_t fl = nc.flags[n];
    const Row r = load_row(nc, n);
    uint64_t pw[4] = {0, 0, 0, 0};
    if (c.has_ports)
        for (int w = 0; w < 4; ++w) if (w < port_win(c, nc)) pw[w] = nc.ports[port_at(c, nc, w, n)];
    const bool st = static_pred_f(cf, c, t, nc, n, fl);
    const int32_t na = (st && cf.score_mult) ? na_weight(c, t, nc, n) : 0;
    const uint64_t k = dyn_key(cf, c, t, nc, r, pw, n, st, na, score_out, passed);
    if (fit) *fit = fit_bits(c, r, *passed);
    return k;
}

// The batched sweep of a session with Backfilled nodes (placement 6): a node
// in the walk that cannot fit yet stays a candidate when it carries Backfilled
// resources — each visit of a walk adds them to its Idle (GetAccessibleResource,
// node_info.go:209-211), so it may fit a later task of the pop — keyed by its
// walk position (score, index; kind bit 0).
KBHIP_HD uint64_t eval_node_walk(const Conf& cf, const TaskClass& c, const DevTables& t,
                                 const NodeCols& nc, int n, uint32_t* fit) {
    const Row r = load_row(nc, n);  // before the predicates' early exits (eval_node)
    uint64_t pw[4] = {0, 0, 0, 0};
    if (c.has_ports)
        for (int w = 0; w < 4; ++w) if (w < port_win(c, nc)) pw[w] = nc.ports[port_at(c, nc, w, n)];
    const bool st = static_pred(cf, c, t, nc, n);
    const int32_t na = (st && cf.score_mult) ? na_weight(c, t, nc, n) : 0;
    int32_t s = 0;
    bool passed = false;
    uint64_t k = dyn_key(cf, c, t, nc, r, pw, n, st, na, &s, &passed);
    if (!k && passed && (r.bf_cpu | r.bf_mem | r.bf_gpu)) k = pack_key(s, n + nc.base, 0);
    *fit = fit_bits(c, r, passed);
    return k;
}

// ---------------------------------------------------------------------------
// pod (anti-)affinity (kbhip_affinity.h): count tables per term class,
// indexed by the node's topology domain.
// ---------------------------------------------------------------------------
// Domain columns are replicated over the whole node array (every shard holds
// them): dom_g takes a global node index, dom_of a local row of this shard.
KBHIP_HD int32_t dom_g(const NodeCols& nc, int space, int g) {
    return nc.dom[(int64_t)space * nc.dom_stride + g];
}
KBHIP_HD int32_t dom_of(const NodeCols& nc, int space, int n) { return dom_g(nc, space, n + nc.base); }

// predicates.go:1293-1458 for one node.
KBHIP_HD bool aff_pred(const TaskClass& c, const DevTables& t, const NodeCols& nc, int n) {
    // existing pods' required anti-affinity: a matching target in n's domain
    for (int i = 0; i < c.ea_n; ++i) {
        const int d = dom_of(nc, t.aff_items[c.ea_off + 2 * i], n);
        if (d >= 0 && t.aff_cnt[t.aff_items[c.ea_off + 2 * i + 1] + d] > 0) return false;
    }
    // own required affinity: a target matching every term in n's domain tuple,
    // or no target matches the terms anywhere and the pod matches them itself
    if (c.pa_space >= 0) {
        const int d = dom_of(nc, c.pa_space, n);
        const bool match = d >= 0 && t.aff_cnt[c.pa_cnt + d] > 0;
        if (!match && !(c.pa_self && t.aff_scalar[c.pa_total] == 0)) return false;
    }
    // own required anti-affinity: a target matching every term in n's domain tuple
    if (c.paa_space >= 0) {
        const int d = dom_of(nc, c.paa_space, n);
        if (d >= 0 && t.aff_cnt[c.paa_cnt + d] > 0) return false;
    }
    return true;
}

// Raw inter-pod affinity count of node n (interpod_affinity.go:119-212):
// sum over the task's term classes of weight x pods of the class in n's
// domain; session-placed pods count at the fallback node F's domain.
KBHIP_HD int64_t ipa_count(const TaskClass& c, const DevTables& t, const NodeCols& nc, int n,
                                             int F) {
    int64_t sum = 0;
    for (int i = 0; i < c.ipa_n; ++i) {
        const int32_t* it = t.aff_items + c.ipa_off + 4 * i;
        const int d = dom_of(nc, it[0], n);
        if (d < 0) continue;
        int64_t x = t.aff_cnt[it[1] + d];
        if (F >= 0 && dom_g(nc, it[0], F) == d) x += t.aff_scalar[it[2]];
        sum += (int64_t)it[3] * x;
    }
    return sum;
}

// Full evaluation for the per-task path: static + affinity predicates, the
// inter-pod score normalised by the prepass's [lo, hi] (interpod_affinity.go:228-237).
KBHIP_HD uint64_t eval_node_aff(const Conf& cf, const TaskClass& c, const DevTables& t,
                                                  const NodeCols& nc, int n, int64_t lo, int64_t hi, int F,
                                                  int32_t* score_out, bool* passed, uint32_t* fit = nullptr,
                                                  const int64_t* ipa_pre = nullptr) {
    bool st = static_pred(cf, c, t, nc, n);
    if (st && c.aff && cf.pred_on) st = aff_pred(c, t, nc, n);
    int32_t ipa = 0;
    if (st && c.ipa_n && hi - lo > 0)  // ipa_pre: the raw counts k_ipa_minmax just computed on this state
        ipa = (int32_t)(10.0 * ((double)((ipa_pre ? ipa_pre[n] : ipa_count(c, t, nc, n, F)) - lo) / (double)(hi - lo)));
    const int32_t na = (st && cf.score_mult) ? na_weight(c, t, nc, n) : 0;
    const Row r = load_row(nc, n);
    uint64_t pw[4] = {0, 0, 0, 0};
    if (c.has_ports)
        for (int w = 0; w < 4; ++w) if (w < port_win(c, nc)) pw[w] = nc.ports[port_at(c, nc, w, n)];
    const uint64_t k = dyn_key(cf, c, t, nc, r, pw, n, st, na, score_out, passed, ipa);
    if (fit) *fit = fit_bits(c, r, *passed);
    return k;
}

// Backfill's node test (backfill.go:51-56): the predicates only — no score,
// no fit — keyed so that the max key is the lowest passing index.
KBHIP_HD uint64_t eval_first_fit(const Conf& cf, const TaskClass& c, const DevTables& t,
                                                   const NodeCols& nc, int n) {
    bool ok = static_pred(cf, c, t, nc, n);
    if (ok && cf.pred_on) {
        if (c.aff) ok = aff_pred(c, t, nc, n);
        if (nc.maxtasks[n] <= nc.pods[n]) ok = false;                    // predicates.go:127
        if (c.has_ports)                                                 // host_ports.go:96-125
            for (int w = 0; w < 4; ++w) if (w < port_win(c, nc))
                if (nc.ports[port_at(c, nc, w, n)] & t.masks[c.pconf_off + w]) ok = false;
    }
    return ok ? pack_key(0, n + nc.base, 0) : 0;
}

// Count-table updates of a committed task (kind 1 Allocated, 2 Pipelined) on
// global node g (every shard applies them).
//   UPD_CNT_ALLOC (0):    Allocated only: a new predicate target in g's domain
//   UPD_SCALAR_ALLOC (1): Allocated only: target total of a PA class
//   UPD_SCALAR_ANY (2):   any commit: a session-placed pod (inter-pod priority)
// Written branch-free on purpose: the if / else-if / else form (one increment
// per branch, two tables) is miscompiled by the ROCm 7.2 gfx950 backend when
// it runs in a single lane — the UPD_SCALAR_ANY branch reused a stale table
// pointer register ("toolchain note").  A node without the
// space's key (domain -1) adds 0 at the table's first entry: the index stays
// inside the table (u[2] + -1 was one word before it — outside the buffer for
// the first table, a fault at full-size C3 with keyless nodes).
KBHIP_HD void commit_aff(const TaskClass& c, const DevTables& t, const NodeCols& nc, int g, int kind) {
    for (int i = 0; i < c.upd_n; ++i) {
        const int32_t* u = t.aff_items + c.upd_off + 3 * i;
        const int typ = u[0];
        const bool to_cnt = typ == 0;
        const int d = to_cnt ? dom_g(nc, u[1], g) : 0;
        const bool apply = (typ == 2 || kind == 1) && d >= 0;
        int32_t* tab = to_cnt ? t.aff_cnt : t.aff_scalar;
        tab[u[2] + (d < 0 ? 0 : d)] += apply ? 1 : 0;  // (a keyless node: +0 at the table's first entry)
    }
}

// Exact inverse of commit_aff (a retracted prediction, or the undo around a
// FitDelta recomputation); same branch-free form.
KBHIP_HD void uncommit_aff(const TaskClass& c, const DevTables& t, const NodeCols& nc, int g, int kind) {
    for (int i = 0; i < c.upd_n; ++i) {
        const int32_t* u = t.aff_items + c.upd_off + 3 * i;
        const int typ = u[0];
        const bool to_cnt = typ == 0;
        const int d = to_cnt ? dom_g(nc, u[1], g) : 0;
        const bool apply = (typ == 2 || kind == 1) && d >= 0;
        int32_t* tab = to_cnt ? t.aff_cnt : t.aff_scalar;
        tab[u[2] + (d < 0 ? 0 : d)] -= apply ? 1 : 0;
    }
}

// Pod-affinity classes the batched pop places (placement 7): predicate terms
// that only ever turn nodes infeasible as pods are placed — existing pods'
// required anti-affinity (EA) and own required anti-affinity (PAA) — with no
// own required affinity (PA: placements make nodes feasible) and no inter-pod
// priority terms (their normalisation moves every node's score).  Lanes keep
// the count-table entries their node's predicate reads in registers.
constexpr int kAffItems = 4;  // EA pairs + PAA the placement tracks per candidate
constexpr int kAffUpd = 8;    // commit updates of the class
KBHIP_HD bool aff_batchable(const TaskClass& c) {
    return c.aff && !c.pred_err && c.pa_space < 0 && c.ipa_n == 0 &&
           c.ea_n + (c.paa_space >= 0 ? 1 : 0) <= kAffItems && c.upd_n <= kAffUpd;
}

// NodeInfo.AddTask for the winner (node_info.go:113-145) + the k8s NodeInfo
// aggregates the predicates/nodeorder read (k8s cache/node_info.go:498-521).
KBHIP_HD void commit_node(const TaskClass& c, const DevTables& t, const NodeCols& nc, int n, int kind) {
    if (c.backfill) { nc.bf_cpu[n] += c.req_cpu; nc.bf_mem[n] += c.req_mem; nc.bf_gpu[n] += c.req_gpu; }
    if (kind == 1) { nc.idle_cpu[n] -= c.req_cpu; nc.idle_mem[n] -= c.req_mem; nc.idle_gpu[n] -= c.req_gpu; }
    else { nc.rel_cpu[n] -= c.req_cpu; nc.rel_mem[n] -= c.req_mem; nc.rel_gpu[n] -= c.req_gpu; }
    nc.pods[n] += 1;
    nc.nzc[n] += c.nz_cpu;
    nc.nzm[n] += c.nz_mem;
    if (c.has_ports)
        for (int w = 0; w < 4; ++w) if (w < port_win(c, nc)) nc.ports[port_at(c, nc, w, n)] |= t.masks[c.pown_off + w];
}

// Exact inverse of commit_node for a batched-path class (integer updates; the
// class's own host-port bits cannot have been set before its commit, since
// they conflict with themselves).  Used to retract a mispredicted pop.
KBHIP_HD void uncommit_node(const TaskClass& c, const DevTables& t, const NodeCols& nc, int n, int kind) {
    if (c.backfill) { nc.bf_cpu[n] -= c.req_cpu; nc.bf_mem[n] -= c.req_mem; nc.bf_gpu[n] -= c.req_gpu; }
    if (kind == 1) { nc.idle_cpu[n] += c.req_cpu; nc.idle_mem[n] += c.req_mem; nc.idle_gpu[n] += c.req_gpu; }
    else { nc.rel_cpu[n] += c.req_cpu; nc.rel_mem[n] += c.req_mem; nc.rel_gpu[n] += c.req_gpu; }
    nc.pods[n] -= 1;
    nc.nzc[n] -= c.nz_cpu;
    nc.nzm[n] -= c.nz_mem;
    if (c.has_ports)
        for (int w = 0; w < 4; ++w) if (w < port_win(c, nc)) nc.ports[port_at(c, nc, w, n)] &= ~t.masks[c.pown_off + w];
}

// Gang bookkeeping after an assignment: allocate.go:191-195 + gang.go:63-66.
KBHIP_HD void after_assign(PopCtrl* ctrl, int i, int kind) {
    if (kind == 1) ctrl->ready_count += 1;  // Pipelined is not an AllocatedStatus (types.go:82-84)
    ctrl->n_done = i + 1;
    if (!ctrl->gang_mode || ctrl->ready_count >= ctrl->min_avail) ctrl->stop = 2;
    else if (i + 1 == ctrl->n_tasks) ctrl->stop = 0;
}


}  // namespace kbhip
