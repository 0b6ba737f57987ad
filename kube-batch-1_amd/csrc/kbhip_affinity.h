// kbhip_affinity.h — pod (anti-)affinity as per-topology-domain count tables.
//
// The reference evaluates pod affinity per (task, node) by listing every
// allocated pod (predicates.go:1293-1458) and inter-pod-affinity priority by
// scanning every pod on every node (interpod_affinity.go:119-240).  Both only
// ever ask "how many pods of a given term class sit in the topology domain of
// node n", so the engine keeps one count table per term class, indexed by the
// node's domain (a dense id over the values — or value tuples — of the term's
// topology key(s)), and updates the tables when a task is committed.
//
// Term classes (identity = resolved namespaces + selector + key(s) [+ weight]):
//   EA   required anti-affinity terms of pods that are or can become targets
//        (satisfiesExistingPodsAntiAffinity, predicates.go:1293-1334)
//   PA   a pending task's own required affinity terms as one conjunction
//        (satisfiesPodsAffinityAntiAffinity, :1402-1458) + a target total for
//        the "no pod matches the terms' properties yet" rule
//   PAA  a pending task's own required anti-affinity terms (conjunction)
//   Q    a pending task's preferred (anti-)affinity terms (IPA, :137-152)
//   R    existing pods' required affinity / preferred (anti-)affinity terms
//        matched by the task (IPA, :154-181)
// Predicate targets are AllocatedStatuses tasks of session jobs at their
// task.NodeName; IPA pods are every pod on a node, at the node named by the
// raw Spec.NodeName — for pods placed in this session that name is "" and the
// reference falls back to the lowest-index node holding such a pod
// (nodeorder.go:78-93), so their contributions are kept
// in per-class session counters applied at that node's domain.
#pragma once
#include <map>
#include <string>
#include <vector>

#include <stdint.h>

#include "../../include/kbsnap.h"

namespace kbhip {

// Commit update item types.
enum : int32_t { UPD_CNT_ALLOC = 0, UPD_SCALAR_ALLOC = 1, UPD_SCALAR_ANY = 2 };

// A task's compiled affinity program (item lists; offsets are absolute in the
// model's count / scalar tables).
struct AffProgram {
    std::vector<int32_t> ea;   // (space, cnt_off) pairs: fail if cnt[off + dom(n)] > 0
    int32_t pa_space = -1, pa_cnt = -1, pa_total = -1, pa_self = 0;
    int32_t paa_space = -1, paa_cnt = -1;
    std::vector<int32_t> ipa;  // (space, cnt_off, sess_idx, weight) quads
    std::vector<int32_t> upd;  // (type, space, off) triples applied on commit
    int32_t pred_err = 0;      // the task's own required term has an invalid selector
    bool empty() const {
        return ea.empty() && pa_space < 0 && paa_space < 0 && ipa.empty() && upd.empty() && !pred_err;
    }
};

struct AffPod {  // what the model needs to know about each pod
    int ns = -1;              // namespace id (index into ns_names)
    int status = 0;           // St code of session/session.h
    bool session_job = false; // belongs to a job of the session
    bool target = false;      // AllocatedStatuses task of a session job, on a node
    bool pending = false;     // pending task of a session job (gets a program)
    int node = -1;            // node index when on a node (node.Pods()), else -1
};

// Canonical affinity rows: rows whose raw contents (flags, node-affinity terms,
// pod (anti-)affinity terms with their selectors, namespaces and topology keys,
// as string-table offsets) are equal get one id, the index of the first such
// row — the snapshot's string table is interned (kbsnap.h), so equal offsets
// are equal strings.  The pods of one gang carry equal rows.
std::vector<int> canon_aff_rows(const kbs::Snapshot& s);

class AffinityModel {
  public:
    bool active = false;         // some pod carries pod (anti-)affinity terms
    int n_spaces = 0;
    std::vector<int32_t> dom;    // [n_spaces][npad] node domain ids (-1: a key is missing)
    std::vector<int32_t> cnt;    // all count tables
    std::vector<int32_t> scalar; // PA totals and session counters

    // Builds classes, tables, initial counts and the pending tasks' programs.
    // Throws std::invalid_argument for inputs outside the supported domain.
    // row_canon: canon_aff_rows(s) (pods whose rows have one id share their terms).
    void build(const kbs::Snapshot& s, int n_nodes, int npad, const std::vector<AffPod>& pods,
               const std::vector<std::string>& ns_names, bool pred_on, bool ipa_on,
               const std::vector<int>& row_canon);
    const AffProgram* program(int pod) const {
        const int k = pod >= 0 && pod < (int)prog_of_.size() ? prog_of_[pod] : -1;
        return k < 0 ? nullptr : &progs_[k];
    }
    // Programs of two pods are the same object (a sufficient test of equality).
    int program_id(int pod) const { return pod >= 0 && pod < (int)prog_of_.size() ? prog_of_[pod] : -1; }
    // Counts of every table for the given pod states (same term classes and
    // programs as built: the pods' statuses / nodes may have changed, e.g. a
    // session carried over or victims evicted).  build() uses it for the
    // initial counts.
    void recount(const std::vector<AffPod>& pods);
    // What pod i contributes while it is a predicate target (an
    // AllocatedStatuses task of a session job on a node): (type, space, off)
    // triples as in AffProgram::upd (UPD_CNT_ALLOC / UPD_SCALAR_ALLOC).  An
    // eviction (Running -> Releasing) withdraws them, an unevict restores them.
    void target_updates(int pod, std::vector<int32_t>& out) const;
    int npad() const { return npad_; }

  private:
    std::vector<AffProgram> progs_;  // distinct programs
    std::vector<int> prog_of_;       // per pod: index into progs_ (-1: none)
    struct CInfo {
        int kind, space, cnt_off, scal;
    };
    std::vector<CInfo> cls_;                          // term classes
    std::vector<int> pod_group_;                      // label group of each pod
    std::vector<std::vector<int>> own_ea_, own_r_;    // per pod: its own EA / R term classes
    std::vector<std::vector<int>> g_tgt_, g_q_;       // per label group: PA / PAA, Q classes it matches
    int npad_ = 0;
};

}  // namespace kbhip
