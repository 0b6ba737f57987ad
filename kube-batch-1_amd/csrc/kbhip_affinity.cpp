// kbhip_affinity.cpp — builds the pod (anti-)affinity count tables and the
// pending tasks' affinity programs (see kbhip_affinity.h for the model).
//
// Reference semantics followed (vendored k8s v1.13 under /root/reference/vendor):
//   selectors     metav1.LabelSelectorAsSelector (nil -> nothing, empty -> everything),
//                 labels.Requirement.Matches (apimachinery/pkg/labels/selector.go:192-236)
//   namespaces    priorityutil.GetNamespacesFromPodAffinityTerm (empty -> the defining pod's)
//   predicate     predicates.go:1293-1334 (existing pods' anti-affinity), 1402-1458 (the
//                 pod's own terms, all terms of a kind as one conjunction, metadata.go:498-509
//                 for the first pod of a self-affine series), targets = AllocatedStatuses
//                 tasks of session jobs (plugins/predicates/predicates.go:59-94)
//   priority      interpod_affinity.go:119-240, hardPodAffinityWeight = 1, existing pods
//                 resolved through nodeorder.go:78-93 (fallback node for NodeName "")
#include "kbhip_affinity.h"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <unordered_map>

namespace kbhip {

using std::string;
using std::vector;

namespace {

struct SDict {
    std::unordered_map<string, int> ids;
    vector<string> strs;
    int get(const string& s) {
        auto it = ids.find(s);
        if (it != ids.end()) return it->second;
        ids.emplace(s, (int)strs.size());
        strs.push_back(s);
        return (int)strs.size() - 1;
    }
};

// Dictionary lookups by string-table offset: the same offset is the same
// string, so each distinct offset is hashed as a string once.
struct ODict {
    SDict& d;
    const kbs::Snapshot& s;
    std::unordered_map<int32_t, int> by_off;
    int get(int32_t off) {
        auto it = by_off.find(off);
        if (it != by_off.end()) return it->second;
        const int id = d.get(s.s(off));
        by_off.emplace(off, id);
        return id;
    }
};

typedef vector<std::pair<int, int>> LSet;  // sorted (key id, value id)
static int lget(const LSet& l, int key) {
    auto it = std::lower_bound(l.begin(), l.end(), std::make_pair(key, -1));
    return (it != l.end() && it->first == key) ? it->second : -1;
}

enum { L_IN = 0, L_NOTIN = 1, L_EXISTS = 2, L_DNE = 3 };
struct LReq {
    int key, op;
    vector<int> vals;  // sorted value ids
};
struct LSel {
    bool nothing = false, err = false;
    vector<LReq> reqs;
    string canon;
};
static bool sel_match(const LSel& s, const LSet& ls) {
    if (s.nothing || s.err) return false;
    for (const LReq& r : s.reqs) {
        const int v = lget(ls, r.key);
        const bool hit = v >= 0 && std::binary_search(r.vals.begin(), r.vals.end(), v);
        switch (r.op) {
            case L_IN: if (!hit) return false; break;
            case L_NOTIN: if (hit) return false; break;
            case L_EXISTS: if (v < 0) return false; break;
            case L_DNE: if (v >= 0) return false; break;
            default: return false;
        }
    }
    return true;
}

struct PTerm {           // a PodAffinityTerm as written in the pod spec
    int sel = -1;        // index into the parsed selectors
    vector<int> ns;      // namespace ids; empty = the defining pod's namespace
    string key;          // topology key
};
struct ARow {
    bool pa = false, paa = false;
    vector<PTerm> pa_req, paa_req;
    vector<std::pair<int32_t, PTerm>> pa_pref, paa_pref;
    bool any() const { return !pa_req.empty() || !paa_req.empty() || !pa_pref.empty() || !paa_pref.empty(); }
};

enum Kind { K_EA = 0, K_PA, K_PAA, K_Q, K_R };
struct Prop {
    vector<int> ns;  // resolved, sorted
    int sel;
};
struct TClass {
    int kind;
    vector<Prop> props;  // conjunction
    int space;
    int cnt_off = 0;
    int scal = -1;       // PA: target total; Q/R: session counter
    int weight = 0;      // R
};

}  // namespace

vector<int> canon_aff_rows(const kbs::Snapshot& s) {
    auto V32 = [&](const char* n) { return s.vec<int32_t>(n); };
    auto a_flags = s.vec<uint8_t>("a_flags");
    const size_t A = a_flags.size();
    vector<int> out(A, -1);
    if (A == 0) return out;
    auto cnt_of = [&](const char* n) {
        auto v = V32(n);
        if (v.size() != A) v.assign(A, 0);
        return v;
    };
    const auto nareq_s = cnt_of("a_nareq_start"), nareq_c = cnt_of("a_nareq_cnt"),
               napref_s = cnt_of("a_napref_start"), napref_c = cnt_of("a_napref_cnt"),
               pareq_s = cnt_of("a_pareq_start"), pareq_c = cnt_of("a_pareq_cnt"),
               papref_s = cnt_of("a_papref_start"), papref_c = cnt_of("a_papref_cnt"),
               paareq_s = cnt_of("a_paareq_start"), paareq_c = cnt_of("a_paareq_cnt"),
               paapref_s = cnt_of("a_paapref_start"), paapref_c = cnt_of("a_paapref_cnt");
    const auto es = V32("nst_expr_start"), ec = V32("nst_expr_cnt"), fs = V32("nst_field_start"),
               fc = V32("nst_field_cnt"), nsr_key = V32("nsr_key"), nsrv = V32("nsrv"), pst_w = V32("pst_weight"),
               pst_t = V32("pst_term");
    const auto nsr_op = s.vec<uint8_t>("nsr_op");
    const auto nsr_voff = s.offs("nsr_val_off", nsr_key.size());
    const auto pat_sel = V32("pat_sel"), pat_topo = V32("pat_topo"), patns = V32("patns");
    const auto pat_ns = s.offs("pat_ns_off", pat_sel.size());
    const auto ls_ml = V32("ls_ml_off"), ls_me = V32("ls_me_off"), lkv_k = V32("lkv_key"), lkv_v = V32("lkv_val");
    const auto lsr_key = V32("lsr_key"), lsrv = V32("lsrv");
    const auto lsr_op = s.vec<uint8_t>("lsr_op");
    const auto lsr_voff = s.offs("lsr_val_off", lsr_key.size());
    const auto wpat_w = V32("wpat_weight"), wpat_t = V32("wpat_term");
    vector<int32_t> sig, prev;
    auto at = [](const vector<int32_t>& v, int64_t i) -> int32_t {
        if (i < 0 || i >= (int64_t)v.size()) throw std::invalid_argument("affinity row reference out of range");
        return v[i];
    };
    auto nsr_row = [&](int k) {  // one NodeSelectorRequirement
        sig.push_back(at(nsr_key, k));
        sig.push_back(k < (int)nsr_op.size() ? nsr_op[k] : -1);
        sig.push_back(nsr_voff[k + 1] - nsr_voff[k]);
        for (int q = nsr_voff[k]; q < nsr_voff[k + 1]; ++q) sig.push_back(at(nsrv, q));
    };
    auto nst = [&](int row) {  // one NodeSelectorTerm
        sig.push_back(at(ec, row));
        for (int k = at(es, row); k < es[row] + ec[row]; ++k) nsr_row(k);
        sig.push_back(at(fc, row));
        for (int k = at(fs, row); k < fs[row] + fc[row]; ++k) nsr_row(k);
    };
    auto pat = [&](int row) {  // one PodAffinityTerm
        const int sr = at(pat_sel, row);
        sig.push_back(sr < 0 ? -1 : 1);
        if (sr >= 0) {
            for (int k = at(ls_ml, sr); k < at(ls_ml, sr + 1); ++k) { sig.push_back(at(lkv_k, k)); sig.push_back(at(lkv_v, k)); }
            sig.push_back(-2);
            for (int k = at(ls_me, sr); k < at(ls_me, sr + 1); ++k) {
                sig.push_back(at(lsr_key, k));
                sig.push_back(k < (int)lsr_op.size() ? lsr_op[k] : -1);
                sig.push_back(lsr_voff[k + 1] - lsr_voff[k]);
                for (int q = lsr_voff[k]; q < lsr_voff[k + 1]; ++q) sig.push_back(at(lsrv, q));
            }
        }
        sig.push_back(pat_ns[row + 1] - pat_ns[row]);
        for (int k = pat_ns[row]; k < pat_ns[row + 1]; ++k) sig.push_back(at(patns, k));
        sig.push_back(at(pat_topo, row));
    };
    std::unordered_map<string, int> ids;
    ids.reserve(A);
    for (size_t a = 0; a < A; ++a) {
        sig.clear();
        sig.push_back(a_flags[a]);
        sig.push_back(nareq_c[a]);
        for (int k = nareq_s[a]; k < nareq_s[a] + nareq_c[a]; ++k) nst(k);
        sig.push_back(napref_c[a]);
        for (int k = napref_s[a]; k < napref_s[a] + napref_c[a]; ++k) { sig.push_back(at(pst_w, k)); nst(at(pst_t, k)); }
        for (auto* r : {&pareq_s, &paareq_s}) {
            const auto& cnt = r == &pareq_s ? pareq_c : paareq_c;
            sig.push_back(cnt[a]);
            for (int k = (*r)[a]; k < (*r)[a] + cnt[a]; ++k) pat(k);
        }
        for (auto* r : {&papref_s, &paapref_s}) {
            const auto& cnt = r == &papref_s ? papref_c : paapref_c;
            sig.push_back(cnt[a]);
            for (int k = (*r)[a]; k < (*r)[a] + cnt[a]; ++k) { sig.push_back(at(wpat_w, k)); pat(at(wpat_t, k)); }
        }
        if (a > 0 && sig == prev) {  // the previous row's content (consecutive pods of a gang)
            out[a] = out[a - 1];
            continue;
        }
        string key((const char*)sig.data(), sig.size() * sizeof(int32_t));
        out[a] = ids.emplace(std::move(key), (int)a).first->second;  // id = the first row with this content
        prev.swap(sig);
    }
    return out;
}

void AffinityModel::build(const kbs::Snapshot& s, int N, int npad, const vector<AffPod>& pods,
                          const vector<string>& ns_names, bool pred_on, bool ipa_on, const vector<int>& canon) {
    auto V32 = [&](const char* n) { return s.vec<int32_t>(n); };
    const int P = (int)pods.size();
    auto paff = V32("p_aff");
    auto a_flags = s.vec<uint8_t>("a_flags");
    const size_t A = a_flags.size();
    auto cnt_of = [&](const char* n) {
        auto v = V32(n);
        if (v.size() != A) v.assign(A, 0);
        return v;
    };
    auto pareq_s = cnt_of("a_pareq_start"), pareq_c = cnt_of("a_pareq_cnt"), papref_s = cnt_of("a_papref_start"),
         papref_c = cnt_of("a_papref_cnt"), paareq_s = cnt_of("a_paareq_start"), paareq_c = cnt_of("a_paareq_cnt"),
         paapref_s = cnt_of("a_paapref_start"), paapref_c = cnt_of("a_paapref_cnt");
    bool any_terms = false;
    for (size_t a = 0; a < A; ++a)
        if (pareq_c[a] + papref_c[a] + paareq_c[a] + paapref_c[a] > 0) any_terms = true;
    bool used = false;
    if (any_terms)
        for (int i = 0; i < P && !used; ++i) {
            const int a = paff.empty() ? -1 : paff[i];
            if (a >= 0 && (size_t)a < A && pareq_c[a] + papref_c[a] + paareq_c[a] + paapref_c[a] > 0) used = true;
        }
    active = used && (pred_on || ipa_on);
    if (!active) return;

    static const bool prof = std::getenv("KBHIP_OPEN_PROFILE") != nullptr;
    auto tp = std::chrono::steady_clock::now();
    auto mark = [&](const char* what) {
        if (!prof) return;
        auto t = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[aff]  %-12s %6.2f ms\n", what, std::chrono::duration<double, std::milli>(t - tp).count());
        tp = t;
    };
    // ---------------- dictionaries, selectors, affinity rows ----------------
    SDict keys, vals, nss;
    for (auto& n : ns_names) nss.get(n);
    ODict okeys{keys, s, {}}, ovals{vals, s, {}}, onss{nss, s, {}};
    auto pat_sel = V32("pat_sel"), pat_topo = V32("pat_topo"), patns = V32("patns");
    auto pat_ns = s.offs("pat_ns_off", pat_sel.size());
    auto ls_ml = V32("ls_ml_off"), ls_me = V32("ls_me_off"), lkv_k = V32("lkv_key"), lkv_v = V32("lkv_val");
    auto lsr_key = V32("lsr_key");
    auto lsr_op = s.vec<uint8_t>("lsr_op");
    auto lsr_voff = s.offs("lsr_val_off", lsr_key.size());
    auto lsrv = V32("lsrv");
    auto wpat_w = V32("wpat_weight"), wpat_t = V32("wpat_term");
    vector<LSel> sels;
    std::map<int, int> sel_of_row;  // lsel row -> parsed selector (-1 row: nil)
    std::unordered_map<string, int> sel_of_canon;  // equal selectors share one index
    auto parse_sel = [&](int sr) -> int {
        auto it = sel_of_row.find(sr);
        if (it != sel_of_row.end()) return it->second;
        LSel L;
        if (sr < 0) {
            L.nothing = true;  // nil LabelSelector -> labels.Nothing()
            L.canon = "N";
        } else {
            if (sr + 1 >= (int)ls_ml.size() || sr + 1 >= (int)ls_me.size())
                throw std::invalid_argument("label selector row out of range");
            // MatchLabels -> Equals requirements; MatchExpressions In/NotIn/Exists/DoesNotExist
            // (metav1.LabelSelectorAsSelector); an invalid requirement errors the selector.
            for (int k = ls_ml[sr]; k < ls_ml[sr + 1]; ++k)
                L.reqs.push_back(LReq{okeys.get(lkv_k[k]), L_IN, {ovals.get(lkv_v[k])}});
            for (int k = ls_me[sr]; k < ls_me[sr + 1]; ++k) {
                LReq r{okeys.get(lsr_key[k]), (int)lsr_op[k], {}};
                for (int q = lsr_voff[k]; q < lsr_voff[k + 1]; ++q) r.vals.push_back(ovals.get(lsrv[q]));
                const bool nv = r.vals.empty();
                if (r.op == L_IN || r.op == L_NOTIN) { if (nv) L.err = true; }
                else if (r.op == L_EXISTS || r.op == L_DNE) { if (!nv) L.err = true; }
                else L.err = true;  // Gt/Lt are not LabelSelectorOperators
                L.reqs.push_back(std::move(r));
            }
            for (auto& r : L.reqs) {
                std::sort(r.vals.begin(), r.vals.end());
                r.vals.erase(std::unique(r.vals.begin(), r.vals.end()), r.vals.end());
            }
            vector<string> parts;
            for (auto& r : L.reqs) {
                string p = std::to_string(r.key) + ":" + std::to_string(r.op) + ":";
                for (int v : r.vals) p += std::to_string(v) + ",";
                parts.push_back(p);
            }
            std::sort(parts.begin(), parts.end());
            L.canon = L.err ? "X" + std::to_string(sr) : "S";
            for (auto& p : parts) L.canon += p + ";";
        }
        auto ci = sel_of_canon.find(L.canon);
        if (ci != sel_of_canon.end()) {
            sel_of_row[sr] = ci->second;
            return ci->second;
        }
        sels.push_back(std::move(L));
        sel_of_canon.emplace(sels.back().canon, (int)sels.size() - 1);
        sel_of_row[sr] = (int)sels.size() - 1;
        return (int)sels.size() - 1;
    };
    auto pterm = [&](int row) {
        if (row < 0 || row >= (int)pat_sel.size()) throw std::invalid_argument("pod affinity term row out of range");
        PTerm t;
        t.sel = parse_sel(pat_sel[row]);
        for (int k = pat_ns[row]; k < pat_ns[row + 1]; ++k) t.ns.push_back(onss.get(patns[k]));
        t.key = s.s(pat_topo[row]);
        return t;
    };
    if (canon.size() != A) throw std::invalid_argument("affinity row ids do not match the rows");
    vector<ARow> rows(A);
    for (size_t a = 0; a < A; ++a) {
        if (canon[a] != (int)a) continue;  // parsed once per content (rows[canon[a]])
        ARow& r = rows[a];
        r.pa = a_flags[a] & KBS_AFF_PA;
        r.paa = a_flags[a] & KBS_AFF_PAA;
        for (int k = pareq_s[a]; k < pareq_s[a] + pareq_c[a]; ++k) r.pa_req.push_back(pterm(k));
        for (int k = paareq_s[a]; k < paareq_s[a] + paareq_c[a]; ++k) r.paa_req.push_back(pterm(k));
        for (int k = papref_s[a]; k < papref_s[a] + papref_c[a]; ++k) r.pa_pref.push_back({wpat_w[k], pterm(wpat_t[k])});
        for (int k = paapref_s[a]; k < paapref_s[a] + paapref_c[a]; ++k)
            r.paa_pref.push_back({wpat_w[k], pterm(wpat_t[k])});
    }
    auto row_of = [&](int i) -> const ARow* {
        const int a = paff.empty() ? -1 : paff[i];
        return (a >= 0 && (size_t)a < A && rows[canon[a]].any()) ? &rows[canon[a]] : nullptr;
    };

    // keys any selector reads (pod labels) / any term's topology key (node labels):
    // labels under other keys never matter here and are not encoded
    vector<char> sel_key(keys.strs.size(), 0);
    for (auto& L : sels)
        for (auto& r : L.reqs) sel_key[r.key] = 1;
    std::unordered_map<string, int> topo_keys;
    for (auto& r : rows) {
        for (auto* v : {&r.pa_req, &r.paa_req})
            for (auto& t : *v) topo_keys.emplace(t.key, 0);
        for (auto* v : {&r.pa_pref, &r.paa_pref})
            for (auto& wt : *v) topo_keys.emplace(wt.second.key, 0);
    }
    for (auto& kv : topo_keys) kv.second = keys.get(kv.first);
    vector<char> topo_key(keys.strs.size(), 0);
    for (auto& kv : topo_keys) topo_key[kv.second] = 1;
    mark("rows");
    // ---------------- pod label groups (namespace + labels) ----------------
    auto plo = s.offs("p_label_off", P);
    auto plk = V32("pl_key"), plv = V32("pl_val");
    vector<int> group(P);
    vector<LSet> g_labels;
    vector<int> g_ns;
    {
        std::map<std::pair<int, LSet>, int> gid;
        for (int i = 0; i < P; ++i) {
            if (i > 0 && pods[i].ns == pods[i - 1].ns && plo[i + 1] - plo[i] == plo[i] - plo[i - 1]) {
                bool same = true;  // the previous pod's labels, offset for offset (a gang's pods)
                for (int k = 0; k < plo[i + 1] - plo[i] && same; ++k)
                    same = plk[plo[i] + k] == plk[plo[i - 1] + k] && plv[plo[i] + k] == plv[plo[i - 1] + k];
                if (same) { group[i] = group[i - 1]; continue; }
            }
            LSet l;
            for (int k = plo[i]; k < plo[i + 1]; ++k) {
                const int key = okeys.get(plk[k]);
                if (key < (int)sel_key.size() && sel_key[key]) l.push_back({key, ovals.get(plv[k])});
            }
            std::sort(l.begin(), l.end());
            auto key = std::make_pair(pods[i].ns, l);
            auto it = gid.find(key);
            if (it == gid.end()) {
                it = gid.emplace(key, (int)g_labels.size()).first;
                g_labels.push_back(std::move(l));
                g_ns.push_back(pods[i].ns);
            }
            group[i] = it->second;
        }
    }

    mark("groups");
    // ---------------- topology spaces ----------------
    auto nlo = s.offs("n_label_off", N);
    auto nlk = V32("nl_key"), nlv = V32("nl_val");
    vector<LSet> n_labels(N);
    for (int n = 0; n < N; ++n) {
        for (int k = nlo[n]; k < nlo[n + 1]; ++k) {
            const int key = okeys.get(nlk[k]);
            if (key < (int)topo_key.size() && topo_key[key]) n_labels[n].push_back({key, ovals.get(nlv[k])});
        }
        std::sort(n_labels[n].begin(), n_labels[n].end());
    }
    std::map<vector<string>, int> space_ids;
    vector<int> space_size;
    auto space_of = [&](const vector<string>& ks) -> int {
        auto it = space_ids.find(ks);
        if (it != space_ids.end()) return it->second;
        const int sp = (int)space_size.size();
        space_ids.emplace(ks, sp);
        dom.resize((size_t)(sp + 1) * npad, -1);
        vector<int> kid;
        for (auto& k : ks) kid.push_back(keys.get(k));
        std::map<vector<int>, int> tuples;
        for (int n = 0; n < N; ++n) {
            vector<int> tup;
            bool ok = true;
            for (int k : kid) {
                const int v = lget(n_labels[n], k);
                if (v < 0) { ok = false; break; }
                tup.push_back(v);
            }
            if (!ok) continue;
            auto t = tuples.emplace(tup, (int)tuples.size()).first;
            dom[(size_t)sp * npad + n] = t->second;
        }
        space_size.push_back((int)tuples.size());
        return sp;
    };

    mark("node labels");
    // ---------------- term classes ----------------
    vector<TClass> classes;
    std::map<string, int> class_ids;
    auto resolve = [&](const PTerm& t, int definer) {
        Prop p;
        p.ns = t.ns.empty() ? vector<int>{pods[definer].ns} : t.ns;
        std::sort(p.ns.begin(), p.ns.end());
        p.ns.erase(std::unique(p.ns.begin(), p.ns.end()), p.ns.end());
        p.sel = t.sel;
        return p;
    };
    auto class_of = [&](int kind, const vector<Prop>& props, const vector<string>& ks, int weight) {
        string sig = std::to_string(kind) + "|" + std::to_string(weight) + "|";
        for (auto& p : props) {
            for (int x : p.ns) sig += std::to_string(x) + ",";
            sig += "/" + std::to_string(p.sel) + "|";  // selectors are deduplicated by canonical form
        }
        for (auto& k : ks) { sig += k; sig.push_back('\0'); }
        auto it = class_ids.find(sig);
        if (it != class_ids.end()) return it->second;
        TClass c;
        c.kind = kind;
        c.props = props;
        c.space = space_of(ks);
        c.weight = weight;
        classes.push_back(std::move(c));
        class_ids.emplace(sig, (int)classes.size() - 1);
        return (int)classes.size() - 1;
    };
    auto bad_sel = [&](const PTerm& t) { return sels[t.sel].err; };

    vector<vector<int>> own_ea(P), own_r(P);
    vector<int> own_pa(P, -1), own_paa(P, -1);
    vector<vector<std::pair<int, int>>> own_q(P);  // (class, weight)
    vector<char> own_pred_err(P, 0);
    // the term classes of a pod follow from its row's content, its namespace
    // (the default of a term's namespaces) and three flags: computed once per
    // combination, then copied
    std::unordered_map<uint64_t, int> tc_memo;  // (canonical row, ns, flags) -> first pod
    uint64_t last_mk = ~0ull;
    int last_j = -1;
    for (int i = 0; i < P; ++i) {
        const ARow* r = row_of(i);
        if (!r) continue;
        const AffPod& p = pods[i];
        const bool can_target = p.session_job && (p.target || p.pending);
        const uint64_t mk = ((uint64_t)(uint32_t)canon[paff[i]] << 32) | ((uint64_t)(uint32_t)p.ns << 3) |
                            (can_target ? 4u : 0u) | (p.pending ? 2u : 0u) | (p.node >= 0 ? 1u : 0u);
        if (p.ns < (1 << 28)) {
            int j = -1;
            if (mk == last_mk) j = last_j;  // the previous pod with a row (a gang's pods)
            else if (auto mi = tc_memo.find(mk); mi != tc_memo.end()) j = mi->second;
            if (j >= 0) {
                last_mk = mk;
                last_j = j;
                own_ea[i] = own_ea[j]; own_r[i] = own_r[j]; own_q[i] = own_q[j];
                own_pa[i] = own_pa[j]; own_paa[i] = own_paa[j]; own_pred_err[i] = own_pred_err[j];
                continue;
            }
            tc_memo.emplace(mk, i);
            last_mk = mk;
            last_j = i;
        }
        if (pred_on && can_target && r->paa) {
            for (auto& t : r->paa_req) {
                if (bad_sel(t)) throw std::invalid_argument("invalid label selector in a required anti-affinity term");
                if (t.key.empty()) continue;  // node.Labels[""] is never set: adds nothing
                own_ea[i].push_back(class_of(K_EA, {resolve(t, i)}, {t.key}, 0));
            }
        }
        if (pred_on && p.pending) {
            for (int kind : {K_PA, K_PAA}) {
                const bool flag = kind == K_PA ? r->pa : r->paa;
                const vector<PTerm>& ts = kind == K_PA ? r->pa_req : r->paa_req;
                if (!flag || ts.empty()) continue;
                vector<Prop> props;
                vector<string> ks;
                bool err = false;
                for (auto& t : ts) {
                    if (bad_sel(t)) err = true;
                    if (t.key.empty()) throw std::invalid_argument("empty topology key in a required pod (anti-)affinity term");
                    props.push_back(resolve(t, i));
                    ks.push_back(t.key);
                }
                if (err) { own_pred_err[i] = 1; continue; }  // the selector error fails every node
                (kind == K_PA ? own_pa : own_paa)[i] = class_of(kind, props, ks, 0);
            }
        }
        if (ipa_on && p.pending) {
            if (r->pa)
                for (auto& wt : r->pa_pref) {
                    if (bad_sel(wt.second)) throw std::invalid_argument("invalid label selector in a preferred pod affinity term");
                    if (wt.second.key.empty() || wt.first == 0) continue;
                    own_q[i].push_back({class_of(K_Q, {resolve(wt.second, i)}, {wt.second.key}, 0), wt.first});
                }
            if (r->paa)
                for (auto& wt : r->paa_pref) {
                    if (bad_sel(wt.second)) throw std::invalid_argument("invalid label selector in a preferred pod anti-affinity term");
                    if (wt.second.key.empty() || wt.first == 0) continue;
                    own_q[i].push_back({class_of(K_Q, {resolve(wt.second, i)}, {wt.second.key}, 0), -wt.first});
                }
        }
        if (ipa_on && (p.node >= 0 || p.pending)) {
            auto add_r = [&](const PTerm& t, int w) {
                if (bad_sel(t)) throw std::invalid_argument("invalid label selector in an existing pod's affinity term");
                if (t.key.empty() || w == 0) return;
                own_r[i].push_back(class_of(K_R, {resolve(t, i)}, {t.key}, w));
            };
            if (r->pa) {
                for (auto& t : r->pa_req) add_r(t, 1);  // hardPodAffinityWeight
                for (auto& wt : r->pa_pref) add_r(wt.second, wt.first);
            }
            if (r->paa)
                for (auto& wt : r->paa_pref) add_r(wt.second, -wt.first);
        }
    }
    mark("term classes");
    n_spaces = (int)space_size.size();
    if (n_spaces == 0) dom.assign(npad, -1);
    // table offsets
    for (auto& c : classes) {
        c.cnt_off = (int)cnt.size();
        cnt.resize(cnt.size() + std::max(space_size[c.space], 1), 0);
        if (c.kind == K_PA || c.kind == K_Q || c.kind == K_R) {
            c.scal = (int)scalar.size();
            scalar.push_back(0);
        }
    }
    if (scalar.empty()) scalar.push_back(0);
    if (cnt.empty()) cnt.push_back(0);

    // membership: does a pod of label group g satisfy every property of class c
    std::unordered_map<int64_t, char> memo;
    auto matches = [&](int c, int g) -> bool {
        const int64_t k = (int64_t)c * (int64_t)g_labels.size() + g;
        auto it = memo.find(k);
        if (it != memo.end()) return it->second;
        bool ok = true;
        for (auto& p : classes[c].props) {
            if (!std::binary_search(p.ns.begin(), p.ns.end(), g_ns[g]) || !sel_match(sels[p.sel], g_labels[g])) {
                ok = false;
                break;
            }
        }
        memo.emplace(k, ok);
        return ok;
    };
    // Candidate classes per label group: a class whose first property's
    // selector requires some (key, value) (an In requirement) can only match a
    // group carrying one of those labels; the rest are checked for every
    // group.  Keeps the membership tests per group proportional to the classes
    // that mention its labels (C3: one self-anti-affinity class per gang).
    std::unordered_map<int64_t, vector<int>> by_label;  // key << 32 | value -> classes (ascending)
    vector<int> unanchored;
    for (int c = 0; c < (int)classes.size(); ++c) {
        const LSel* sl = classes[c].props.empty() ? nullptr : &sels[classes[c].props[0].sel];
        const LReq* in = nullptr;
        if (sl && !sl->nothing && !sl->err)
            for (const LReq& r : sl->reqs)
                if (r.op == L_IN && (!in || r.vals.size() < in->vals.size())) in = &r;
        if (!in) { unanchored.push_back(c); continue; }
        for (int v : in->vals) by_label[((int64_t)in->key << 32) | (uint32_t)v].push_back(c);
    }
    vector<vector<int>> g_cands(g_labels.size());
    vector<char> g_cands_built(g_labels.size(), 0);
    auto cands = [&](int g) -> const vector<int>& {
        vector<int>& v = g_cands[g];
        if (g_cands_built[g]) return v;
        g_cands_built[g] = 1;
        v = unanchored;
        for (auto& kv : g_labels[g]) {
            auto it = by_label.find(((int64_t)kv.first << 32) | (uint32_t)kv.second);
            if (it != by_label.end()) v.insert(v.end(), it->second.begin(), it->second.end());
        }
        std::sort(v.begin(), v.end());
        v.erase(std::unique(v.begin(), v.end()), v.end());
        return v;
    };

    mark("tables+index");
    // ---------------- retained for recount / target_updates ----------------
    npad_ = npad;
    cls_.clear();
    for (auto& c : classes) cls_.push_back(CInfo{c.kind, c.space, c.cnt_off, c.scal});
    pod_group_ = group;
    own_ea_ = own_ea;
    own_r_ = own_r;
    g_tgt_.assign(g_labels.size(), {});
    g_q_.assign(g_labels.size(), {});
    for (int g = 0; g < (int)g_labels.size(); ++g)
        for (int c : cands(g)) {
            const int k = classes[c].kind;
            if ((k == K_PA || k == K_PAA) && matches(c, g)) g_tgt_[g].push_back(c);
            else if (k == K_Q && matches(c, g)) g_q_[g].push_back(c);
        }
    // ---------------- initial counts ----------------
    recount(pods);
    mark("counts");
    // ---------------- programs of pending tasks ----------------
    // (label group, the pod's own term classes) -> program
    std::map<vector<int>, int> cache;  // -> index into progs_ (-1: empty program)
    progs_.clear();
    prog_of_.assign(P, -1);
    vector<int> ck, prev_ck;
    int prev_prog = -1;
    for (int i = 0; i < P; ++i) {
        if (!pods[i].pending) continue;
        ck.assign({group[i], own_pred_err[i], own_pa[i], own_paa[i], (int)own_ea[i].size(), (int)own_q[i].size()});
        ck.insert(ck.end(), own_ea[i].begin(), own_ea[i].end());
        for (auto& q : own_q[i]) ck.insert(ck.end(), {q.first, q.second});
        ck.insert(ck.end(), own_r[i].begin(), own_r[i].end());
        if (!prev_ck.empty() && ck == prev_ck) {  // the previous pending pod's (a gang's pods)
            prog_of_[i] = prev_prog;
            continue;
        }
        auto it = cache.find(ck);
        if (it == cache.end()) {
            AffProgram pg;
            const int g = group[i];
            pg.pred_err = own_pred_err[i];
            const vector<int>& cg = cands(g);
            for (int c : cg)
                if (classes[c].kind == K_EA && matches(c, g)) { pg.ea.push_back(classes[c].space); pg.ea.push_back(classes[c].cnt_off); }
            if (own_pa[i] >= 0) {
                const TClass& c = classes[own_pa[i]];
                pg.pa_space = c.space; pg.pa_cnt = c.cnt_off; pg.pa_total = c.scal;
                pg.pa_self = matches(own_pa[i], g) ? 1 : 0;
            }
            if (own_paa[i] >= 0) {
                const TClass& c = classes[own_paa[i]];
                pg.paa_space = c.space; pg.paa_cnt = c.cnt_off;
            }
            for (auto& q : own_q[i]) {
                const TClass& c = classes[q.first];
                pg.ipa.insert(pg.ipa.end(), {c.space, c.cnt_off, c.scal, q.second});
            }
            for (int c : cg)
                if (classes[c].kind == K_R && matches(c, g)) {
                    const TClass& rc = classes[c];
                    pg.ipa.insert(pg.ipa.end(), {rc.space, rc.cnt_off, rc.scal, rc.weight});
                }
            // commit updates: what this task changes once it is placed
            for (int c : own_ea[i]) pg.upd.insert(pg.upd.end(), {UPD_CNT_ALLOC, classes[c].space, classes[c].cnt_off});
            for (int c : cg)
                if ((classes[c].kind == K_PA || classes[c].kind == K_PAA) && matches(c, g)) {
                    pg.upd.insert(pg.upd.end(), {UPD_CNT_ALLOC, classes[c].space, classes[c].cnt_off});
                    if (classes[c].kind == K_PA) pg.upd.insert(pg.upd.end(), {UPD_SCALAR_ALLOC, 0, classes[c].scal});
                }
            for (int c : cg)
                if (classes[c].kind == K_Q && matches(c, g)) pg.upd.insert(pg.upd.end(), {UPD_SCALAR_ANY, 0, classes[c].scal});
            for (int c : own_r[i]) pg.upd.insert(pg.upd.end(), {UPD_SCALAR_ANY, 0, classes[c].scal});
            int k = -1;
            if (!pg.empty()) {
                k = (int)progs_.size();
                progs_.push_back(std::move(pg));
            }
            it = cache.emplace(ck, k).first;
        }
        prog_of_[i] = it->second;
        prev_ck.swap(ck);
        prev_prog = it->second;
    }
    mark("programs");
}

void AffinityModel::recount(const vector<AffPod>& pods) {
    if (!active) return;
    std::fill(cnt.begin(), cnt.end(), 0);
    std::fill(scalar.begin(), scalar.end(), 0);
    auto dom_at = [&](int c, int n) { return dom[(size_t)cls_[c].space * npad_ + n]; };
    for (int i = 0; i < (int)pods.size(); ++i) {
        const AffPod& p = pods[i];
        const int g = pod_group_[i];
        if (p.target && p.node >= 0) {  // predicate targets (predicates.go:59-94)
            for (int c : own_ea_[i]) {
                const int d = dom_at(c, p.node);
                if (d >= 0) cnt[cls_[c].cnt_off + d]++;
            }
            for (int c : g_tgt_[g]) {
                if (cls_[c].kind == K_PA) scalar[cls_[c].scal]++;
                const int d = dom_at(c, p.node);
                if (d >= 0) cnt[cls_[c].cnt_off + d]++;
            }
        }
        if (p.node >= 0) {  // IPA pods: every pod on a node, at its (raw) node
            for (int c : g_q_[g]) {
                const int d = dom_at(c, p.node);
                if (d >= 0) cnt[cls_[c].cnt_off + d]++;
            }
            for (int c : own_r_[i]) {
                const int d = dom_at(c, p.node);
                if (d >= 0) cnt[cls_[c].cnt_off + d]++;
            }
        }
    }
}

void AffinityModel::target_updates(int pod, vector<int32_t>& out) const {
    out.clear();
    if (!active || pod < 0 || pod >= (int)pod_group_.size()) return;
    for (int c : own_ea_[pod]) out.insert(out.end(), {UPD_CNT_ALLOC, cls_[c].space, cls_[c].cnt_off});
    for (int c : g_tgt_[pod_group_[pod]]) {
        out.insert(out.end(), {UPD_CNT_ALLOC, cls_[c].space, cls_[c].cnt_off});
        if (cls_[c].kind == K_PA) out.insert(out.end(), {UPD_SCALAR_ALLOC, 0, cls_[c].scal});
    }
}

}  // namespace kbhip
