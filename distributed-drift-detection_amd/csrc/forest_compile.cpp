// Host compiler from the packed node forest (ddm_node, BFS, adjacent children) to the
// blob the fast predict kernels evaluate (include/ddm_amd.h, ddm_cforest_head).
//
// predict_rf (DDM_Process.py:110-128) runs sklearn's forest.predict: per tree the leaf
// reached by `(double)x_f32 <= threshold` tests, votes summed over trees, first argmax.
// For a pure forest (one-hot leaves) the vote of a tree is the class of its exit leaf,
// so the forest is rewritten without changing any decision:
//   * a float32 x satisfies (double)x <= t exactly when x <= t32, t32 = the largest
//     float32 <= t, so every test becomes one float32 compare;
//   * single-leaf trees always vote the same class: folded into base_votes;
//   * stumps vote cl or cr: base_votes takes cl, the kernel adds (cr - cl) when x > t32
//     (u8 counters packed in uint32 words; the packed sum is exact because every final
//     count is <= n_trees <= 255);
//   * other trees: QuickScorer masks (a node that sends the row right clears the leaves
//     of its left subtree; the exit leaf is the leftmost leaf left standing).
// Only the feature columns the forest reads are loaded (slots).
#include <math.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../../include/ddm_amd.h"

namespace ddm {
void set_error(const char* fmt, ...);
}

namespace {

constexpr int kMaxSlots = 32;
constexpr int kMaxClasses = 16;
constexpr int kMaxLeaves = 64;

float float_floor_of(double t) {
    float f = (float)t;
    if ((double)f > t) f = nextafterf(f, -INFINITY);
    return f;
}

int64_t align16(int64_t v) { return (v + 15) & ~(int64_t)15; }

struct Stump {
    int slot;
    float thr;
    int cl, cr;
    int nanleft;
};

}  // namespace

extern "C" int ddm_forest_compile(const ddm_node* nodes, int32_t n_nodes, const int32_t* roots, int32_t n_trees,
                                  const int32_t* classes, int32_t n_classes, int32_t pure, uint8_t* out, int64_t cap,
                                  int64_t* out_bytes) {
    if (!nodes || !roots || !classes || n_nodes <= 0 || n_trees <= 0 || n_classes <= 0 || !out_bytes) {
        ddm::set_error("ddm_forest_compile: invalid argument");
        return DDM_E_ARG;
    }
    if (!pure || n_trees > 255 || n_classes > kMaxClasses) {
        ddm::set_error("ddm_forest_compile: not compilable (pure=%d trees=%d classes=%d)", pure, n_trees, n_classes);
        return DDM_E_FOREST;
    }
    const int vr = n_classes <= 4 ? 1 : n_classes <= 8 ? 2 : 4;
    std::vector<int> slot_of_col;   // feature column -> slot (grown on demand)
    std::vector<int> cols;
    auto slot = [&](int col) -> int {
        if (col >= (int)slot_of_col.size()) slot_of_col.resize(col + 1, -1);
        if (slot_of_col[col] < 0) {
            slot_of_col[col] = (int)cols.size();
            cols.push_back(col);
        }
        return slot_of_col[col];
    };
    auto inc = [&](int c, uint32_t* v) { v[c >> 2] += 1u << (8 * (c & 3)); };

    uint32_t base[4] = {0, 0, 0, 0};
    std::vector<Stump> stumps;
    std::vector<ddm_cforest_tree> trees;
    std::vector<ddm_cforest_node> gnodes;
    std::vector<uint8_t> leaf_cls;    // class of every general-tree leaf
    bool any_nanleft = false;

    for (int t = 0; t < n_trees; ++t) {
        const int r = roots[t];
        if (r < 0 || r >= n_nodes) {
            ddm::set_error("ddm_forest_compile: bad root %d", r);
            return DDM_E_ARG;
        }
        const ddm_node& root = nodes[r];
        if (root.feature < 0) {                       // single leaf
            if (root.child < 0 || root.child >= n_classes) return DDM_E_FOREST;
            inc(root.child, base);
            continue;
        }
        const ddm_node& L = nodes[root.child];
        const ddm_node& R = nodes[root.child + 1];
        const int col = root.feature & 0x3fffffff;
        const int nl = (root.feature >> 30) & 1;
        if (L.feature < 0 && R.feature < 0) {         // stump
            if (L.child < 0 || L.child >= n_classes || R.child < 0 || R.child >= n_classes) return DDM_E_FOREST;
            stumps.push_back({slot(col), float_floor_of(root.threshold), L.child, R.child, nl});
            any_nanleft |= nl != 0;
            inc(L.child, base);
            continue;
        }
        // general tree: in-order leaf numbering, left-subtree leaf masks
        ddm_cforest_tree tr;
        tr.node_begin = (int)gnodes.size();
        tr.leaf_begin = (int)leaf_cls.size();
        int n_leaves = 0;
        // iterative post-order: returns [first leaf, end leaf) of each subtree
        struct Frame { int node; int stage; int lo; int node_idx; };
        std::vector<Frame> st;
        st.push_back({r, 0, 0, -1});
        int ret_lo = 0, ret_hi = 0;
        while (!st.empty()) {
            Frame& f = st.back();
            const ddm_node& nd = nodes[f.node];
            if (nd.feature < 0) {
                if (nd.child < 0 || nd.child >= n_classes || n_leaves >= kMaxLeaves) {
                    ddm::set_error("ddm_forest_compile: tree %d exceeds %d leaves", t, kMaxLeaves);
                    return DDM_E_FOREST;
                }
                leaf_cls.push_back((uint8_t)nd.child);
                ret_lo = n_leaves;
                ret_hi = ++n_leaves;
                st.pop_back();
                continue;
            }
            if (f.stage == 0) {
                ddm_cforest_node cn;
                cn.threshold = float_floor_of(nd.threshold);
                const int nlb = (nd.feature >> 30) & 1;
                any_nanleft |= nlb != 0;
                cn.slot_nanleft = slot(nd.feature & 0x3fffffff) | (nlb << 8);
                cn.left_lo = cn.left_hi = 0;
                f.node_idx = (int)gnodes.size();
                gnodes.push_back(cn);
                f.stage = 1;
                st.push_back({nd.child, 0, 0, -1});
            } else if (f.stage == 1) {               // left subtree done: [ret_lo, ret_hi)
                uint64_t m = 0;
                for (int k = ret_lo; k < ret_hi; ++k) m |= 1ull << k;
                gnodes[f.node_idx].left_lo = (uint32_t)m;
                gnodes[f.node_idx].left_hi = (uint32_t)(m >> 32);
                f.lo = ret_lo;
                f.stage = 2;
                st.push_back({nd.child + 1, 0, 0, -1});
            } else {                                 // right subtree done
                ret_lo = f.lo;
                st.pop_back();
            }
        }
        tr.n_nodes = (int)gnodes.size() - tr.node_begin;
        tr.n_leaves = n_leaves;
        trees.push_back(tr);
    }
    if ((int)cols.size() > kMaxSlots) {
        ddm::set_error("ddm_forest_compile: %d feature columns > %d", (int)cols.size(), kMaxSlots);
        return DDM_E_FOREST;
    }
    std::stable_sort(stumps.begin(), stumps.end(), [](const Stump& a, const Stump& b) {
        return a.nanleft != b.nanleft ? a.nanleft < b.nanleft : a.slot < b.slot;
    });

    const int S = (int)stumps.size();
    const int64_t stumps_off = align16(sizeof(ddm_cforest_head));
    const int sw = vr <= 2 ? 4 : 8;                 // 16- or 32-byte stump records
    const int64_t trees_off = align16(stumps_off + 4 * (int64_t)S * sw);
    const int64_t nodes_off = align16(trees_off + (int64_t)sizeof(ddm_cforest_tree) * trees.size());
    const int64_t leafcls_off = align16(nodes_off + (int64_t)sizeof(ddm_cforest_node) * gnodes.size());
    // per-slot rank thresholds and prefix-vote tables (ddm_cforest_slot)
    std::vector<std::vector<int>> by_slot(cols.size());
    for (int k = 0; k < S; ++k) by_slot[stumps[k].slot].push_back(k);
    // records padded with empty slots (n4 = 0) to a multiple of 8: the kernel walks slots
    // eight at a time
    std::vector<ddm_cforest_slot> srec((cols.size() + 7) & ~(size_t)7);
    for (ddm_cforest_slot& rs : srec) {
        memset(&rs, 0, sizeof(rs));
        rs.col = cols.empty() ? 0 : cols.back();
    }
    std::vector<float> xthr;
    std::vector<uint32_t> rtab;
    for (size_t sl = 0; sl < cols.size(); ++sl) {
        std::vector<int>& ks = by_slot[sl];
        std::stable_sort(ks.begin(), ks.end(), [&](int a, int b) { return stumps[a].thr < stumps[b].thr; });
        const int m = (int)ks.size();
        ddm_cforest_slot& rs = srec[sl];
        rs.col = cols[sl];
        rs.n4 = m ? m / 4 + 1 : 0;
        rs.tab = (int32_t)(rtab.size() / vr);
        rs.xthr = (int32_t)(xthr.size() / 4);
        for (int q = 0; q < 4; ++q) rs.thr[q] = q < m ? stumps[ks[q]].thr : INFINITY;
        for (int q = 4; q < 4 * rs.n4; ++q) xthr.push_back(q < m ? stumps[ks[q]].thr : INFINITY);
        if (!m) continue;
        uint32_t acc[4] = {0, 0, 0, 0}, nan_acc[4] = {0, 0, 0, 0};
        for (int q = 0; q < 4 * rs.n4; ++q) {       // entry q = deltas of the min(q, m) lowest
            for (int j = 0; j < vr; ++j) rtab.push_back(acc[j]);
            if (q >= m) continue;
            const Stump& st = stumps[ks[q]];
            uint32_t vl[4] = {0, 0, 0, 0}, vrr[4] = {0, 0, 0, 0};
            inc(st.cl, vl);
            inc(st.cr, vrr);
            for (int j = 0; j < vr; ++j) {
                acc[j] += vrr[j] - vl[j];
                if (!st.nanleft) nan_acc[j] += vrr[j] - vl[j];
            }
        }
        for (int j = 0; j < vr; ++j) rtab.push_back(nan_acc[j]);   // entry 4*n4: x is NaN
    }
    const int64_t slots_off = align16(leafcls_off + (int64_t)leaf_cls.size());
    const int64_t xthr_off = align16(slots_off + (int64_t)sizeof(ddm_cforest_slot) * srec.size());
    const int64_t rank_tab_off = align16(xthr_off + 4 * (int64_t)xthr.size());
    const int64_t total = align16(rank_tab_off + 4 * (int64_t)rtab.size());
    *out_bytes = total;
    if (!out || cap == 0) return 0;
    if (cap < total) {
        ddm::set_error("ddm_forest_compile: blob needs %lld bytes, cap %lld", (long long)total, (long long)cap);
        return DDM_E_ARG;
    }
    memset(out, 0, total);
    ddm_cforest_head h;
    memset(&h, 0, sizeof(h));
    h.n_slots = (int)cols.size();
    h.n_classes = n_classes;
    h.vote_regs = vr;
    h.n_stumps = S;
    h.n_general = (int)trees.size();
    h.n_leaves = (int)leaf_cls.size();
    h.total_bytes = (int)total;
    h.any_nanleft = any_nanleft ? 1 : 0;
    h.stumps_off = (int)stumps_off;
    h.stump_words = sw;
    h.trees_off = (int)trees_off;
    h.nodes_off = (int)nodes_off;
    h.leafcls_off = (int)leafcls_off;
    for (int k = 0; k < 4; ++k) h.base_votes[k] = base[k];
    for (int s = 0; s < kMaxSlots; ++s)               // past n_slots: the last column (the
        h.cols[s] = cols.empty() ? 0 : cols[std::min<int>(s, (int)cols.size() - 1)];   // kernel loads 8 at a time)
    int n_right = 0;
    while (n_right < S && stumps[n_right].nanleft == 0) ++n_right;
    h.n_stumps_right = n_right;
    for (int c = 0; c < n_classes; ++c) h.classes[c] = classes[c];
    memcpy(out, &h, sizeof(h));
    uint32_t* rec = reinterpret_cast<uint32_t*>(out + stumps_off);
    for (int k = 0; k < S; ++k, rec += sw) {
        memcpy(rec, &stumps[k].thr, 4);
        rec[1] = (uint32_t)stumps[k].slot;
        uint32_t vl[4] = {0, 0, 0, 0}, vrr[4] = {0, 0, 0, 0};
        inc(stumps[k].cl, vl);
        inc(stumps[k].cr, vrr);
        for (int j = 0; j < vr; ++j) rec[2 + j] = vrr[j] - vl[j];
    }
    if (!trees.empty()) memcpy(out + trees_off, trees.data(), sizeof(ddm_cforest_tree) * trees.size());
    if (!gnodes.empty()) memcpy(out + nodes_off, gnodes.data(), sizeof(ddm_cforest_node) * gnodes.size());
    if (!leaf_cls.empty()) memcpy(out + leafcls_off, leaf_cls.data(), leaf_cls.size());
    ddm_cforest_head* hp = reinterpret_cast<ddm_cforest_head*>(out);
    hp->slots_off = (int)slots_off;
    hp->xthr_off = (int)xthr_off;
    hp->rank_tab_off = (int)rank_tab_off;
    hp->rank_tab_entries = (int)(rtab.size() / vr);
    if (!srec.empty()) memcpy(out + slots_off, srec.data(), sizeof(ddm_cforest_slot) * srec.size());
    if (!xthr.empty()) memcpy(out + xthr_off, xthr.data(), 4 * xthr.size());
    if (!rtab.empty()) memcpy(out + rank_tab_off, rtab.data(), 4 * rtab.size());
    return 0;
}
