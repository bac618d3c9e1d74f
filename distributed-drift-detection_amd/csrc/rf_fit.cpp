// Native forest refit: train_rf (DDM_Process.py:98-105) without the Python overhead.
//
// RandomForestClassifier(n_estimators=T, defaults) .fit on one shuffled 100-row batch,
// restated from scikit-learn 1.7.2 so that the trees are IDENTICAL to sklearn's:
//   ensemble/_forest.py  _parallel_build_trees / _generate_sample_indices:
//       bootstrap = RandomState(seed_t).randint(0, n, n) -> sample_weight = bincount
//   tree/_classes.py     max_features="sqrt" -> max(1, int(sqrt(F))), min_samples_split 2,
//                        min_samples_leaf 1, max_depth None -> DepthFirstTreeBuilder
//   tree/_tree.pyx       DepthFirstTreeBuilder.build (stack: right child pushed first)
//   tree/_splitter.pyx   Splitter.init (samples = indices with weight != 0,
//                        rand_r_state = RandomState(seed_t).randint(0, 2**31-1)),
//                        node_split_best (Fisher-Yates feature draw with our_rand_r and
//                        constant-feature bookkeeping, best proxy improvement, threshold
//                        = midpoint of float32 neighbours)
//   tree/_partitioner.pyx next_p / constant test in float32 (+FEATURE_THRESHOLD 1e-7f),
//                        partition_samples_final (x <= threshold goes left)
//   tree/_criterion.pyx  Gini node/children impurity, proxy and impurity improvement,
//                        node_value = sum_total / weighted_n_node_samples
// Class counts and weights are integers, so every sum is exact whatever the order of
// samples with equal feature values; only the formulas' operation order matters, and
// it is kept (compiled without FMA contraction).  Inputs with NaN are rejected
// (DDM_E_NAN); the caller then uses sklearn itself.
//
// Output: the forest already packed in the ddm_node layout (same BFS renumbering as
// ddm_amd/treepack.py:pack), ready for ddm_forest_predict.
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../../include/ddm_amd.h"

namespace {

// ---- numpy legacy MT19937 seeded by init_genrand (RandomState(int)) -------------------
struct MT {
    uint32_t mt[624];
    int pos;
    explicit MT(uint32_t s) {
        mt[0] = s;
        for (int i = 1; i < 624; ++i) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
        pos = 624;
    }
    uint32_t next() {
        if (pos >= 624) {
            for (int i = 0; i < 624; ++i) {
                const uint32_t y = (mt[i] & 0x80000000u) | (mt[(i + 1) % 624] & 0x7fffffffu);
                mt[i] = mt[(i + 397) % 624] ^ (y >> 1) ^ (-(y & 1u) & 0x9908b0dfu);
            }
            pos = 0;
        }
        uint32_t y = mt[pos++];
        y ^= y >> 11;
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= y >> 18;
        return y;
    }
    uint32_t interval(uint32_t mx) {
        if (mx == 0) return 0;
        uint32_t mask = mx;
        mask |= mask >> 1;
        mask |= mask >> 2;
        mask |= mask >> 4;
        mask |= mask >> 8;
        mask |= mask >> 16;
        uint32_t v;
        while ((v = next() & mask) > mx) {
        }
        return v;
    }
};

constexpr uint32_t kRandRMax = 0x7fffffffu;
constexpr float kFeatureThreshold = 1e-7f;
constexpr double kEpsilon = 2.220446049250313e-16;   // np.finfo('double').eps (_tree.pyx:44)

inline uint32_t our_rand_r(uint32_t* seed) {
    if (seed[0] == 0) seed[0] = 1;
    seed[0] ^= (uint32_t)(seed[0] << 13);
    seed[0] ^= (uint32_t)(seed[0] >> 17);
    seed[0] ^= (uint32_t)(seed[0] << 5);
    return seed[0] % (kRandRMax + 1u);
}

inline int64_t rand_int(int64_t low, int64_t high, uint32_t* seed) {
    return low + (int64_t)our_rand_r(seed) % (high - low);
}

// sklearn-ordered tree (node ids in _add_node order)
struct Tree {
    std::vector<int32_t> left, right, feature;
    std::vector<double> threshold;
    std::vector<uint8_t> missing_left;
    std::vector<double> value;   // [node][K]
};

struct Builder {
    const float* X;
    int n, F, K, max_features;
    const int32_t* y;
    std::vector<double> w;            // bootstrap counts
    std::vector<int64_t> samples;
    std::vector<float> fv;
    std::vector<int64_t> features, constant;
    std::vector<double> sum_total, sum_left, sum_right;
    double weighted_n_samples = 0, wn_node = 0, wn_left = 0, wn_right = 0;
    int64_t start = 0, end = 0, pos = 0;
    uint32_t rand_r_state = 0;
    std::vector<std::pair<float, int64_t>> sortbuf;

    float x(int64_t s, int64_t f) const { return X[s * F + f]; }

    // ClassificationCriterion.init over samples[start:end]
    void crit_init(int64_t s0, int64_t s1) {
        start = s0;
        end = s1;
        std::fill(sum_total.begin(), sum_total.end(), 0.0);
        wn_node = 0.0;
        for (int64_t p = s0; p < s1; ++p) {
            const int64_t i = samples[p];
            sum_total[y[i]] += w[i];
            wn_node += w[i];
        }
        crit_reset();
    }
    void crit_reset() {
        pos = start;
        std::fill(sum_left.begin(), sum_left.end(), 0.0);
        for (int c = 0; c < K; ++c) sum_right[c] = sum_total[c];
        wn_left = 0.0;
        wn_right = wn_node;
    }
    void crit_update(int64_t new_pos) {   // exact integer sums: forward accumulation suffices
        for (int64_t p = pos; p < new_pos; ++p) {
            const int64_t i = samples[p];
            sum_left[y[i]] += w[i];
            wn_left += w[i];
        }
        wn_right = wn_node - wn_left;
        for (int c = 0; c < K; ++c) sum_right[c] = sum_total[c] - sum_left[c];
        pos = new_pos;
    }
    double node_impurity() const {
        double sq = 0.0;
        for (int c = 0; c < K; ++c) sq += sum_total[c] * sum_total[c];
        const double gini = 1.0 - sq / (wn_node * wn_node);
        return gini / 1.0;
    }
    void children_impurity(double* il, double* ir) const {
        double sl = 0.0, sr = 0.0;
        for (int c = 0; c < K; ++c) {
            sl += sum_left[c] * sum_left[c];
            sr += sum_right[c] * sum_right[c];
        }
        const double gl = 1.0 - sl / (wn_left * wn_left);
        const double gr = 1.0 - sr / (wn_right * wn_right);
        *il = gl / 1.0;
        *ir = gr / 1.0;
    }
    double proxy_improvement() const {
        double il, ir;
        children_impurity(&il, &ir);
        return (-wn_right * ir) - wn_left * il;
    }
    double impurity_improvement(double parent, double il, double ir) const {
        return (wn_node / weighted_n_samples) * (parent - (wn_right / wn_node * ir) - (wn_left / wn_node * il));
    }

    void sort_feature(int64_t f) {
        sortbuf.clear();
        for (int64_t p = start; p < end; ++p) sortbuf.emplace_back(x(samples[p], f), samples[p]);
        std::sort(sortbuf.begin(), sortbuf.end(),
                  [](const std::pair<float, int64_t>& a, const std::pair<float, int64_t>& b) { return a.first < b.first; });
        for (int64_t p = start; p < end; ++p) {
            fv[p] = sortbuf[p - start].first;
            samples[p] = sortbuf[p - start].second;
        }
    }

    struct Split {
        int64_t pos, feature;
        double threshold, improvement, il, ir;
        bool missing_left;
    };

    // node_split_best (no missing values)
    Split node_split(double impurity, int64_t* n_constant_features) {
        Split best{end, 0, 0.0, -INFINITY, INFINITY, INFINITY, false}, cur = best;
        double best_proxy = -INFINITY;
        int64_t f_i = F, n_visited = 0, n_found_c = 0, n_drawn_c = 0;
        const int64_t n_known_c = *n_constant_features;
        int64_t n_total_c = n_known_c;
        while (f_i > n_total_c && (n_visited < max_features || n_visited <= n_found_c + n_drawn_c)) {
            ++n_visited;
            int64_t f_j = rand_int(n_drawn_c, f_i - n_found_c, &rand_r_state);
            if (f_j < n_known_c) {
                std::swap(features[n_drawn_c], features[f_j]);
                ++n_drawn_c;
                continue;
            }
            f_j += n_found_c;
            cur.feature = features[f_j];
            sort_feature(cur.feature);
            if (end == start || fv[end - 1] <= fv[start] + kFeatureThreshold) {
                std::swap(features[f_j], features[n_total_c]);
                ++n_found_c;
                ++n_total_c;
                continue;
            }
            --f_i;
            std::swap(features[f_i], features[f_j]);
            crit_reset();
            int64_t p = start, p_prev = start;
            while (p < end) {
                while (p + 1 < end && fv[p + 1] <= fv[p] + kFeatureThreshold) ++p;   // next_p
                p_prev = p;
                ++p;
                if (p >= end) continue;
                const int64_t n_left = p - start, n_right = end - p;
                if (n_left < 1 || n_right < 1) continue;
                cur.pos = p;
                crit_update(p);
                const double proxy = proxy_improvement();
                if (proxy > best_proxy) {
                    best_proxy = proxy;
                    cur.threshold = (double)fv[p_prev] / 2.0 + (double)fv[p] / 2.0;
                    if (cur.threshold == (double)fv[p] || cur.threshold == INFINITY || cur.threshold == -INFINITY)
                        cur.threshold = (double)fv[p_prev];
                    cur.missing_left = n_left > n_right;
                    best = cur;
                }
            }
        }
        if (best.pos < end) {
            // partition_samples_final
            int64_t p = start, pend = end;
            while (p < pend) {
                if ((double)x(samples[p], best.feature) <= best.threshold) ++p;
                else {
                    --pend;
                    std::swap(samples[p], samples[pend]);
                }
            }
            crit_reset();
            crit_update(best.pos);
            children_impurity(&best.il, &best.ir);
            best.improvement = impurity_improvement(impurity, best.il, best.ir);
        }
        memcpy(features.data(), constant.data(), sizeof(int64_t) * n_known_c);
        memcpy(constant.data() + n_known_c, features.data() + n_known_c, sizeof(int64_t) * n_found_c);
        *n_constant_features = n_total_c;
        return best;
    }

    void build(uint32_t seed, Tree& t) {
        // bootstrap (ensemble/_forest.py _generate_sample_indices)
        MT boot(seed);
        std::fill(w.begin(), w.end(), 0.0);
        for (int i = 0; i < n; ++i) w[boot.interval((uint32_t)(n - 1))] += 1.0;
        // splitter RNG: a fresh RandomState(seed) (tree/_classes.py check_random_state)
        MT split_rs(seed);
        rand_r_state = split_rs.interval(kRandRMax - 1u);
        samples.clear();
        weighted_n_samples = 0.0;
        for (int i = 0; i < n; ++i) {
            if (w[i] != 0.0) samples.push_back(i);
            weighted_n_samples += w[i];
        }
        for (int f = 0; f < F; ++f) features[f] = f;
        t = Tree();
        struct Rec {
            int64_t start, end, depth, parent;
            int is_left;
            double impurity;
            int64_t n_const;
        };
        std::vector<Rec> stack;
        stack.push_back({0, (int64_t)samples.size(), 0, -1, 0, INFINITY, 0});
        bool first = true;
        while (!stack.empty()) {
            Rec r = stack.back();
            stack.pop_back();
            const int64_t n_node = r.end - r.start;
            crit_init(r.start, r.end);
            bool is_leaf = n_node < 2 || wn_node < 0.0;
            double impurity = r.impurity;
            if (first) {
                impurity = node_impurity();
                first = false;
            }
            is_leaf = is_leaf || impurity <= kEpsilon;
            Split sp{r.end, 0, 0.0, -INFINITY, INFINITY, INFINITY, false};
            int64_t n_const = r.n_const;
            if (!is_leaf) {
                sp = node_split(impurity, &n_const);
                is_leaf = sp.pos >= r.end || sp.improvement + kEpsilon < 0.0;
            }
            const int32_t id = (int32_t)t.left.size();
            t.left.push_back(-1);
            t.right.push_back(-1);
            t.feature.push_back(is_leaf ? -2 : (int32_t)sp.feature);
            t.threshold.push_back(is_leaf ? -2.0 : sp.threshold);
            t.missing_left.push_back(sp.missing_left);
            for (int c = 0; c < K; ++c) t.value.push_back(sum_total[c] / wn_node);
            if (r.parent >= 0) (r.is_left ? t.left : t.right)[r.parent] = id;
            if (!is_leaf) {
                stack.push_back({sp.pos, r.end, r.depth + 1, id, 0, sp.ir, n_const});
                stack.push_back({r.start, sp.pos, r.depth + 1, id, 1, sp.il, n_const});
            }
        }
    }
};

}  // namespace

extern "C" int ddm_rf_fit(const float* X, int32_t n, int32_t n_features, const int32_t* y_idx, int32_t n_classes,
                          const int64_t* seeds, int32_t n_trees, int32_t max_features, ddm_node* nodes,
                          int64_t nodes_cap, int32_t* roots, double* leaf_value, int64_t leaf_rows_cap,
                          int64_t* out_info) {
    if (!X || !y_idx || !seeds || !nodes || !roots || !out_info || n <= 0 || n_features <= 0 || n_classes <= 0 ||
        n_trees <= 0 || max_features <= 0 || nodes_cap < (int64_t)n_trees * (2 * (int64_t)n - 1))
        return DDM_E_ARG;
    for (int64_t i = 0; i < (int64_t)n * n_features; ++i)
        if (X[i] != X[i]) return DDM_E_NAN;
    for (int i = 0; i < n; ++i)
        if (y_idx[i] < 0 || y_idx[i] >= n_classes) return DDM_E_ARG;
    Builder b;
    b.X = X;
    b.n = n;
    b.F = n_features;
    b.K = n_classes;
    b.max_features = max_features;
    b.y = y_idx;
    b.w.assign(n, 0.0);
    b.fv.assign(n, 0.0f);
    b.features.assign(n_features, 0);
    b.constant.assign(n_features, 0);
    b.sum_total.assign(n_classes, 0.0);
    b.sum_left.assign(n_classes, 0.0);
    b.sum_right.assign(n_classes, 0.0);
    b.samples.reserve(n);
    std::vector<Tree> trees(n_trees);
    bool pure = n_trees <= 255;
    for (int t = 0; t < n_trees; ++t) {
        b.build((uint32_t)seeds[t], trees[t]);
        const Tree& tr = trees[t];
        for (size_t u = 0; pure && u < tr.left.size(); ++u) {
            if (tr.left[u] != -1) continue;
            int ones = 0, others = 0;
            for (int c = 0; c < n_classes; ++c) {
                const double v = tr.value[u * n_classes + c];
                ones += v == 1.0;
                others += (v != 0.0 && v != 1.0);
            }
            pure = (ones == 1 && others == 0);
        }
    }
    // pack: BFS renumbering with adjacent siblings (treepack.py:pack)
    int64_t base = 0, leaf_rows = 0;
    std::vector<int64_t> order, new_id;
    for (int t = 0; t < n_trees; ++t) {
        const Tree& tr = trees[t];
        const int64_t m = (int64_t)tr.left.size();
        new_id.assign(m, 0);
        order.assign(1, 0);
        int64_t nxt = 1;
        for (size_t qi = 0; qi < order.size(); ++qi) {
            const int64_t u = order[qi];
            if (tr.left[u] != -1) {
                new_id[tr.left[u]] = nxt;
                new_id[tr.right[u]] = nxt + 1;
                order.push_back(tr.left[u]);
                order.push_back(tr.right[u]);
                nxt += 2;
            }
        }
        roots[t] = (int32_t)base;
        for (int64_t u = 0; u < m; ++u) {
            ddm_node& nd = nodes[base + new_id[u]];
            if (tr.left[u] != -1) {
                nd.threshold = tr.threshold[u];
                nd.feature = tr.feature[u] | (tr.missing_left[u] ? (1 << 30) : 0);
                nd.child = (int32_t)(base + new_id[tr.left[u]]);
            } else {
                nd.threshold = 0.0;
                nd.feature = -1;
                if (pure) {
                    int best = 0;
                    for (int c = 1; c < n_classes; ++c)
                        if (tr.value[u * n_classes + c] > tr.value[u * n_classes + best]) best = c;
                    nd.child = best;
                } else {
                    if (!leaf_value || leaf_rows >= leaf_rows_cap) return DDM_E_IMPURE;
                    memcpy(leaf_value + leaf_rows * n_classes, &tr.value[u * n_classes], sizeof(double) * n_classes);
                    nd.child = (int32_t)leaf_rows++;
                }
            }
        }
        base += m;
    }
    out_info[0] = base;
    out_info[1] = pure ? 1 : 0;
    out_info[2] = leaf_rows;
    return 0;
}
