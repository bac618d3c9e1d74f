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
#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/ddm_amd.h"

namespace {

// ---- numpy legacy MT19937 seeded by init_genrand (RandomState(int)) -------------------
// The twist is done lazily, word by word: new word i needs old words i, i+1 and i+397
// (or the new word i-227), all available in order, so a tree pays for the ~130 words
// its bootstrap draws instead of a full 624-word block.
struct MT {
    uint32_t mt[624];
    int pos;          // next word to return
    int twisted;      // words [0, twisted) of the current block are already regenerated
    explicit MT(uint32_t s) {
        mt[0] = s;
        for (int i = 1; i < 624; ++i) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
        pos = 624;
        twisted = 624;
    }
    uint32_t raw(int i) {                       // word i of the next block, twisting on demand
        while (twisted <= i) {
            const int k = twisted++;
            const uint32_t y = (mt[k] & 0x80000000u) | (mt[(k + 1) % 624] & 0x7fffffffu);
            mt[k] = mt[(k + 397) % 624] ^ (y >> 1) ^ (-(y & 1u) & 0x9908b0dfu);
        }
        return mt[i];
    }
    static uint32_t temper(uint32_t y) {
        y ^= y >> 11;
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= y >> 18;
        return y;
    }
    uint32_t next() {
        if (pos >= 624) {
            if (twisted < 624) raw(623);            // finish the block before starting another
            pos = 0;
            twisted = 0;
        }
        return temper(raw(pos++));
    }
    // tempered word k positions ahead of the next one (k small), without consuming it
    uint32_t peek(int k) {
        if (pos >= 624) {
            if (twisted < 624) raw(623);
            pos = 0;
            twisted = 0;
        }
        return temper(raw(pos + k));
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
    // Presorted features: order[f] = the n training rows by ascending X[:, f], shared by
    // every tree and node.  A node's samples carry the node's tag, so its values sorted
    // by f are a filtered pass over order[f] (O(n)) instead of a sort.  Equal values may
    // come out in another order than sklearn's sort leaves them; split search and
    // partition depend only on the values and the (exact, integer) class sums.
    std::vector<int32_t> own_order;   // [F][n] when this builder sorted itself
    const int32_t* order = nullptr;   // [F][n] (own_order or a job's shared copy)
    std::vector<uint32_t> tag;        // [n]
    uint32_t cur_tag = 0;

    float x(int64_t s, int64_t f) const { return X[s * F + f]; }

    static void presort_into(const float* X, int n, int F, int32_t* order) {
        std::vector<std::pair<float, int32_t>> buf(n);
        for (int f = 0; f < F; ++f) {
            for (int i = 0; i < n; ++i) buf[i] = {X[(int64_t)i * F + f], i};
            std::sort(buf.begin(), buf.end(),
                      [](const std::pair<float, int32_t>& a, const std::pair<float, int32_t>& b) { return a.first < b.first; });
            for (int i = 0; i < n; ++i) order[(size_t)f * n + i] = buf[i].second;
        }
    }
    void use_order(const int32_t* shared) {
        if (shared) {
            order = shared;
        } else {
            own_order.assign((size_t)F * n, 0);
            presort_into(X, n, F, own_order.data());
            order = own_order.data();
        }
        tag.assign(n, 0);
        cur_tag = 0;
    }
    void tag_node() {                 // samples[start:end] belong to the node being split
        ++cur_tag;
        for (int64_t p = start; p < end; ++p) tag[samples[p]] = cur_tag;
    }

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
        const int32_t* o = order + (size_t)f * n;
        int64_t k = start;
        for (int i = 0; i < n; ++i) {
            const int32_t r = o[i];
            if (tag[r] == cur_tag) {
                samples[k] = r;
                fv[k] = x(r, f);
                ++k;
            }
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

    struct Rec {
        int64_t start, end, depth, parent;
        int is_left;
        double impurity;
        int64_t n_const;
    };
    std::vector<Rec> stack;

    void build(uint32_t seed, Tree& t) {
        // bootstrap (ensemble/_forest.py _generate_sample_indices) and the splitter seed,
        // which is the first randint(0, 2**31-1) of a fresh RandomState(seed)
        // (tree/_classes.py check_random_state): the same stream, so it is peeked from the
        // bootstrap generator before that consumes anything
        MT boot(seed);
        {
            int k = 0;
            uint32_t v;
            while ((v = boot.peek(k) & 0x7fffffffu) > kRandRMax - 1u) ++k;
            rand_r_state = v;
        }
        std::fill(w.begin(), w.end(), 0.0);
        for (int i = 0; i < n; ++i) w[boot.interval((uint32_t)(n - 1))] += 1.0;
        samples.clear();
        weighted_n_samples = 0.0;
        for (int i = 0; i < n; ++i) {
            if (w[i] != 0.0) samples.push_back(i);
            weighted_n_samples += w[i];
        }
        for (int f = 0; f < F; ++f) features[f] = f;
        t.left.clear();                 // keep the capacity of a reused tree
        t.right.clear();
        t.feature.clear();
        t.threshold.clear();
        t.missing_left.clear();
        t.value.clear();
        stack.clear();
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
                tag_node();
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

// Pack trees into the ddm_node layout: BFS renumbering with adjacent siblings
// (treepack.py:pack).  Returns 0 or DDM_E_IMPURE (leaf_value missing / too small).
int pack_trees(const Tree* trees, int n_trees, int n_classes, bool pure, ddm_node* nodes, int32_t* roots,
               double* leaf_value, int64_t leaf_rows_cap, int64_t* out_info) {
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

bool tree_is_pure(const Tree& tr, int n_classes) {
    for (size_t u = 0; u < tr.left.size(); ++u) {
        if (tr.left[u] != -1) continue;
        int ones = 0, others = 0;
        for (int c = 0; c < n_classes; ++c) {
            const double v = tr.value[u * n_classes + c];
            ones += v == 1.0;
            others += (v != 0.0 && v != 1.0);
        }
        if (!(ones == 1 && others == 0)) return false;
    }
    return true;
}

void builder_init(Builder& b, const float* X, int n, int F, const int32_t* y, int K, int max_features,
                  const int32_t* shared_order = nullptr) {
    b.X = X;
    b.n = n;
    b.F = F;
    b.K = K;
    b.max_features = max_features;
    b.y = y;
    b.w.assign(n, 0.0);
    b.fv.assign(n, 0.0f);
    b.features.assign(F, 0);
    b.constant.assign(F, 0);
    b.sum_total.assign(K, 0.0);
    b.sum_left.assign(K, 0.0);
    b.sum_right.assign(K, 0.0);
    b.samples.reserve(n);
    b.use_order(shared_order);
}

int check_inputs(const float* X, int32_t n, int32_t n_features, const int32_t* y_idx, int32_t n_classes) {
    for (int64_t i = 0; i < (int64_t)n * n_features; ++i)
        if (X[i] != X[i]) return DDM_E_NAN;
    for (int i = 0; i < n; ++i)
        if (y_idx[i] < 0 || y_idx[i] >= n_classes) return DDM_E_ARG;
    return 0;
}

// ---- a small persistent worker pool for ddm_rf_fit_many ------------------------------
class Pool {
  public:
    // Runs fn(i) for i in [0, n) on up to `threads` threads (the caller included).
    void run(int threads, int64_t n, const std::function<void(int64_t)>& fn) {
        if (threads <= 1 || n <= 1) {
            for (int64_t i = 0; i < n; ++i) fn(i);
            return;
        }
        std::unique_lock<std::mutex> lk(mu_);     // one batch at a time
        ensure(threads - 1);
        fn_ = &fn;
        n_ = n;
        next_.store(0);
        active_ = (int)std::min<int64_t>(threads - 1, (int64_t)workers_.size());
        done_ = 0;
        ++gen_;
        cv_.notify_all();
        lk.unlock();
        drain();
        lk.lock();
        cv_done_.wait(lk, [&] { return done_ == active_; });
        fn_ = nullptr;
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
            ++gen_;
        }
        cv_.notify_all();
        for (auto& t : workers_) t.join();
    }

  private:
    void ensure(int k) {
        while ((int)workers_.size() < k) {
            const int id = (int)workers_.size();
            workers_.emplace_back([this, id] { loop(id); });
        }
    }
    void drain() {
        for (;;) {
            const int64_t i = next_.fetch_add(1);
            if (i >= n_) break;
            (*fn_)(i);
        }
    }
    void loop(int id) {
        uint64_t seen = 0;
        std::unique_lock<std::mutex> lk(mu_);
        for (;;) {
            cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
            if (stop_) return;
            seen = gen_;
            if (id >= active_) continue;
            lk.unlock();
            drain();
            lk.lock();
            if (++done_ == active_) cv_done_.notify_all();
        }
    }
    std::mutex mu_;
    std::condition_variable cv_, cv_done_;
    std::vector<std::thread> workers_;
    const std::function<void(int64_t)>* fn_ = nullptr;
    std::atomic<int64_t> next_{0};
    int64_t n_ = 0;
    int active_ = 0, done_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
};

Pool& pool() {
    static Pool p;
    return p;
}

}  // namespace

extern "C" int ddm_rf_fit(const float* X, int32_t n, int32_t n_features, const int32_t* y_idx, int32_t n_classes,
                          const int64_t* seeds, int32_t n_trees, int32_t max_features, ddm_node* nodes,
                          int64_t nodes_cap, int32_t* roots, double* leaf_value, int64_t leaf_rows_cap,
                          int64_t* out_info) {
    if (!X || !y_idx || !seeds || !nodes || !roots || !out_info || n <= 0 || n_features <= 0 || n_classes <= 0 ||
        n_trees <= 0 || max_features <= 0 || nodes_cap < (int64_t)n_trees * (2 * (int64_t)n - 1))
        return DDM_E_ARG;
    if (int rc = check_inputs(X, n, n_features, y_idx, n_classes)) return rc;
    Builder b;
    builder_init(b, X, n, n_features, y_idx, n_classes, max_features);
    std::vector<Tree> trees(n_trees);
    bool pure = n_trees <= 255;
    for (int t = 0; t < n_trees; ++t) {
        b.build((uint32_t)seeds[t], trees[t]);
        pure = pure && tree_is_pure(trees[t], n_classes);
    }
    return pack_trees(trees.data(), n_trees, n_classes, pure, nodes, roots, leaf_value, leaf_rows_cap, out_info);
}

extern "C" int ddm_rf_fit_many(ddm_fit_job* jobs, int32_t n_jobs, int32_t n_threads) {
    if (!jobs || n_jobs < 0) return DDM_E_ARG;
    // trees persist across calls so their node vectors keep their capacity
    static std::vector<std::vector<Tree>> trees;
    static std::mutex trees_mu;
    std::lock_guard<std::mutex> trees_lock(trees_mu);
    if ((int)trees.size() < n_jobs) trees.resize(n_jobs);
    std::vector<int64_t> first(n_jobs + 1, 0);
    for (int j = 0; j < n_jobs; ++j) {
        ddm_fit_job& jb = jobs[j];
        jb.status = 0;
        jb.blob_bytes = 0;
        if (!jb.X || !jb.y_idx || !jb.seeds || !jb.nodes || !jb.roots || !jb.classes || jb.n <= 0 ||
            jb.n_features <= 0 || jb.n_classes <= 0 || jb.n_trees <= 0 || jb.max_features <= 0 ||
            jb.nodes_cap < (int64_t)jb.n_trees * (2 * (int64_t)jb.n - 1))
            jb.status = DDM_E_ARG;
        else
            jb.status = check_inputs(jb.X, jb.n, jb.n_features, jb.y_idx, jb.n_classes);
        if (!jb.status && (int)trees[j].size() < jb.n_trees) trees[j].resize(jb.n_trees);
        first[j + 1] = first[j] + (jb.status ? 0 : jb.n_trees);
    }
    // presorted feature orders, one per job, shared read-only by the tree tasks
    std::vector<std::vector<int32_t>> orders(n_jobs);
    pool().run(std::max(1, (int)n_threads), n_jobs, [&](int64_t j) {
        const ddm_fit_job& jb = jobs[j];
        if (jb.status) return;
        orders[j].assign((size_t)jb.n_features * jb.n, 0);
        Builder::presort_into(jb.X, jb.n, jb.n_features, orders[j].data());
    });
    // every (job, tree) is an independent task
    // each thread keeps one Builder, re-initialised when it moves to another job (or call)
    static std::atomic<uint64_t> calls{0};
    const uint64_t call = ++calls;
    static thread_local Builder tb;
    static thread_local uint64_t tb_call = 0;
    static thread_local int tb_job = -1;
    pool().run(std::max(1, (int)n_threads), first[n_jobs], [&](int64_t task) {
        const int j = (int)(std::upper_bound(first.begin(), first.end(), task) - first.begin()) - 1;
        const ddm_fit_job& jb = jobs[j];
        if (tb_call != call || tb_job != j) {
            builder_init(tb, jb.X, jb.n, jb.n_features, jb.y_idx, jb.n_classes, jb.max_features, orders[j].data());
            tb_call = call;
            tb_job = j;
        }
        const int t = (int)(task - first[j]);
        tb.build((uint32_t)jb.seeds[t], trees[j][t]);
    });
    // pack + compile each job
    pool().run(std::max(1, (int)n_threads), n_jobs, [&](int64_t j) {
        ddm_fit_job& jb = jobs[j];
        if (jb.status) return;
        bool pure = jb.n_trees <= 255;
        for (int t = 0; t < jb.n_trees; ++t) pure = pure && tree_is_pure(trees[j][t], jb.n_classes);
        jb.status = pack_trees(trees[j].data(), jb.n_trees, jb.n_classes, pure, jb.nodes, jb.roots, jb.leaf_value,
                               jb.leaf_rows_cap, jb.info);
        if (jb.status || !jb.blob) return;
        int64_t bytes = 0;
        const int rc = ddm_forest_compile(jb.nodes, (int32_t)jb.info[0], jb.roots, jb.n_trees, jb.classes,
                                          jb.n_classes, (int32_t)jb.info[1], jb.blob, jb.blob_cap, &bytes);
        if (rc == 0) {
            jb.blob_bytes = bytes;
            const ddm_cforest_head* h = reinterpret_cast<const ddm_cforest_head*>(jb.blob);
            jb.cf_slots = h->n_slots;
            jb.cf_vote_regs = h->vote_regs;
            jb.cf_leaves = h->n_leaves;
            jb.cf_tab_words = h->rank_tab_entries * h->vote_regs;
        }
    });
    for (int j = 0; j < n_jobs; ++j)
        if (jobs[j].status) return jobs[j].status;
    return 0;
}
