// Forest predict + error flag: predict_rf (DDM_Process.py:110-128).
//
// sklearn semantics reproduced (1.7.2, ensemble/_forest.py:903-962, tree/_tree.pyx):
//   * X cast to float32; node test (double)x <= threshold (f64); NaN -> missing_go_to_left
//   * per tree the leaf's class-fraction row; forest sums rows in tree order, divides
//     by n_trees, argmax takes the first maximum, label = classes_[argmax]
//   * error = label != y   (DDM_Process.py:117)
// Pure forests (every leaf one-hot, the normal case for fully grown trees) vote with
// u8 counters packed four to a register: the sum of one-hot rows is an exact integer
// count and dividing distinct integers <= 255 by n_trees keeps them distinct, so
// argmax over counts == sklearn's argmax bit for bit.  Impure forests accumulate
// the f64 leaf rows in tree order and divide by n_trees like sklearn.
//
// Not a GEMM: the work is data-dependent tree traversal, so no MFMA.  Rows are
// addressed through the batch shuffle (row = batch*per_batch + perm[g]) so the
// error vector comes out already in DDM order.  The forest (16-byte nodes) sits in
// LDS when it fits, shared by the workgroup's rows for its whole grid-stride loop.
// The first error position is reduced per wave with a ballot and one atomicMin.
#include <vector>

#include "common.h"

namespace {

constexpr int kThreads = 256;
constexpr int kMaxLdsForest = 64 * 1024;

template <bool kLdsForest>
__device__ __forceinline__ int leaf_of(const ddm_node* __restrict__ nodes, int nd, const float* __restrict__ X,
                                       int64_t ld, int64_t row) {
    for (;;) {
        const ddm_node n = nodes[nd];
        if (n.feature < 0) return n.child;
        const float xv = X[(int64_t)(n.feature & 0x3fffffff) * ld + row];
        bool left = (double)xv <= n.threshold;
        if (xv != xv) left = (n.feature >> 30) & 1;
        nd = n.child + (left ? 0 : 1);
    }
}

// One segment of predict work: DDM positions [pos_begin, pos_end) of one partition with
// its forest.  The batch entry point takes a device array of these (one per partition).
struct Seg {
    const float* X;
    int64_t ld;
    const int32_t* y;
    const uint8_t* perm;
    uint8_t* err;
    int32_t* pred;
    unsigned long long* first_err;
    int64_t pos_begin, pos_end;
    const ddm_node* nodes;
    const int32_t* roots;
    const double* leaf_value;
    const int32_t* classes;
    int32_t n_trees, n_classes, n_nodes, pure;
    int64_t row_base;            // rows are (g / per_batch) * per_batch + perm[g] - row_base
    int64_t block0, nblocks;     // this segment's blocks in the launch grid
};
static_assert(sizeof(Seg) == sizeof(ddm_predict_segment) && sizeof(Seg) == 144, "Seg must mirror ddm_predict_segment");

template <bool kPure, int kK, bool kLdsForest>
__device__ __forceinline__ void predict_segment(const Seg& sg, int64_t blk, int64_t nblk, int64_t per_batch,
                                                unsigned char* smem) {
    const ddm_node* nodes = sg.nodes;
    const int32_t* roots = sg.roots;
    const float* __restrict__ X = sg.X;
    const int64_t ld = sg.ld;
    const int n_trees = sg.n_trees, n_classes = sg.n_classes;
    if constexpr (kLdsForest) {
        uint4* dst = reinterpret_cast<uint4*>(smem);
        const uint4* src = reinterpret_cast<const uint4*>(sg.nodes);
        for (int k = threadIdx.x; k < sg.n_nodes; k += kThreads) dst[k] = src[k];
        int32_t* r = reinterpret_cast<int32_t*>(smem + (size_t)sg.n_nodes * sizeof(ddm_node));
        for (int k = threadIdx.x; k < n_trees; k += kThreads) r[k] = sg.roots[k];
        __syncthreads();
        nodes = reinterpret_cast<const ddm_node*>(smem);
        roots = r;
    }
    const int lane = threadIdx.x & 63;
    const int64_t stride = nblk * kThreads;
    for (int64_t base = sg.pos_begin + blk * kThreads + (threadIdx.x & ~63); base < sg.pos_end; base += stride) {
        const int64_t g = base + lane;
        const bool valid = g < sg.pos_end;
        int e = 0;
        if (valid) {
            const int64_t row = (g / per_batch) * per_batch + sg.perm[g] - sg.row_base;
            int best_k = 0;
            if constexpr (kPure) {
                constexpr int kRegs = (kK + 3) / 4;
                uint32_t votes[kRegs];
#pragma unroll
                for (int r = 0; r < kRegs; ++r) votes[r] = 0;
                for (int t = 0; t < n_trees; ++t) {
                    const int c = leaf_of<kLdsForest>(nodes, roots[t], X, ld, row);
                    const uint32_t inc = 1u << ((c & 3) << 3);
#pragma unroll
                    for (int r = 0; r < kRegs; ++r) votes[r] += ((c >> 2) == r) ? inc : 0u;
                }
                int best = -1;
#pragma unroll
                for (int k = 0; k < 4 * kRegs; ++k) {
                    const int v = (int)((votes[k >> 2] >> ((k & 3) << 3)) & 0xffu);
                    if (k < n_classes && v > best) {
                        best = v;
                        best_k = k;
                    }
                }
            } else {
                double acc[kK];
#pragma unroll
                for (int k = 0; k < kK; ++k) acc[k] = 0.0;
                for (int t = 0; t < n_trees; ++t) {
                    const int lr = leaf_of<kLdsForest>(nodes, roots[t], X, ld, row);
                    const double* lv = sg.leaf_value + (int64_t)lr * n_classes;
#pragma unroll
                    for (int k = 0; k < kK; ++k)
                        if (k < n_classes) acc[k] += lv[k];
                }
                const double nt = (double)n_trees;
                double best = -1.0;
#pragma unroll
                for (int k = 0; k < kK; ++k) {
                    const double v = acc[k] / nt;
                    if (k < n_classes && v > best) {
                        best = v;
                        best_k = k;
                    }
                }
            }
            const int32_t label = sg.classes[best_k];
            e = label != sg.y[row];
            sg.err[g] = (uint8_t)e;
            if (sg.pred) sg.pred[g] = label;
        }
        if (sg.first_err) {
            const unsigned long long m = __ballot(e);
            if (m && lane == __ffsll((long long)m) - 1) atomicMin(sg.first_err, (unsigned long long)g);
        }
    }
}

template <bool kPure, int kK, bool kLdsForest>
__global__ __launch_bounds__(kThreads) void k_forest_predict(Seg sg, int64_t per_batch) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    predict_segment<kPure, kK, kLdsForest>(sg, blockIdx.x, gridDim.x, per_batch, smem);
}

// Batched: every block finds its segment (one per partition) and works on it.  Segments
// are ordered by their global block range; this launch covers blocks [block_base, ...).
template <bool kPure, int kK, bool kLdsForest>
__global__ __launch_bounds__(kThreads) void k_forest_predict_batch(const Seg* __restrict__ segs, int n_segs,
                                                                   int64_t block_base, int64_t per_batch) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int64_t gb = block_base + blockIdx.x;
    int s = 0;
    while (s < n_segs && !(segs[s].block0 <= gb && gb < segs[s].block0 + segs[s].nblocks)) ++s;
    if (s == n_segs) return;
    const Seg sg = segs[s];
    predict_segment<kPure, kK, kLdsForest>(sg, gb - sg.block0, sg.nblocks, per_batch, smem);
}

using predict_fn = void (*)(Seg, int64_t);
using predict_batch_fn = void (*)(const Seg*, int, int64_t, int64_t);

template <bool kLds>
predict_fn pick(bool pure, int k) {
    if (pure) {
        if (k <= 4) return k_forest_predict<true, 4, kLds>;
        if (k <= 8) return k_forest_predict<true, 8, kLds>;
        if (k <= 16) return k_forest_predict<true, 16, kLds>;
        return k_forest_predict<true, 64, kLds>;
    }
    if (k <= 4) return k_forest_predict<false, 4, kLds>;
    if (k <= 16) return k_forest_predict<false, 16, kLds>;
    return k_forest_predict<false, 64, kLds>;
}

template <bool kLds>
predict_batch_fn pick_batch(bool pure, int k) {
    if (pure) {
        if (k <= 4) return k_forest_predict_batch<true, 4, kLds>;
        if (k <= 8) return k_forest_predict_batch<true, 8, kLds>;
        if (k <= 16) return k_forest_predict_batch<true, 16, kLds>;
        return k_forest_predict_batch<true, 64, kLds>;
    }
    if (k <= 4) return k_forest_predict_batch<false, 4, kLds>;
    if (k <= 16) return k_forest_predict_batch<false, 16, kLds>;
    return k_forest_predict_batch<false, 64, kLds>;
}

size_t forest_lds_bytes(int n_nodes, int n_trees) {
    return ((size_t)n_nodes * sizeof(ddm_node) + (size_t)n_trees * 4 + 15) & ~(size_t)15;
}

}  // namespace

extern "C" int ddm_forest_predict(const float* X, int64_t ld, int32_t n_features, const int32_t* y,
                                  const uint8_t* perm, int64_t pos_begin, int64_t pos_end, int32_t per_batch,
                                  const ddm_forest* forest, uint8_t* err_out, uint64_t* first_err,
                                  int32_t* pred_out, ddm_stream_t stream, ddm_event_t ev_begin,
                                  ddm_event_t ev_end) {
    if (!X || !y || !perm || !forest || !err_out || !forest->nodes || !forest->roots || !forest->classes ||
        per_batch <= 0 || per_batch > 256 || pos_begin < 0 || pos_end < pos_begin || n_features <= 0 ||
        ld <= 0 || forest->n_trees <= 0 || forest->n_nodes <= 0 || forest->n_classes <= 0) {
        ddm::set_error("ddm_forest_predict: invalid argument");
        return DDM_E_ARG;
    }
    if (forest->n_classes > 64 || (forest->pure && forest->n_trees > 255) || (!forest->pure && !forest->leaf_value)) {
        ddm::set_error("ddm_forest_predict: unsupported forest (classes=%d trees=%d pure=%d)", forest->n_classes,
                       forest->n_trees, forest->pure);
        return DDM_E_FOREST;
    }
    hipStream_t s = ddm::as_hip(stream);
    if (first_err) {
        if (int rc = ddm::hip_status(hipMemsetAsync(first_err, 0xff, sizeof(uint64_t), s), "ddm_forest_predict"))
            return rc;
    }
    const int64_t n = pos_end - pos_begin;
    if (n == 0) return 0;
    const size_t lds = forest_lds_bytes(forest->n_nodes, forest->n_trees);
    const bool use_lds = lds <= (size_t)kMaxLdsForest;
    const predict_fn fn = use_lds ? pick<true>(forest->pure, forest->n_classes)
                                  : pick<false>(forest->pure, forest->n_classes);
    const int64_t blocks = std::min<int64_t>(ddm::ceil_div(n, kThreads), 256 * 8);
    Seg sg{X, ld, y, perm, err_out, pred_out, reinterpret_cast<unsigned long long*>(first_err), pos_begin, pos_end,
           forest->nodes, forest->roots, forest->leaf_value, forest->classes, forest->n_trees, forest->n_classes,
           forest->n_nodes, forest->pure, 0, 0, blocks};
    if (ev_begin)
        if (int rc = ddm::hip_status(hipEventRecord(reinterpret_cast<hipEvent_t>(ev_begin), s), "event record")) return rc;
    hipLaunchKernelGGL(fn, dim3((unsigned)blocks), dim3(kThreads), use_lds ? lds : 0, s, sg, (int64_t)per_batch);
    if (ev_end)
        if (int rc = ddm::hip_status(hipEventRecord(reinterpret_cast<hipEvent_t>(ev_end), s), "event record")) return rc;
    return ddm::launch_status("ddm_forest_predict");
}

static_assert(sizeof(Seg) == sizeof(ddm_predict_segment), "ddm_predict_segment layout");

extern "C" int ddm_forest_predict_batch(const ddm_predict_segment* segs_host, ddm_predict_segment* segs_dev,
                                        int32_t n_segs, int32_t per_batch, ddm_stream_t stream, ddm_event_t ev_begin,
                                        ddm_event_t ev_end) {
    if (!segs_host || !segs_dev || n_segs <= 0 || per_batch <= 0 || per_batch > 256) {
        ddm::set_error("ddm_forest_predict_batch: invalid argument");
        return DDM_E_ARG;
    }
    hipStream_t s = ddm::as_hip(stream);
    // One launch per kernel variant (pure/impure x classes x LDS-resident forest); every
    // launch walks the whole device table and only the blocks assigned to its segments
    // work.  Block counts are proportional to rows, 2048 blocks in total per variant.
    Seg* hs = reinterpret_cast<Seg*>(const_cast<ddm_predict_segment*>(segs_host));
    for (int i = 0; i < n_segs; ++i) {
        const Seg& g = hs[i];
        if (!g.X || !g.y || !g.perm || !g.err || !g.nodes || !g.roots || !g.classes || g.pos_end < g.pos_begin ||
            g.n_classes <= 0 || g.n_classes > 64 || g.n_trees <= 0 || (g.pure && g.n_trees > 255) ||
            (!g.pure && !g.leaf_value)) {
            ddm::set_error("ddm_forest_predict_batch: invalid segment %d", i);
            return DDM_E_ARG;
        }
        if (g.first_err)
            if (int rc = ddm::hip_status(hipMemsetAsync(g.first_err, 0xff, sizeof(uint64_t), s), "predict_batch memset"))
                return rc;
    }
    if (ev_begin)
        if (int rc = ddm::hip_status(hipEventRecord(reinterpret_cast<hipEvent_t>(ev_begin), s), "event record")) return rc;
    // Variants (pure/impure x classes x LDS-resident forest) get disjoint global block
    // ranges, so ONE copy of the table serves one launch per variant present.
    std::vector<int> variant(n_segs);
    for (int i = 0; i < n_segs; ++i) {
        const Seg& g = hs[i];
        const bool lds = forest_lds_bytes(g.n_nodes, g.n_trees) <= (size_t)kMaxLdsForest;
        const int kc = g.n_classes <= 4 ? 0 : g.n_classes <= 8 ? 1 : g.n_classes <= 16 ? 2 : 3;
        variant[i] = (g.pure ? 1 : 0) * 8 + (lds ? 4 : 0) + kc;
    }
    int64_t vbase[17] = {0};
    size_t vlds[16] = {0};
    int64_t b0 = 0;
    for (int v = 0; v < 16; ++v) {
        vbase[v] = b0;
        int64_t rows = 0;
        for (int i = 0; i < n_segs; ++i)
            if (variant[i] == v) {
                rows += hs[i].pos_end - hs[i].pos_begin;
                vlds[v] = std::max(vlds[v], forest_lds_bytes(hs[i].n_nodes, hs[i].n_trees));
            }
        const int64_t total_blocks = rows ? std::min<int64_t>(ddm::ceil_div(rows, kThreads), 256 * 8) : 0;
        for (int i = 0; i < n_segs; ++i) {
            if (variant[i] != v) continue;
            Seg& g = hs[i];
            const int64_t r = g.pos_end - g.pos_begin;
            g.block0 = b0;
            g.nblocks = r == 0 ? 0 : std::max<int64_t>(1, (total_blocks * r + rows - 1) / rows);
            b0 += g.nblocks;
        }
    }
    vbase[16] = b0;
    if (b0 > 0) {
        if (int rc = ddm::hip_status(hipMemcpyAsync(segs_dev, hs, sizeof(Seg) * n_segs, hipMemcpyHostToDevice, s),
                                     "predict_batch table"))
            return rc;
    }
    for (int v = 0; v < 16; ++v) {
        const int64_t nb = vbase[v + 1] - vbase[v];
        if (nb == 0) continue;
        const bool lds = (v & 4) != 0;
        const bool pure = (v & 8) != 0;
        const int kmax = (v & 3) == 0 ? 4 : (v & 3) == 1 ? 8 : (v & 3) == 2 ? 16 : 64;
        const predict_batch_fn fn = lds ? pick_batch<true>(pure, kmax) : pick_batch<false>(pure, kmax);
        hipLaunchKernelGGL(fn, dim3((unsigned)nb), dim3(kThreads), lds ? vlds[v] : 0, s,
                           reinterpret_cast<const Seg*>(segs_dev), n_segs, vbase[v],
                           (int64_t)per_batch);
        if (int rc = ddm::launch_status("ddm_forest_predict_batch")) return rc;
    }
    if (ev_end)
        if (int rc = ddm::hip_status(hipEventRecord(reinterpret_cast<hipEvent_t>(ev_end), s), "event record")) return rc;
    return 0;
}
