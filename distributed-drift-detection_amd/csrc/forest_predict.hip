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

template <bool kPure, int kK, bool kLdsForest>
__global__ __launch_bounds__(kThreads) void k_forest_predict(
    const float* __restrict__ X, int64_t ld, const int32_t* __restrict__ y, const uint8_t* __restrict__ perm,
    int64_t pos_begin, int64_t pos_end, int64_t per_batch, const ddm_node* __restrict__ g_nodes,
    const int32_t* __restrict__ g_roots, const double* __restrict__ leaf_value, const int32_t* __restrict__ classes,
    int n_trees, int n_classes, int n_nodes, uint8_t* __restrict__ err_out, unsigned long long* __restrict__ first_err,
    int32_t* __restrict__ pred_out) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const ddm_node* nodes = g_nodes;
    const int32_t* roots = g_roots;
    if constexpr (kLdsForest) {
        uint4* dst = reinterpret_cast<uint4*>(smem);
        const uint4* src = reinterpret_cast<const uint4*>(g_nodes);
        for (int k = threadIdx.x; k < n_nodes; k += kThreads) dst[k] = src[k];
        int32_t* r = reinterpret_cast<int32_t*>(smem + (size_t)n_nodes * sizeof(ddm_node));
        for (int k = threadIdx.x; k < n_trees; k += kThreads) r[k] = g_roots[k];
        __syncthreads();
        nodes = reinterpret_cast<const ddm_node*>(smem);
        roots = r;
    }
    const int lane = threadIdx.x & 63;
    const int64_t stride = (int64_t)gridDim.x * kThreads;
    for (int64_t base = pos_begin + (int64_t)blockIdx.x * kThreads + (threadIdx.x & ~63); base < pos_end;
         base += stride) {
        const int64_t g = base + lane;
        const bool valid = g < pos_end;
        int e = 0;
        if (valid) {
            const int64_t row = (g / per_batch) * per_batch + perm[g];
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
                    const double* lv = leaf_value + (int64_t)lr * n_classes;
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
            const int32_t label = classes[best_k];
            e = label != y[row];
            err_out[g] = (uint8_t)e;
            if (pred_out) pred_out[g] = label;
        }
        if (first_err) {
            const unsigned long long m = __ballot(e);
            if (m && lane == __ffsll((long long)m) - 1) atomicMin(first_err, (unsigned long long)g);
        }
    }
}

using predict_fn = void (*)(const float*, int64_t, const int32_t*, const uint8_t*, int64_t, int64_t, int64_t,
                            const ddm_node*, const int32_t*, const double*, const int32_t*, int, int, int, uint8_t*,
                            unsigned long long*, int32_t*);

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
    const size_t lds = ((size_t)forest->n_nodes * sizeof(ddm_node) + (size_t)forest->n_trees * 4 + 15) & ~(size_t)15;
    const bool use_lds = lds <= (size_t)kMaxLdsForest;
    const predict_fn fn = use_lds ? pick<true>(forest->pure, forest->n_classes)
                                  : pick<false>(forest->pure, forest->n_classes);
    const int64_t blocks = std::min<int64_t>(ddm::ceil_div(n, kThreads), 256 * 8);
    if (ev_begin)
        if (int rc = ddm::hip_status(hipEventRecord(reinterpret_cast<hipEvent_t>(ev_begin), s), "event record")) return rc;
    hipLaunchKernelGGL(fn, dim3((unsigned)blocks), dim3(kThreads), use_lds ? lds : 0, s, X, ld, y, perm, pos_begin,
                       pos_end, (int64_t)per_batch, forest->nodes, forest->roots, forest->leaf_value,
                       forest->classes, forest->n_trees, forest->n_classes, forest->n_nodes, err_out,
                       reinterpret_cast<unsigned long long*>(first_err), pred_out);
    if (ev_end)
        if (int rc = ddm::hip_status(hipEventRecord(reinterpret_cast<hipEvent_t>(ev_end), s), "event record")) return rc;
    return ddm::launch_status("ddm_forest_predict");
}
