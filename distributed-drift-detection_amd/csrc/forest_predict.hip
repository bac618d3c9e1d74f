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
// The first error position is reduced per wave with a ballot; a wave's positions only
// grow along its grid-stride loop, so it issues at most one atomicMin (and none when the
// global minimum is already smaller): hot single-address atomics would otherwise
// serialise every wave that sees an error.
#include <type_traits>
#include <vector>

#include "common.h"

namespace {

constexpr int kThreads = 256;
constexpr int kMaxLdsForest = 64 * 1024;

// first_err reduction: at most one atomicMin per wave (see the file comment).
__device__ __forceinline__ void note_first_error(ddm::gptr<unsigned long long> first_err, int e, int64_t g, int lane,
                                                 bool& wave_done) {
    const unsigned long long m = __ballot(e);
    if (m && !wave_done) {
        wave_done = true;
        if (lane == __ffsll((long long)m) - 1 &&
            (unsigned long long)g < __hip_atomic_load(first_err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
            __hip_atomic_fetch_min(first_err, (unsigned long long)g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

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
// The row / position pointers as the global address space: their loads and stores are
// global_* instructions, not flat_* (a flat load also counts on lgkmcnt, so every LDS wait
// of the row phase -- rank tables, labels -- would wait for the next rows' prefetched labels)
using ddm::gptr;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
using ddm::ld_int4;
struct Seg {
    const float* X;
    int64_t ld;
    gptr<const int32_t> y;
    gptr<const uint8_t> perm;
    gptr<uint8_t> err;
    gptr<int32_t> pred;
    gptr<unsigned long long> first_err;
    int64_t pos_begin, pos_end;
    const ddm_node* nodes;
    const int32_t* roots;
    const double* leaf_value;
    const int32_t* classes;
    int32_t n_trees, n_classes, n_nodes, pure;
    int64_t row_base;            // rows are (g / per_batch) * per_batch + perm[g] - row_base
    int64_t block0, nblocks;     // this segment's blocks in the launch grid
    const uint8_t* cforest;      // compiled forest or NULL
    int32_t cf_slots, cf_vote_regs, cf_leaves, flags;
    int32_t cf_tab_words, pad;
};
static_assert(sizeof(Seg) == sizeof(ddm_predict_segment) && sizeof(Seg) == 176, "Seg must mirror ddm_predict_segment");

// Internal segment flag (device-resident epochs, ddm_forest_predict_dev_orig): err is written
// in ROW order (position g gets the error of row g - row_base, no perm read; first_err notes
// the first error row) and ddm_err_permute_dev puts the bytes into DDM order once the
// window's shuffles are done.  The predict then needs the forest only, not the shuffle.
constexpr int32_t kSegRowOrder = 1 << 8;

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
    bool wave_done = false;
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
        if (sg.first_err) note_first_error(sg.first_err, e, g, lane, wave_done);
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

// ---------------------------------------------------------------------------------
// Compiled-forest path (ddm_forest_compile, csrc/forest_compile.cpp).
//
// A workgroup of 512 threads owns a tile of whole batches (tile = floor(512/pb)*pb
// positions, so a tile's DDM positions and its rows are the same set):
//   1. row phase: thread t owns ROW g0+t of the tile.  It loads only the forest's
//      feature columns (slot s <- X[cols[s]*ld + row], 4-byte coalesced loads), runs the
//      compiled forest out of registers (node data arrive through uniform/scalar loads)
//      and keeps err/label in LDS at t;
//   2. position phase: thread t owns DDM POSITION g0+t and picks the error of row
//      tb + perm[g] from LDS, so err (and pred) are written in DDM order, coalesced.
// Bytes per row from HBM: 4*n_slots (X) + 4 (y) + 1 (perm) + 1 (err).
constexpr int kCfThreads = 512;

// Uniform loads: the blob and the segment table are read-only for the kernel's lifetime,
// so they are read through the constant address space (scalar s_load into SGPRs).
#define DDM_CONST __attribute__((address_space(4)))
template <class T>
__device__ __forceinline__ T ldu(const T* p) {
    if constexpr (std::is_arithmetic<T>::value) {
        return *(const DDM_CONST T*)(p);
    } else {
        static_assert(sizeof(T) % 4 == 0, "records are dword multiples");
        T out;
        uint32_t* o = reinterpret_cast<uint32_t*>(&out);
        const DDM_CONST uint32_t* q = (const DDM_CONST uint32_t*)(p);
#pragma unroll
        for (int i = 0; i < (int)(sizeof(T) / 4); ++i) o[i] = q[i];
        return out;
    }
}

// Feature columns are read through pointers kept in LDS, i.e. generic (flat) pointers: a
// flat load also counts on lgkmcnt, so the next chunk's prefetch would be waited for by the
// first scalar load of the slot records.  As global loads they count on vmcnt only.
__device__ __forceinline__ float ldg1(const float* p) { return *(const __attribute__((address_space(1))) float*)(p); }
__device__ __forceinline__ float4 ldg4(const float* p) {
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    const f32x4 v = *(const __attribute__((address_space(1))) f32x4*)(p);
    return make_float4(v.x, v.y, v.z, v.w);
}

// Stumps are evaluated per feature slot through the blob's rank tables
// (ddm_cforest_slot): r = #{k : !(x <= t_k)} over the slot's padded ascending thresholds
// (2 VALU per threshold against uniform operands; NaN counts every entry), then one LDS
// read of the table entry and vote_regs adds, instead of a compare and masked adds per
// stump.
__device__ __forceinline__ int rank4(const float x, const float* t) {
    return (!(x <= t[0]) ? 1 : 0) + (!(x <= t[1]) ? 1 : 0) + (!(x <= t[2]) ? 1 : 0) + (!(x <= t[3]) ? 1 : 0);
}

template <int kVR>
__device__ __forceinline__ void add_votes(const uint32_t* e, uint32_t (&votes)[kVR]) {
    if constexpr (kVR == 4) {
        const uint4 d = *reinterpret_cast<const uint4*>(e);
        votes[0] += d.x;
        votes[1] += d.y;
        votes[2] += d.z;
        votes[3] += d.w;
    } else if constexpr (kVR == 2) {
        const uint2 d = *reinterpret_cast<const uint2*>(e);
        votes[0] += d.x;
        votes[1] += d.y;
    } else {
        votes[0] += e[0];
    }
}

// A thread evaluates kRows rows (2 for stump forests: one in each half of a double
// tile; 1 with general trees, whose LDS row columns grow with kRows), so every
// scalar instruction of the slot walk (records, thresholds, loop control: the scalar
// unit is shared by the CU's four SIMDs) serves 128 rows of a wave.  Feature values are
// loaded 8 slots at a time, one chunk ahead of the chunk being evaluated (and the next
// double tile's first chunk during the current one's last), so a row's loads stay in
// flight behind the compares.  Column pointers X + col*ld come from LDS (no 64-bit
// scalar multiplies per load).
constexpr int kChunk = 8;

template <int kVR, int kRows>
__device__ __forceinline__ void cf_segment(const Seg& sg, int64_t blk, int64_t nblk, int pb, unsigned char* smem) {
    const uint8_t* blob = sg.cforest;
    const ddm_cforest_head* H = reinterpret_cast<const ddm_cforest_head*>(blob);
    const int U = ldu(&H->n_slots), K = ldu(&H->n_classes), n_general = ldu(&H->n_general);
    const int n_leaves = ldu(&H->n_leaves);
    const int tab_words = ldu(&H->rank_tab_entries) * kVR;
    const ddm_cforest_slot* slots = reinterpret_cast<const ddm_cforest_slot*>(blob + ldu(&H->slots_off));
    const float4* xthr = reinterpret_cast<const float4*>(blob + ldu(&H->xthr_off));
    const ddm_cforest_tree* trees = reinterpret_cast<const ddm_cforest_tree*>(blob + ldu(&H->trees_off));
    const ddm_cforest_node* gnodes = reinterpret_cast<const ddm_cforest_node*>(blob + ldu(&H->nodes_off));
    const uint8_t* leafcls = blob + ldu(&H->leafcls_off);
    const int U8 = (U + kChunk - 1) & ~(kChunk - 1);

    const int tid = threadIdx.x;
    // LDS (cf_lds_bytes): column pointers [32] | rank tables | labels [2][512] |
    // classes [16] | err [2][512] | leaf classes | row slots [kRows][U8][512] (only with
    // general trees, which index x by a node's slot at run time)
    const float** s_colp = reinterpret_cast<const float**>(smem);
    uint32_t* s_tab = reinterpret_cast<uint32_t*>(s_colp + 32);
    int32_t* s_pred = reinterpret_cast<int32_t*>(s_tab + ((tab_words + 3) & ~3));
    int32_t* s_cls = s_pred + kRows * kCfThreads;
    uint8_t* s_e = reinterpret_cast<uint8_t*>(s_cls + 16);
    uint8_t* s_leaf = s_e + kRows * kCfThreads;
    float* s_x = reinterpret_cast<float*>(s_leaf + ((n_leaves + 15) & ~15));
    {
        gptr<const uint32_t> gt = (gptr<const uint32_t>)(blob + ldu(&H->rank_tab_off));
        for (int k = tid; k < tab_words; k += kCfThreads) s_tab[k] = gt[k];
    }
    for (int k = tid; k < n_leaves; k += kCfThreads) s_leaf[k] = ((gptr<const uint8_t>)leafcls)[k];
    if (tid < 16) s_cls[tid] = ((gptr<const int32_t>)H->classes)[tid];
    if (tid < 32) s_colp[tid] = sg.X + (int64_t)H->cols[tid] * sg.ld;
    uint32_t base_votes[kVR];
#pragma unroll
    for (int j = 0; j < kVR; ++j) base_votes[j] = ldu(&H->base_votes[j]);

    const int tile = (kCfThreads / pb) * pb;
    const int tb = (tid / pb) * pb;
    const int lane = tid & 63;
    bool wave_done = false;
    const int64_t step = nblk * kRows * tile;
    // every lane runs the row phase, on a clamped row, so the forest loops stay
    // wave-uniform and their records stay in SGPRs
    auto row_of = [&](int64_t gt0) -> int64_t {
        const int64_t gg = gt0 + tid;
        return ((tid < tile && gg < sg.pos_end) ? gg : min(gt0, sg.pos_end - 1)) - sg.row_base;
    };
    auto load_chunk = [&](int c, const int64_t (&row)[kRows], float (&xc)[kRows][kChunk]) {
        const float* p[kChunk];
#pragma unroll
        for (int k = 0; k < kChunk; ++k) p[k] = s_colp[c + k];
#pragma unroll
        for (int i = 0; i < kRows; ++i)
#pragma unroll
            for (int k = 0; k < kChunk; ++k) xc[i][k] = ldg1(p[k] + row[i]);
    };
    float xa[kRows][kChunk], xb[kRows][kChunk];
#pragma unroll
    for (int i = 0; i < kRows; ++i)
#pragma unroll
        for (int k = 0; k < kChunk; ++k) xa[i][k] = xb[i][k] = 0.f;
    int32_t ynext[kRows];
#pragma unroll
    for (int i = 0; i < kRows; ++i) ynext[i] = 0;
    int64_t g0 = sg.pos_begin + blk * kRows * tile;
    __syncthreads();                            // column pointers, tables
    if (g0 < sg.pos_end) {
        int64_t row[kRows];
#pragma unroll
        for (int i = 0; i < kRows; ++i) row[i] = row_of(g0 + i * tile);
        if (U > 0) load_chunk(0, row, xa);
#pragma unroll
        for (int i = 0; i < kRows; ++i) ynext[i] = sg.y[row[i]];
    }
    for (; g0 < sg.pos_end; g0 += step) {
        int64_t row[kRows], nrow[kRows];
        const bool has_next = g0 + step < sg.pos_end;
#pragma unroll
        for (int i = 0; i < kRows; ++i) {
            row[i] = row_of(g0 + i * tile);
            nrow[i] = has_next ? row_of(g0 + step + i * tile) : row[i];
        }
        int32_t yv[kRows];
#pragma unroll
        for (int i = 0; i < kRows; ++i) {
            yv[i] = ynext[i];
            if (has_next) ynext[i] = sg.y[nrow[i]];
        }
        uint32_t votes[kRows][kVR];
#pragma unroll
        for (int i = 0; i < kRows; ++i)
#pragma unroll
            for (int j = 0; j < kVR; ++j) votes[i][j] = base_votes[j];
        // ---- row phase.  Each thread only reads the LDS columns it wrote itself, so no
        // barrier is needed before the general trees.
        for (int c = 0; c < U; c += kChunk) {
            if (c + kChunk < U) load_chunk(c + kChunk, row, xb);
            else if (has_next) load_chunk(0, nrow, xb);
            const ddm_cforest_slot* sc = slots + c;
#pragma unroll
            for (int k = 0; k < kChunk; ++k) {
                if (n_leaves > 0) {
#pragma unroll
                    for (int i = 0; i < kRows; ++i) s_x[((i * U8) + c + k) * kCfThreads + tid] = xa[i][k];
                }
                const int n4 = ldu(&sc[k].n4);
                if (n4 > 0) {
                    const float4 t0 = ldu(reinterpret_cast<const float4*>(sc[k].thr));
                    const float tt0[4] = {t0.x, t0.y, t0.z, t0.w};
                    int r[kRows];
#pragma unroll
                    for (int i = 0; i < kRows; ++i) r[i] = rank4(xa[i][k], tt0);
                    if (n4 > 1) {
                        const float4* xt = xthr + ldu(&sc[k].xthr);
                        for (int q = 0; q < n4 - 1; ++q) {
                            const float4 t = ldu(xt + q);
                            const float tt[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
                            for (int i = 0; i < kRows; ++i) r[i] += rank4(xa[i][k], tt);
                        }
                    }
                    const uint32_t* tab = s_tab + ldu(&sc[k].tab) * kVR;
#pragma unroll
                    for (int i = 0; i < kRows; ++i) add_votes<kVR>(tab + r[i] * kVR, votes[i]);
                }
            }
#pragma unroll
            for (int i = 0; i < kRows; ++i)
#pragma unroll
                for (int k = 0; k < kChunk; ++k) xa[i][k] = xb[i][k];
        }
#pragma unroll
        for (int i = 0; i < kRows; ++i) {
            // deeper trees: QuickScorer exit-leaf masks
            const float* xl = s_x + (size_t)i * U8 * kCfThreads + tid;
            for (int t = 0; t < n_general; ++t) {
                const ddm_cforest_tree T = ldu(trees + t);
                uint32_t mlo = 0xffffffffu, mhi = 0xffffffffu;
                for (int k = T.node_begin; k < T.node_begin + T.n_nodes; ++k) {
                    const ddm_cforest_node nd = ldu(gnodes + k);
                    const float v = xl[(nd.slot_nanleft & 0xff) * kCfThreads];
                    const bool right = (nd.slot_nanleft >> 8) ? (v > nd.threshold) : !(v <= nd.threshold);
                    mlo = right ? (mlo & ~nd.left_lo) : mlo;
                    mhi = right ? (mhi & ~nd.left_hi) : mhi;
                }
                const int leaf = mlo ? __builtin_ctz(mlo) : 32 + __builtin_ctz(mhi);
                const int c = s_leaf[T.leaf_begin + leaf];
                const uint32_t inc = 1u << (8 * (c & 3));
#pragma unroll
                for (int j = 0; j < kVR; ++j) votes[i][j] += (c >> 2) == j ? inc : 0u;
            }
            // first argmax over the vote counters
            int best = 0, bestv = -1;
#pragma unroll
            for (int c = 0; c < 4 * kVR; ++c) {
                const int v = (int)((votes[i][c >> 2] >> (8 * (c & 3))) & 0xffu);
                const bool better = c < K && v > bestv;
                bestv = better ? v : bestv;
                best = better ? c : best;
            }
            const int32_t label = s_cls[best];
            if (tid < tile) {
                s_e[i * kCfThreads + tid] = (uint8_t)(label != yv[i]);
                if (sg.pred) s_pred[i * kCfThreads + tid] = label;
            }
        }
        __syncthreads();
        // ---- position phase
#pragma unroll
        for (int i = 0; i < kRows; ++i) {
            const int64_t g = g0 + i * tile + tid;
            int e = 0;
            if (tid < tile && g < sg.pos_end) {
                const int k = i * kCfThreads + ((sg.flags & kSegRowOrder) ? tid : tb + (int)sg.perm[g]);
                e = s_e[k];
                sg.err[g] = (uint8_t)e;
                if (sg.pred) sg.pred[g] = s_pred[k];
            }
            if (sg.first_err) note_first_error(sg.first_err, e, g, lane, wave_done);
        }
        __syncthreads();                        // s_e / s_pred / s_x consumed
    }
}

// Stump forests with per_batch % 4 == 0: a thread owns FOUR consecutive rows and reads
// each feature slot of them with one 16-byte load (a wave: 1 KiB contiguous per slot),
// labels with one 16-byte load, and in the position phase four DDM positions (one
// 4-byte perm load, one 4-byte err store).  A tile is floor(2048 / pb) * pb rows; the
// next tile's first slot chunk and labels are loaded during the current tile.  Rows of a
// partition start 16-byte aligned (ld % 64 == 0, windows start on batches of a multiple
// of 4 rows) and ld covers every row a clamped lane may read.
constexpr int kVecRows = 4;
constexpr int kVecChunk = 4;     // slots per load chunk (8 held 166 VGPRs: 3 waves per SIMD)

template <int kVR>
__device__ __forceinline__ void cf_segment_vec(const Seg& sg, int64_t blk, int64_t nblk, int pb, unsigned char* smem) {
    const uint8_t* blob = sg.cforest;
    const ddm_cforest_head* H = reinterpret_cast<const ddm_cforest_head*>(blob);
    const int U = ldu(&H->n_slots), K = ldu(&H->n_classes);
    const int tab_words = ldu(&H->rank_tab_entries) * kVR;
    const ddm_cforest_slot* slots = reinterpret_cast<const ddm_cforest_slot*>(blob + ldu(&H->slots_off));
    const float4* xthr = reinterpret_cast<const float4*>(blob + ldu(&H->xthr_off));
    const int tid = threadIdx.x;
    // LDS (cf_lds_bytes with rows 4): column pointers [32] | rank tables | labels [2048] |
    // classes [16] | err [2048]
    const float** s_colp = reinterpret_cast<const float**>(smem);
    uint32_t* s_tab = reinterpret_cast<uint32_t*>(s_colp + 32);
    int32_t* s_pred = reinterpret_cast<int32_t*>(s_tab + ((tab_words + 3) & ~3));
    int32_t* s_cls = s_pred + kVecRows * kCfThreads;
    uint8_t* s_e = reinterpret_cast<uint8_t*>(s_cls + 16);
    {
        gptr<const uint32_t> gt = (gptr<const uint32_t>)(blob + ldu(&H->rank_tab_off));
        for (int k = tid; k < tab_words; k += kCfThreads) s_tab[k] = gt[k];
    }
    if (tid < 16) s_cls[tid] = ((gptr<const int32_t>)H->classes)[tid];
    if (tid < 32) s_colp[tid] = sg.X + (int64_t)H->cols[tid] * sg.ld;
    uint32_t base_votes[kVR];
#pragma unroll
    for (int j = 0; j < kVR; ++j) base_votes[j] = ldu(&H->base_votes[j]);

    const int tile = ((kVecRows * kCfThreads) / pb) * pb;
    const int q0 = kVecRows * tid;                  // this thread's rows / positions in the tile
    const int lane = tid & 63;
    bool wave_done = false;
    const int64_t step = nblk * tile;
    const int64_t last_row = ((sg.pos_end - 1 - sg.row_base) & ~(int64_t)3);
    auto row_of = [&](int64_t gt0) -> int64_t {    // first of the 4 rows (clamped: in bounds)
        const int64_t r = gt0 + q0 - sg.row_base;
        return (q0 < tile && r <= last_row) ? r : last_row;
    };
    auto load_chunk = [&](int c, int64_t row, float4 (&xc)[kVecChunk]) {
#pragma unroll
        for (int k = 0; k < kVecChunk; ++k) xc[k] = ldg4(s_colp[c + k] + row);
    };
    float4 xa[kVecChunk], xb[kVecChunk];
#pragma unroll
    for (int k = 0; k < kVecChunk; ++k) xa[k] = xb[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    int4 ynext = make_int4(0, 0, 0, 0);
    int64_t g0 = sg.pos_begin + blk * tile;
    __syncthreads();                                // column pointers, tables
    if (g0 < sg.pos_end) {
        const int64_t row = row_of(g0);
        if (U > 0) load_chunk(0, row, xa);
        ynext = ld_int4(sg.y + row);
    }
    for (; g0 < sg.pos_end; g0 += step) {
        const int64_t row = row_of(g0);
        const bool has_next = g0 + step < sg.pos_end;
        const int64_t nrow = has_next ? row_of(g0 + step) : row;
        const int4 yv = ynext;
        if (has_next) ynext = ld_int4(sg.y + nrow);
        uint32_t votes[kVecRows][kVR];
#pragma unroll
        for (int i = 0; i < kVecRows; ++i)
#pragma unroll
            for (int j = 0; j < kVR; ++j) votes[i][j] = base_votes[j];
        // ---- row phase
        for (int c = 0; c < U; c += kVecChunk) {
            if (c + kVecChunk < U) load_chunk(c + kVecChunk, row, xb);
            else if (has_next) load_chunk(0, nrow, xb);
            const ddm_cforest_slot* sc = slots + c;
#pragma unroll
            for (int k = 0; k < kVecChunk; ++k) {
                const int n4 = ldu(&sc[k].n4);
                if (n4 > 0) {
                    const float xv[kVecRows] = {xa[k].x, xa[k].y, xa[k].z, xa[k].w};
                    const float4 t0 = ldu(reinterpret_cast<const float4*>(sc[k].thr));
                    const float tt0[4] = {t0.x, t0.y, t0.z, t0.w};
                    int r[kVecRows];
#pragma unroll
                    for (int i = 0; i < kVecRows; ++i) r[i] = rank4(xv[i], tt0);
                    if (n4 > 1) {
                        const float4* xt = xthr + ldu(&sc[k].xthr);
                        for (int q = 0; q < n4 - 1; ++q) {
                            const float4 t = ldu(xt + q);
                            const float tt[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
                            for (int i = 0; i < kVecRows; ++i) r[i] += rank4(xv[i], tt);
                        }
                    }
                    const uint32_t* tab = s_tab + ldu(&sc[k].tab) * kVR;
#pragma unroll
                    for (int i = 0; i < kVecRows; ++i) add_votes<kVR>(tab + r[i] * kVR, votes[i]);
                }
            }
#pragma unroll
            for (int k = 0; k < kVecChunk; ++k) xa[k] = xb[k];
        }
        const int yl[kVecRows] = {yv.x, yv.y, yv.z, yv.w};
        uint32_t e4 = 0;
#pragma unroll
        for (int i = 0; i < kVecRows; ++i) {
            int best = 0, bestv = -1;               // first argmax over the vote counters
#pragma unroll
            for (int c = 0; c < 4 * kVR; ++c) {
                const int v = (int)((votes[i][c >> 2] >> (8 * (c & 3))) & 0xffu);
                const bool better = c < K && v > bestv;
                bestv = better ? v : bestv;
                best = better ? c : best;
            }
            const int32_t label = s_cls[best];
            e4 |= (uint32_t)(label != yl[i]) << (8 * i);
            if (sg.pred && q0 < tile) s_pred[q0 + i] = label;
        }
        if (q0 < tile) *reinterpret_cast<uint32_t*>(s_e + q0) = e4;
        __syncthreads();
        // ---- position phase: positions g0 + q0 .. g0 + q0 + 3
        const int64_t g = g0 + q0;
        int e_any = 0;
        int64_t g_first = g;
        if (q0 < tile && g < sg.pos_end) {
            const uint32_t p4 = (sg.flags & kSegRowOrder) ? 0x03020100u + (uint32_t)(q0 % pb) * 0x01010101u
                                                          : *(gptr<const uint32_t>)(sg.perm + g);
            uint32_t out = 0;
            int first = -1;
#pragma unroll
            for (int i = 0; i < kVecRows; ++i) {
                const int q = q0 + i;
                const int k = (q / pb) * pb + (int)((p4 >> (8 * i)) & 0xffu);
                const uint32_t e = s_e[k];
                const bool ok = g + i < sg.pos_end;
                out |= (ok ? e : 0u) << (8 * i);
                if (ok && e && first < 0) first = i;
            }
            if (g + kVecRows <= sg.pos_end) {
                *(gptr<uint32_t>)(sg.err + g) = out;
            } else {
                for (int i = 0; g + i < sg.pos_end; ++i) sg.err[g + i] = (uint8_t)((out >> (8 * i)) & 0xffu);
            }
            if (sg.pred) {
                for (int i = 0; i < kVecRows && g + i < sg.pos_end; ++i) {
                    const int q = q0 + i;
                    sg.pred[g + i] = s_pred[(q / pb) * pb + (int)((p4 >> (8 * i)) & 0xffu)];
                }
            }
            e_any = first >= 0;
            g_first = g + (first >= 0 ? first : 0);
        }
        if (sg.first_err) note_first_error(sg.first_err, e_any, g_first, lane, wave_done);
        __syncthreads();                            // s_e / s_pred consumed
    }
}

template <int kVR, int kRows>
__device__ __forceinline__ void cf_dispatch(const Seg& sg, int64_t blk, int64_t nblk, int pb, unsigned char* smem) {
    if constexpr (kRows == kVecRows) cf_segment_vec<kVR>(sg, blk, nblk, pb, smem);
    else cf_segment<kVR, kRows>(sg, blk, nblk, pb, smem);
}

template <int kVR, int kRows>
__global__ __launch_bounds__(kCfThreads) void k_cforest_predict(Seg sg, int pb) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    cf_dispatch<kVR, kRows>(sg, blockIdx.x, gridDim.x, pb, smem);
}

template <int kVR, int kRows>
__global__ __launch_bounds__(kCfThreads) void k_cforest_predict_batch(const Seg* __restrict__ segs, int n_segs,
                                                                      int64_t block_base, int pb) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int64_t gb = block_base + blockIdx.x;
    int s = 0;
    while (s < n_segs && !(ldu(&segs[s].block0) <= gb && gb < ldu(&segs[s].block0) + ldu(&segs[s].nblocks))) ++s;
    if (s == n_segs) return;
    const Seg sg = ldu(segs + s);
    cf_dispatch<kVR, kRows>(sg, gb - sg.block0, sg.nblocks, pb, smem);
}

// The same kernel with the segment table passed by value in the kernel arguments (up to
// kArgSegs segments: a C3 GPU runs 8 partitions), so an epoch's predict needs no
// host->device table copy ahead of it on the stream.  The table lives in the kernarg
// segment; the lookup and the copy of the selected segment are scalar loads.
constexpr int kArgSegs = 8;
struct SegTab {
    Seg s[kArgSegs];
};

template <int kVR, int kRows>
__global__ __launch_bounds__(kCfThreads) void k_cforest_predict_arg(const SegTab tab, int n_segs, int64_t block_base,
                                                                    int pb) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int64_t gb = block_base + blockIdx.x;
    int s = 0;
    while (s < n_segs && !(tab.s[s].block0 <= gb && gb < tab.s[s].block0 + tab.s[s].nblocks)) ++s;
    if (s == n_segs) return;
    const Seg sg = tab.s[s];
    cf_dispatch<kVR, kRows>(sg, gb - sg.block0, sg.nblocks, pb, smem);
}

using cf_fn = void (*)(Seg, int);
using cf_batch_fn = void (*)(const Seg*, int, int64_t, int);

int cf_vkind(int vr) { return vr <= 1 ? 0 : vr <= 2 ? 1 : 2; }
// rows per thread: 1 with general trees, 4 consecutive (16-byte loads) for stump forests
// whose rows and positions are 16- / 4-byte aligned, else 2
bool vec_env() {
#ifdef DDM_TUNING                                   // tuning builds only (tools/build_variant.sh)
    static const bool on = [] {
        const char* e = getenv("DDM_PREDICT_VEC");
        return e ? atoi(e) != 0 : true;
    }();
    return on;
#else
    return true;
#endif
}
int cf_rows(const Seg& g, int pb) {
    if (g.cf_leaves > 0) return 1;
    const bool aligned = pb % 4 == 0 && g.ld % 4 == 0 && g.row_base % 4 == 0 &&
                         ((reinterpret_cast<uintptr_t>(g.X) | reinterpret_cast<uintptr_t>(g.y)) & 15) == 0 &&
                         ((reinterpret_cast<uintptr_t>(g.perm) | reinterpret_cast<uintptr_t>(g.err)) & 3) == 0;
    return aligned && vec_env() ? kVecRows : 2;
}
int cf_rows_idx(int rows) { return rows == 1 ? 0 : rows == 2 ? 1 : 2; }
int cf_rows_of_idx(int i) { return i == 0 ? 1 : i == 1 ? 2 : kVecRows; }
// positions one block step covers
int cf_unit(int rows, int pb) {
    return rows == kVecRows ? ((kVecRows * kCfThreads) / pb) * pb : rows * ((kCfThreads / pb) * pb);
}
template <int kRows>
cf_fn pick_cf_r(int vk) {
    return vk == 0 ? k_cforest_predict<1, kRows> : vk == 1 ? k_cforest_predict<2, kRows> : k_cforest_predict<4, kRows>;
}
cf_fn pick_cf(int vk, int rows) {
    return rows == 1 ? pick_cf_r<1>(vk) : rows == 2 ? pick_cf_r<2>(vk) : pick_cf_r<kVecRows>(vk);
}
template <int kRows>
cf_batch_fn pick_cf_batch_r(int vk) {
    return vk == 0 ? k_cforest_predict_batch<1, kRows>
                   : vk == 1 ? k_cforest_predict_batch<2, kRows> : k_cforest_predict_batch<4, kRows>;
}
cf_batch_fn pick_cf_batch(int vk, int rows) {
    return rows == 1 ? pick_cf_batch_r<1>(vk) : rows == 2 ? pick_cf_batch_r<2>(vk) : pick_cf_batch_r<kVecRows>(vk);
}
using cf_arg_fn = void (*)(SegTab, int, int64_t, int);
template <int kRows>
cf_arg_fn pick_cf_arg_r(int vk) {
    return vk == 0 ? k_cforest_predict_arg<1, kRows>
                   : vk == 1 ? k_cforest_predict_arg<2, kRows> : k_cforest_predict_arg<4, kRows>;
}
cf_arg_fn pick_cf_arg(int vk, int rows) {
    return rows == 1 ? pick_cf_arg_r<1>(vk) : rows == 2 ? pick_cf_arg_r<2>(vk) : pick_cf_arg_r<kVecRows>(vk);
}

// LDS of the compiled path (cf_segment / cf_segment_vec): column pointers + rank tables
// + labels + classes + err + leaf classes + row slots [kRows][slots rounded to 8][512]
// when the forest has general trees (leaves > 0).
__host__ __device__ size_t cf_lds_bytes(int leaves, int slots, int tab_words, int kRows) {
    const size_t slots8 = (size_t)((slots + kChunk - 1) & ~(kChunk - 1));
    return 8 * 32 + (size_t)4 * ((tab_words + 3) & ~3) + (size_t)4 * kRows * kCfThreads + 64 +
           (size_t)kRows * kCfThreads + (size_t)((leaves + 15) & ~15) +
           (leaves > 0 ? (size_t)4 * kRows * kCfThreads * slots8 : 0);
}

size_t cf_lds_bound(const Seg& g, int pb) { return cf_lds_bytes(g.cf_leaves, g.cf_slots, g.cf_tab_words, cf_rows(g, pb)); }

bool cf_usable(const Seg& g, int pb) {
    return g.cforest && g.cf_slots >= 0 && g.cf_slots <= 32 && g.cf_vote_regs >= 1 && g.cf_vote_regs <= 4 &&
           g.cf_tab_words >= 0 &&
           g.pos_begin % pb == 0 && cf_lds_bound(g, pb) <= 80 * 1024;
}

// ---------------------------------------------------------------------------------
// The device-resident runner's predict (csrc/ctl.hip): one launch with a fixed grid; the
// segment table and its block split were written on the device, and a segment whose
// forest is a device refit (res[s] != NULL) takes the compiled forest's shape from the
// refit's result words.  A forest that cannot run here (the refit reported a status, did
// not compile, or needs more LDS than the launch has) sets stall[s]: the partition waits
// for the host, which refits or walks it.
constexpr size_t kDevLds = 80 * 1024;
constexpr size_t kDevLdsRowOrderDefault = 24 * 1024;
// the row-order launch's LDS per workgroup (tuning builds: DDM_ROW_LDS_KB)
size_t row_order_lds() {
#ifdef DDM_TUNING
    static const size_t v = [] {
        const char* e = getenv("DDM_ROW_LDS_KB");
        return e ? (size_t)atoi(e) * 1024 : kDevLdsRowOrderDefault;
    }();
    return v;
#else
    return kDevLdsRowOrderDefault;
#endif
}

__device__ __forceinline__ int cf_rows_dev(const Seg& g, int pb) {
    if (g.cf_leaves > 0) return 1;
    const bool aligned = pb % 4 == 0 && g.ld % 4 == 0 && g.row_base % 4 == 0 &&
                         ((reinterpret_cast<uintptr_t>(g.X) | reinterpret_cast<uintptr_t>(g.y)) & 15) == 0 &&
                         ((reinterpret_cast<uintptr_t>(g.perm) | reinterpret_cast<uintptr_t>(g.err)) & 3) == 0;
    return aligned ? kVecRows : 2;
}

__device__ __forceinline__ void predict_dev_body(const Seg* __restrict__ segs, const int64_t* const* __restrict__ res,
                                                 int n_segs, int pb, int32_t* __restrict__ stall,
                                                 int64_t row_order_delta, int lds_cap) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int64_t gb = blockIdx.x;
    int s = 0;
    while (s < n_segs && !(ldu(&segs[s].block0) <= gb && gb < ldu(&segs[s].block0) + ldu(&segs[s].nblocks))) ++s;
    if (s == n_segs) return;
    Seg sg = ldu(segs + s);
    if (sg.pos_end <= sg.pos_begin) return;
    if (row_order_delta) {                          // row order into err + delta (kSegRowOrder)
        sg.err += row_order_delta;                  // first_err: the first error ROW (a valid hint)
        sg.flags |= kSegRowOrder;
    }
    const int64_t* r = ldu(res + s);
    if (r) {       // the refit's result words (written by an earlier kernel: read-only here)
        sg.n_classes = (int32_t)ldu(r + DDM_DFIT_CLASSES);
        sg.n_nodes = (int32_t)ldu(r + DDM_DFIT_NODES);
        sg.pure = (int32_t)ldu(r + DDM_DFIT_PURE);
        sg.cf_slots = (int32_t)ldu(r + DDM_DFIT_CF_SLOTS);
        sg.cf_vote_regs = (int32_t)ldu(r + DDM_DFIT_CF_VR);
        sg.cf_leaves = (int32_t)ldu(r + DDM_DFIT_CF_LEAVES);
        sg.cf_tab_words = (int32_t)ldu(r + DDM_DFIT_CF_TAB);
        if (ldu(r + DDM_DFIT_STATUS) != 0 || ldu(r + DDM_DFIT_BLOB) <= 0) sg.cforest = nullptr;
    }
    const int rows = cf_rows_dev(sg, pb);
    const bool usable = sg.cforest && sg.cf_slots >= 0 && sg.cf_slots <= 32 && sg.cf_vote_regs >= 1 &&
                        sg.cf_vote_regs <= 4 && sg.cf_tab_words >= 0 && sg.pos_begin % pb == 0 &&
                        cf_lds_bytes(sg.cf_leaves, sg.cf_slots, sg.cf_tab_words, rows) <= (size_t)lds_cap;
    if (!usable) {
        if (threadIdx.x == 0) stall[s] = 1;
        return;
    }
    const int64_t blk = gb - sg.block0, nblk = sg.nblocks;
    const int vk = sg.cf_vote_regs <= 1 ? 0 : sg.cf_vote_regs <= 2 ? 1 : 2;
    switch (3 * (rows == 1 ? 0 : rows == 2 ? 1 : 2) + vk) {
        case 0: cf_dispatch<1, 1>(sg, blk, nblk, pb, smem); break;
        case 1: cf_dispatch<2, 1>(sg, blk, nblk, pb, smem); break;
        case 2: cf_dispatch<4, 1>(sg, blk, nblk, pb, smem); break;
        case 3: cf_dispatch<1, 2>(sg, blk, nblk, pb, smem); break;
        case 4: cf_dispatch<2, 2>(sg, blk, nblk, pb, smem); break;
        case 5: cf_dispatch<4, 2>(sg, blk, nblk, pb, smem); break;
        case 6: cf_dispatch<1, kVecRows>(sg, blk, nblk, pb, smem); break;
        case 7: cf_dispatch<2, kVecRows>(sg, blk, nblk, pb, smem); break;
        default: cf_dispatch<4, kVecRows>(sg, blk, nblk, pb, smem); break;
    }
}

// clk (ddm_ctl.predict_clock): the launch's span on the 100 MHz device clock, as the
// kernel's own time (a rocprofv3 kernel record's, without the queue time HIP events add):
// workgroups 0-7 (one per XCD) stamp their start, every workgroup its end, into 8 shards
// (block b -> shard b & 7) so that no one word takes 2,048 atomics; k_stage_ctl folds them.
__global__ __launch_bounds__(kCfThreads) void k_cforest_predict_dev(const Seg* __restrict__ segs,
                                                                    const int64_t* const* __restrict__ res,
                                                                    int n_segs, int pb, int32_t* __restrict__ stall,
                                                                    int64_t row_order_delta, int lds_cap,
                                                                    unsigned long long* clk, const uint32_t* join_flag,
                                                                    uint32_t join_v, uint32_t* timeouts) {
    if (clk && blockIdx.x < 8 && threadIdx.x == 0) atomicMin(clk + blockIdx.x, (unsigned long long)wall_clock64());
    predict_dev_body(segs, res, n_segs, pb, stall, row_order_delta, lds_cap);
    if (clk) {
        __syncthreads();
        if (threadIdx.x == 0) atomicMax(clk + 8 + (blockIdx.x & 7), (unsigned long long)wall_clock64());
    }
    // join_flag (decoupled epochs, ctl.hip): workgroup 0 -- the first to finish -- holds the
    // kernel's end until the side stream's shuffles of this window are done, so the
    // permutation after it needs no poll of its own (the other workgroups never wait)
    if (join_flag && blockIdx.x == 0 && threadIdx.x == 0) ddm::flag_poll(join_flag, join_v, timeouts);
}

using predict_fn = void (*)(Seg, int64_t);
using predict_batch_fn = void (*)(const Seg*, int, int64_t, int64_t);

// Up to kMaxClasses classes: a batch of per_batch <= 256 rows holds at most 256.  More than
// 64 is a rare shape (the wide variants' vote arrays live partly in scratch), kept so that
// such a batch's forest (refit by sklearn on the host: the device and native trainers take
// up to 64) is still predicted on the device instead of failing.
constexpr int kMaxClasses = 256;

template <bool kLds>
predict_fn pick(bool pure, int k) {
    if (pure) {
        if (k <= 4) return k_forest_predict<true, 4, kLds>;
        if (k <= 8) return k_forest_predict<true, 8, kLds>;
        if (k <= 16) return k_forest_predict<true, 16, kLds>;
        if (k <= 64) return k_forest_predict<true, 64, kLds>;
        return k_forest_predict<true, kMaxClasses, kLds>;
    }
    if (k <= 4) return k_forest_predict<false, 4, kLds>;
    if (k <= 16) return k_forest_predict<false, 16, kLds>;
    if (k <= 64) return k_forest_predict<false, 64, kLds>;
    return k_forest_predict<false, kMaxClasses, kLds>;
}

template <bool kLds>
predict_batch_fn pick_batch(bool pure, int k) {
    if (pure) {
        if (k <= 4) return k_forest_predict_batch<true, 4, kLds>;
        if (k <= 8) return k_forest_predict_batch<true, 8, kLds>;
        if (k <= 16) return k_forest_predict_batch<true, 16, kLds>;
        if (k <= 64) return k_forest_predict_batch<true, 64, kLds>;
        return k_forest_predict_batch<true, kMaxClasses, kLds>;
    }
    if (k <= 4) return k_forest_predict_batch<false, 4, kLds>;
    if (k <= 16) return k_forest_predict_batch<false, 16, kLds>;
    if (k <= 64) return k_forest_predict_batch<false, 64, kLds>;
    return k_forest_predict_batch<false, kMaxClasses, kLds>;
}

size_t forest_lds_bytes(int n_nodes, int n_trees) {
    return ((size_t)n_nodes * sizeof(ddm_node) + (size_t)n_trees * 4 + 15) & ~(size_t)15;
}

constexpr int kMaxBlocks = 256 * 8;

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
    if (forest->n_classes > kMaxClasses || (forest->pure && forest->n_trees > 255) ||
        (!forest->pure && !forest->leaf_value)) {
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
    Seg sg{X, ld, (gptr<const int32_t>)y, (gptr<const uint8_t>)perm, (gptr<uint8_t>)err_out, (gptr<int32_t>)pred_out,
           (gptr<unsigned long long>)first_err, pos_begin, pos_end,
           forest->nodes, forest->roots, forest->leaf_value, forest->classes, forest->n_trees, forest->n_classes,
           forest->n_nodes, forest->pure, 0, 0, 0, forest->cforest, forest->cf_slots, forest->cf_vote_regs,
           forest->cf_leaves, 0, forest->cf_tab_words, 0};
    if (ev_begin)
        if (int rc = ddm::hip_status(hipEventRecord(reinterpret_cast<hipEvent_t>(ev_begin), s), "event record")) return rc;
    if (cf_usable(sg, per_batch)) {
        const int rows = cf_rows(sg, per_batch);
        const int tile = cf_unit(rows, per_batch);
        sg.nblocks = std::min<int64_t>(ddm::ceil_div(n, tile), kMaxBlocks);
        hipLaunchKernelGGL(pick_cf(cf_vkind(sg.cf_vote_regs), rows), dim3((unsigned)sg.nblocks),
                           dim3(kCfThreads), cf_lds_bound(sg, per_batch), s, sg, (int)per_batch);
    } else {
        const size_t lds = forest_lds_bytes(forest->n_nodes, forest->n_trees);
        const bool use_lds = lds <= (size_t)kMaxLdsForest;
        const predict_fn fn = use_lds ? pick<true>(forest->pure, forest->n_classes)
                                      : pick<false>(forest->pure, forest->n_classes);
        sg.nblocks = std::min<int64_t>(ddm::ceil_div(n, kThreads), kMaxBlocks);
        hipLaunchKernelGGL(fn, dim3((unsigned)sg.nblocks), dim3(kThreads), use_lds ? lds : 0, s, sg,
                           (int64_t)per_batch);
    }
    if (int rc = ddm::launch_status("ddm_forest_predict")) return rc;
    if (ev_end)
        if (int rc = ddm::hip_status(hipEventRecord(reinterpret_cast<hipEvent_t>(ev_end), s), "event record")) return rc;
    return 0;
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
    // One launch per kernel variant; every launch walks the whole device table and only
    // the blocks assigned to its segments work.  Variants: 16 node-walk kinds (pure x
    // classes <= 64 x LDS-resident forest), 9 compiled kinds (vote registers x rows/lane)
    // and 4 wide node-walk kinds (pure x LDS, up to kMaxClasses classes).
    Seg* hs = reinterpret_cast<Seg*>(const_cast<ddm_predict_segment*>(segs_host));
    for (int i = 0; i < n_segs; ++i) {
        const Seg& g = hs[i];
        if (!g.X || !g.y || !g.perm || !g.err || !g.nodes || !g.roots || !g.classes || g.pos_end < g.pos_begin ||
            g.pos_begin < 0 || g.n_classes <= 0 || g.n_classes > kMaxClasses || g.n_trees <= 0 ||
            (g.pure && g.n_trees > 255) || (!g.pure && !g.leaf_value)) {
            ddm::set_error("ddm_forest_predict_batch: invalid segment %d", i);
            return DDM_E_ARG;
        }
        if (g.first_err && !(g.flags & DDM_SEG_FIRST_ERR_PRESET))
            if (int rc = ddm::hip_status(hipMemsetAsync((void*)g.first_err, 0xff, sizeof(uint64_t), s), "predict_batch memset"))
                return rc;
    }
    if (ev_begin)
        if (int rc = ddm::hip_status(hipEventRecord(reinterpret_cast<hipEvent_t>(ev_begin), s), "event record")) return rc;
    constexpr int kCf0 = 16, kWide0 = 16 + 9, kNV = 16 + 9 + 4;
    const auto is_cf = [](int v) { return v >= kCf0 && v < kWide0; };
    std::vector<int> variant(n_segs);
    for (int i = 0; i < n_segs; ++i) {
        const Seg& g = hs[i];
        if (cf_usable(g, per_batch)) {
            variant[i] = kCf0 + 3 * cf_rows_idx(cf_rows(g, per_batch)) + cf_vkind(g.cf_vote_regs);
        } else {
            const bool lds = forest_lds_bytes(g.n_nodes, g.n_trees) <= (size_t)kMaxLdsForest;
            if (g.n_classes > 64) {
                variant[i] = kWide0 + (g.pure ? 2 : 0) + (lds ? 1 : 0);
            } else {
                const int kc = g.n_classes <= 4 ? 0 : g.n_classes <= 8 ? 1 : g.n_classes <= 16 ? 2 : 3;
                variant[i] = (g.pure ? 1 : 0) * 8 + (lds ? 4 : 0) + kc;
            }
        }
    }
    int64_t vbase[kNV + 1] = {0};
    size_t vlds[kNV] = {0};
    int64_t b0 = 0;
    for (int v = 0; v < kNV; ++v) {
        vbase[v] = b0;
        const int unit = is_cf(v) ? cf_unit(cf_rows_of_idx((v - kCf0) / 3), per_batch) : kThreads;
        int64_t rows = 0;
        for (int i = 0; i < n_segs; ++i)
            if (variant[i] == v) {
                rows += hs[i].pos_end - hs[i].pos_begin;
                vlds[v] = std::max(vlds[v], is_cf(v) ? cf_lds_bound(hs[i], per_batch)
                                                     : forest_lds_bytes(hs[i].n_nodes, hs[i].n_trees));
            }
        const int64_t total_blocks = rows ? std::min<int64_t>(ddm::ceil_div(rows, unit), kMaxBlocks) : 0;
        for (int i = 0; i < n_segs; ++i) {
            if (variant[i] != v) continue;
            Seg& g = hs[i];
            const int64_t r = g.pos_end - g.pos_begin;
            g.block0 = b0;
            g.nblocks = r == 0 ? 0 : std::max<int64_t>(1, (total_blocks * r + rows - 1) / rows);
            b0 += g.nblocks;
        }
    }
    vbase[kNV] = b0;
    bool all_cf = true;
    for (int i = 0; i < n_segs; ++i) all_cf = all_cf && is_cf(variant[i]);
    if (all_cf && n_segs <= kArgSegs) {
        // compiled forests only: the table rides in the kernel arguments (no table copy)
        SegTab tab{};
        for (int i = 0; i < n_segs; ++i) tab.s[i] = hs[i];
        for (int v = kCf0; v < kWide0; ++v) {
            const int64_t nb = vbase[v + 1] - vbase[v];
            if (nb == 0) continue;
            hipLaunchKernelGGL(pick_cf_arg((v - kCf0) % 3, cf_rows_of_idx((v - kCf0) / 3)), dim3((unsigned)nb),
                               dim3(kCfThreads), vlds[v],
                               s, tab, n_segs, vbase[v], (int)per_batch);
            if (int rc = ddm::launch_status("ddm_forest_predict_batch")) return rc;
        }
        if (ev_end)
            if (int rc = ddm::hip_status(hipEventRecord(reinterpret_cast<hipEvent_t>(ev_end), s), "event record")) return rc;
        return 0;
    }
    if (b0 > 0) {
        if (int rc = ddm::hip_status(hipMemcpyAsync(segs_dev, hs, sizeof(Seg) * n_segs, hipMemcpyHostToDevice, s),
                                     "predict_batch table"))
            return rc;
    }
    for (int v = 0; v < kNV; ++v) {
        const int64_t nb = vbase[v + 1] - vbase[v];
        if (nb == 0) continue;
        if (is_cf(v)) {
            hipLaunchKernelGGL(pick_cf_batch((v - kCf0) % 3, cf_rows_of_idx((v - kCf0) / 3)), dim3((unsigned)nb),
                               dim3(kCfThreads), vlds[v], s,
                               reinterpret_cast<const Seg*>(segs_dev), n_segs, vbase[v], (int)per_batch);
        } else {
            const bool wide = v >= kWide0;
            const bool lds = wide ? ((v - kWide0) & 1) != 0 : (v & 4) != 0;
            const bool pure = wide ? ((v - kWide0) & 2) != 0 : (v & 8) != 0;
            const int kmax = wide ? kMaxClasses : (v & 3) == 0 ? 4 : (v & 3) == 1 ? 8 : (v & 3) == 2 ? 16 : 64;
            const predict_batch_fn fn = lds ? pick_batch<true>(pure, kmax) : pick_batch<false>(pure, kmax);
            hipLaunchKernelGGL(fn, dim3((unsigned)nb), dim3(kThreads), lds ? vlds[v] : 0, s,
                               reinterpret_cast<const Seg*>(segs_dev), n_segs, vbase[v], (int64_t)per_batch);
        }
        if (int rc = ddm::launch_status("ddm_forest_predict_batch")) return rc;
    }
    if (ev_end)
        if (int rc = ddm::hip_status(hipEventRecord(reinterpret_cast<hipEvent_t>(ev_end), s), "event record")) return rc;
    return 0;
}

int forest_predict_dev_clk(const ddm_predict_segment* segs_dev, const int64_t* const* res_dev, int32_t n_segs,
                           int32_t per_batch, int64_t grid, int32_t* stall, uint64_t* clk, ddm_stream_t stream);

extern "C" int ddm_forest_predict_dev(const ddm_predict_segment* segs_dev, const int64_t* const* res_dev,
                                      int32_t n_segs, int32_t per_batch, int64_t grid, int32_t* stall,
                                      ddm_stream_t stream, ddm_event_t ev_begin, ddm_event_t ev_end) {
    if (!segs_dev || !res_dev || !stall || n_segs <= 0 || per_batch <= 0 || per_batch > 256 || grid <= 0 ||
        grid >= ((int64_t)1 << 31)) {
        ddm::set_error("ddm_forest_predict_dev: invalid argument");
        return DDM_E_ARG;
    }
    hipStream_t s = ddm::as_hip(stream);
    if (ev_begin)
        if (int rc = ddm::hip_status(hipEventRecord(reinterpret_cast<hipEvent_t>(ev_begin), s), "event record")) return rc;
    if (int rc = forest_predict_dev_clk(segs_dev, res_dev, n_segs, per_batch, grid, stall, nullptr, stream)) return rc;
    if (ev_end)
        if (int rc = ddm::hip_status(hipEventRecord(reinterpret_cast<hipEvent_t>(ev_end), s), "event record")) return rc;
    return 0;
}

// The same launch, stamping clk (ddm_ctl.predict_clock) when non-null (csrc/ctl.hip).
int forest_predict_dev_clk(const ddm_predict_segment* segs_dev, const int64_t* const* res_dev, int32_t n_segs,
                           int32_t per_batch, int64_t grid, int32_t* stall, uint64_t* clk, ddm_stream_t stream) {
    hipLaunchKernelGGL(k_cforest_predict_dev, dim3((unsigned)grid), dim3(kCfThreads), kDevLds, ddm::as_hip(stream),
                       reinterpret_cast<const Seg*>(segs_dev), res_dev, (int)n_segs, (int)per_batch, stall,
                       (int64_t)0, (int)kDevLds, reinterpret_cast<unsigned long long*>(clk), nullptr, 0u, nullptr);
    return ddm::launch_status("ddm_forest_predict_dev");
}

// ---- row-order predict + the permutation into DDM order (device-resident epochs) --------
namespace {

// err[g] = err_rows[(g / pb) * pb + perm[g]] over every segment's positions (err_rows =
// err + delta, written by ddm_forest_predict_dev_orig).  The row-order predict noted its
// first error ROW in first_err: every batch before that row's batch is error-free, so
// those positions are only zero-filled (16-byte stores), and the hint the scan gets is that
// batch's first position (the row itself is no hint: the batch's shuffle may put an error
// row ahead of it).  From that batch on, a thread takes 4 positions of one batch
// (pb % 4 == 0) or single positions otherwise.
constexpr int kPermThreads = 256;

__global__ __launch_bounds__(kPermThreads) void k_err_permute(const Seg* __restrict__ segs, int64_t delta, int pb) {
    const Seg sg = ldu(segs + blockIdx.y);
    if (sg.pos_end <= sg.pos_begin) return;
    gptr<const uint8_t> src = sg.err + delta;
    const int64_t tid = (int64_t)blockIdx.x * kPermThreads + threadIdx.x;
    const int64_t step = (int64_t)gridDim.x * kPermThreads;
    const unsigned long long f = sg.first_err ? *sg.first_err : ~0ull;
    const int64_t zend = f >= (unsigned long long)sg.pos_end
                             ? sg.pos_end
                             : max(sg.pos_begin, ((int64_t)f / pb) * pb);
    // every block computes the same zend from f or from zend itself: the store is idempotent
    if (blockIdx.x == 0 && threadIdx.x == 0 && zend < sg.pos_end) *sg.first_err = (unsigned long long)zend;
    // zeros: [pos_begin, zend)
    {
        const int64_t a0 = min(zend, (sg.pos_begin + 15) & ~(int64_t)15), a1 = max(a0, zend & ~(int64_t)15);
        for (int64_t g = sg.pos_begin + tid; g < a0; g += step) sg.err[g] = 0;
        for (int64_t w = a0 / 16 + tid; w < a1 / 16; w += step) ((gptr<u32x4>)sg.err)[w] = u32x4{0u, 0u, 0u, 0u};
        for (int64_t g = a1 + tid; g < zend; g += step) sg.err[g] = 0;
    }
    // the permutation: [zend, pos_end); zend is batch-aligned
    if (pb % 4 == 0 && zend % 4 == 0) {
        for (int64_t g = zend + 4 * tid; g < sg.pos_end; g += 4 * step) {
            const int64_t b0 = (g / pb) * pb;
            const uint32_t p4 = *(gptr<const uint32_t>)(sg.perm + g);
            uint32_t out = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const bool ok = g + i < sg.pos_end;
                const uint32_t e = ok ? src[b0 + ((p4 >> (8 * i)) & 0xffu)] : 0u;
                out |= e << (8 * i);
            }
            if (g + 4 <= sg.pos_end) {
                *(gptr<uint32_t>)(sg.err + g) = out;
            } else {
                for (int i = 0; g + i < sg.pos_end; ++i) sg.err[g + i] = (uint8_t)((out >> (8 * i)) & 0xffu);
            }
        }
    } else {
        for (int64_t g = zend + tid; g < sg.pos_end; g += step) sg.err[g] = src[(g / pb) * pb + sg.perm[g]];
    }
}

}  // namespace

// Internal (csrc/ctl.hip): the device-table predict writing err + delta in row order.
extern "C" int ddm_forest_predict_dev_orig(const ddm_predict_segment* segs_dev, const int64_t* const* res_dev,
                                           int32_t n_segs, int32_t per_batch, int64_t grid, int32_t* stall,
                                           int64_t delta, uint64_t* clk, const uint32_t* join_flag, uint32_t join_v,
                                           uint32_t* timeouts, ddm_stream_t stream) {
    if (!segs_dev || !res_dev || !stall || n_segs <= 0 || per_batch <= 0 || per_batch > 256 || grid <= 0 ||
        grid >= ((int64_t)1 << 31) || delta == 0) {
        ddm::set_error("ddm_forest_predict_dev_orig: invalid argument");
        return DDM_E_ARG;
    }
    // 24 KB of LDS per workgroup instead of 80 (a stump forest's tables, labels and errors
    // take ~16 KB): the side stream's replay workgroups hold ~134 KB of a CU's 160 while they
    // run, and a predict workgroup that does not fit waits for them (a 20 us gap per C3
    // epoch at 48 KB).  A forest that needs more stalls its partition to the host, as any
    // unusable forest, and the runner stops decoupling (ddm_amd/devctl.py).
    const size_t lds = row_order_lds();
    hipLaunchKernelGGL(k_cforest_predict_dev, dim3((unsigned)grid), dim3(kCfThreads), lds, ddm::as_hip(stream),
                       reinterpret_cast<const Seg*>(segs_dev), res_dev, (int)n_segs, (int)per_batch, stall, delta,
                       (int)lds, reinterpret_cast<unsigned long long*>(clk), join_flag, join_v, timeouts);
    return ddm::launch_status("ddm_forest_predict_dev_orig");
}

// Internal (csrc/ctl.hip): row-order errors (err + delta) into DDM order, every segment.
extern "C" int ddm_err_permute_dev(const ddm_predict_segment* segs_dev, int32_t n_segs, int32_t per_batch,
                                   int64_t delta, int32_t blocks_per_seg, ddm_stream_t stream) {
    if (!segs_dev || n_segs <= 0 || n_segs > 65535 || per_batch <= 0 || per_batch > 256 || delta == 0 ||
        blocks_per_seg <= 0) {
        ddm::set_error("ddm_err_permute_dev: invalid argument");
        return DDM_E_ARG;
    }
    hipLaunchKernelGGL(k_err_permute, dim3((unsigned)blocks_per_seg, (unsigned)n_segs), dim3(kPermThreads), 0,
                       ddm::as_hip(stream), reinterpret_cast<const Seg*>(segs_dev), delta, (int)per_batch);
    return ddm::launch_status("ddm_err_permute_dev");
}
