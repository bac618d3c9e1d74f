// Device forest refit: train_rf (DDM_Process.py:98-105) on the GPU.
//
// The host trainer (rf_fit.cpp, pinned to scikit-learn 1.7.2 by tests/test_trainer.py)
// is restated here with the same arithmetic, so that both build the same trees:
//   k_dfit_prep    one workgroup per job: gate, NaN check, classes_ (np.unique) and the
//                  class index of every row, per-feature presorted row orders; beside
//                  it, boot workgroups (one wave per tree):
//                    * RandomState(seed): init_genrand on lane 0 (a serial recurrence),
//                      the 624-word twist in three lane-parallel phases, tempering;
//                    * the splitter seed = the first randint(0, 2**31-1) of that stream
//                      (peeked) and the bootstrap = randint(0, L, L) from the same start
//                      (accept/reject by ballot, counts by LDS atomics);
//   k_dfit_trees   one wave per (job, tree), from the boot workgroups' draws:
//                    * depth-first BestSplitter: the feature draws (our_rand_r) and the
//                      constant-feature bookkeeping run identically in every lane; a
//                      node's rows in feature order come from the presorted order by a
//                      ballot compaction, the class sums left of every split position
//                      by wave prefix sums (exact integers), the Gini proxy of every
//                      position is evaluated by its lane and the first maximum wins;
//   k_dfit_pack    one workgroup per job: BFS packing (ddm_node, adjacent children)
//                  and the forest compiler of forest_compile.cpp (run by one lane).
// Floating point: the proxy, impurity and improvement formulas are evaluated in the
// host's operation order with contraction off (Makefile: -ffp-contract=off), on
// exact integer class sums, so every comparison matches the host bit for bit.
#include <math.h>

#include "common.h"

namespace {

constexpr int kMaxL = 256;
constexpr int kMaxF = 256;
constexpr int kMaxK = 64;
constexpr int kWaves = 4;                      // trees per workgroup
constexpr int kPrepTile = 8192;                // floats of X staged per presort round
constexpr int kMaxSlots = 32;
constexpr int kMaxCfLeaves = 64;
constexpr int kMaxTabWords = 4 * (255 + 5 * kMaxSlots);   // rank-table words of <= 255 stumps
constexpr uint32_t kRandRMax = 0x7fffffffu;
constexpr float kFeatureThreshold = 1e-7f;
constexpr double kEpsilon = 2.220446049250313e-16;

// The job's pointers as the global address space (device memory): the kernels' accesses
// through them are global_* instructions instead of flat_* (which also count on lgkmcnt,
// so every LDS wait waited for them too); pass (T*) casts where a callee also takes LDS.
using ddm::gget;
using ddm::lptr;
using ddm::gptr;
using ddm::gput;
struct Job {
    gptr<const float> X;
    gptr<const int32_t> y;
    gptr<const int64_t> seeds;
    gptr<const int64_t> gate;
    gptr<const int64_t> gate2;
    int32_t L, F, n_trees, max_features;
    int32_t k_cap, pad;
    gptr<uint8_t> scratch;
    gptr<ddm_node> nodes;
    gptr<int32_t> roots;
    gptr<double> leaf_value;
    gptr<int32_t> classes;
    gptr<uint8_t> blob;
    int64_t blob_cap;
    gptr<int64_t> result;
};
static_assert(sizeof(Job) == sizeof(ddm_dfit_job), "Job must mirror ddm_dfit_job");

// A job whose gate says "no refit this epoch" (no change: *gate < 0; or batch d+1's shuffle
// and the seeds were not staged: *gate2 != 1).  Every kernel of the refit checks it, and
// nothing is written: the result words keep the partition's last refit, whose forest the
// device-resident runner's predict is still using.
__device__ __forceinline__ bool gated_off(const Job& jb) {
    return (jb.gate && *jb.gate < 0) || (jb.gate2 && *jb.gate2 != 1);
}

// Tree node in creation (_add_node) order, which is pre-order (depth first, left child
// first): a node's left subtree is the id range [id + 1, right).
struct TNode {
    int16_t left, right, feature;
    uint8_t missing_left, leaf;
    double threshold;
};
static_assert(sizeof(TNode) == 16, "TNode");

struct Stump {
    int32_t slot;
    float thr;
    int32_t cl, cr, nanleft;
};

// ---- per-job scratch layout -------------------------------------------------------
struct Layout {
    int64_t yidx, order, tnodes, tvals, tmeta, bfs, cslot, cstump, ctree, cnode, cleaf, cframe, csort, boot, total;
};

__host__ __device__ inline int64_t al16(int64_t v) { return (v + 15) & ~(int64_t)15; }

__host__ __device__ inline Layout layout(int L, int F, int T, int K) {
    Layout o;
    const int64_t M = 2 * (int64_t)L - 1;      // nodes per tree
    o.yidx = 64;
    o.order = al16(o.yidx + L);
    o.tnodes = al16(o.order + (int64_t)F * L);
    o.tvals = al16(o.tnodes + 16 * (int64_t)T * M);
    o.tmeta = al16(o.tvals + 8 * (int64_t)T * M * K);
    o.bfs = al16(o.tmeta + 16 * (int64_t)T);
    o.cslot = al16(o.bfs + 4 * (int64_t)T * M);
    o.cstump = al16(o.cslot + 4 * (int64_t)F);
    o.ctree = al16(o.cstump + (int64_t)sizeof(Stump) * T);
    o.cnode = al16(o.ctree + (int64_t)sizeof(ddm_cforest_tree) * T);
    o.cleaf = al16(o.cnode + (int64_t)sizeof(ddm_cforest_node) * T * (kMaxCfLeaves - 1));
    o.cframe = al16(o.cleaf + (int64_t)T * kMaxCfLeaves);
    o.csort = al16(o.cframe + 16 * (int64_t)2 * kMaxCfLeaves);
    o.boot = al16(o.csort + 4 * (int64_t)T);
    o.total = al16(o.boot + 4 * (int64_t)T * (L + 1));
    return o;
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ uint64_t lanemask_lt(int lane) { return lane ? (~0ull >> (64 - lane)) : 0ull; }

__device__ __forceinline__ uint32_t temper(uint32_t y) {
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

__device__ __forceinline__ uint32_t mt_word(uint32_t a, uint32_t b, uint32_t c) {
    const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
    return c ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}

// One MT19937 twist of mt[624] in place by one wave: words 0..226 from old words,
// 227..453 from old words and new 0..226, 454..623 from old words and new 227..396
// (and new 0 for the last).  Each phase computes into registers before it writes.
__device__ void twist(lptr<uint32_t> mt, int lane) {
    uint32_t v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int i = lane + 64 * k;
        v[k] = i < 227 ? mt_word(mt[i], mt[i + 1], mt[i + 397]) : 0u;
    }
    wave_sync();
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int i = lane + 64 * k;
        if (i < 227) mt[i] = v[k];
    }
    wave_sync();
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int i = 227 + lane + 64 * k;
        v[k] = i < 454 ? mt_word(mt[i], mt[i + 1], mt[i - 227]) : 0u;
    }
    wave_sync();
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int i = 227 + lane + 64 * k;
        if (i < 454) mt[i] = v[k];
    }
    wave_sync();
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const int i = 454 + lane + 64 * k;
        v[k] = i < 623 ? mt_word(mt[i], mt[i + 1], mt[i - 227]) : (i == 623 ? mt_word(mt[623], mt[0], mt[396]) : 0u);
    }
    wave_sync();
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const int i = 454 + lane + 64 * k;
        if (i < 624) mt[i] = v[k];
    }
    wave_sync();
}

__device__ __forceinline__ uint32_t our_rand_r(uint32_t& s) {
    if (s == 0) s = 1;
    s ^= s << 13;
    s ^= s >> 17;
    s ^= s << 5;
    return s % (kRandRMax + 1u);
}

// One step of a wave scan / reduction by DPP: the value from the lane kCtrl names
// (row_shr:n, or row_bcast:15/31 into the rows of kRowMask), `ident` where there is none.
template <int kCtrl, int kRowMask>
__device__ __forceinline__ int dpp_i(int v, int ident) {
    return __builtin_amdgcn_update_dpp(ident, v, kCtrl, kRowMask, 0xF, false);
}

template <int kCtrl, int kRowMask>
__device__ __forceinline__ double dpp_d(double v, double ident) {
    const long long b = __double_as_longlong(v), e = __double_as_longlong(ident);
    const int lo = __builtin_amdgcn_update_dpp((int)e, (int)b, kCtrl, kRowMask, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp((int)(e >> 32), (int)(b >> 32), kCtrl, kRowMask, 0xF, false);
    return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}

__device__ __forceinline__ double readlane_d(double v, int src) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, src);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), src);
    return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}

// Wave reductions, uniform results: the inclusive DPP scan's last lane, read by readlane.
__device__ __forceinline__ int wave_sum_i(int v) {
    v += dpp_i<0x111, 0xF>(v, 0);
    v += dpp_i<0x112, 0xF>(v, 0);
    v += dpp_i<0x114, 0xF>(v, 0);
    v += dpp_i<0x118, 0xF>(v, 0);
    v += dpp_i<0x142, 0xA>(v, 0);
    v += dpp_i<0x143, 0xC>(v, 0);
    return __builtin_amdgcn_readlane(v, 63);
}

__device__ __forceinline__ int wave_min_i(int v) {
    constexpr int kId = 0x7fffffff;
    v = min(v, dpp_i<0x111, 0xF>(v, kId));
    v = min(v, dpp_i<0x112, 0xF>(v, kId));
    v = min(v, dpp_i<0x114, 0xF>(v, kId));
    v = min(v, dpp_i<0x118, 0xF>(v, kId));
    v = min(v, dpp_i<0x142, 0xA>(v, kId));
    v = min(v, dpp_i<0x143, 0xC>(v, kId));
    return __builtin_amdgcn_readlane(v, 63);
}

__device__ __forceinline__ double wave_max_d(double v) {
    const double kId = -__builtin_huge_val();
    v = fmax(v, dpp_d<0x111, 0xF>(v, kId));
    v = fmax(v, dpp_d<0x112, 0xF>(v, kId));
    v = fmax(v, dpp_d<0x114, 0xF>(v, kId));
    v = fmax(v, dpp_d<0x118, 0xF>(v, kId));
    v = fmax(v, dpp_d<0x142, 0xA>(v, kId));
    v = fmax(v, dpp_d<0x143, 0xC>(v, kId));
    return readlane_d(v, 63);
}

// inclusive prefix sum over the wave by DPP (rows of 16 by row_shr 1/2/4/8, then across
// rows by row_bcast 15/31; a lane without a source adds 0): six VALU operations instead of
// six LDS-crossbar shuffles (the split search's per-class scans are its inner loop)
__device__ __forceinline__ int wave_scan_i(int v, int lane) {
    (void)lane;
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false);
    return v;
}

// the last lane's value (uniform)
__device__ __forceinline__ int wave_last_i(int v) { return __builtin_amdgcn_readlane(v, 63); }

// RandomState(seed) of one tree (init_genrand on lane 0: a serial recurrence, on the
// scalar unit it made the trees kernel slower, 46 -> 54 us with 800 waves sharing one
// scalar unit per CU; the 624-word twist lane-parallel), the splitter seed = the first
// randint(0, 2**31 - 1) of that stream (peeked, not consumed) and the bootstrap =
// randint(0, L, L) from the same start, as multiplicities in cnt[0..L).  One wave; returns
// the splitter seed.
#ifdef DDM_PREP_PROFILE
__device__ uint64_t g_boot_prof[3];   // the last boot's stamps: init done, twist done, end
#endif

// init_genrand words base + k0 .. base + k1 - 1 (v holds word base + k0 - 1), each written
// into lane k of buf
template <int k0, int k1>
__device__ __forceinline__ void init_block(uint32_t& v, uint32_t& buf, uint32_t base) {
#pragma unroll
    for (int k = k0; k < k1; ++k) {
        v = 1812433253u * (v ^ (v >> 30)) + (base + (uint32_t)k);
        asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(buf) : "s"(v), "i"(k));
    }
}

__device__ uint32_t tree_boot(uint32_t seed, int L, lptr<uint32_t> mt, lptr<int32_t> cnt, int lane) {
    // init_genrand: the recurrence on the scalar unit (a uniform value: s_mul_i32 and
    // friends, instead of quarter-rate wave64 VALU operations on one lane), each word put
    // into its lane of a VGPR by v_writelane (off the chain; 64 steps unrolled, so no branch
    // or compare per step) and stored 64 words at a time
    uint32_t v = __builtin_amdgcn_readfirstlane(seed);
    uint32_t buf = v;                               // word 0 in every lane, lane 0 kept
    init_block<1, 64>(v, buf, 0u);
    mt[lane] = buf;
    for (uint32_t base = 64; base < 576; base += 64) {
        init_block<0, 64>(v, buf, base);
        mt[base + lane] = buf;
    }
    init_block<0, 48>(v, buf, 576u);
    if (lane < 48) mt[576 + lane] = buf;            // words 576..623
    wave_sync();
#ifdef DDM_PREP_PROFILE
    const uint64_t tq1 = wall_clock64();
#endif
    twist(mt, lane);
    for (int k = lane; k < L; k += 64) cnt[k] = 0;
    wave_sync();
#ifdef DDM_PREP_PROFILE
    const uint64_t tq2 = wall_clock64();
#endif
    uint32_t rstate = 0;
    for (int j0 = 0; j0 < 624; j0 += 64) {
        const int j = j0 + lane;
        const uint32_t v = j < 624 ? (temper(mt[j]) & 0x7fffffffu) : 0xffffffffu;
        const uint64_t m = __ballot(j < 624 && v <= kRandRMax - 1u);
        if (m) {
            rstate = __shfl(v, __builtin_ctzll(m), 64);
            break;
        }
    }
    if (L > 1) {
        const uint32_t mx = (uint32_t)(L - 1);
        const uint32_t mask = 0xffffffffu >> __builtin_clz(mx);
        int taken = 0;
        for (;;) {
            for (int j0 = 0; j0 < 624 && taken < L; j0 += 64) {
                const int j = j0 + lane;
                const uint32_t v = j < 624 ? (temper(mt[j]) & mask) : 0xffffffffu;
                const bool acc = j < 624 && v <= mx;
                const uint64_t m = __ballot(acc);
                if (acc && taken + __popcll(m & lanemask_lt(lane)) < L)
                    __hip_atomic_fetch_add(cnt + v, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
                taken += __popcll(m);
            }
            if (taken >= L) break;
            twist(mt, lane);
        }
    } else if (lane == 0) {
        cnt[0] = 1;                                 // interval(0) draws nothing
    }
    wave_sync();
#ifdef DDM_PREP_PROFILE
    g_boot_prof[0] = tq1;
    g_boot_prof[1] = tq2;
    g_boot_prof[2] = wall_clock64();
#endif
    return rstate;
}

// k_dfit_prep's boot workgroups (blockIdx.y >= kSortBlocks): one tree per wave, the draws tree_boot
// makes, stored for k_dfit_trees (rstate, then the L bootstrap counts).  They run beside
// the presort instead of at the head of every tree wave (init_genrand alone is ~15 us).
// Only the first wave of each SIMD works: the init recurrence runs on one lane, but every
// wave64 VALU instruction holds its SIMD for 4 cycles, so 16 such waves per CU (4 per
// SIMD) took 58 us instead of ~20 and slowed the window shuffles beside them.
constexpr int kPrepThreads = 1024;         // presort tasks: every (feature, row) pair
constexpr int kBootWaves = 4;              // working waves (trees) per boot workgroup
// presort workgroups per job: the (feature, row) rank tasks are ALU work (100 comparisons
// each, 2,700 for a 100 x 27 batch), ~10 us on one CU; each workgroup also redoes the
// label pass (~1 us) so that all agree on NaN / class-count exits
constexpr int kSortBlocks = 4;

__device__ void dfit_boot(const Job& jb, int bblk) {
    __shared__ uint32_t s_mt[kBootWaves][624];
    __shared__ int32_t s_cnt[kBootWaves][kMaxL];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int tree = bblk * kBootWaves + w;
    const int L = jb.L;
    if (w >= kBootWaves || gated_off(jb) || L < 1 || L > kMaxL || jb.F < 1 || jb.F > kMaxF || jb.n_trees < 1 || jb.n_trees > 256 ||
        jb.k_cap < 1 || jb.k_cap > kMaxK || jb.max_features < 1 || tree >= jb.n_trees)
        return;
    const Layout lo = layout(L, jb.F, jb.n_trees, jb.k_cap);
    gptr<int32_t> bt = (gptr<int32_t>)(jb.scratch + lo.boot) + (int64_t)tree * (L + 1);
#ifdef DDM_PREP_PROFILE
    const uint64_t tb0 = wall_clock64();
#endif
    const uint32_t rs = tree_boot((uint32_t)jb.seeds[tree], L, (lptr<uint32_t>)s_mt[w], (lptr<int32_t>)s_cnt[w], lane);
    if (lane == 0) bt[0] = (int32_t)rs;
    for (int k = lane; k < L; k += 64) bt[1 + k] = s_cnt[w][k];
#ifdef DDM_PREP_PROFILE
    if (tree == 0 && lane == 0) {   // boot of tree 0: start (vs the presort's start), duration
        __threadfence();
        // init done / twist done / draws done / end: 16-bit fields of 10-ns ticks from tb0
        jb.result[11] = (int64_t)((g_boot_prof[0] - tb0) | ((g_boot_prof[1] - tb0) << 16) |
                                  ((g_boot_prof[2] - tb0) << 32) | ((wall_clock64() - tb0) << 48));
    }
#endif
}

// ---- k_dfit_prep --------------------------------------------------------------------
// The refit kernels are the epoch's critical path while the next windows' shuffles run on
// the side stream on the same CUs: their waves take issue priority over the shuffles'.
#ifndef DDM_REFIT_PRIO
#define DDM_REFIT_PRIO 2
#endif
__device__ __forceinline__ void refit_priority() { __builtin_amdgcn_s_setprio(DDM_REFIT_PRIO); }

__global__ __launch_bounds__(kPrepThreads) void k_dfit_prep(const Job* __restrict__ jobs) {
    refit_priority();
    const Job jb = jobs[blockIdx.x];
    if (blockIdx.y >= kSortBlocks) {
        dfit_boot(jb, (int)blockIdx.y - kSortBlocks);
        return;
    }
    const int t = threadIdx.x;
    const int part = (int)blockIdx.y;            // this workgroup's share of the rank tasks
    const bool lead = part == 0;                 // writes classes_, yidx and the status
#ifdef DDM_PREP_PROFILE
    const uint64_t tp0 = wall_clock64();
#endif
    __shared__ int32_t s_y[kMaxL];
    __shared__ float s_tile[kPrepTile];
    __shared__ uint8_t s_first[kMaxL];
    __shared__ int s_nan, s_K, s_skip;
    const int L = jb.L, F = jb.F;
    const bool args_ok = !(L < 1 || L > kMaxL || F < 1 || F > kMaxF || jb.n_trees < 1 || jb.n_trees > 256 ||
                           jb.k_cap < 1 || jb.k_cap > kMaxK || jb.max_features < 1);
    // the labels and (when every feature fits one tile, the controller's batches) X itself
    // are loaded beside the gate words instead of after them: one round trip to HBM, not
    // three; the NaN check reads the tile
    const int G = args_ok ? max(1, min(F, kPrepTile / L)) : 1;
    const bool one_tile = args_ok && G == F;
    if (t == 0) {
        s_skip = gated_off(jb);
        s_nan = 0;
        s_K = 0;
    }
    if (args_ok) {
        if (t < L) s_y[t] = jb.y[t];
        if (one_tile) {
            for (int e = t; e < L * F; e += kPrepThreads) {
                const float x = jb.X[e];
                const int r = e / F, k = e % F;
                s_tile[k * L + r] = x;
                if (x != x) s_nan = 1;
            }
        }
    }
    __syncthreads();
    if (s_skip) return;                          // the result words keep the last refit's
    if (!args_ok) {
        if (lead && t == 0) jb.result[DDM_DFIT_STATUS] = DDM_E_ARG;
        return;
    }
    const Layout lo = layout(L, F, jb.n_trees, jb.k_cap);
    gptr<uint8_t> yidx = jb.scratch + lo.yidx;
    gptr<uint8_t> order = jb.scratch + lo.order;
    if (!one_tile) {
        for (int e = t; e < L * F; e += kPrepThreads)
            if (jb.X[e] != jb.X[e]) s_nan = 1;
        __syncthreads();
    }
    // classes_ = np.unique(y): first occurrences ranked by value
    if (t < L) {
        int first = 1;
#pragma unroll 16
        for (int j = 0; j < t; ++j) first &= s_y[j] != s_y[t];
        s_first[t] = (uint8_t)first;
        if (first) atomicAdd(&s_K, 1);
    }
    __syncthreads();
    const int K = s_K;
    if (t < L) {
        int rank = 0;
#pragma unroll 16
        for (int j = 0; j < L; ++j) rank += (s_first[j] && s_y[j] < s_y[t]) ? 1 : 0;
        if (lead) {
            yidx[t] = (uint8_t)min(rank, 255);
            if (s_first[t] && rank < jb.k_cap) jb.classes[rank] = s_y[t];
        }
    }
    if (s_nan || K > jb.k_cap) {
        if (lead && t == 0) {
            jb.result[DDM_DFIT_STATUS] = s_nan ? DDM_E_NAN : DDM_E_FOREST;
            jb.result[DDM_DFIT_CLASSES] = K;
        }
        return;
    }
#ifdef DDM_PREP_PROFILE
    const uint64_t tp1 = wall_clock64();
#endif
    // presorted orders: the stable rank of every row in every feature, for as many
    // features at once as fit the LDS tile (every (feature, row) pair is one task)
    for (int f0 = 0; f0 < F; f0 += G) {
        const int g = min(G, F - f0);
        if (!one_tile) {
            __syncthreads();
            for (int e = t; e < L * g; e += kPrepThreads) {
                const int r = e / g, k = e % g;
                s_tile[k * L + r] = jb.X[(int64_t)r * F + f0 + k];
            }
        }
        __syncthreads();
        for (int e = part * kPrepThreads + t; e < L * g; e += kSortBlocks * kPrepThreads) {
            const int k = e / L, i = e % L;
            const float* col = s_tile + k * L;
            const float x = col[i];
            int r = 0;
#pragma unroll 16
            for (int j = 0; j < L; ++j) {
                const float u = col[j];
                r += (u < x || (u == x && j < i)) ? 1 : 0;
            }
            order[(int64_t)(f0 + k) * L + r] = (uint8_t)i;
        }
    }
    if (lead && t == 0) {
        jb.result[DDM_DFIT_STATUS] = 0;
        jb.result[DDM_DFIT_CLASSES] = K;
    }
#ifdef DDM_PREP_PROFILE
    __syncthreads();
    if (lead && t == 0)   // presort: start, classes done, end (10-ns ticks from the start)
        jb.result[10] = (int64_t)(tp0 | ((tp1 - tp0) << 40) | ((wall_clock64() - tp0) << 52));
#endif
}

// ---- k_dfit_trees -------------------------------------------------------------------
struct TreeLds {            // one tree's build state
    int32_t cnt[kMaxL];    // bootstrap multiplicity
    int16_t key[kMaxL];    // node key of each in-bag row (-1: out of bag)
    uint8_t crow[kMaxL];   // the node's rows in the current feature's order
    float cfv[kMaxL];      // their feature values
    int16_t feats[kMaxF];
    int16_t consts[kMaxF];
    int32_t ccnt[kMaxK];   // class weights of the node
    int16_t st_parent[kMaxL];
    uint8_t st_left[kMaxL];
    int16_t st_nconst[kMaxL];
    double st_imp[kMaxL];
};

struct WaveLds : TreeLds {
    uint32_t mt[624];      // raw MT state (RandomState drawn in the tree kernel itself)
};

struct Best {
    double proxy, thr, il, ir;
    int feature, pos, ml;
};

__device__ __forceinline__ int node_key(int parent, int is_left) {
    return parent < 0 ? 0 : 1 + 2 * parent + (is_left ? 0 : 1);
}

// The node's rows (key == nk) in ascending order of feature f: crow/cfv[0..n).
__device__ __forceinline__ int sort_feature(const int16_t* key, uint8_t* crow, float* cfv,
                                            const float* __restrict__ X, const uint8_t* __restrict__ order, int L,
                                            int F, int f, int nk, int lane) {
    int n = 0;
    for (int q0 = 0; q0 < L; q0 += 64) {
        const int q = q0 + lane;
        const int r = q < L ? order[(int64_t)f * L + q] : 0;
        const bool in = q < L && key[r] == nk;
        const uint64_t m = __ballot(in);
        if (in) {
            const int p = n + __popcll(m & lanemask_lt(lane));
            crow[p] = (uint8_t)r;
            cfv[p] = X[(int64_t)r * F + f];
        }
        n += __popcll(m);
    }
    wave_sync();
    return n;
}

__device__ void swap_feats(TreeLds& S, int a, int b) {
    const int16_t fa = S.feats[a], fb = S.feats[b];
    wave_sync();
    S.feats[a] = fb;
    S.feats[b] = fa;
    wave_sync();
}

// The best split position of one feature (rf_fit.cpp Builder::node_split, the body for one
// feature that is not constant): the node's n rows in the feature's order in crow / cfv.
// Every split position p in [1, n): left = positions [0, p).  Lane owns positions
// lane + 64k; the class weights left of every position come from wave prefix sums, three
// classes per sum (exact integers; absent classes add 0 to every sum), summed into
// sum-of-squares per position.  pos < 0: no split position.
struct FeatBest {
    double mx, thr, il, ir;
    int pos, ml;
};

__device__ __forceinline__ FeatBest eval_feature(const uint8_t* crow, const float* cfv, const int32_t* cnt,
                                                 const int32_t* ccnt, const uint8_t* __restrict__ yidx, int n, int K,
                                                 double wn_node, int lane) {
    constexpr int kR = kMaxL / 64;
    int wq[kR], cq[kR], wl[kR], sql[kR], sqr[kR];
    int carry = 0;
#pragma unroll
    for (int k = 0; k < kR; ++k) {
        const int q = 64 * k + lane;
        const bool inq = q < n;
        const int r = inq ? crow[q] : 0;
        wq[k] = inq ? cnt[r] : 0;
        cq[k] = inq ? (int)yidx[r] : -1;
        const int incl = wave_scan_i(wq[k], lane);
        wl[k] = carry + incl - wq[k];
        carry += wave_last_i(incl);
        sql[k] = 0;
        sqr[k] = 0;
    }
    // three classes per scan: 10-bit fields of one int (a field's running sum is at most the
    // node's weight <= L <= 256, so fields never carry into each other)
    for (int c0 = 0; c0 < K; c0 += 3) {
        const int t0 = ccnt[c0], t1 = c0 + 1 < K ? ccnt[c0 + 1] : 0, t2 = c0 + 2 < K ? ccnt[c0 + 2] : 0;
        if ((t0 | t1 | t2) == 0) continue;
        int cc = 0;
#pragma unroll
        for (int k = 0; k < kR; ++k) {
            if (64 * k >= n) break;
            const int d = cq[k] - c0;
            const int v = (d >= 0 && d < 3) ? wq[k] << (10 * d) : 0;
            const int incl = wave_scan_i(v, lane);
            const int slp = cc + incl - v;
            const int sl0 = slp & 1023, sl1 = (slp >> 10) & 1023, sl2 = (slp >> 20) & 1023;
            const int sr0 = t0 - sl0, sr1 = t1 - sl1, sr2 = t2 - sl2;
            sql[k] += sl0 * sl0 + sl1 * sl1 + sl2 * sl2;
            sqr[k] += sr0 * sr0 + sr1 * sr1 + sr2 * sr2;
            cc += wave_last_i(incl);
        }
    }
    double bp = -INFINITY, bil = 0.0, bir = 0.0;
    int bpos = -1;
#pragma unroll
    for (int k = 0; k < kR; ++k) {
        const int q = 64 * k + lane;
        const bool cand = q < n && q >= 1 && !(cfv[q] <= cfv[q - 1] + kFeatureThreshold);
        if (cand) {
            const double dwl = (double)wl[k], dwr = wn_node - dwl;
            const double il = 1.0 - (double)sql[k] / (dwl * dwl);
            const double ir = 1.0 - (double)sqr[k] / (dwr * dwr);
            const double proxy = (-dwr * ir) - dwl * il;
            if (proxy > bp) {                   // positions ascend within a lane
                bp = proxy;
                bpos = q;
                bil = il;
                bir = ir;
            }
        }
    }
    // first maximum over the wave: the largest proxy, then the smallest position
    const double mx = wave_max_d(bp);
    const int mpos = wave_min_i((bpos >= 0 && bp == mx) ? bpos : 0x7fffffff);
    FeatBest r{mx, 0.0, 0.0, 0.0, -1, 0};
    if (mpos != 0x7fffffff) {
        const int src = mpos & 63;                // the lane that owns position mpos (uniform)
        r.pos = mpos;
        r.il = readlane_d(bil, src);
        r.ir = readlane_d(bir, src);
        double thr = (double)cfv[mpos - 1] / 2.0 + (double)cfv[mpos] / 2.0;
        if (thr == (double)cfv[mpos] || thr == INFINITY || thr == -INFINITY) thr = (double)cfv[mpos - 1];
        r.thr = thr;
        r.ml = mpos > n - mpos ? 1 : 0;
    }
    return r;
}

// node_split_best without missing values (rf_fit.cpp Builder::node_split).
__device__ __forceinline__ Best node_split(TreeLds& S, const float* __restrict__ X, const uint8_t* __restrict__ order,
                           const uint8_t* __restrict__ yidx, int L, int F, int K, int max_features, int nk,
                           int n_node, double wn_node, uint32_t& rstate, int& n_const, int lane) {
    Best best{-INFINITY, 0.0, INFINITY, INFINITY, 0, -1, 0};
    int f_i = F, n_visited = 0, n_found_c = 0, n_drawn_c = 0;
    const int n_known_c = n_const;
    int n_total_c = n_known_c;
    while (f_i > n_total_c && (n_visited < max_features || n_visited <= n_found_c + n_drawn_c)) {
        ++n_visited;
        const int lo = n_drawn_c, hi = f_i - n_found_c;
        int f_j = lo + (int)((int64_t)our_rand_r(rstate) % (hi - lo));
        if (f_j < n_known_c) {
            swap_feats(S, n_drawn_c, f_j);
            ++n_drawn_c;
            continue;
        }
        f_j += n_found_c;
        const int feature = S.feats[f_j];
        const int n = sort_feature(S.key, S.crow, S.cfv, X, order, L, F, feature, nk, lane);
        if (n == 0 || S.cfv[n - 1] <= S.cfv[0] + kFeatureThreshold) {
            swap_feats(S, f_j, n_total_c);
            ++n_found_c;
            ++n_total_c;
            continue;
        }
        --f_i;
        swap_feats(S, f_i, f_j);
        const FeatBest fb = eval_feature(S.crow, S.cfv, S.cnt, S.ccnt, yidx, n, K, wn_node, lane);
        if (fb.pos >= 0 && fb.mx > best.proxy) {
            best.proxy = fb.mx;
            best.pos = fb.pos;
            best.feature = feature;
            best.il = fb.il;
            best.ir = fb.ir;
            best.thr = fb.thr;
            best.ml = fb.ml;
        }
    }
    // features[0:n_known_c] = constant[0:n_known_c];
    // constant[n_known_c:n_known_c+n_found_c] = features[n_known_c:n_known_c+n_found_c]
    wave_sync();
    for (int k = lane; k < n_known_c; k += 64) S.feats[k] = S.consts[k];
    for (int k = lane; k < n_found_c; k += 64) S.consts[n_known_c + k] = S.feats[n_known_c + k];
    wave_sync();
    n_const = n_total_c;
    return best;
}

// One tree, one wave; mt: RandomState drawn here (boot == nullptr, the fused kernel).
__device__ __forceinline__ void build_tree(const Job& jb, const Layout& lo, int tree, int K, TreeLds& S, int lane,
                                           const float* __restrict__ X, const uint8_t* __restrict__ order,
                                           const uint8_t* __restrict__ yidx, const int32_t* __restrict__ boot,
                                           uint32_t* mt) {
    const int L = jb.L, F = jb.F;
    const int64_t M = 2 * (int64_t)L - 1;
    gptr<TNode> nodes = (gptr<TNode>)(jb.scratch + lo.tnodes) + tree * M;
    gptr<double> vals = (gptr<double>)(jb.scratch + lo.tvals) + tree * M * jb.k_cap;
    gptr<int32_t> meta = (gptr<int32_t>)(jb.scratch + lo.tmeta) + 4 * tree;

#ifdef DDM_DFIT_PROFILE
    const uint64_t t_a = wall_clock64();
#endif
    // ---- RandomState(seed), the splitter seed and the bootstrap counts: drawn by
    // k_dfit_prep's boot workgroups beside the presort when it ran (boot != nullptr)
    uint32_t rstate = 0;
    if (boot) {
        const int32_t* bt = boot + (int64_t)tree * (L + 1);
        for (int k = lane; k < L; k += 64) S.cnt[k] = bt[1 + k];
        rstate = (uint32_t)bt[0];
        wave_sync();
    } else {
        rstate = tree_boot((uint32_t)jb.seeds[tree], L, (lptr<uint32_t>)mt, (lptr<int32_t>)S.cnt, lane);
    }
#ifdef DDM_DFIT_PROFILE
    const uint64_t t_a1 = wall_clock64();
    const uint64_t t_b = t_a1;
#endif
    for (int k = lane; k < L; k += 64) S.key[k] = S.cnt[k] > 0 ? 0 : -1;
    for (int f = lane; f < F; f += 64) S.feats[f] = (int16_t)f;
    wave_sync();
#ifdef DDM_DFIT_PROFILE
    const uint64_t t_c = wall_clock64();
#endif
    const double wns = (double)L;               // weighted_n_samples = sum of the counts
    // ---- depth-first build (rf_fit.cpp Builder::build)
    int sp = 0, n_nodes = 0, n_leaves = 0, impure = 0;
    if (lane == 0) {
        S.st_parent[0] = -1;
        S.st_left[0] = 0;
        S.st_nconst[0] = 0;
        S.st_imp[0] = INFINITY;
    }
    sp = 1;
    bool first = true;
    wave_sync();
    while (sp > 0) {
        --sp;
        const int parent = S.st_parent[sp], is_left = S.st_left[sp];
        int n_const = S.st_nconst[sp];
        const double rimp = S.st_imp[sp];
        const int nk = node_key(parent, is_left);
        wave_sync();
        // crit_init: class weights and row count of the node
        for (int c = lane; c < K; c += 64) S.ccnt[c] = 0;
        wave_sync();
        int my_n = 0;
        for (int r = lane; r < L; r += 64)
            if (S.key[r] == nk) {
                atomicAdd(&S.ccnt[yidx[r]], S.cnt[r]);
                ++my_n;
            }
        const int n_node = wave_sum_i(my_n);
        wave_sync();
        double wn_node = 0.0;
        for (int c = 0; c < K; ++c) wn_node += (double)S.ccnt[c];
        bool is_leaf = n_node < 2 || wn_node < 0.0;
        double impurity = rimp;
        if (first) {
            double sq = 0.0;
            for (int c = 0; c < K; ++c) sq += (double)S.ccnt[c] * (double)S.ccnt[c];
            impurity = (1.0 - sq / (wn_node * wn_node)) / 1.0;
            first = false;
        }
        is_leaf = is_leaf || impurity <= kEpsilon;
        Best sp_best{-INFINITY, 0.0, INFINITY, INFINITY, 0, -1, 0};
        double improvement = -INFINITY;
        if (!is_leaf) {
            sp_best = node_split(S, X, order, yidx, L, F, K, jb.max_features, nk, n_node, wn_node, rstate, n_const,
                                 lane);
            if (sp_best.pos >= 0) {
                const double wl = [&] {
                    // weight of the rows left of the split = rows with x <= thr
                    int w = 0;
                    for (int r = lane; r < L; r += 64)
                        if (S.key[r] == nk && (double)X[(int64_t)r * F + sp_best.feature] <= sp_best.thr) w += S.cnt[r];
                    return (double)wave_sum_i(w);
                }();
                const double wr = wn_node - wl;
                improvement = (wn_node / wns) *
                              (impurity - (wr / wn_node * sp_best.ir) - (wl / wn_node * sp_best.il));
            }
            is_leaf = sp_best.pos < 0 || improvement + kEpsilon < 0.0;
        }
        const int id = n_nodes++;
        if (lane == 0) {
            TNode nd;
            nd.left = -1;
            nd.right = -1;
            nd.feature = (int16_t)(is_leaf ? -2 : sp_best.feature);
            nd.missing_left = (uint8_t)(sp_best.pos >= 0 ? sp_best.ml : 0);
            int lc = 0;                              // first argmax of the class weights
            for (int c = 1; c < K; ++c)
                if (S.ccnt[c] > S.ccnt[lc]) lc = c;
            nd.leaf = (uint8_t)(is_leaf ? 1 + lc : 0);   // 1 + leaf class, 0: internal
            nd.threshold = is_leaf ? -2.0 : sp_best.thr;
            gput(nodes + id, nd);
            if (parent >= 0) {
                if (is_left) nodes[parent].left = (int16_t)id;
                else nodes[parent].right = (int16_t)id;
            }
        }
        for (int c = lane; c < K; c += 64) vals[id * (int64_t)jb.k_cap + c] = (double)S.ccnt[c] / wn_node;
        if (is_leaf) {
            ++n_leaves;
            int nz = 0, ones = 0;
            for (int c = 0; c < K; ++c) {
                nz += S.ccnt[c] != 0;
                ones += (double)S.ccnt[c] / wn_node == 1.0;
            }
            impure |= !(ones == 1 && nz == 1);
        } else {
            const int kl = node_key(id, 1), kr = node_key(id, 0);
            for (int r = lane; r < L; r += 64)
                if (S.key[r] == nk)
                    S.key[r] = (int16_t)((double)X[(int64_t)r * F + sp_best.feature] <= sp_best.thr ? kl : kr);
            if (lane == 0) {
                S.st_parent[sp] = (int16_t)id;
                S.st_left[sp] = 0;
                S.st_nconst[sp] = (int16_t)n_const;
                S.st_imp[sp] = sp_best.ir;
                S.st_parent[sp + 1] = (int16_t)id;
                S.st_left[sp + 1] = 1;
                S.st_nconst[sp + 1] = (int16_t)n_const;
                S.st_imp[sp + 1] = sp_best.il;
            }
            sp += 2;
        }
        wave_sync();
    }
    if (lane == 0) {
        meta[0] = n_nodes;
        meta[1] = n_leaves;
        meta[2] = impure;
#ifdef DDM_DFIT_PROFILE
        if (tree == 0)   // rng init | bootstrap | build, 10-ns ticks
            jb.result[10] = (int64_t)((t_b - t_a) | ((t_c - t_b) << 16) | (((wall_clock64() - t_c) & 0xffff) << 32) |
                                      ((t_a1 - t_a) << 48));
#endif
    }
}

// X, the presorted orders and the class indices are staged in LDS for the workgroup's
// trees when they fit (L*F <= kTreeTile); otherwise the builder reads them from HBM.
constexpr int kTreeTile = 4096;

// Small jobs (L*F <= kTreeTile, the controller's refits: 100 rows x 27 features) skip
// k_dfit_prep: every workgroup gates, checks and presorts the batch itself in LDS (the
// ~270k rank comparisons of a 100 x 27 batch are ~1k per thread), and workgroup 0 writes
// the job's status, classes_ and class count for k_dfit_pack.  One launch fewer per refit.
template <bool kFused>
__device__ __forceinline__ bool fused_prep(const Job& jb, float* s_X, uint8_t* s_ord, uint8_t* s_yi, int& K_out) {
    __shared__ int32_t s_y[kMaxL];
    __shared__ uint8_t s_first[kMaxL];
    __shared__ int s_nan, s_K, s_skip;
    const int t = threadIdx.x;
    constexpr int kT = 64 * kWaves;
    const bool lead = blockIdx.x == 0;
    if (t == 0) {
        s_skip = gated_off(jb);
        s_nan = 0;
        s_K = 0;
    }
    __syncthreads();
    if (s_skip) return false;                    // the result words keep the last refit's
    const int L = jb.L, F = jb.F;
    if (L < 1 || L > kMaxL || F < 1 || F > kMaxF || jb.n_trees < 1 || jb.n_trees > 256 || jb.k_cap < 1 ||
        jb.k_cap > kMaxK || jb.max_features < 1) {
        if (lead && t == 0) jb.result[DDM_DFIT_STATUS] = DDM_E_ARG;
        return false;
    }
    const int LF = L * F;
    for (int e = t; e < LF; e += kT) {
        const float x = jb.X[e];
        s_X[e] = x;
        if (x != x) s_nan = 1;
    }
    if (t < L) s_y[t] = jb.y[t];
    __syncthreads();
    // classes_ = np.unique(y): first occurrences ranked by value
    if (t < L) {
        int first = 1;
        for (int j = 0; j < t; ++j) first &= s_y[j] != s_y[t];
        s_first[t] = (uint8_t)first;
        if (first) atomicAdd(&s_K, 1);
    }
    __syncthreads();
    const int K = s_K;
    if (t < L) {
        int rank = 0;
        for (int j = 0; j < L; ++j) rank += (s_first[j] && s_y[j] < s_y[t]) ? 1 : 0;
        s_yi[t] = (uint8_t)min(rank, 255);
        if (lead && s_first[t] && rank < jb.k_cap) jb.classes[rank] = s_y[t];
    }
    if (s_nan || K > jb.k_cap) {
        if (lead && t == 0) {
            jb.result[DDM_DFIT_STATUS] = s_nan ? DDM_E_NAN : DDM_E_FOREST;
            jb.result[DDM_DFIT_CLASSES] = K;
        }
        return false;
    }
    // presorted orders (stable rank of every row in every feature), straight into LDS
    for (int e = t; e < LF; e += kT) {
        const int k = e / L, i = e % L;
        const float x = s_X[i * F + k];
        int r = 0;
        for (int j = 0; j < L; ++j) {
            const float u = s_X[j * F + k];
            r += (u < x || (u == x && j < i)) ? 1 : 0;
        }
        s_ord[k * L + r] = (uint8_t)i;
    }
    if (lead && t == 0) {
        jb.result[DDM_DFIT_STATUS] = 0;
        jb.result[DDM_DFIT_CLASSES] = K;
    }
    __syncthreads();
    K_out = K;
    return true;
}

template <bool kFused>
__global__ __launch_bounds__(64 * kWaves) void k_dfit_trees(const Job* __restrict__ jobs) {
    __shared__ WaveLds lds[kWaves];
    __shared__ float s_X[kTreeTile];
    __shared__ uint8_t s_ord[kTreeTile];
    __shared__ uint8_t s_yi[kMaxL];
    refit_priority();
    const Job jb = jobs[blockIdx.y];
    const int w = threadIdx.x / 64, lane = threadIdx.x & 63;
    const int tree = blockIdx.x * kWaves + w;
    if constexpr (kFused) {
        int K = 0;
        if (!fused_prep<true>(jb, s_X, s_ord, s_yi, K)) return;
        const Layout lo = layout(jb.L, jb.F, jb.n_trees, jb.k_cap);
        if (tree < jb.n_trees) build_tree(jb, lo, tree, K, lds[w], lane, s_X, s_ord, s_yi, nullptr, lds[w].mt);
        return;
    }
    if (gated_off(jb) || jb.result[DDM_DFIT_STATUS] != 0) return;
    const int K = (int)jb.result[DDM_DFIT_CLASSES];
    const Layout lo = layout(jb.L, jb.F, jb.n_trees, jb.k_cap);
    const int LF = jb.L * jb.F;
    const uint8_t* yidx = (const uint8_t*)(jb.scratch + lo.yidx);
    const uint8_t* order = (const uint8_t*)(jb.scratch + lo.order);
    const int32_t* boot = (const int32_t*)(gptr<const int32_t>)(jb.scratch + lo.boot);
    if (LF <= kTreeTile) {
        for (int e = threadIdx.x; e < LF; e += 64 * kWaves) {
            s_X[e] = jb.X[e];
            s_ord[e] = order[e];
        }
        for (int e = threadIdx.x; e < jb.L; e += 64 * kWaves) s_yi[e] = yidx[e];
        __syncthreads();
        if (tree < jb.n_trees) build_tree(jb, lo, tree, K, lds[w], lane, s_X, s_ord, s_yi, boot, nullptr);
    } else if (tree < jb.n_trees) {
        build_tree(jb, lo, tree, K, lds[w], lane, (const float*)jb.X, order, yidx, boot, nullptr);
    }
}

// ---- k_dfit_pack: BFS packing (rf_fit.cpp pack_trees) and the forest compiler ----------
__device__ float float_floor_of(double t) {
    float f = (float)t;
    if ((double)f > t) f = nextafterf(f, -INFINITY);
    return f;
}

__device__ __forceinline__ void inc_vote(int c, uint32_t* v) { atomicAdd(&v[c >> 2], 1u << (8 * (c & 3))); }
__device__ __forceinline__ uint32_t vote_word(int c, int j) { return (c >> 2) == j ? 1u << (8 * (c & 3)) : 0u; }

constexpr int kPackThreads = 256;
constexpr int kPackLdsNodes = 1024;          // forests up to this many nodes are packed in LDS

// Block-wide exclusive prefix sum of one int per thread (kPackThreads threads): a wave
// scan (DPP), then the wave totals through LDS (two barriers).
__device__ int block_scan_excl(int v, int* tmp, int& total) {
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int inc = wave_scan_i(v, lane);
    if (lane == 63) tmp[wv] = inc;
    __syncthreads();
    int base = 0, all = 0;
#pragma unroll
    for (int w = 0; w < kPackThreads / 64; ++w) {
        const int x = tmp[w];
        base += w < wv ? x : 0;
        all += x;
    }
    total = all;
    __syncthreads();
    return base + inc - v;
}

// ddm_forest_compile (forest_compile.cpp) for a pure forest given as creation-order tree
// nodes, by the whole workgroup.  The blob is byte for byte the host compiler's:
//   * slots in order of first use over (tree, pre-order internal node): a min-key per
//     column, ranked;
//   * stumps stable-sorted by (NaN-left, slot) and, per slot, by threshold: ranks by
//     counting; rank-table entries are sums over the ranked stumps;
//   * general trees: internal nodes and leaves in pre-order (the host's post-order walk
//     emits nodes on entry and numbers leaves left to right); the left-subtree leaf mask
//     of node u covers the leaves with ids in [u + 1, right(u)).
// Returns the blob size, or 0 when the forest does not compile.
// tn_lds: when not null, this thread's tree (> 3 nodes) is at tn_lds[my_base ...] in LDS and
// lrank_lds[my_base ...] is its scratch (k_dfit_pack copied it there)
__device__ int64_t compile_forest(const TNode* tn, int64_t M, const int32_t* meta, int T, const int32_t* classes,
                                  int K, int F, int16_t* lrank, uint8_t* out, int64_t cap, const TNode* tn_lds,
                                  int16_t* lrank_lds, int my_base) {
    __shared__ int s_tmp[kPackThreads];
    __shared__ uint32_t s_first[kMaxF];
    __shared__ int16_t s_slot_of[kMaxF];
    __shared__ int s_cols[kMaxSlots];
    __shared__ uint8_t s_kind[256];
    __shared__ int16_t s_col[256], s_cl[256], s_cr[256], s_srank[256], s_prank[256], s_sid[256];
    __shared__ uint8_t s_nl[256];
    __shared__ float s_thr[256];
    __shared__ int16_t s_skey[256];
    __shared__ float s_sthr[256];
    __shared__ uint32_t s_key32[256];
    __shared__ uint64_t s_pkey[256];
    __shared__ uint32_t s_sdel[256][4];
    __shared__ uint32_t s_rtab[kMaxTabWords];
    __shared__ int s_gnode[256], s_gleaf[256], s_gtree[256], s_nint[256], s_nlv[256];
    __shared__ int s_m[kMaxSlots], s_n4[kMaxSlots], s_tab[kMaxSlots], s_xq[kMaxSlots];
    __shared__ uint32_t s_base[4];
    __shared__ int s_bad, s_anynl, s_U;
    __shared__ int64_t s_off[8];
#ifdef DDM_DFIT_PROFILE
    __shared__ uint64_t s_prof[4];
    if (threadIdx.x == 0) s_prof[0] = wall_clock64();
#endif
    const int t = threadIdx.x;
    if (T > 255 || K > 16) return 0;
    const int vr = K <= 4 ? 1 : K <= 8 ? 2 : 4;
    for (int f = t; f < F; f += kPackThreads) s_first[f] = 0xffffffffu;
    if (t < 4) s_base[t] = 0;
    if (t == 0) {
        s_bad = 0;
        s_anynl = 0;
    }
    if (t < kMaxSlots) s_m[t] = 0;
    __syncthreads();
    // ---- A: classify every tree
    int kind = 3, nint = 0, nlv = 0;
    if (t < T) {
        const TNode* nd = tn_lds && meta[4 * t] > 3 ? tn_lds + my_base : tn + t * M;
        const int n = meta[4 * t];
        const TNode r = nd[0];
        if (r.leaf) {
            kind = 0;
            inc_vote(r.leaf - 1, s_base);
        } else if (n == 3 && nd[1].leaf && nd[2].leaf) {
            kind = 1;
            s_col[t] = r.feature;
            s_thr[t] = float_floor_of(r.threshold);
            s_cl[t] = nd[1].leaf - 1;
            s_cr[t] = nd[2].leaf - 1;
            s_nl[t] = r.missing_left;
            if (r.missing_left) s_anynl = 1;
            inc_vote(nd[1].leaf - 1, s_base);
            atomicMin(&s_first[r.feature], (uint32_t)t << 9);
        } else {
            kind = 2;
            for (int u = 0; u < n; ++u) {
                const TNode x = nd[u];
                if (x.leaf) {
                    ++nlv;
                } else {
                    atomicMin(&s_first[x.feature], ((uint32_t)t << 9) | (uint32_t)nint);
                    if (x.missing_left) s_anynl = 1;
                    ++nint;
                }
            }
            if (nlv > kMaxCfLeaves) s_bad = 1;
        }
        s_kind[t] = (uint8_t)kind;
    }
    s_nint[t] = kind == 2 ? nint : 0;
    s_nlv[t] = kind == 2 ? nlv : 0;
    __syncthreads();
#ifdef DDM_DFIT_PROFILE
    if (threadIdx.x == 0) s_prof[1] = wall_clock64();
#endif
    // ---- B: slots
    int used = 0;
    for (int f = t; f < F; f += kPackThreads) used += s_first[f] != 0xffffffffu;
    int U = 0;
    block_scan_excl(used, s_tmp, U);
    for (int f = t; f < F; f += kPackThreads) {
        if (s_first[f] == 0xffffffffu) continue;
        int r = 0;
#pragma unroll 8
        for (int g = 0; g < F; ++g) r += s_first[g] < s_first[f];
        s_slot_of[f] = (int16_t)r;
        if (r < kMaxSlots) s_cols[r] = f;
    }
    if (U > kMaxSlots) return 0;
    // ---- C: stump ids, general-tree offsets
    int S = 0, n_gtrees = 0, n_gnodes = 0, n_leaf = 0;
    const int sid = block_scan_excl(t < T && kind == 1 ? 1 : 0, s_tmp, S);
    const int gid = block_scan_excl(t < T && kind == 2 ? 1 : 0, s_tmp, n_gtrees);
    const int goff = block_scan_excl(s_nint[t], s_tmp, n_gnodes);
    const int loff = block_scan_excl(s_nlv[t], s_tmp, n_leaf);
    if (s_bad) return 0;
    if (t < T && kind == 1) s_sid[sid] = (int16_t)t;   // stump sid -> tree
    if (t < T && kind == 2) {
        s_gtree[t] = gid;
        s_gnode[t] = goff;
        s_gleaf[t] = loff;
    }
    __syncthreads();
    // per stump (by sid): sort key (nanleft, slot), threshold, delta words
    if (t < S) {
        const int ti = s_sid[t];
        const int sl = s_slot_of[s_col[ti]];
        s_skey[t] = (int16_t)(s_nl[ti] * kMaxSlots + sl);
        s_sthr[t] = s_thr[ti];
        for (int w = 0; w < 4; ++w) s_sdel[t][w] = vote_word(s_cr[ti], w) - vote_word(s_cl[ti], w);
        atomicAdd(&s_m[sl], 1);
    }
    __syncthreads();
    // stump ranks: sorted by (nanleft, slot, sid); per slot by (threshold, sorted rank).
    // Both are counts of smaller packed keys (distinct by construction), over the keys
    // padded to a multiple of 8 with the largest key: 8 broadcast LDS reads per round
    const int S8 = (S + 7) & ~7;
    if (t < S8) s_key32[t] = t < S ? ((uint32_t)s_skey[t] << 16) | (uint32_t)t : 0xffffffffu;
    __syncthreads();
    if (t < S) {
        const uint32_t key = s_key32[t];
        int r = 0;
#pragma unroll 8
        for (int j = 0; j < S8; ++j) r += s_key32[j] < key ? 1 : 0;
        s_srank[t] = (int16_t)r;
        // (slot, threshold as an order-preserving u32 (-0 as +0), sorted rank)
        const float th = s_sthr[t];
        const uint32_t b = th == 0.0f ? 0u : __float_as_uint(th);
        const uint32_t ob = (b & 0x80000000u) ? ~b : (b | 0x80000000u);
        s_pkey[t] = ((uint64_t)(s_skey[t] % kMaxSlots) << 56) | ((uint64_t)ob << 24) | (uint64_t)r;
    } else if (t < S8) {
        s_pkey[t] = ~0ull;
    }
    __syncthreads();
    if (t < S) {
        // rank within the slot = smaller keys - keys of lower slots
        const uint64_t key = s_pkey[t];
        const uint64_t lo = key & ~((1ull << 56) - 1);
        int r = 0;
#pragma unroll 8
        for (int j = 0; j < S8; ++j) {
            const uint64_t kj = s_pkey[j];
            r += (kj < key ? 1 : 0) - (kj < lo ? 1 : 0);
        }
        s_prank[t] = (int16_t)r;
    }
    if (t == 0) {
        int tab = 0, xq = 0;
        for (int sl = 0; sl < U; ++sl) {
            const int m = s_m[sl];
            s_n4[sl] = m ? m / 4 + 1 : 0;
            s_tab[sl] = tab;
            s_xq[sl] = xq;
            if (m) {
                tab += 4 * s_n4[sl] + 1;
                xq += s_n4[sl] - 1;
            }
        }
        const int sw = vr <= 2 ? 4 : 8;
        const int n_srec = (U + 7) & ~7;
        s_off[0] = al16(sizeof(ddm_cforest_head));                                        // stumps
        s_off[1] = al16(s_off[0] + 4 * (int64_t)S * sw);                                   // trees
        s_off[2] = al16(s_off[1] + (int64_t)sizeof(ddm_cforest_tree) * n_gtrees);          // nodes
        s_off[3] = al16(s_off[2] + (int64_t)sizeof(ddm_cforest_node) * n_gnodes);          // leaf cls
        s_off[4] = al16(s_off[3] + n_leaf);                                                 // slots
        s_off[5] = al16(s_off[4] + (int64_t)sizeof(ddm_cforest_slot) * n_srec);            // xthr
        s_off[6] = al16(s_off[5] + 16 * (int64_t)xq);                                      // tables
        s_off[7] = al16(s_off[6] + 4 * (int64_t)tab * vr);                                 // total
        s_U = tab;                                                                         // entries
    }
    __syncthreads();
    const int64_t total = s_off[7];
#ifdef DDM_DFIT_PROFILE
    if (threadIdx.x == 0) s_prof[2] = wall_clock64();
#endif
    const int n_entries = s_U;
    if (total > cap || n_entries * vr > kMaxTabWords) return 0;
    // ---- D: write the blob
    for (int64_t k = t; k < total / 16; k += kPackThreads) reinterpret_cast<uint4*>(out)[k] = uint4{0, 0, 0, 0};
    __syncthreads();
#ifdef DDM_DFIT_PROFILE
    if (threadIdx.x == 0) s_prof[3] = wall_clock64();
#endif
    ddm_cforest_head* h = reinterpret_cast<ddm_cforest_head*>(out);
    const int n_right = __syncthreads_count(t < S && s_nl[s_sid[t]] == 0);   // stumps sending NaN right
    const int sw = vr <= 2 ? 4 : 8;
    if (t == 0) {
        h->n_slots = U;
        h->n_classes = K;
        h->vote_regs = vr;
        h->n_stumps = S;
        h->n_general = n_gtrees;
        h->n_leaves = n_leaf;
        h->total_bytes = (int)total;
        h->any_nanleft = s_anynl;
        h->stumps_off = (int)s_off[0];
        h->stump_words = sw;
        h->trees_off = (int)s_off[1];
        h->nodes_off = (int)s_off[2];
        h->leafcls_off = (int)s_off[3];
        for (int k = 0; k < 4; ++k) h->base_votes[k] = s_base[k];
        h->n_stumps_right = n_right;
        h->slots_off = (int)s_off[4];
        h->xthr_off = (int)s_off[5];
        h->rank_tab_off = (int)s_off[6];
        h->rank_tab_entries = n_entries;
    }
    if (t < kMaxSlots) h->cols[t] = U == 0 ? 0 : s_cols[t < U ? t : U - 1];
    if (t < K) h->classes[t] = classes[t];
    // stump records
    if (t < S) {
        const int ti = s_sid[t];
        uint32_t* rec = reinterpret_cast<uint32_t*>(out + s_off[0]) + (int64_t)s_srank[t] * sw;
        rec[0] = __float_as_uint(s_thr[ti]);
        rec[1] = (uint32_t)s_slot_of[s_col[ti]];
        for (int j = 0; j < vr; ++j) rec[2 + j] = vote_word(s_cr[ti], j) - vote_word(s_cl[ti], j);
    }
    // slot records and thresholds
    ddm_cforest_slot* srec = reinterpret_cast<ddm_cforest_slot*>(out + s_off[4]);
    float* xthr = reinterpret_cast<float*>(out + s_off[5]);
    const int n_srec = (U + 7) & ~7;
    if (t < n_srec) {
        ddm_cforest_slot rs;
        rs.col = U == 0 ? 0 : s_cols[t < U ? t : U - 1];
        rs.n4 = t < U ? s_n4[t] : 0;
        rs.tab = t < U ? s_tab[t] : 0;
        rs.xthr = t < U ? s_xq[t] : 0;
        for (int q = 0; q < 4; ++q) rs.thr[q] = t < U ? INFINITY : 0.0f;
        srec[t] = rs;
    }
    __syncthreads();
    if (t < S) {
        const int ti = s_sid[t];
        const int sl = s_slot_of[s_col[ti]], q = s_prank[t];
        if (q < 4) srec[sl].thr[q] = s_thr[ti];
        else xthr[4 * s_xq[sl] + (q - 4)] = s_thr[ti];
    }
    for (int sl = 0; sl < U; ++sl) {                          // +inf pads past m
        const int m = s_m[sl];
        for (int q = max(m, 4) + t; q < 4 * s_n4[sl]; q += kPackThreads) xthr[4 * s_xq[sl] + (q - 4)] = INFINITY;
    }
    // rank tables: entry q < 4*n4: deltas of the min(q, m) lowest; entry 4*n4: NaN.
    // Each stump adds its delta to the entries above its rank (and to the NaN entry when
    // it sends NaN right): wrapping u32 sums, so the order of the additions is free.
    uint32_t* rtab = reinterpret_cast<uint32_t*>(out + s_off[6]);
    for (int k = t; k < n_entries * vr; k += kPackThreads) s_rtab[k] = 0;
    __syncthreads();
    if (t < S) {
        const int sl = s_skey[t] % kMaxSlots, q0 = s_prank[t];
        const int ne = 4 * s_n4[sl] + 1;
        uint32_t* e = s_rtab + (int64_t)s_tab[sl] * vr;
        for (int q = q0 + 1; q < ne - 1; ++q)
            for (int w = 0; w < vr; ++w) atomicAdd(&e[q * vr + w], s_sdel[t][w]);
        if (s_skey[t] < kMaxSlots)                      // nanleft == 0
            for (int w = 0; w < vr; ++w) atomicAdd(&e[(ne - 1) * vr + w], s_sdel[t][w]);
    }
    __syncthreads();
    for (int k = t; k < n_entries * vr; k += kPackThreads) rtab[k] = s_rtab[k];
    // general trees: one thread per tree
    if (t < T && kind == 2) {
        const TNode* nd = tn_lds && meta[4 * t] > 3 ? tn_lds + my_base : tn + t * M;
        const int n = meta[4 * t];
        int16_t* lr = tn_lds ? lrank_lds + my_base : lrank + t * M;   // leaves before node u
        int c = 0;
        for (int u = 0; u < n; ++u) {
            lr[u] = (int16_t)c;
            c += nd[u].leaf ? 1 : 0;
        }
        ddm_cforest_tree tr;
        tr.node_begin = s_gnode[t];
        tr.n_nodes = nint;
        tr.leaf_begin = s_gleaf[t];
        tr.n_leaves = nlv;
        reinterpret_cast<ddm_cforest_tree*>(out + s_off[1])[s_gtree[t]] = tr;
        ddm_cforest_node* gn = reinterpret_cast<ddm_cforest_node*>(out + s_off[2]) + s_gnode[t];
        uint8_t* lc = out + s_off[3] + s_gleaf[t];
        int ki = 0, kl = 0;
        for (int u = 0; u < n; ++u) {
            const TNode x = nd[u];
            if (x.leaf) {
                lc[kl++] = (uint8_t)(x.leaf - 1);
                continue;
            }
            const int lo = lr[u + 1], hi = lr[x.right];
            const uint64_t m = (hi - lo >= 64 ? ~0ull : ((1ull << (hi - lo)) - 1)) << lo;
            ddm_cforest_node cn;
            cn.threshold = float_floor_of(x.threshold);
            cn.slot_nanleft = s_slot_of[x.feature] | (x.missing_left << 8);
            cn.left_lo = (uint32_t)m;
            cn.left_hi = (uint32_t)(m >> 32);
            gn[ki++] = cn;
        }
    }
#ifdef DDM_DFIT_PROFILE
    if (threadIdx.x == 0) {   // 8-bit fields in 80 ns: A, B-C, zero fill, D
        const uint64_t e = wall_clock64();
        const auto f8 = [](uint64_t dt) { return min((uint64_t)255, dt >> 3); };
        s_prof[0] = f8(s_prof[1] - s_prof[0]) | (f8(s_prof[2] - s_prof[1]) << 8) | (f8(s_prof[3] - s_prof[2]) << 16) |
                    (f8(e - s_prof[3]) << 24);
        *reinterpret_cast<uint32_t*>(lrank) = (uint32_t)s_prof[0];
    }
#endif
    return total;
}

__device__ void pack_tree(const TNode* tn, int m, int16_t* new_id, int16_t* queue, gptr<ddm_node> out, int64_t base,
                          bool pure, gptr<const double> vals, int K, int kcap, gptr<double> leaf_value, int64_t leaf_row) {
    if (m <= 3) {
        // a single leaf or a stump: pre-order ids are already the BFS ids (C3's trees), so
        // no queue; the nodes are loaded before anything is stored
        TNode xs[3];
#pragma unroll
        for (int u = 0; u < 3; ++u) xs[u] = tn[u < m ? u : 0];
#pragma unroll
        for (int u = 0; u < 3; ++u) {
            if (u >= m) break;
            const TNode x = xs[u];
            ddm_node nd;
            if (x.left != -1) {
                nd.threshold = x.threshold;
                nd.feature = x.feature | (x.missing_left ? (1 << 30) : 0);
                nd.child = (int32_t)(base + x.left);
            } else {
                nd.threshold = 0.0;
                nd.feature = -1;
                if (pure) {
                    nd.child = x.leaf - 1;
                } else {
                    for (int c = 0; c < K; ++c) leaf_value[leaf_row * K + c] = vals[(int64_t)u * kcap + c];
                    nd.child = (int32_t)leaf_row++;
                }
            }
            gput(out + base + u, nd);
        }
        return;
    }
    int head = 0, tail = 0, nxt = 1;
    queue[tail++] = 0;
    new_id[0] = 0;
    while (head < tail) {
        const int u = queue[head++];
        if (tn[u].left != -1) {
            new_id[tn[u].left] = (int16_t)nxt;
            new_id[tn[u].right] = (int16_t)(nxt + 1);
            queue[tail++] = tn[u].left;
            queue[tail++] = tn[u].right;
            nxt += 2;
        }
    }
    for (int u = 0; u < m; ++u) {
        const TNode x = tn[u];
        ddm_node nd;
        if (x.left != -1) {
            nd.threshold = x.threshold;
            nd.feature = x.feature | (x.missing_left ? (1 << 30) : 0);
            nd.child = (int32_t)(base + new_id[x.left]);
        } else {
            nd.threshold = 0.0;
            nd.feature = -1;
            if (pure) {
                nd.child = x.leaf - 1;
            } else {
                for (int c = 0; c < K; ++c) leaf_value[leaf_row * K + c] = vals[(int64_t)u * kcap + c];
                nd.child = (int32_t)leaf_row++;
            }
        }
        gput(out + base + new_id[u], nd);
    }
}

__device__ __forceinline__ void pack_job(const Job& jb) {
#ifdef DDM_DFIT_PROFILE
    const uint64_t t_pack0 = wall_clock64();
#endif
    if (gated_off(jb) || jb.result[DDM_DFIT_STATUS] != 0) return;
    const int t = threadIdx.x;
    const int T = jb.n_trees, K = (int)jb.result[DDM_DFIT_CLASSES];
    const Layout lo = layout(jb.L, jb.F, T, jb.k_cap);
    const int64_t M = 2 * (int64_t)jb.L - 1;
    gptr<const int32_t> meta = (gptr<const int32_t>)(jb.scratch + lo.tmeta);
    gptr<const TNode> tn = (gptr<const TNode>)(jb.scratch + lo.tnodes);
    gptr<const double> tv = (gptr<const double>)(jb.scratch + lo.tvals);
    gptr<int16_t> bfs = (gptr<int16_t>)(jb.scratch + lo.bfs);
    __shared__ int s_tmp[kPackThreads];
    __shared__ int s_impure;
    __shared__ TNode s_tn[kPackLdsNodes];
    __shared__ int16_t s_bid[2 * kPackLdsNodes];
    if (t == 0) s_impure = 0;
    __syncthreads();
    const int nn = t < T ? meta[4 * t] : 0;
    const int nl = t < T ? meta[4 * t + 1] : 0;
    if (t < T && meta[4 * t + 2]) s_impure = 1;
    int n_nodes = 0, n_leaf = 0;
    const int base = block_scan_excl(nn, s_tmp, n_nodes);
    const int lbase = block_scan_excl(nl, s_tmp, n_leaf);
    const bool pure = T <= 255 && !s_impure;
    if (t < T) {
        if (nn > 3 && n_nodes <= kPackLdsNodes) {
            // the tree's nodes, its BFS ids and queue in LDS (each thread its own range): the
            // queue walk and the node loop wait on LDS, not on a global round trip per node
#pragma unroll 4
            for (int u = 0; u < nn; ++u) s_tn[base + u] = gget(tn + t * M + u);
            pack_tree(s_tn + base, nn, s_bid + base, s_bid + n_nodes + base, jb.nodes, base, pure,
                      tv + t * M * jb.k_cap, K, jb.k_cap, jb.leaf_value, lbase);
        } else {
            pack_tree((const TNode*)(tn + t * M), nn, (int16_t*)(bfs + 2 * t * M), (int16_t*)(bfs + 2 * t * M + M), jb.nodes, base, pure, tv + t * M * jb.k_cap,
                      K, jb.k_cap, jb.leaf_value, lbase);
        }
        jb.roots[t] = base;
    }
#ifdef DDM_DFIT_PROFILE
    const uint64_t t_p = wall_clock64();
#endif
    int64_t bytes = 0;
    if (pure && jb.blob)
        bytes = compile_forest((const TNode*)tn, M, (const int32_t*)meta, T, (const int32_t*)jb.classes, K, jb.F, (int16_t*)bfs,
                               (uint8_t*)jb.blob, jb.blob_cap,
                               n_nodes <= kPackLdsNodes ? s_tn : nullptr, s_bid, base);
#ifdef DDM_DFIT_PROFILE
    if (t == 0)
        jb.result[11] = (int64_t)((t_p - t_pack0) | ((wall_clock64() - t_p) << 16) |
                                  (bytes ? (uint64_t)*(gptr<const uint32_t>)bfs << 32 : 0));
#endif
    if (t == 0) {
        jb.result[DDM_DFIT_NODES] = n_nodes;
        jb.result[DDM_DFIT_PURE] = pure ? 1 : 0;
        jb.result[DDM_DFIT_LEAF_ROWS] = pure ? 0 : n_leaf;
        jb.result[DDM_DFIT_BLOB] = bytes;
        if (bytes) {
            gptr<const ddm_cforest_head> h = (gptr<const ddm_cforest_head>)jb.blob;
            jb.result[DDM_DFIT_CF_SLOTS] = h->n_slots;
            jb.result[DDM_DFIT_CF_VR] = h->vote_regs;
            jb.result[DDM_DFIT_CF_LEAVES] = h->n_leaves;
            jb.result[DDM_DFIT_CF_TAB] = (int64_t)h->rank_tab_entries * h->vote_regs;
        }
    }
}

// join_flag: one thread of workgroup 0 polls it after its job (ctl.hip: the side stream's
// shuffles of the next window, which the next predict reads), so the kernel ends only once
// they are done.
__global__ __launch_bounds__(kPackThreads) void k_dfit_pack(const Job* __restrict__ jobs, const uint32_t* join_flag,
                                                            uint32_t join_v, uint32_t* timeouts) {
    refit_priority();
    pack_job(jobs[blockIdx.x]);
    if (join_flag && blockIdx.x == 0 && threadIdx.x == 0) ddm::flag_poll(join_flag, join_v, timeouts);
}

}  // namespace

int rf_fit_device_join(const ddm_dfit_job* jobs_dev, int32_t n_jobs, int32_t max_trees, int64_t max_lf,
                       const uint32_t* join_flag, uint32_t join_v, uint32_t* timeouts, ddm_stream_t stream);

extern "C" int64_t ddm_rf_device_scratch_bytes(int32_t L, int32_t F, int32_t n_trees, int32_t k_cap) {
    if (L < 1 || F < 1 || n_trees < 1 || k_cap < 1) return 0;
    return layout(L, F, n_trees, k_cap).total;
}

extern "C" int ddm_rf_fit_device_lf(const ddm_dfit_job* jobs_dev, int32_t n_jobs, int32_t max_trees, int64_t max_lf,
                                    ddm_stream_t stream) {
    return rf_fit_device_join(jobs_dev, n_jobs, max_trees, max_lf, nullptr, 0, nullptr, stream);
}

// The same; join_flag != NULL: the pack kernel ends only once *join_flag reaches join_v
// (ctl.hip), n_jobs >= 1.
int rf_fit_device_join(const ddm_dfit_job* jobs_dev, int32_t n_jobs, int32_t max_trees, int64_t max_lf,
                       const uint32_t* join_flag, uint32_t join_v, uint32_t* timeouts, ddm_stream_t stream) {
    if (!jobs_dev || n_jobs < 0 || max_trees < 1 || max_trees > 256 || (join_flag && (!timeouts || n_jobs < 1))) {
        ddm::set_error("ddm_rf_fit_device: invalid argument");
        return DDM_E_ARG;
    }
    if (n_jobs == 0) return 0;
    hipStream_t s = ddm::as_hip(stream);
    const Job* jobs = reinterpret_cast<const Job*>(jobs_dev);
    const bool fused = max_lf > 0 && max_lf <= kTreeTile;
    if (!fused) {
        hipLaunchKernelGGL(k_dfit_prep, dim3((unsigned)n_jobs, kSortBlocks + (unsigned)ddm::ceil_div(max_trees, kBootWaves)),
                           dim3(kPrepThreads), 0, s, jobs);
        if (int rc = ddm::launch_status("ddm_rf_fit_device/prep")) return rc;
    }
    hipLaunchKernelGGL(fused ? k_dfit_trees<true> : k_dfit_trees<false>,
                       dim3((unsigned)ddm::ceil_div(max_trees, kWaves), (unsigned)n_jobs), dim3(64 * kWaves), 0, s,
                       jobs);
    if (int rc = ddm::launch_status("ddm_rf_fit_device/trees")) return rc;
    hipLaunchKernelGGL(k_dfit_pack, dim3((unsigned)n_jobs), dim3(kPackThreads), 0, s, jobs, join_flag, join_v, timeouts);
    return ddm::launch_status("ddm_rf_fit_device/pack");
}

extern "C" int ddm_rf_fit_device(const ddm_dfit_job* jobs_dev, int32_t n_jobs, int32_t max_trees, ddm_stream_t stream) {
    return ddm_rf_fit_device_lf(jobs_dev, n_jobs, max_trees, -1, stream);
}
