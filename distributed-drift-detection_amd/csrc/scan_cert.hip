// Certified long carried DDM segments: run_DDM (DDM_Process.py:135-159) over streams whose
// detector carries across very many rows (:144-152, :202), evaluated row-parallel.
//
// The reference's p is a rounded running mean, p += (x - p) / n, so the exact value of row
// i needs every row before it (ddm_scan_long runs that chain: ~50 ns per row).  But the
// DECISIONS only need p to the precision that separates them.  In exact arithmetic the
// recurrence is the running mean: from a detector holding p0 over c0 samples, row i (the
// c_i = c0 + i'th sample, K_i errors in the window so far) has
//     pa_i = (c0 * p0 + K_i) / c_i.
// Each reference step adds a rounding error rho_k (|rho_k| <= u (p_k + 2 / c_k), u = 2^-53:
// the subtraction, the division and the addition), and the step contracts older errors by
// (c_k - 1) / c_k, so c_i e_i = c_m e_m + sum_{m<k<=i} c_k rho_k for the error e = p_ref - pa.
// Hence (the sums are closed forms of prefix counts, computed exactly in integers):
//   * |e_i| <= B_i = (c0 B0 + u S_i) / c_i,   S_i = sum_{k<=i} (c0 p0 + K_k + 2 + c_k 2^-30);
//   * and, what makes it work, for two rows m < i of the window
//     |e_i - e_m| <= D = B_m (c_i - c_m) / c_i + u (S_i - S_m) / c_i,
//     i.e. comparing a row with a recent one (the running arg-min) cancels the long
//     history's error and leaves only the rounding of the rows in between.
// Every decision the reference takes compares row i with its arg-min row m: the min update
// ps_i <= ps_min and the tests ps_i > p_min + k s_min (k = out_control / warning level).
// With s' = ds/dp the margin's error is at most
//   (D + 3u (p_i + p_m)) (1 + 2|s'_i|) + 2 |s'_i - k s'_m| B_m + 2^-50 (the operands)
// (the 3u terms: pa's own evaluation; 2^-50: s, p + s and the thresholds' roundings, ours
// and the reference's); a decision whose margin exceeds that bound is the reference's
// decision.  A cheap per-thread form of the bound (D <= B_i + B_m) settles almost every
// row; the exact form only runs near ties.  Rows in the exact regime (p stays exactly 0 or
// 1 from an exact start) compare exactly.  A stream with any uncertified decision up to its
// stop (or the end) is rescanned by the exact kernel (ddm_scan_long), so decisions and
// events are always the reference's; the state handed back is pa's (|p - p_ref| <= B, in
// practice ~1e-13 relative; north_star allows p/s within 1e-12 relative) together with its
// bound (bound_io), which a following call continues from.
//
// Kernels per round (a stream is cut into chunks of 4096 rows, 16 per thread):
//   count   per chunk: errors, sum of in-chunk prefix counts, first 0 / first 1; event rows
//           of the chunk's batches preset
//   scan1   per stream: chunk prefix counts; the incoming detector (c0, p0, its minimum,
//           the exact regime)
//   eval    per chunk: every row's p + s; each thread's and the chunk's arg-min
//   scan2   per stream: the arg-min before each chunk (the incoming minimum first)
//   decide  per chunk: every row's decisions against its arg-min, certified; first change,
//           first uncertified row, first warning of each batch
//   final   per stream: stop, state, bound, or the exact fallback
//   fix     per chunk: the event rows up to the stop (perm_map labels), event counts
// Scans run on (p + s, index) keys with wave shuffles; the full arg-min element is fetched
// by index.  Mode 1 (a change drops the detector, a fresh one takes the next batch)
// repeats the round from the batch after the change, up to kCertRounds rounds; what is
// left runs exact.
#include <cstddef>

#include "common.h"

namespace {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
constexpr int kRowsPerThread = 16;
constexpr int kChunk = kThreads * kRowsPerThread;   // rows per chunk
constexpr int kMaxBatch = 256;                      // ddm_scan_long's limit (the fallback)
constexpr int kSlots = kChunk + 2;                  // batches a chunk can touch (per_batch 1)
constexpr int kCertRounds = 4;                      // mode 1: certified rounds before the exact kernel
constexpr double kU = 0x1p-53;
constexpr double kG = 0x1p-30;                      // guard: |p_ref - pa| <= 2^-30 (checked)
constexpr unsigned long long kNone = ~0ull;

struct MinEl {                 // the arg-min element: a row of the window or the incoming minimum
    double ps, p, s, B;        // p + s, p, s, error bound of p
    double sd;                 // ds/dp at the row
    int64_t c;                 // sample count c of the row (in-window)
    int64_t sk;                // prefix sum of the window's prefix error counts at the row
    int32_t kind;              // 0 none, 1 the incoming minimum, 2 a window row
    int32_t pad;
};

struct Key {                   // an arg-min candidate: p + s and where its element is
    double ps;
    int32_t idx;               // -1 none
    int32_t pad;
};

struct Rec {                   // the detector after a row (state handed back)
    double p, s, B;
    MinEl m;
    int64_t n;
    int32_t chg, warn;
};

struct Hdr {                   // per stream
    int64_t lo0;               // the stream's first row (batch numbering)
    int64_t lo, hi;            // this round's rows
    int64_t next_lo;           // mode 1: the next round's first row
    int64_t c0;                // samples in the incoming p (0: fresh)
    double p0, A, B0, Bmin;    // incoming p, c0 * p0, bound of p0, bound of the incoming minimum
    MinEl inmin;
    int64_t rstar;             // window rows before rstar are exact (p stays 0 or 1)
    int64_t skr;               // prefix-count sum over the exact rows
    unsigned long long fc, fu; // first change / first uncertified row of the window (kNone)
    int32_t regime;            // -1 none, 0 / 1 the exact regime's p
    int32_t touched;           // non-empty stream: results are written
    int32_t active;            // this round scans the stream
    int32_t cont;              // mode 1: another round from next_lo
    int32_t fb;                // exact fallback from lo
    int32_t status;            // 0 certified, 1 uncertified decision, 2 rounds exhausted,
                               // 3 uncertified decision from an inexact incoming state (void)
};

__device__ __forceinline__ MinEl mcomb(const MinEl& L, const MinEl& R) {
    if (R.kind == 0) return L;
    if (L.kind == 0) return R;
    return R.ps <= L.ps ? R : L;                    // the reference's `<=`: the later row on ties
}

__device__ __forceinline__ Key kcomb(const Key& L, const Key& R) {
    if (R.idx < 0) return L;
    if (L.idx < 0) return R;
    return R.ps <= L.ps ? R : L;
}

__device__ __forceinline__ Key key_none() { return Key{0.0, -1, 0}; }

__device__ __forceinline__ double sd_of(double p, double s) {   // ds/dp at (p, s = sqrt(p(1-p)/c))
    return (s > 0.0 && p > 0.0 && p < 1.0) ? (1.0 - 2.0 * p) * s / (2.0 * p * (1.0 - p)) : 0.0;
}

// sum_{k=lo..w} (A + 2 + K_k + 2^-30 c_k) for window rows lo..w, sum K_k = skd (exact)
__device__ __forceinline__ double s_sum(const Hdr& H, int64_t lo, int64_t w, int64_t skd) {
    if (w < lo) return 0.0;
    const int64_t nr = w - lo + 1;
    const int64_t sc = nr * (H.c0 + 1) + (w * (w + 1) - (lo - 1) * lo) / 2;   // sum of c_k
    return (double)nr * (H.A + 2.0) + (double)skd + kG * (double)sc;
}

// B_i: the bound of |p_ref - pa| at window row w (its c, its prefix-count sum SK)
__device__ __forceinline__ double bound_at(const Hdr& H, int64_t w, int64_t SK) {
    const double cd = (double)(H.c0 + w + 1);
    if (w < H.rstar) return H.B0 > 0.0 ? (double)H.c0 * H.B0 / cd * (1.0 + 0x1p-50) : 0.0;
    return ((double)H.c0 * H.B0 + kU * s_sum(H, H.rstar, w, SK - H.skr) * (1.0 + 0x1p-40)) / cd * (1.0 + 0x1p-48);
}

struct RowP {                  // the values a row compares
    double pa, sa, ps, q, r;   // q = pa (1 - pa) / c, r = 1 / c
};

// pa = (A + K) r is within 2u of (A + K) / c; a quotient that is exactly 0 or 1 (the exact
// regime) is taken as the division's, which is exact there
__device__ __forceinline__ RowP row_p(const Hdr& H, int64_t c, int64_t K) {
    RowP v;
    const double num = H.A + (double)K;
    const double cd = (double)c;
    v.r = 1.0 / cd;
    v.pa = (num == 0.0 || num == cd) ? num / cd : num * v.r;
    v.q = v.pa * (1.0 - v.pa) * v.r;
    v.sa = sqrt(v.q);
    v.ps = v.pa + v.sa;
    return v;
}

// s' = (1/2 - pa) / (c s) for the bounds (1/s by a refined reciprocal square root: within
// 2^-40, covered by the 2^-20 slack the bounds give s')
__device__ __forceinline__ double sd_row(const RowP& v, int64_t) {
    if (!(v.sa > 0.0)) return 0.0;
    double y = __builtin_amdgcn_rsq(v.q);
    y = y * (1.5 - 0.5 * v.q * y * y);
    y = y * (1.5 - 0.5 * v.q * y * y);
    return (0.5 - v.pa) * v.r * y;
}

__device__ __forceinline__ MinEl row_el(const Hdr& H, const RowP& v, int64_t w, int64_t SK) {
    MinEl m;
    m.ps = v.ps;
    m.p = v.pa;
    m.s = v.sa;
    m.c = H.c0 + w + 1;
    m.B = bound_at(H, w, SK);
    m.sd = sd_row(v, m.c);
    m.sk = SK;
    m.kind = 2;
    m.pad = 0;
    return m;
}

// Is the comparison ps_v vs (M.p + k M.s) (the min test: M.ps with k = 1) decided the
// reference's way?  margin = our value of the compared difference; Bthr bounds B over the
// thread's rows (the cheap form), the exact D is formed only when that does not settle it.
__device__ __forceinline__ bool certain(const Hdr& H, const RowP& v, double sdv, int64_t w, int64_t SK, double Bthr,
                                        const MinEl& M, double k, double margin, double scale) {
    const bool inc = M.kind == 1;
    const double Bm = inc ? H.Bmin : M.B;
    if (Bthr == 0.0 && Bm == 0.0) return true;      // both exact (the regime): compare as they are
    const double evp = 3.0 * kU * (inc ? v.pa : v.pa + M.p);
    const double bmp = inc ? Bm : Bm + 3.0 * kU * M.p;
    const double sdm = inc && Bm == 0.0 ? 0.0 : M.sd;
    const double lin = 2.0 * (fabs(sdv - k * sdm) + 0x1p-20 * (fabs(sdv) + k * fabs(sdm))) * bmp +
                       0x1p-50 * (v.ps + M.ps + M.p + k * M.s);
    const double amar = fabs(margin);
    // cheap: |e_v - e_m| <= B_v + B_m
    if (amar > ((Bthr + Bm + evp) * (1.0 + 2.0 * fabs(sdv)) + lin) * scale) return true;
    // exact D
    const int64_t c = H.c0 + w + 1;
    const double Bv = bound_at(H, w, SK);
    if (Bv > 0.0 && (v.sa == 0.0 || Bv > 0x1p-20 * fmin(v.pa, 1.0 - v.pa))) return false;
    double D;
    if (inc) {
        D = Bv + Bm;
    } else if (M.c == c) {
        D = 0.0;
    } else {
        const int64_t mw = M.c - H.c0 - 1;          // window row of the minimum
        const int64_t lo = max(mw + 1, H.rstar);
        const int64_t skd = lo == mw + 1 ? SK - M.sk : SK - H.skr;
        D = (M.B * (double)(c - M.c) + kU * s_sum(H, lo, w, skd) * (1.0 + 0x1p-40)) / (double)c * (1.0 + 0x1p-48);
    }
    if (Bv == 0.0 && Bm == 0.0 && D == 0.0) return true;
    return amar > ((D + evp) * (1.0 + 2.0 * fabs(sdv)) + lin) * scale;
}

// ---- wave / block scans (shuffles; 4 waves per block)
struct Tri {                   // (errors, sum of prefix counts, rows) of a run of rows
    int64_t k, sk, l;
};
__device__ __forceinline__ Tri tcomb(const Tri& a, const Tri& b) { return {a.k + b.k, a.sk + b.sk + a.k * b.l, a.l + b.l}; }

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

__device__ Tri wave_incl_tri(Tri t) {
    const int lane = lane_id();
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        Tri o{__shfl_up(t.k, d), __shfl_up(t.sk, d), __shfl_up(t.l, d)};
        if (lane >= d) t = tcomb(o, t);
    }
    return t;
}

__device__ Key wave_incl_key(Key k) {
    const int lane = lane_id();
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        Key o{__shfl_up(k.ps, d), __shfl_up(k.idx, d), 0};
        if (lane >= d) k = kcomb(o, k);
    }
    return k;
}

// exclusive block scan of Tri over threads; returns the thread's exclusive prefix
__device__ Tri block_excl_tri(Tri x, Tri* sw, Tri* total) {
    const int lane = lane_id(), wv = threadIdx.x >> 6;
    const Tri inc = wave_incl_tri(x);
    if (lane == 63) sw[wv] = inc;
    __syncthreads();
    Tri pre{0, 0, 0};
    for (int q = 0; q < wv; ++q) pre = tcomb(pre, sw[q]);
    Tri ex{__shfl_up(inc.k, 1), __shfl_up(inc.sk, 1), __shfl_up(inc.l, 1)};
    if (lane == 0) ex = Tri{0, 0, 0};
    if (total) {
        Tri t{0, 0, 0};
        for (int q = 0; q < kWaves; ++q) t = tcomb(t, sw[q]);
        *total = t;
    }
    __syncthreads();
    return tcomb(pre, ex);
}

__device__ Key block_excl_key(Key x, Key* sw, Key* total) {
    const int lane = lane_id(), wv = threadIdx.x >> 6;
    const Key inc = wave_incl_key(x);
    if (lane == 63) sw[wv] = inc;
    __syncthreads();
    Key pre = key_none();
    for (int q = 0; q < wv; ++q) pre = kcomb(pre, sw[q]);
    Key ex{__shfl_up(inc.ps, 1), __shfl_up(inc.idx, 1), 0};
    if (lane == 0) ex = key_none();
    if (total) {
        Key t = key_none();
        for (int q = 0; q < kWaves; ++q) t = kcomb(t, sw[q]);
        *total = t;
    }
    __syncthreads();
    return kcomb(pre, ex);
}

// a thread's rows of a chunk
struct ThreadRows {
    uint32_t bits;             // bit j: row j is an error
    int n;                     // rows present
};

__device__ __forceinline__ ThreadRows load_rows(const uint8_t* __restrict__ err, int64_t r0, int64_t L) {
    ThreadRows tr;
    const int64_t o = (int64_t)threadIdx.x * kRowsPerThread;
    const int64_t a = r0 + o;
    tr.n = (int)max((int64_t)0, min((int64_t)kRowsPerThread, L - o));
    tr.bits = 0;
    if (tr.n == kRowsPerThread && (a & 15) == 0) {
        const uint4 q = *reinterpret_cast<const uint4*>(err + a);
        const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int j = 0; j < 16; ++j) tr.bits |= (((w[j >> 2] >> (8 * (j & 3))) & 0xffu) != 0 ? 1u : 0u) << j;
    } else {
        for (int j = 0; j < tr.n; ++j) tr.bits |= (err[a + j] != 0 ? 1u : 0u) << j;
    }
    return tr;
}

__device__ __forceinline__ Tri thread_tri(const ThreadRows& tr) {
    Tri t{__builtin_popcount(tr.bits), 0, tr.n};
    for (uint32_t b = tr.bits; b; b &= b - 1) t.sk += tr.n - __builtin_ctz(b);   // rows counting the error
    return t;
}

// the thread's (K, SK) before its rows: the chunk's prefix, then the block's
__device__ __forceinline__ void thread_base(int64_t kb, int64_t skb, const Tri& ex, int64_t& K, int64_t& SK) {
    K = kb + ex.k;
    SK = skb + ex.sk + kb * ex.l;
}

// ---- kernels
__global__ __launch_bounds__(64) void k_cert_setup(Hdr* __restrict__ hdr, const int64_t* __restrict__ off,
                                                    const int64_t* __restrict__ end, int64_t n_streams,
                                                    int32_t* __restrict__ any_fb, uint32_t* __restrict__ zero,
                                                    int64_t zero_words, int32_t* __restrict__ evc, int64_t n_evc) {
    const int64_t s = (int64_t)blockIdx.x * 64 + threadIdx.x;
    for (int64_t q = s; q < zero_words; q += (int64_t)gridDim.x * 64) zero[q] = 0;   // the exact kernel's flags
    for (int64_t q = s; q < n_evc; q += (int64_t)gridDim.x * 64) evc[q] = 0;
    if (s == 0) *any_fb = 0;
    if (s >= n_streams) return;
    Hdr H = {};
    H.lo0 = H.lo = off[s];
    H.hi = end ? end[s] : off[s + 1];
    H.touched = H.hi > H.lo;
    H.active = H.touched;
    hdr[s] = H;
}

__global__ __launch_bounds__(64) void k_cert_advance(Hdr* __restrict__ hdr, int64_t n_streams) {
    const int64_t s = (int64_t)blockIdx.x * 64 + threadIdx.x;
    if (s >= n_streams) return;
    Hdr& H = hdr[s];
    H.active = H.cont;                              // done, or the fallback's: no further rounds
    if (H.cont) H.lo = H.next_lo;
    H.cont = 0;
}

__global__ __launch_bounds__(kThreads) void k_cert_count(const Hdr* __restrict__ hdr, const uint8_t* __restrict__ err,
                                                         int64_t n_streams, int64_t n_chunks, int pb,
                                                         int32_t* __restrict__ cnt, int64_t* __restrict__ skl,
                                                         int32_t* __restrict__ f0, int32_t* __restrict__ f1,
                                                         int32_t* __restrict__ ev, const int64_t* __restrict__ bbase) {
    const int64_t s = blockIdx.x % n_streams, c = blockIdx.x / n_streams;
    const Hdr& H = hdr[s];
    if (!H.active) return;
    const int64_t r0 = H.lo + c * kChunk;
    if (r0 >= H.hi) return;
    const int64_t L = min((int64_t)kChunk, H.hi - r0);
    const ThreadRows tr = load_rows(err, r0, L);
    __shared__ Tri sw[kWaves];
    Tri tot;
    block_excl_tri(thread_tri(tr), sw, &tot);
    // first 0 / first 1 of the chunk
    const int o = threadIdx.x * kRowsPerThread;
    const uint32_t pres = (1u << tr.n) - 1;
    int a0 = (~tr.bits & pres) ? o + __builtin_ctz(~tr.bits & pres) : 0x7fffffff;
    int a1 = tr.bits ? o + __builtin_ctz(tr.bits) : 0x7fffffff;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        a0 = min(a0, __shfl_xor(a0, d));
        a1 = min(a1, __shfl_xor(a1, d));
    }
    __shared__ int s_f[2][kWaves];
    if (lane_id() == 0) {
        s_f[0][threadIdx.x >> 6] = a0;
        s_f[1][threadIdx.x >> 6] = a1;
    }
    __syncthreads();
    const int64_t q = s * n_chunks + c;
    if (threadIdx.x == 0) {
        int m0 = 0x7fffffff, m1 = 0x7fffffff;
        for (int w = 0; w < kWaves; ++w) {
            m0 = min(m0, s_f[0][w]);
            m1 = min(m1, s_f[1][w]);
        }
        cnt[q] = (int32_t)tot.k;
        skl[q] = tot.sk;
        f0[q] = m0 == 0x7fffffff ? 0x7fffffff : (int32_t)(c * kChunk + m0);
        f1[q] = m1 == 0x7fffffff ? 0x7fffffff : (int32_t)(c * kChunk + m1);
    }
    // event rows of the batches that start in this chunk: (no warning yet, no change)
    const int64_t b_first = (r0 - H.lo0 + pb - 1) / pb, b_last = (r0 + L - 1 - H.lo0) / pb;
    int32_t* e = ev + 2 * bbase[s];
    for (int64_t b = b_first + threadIdx.x; b <= b_last; b += kThreads)
        *reinterpret_cast<int2*>(e + 2 * b) = make_int2(0x7fffffff, -1);
}

__global__ __launch_bounds__(kThreads) void k_cert_scan1(Hdr* __restrict__ hdr, int64_t n_chunks,
                                                         const int32_t* __restrict__ cnt,
                                                         const int64_t* __restrict__ skl,
                                                         const int32_t* __restrict__ f0, const int32_t* __restrict__ f1,
                                                         int64_t* __restrict__ kb, int64_t* __restrict__ skb,
                                                         const ddm_state* __restrict__ state,
                                                         const double* __restrict__ bound_in, int round) {
    const int64_t s = blockIdx.x;
    Hdr& H = hdr[s];
    if (!H.active) return;
    __shared__ Tri sw[kWaves];
    __shared__ int s_f[2][kWaves];
    const int64_t rows = H.hi - H.lo;
    const int64_t nck = (rows + kChunk - 1) / kChunk;
    Tri carry{0, 0, 0};
    int m0 = 0x7fffffff, m1 = 0x7fffffff;
    for (int64_t base = 0; base < nck; base += kThreads) {
        const int64_t c = base + threadIdx.x;
        Tri x{0, 0, 0};
        if (c < nck) {
            const int64_t q = s * n_chunks + c;
            x = Tri{cnt[q], skl[q], min((int64_t)kChunk, rows - c * kChunk)};
            m0 = min(m0, f0[q]);
            m1 = min(m1, f1[q]);
        }
        Tri tot;
        const Tri ex = tcomb(carry, block_excl_tri(x, sw, &tot));
        if (c < nck) {
            kb[s * n_chunks + c] = ex.k;
            skb[s * n_chunks + c] = ex.sk;
        }
        carry = tcomb(carry, tot);
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        m0 = min(m0, __shfl_xor(m0, d));
        m1 = min(m1, __shfl_xor(m1, d));
    }
    if (lane_id() == 0) {
        s_f[0][threadIdx.x >> 6] = m0;
        s_f[1][threadIdx.x >> 6] = m1;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 0; w < kWaves; ++w) {
            m0 = min(m0, s_f[0][w]);
            m1 = min(m1, s_f[1][w]);
        }
        const ddm_state st = state[s];
        const bool dropped = st.in_concept_change != 0;
        H.c0 = dropped ? 0 : st.sample_count - 1;
        H.p0 = dropped ? 0.0 : st.miss_prob;
        H.A = (double)H.c0 * H.p0;
        H.B0 = (!dropped && bound_in && round == 0) ? bound_in[2 * s] : 0.0;
        H.Bmin = (!dropped && bound_in && round == 0) ? bound_in[2 * s + 1] : 0.0;
        H.inmin.kind = 0;
        if (!dropped && !__builtin_isinf(st.miss_prob_sd_min)) {
            H.inmin.kind = 1;
            H.inmin.ps = st.miss_prob_sd_min;
            H.inmin.p = st.miss_prob_min;
            H.inmin.s = st.miss_sd_min;
            H.inmin.B = H.Bmin;
            H.inmin.sd = sd_of(H.inmin.p, H.inmin.s);
            H.inmin.c = 0;
            H.inmin.sk = 0;
        }
        if (H.c0 == 0) H.regime = m0 == 0 ? 0 : 1;  // a fresh detector: p = x of the first row
        else if (H.B0 == 0.0 && (H.p0 == 0.0 || H.p0 == 1.0)) H.regime = (int)H.p0;
        else H.regime = -1;
        const int64_t fo = H.regime == 0 ? m1 : m0;
        H.rstar = H.regime < 0 ? 0 : min(rows, (int64_t)fo);
        H.skr = H.regime == 1 ? H.rstar * (H.rstar + 1) / 2 : 0;
        H.fc = H.fu = kNone;
    }
}

// The thread's own arg-min over its rows (ps only), as (ps, local row).
__device__ __forceinline__ Key thread_min(const Hdr& H, const ThreadRows& tr, int64_t w0, int64_t K, int min_inst) {
    Key m = key_none();
    for (int j = 0; j < tr.n; ++j) {
        K += (tr.bits >> j) & 1u;
        const int64_t c = H.c0 + w0 + j + 1;
        if (c + 1 < min_inst) continue;             // the gate: n (after the row) < min_num_instances
        const RowP v = row_p(H, c, K);
        if (m.idx < 0 || v.ps <= m.ps) m = Key{v.ps, j, 0};
    }
    return m;
}

// the element of the thread's row j
__device__ __forceinline__ MinEl thread_el(const Hdr& H, const ThreadRows& tr, int64_t w0, int64_t K, int64_t SK,
                                           int j) {
    for (int i = 0; i <= j; ++i) {
        K += (tr.bits >> i) & 1u;
        SK += K;
    }
    return row_el(H, row_p(H, H.c0 + w0 + j + 1, K), w0 + j, SK);
}

__global__ __launch_bounds__(kThreads) void k_cert_eval(const Hdr* __restrict__ hdr, const uint8_t* __restrict__ err,
                                                        int64_t n_streams, int64_t n_chunks, int min_inst,
                                                        const int64_t* __restrict__ kb, const int64_t* __restrict__ skb,
                                                        MinEl* __restrict__ agg, Key* __restrict__ tkey) {
    const int64_t s = blockIdx.x % n_streams, c = blockIdx.x / n_streams;
    const Hdr& H = hdr[s];
    if (!H.active) return;
    const int64_t r0 = H.lo + c * kChunk;
    if (r0 >= H.hi) return;
    const int64_t L = min((int64_t)kChunk, H.hi - r0);
    __shared__ Tri sw[kWaves];
    __shared__ Key skw[kWaves];
    const ThreadRows tr = load_rows(err, r0, L);
    const Tri ex = block_excl_tri(thread_tri(tr), sw, nullptr);
    const int64_t q = s * n_chunks + c;
    int64_t K, SK;
    thread_base(kb[q], skb[q], ex, K, SK);
    const int64_t w0 = c * kChunk + (int64_t)threadIdx.x * kRowsPerThread;
    const Key m = thread_min(H, tr, w0, K, min_inst);
    tkey[q * kThreads + threadIdx.x] = m;           // decide's thread prefixes start from these
    Key tot;
    block_excl_key(Key{m.ps, m.idx < 0 ? -1 : (int32_t)threadIdx.x, 0}, skw, &tot);
    if (tot.idx == (int32_t)threadIdx.x) agg[q] = thread_el(H, tr, w0, K, SK, m.idx);
    if (tot.idx < 0 && threadIdx.x == 0) agg[q].kind = 0;
}

constexpr int32_t kIn = 0x7ffffffe;                 // the incoming minimum's index (before every chunk)

__global__ __launch_bounds__(kThreads) void k_cert_scan2(const Hdr* __restrict__ hdr, int64_t n_chunks,
                                                         const MinEl* __restrict__ agg, int32_t* __restrict__ minb) {
    const int64_t s = blockIdx.x;
    const Hdr& H = hdr[s];
    if (!H.active) return;
    __shared__ Key skw[kWaves];
    const int64_t nck = (H.hi - H.lo + kChunk - 1) / kChunk;
    // keys: the chunk index, or kIn for the incoming minimum
    Key carry = H.inmin.kind ? Key{H.inmin.ps, kIn, 0} : key_none();
    for (int64_t base = 0; base < nck; base += kThreads) {
        const int64_t c = base + threadIdx.x;
        Key x = key_none();
        if (c < nck) {
            const MinEl& a = agg[s * n_chunks + c];
            if (a.kind) x = Key{a.ps, (int32_t)c, 0};
        }
        Key tot;
        const Key ex = kcomb(carry, block_excl_key(x, skw, &tot));
        if (c < nck) minb[s * n_chunks + c] = ex.idx;
        carry = kcomb(carry, tot);
    }
}

__global__ __launch_bounds__(kThreads) void k_cert_decide(Hdr* __restrict__ hdr, const uint8_t* __restrict__ err,
                                                          int64_t n_streams, int64_t n_chunks, ddm_params P,
                                                          const int64_t* __restrict__ kb,
                                                          const int64_t* __restrict__ skb,
                                                          const MinEl* __restrict__ agg,
                                                          const int32_t* __restrict__ minb, const Key* __restrict__ tkey,
                                                          Rec* __restrict__ rec_chg, Rec* __restrict__ rec_end,
                                                          int32_t* __restrict__ ev, const int64_t* __restrict__ bbase,
                                                          double scale) {
    const int64_t s = blockIdx.x % n_streams, c = blockIdx.x / n_streams;
    Hdr& H = hdr[s];
    if (!H.active) return;
    const int64_t r0 = H.lo + c * kChunk;
    if (r0 >= H.hi) return;
    const int64_t L = min((int64_t)kChunk, H.hi - r0);
    const int pb = P.per_batch, min_inst = P.min_num_instances;
    const double wl = P.warning_level, cl = P.out_control_level;
    __shared__ Tri sw[kWaves];
    __shared__ Key skw[kWaves];
    __shared__ MinEl s_el[kThreads];
    __shared__ int32_t s_warn[kSlots];
    __shared__ unsigned long long s_fc, s_fu;
    const int64_t b_lo = (r0 - H.lo0) / pb;          // the first batch a row of the chunk is in
    const int nslot = (int)((r0 + L - 1 - H.lo0) / pb - b_lo + 1);
    for (int k = threadIdx.x; k < nslot; k += kThreads) s_warn[k] = 0x7fffffff;
    if (threadIdx.x == 0) s_fc = s_fu = kNone;
    const ThreadRows tr = load_rows(err, r0, L);
    const Tri ex = block_excl_tri(thread_tri(tr), sw, nullptr);
    const int64_t q = s * n_chunks + c;
    int64_t K0, SK0;
    thread_base(kb[q], skb[q], ex, K0, SK0);
    const int64_t w0 = c * kChunk + (int64_t)threadIdx.x * kRowsPerThread;
    // the arg-min before the thread's rows: the chunk's prefix, then the earlier threads' minima
    const Key tk = tkey[q * kThreads + threadIdx.x];
    if (tk.idx >= 0) s_el[threadIdx.x] = thread_el(H, tr, w0, K0, SK0, tk.idx);
    const Key pk = block_excl_key(Key{tk.ps, tk.idx < 0 ? -1 : (int32_t)threadIdx.x, 0}, skw, nullptr);
    const int32_t mi = minb[q];
    MinEl M;
    if (mi == kIn) M = H.inmin;
    else if (mi >= 0) M = agg[s * n_chunks + mi];
    else M.kind = 0;
    if (pk.idx >= 0) M = mcomb(M, s_el[pk.idx]);
    // a ceiling of B over the thread's rows: S grows row by row, c is smallest at the first
    double Bthr = 0.0;
    if (tr.n > 0) {
        int64_t K = K0, SK = SK0;
        for (int j = 0; j < tr.n; ++j) {
            K += (tr.bits >> j) & 1u;
            SK += K;
        }
        const int64_t wlast = w0 + tr.n - 1;
        if (wlast >= H.rstar)
            Bthr = ((double)H.c0 * H.B0 + kU * s_sum(H, H.rstar, wlast, SK - H.skr) * (1.0 + 0x1p-40)) /
                   (double)(H.c0 + w0 + 1) * (1.0 + 0x1p-48);
        else
            Bthr = bound_at(H, w0, SK0);
    }
    // the decisions, in row order, against the running arg-min
    unsigned long long fc = kNone, fu = kNone;
    int64_t K = K0, SK = SK0;
    int chg = 0, warn = 0, jl = -1;
    RowP v{};
    const int64_t rr0 = r0 + (w0 - c * kChunk) - H.lo0;   // the thread's first stream row
    int bslot = (int)(rr0 / pb - b_lo), bpos = (int)(rr0 % pb);
    bool wdone = false;                             // this batch's first warning (of the thread) recorded
    for (int j = 0; j < tr.n; ++j, ++bpos) {
        if (bpos == pb) {
            bpos = 0;
            ++bslot;
            wdone = false;
        }
        K += (tr.bits >> j) & 1u;
        SK += K;
        const int64_t w = w0 + j;
        const int64_t cr = H.c0 + w + 1;
        jl = j;
        chg = warn = 0;
        v = row_p(H, cr, K);
        if (cr + 1 < min_inst) continue;
        const double sdv = sd_row(v, cr);
        if (M.kind != 0 && fu == kNone && !certain(H, v, sdv, w, SK, Bthr, M, 1.0, v.ps - M.ps, scale))
            fu = (unsigned long long)w;
        if (M.kind == 0 || v.ps <= M.ps) M = row_el(H, v, w, SK);
        const double tc = M.p + cl * M.s;
        const double tw = M.p + wl * M.s;
        if (fu == kNone && (!certain(H, v, sdv, w, SK, Bthr, M, cl, v.ps - tc, scale) ||
                            (!(v.ps > tc) && !certain(H, v, sdv, w, SK, Bthr, M, wl, v.ps - tw, scale))))
            fu = (unsigned long long)w;
        if (v.ps > tc) {
            chg = 1;
            fc = (unsigned long long)w;
            break;                                  // later rows of the thread follow the stream's change
        }
        if (v.ps > tw) {
            warn = 1;
            if (!wdone) {
                atomicMin(&s_warn[bslot], bpos);
                wdone = true;
            }
        }
    }
    if (fc != kNone) atomicMin(&s_fc, fc);
    if (fu != kNone) atomicMin(&s_fu, fu);
    __syncthreads();
    // the detector after the chunk's first change (its thread), after the window's last row
    if (tr.n > 0 && ((fc != kNone && fc == s_fc) || (fc == kNone && r0 + (w0 - c * kChunk) + tr.n == H.hi))) {
        const int64_t w = w0 + jl;
        Rec r;
        r.p = v.pa;
        r.s = v.sa;
        r.B = bound_at(H, w, SK);
        r.m = M;
        r.n = H.c0 + w + 2;
        r.chg = chg;
        r.warn = warn;
        if (fc != kNone) rec_chg[q] = r;
        else rec_end[s] = r;
    }
    if (threadIdx.x == 0) {
        if (s_fc != kNone) atomicMin(&H.fc, s_fc);
        if (s_fu != kNone) atomicMin(&H.fu, s_fu);
    }
    int32_t* e = ev + 2 * bbase[s];
    for (int k = threadIdx.x; k < nslot; k += kThreads)
        if (s_warn[k] != 0x7fffffff) atomicMin(&e[2 * (b_lo + k)], s_warn[k]);
}

__global__ __launch_bounds__(64) void k_cert_final(Hdr* __restrict__ hdr, int64_t n_streams, int64_t n_chunks, int pb,
                                                   int mode, const Rec* __restrict__ rec_chg,
                                                   const Rec* __restrict__ rec_end, ddm_state* __restrict__ state,
                                                   double* __restrict__ bound_out, int32_t* __restrict__ stop_out) {
    const int64_t s = (int64_t)blockIdx.x * 64 + threadIdx.x;
    if (s >= n_streams) return;
    Hdr& H = hdr[s];
    if (!H.active) return;
    const unsigned long long fc = H.fc, fu = H.fu;
    if (fu != kNone && (fc == kNone || fu <= fc)) {  // an uncertified decision before the stop
        H.fb = 1;
        H.status = 1;
        H.active = 0;
        return;
    }
    const Rec r = fc != kNone ? rec_chg[s * n_chunks + (int64_t)(fc / kChunk)] : rec_end[s];
    ddm_state st;
    st.miss_prob = r.p;
    st.miss_std = r.s;
    if (r.m.kind == 0) {
        st.miss_prob_min = st.miss_sd_min = st.miss_prob_sd_min = __builtin_inf();
    } else {
        st.miss_prob_min = r.m.p;
        st.miss_sd_min = r.m.s;
        st.miss_prob_sd_min = r.m.ps;
    }
    st.sample_count = r.n;
    st.in_concept_change = r.chg;
    st.in_warning_zone = r.warn;
    const bool dropped = mode == 1 && fc != kNone;  // a fresh DDM takes the next batch (:209, :136-139)
    if (dropped) {
        st.miss_prob = 1.0;
        st.miss_std = 0.0;
        st.miss_prob_min = st.miss_sd_min = st.miss_prob_sd_min = __builtin_inf();
        st.sample_count = 1;
        st.in_concept_change = st.in_warning_zone = 0;
    }
    state[s] = st;
    if (bound_out) {
        bound_out[2 * s] = dropped ? 0.0 : r.B;
        bound_out[2 * s + 1] = dropped ? 0.0 : r.m.kind == 2 ? r.m.B : r.m.kind == 1 ? H.Bmin : 0.0;
    }
    if (mode == 0) {
        if (stop_out) stop_out[s] = fc == kNone ? -1 : (int32_t)((H.lo - H.lo0 + (int64_t)fc) / pb);
    } else {
        if (stop_out) stop_out[s] = -1;
        if (fc != kNone) {
            const int64_t b = (H.lo - H.lo0 + (int64_t)fc) / pb;
            const int64_t nl = H.lo0 + (b + 1) * pb;
            if (nl < H.hi) {
                H.next_lo = nl;
                H.cont = 1;
            }
        }
    }
}

__global__ __launch_bounds__(kThreads) void k_cert_fix(Hdr* __restrict__ hdr, int64_t n_streams, int64_t n_chunks,
                                                       int pb, int mode, int32_t* __restrict__ ev,
                                                       const int64_t* __restrict__ bbase,
                                                       const uint8_t* __restrict__ pmap, int32_t* __restrict__ evc) {
    const int64_t s = blockIdx.x % n_streams, c = blockIdx.x / n_streams;
    Hdr& H = hdr[s];
    if (!H.active) return;
    const int64_t r0 = H.lo + c * kChunk;
    if (r0 >= H.hi) return;
    const int64_t L = min((int64_t)kChunk, H.hi - r0);
    const unsigned long long fc = H.fc;
    const int64_t sb = fc == kNone ? INT64_MAX : (H.lo - H.lo0 + (int64_t)fc) / pb;
    const int32_t sy = fc == kNone ? -1 : (int32_t)((H.lo - H.lo0 + (int64_t)fc) % pb);
    const int64_t b_first = (r0 - H.lo0 + pb - 1) / pb, b_last = (r0 + L - 1 - H.lo0) / pb;
    int32_t* e = ev + 2 * bbase[s];
    int n = 0;
    for (int64_t b = b_first + threadIdx.x; b <= b_last; b += kThreads) {
        if (b > sb) {
            if (mode == 0) *reinterpret_cast<int2*>(e + 2 * b) = make_int2(-1, -1);
            continue;                               // mode 1: the next round's
        }
        int32_t x = e[2 * b], y = -1;
        if (x == 0x7fffffff) x = -1;
        if (b == sb) {
            y = sy;
            if (x > y) x = -1;                      // a warning after the change is never fed
        }
        n += (x >= 0 || y >= 0);
        if (pmap) {
            const int64_t bs = H.lo0 + b * pb;
            if (x >= 0) x = pmap[bs + x];
            if (y >= 0) y = pmap[bs + y];
        }
        *reinterpret_cast<int2*>(e + 2 * b) = make_int2(x, y);
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) n += __shfl_xor(n, d);
    __shared__ int s_n[kWaves];
    if (lane_id() == 0) s_n[threadIdx.x >> 6] = n;
    __syncthreads();
    if (threadIdx.x == 0) {                         // summed per stream by k_cert_done (rounds add up)
        int t = 0;
        for (int w = 0; w < kWaves; ++w) t += s_n[w];
        evc[s * n_chunks + c] += t;
    }
}

// the exact fallback's arguments: streams still active after the rounds, or uncertified
__global__ __launch_bounds__(64) void k_cert_prep_fb(Hdr* __restrict__ hdr, int64_t n_streams, int pb,
                                                     const int64_t* __restrict__ bbase, int64_t* __restrict__ fb_off,
                                                     int64_t* __restrict__ fb_end, int64_t* __restrict__ fb_bb,
                                                     int32_t* __restrict__ only, int32_t* __restrict__ any_fb) {
    const int64_t s = (int64_t)blockIdx.x * 64 + threadIdx.x;
    if (s >= n_streams) return;
    Hdr& H = hdr[s];
    if (H.cont) {                                   // mode 1: rounds exhausted
        H.lo = H.next_lo;
        H.fb = 1;
        H.status = 2;
        H.cont = 0;
    }
    // The exact kernel is the reference only from the reference's state.  A fallback from the
    // stream's first row starts from the caller's state, which is pa's (not the reference's
    // rounded p) when it came with a bound: the near-tie the rescan exists for could then be
    // decided wrongly, and the bound zeroed after it would certify what follows.  Such a
    // stream is left alone with status 3 (every output void); the caller redoes the run from
    // its last exact carry (ddm_amd/longstream.py).  Later rounds (mode 1) start fresh.
    if (H.fb && H.lo == H.lo0 && (H.B0 != 0.0 || H.Bmin != 0.0)) {
        H.fb = 0;
        H.status = 3;
    }
    fb_off[s] = H.lo;
    fb_end[s] = H.hi;
    fb_bb[s] = bbase[s] + (H.lo - H.lo0) / pb;
    only[s] = H.fb;
    if (H.fb) atomicOr(any_fb, 1);
}

__global__ __launch_bounds__(kThreads) void k_cert_done(const Hdr* __restrict__ hdr, int64_t n_chunks,
                                                        const int32_t* __restrict__ evc,
                                                        const int64_t* __restrict__ nev_fb, int64_t* __restrict__ nev_out,
                                                        double* __restrict__ bound_out, int32_t* __restrict__ status) {
    const int64_t s = blockIdx.x;
    const Hdr& H = hdr[s];
    if (!H.touched) return;
    int64_t n = 0;
    for (int64_t c = threadIdx.x; c < n_chunks; c += kThreads) n += evc[s * n_chunks + c];
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) n += __shfl_xor(n, d);
    __shared__ int64_t s_n[kWaves];
    if (lane_id() == 0) s_n[threadIdx.x >> 6] = n;
    __syncthreads();
    if (threadIdx.x) return;
    for (int w = 1; w < kWaves; ++w) n += s_n[w];
    if (nev_out) nev_out[s] = n + (H.fb ? nev_fb[s] : 0);
    if (H.fb && bound_out) {                        // the exact kernel's state is the reference's
        bound_out[2 * s] = 0.0;
        bound_out[2 * s + 1] = 0.0;
    }
    if (status) status[s] = H.status;
}

struct CertScratch {
    Hdr* hdr;
    int32_t *cnt, *f0, *f1, *only, *evc;
    int64_t *skl, *kb, *skb, *fb_off, *fb_end, *fb_bb, *nev_fb;
    MinEl* agg;
    int32_t* minb;
    Key* tkey;
    Rec *rec_chg, *rec_end;
    void* exact;
    int64_t bytes;
};

CertScratch cert_scratch(void* base, int64_t n, int64_t nc, int64_t exact_bytes) {
    const auto up = [](int64_t x) { return (x + 255) & ~(int64_t)255; };
    CertScratch sc{};
    int64_t o = 0;
    uint8_t* b = static_cast<uint8_t*>(base);
    const auto take = [&](int64_t bytes) {
        uint8_t* p = b ? b + o : nullptr;
        o += up(bytes);
        return p;
    };
    sc.hdr = reinterpret_cast<Hdr*>(take(sizeof(Hdr) * n));
    sc.evc = reinterpret_cast<int32_t*>(take(4 * n * nc));      // first: the setup zeroes it
    sc.cnt = reinterpret_cast<int32_t*>(take(4 * n * nc));
    sc.f0 = reinterpret_cast<int32_t*>(take(4 * n * nc));
    sc.f1 = reinterpret_cast<int32_t*>(take(4 * n * nc));
    sc.only = reinterpret_cast<int32_t*>(take(4 * (n + 1)));   // [n]: any stream needs the exact kernel
    sc.skl = reinterpret_cast<int64_t*>(take(8 * n * nc));
    sc.kb = reinterpret_cast<int64_t*>(take(8 * n * nc));
    sc.skb = reinterpret_cast<int64_t*>(take(8 * n * nc));
    sc.fb_off = reinterpret_cast<int64_t*>(take(8 * n));
    sc.fb_end = reinterpret_cast<int64_t*>(take(8 * n));
    sc.fb_bb = reinterpret_cast<int64_t*>(take(8 * n));
    sc.nev_fb = reinterpret_cast<int64_t*>(take(8 * n));
    sc.agg = reinterpret_cast<MinEl*>(take(sizeof(MinEl) * n * nc));
    sc.minb = reinterpret_cast<int32_t*>(take(4 * n * nc));
    sc.tkey = reinterpret_cast<Key*>(take(sizeof(Key) * n * nc * kThreads));
    sc.rec_chg = reinterpret_cast<Rec*>(take(sizeof(Rec) * n * nc));
    sc.rec_end = reinterpret_cast<Rec*>(take(sizeof(Rec) * n));
    sc.exact = take(exact_bytes);
    sc.bytes = o;
    return sc;
}

double g_tol_scale = 1.0;

}  // namespace

extern "C" int ddm_scan_long_only(const uint8_t* err, const int64_t* stream_off, const int64_t* stream_end,
                                  int64_t n_streams, int64_t max_rows, const ddm_params* prm, ddm_state* state_io,
                                  const int64_t* batch_base, int32_t* ev_out, int32_t* stop_out, int64_t* nev_out,
                                  int32_t mode, const uint8_t* perm_map, void* scratch, const int32_t* only,
                                  const int32_t* any, ddm_stream_t stream);
extern "C" int64_t ddm_scan_long_flag_bytes(int64_t n_streams, int64_t max_rows, int32_t per_batch);

extern "C" int64_t ddm_scan_certified_scratch_bytes(int64_t n_streams, int64_t max_rows, int32_t per_batch) {
    if (n_streams < 0 || max_rows < 0 || per_batch <= 0 || per_batch > kMaxBatch) return -1;
    const int64_t nc = std::max<int64_t>(1, ddm::ceil_div(max_rows, kChunk));
    const int64_t eb = ddm_scan_long_scratch_bytes(n_streams, max_rows, per_batch);
    return cert_scratch(nullptr, std::max<int64_t>(1, n_streams), nc, eb).bytes;
}

extern "C" int ddm_scan_certified(const uint8_t* err, const int64_t* stream_off, const int64_t* stream_end,
                                  int64_t n_streams, int64_t max_rows, const ddm_params* prm, ddm_state* state_io,
                                  double* bound_io, const int64_t* batch_base, int32_t* ev_out, int32_t* stop_out,
                                  int64_t* nev_out, int32_t mode, const uint8_t* perm_map, int32_t* status_out,
                                  void* scratch, ddm_stream_t stream, ddm_event_t ev_begin, ddm_event_t ev_end) {
    if (!err || !stream_off || !prm || !state_io || !batch_base || !ev_out || !scratch || n_streams < 0 ||
        max_rows < 0 || prm->per_batch <= 0 || prm->per_batch > kMaxBatch || (mode != 0 && mode != 1)) {
        ddm::set_error("ddm_scan_certified: invalid argument (per_batch must be 1..%d)", kMaxBatch);
        return DDM_E_ARG;
    }
    if (n_streams == 0 || max_rows == 0) return 0;
    const int64_t nc = ddm::ceil_div(max_rows, kChunk);
    if (n_streams * nc >= ((int64_t)1 << 31) / kThreads || max_rows >= ((int64_t)1 << 31) - kChunk) {
        ddm::set_error("ddm_scan_certified: too many chunks");
        return DDM_E_ARG;
    }
    const CertScratch sc = cert_scratch(scratch, n_streams, nc, ddm_scan_long_scratch_bytes(n_streams, max_rows,
                                                                                              prm->per_batch));
    const int64_t zero_words = ddm_scan_long_flag_bytes(n_streams, max_rows, prm->per_batch) / 4;
    hipStream_t s = ddm::as_hip(stream);
    if (ev_begin)
        if (int rc = ddm::hip_status(hipEventRecord(reinterpret_cast<hipEvent_t>(ev_begin), s), "event record")) return rc;
    const dim3 gs((unsigned)ddm::ceil_div(n_streams, 64)), gc((unsigned)(n_streams * nc));
    const int pb = prm->per_batch;
    int32_t* any_fb = sc.only + n_streams;
    hipLaunchKernelGGL(k_cert_setup, dim3((unsigned)std::max<int64_t>(ddm::ceil_div(n_streams, 64), 64)), dim3(64), 0,
                       s, sc.hdr, stream_off, stream_end, n_streams, any_fb, static_cast<uint32_t*>(sc.exact),
                       zero_words, sc.evc, n_streams * nc);
    const int rounds = mode == 0 ? 1 : kCertRounds;
    for (int r = 0; r < rounds; ++r) {
        if (r) hipLaunchKernelGGL(k_cert_advance, gs, dim3(64), 0, s, sc.hdr, n_streams);
        hipLaunchKernelGGL(k_cert_count, gc, dim3(kThreads), 0, s, sc.hdr, err, n_streams, nc, pb, sc.cnt, sc.skl,
                           sc.f0, sc.f1, ev_out, batch_base);
        hipLaunchKernelGGL(k_cert_scan1, dim3((unsigned)n_streams), dim3(kThreads), 0, s, sc.hdr, nc, sc.cnt, sc.skl,
                           sc.f0, sc.f1, sc.kb, sc.skb, state_io, bound_io, r);
        hipLaunchKernelGGL(k_cert_eval, gc, dim3(kThreads), 0, s, sc.hdr, err, n_streams, nc, prm->min_num_instances,
                           sc.kb, sc.skb, sc.agg, sc.tkey);
        hipLaunchKernelGGL(k_cert_scan2, dim3((unsigned)n_streams), dim3(kThreads), 0, s, sc.hdr, nc, sc.agg,
                           sc.minb);
        hipLaunchKernelGGL(k_cert_decide, gc, dim3(kThreads), 0, s, sc.hdr, err, n_streams, nc, *prm, sc.kb, sc.skb,
                           sc.agg, sc.minb, sc.tkey, sc.rec_chg, sc.rec_end, ev_out, batch_base, g_tol_scale);
        hipLaunchKernelGGL(k_cert_final, gs, dim3(64), 0, s, sc.hdr, n_streams, nc, pb, (int)mode, sc.rec_chg,
                           sc.rec_end, state_io, bound_io, stop_out);
        hipLaunchKernelGGL(k_cert_fix, gc, dim3(kThreads), 0, s, sc.hdr, n_streams, nc, pb, (int)mode, ev_out,
                           batch_base, perm_map, sc.evc);
        if (int rc = ddm::launch_status("ddm_scan_certified")) return rc;
    }
    hipLaunchKernelGGL(k_cert_prep_fb, gs, dim3(64), 0, s, sc.hdr, n_streams, pb, batch_base, sc.fb_off, sc.fb_end,
                       sc.fb_bb, sc.only, any_fb);
    if (int rc = ddm::launch_status("ddm_scan_certified")) return rc;
    // the exact kernel for the streams that need it (every block exits at once when none
    // does); it writes their events, state, stop and event count from their current start
    if (int rc = ddm_scan_long_only(err, sc.fb_off, sc.fb_end, n_streams, max_rows, prm, state_io, sc.fb_bb, ev_out,
                                    stop_out, sc.nev_fb, mode, perm_map, sc.exact, sc.only, any_fb, stream))
        return rc;
    hipLaunchKernelGGL(k_cert_done, dim3((unsigned)n_streams), dim3(kThreads), 0, s, sc.hdr, nc, sc.evc, sc.nev_fb,
                       nev_out, bound_io, status_out);
    if (int rc = ddm::launch_status("ddm_scan_certified")) return rc;
    if (ev_end)
        if (int rc = ddm::hip_status(hipEventRecord(reinterpret_cast<hipEvent_t>(ev_end), s), "event record")) return rc;
    return 0;
}

extern "C" int ddm_scan_certified_set_tol_scale(double scale) {
    if (!(scale >= 1.0)) {
        ddm::set_error("ddm_scan_certified_set_tol_scale: scale must be >= 1");
        return DDM_E_ARG;
    }
    g_tol_scale = scale;
    return 0;
}
