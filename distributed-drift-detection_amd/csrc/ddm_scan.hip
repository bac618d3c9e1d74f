// DDM scan over error streams: run_DDM (DDM_Process.py:135-159) batch after batch.
//
// One lane owns one stream and runs scikit-multiflow's DDM recurrence exactly
// (fp64, no FMA contraction: built with -ffp-contract=off), so p, s and every
// decision are bit-identical to the reference arithmetic.  Throughput comes from
// (a) many streams in flight (C4: 1M streams = 16k waves) and (b) the zero-run
// fast path: while the detector is in its trivial state (every error so far 0:
// p = s = p_min = s_min = 0 after the gate) a 0 leaves the state unchanged except
// sample_count, so runs of zeros are skipped with `ctz` over 16-byte chunks and,
// with the `first_nz` hint produced by the predict kernel, in one jump.
//
// HBM layout: err is one uint8 per row in DDM order (the shuffled order of
// DDM_Process.py:190), streams back to back; events are int32 pairs per batch.
#include "common.h"
#include "det.h"
#include "wave_det.h"

namespace {

// First byte index t in [k, limit) of the 16-byte chunk (lo | hi << 64) that is
// nonzero, or limit.
__device__ __forceinline__ int first_nonzero_byte(uint64_t lo, uint64_t hi, int k, int limit) {
    if (k >= 8) {
        lo = 0;
        hi &= ~0ull << (8 * (k - 8));
    } else {
        lo &= ~0ull << (8 * k);
    }
    int t = lo ? (__builtin_ctzll(lo) >> 3) : (hi ? 8 + (__builtin_ctzll(hi) >> 3) : 16);
    return t < limit ? t : limit;
}

__global__ __launch_bounds__(256) void k_scan_streams(
    const uint8_t* __restrict__ err, const int64_t* __restrict__ off, int64_t n_streams,
    ddm_params P, ddm_state* __restrict__ state, const uint64_t* __restrict__ first_nz,
    const int64_t* __restrict__ batch_base, int32_t* __restrict__ ev, int32_t* __restrict__ stop_out,
    int64_t* __restrict__ nev_out, int mode, double* __restrict__ ps_out, const uint8_t* __restrict__ pmap,
    const int64_t* __restrict__ stream_end) {
    const int64_t sid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (sid >= n_streams) return;
    const int64_t lo = off[sid], hi = stream_end ? stream_end[sid] : off[sid + 1];
    const int64_t pb = P.per_batch;
    const int min_inst = P.min_num_instances;
    const double wl = P.warning_level, cl = P.out_control_level;

    Det d;
    {
        const ddm_state st = state[sid];
        d.p = st.miss_prob;
        d.s = st.miss_std;
        d.pmin = st.miss_prob_min;
        d.smin = st.miss_sd_min;
        d.psmin = st.miss_prob_sd_min;
        d.n = st.sample_count;
        d.chg = st.in_concept_change;
        d.warn = st.in_warning_zone;
    }
    const uint64_t hint = first_nz ? first_nz[sid] : 0ull;
    int32_t* evs = ev + 2 * batch_base[sid];
    int64_t nev = 0;
    int32_t stop = -1;
    int64_t b = 0, bstart = lo, bend = min(lo + pb, hi);
    int wpos = -1;
    int64_t i = lo;
    int64_t cbase = -1;
    uint64_t clo = 0, chi = 0;

    while (i < hi) {
        if (det_trivial(d)) {
            // Jump over a zero run: to the hinted first nonzero row, or past the zero
            // bytes of the current chunk (never past the current batch).
            int64_t j = i;
            if (hint > (uint64_t)i) {
                j = hint < (uint64_t)hi ? (int64_t)hint : hi;
            } else {
                const int64_t cb = i & ~(int64_t)15;
                if (cb != cbase) {
                    const uint4 v = *reinterpret_cast<const uint4*>(err + cb);
                    clo = (uint64_t)v.x | ((uint64_t)v.y << 32);
                    chi = (uint64_t)v.z | ((uint64_t)v.w << 32);
                    cbase = cb;
                }
                const int lim = (int)min((int64_t)16, min(hi, bend) - cb);
                j = cb + first_nonzero_byte(clo, chi, (int)(i - cb), lim);
            }
            if (j > i) {
                if (ps_out)
                    for (int64_t k = i; k < j; ++k) ps_out[2 * k] = ps_out[2 * k + 1] = 0.0;
                d.n += j - i;
                d.warn = 0;
                i = j;
                if (i >= bend) {  // whole batches of zeros: no event can have occurred
                    b = (i - lo) / pb;
                    bstart = lo + b * pb;
                    bend = min(bstart + pb, hi);
                    wpos = -1;
                }
                continue;
            }
        }
        const int64_t cb = i & ~(int64_t)15;
        if (cb != cbase) {
            const uint4 v = *reinterpret_cast<const uint4*>(err + cb);
            clo = (uint64_t)v.x | ((uint64_t)v.y << 32);
            chi = (uint64_t)v.z | ((uint64_t)v.w << 32);
            cbase = cb;
        }
        const int k = (int)(i - cb);
        const int x = (int)(((k < 8 ? clo >> (8 * k) : chi >> (8 * (k - 8)))) & 0xff) != 0;
        det_add(d, x, min_inst, wl, cl);
        if (ps_out) {
            ps_out[2 * i] = d.p;
            ps_out[2 * i + 1] = d.s;
        }
        if (d.warn && wpos < 0) wpos = (int)(i - bstart);
        ++i;
        if (d.chg) {
            const int cpos = (int)(i - 1 - bstart);
            evs[2 * b] = (pmap && wpos >= 0) ? (int)pmap[bstart + wpos] : wpos;
            evs[2 * b + 1] = pmap ? (int)pmap[bstart + cpos] : cpos;
            ++nev;
            if (mode == 0) {
                stop = (int32_t)b;
                break;
            }
            det_reset(d);  // DDM dropped (DDM_Process.py:209), fresh one next batch
            i = bend;
        } else if (i >= bend && wpos >= 0) {
            evs[2 * b] = pmap ? (int)pmap[bstart + wpos] : wpos;
            ++nev;
        }
        if (i >= bend) {
            ++b;
            bstart = bend;
            bend = min(bstart + pb, hi);
            wpos = -1;
        }
    }

    ddm_state st;
    st.miss_prob = d.p;
    st.miss_std = d.s;
    st.miss_prob_min = d.pmin;
    st.miss_sd_min = d.smin;
    st.miss_prob_sd_min = d.psmin;
    st.sample_count = d.n;
    st.in_concept_change = d.chg;
    st.in_warning_zone = d.warn;
    state[sid] = st;
    if (stop_out) stop_out[sid] = stop;
    if (nev_out) nev_out[sid] = nev;
}


// ---------------------------------------------------------------------------------
// Production scan (no p/s trace): the same decisions and states, bit for bit, with a
// cheaper exact row and shortcuts that need no arithmetic at all.
//
//  * Division by n: q = RN(a / n) from r = RN(1/n) with one Markstein correction,
//    q0 = a*r, e = fma(-q0, n, a), q = fma(e, r, q0) (exact remainder; correctly rounded
//    quotient for a correctly rounded reciprocal).  RN(1/n) comes from an LDS table for
//    n < kRcpN, otherwise from an IEEE division.
//  * Fresh detector + two zero rows == the trivial state with n = 3 (p, s and the three
//    minima all 0) without evaluating them.
//  * Trivial state (gate passed) + an error row: p + s > 0 = p_min + c * s_min, i.e. a
//    change at that row (and no warning, the `elif`).  In mode 1 the detector is then
//    dropped, so nothing of that row needs computing; mode 0 stops there and computes the
//    row exactly for the carried state.
//  * Each lane works through several streams (grid-stride), which evens out the very
//    different amounts of exact rows per stream across the 64 lanes of a wave.
constexpr int kFastThreads = 256;

__device__ __forceinline__ int byte_at(uint64_t lo, uint64_t hi, int k) {
    return (int)(((k < 8 ? lo >> (8 * k) : hi >> (8 * (k - 8)))) & 0xff);
}

// One lane = a persistent worker over streams sid, sid + nthreads, ...  The body is ONE
// flat loop whose iterations each do one step of one kind (start/finish a stream, two
// leading zeros, a zero run, a trivial-state change, or an exact row): no nested loops,
// so a lane that finishes a stream starts its next one at once instead of idling until
// the slowest lane of its wave is done with the same round.
__global__ __launch_bounds__(kFastThreads) void k_scan_fast(
    const uint8_t* __restrict__ err, const int64_t* __restrict__ off, int64_t n_streams, ddm_params P,
    ddm_state* __restrict__ state, const uint64_t* __restrict__ first_nz, const int64_t* __restrict__ batch_base,
    int32_t* __restrict__ ev, int32_t* __restrict__ stop_out, int64_t* __restrict__ nev_out, int mode,
    const uint8_t* __restrict__ pmap, const int64_t* __restrict__ stream_end) {
    __shared__ double rcp[kRcpN];
    for (int k = threadIdx.x; k < kRcpN; k += kFastThreads) rcp[k] = 1.0 / (double)(k > 0 ? k : 1);
    __syncthreads();
    const int64_t pb = P.per_batch;
    const int min_inst = P.min_num_instances;
    const double wl = P.warning_level, cl = P.out_control_level;
    const bool shortcuts = min_inst == 3;   // the trivial-state shortcuts assume the reference gate
    const int64_t nthreads = (int64_t)gridDim.x * kFastThreads;

    int64_t sid = (int64_t)blockIdx.x * kFastThreads + threadIdx.x - nthreads;   // advanced on the first step
    int64_t lo = 0, hi = 0, b = 0, bstart = 0, bend = 0, i = 0, cbase = -1, nev = 0;
    uint64_t hint = 0, clo = 0, chi = 0;
    int32_t* evs = ev;
    int32_t stop = -1;
    int wpos = -1;
    bool open = false;                      // a stream is loaded
    Det d;
    d.p = d.s = d.pmin = d.smin = d.psmin = 0.0;
    d.n = 1;
    d.chg = d.warn = 0;

    for (;;) {
        if (!open || i >= hi) {
            if (open) {                     // finish the stream
                ddm_state st;
                st.miss_prob = d.p;
                st.miss_std = d.s;
                st.miss_prob_min = d.pmin;
                st.miss_sd_min = d.smin;
                st.miss_prob_sd_min = d.psmin;
                st.sample_count = d.n;
                st.in_concept_change = d.chg;
                st.in_warning_zone = d.warn;
                state[sid] = st;
                if (stop_out) stop_out[sid] = stop;
                if (nev_out) nev_out[sid] = nev;
            }
            sid += nthreads;
            if (sid >= n_streams) break;
            lo = off[sid];
            hi = stream_end ? stream_end[sid] : off[sid + 1];
            const ddm_state st = state[sid];
            d.p = st.miss_prob;
            d.s = st.miss_std;
            d.pmin = st.miss_prob_min;
            d.smin = st.miss_sd_min;
            d.psmin = st.miss_prob_sd_min;
            d.n = st.sample_count;
            d.chg = st.in_concept_change;
            d.warn = st.in_warning_zone;
            hint = first_nz ? first_nz[sid] : 0ull;
            evs = ev + 2 * batch_base[sid];
            nev = 0;
            stop = -1;
            b = 0;
            bstart = lo;
            bend = min(lo + pb, hi);
            wpos = -1;
            i = lo;
            cbase = -1;
            open = true;
            continue;
        }
        // the 16-byte chunk holding row i (and row i+1 for the two-zero test)
        const int64_t cb = i & ~(int64_t)15;
        if (cb != cbase) {
            const uint4 v = *reinterpret_cast<const uint4*>(err + cb);
            clo = (uint64_t)v.x | ((uint64_t)v.y << 32);
            chi = (uint64_t)v.z | ((uint64_t)v.w << 32);
            cbase = cb;
        }
        const int k = (int)(i - cb);
        const int xi = byte_at(clo, chi, k);
        const bool triv = det_trivial(d);
        bool changed = false;
        if (shortcuts && !triv && i + 1 < bend && det_fresh(d) && xi == 0 &&
            (k < 15 ? byte_at(clo, chi, k + 1) : (int)err[i + 1]) == 0) {
            // fresh detector, two zero rows: the trivial state with the gate passed
            d.p = d.s = d.pmin = d.smin = d.psmin = 0.0;
            d.n = 3;
            d.chg = d.warn = 0;
            i += 2;
        } else if (triv && xi == 0) {
            // a zero run in the trivial state: to the hinted first nonzero row, or past the
            // zero bytes of this chunk (never past the current batch)
            int64_t j;
            if (hint > (uint64_t)i) {
                j = hint < (uint64_t)hi ? (int64_t)hint : hi;
            } else {
                const int lim = (int)min((int64_t)16, min(hi, bend) - cb);
                j = cb + first_nonzero_byte(clo, chi, k, lim);
            }
            d.n += j - i;
            d.warn = 0;
            i = j;
            if (i >= bend) {                // whole batches of zeros: no event can have occurred
                b = (i - lo) / pb;
                bstart = lo + b * pb;
                bend = min(bstart + pb, hi);
                wpos = -1;
            }
        } else if (shortcuts && triv && mode == 1 && d.n >= 3) {
            // an error row in the trivial state: change here (p + s > 0); the detector is
            // dropped, so the row needs no arithmetic
            changed = true;
            det_reset(d);
            ++i;
        } else {
            det_add_fast(d, xi != 0, min_inst, wl, cl, rcp);
            if (d.warn && wpos < 0) wpos = (int)(i - bstart);
            ++i;
            changed = d.chg != 0;
            if (changed && mode == 1) det_reset(d);   // DDM dropped (DDM_Process.py:209)
        }
        if (changed) {
            const int cpos = (int)(i - 1 - bstart);
            evs[2 * b] = (pmap && wpos >= 0) ? (int)pmap[bstart + wpos] : wpos;
            evs[2 * b + 1] = pmap ? (int)pmap[bstart + cpos] : cpos;
            ++nev;
            if (mode == 0) {
                stop = (int32_t)b;
                i = hi;                     // finish this stream
                continue;
            }
            i = bend;                       // fresh detector from the next batch
        } else if (i >= bend && wpos >= 0) {
            evs[2 * b] = pmap ? (int)pmap[bstart + wpos] : wpos;
            ++nev;
        }
        if (i >= bend && i < hi) {
            ++b;
            bstart = bend;
            bend = min(bstart + pb, hi);
            wpos = -1;
        }
    }
}

// ---------------------------------------------------------------------------------
// Batch-parallel scan for many independent, equal-length, back-to-back streams in mode 1
// (configs[3]: 1M streams x 4096 rows, reset-heavy).
//
// In mode 1 a change drops the detector and the next batch starts fresh
// (DDM_Process.py:207-210), so every batch whose predecessor changed is independent of
// everything before it.  On reset-heavy streams that is nearly every batch, so:
//
//  * k_scan_batches_spec: every batch of every stream is scanned on its own with a FRESH
//    detector (speculation).  A batch is one work item; a wave owns a contiguous range of
//    items and hands them to its lanes dynamically (refill when >= kRefill lanes are idle),
//    so the short trivial items and the long exact ones even out over the wave and each
//    wave-iteration is either a refill or an exact row, never both.  Starting an item
//    loads its <= 128 bytes as 16-byte chunks, folds them into a 128-bit nonzero mask
//    and resolves the trivial case at once (two leading zeros then the first error is
//    the change, or no error at all); otherwise the lane runs exact rows, x from the mask,
//    1/n from a 1 KB LDS table (n <= 129 inside one batch).
//    It writes the item's (warning, change) pair and a flag byte (bit 0 change, bit 1 any
//    event).
//  * k_scan_batches_fix: one lane per stream walks its flag bytes.  A batch whose
//    detector really is fresh (the carried state for batch 0, a change before it
//    otherwise) keeps the speculative result; every other batch (the successor of an
//    unchanged batch) is rescanned exactly with the carried detector, which also
//    rebuilds the carry through unchanged batches.  It writes the carried state and the
//    per-stream event count.
//
// Decisions are those of k_scan_streams bit for bit: the same recurrence, the same
// shortcuts (gate 3 only), the same event positions.
constexpr int kBatchRcp = 160;
constexpr int kSpecThreads = 256;
constexpr int kMaxBatch = 128;

// bit k set <=> byte k of w is nonzero
__device__ __forceinline__ uint32_t nz4(uint32_t w) {
    const uint32_t t = (((w & 0x7f7f7f7fu) + 0x7f7f7f7fu) | w) & 0x80808080u;
    return (((t >> 7) * 0x00204081u) >> 21) & 0xfu;
}

__device__ __forceinline__ uint32_t nz16(uint4 v) {
    return nz4(v.x) | (nz4(v.y) << 4) | (nz4(v.z) << 8) | (nz4(v.w) << 12);
}

// nz4 for a word whose bytes are 0 or 1 (what predict writes): the multiply moves byte
// k's bit 0 to bit 21 + k with no two partial products on the same bit (no carries).
__device__ __forceinline__ uint32_t bin4(uint32_t w) { return ((w * 0x00204081u) >> 21) & 0xfu; }

__device__ __forceinline__ uint32_t bin16(uint4 v) {
    return bin4(v.x) | (bin4(v.y) << 4) | (bin4(v.z) << 8) | (bin4(v.w) << 12);
}

// 128-bit nonzero mask of the rows [bstart, bstart + blen), blen in 1..128: bit t of
// (m0, m1) = row bstart + t is an error.  All nine 16-byte loads are issued before any
// is used (chunk addresses past the batch are clamped to its last chunk, their bits
// dropped).
__device__ __forceinline__ void batch_load(const uint8_t* __restrict__ err, int64_t bstart, int blen, uint4 (&v)[9]) {
    const int64_t c0 = bstart & ~(int64_t)15;
    const int64_t clast = (bstart + blen - 1) & ~(int64_t)15;
#pragma unroll
    for (int k = 0; k < 9; ++k) v[k] = *reinterpret_cast<const uint4*>(err + min(c0 + 16 * k, clast));
}

__device__ __forceinline__ void batch_mask_of(const uint4 (&v)[9], int64_t bstart, int blen, uint64_t& m0,
                                              uint64_t& m1) {
    const int off = (int)(bstart & 15);
    const int nch = (off + blen + 15) >> 4;
    uint32_t c[9];
    uint32_t any = 0;
#pragma unroll
    for (int k = 0; k < 9; ++k) any |= v[k].x | v[k].y | v[k].z | v[k].w;
    if ((any & 0xfefefefeu) == 0u) {            // 0/1 bytes only: the cheap fold
#pragma unroll
        for (int k = 0; k < 9; ++k) c[k] = k < nch ? bin16(v[k]) : 0u;
    } else {
#pragma unroll
        for (int k = 0; k < 9; ++k) c[k] = k < nch ? nz16(v[k]) : 0u;
    }
    const uint64_t a0 = (uint64_t)c[0] | ((uint64_t)c[1] << 16) | ((uint64_t)c[2] << 32) | ((uint64_t)c[3] << 48);
    const uint64_t a1 = (uint64_t)c[4] | ((uint64_t)c[5] << 16) | ((uint64_t)c[6] << 32) | ((uint64_t)c[7] << 48);
    const uint64_t a2 = c[8];
    m0 = off ? (a0 >> off) | (a1 << (64 - off)) : a0;
    m1 = off ? (a1 >> off) | (a2 << (64 - off)) : a1;
    if (blen < 64) {
        m0 &= (1ull << blen) - 1;
        m1 = 0;
    } else if (blen < 128) {
        m1 &= (1ull << (blen - 64)) - 1;
    }
}

__device__ __forceinline__ void batch_mask(const uint8_t* __restrict__ err, int64_t bstart, int blen,
                                           uint64_t& m0, uint64_t& m1) {
    uint4 v[9];
    batch_load(err, bstart, blen, v);
    batch_mask_of(v, bstart, blen, m0, m1);
}

__device__ __forceinline__ int mask_bit(uint64_t m0, uint64_t m1, int i) {
    return (int)((i < 64 ? m0 >> i : m1 >> (i - 64)) & 1ull);
}

// first set bit at or after i (128 if none)
__device__ __forceinline__ int mask_next(uint64_t m0, uint64_t m1, int i) {
    if (i < 64) {
        const uint64_t t = m0 & (~0ull << i);
        if (t) return __builtin_ctzll(t);
        return m1 ? 64 + __builtin_ctzll(m1) : 128;
    }
    if (i >= 128) return 128;
    const uint64_t t = m1 & (~0ull << (i - 64));
    return t ? 64 + __builtin_ctzll(t) : 128;
}

struct SmallDet {          // a detector inside one batch: n <= kMaxBatch + 1
    double p, s, pmin, smin, psmin;
    int n;
};

// returns 2 = change, 1 = warning, 0 = neither
__device__ __forceinline__ int small_add(SmallDet& d, int x, int min_inst, double wl, double cl,
                                         const double* __restrict__ rcp) {
    const double n = (double)d.n;
    const double r = rcp[d.n];
    const double p = d.p + div_rn((double)x - d.p, n, r);
    const double s = sqrt_q(div_rn(p * (1.0 - p), n, r));
    d.p = p;
    d.s = s;
    d.n += 1;
    if (d.n < min_inst) return 0;
    const double ps = p + s;
    if (ps <= d.psmin) {
        d.pmin = p;
        d.smin = s;
        d.psmin = ps;
    }
    if (ps > d.pmin + cl * d.smin) return 2;
    return ps > d.pmin + wl * d.smin ? 1 : 0;
}

// Prefix table: a fresh detector's first kPre rows depend only on their kPre error bits,
// so the spec kernel looks them up instead of stepping them.  Entry m (bit t = row t is
// an error) holds the first warning row and the change row inside the prefix (-1 = none)
// and, without a change, the detector after row kPre - 1 (p, p_min, s_min, psmin; n =
// kPre + 1).  It is built with small_add itself and the same reciprocal table, so a
// looked-up prefix is the stepped one bit for bit.
constexpr int kPre = 16;
constexpr int kPreN = 1 << kPre;

__global__ __launch_bounds__(256) void k_scan_prefix_table(ddm_params P, double4* __restrict__ pst,
                                                           int2* __restrict__ pinfo) {
    __shared__ double rcp[kBatchRcp];
    for (int k = threadIdx.x; k < kBatchRcp; k += 256) rcp[k] = 1.0 / (double)(k > 0 ? k : 1);
    __syncthreads();
    const int m = blockIdx.x * 256 + threadIdx.x;
    if (m >= kPreN) return;
    SmallDet d;
    d.p = 1.0;
    d.s = 0.0;
    d.pmin = d.smin = d.psmin = __builtin_huge_val();
    d.n = 1;
    int wpos = -1, cpos = -1;
    for (int i = 0; i < kPre; ++i) {
        const int r = small_add(d, (m >> i) & 1, P.min_num_instances, P.warning_level, P.out_control_level, rcp);
        if (r == 1 && wpos < 0) wpos = i;
        if (r == 2) {
            cpos = i;
            break;
        }
    }
    pinfo[m] = make_int2(wpos, cpos);
    pst[m] = make_double4(d.p, d.pmin, d.smin, d.psmin);
}

// The tests of one row whose p and s are already computed (small_add's second half).
__device__ __forceinline__ int small_test(SmallDet& d, double p, double s, int min_inst, double wl, double cl) {
    d.p = p;
    d.s = s;
    d.n += 1;
    if (d.n < min_inst) return 0;
    const double ps = p + s;
    if (ps <= d.psmin) {
        d.pmin = p;
        d.smin = s;
        d.psmin = ps;
    }
    if (ps > d.pmin + cl * d.smin) return 2;
    return ps > d.pmin + wl * d.smin ? 1 : 0;
}

__device__ __forceinline__ bool state_fresh(const ddm_state& st) {
    return st.in_concept_change || (st.sample_count == 1 && st.miss_prob == 1.0 && st.miss_std == 0.0 &&
                                    st.miss_prob_sd_min == __builtin_huge_val() &&
                                    st.miss_prob_min == __builtin_huge_val() && st.miss_sd_min == __builtin_huge_val());
}

// The fix-up list: streams with an unchanged batch (need[s], stored by the speculative
// pass) or a carry-in that is not fresh.  Every other stream's speculation is its result:
// the reset state (its last batch changed) and nb batches with an event.  A thread looks
// at kListPer streams (coalesced, 256 apart) and a block takes its list slots with ONE
// atomic (one per wave made the counter a serialisation point: 0.19 ms on 1M streams).
constexpr int kListPer = 8;

__global__ __launch_bounds__(256) void k_scan_batches_list(int64_t n_streams, int64_t nb,
                                                           ddm_state* __restrict__ state,
                                                           const uint32_t* __restrict__ need,
                                                           int64_t* __restrict__ nev_out, int32_t* __restrict__ list,
                                                           uint32_t* __restrict__ ctr) {
    __shared__ uint32_t wcount[4], wbase[4];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t below = (1ull << lane) - 1;
    const int64_t t0 = (int64_t)blockIdx.x * 256 * kListPer + threadIdx.x;
    uint32_t bits = 0, cnt = 0;
#pragma unroll
    for (int k = 0; k < kListPer; ++k) {
        const int64_t t = t0 + (int64_t)k * 256;
        bool fix = false;
        if (t < n_streams) {
            fix = need[t] != 0u || !state_fresh(state[t]);
            if (!fix) {
                if (nb > 0) {
                    ddm_state st;
                    st.miss_prob = 1.0;
                    st.miss_std = 0.0;
                    st.miss_prob_min = st.miss_sd_min = st.miss_prob_sd_min = __builtin_huge_val();
                    st.sample_count = 1;
                    st.in_concept_change = 0;
                    st.in_warning_zone = 0;
                    state[t] = st;
                }
                if (nev_out) nev_out[t] = nb;
            }
        }
        bits |= (fix ? 1u : 0u) << k;
        cnt += (uint32_t)__popcll(__ballot(fix));
    }
    if (lane == 0) wcount[wv] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t total = wcount[0] + wcount[1] + wcount[2] + wcount[3];
        uint32_t b = total ? atomicAdd(ctr, total) : 0u;
        for (int w = 0; w < 4; ++w) {
            wbase[w] = b;
            b += wcount[w];
        }
    }
    __syncthreads();
    uint32_t off = wbase[wv];
#pragma unroll
    for (int k = 0; k < kListPer; ++k) {
        const bool fix = (bits >> k) & 1u;
        const uint64_t m = __ballot(fix);
        if (fix) list[off + __popcll(m & below)] = (int32_t)(t0 + (int64_t)k * 256);
        off += (uint32_t)__popcll(m);
    }
}

// Flag byte of a batch (k_scan_batches_spec -> k_scan_batches_fix): bit 0 change, bit 1
// any event, bit 2 end state stored (pend), and what a TRIVIAL carried detector (every
// error so far 0, gate passed) makes of the batch, without its bytes: bit 5 no error at
// all (it stays trivial), bit 3 an error in row 0 or 1 (the change is that row; bit 4:
// row 1), else the change is the batch's first error row, as the fresh speculation found.
constexpr uint8_t kFlagLead01 = 8, kFlagLeadRow1 = 16, kFlagNoError = 32;

__device__ __forceinline__ uint8_t lead_bits(uint64_t m0, uint64_t m1) {
    if ((m0 | m1) == 0) return kFlagNoError;
    if (m0 & 3ull) return (uint8_t)(kFlagLead01 | ((m0 & 1ull) ? 0 : kFlagLeadRow1));
    return 0;
}

// Per-wave LDS queue of the batches that need exact rows (mask + batch), see below.
constexpr int kSpecQ = 256;
constexpr bool kSpecPrefetch = false;   // next fill's bytes ahead (36 VGPRs; measured no gain)

template <bool kPmap>
__global__ __launch_bounds__(kSpecThreads) void k_scan_batches_spec(
    const uint8_t* __restrict__ err, int64_t n_items, int64_t L, int64_t nb, int64_t nbp, ddm_params P,
    int2* __restrict__ ev, uint8_t* __restrict__ flags, const uint8_t* __restrict__ pmap,
    int64_t items_per_wave, int fill_below, int pop_min, uint32_t* __restrict__ need,
    const double4* __restrict__ pst, const int2* __restrict__ pinfo, double2* __restrict__ pend) {
    __shared__ double rcp[kBatchRcp];
    __shared__ uint64_t qm0[kSpecThreads / 64][kSpecQ], qm1[kSpecThreads / 64][kSpecQ];
    __shared__ uint32_t qitem[kSpecThreads / 64][kSpecQ], qsid[kSpecThreads / 64][kSpecQ];
    __shared__ uint32_t qjl[kSpecThreads / 64][kSpecQ];
    for (int k = threadIdx.x; k < kBatchRcp; k += kSpecThreads) rcp[k] = 1.0 / (double)(k > 0 ? k : 1);
    __syncthreads();
    const int pb = (int)P.per_batch;
    const int min_inst = P.min_num_instances;
    const double wl = P.warning_level, cl = P.out_control_level;
    const bool shortcuts = min_inst == 3;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t below = (1ull << lane) - 1;
    const int64_t wave = (int64_t)blockIdx.x * (kSpecThreads / 64) + wv;
    const int64_t wstart = wave * items_per_wave;
    const int64_t wend = min(wstart + items_per_wave, n_items);
    int64_t cursor = wstart;
    const double inv_nb = 1.0 / (double)nb;
    int qhead = 0, qcount = 0;                      // wave-uniform ring state
    // the next fill's batch bytes, loaded right after the current fill so that their
    // latency hides behind the exact rows in between
    uint4 nv[9];
    bool nv_ok = false;

    bool busy = false;
    int64_t item = 0, bstart = 0, fpos = 0, sid = 0;
    int blen = 0, i = 0, wpos = -1;
    uint64_t m0 = 0, m1 = 0;
    SmallDet d;
    d.p = d.s = d.pmin = d.smin = d.psmin = 0.0;
    d.n = 1;

    auto locate = [&](int64_t it) {                 // item -> stream, batch, rows, flag slot
        int64_t s = (int64_t)((double)it * inv_nb);
        if (s * nb > it) --s;
        else if ((s + 1) * nb <= it) ++s;
        const int64_t j = it - s * nb;
        sid = s;
        bstart = s * L + j * pb;
        fpos = s * nbp + j;
        blen = (int)min((int64_t)pb, L - j * pb);
    };
    auto finish = [&](bool chg, int wp, int c) {    // the batch's result (c: change row)
        // without a perm map no load precedes the stores (a load here made every store
        // wait for all outstanding memory operations)
        const int w = wp < 0 ? -1 : (kPmap ? (int)pmap[bstart + wp] : wp);
        const int cp = chg ? (kPmap ? (int)pmap[bstart + c] : c) : -1;
        ev[item] = make_int2(w, cp);
        flags[fpos] = (uint8_t)((chg ? 1 : 0) | ((chg || wp >= 0) ? 2 : 0) | lead_bits(m0, m1));
        if (!chg) need[sid] = 1u;
    };

    for (;;) {
        const uint64_t idle_m = __ballot(!busy);
        int nidle = __popcll(idle_m);
        if (qcount > 0 && (nidle >= pop_min || nidle == 64 || (nidle > 0 && cursor >= wend))) {
            // pop: idle lanes take queued batches in lane order (LDS only; the queue entry
            // carries the batch's stream and index, so no division here)
            const int take = min(nidle, qcount);
            if (!busy) {
                const int rank = __popcll(idle_m & below);
                if (rank < take) {
                    const int q = (qhead + rank) & (kSpecQ - 1);
                    m0 = qm0[wv][q];
                    m1 = qm1[wv][q];
                    item = wstart + qitem[wv][q];
                    sid = qsid[wv][q];
                    const uint32_t jl = qjl[wv][q];
                    const int64_t j = jl >> 8;
                    blen = (int)(jl & 0xffu);
                    bstart = sid * L + j * pb;
                    fpos = sid * nbp + j;
                    busy = true;
                    i = 0;
                    wpos = -1;
                    d.p = 1.0;
                    d.s = 0.0;
                    d.pmin = d.smin = d.psmin = __builtin_huge_val();
                    d.n = 1;
                    if (pinfo && blen >= kPre) {
                        // the first kPre rows from the prefix table
                        // both table loads issued together: one wait per pop
                        const uint32_t ix = (uint32_t)(m0 & (uint64_t)(kPreN - 1));
                        const int2 inf = pinfo[ix];
                        const double4 q = pst[ix];
                        if (inf.y >= 0 || blen == kPre) {
                            finish(inf.y >= 0, inf.x, inf.y);
                            busy = false;
                        } else {
                            d.p = q.x;
                            d.pmin = q.y;
                            d.smin = q.z;
                            d.psmin = q.w;
                            d.n = kPre + 1;
                            i = kPre;
                            wpos = inf.x;
                        }
                    }
                }
            }
            qhead = (qhead + take) & (kSpecQ - 1);
            qcount -= take;
            nidle -= take;
        }
        if (cursor < wend && qcount < fill_below) {
            // fill: the next 64 items, one per lane (all lanes; busy ones pause a step).
            // Trivial batches are resolved here; the others go to the queue.
            bool exact = false;
            uint64_t a0 = 0, a1 = 0;
            uint32_t e_sid = 0, e_jl = 0;
            const int64_t it = cursor + lane;
            if (it < wend) {
                const int64_t keep_item = item, keep_b = bstart, keep_f = fpos, keep_s = sid;
                const int keep_len = blen;
                locate(it);
                if (kSpecPrefetch) {
                    if (!nv_ok) batch_load(err, bstart, blen, nv);
                    batch_mask_of(nv, bstart, blen, a0, a1);
                } else {
                    batch_mask(err, bstart, blen, a0, a1);
                }
                if (shortcuts && blen >= 2 && (a0 & 3ull) == 0) {
                    // fresh + two zero rows = trivial state (n = 3); its first error row
                    // is the change (p + s > 0), and zeros raise nothing
                    const int t = mask_next(a0, a1, 2);
                    if (t < blen) {
                        ev[it] = make_int2(-1, pmap ? (int)pmap[bstart + t] : t);
                        flags[fpos] = 3;
                    } else {
                        ev[it] = make_int2(-1, -1);
                        flags[fpos] = kFlagNoError;
                        need[sid] = 1u;
                    }
                } else {
                    exact = true;
                    e_sid = (uint32_t)sid;
                    e_jl = (uint32_t)(((fpos - sid * nbp) << 8) | (int64_t)blen);
                }
                // prefetch the next fill's item (this lane's, 64 on)
                nv_ok = false;
                if (kSpecPrefetch && it + 64 < wend) {
                    locate(it + 64);
                    batch_load(err, bstart, blen, nv);
                    nv_ok = true;
                }
                item = keep_item;
                bstart = keep_b;
                fpos = keep_f;
                sid = keep_s;
                blen = keep_len;
            }
            const uint64_t ex_m = __ballot(exact);
            if (exact) {
                const int q = (qhead + qcount + __popcll(ex_m & below)) & (kSpecQ - 1);
                qm0[wv][q] = a0;
                qm1[wv][q] = a1;
                qitem[wv][q] = (uint32_t)(it - wstart);
                qsid[wv][q] = e_sid;
                qjl[wv][q] = e_jl;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            qcount += __popcll(ex_m);
            cursor += 64;
            continue;
        }
        if (nidle == 64) {
            if (cursor >= wend && qcount == 0) break;
            continue;
        }
        if (busy) {
            // two exact rows of the lane's batch.  p and s of row i+1 depend on p_i
            // alone, so both rows' arithmetic is computed first (two overlapping fp64
            // chains, the same operations as small_add), then the tests in row order;
            // row i+1 counts only if row i did not change.
            const bool two = i + 1 < blen;
            const int n0 = d.n;
            const double nd0 = (double)n0, r0 = rcp[n0], nd1 = (double)(n0 + 1), r1 = rcp[n0 + 1];
            const double p0 = d.p + div_rn((double)mask_bit(m0, m1, i) - d.p, nd0, r0);
            const double p1 = p0 + div_rn((double)(two ? mask_bit(m0, m1, i + 1) : 0) - p0, nd1, r1);
            const double s0 = sqrt_q(div_rn(p0 * (1.0 - p0), nd0, r0));
            const double s1 = sqrt_q(div_rn(p1 * (1.0 - p1), nd1, r1));
            int r = small_test(d, p0, s0, min_inst, wl, cl);
            if (r == 1 && wpos < 0) wpos = i;
            ++i;
            if (r != 2 && two) {
                r = small_test(d, p1, s1, min_inst, wl, cl);
                if (r == 1 && wpos < 0) wpos = i;
                ++i;
            }
            if (r == 2 || i >= blen) {
                finish(r == 2, wpos, i - 1);
                if (r != 2 && pend) {
                    // an unchanged batch: its end state, so the fix-up carries it on
                    // without rescanning the batch (flag bit 2)
                    double2* e = pend + 3 * item;
                    e[0] = make_double2(d.p, d.s);
                    e[1] = make_double2(d.pmin, d.smin);
                    e[2] = make_double2(d.psmin, (double)(2 * d.n + (r == 1 ? 1 : 0)));
                    flags[fpos] = (uint8_t)(((wpos >= 0) ? 2 : 0) | 4 | lead_bits(m0, m1));
                }
                busy = false;
            }
        }
    }
}

__device__ __forceinline__ void load_det(Det& d, const ddm_state& st) {
    d.p = st.miss_prob;
    d.s = st.miss_std;
    d.pmin = st.miss_prob_min;
    d.smin = st.miss_sd_min;
    d.psmin = st.miss_prob_sd_min;
    d.n = st.sample_count;
    d.chg = st.in_concept_change;
    d.warn = st.in_warning_zone;
}

__device__ __forceinline__ ddm_state store_det(const Det& d) {
    ddm_state st;
    st.miss_prob = d.p;
    st.miss_std = d.s;
    st.miss_prob_min = d.pmin;
    st.miss_sd_min = d.smin;
    st.miss_prob_sd_min = d.psmin;
    st.sample_count = d.n;
    st.in_concept_change = d.chg;
    st.in_warning_zone = d.warn;
    return st;
}

// Fix-up: persistent lanes take the streams of the fix-up list and run each batch after
// batch through one flat loop.  A lane is idle, waiting to open a batch, or stepping
// through one; each wave-iteration does one kind of work for the lanes in that state, so
// memory latency (claiming streams: state + flags; opening a batch: its 128-bit mask) is
// paid once for many lanes, and stepping never waits on memory:
//   claim  when >= refill lanes are idle: the next list entries, their carried state and
//          first 64-batch window of flags;
//   open   when >= open_thr lanes wait: skip the run of batches whose speculative change
//          stands (a fresh detector and a change flag: bit operations on the window),
//          finish the stream at its end, else load the batch mask;
//   step   one row step of the rescan (k_scan_fast's mode-1 rules, Markstein division).
constexpr int kFixThreads = 256;

// One 64-batch window of flag bytes as bit masks: bit 0 of each byte (change) into the
// result, bit 2 (end state stored) into sm, bit 1 (event) into em.
// bits [i, i + 64) of the 128-bit mask (a0 | a1 << 64), i < 64
__device__ __forceinline__ uint64_t m0_shift(uint64_t a0, uint64_t a1, int i) {
    return i == 0 ? a0 : (a0 >> i) | (a1 << (64 - i));
}

struct LeadMasks {           // flag bits 3, 4, 5 of a 64-batch window as bit masks
    uint64_t l01, row1, none;
};

__device__ __forceinline__ uint64_t change_window(const uint8_t* __restrict__ fl, int64_t wbase, int64_t nb,
                                                  uint64_t& sm, uint64_t& em, LeadMasks& lm) {
    uint64_t m = 0, ms = 0, me = 0, ml = 0, mr = 0, mz = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint4 v = *reinterpret_cast<const uint4*>(fl + wbase + 16 * q);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int sh = 16 * q + 4 * k;
            m |= (uint64_t)(((((w[k] >> 0) & 0x01010101u) * 0x00204081u) >> 21) & 0xfu) << sh;
            me |= (uint64_t)(((((w[k] >> 1) & 0x01010101u) * 0x00204081u) >> 21) & 0xfu) << sh;
            ms |= (uint64_t)(((((w[k] >> 2) & 0x01010101u) * 0x00204081u) >> 21) & 0xfu) << sh;
            ml |= (uint64_t)(((((w[k] >> 3) & 0x01010101u) * 0x00204081u) >> 21) & 0xfu) << sh;
            mr |= (uint64_t)(((((w[k] >> 4) & 0x01010101u) * 0x00204081u) >> 21) & 0xfu) << sh;
            mz |= (uint64_t)(((((w[k] >> 5) & 0x01010101u) * 0x00204081u) >> 21) & 0xfu) << sh;
        }
    }
    const int64_t valid = nb - wbase;
    const uint64_t vm = valid < 64 ? (1ull << valid) - 1 : ~0ull;
    sm = ms & vm;
    em = me & vm;
    lm.l01 = ml & vm;
    lm.row1 = mr & vm;
    lm.none = mz & vm;
    return m & vm;
}

__global__ __launch_bounds__(kFixThreads) void k_scan_batches_fix(
    const uint8_t* __restrict__ err, int64_t L, int64_t nb, int64_t nbp, ddm_params P,
    ddm_state* __restrict__ state, int2* __restrict__ ev, const uint8_t* __restrict__ flags,
    int64_t* __restrict__ nev_out, const uint8_t* __restrict__ pmap, const int32_t* __restrict__ list,
    uint32_t* __restrict__ ctr, int refill, int open_thr, const double2* __restrict__ pend) {
    __shared__ double rcp[kRcpN];
    __shared__ double s_nr[kFixThreads / 64][2][64];       // wave_tile scratch per wave
    for (int k = threadIdx.x; k < kRcpN; k += kFixThreads) rcp[k] = 1.0 / (double)(k > 0 ? k : 1);
    __syncthreads();
    const int64_t pb = P.per_batch;
    const int min_inst = P.min_num_instances;
    const double wl = P.warning_level, cl = P.out_control_level;
    const bool shortcuts = min_inst == 3;
    const int lane = threadIdx.x & 63;
    const uint64_t below = (1ull << lane) - 1;
    const uint32_t n_list = __atomic_load_n(ctr, __ATOMIC_RELAXED);
    uint32_t claimed = 0;                           // wave-uniform: claims exhausted once >= n_list

    enum { IDLE = 0, OPEN = 1, STEP = 2, COOP = 3 };
    bool fin = false;                               // a COOP batch came back: finish it
    int fin_cpos = -1;
    double* const s_n = s_nr[threadIdx.x >> 6][0];
    double* const s_r = s_nr[threadIdx.x >> 6][1];
    Det d;
    d.p = d.s = d.pmin = d.smin = d.psmin = 0.0;
    d.n = 1;
    d.chg = d.warn = 0;
    int64_t sid = 0, j = 0, wbase = 0, nev = 0, bstart = 0;
    uint64_t chg_m = 0, st_m = 0, ev_m = 0, m0 = 0, m1 = 0;
    LeadMasks lm{0, 0, 0};
    int blen = 0, i = 0, wpos = -1, mode = IDLE;
    for (;;) {
        const uint64_t idle_m = __ballot(mode == IDLE);
        const uint64_t open_m = __ballot(mode == OPEN);
        const int nidle = __popcll(idle_m), nopen = __popcll(open_m);
        const bool stepping = nidle + nopen < 64;
        if (claimed < n_list && (nidle >= refill || (!stepping && nopen == 0))) {
            const int lead = __builtin_ctzll(idle_m);
            uint32_t base = 0;
            if (lane == lead) base = atomicAdd(ctr + 1, (uint32_t)nidle);
            base = __shfl(base, lead);
            claimed = base + (uint32_t)nidle;
            if (mode == IDLE) {
                const uint32_t k = base + (uint32_t)__popcll(idle_m & below);
                if (k < n_list) {
                    sid = list[k];
                    load_det(d, state[sid]);
                    j = 0;
                    wbase = 0;
                    chg_m = nb > 0 ? change_window(flags + sid * nbp, 0, nb, st_m, ev_m, lm) : 0;
                    nev = 0;
                    mode = OPEN;
                }
            }
            continue;
        }
        if (nopen > 0 && (nopen >= open_thr || !stepping)) {
            if (mode == OPEN) {
                for (;;) {
                    if (j >= nb) break;
                    if (j >= wbase + 64) {          // next 64-batch window (nb > 64 only)
                        wbase = j & ~(int64_t)63;
                        chg_m = change_window(flags + sid * nbp, wbase, nb, st_m, ev_m, lm);
                    }
                    if (shortcuts && det_trivial(d)) {
                        // a trivial detector (after a batch of zeros): the batch's flag
                        // bits give its result without its bytes (see kFlagNoError)
                        const int o = (int)(j - wbase);
                        if ((lm.none >> o) & 1ull) {
                            d.n += min(pb, L - j * pb);
                            d.warn = 0;
                        } else {
                            if ((lm.l01 >> o) & 1ull) {     // the change is row 0 or 1
                                const int t = (int)((lm.row1 >> o) & 1ull);
                                ev[sid * nb + j] = make_int2(-1, pmap ? (int)pmap[sid * L + j * pb + t] : t);
                            }                               // else: the speculative change stands
                            ++nev;
                            det_reset(d);
                        }
                        ++j;
                        continue;
                    }
                    if (!det_fresh(d)) break;
                    if (shortcuts && ((lm.none >> (j - wbase)) & 1ull)) {
                        // a fresh detector and a batch without an error: two zeros make it
                        // trivial (n = 3), the rest only move n (no bytes needed)
                        const int bl = (int)min(pb, L - j * pb);
                        if (bl >= 2) {
                            d.p = d.s = d.pmin = d.smin = d.psmin = 0.0;
                            d.n = 1 + bl;
                            d.chg = d.warn = 0;
                            ++j;
                            continue;
                        }
                    }
                    const uint64_t rel = chg_m >> (j - wbase);
                    const int run = (int)min((int64_t)(rel == ~0ull ? 64 : __builtin_ctzll(~rel)), wbase + 64 - j);
                    if (run == 0) {
                        if (pend && ((st_m >> (j - wbase)) & 1ull)) {
                            // fresh detector, unchanged batch whose end state the
                            // speculative pass stored: carry it on without a rescan
                            const double2* e = pend + 3 * (sid * nb + j);
                            const double2 a = e[0], b = e[1], c = e[2];
                            const int64_t nw = (int64_t)c.y;
                            d.p = a.x;
                            d.s = a.y;
                            d.pmin = b.x;
                            d.smin = b.y;
                            d.psmin = c.x;
                            d.n = nw >> 1;
                            d.warn = (int)(nw & 1);
                            d.chg = 0;
                            nev += (int64_t)((ev_m >> (j - wbase)) & 1ull);
                            ++j;
                        }
                        break;
                    }
                    nev += run;                     // batches whose speculative change stands
                    j += run;
                    det_reset(d);
                }
                if (j >= nb) {                      // stream done
                    state[sid] = store_det(d);
                    if (nev_out) nev_out[sid] = nev;
                    mode = IDLE;
                } else {
                    bstart = sid * L + j * pb;
                    blen = (int)min(pb, L - j * pb);
                    batch_mask(err, bstart, blen, m0, m1);
                    i = 0;
                    wpos = -1;
                    mode = STEP;
                }
            }
            continue;
        }
        if (!stepping) break;                       // all idle, claims exhausted
        // Exact rows of a carried detector (rare, but a long carried chain is the whole
        // kernel's tail when one lane steps it): the wave runs them for one lane at a time,
        // the p chain once and everything else lane-parallel (wave_det.h)
        uint64_t coop_m = __ballot(mode == COOP);
        while (coop_m) {
            const int ld = __builtin_ctzll(coop_m);
            coop_m &= coop_m - 1;
            Det c;
            c.p = shfl_d(d.p, ld);
            c.s = shfl_d(d.s, ld);
            c.pmin = shfl_d(d.pmin, ld);
            c.smin = shfl_d(d.smin, ld);
            c.psmin = shfl_d(d.psmin, ld);
            c.n = (int64_t)(((uint64_t)(uint32_t)__shfl((int)(d.n >> 32), ld, 64) << 32) |
                            (uint64_t)(uint32_t)__shfl((int)d.n, ld, 64));
            c.chg = 0;
            c.warn = __shfl(d.warn, ld, 64);
            const uint64_t a0 = ((uint64_t)(uint32_t)__shfl((int)(m0 >> 32), ld, 64) << 32) |
                                (uint64_t)(uint32_t)__shfl((int)m0, ld, 64);
            const uint64_t a1 = ((uint64_t)(uint32_t)__shfl((int)(m1 >> 32), ld, 64) << 32) |
                                (uint64_t)(uint32_t)__shfl((int)m1, ld, 64);
            int ci = __shfl(i, ld, 64), cw = __shfl(wpos, ld, 64);
            const int cb = __shfl(blen, ld, 64);
            int cp = -1;
            while (ci < cb) {
                const int cnt = min(64, cb - ci);
                const uint64_t m = ci < 64 ? ((m0_shift(a0, a1, ci))) : (a1 >> (ci - 64));
                const TileOut to = wave_tile(c, m, cnt, min_inst, wl, cl, s_n, s_r);
                const uint64_t upto = to.last >= 63 ? ~0ull : ((1ull << (to.last + 1)) - 1);
                const uint64_t wb = to.warn & upto;
                if (cw < 0 && wb) cw = ci + __builtin_ctzll(wb);
                if (to.kc >= 0) {
                    cp = ci + to.kc;
                    break;
                }
                ci += cnt;
            }
            if (lane == ld) {
                d = c;
                i = cp >= 0 ? cp + 1 : cb;
                wpos = cw;
                fin = true;
                fin_cpos = cp;
                mode = STEP;
            }
        }
        if (mode != STEP) continue;
        int cpos = -1;
        if (fin) {                                  // a batch the wave finished for this lane
            fin = false;
            cpos = fin_cpos;
        } else {
        // one step of the rescan of batch j
        const int xi = mask_bit(m0, m1, i);
        const bool triv = det_trivial(d);
        if (shortcuts && !triv && i + 1 < blen && det_fresh(d) && xi == 0 && mask_bit(m0, m1, i + 1) == 0) {
            d.p = d.s = d.pmin = d.smin = d.psmin = 0.0;
            d.n = 3;
            d.chg = d.warn = 0;
            i += 2;
        } else if (triv && xi == 0) {
            const int t = min(mask_next(m0, m1, i), blen);
            d.n += t - i;
            d.warn = 0;
            i = t;
        } else if (shortcuts && triv && d.n >= 3) {
            cpos = i;
            ++i;
        } else {
            mode = COOP;                            // exact rows: the wave runs them (above)
            continue;
        }
        }
        if (cpos >= 0 || i >= blen) {
            int w = wpos, c = cpos;
            if (pmap) {
                if (w >= 0) w = pmap[bstart + w];
                if (c >= 0) c = pmap[bstart + c];
            }
            ev[sid * nb + j] = make_int2(w, c);
            nev += (w >= 0 || c >= 0);
            if (cpos >= 0) det_reset(d);            // DDM dropped (DDM_Process.py:209)
            ++j;
            mode = OPEN;
        }
    }
}

}  // namespace

namespace {
struct BatchScratch {
    uint32_t* ctr;      // [0] fix-up list length, [1] claim cursor
    uint32_t* need;     // [n_streams]
    int32_t* list;      // [n_streams]
    uint8_t* flags;     // [n_streams * nbp], 64-byte aligned rows
    double2* pend;      // [n_streams * nb][3] end states of unchanged speculative batches
    double4* pst;       // [kPreN] prefix table (k_scan_prefix_table)
    int2* pinfo;        // [kPreN]
    int64_t bytes;
};

BatchScratch batch_scratch(void* base, int64_t n_streams, int64_t nb) {
    const auto up = [](int64_t x) { return (x + 255) & ~(int64_t)255; };
    const int64_t nbp = ddm::ceil_div(nb, 64) * 64;
    const int64_t o_need = 256, o_list = o_need + up(4 * n_streams), o_flags = o_list + up(4 * n_streams);
    const int64_t o_pend = o_flags + up(n_streams * nbp), o_pst = o_pend + up(48 * n_streams * nb);
    const int64_t o_pinfo = o_pst + 32 * (int64_t)kPreN;
    uint8_t* b = static_cast<uint8_t*>(base);
    return {reinterpret_cast<uint32_t*>(b),      reinterpret_cast<uint32_t*>(b + o_need),
            reinterpret_cast<int32_t*>(b + o_list), b + o_flags,
            reinterpret_cast<double2*>(b + o_pend),
            reinterpret_cast<double4*>(b + o_pst), reinterpret_cast<int2*>(b + o_pinfo),
            o_pinfo + 8 * (int64_t)kPreN};
}
}  // namespace

extern "C" int64_t ddm_scan_batches_scratch_bytes(int64_t n_streams, int64_t stream_len, int32_t per_batch) {
    if (n_streams < 0 || stream_len < 0 || per_batch <= 0) return -1;
    return batch_scratch(nullptr, n_streams, ddm::ceil_div(stream_len, per_batch)).bytes;
}

extern "C" int ddm_scan_batches(const uint8_t* err, int64_t n_streams, int64_t stream_len, const ddm_params* prm,
                                ddm_state* state_io, int32_t* ev_out, int64_t* nev_out, void* scratch,
                                const uint8_t* perm_map, ddm_stream_t stream, ddm_event_t ev_begin,
                                ddm_event_t ev_end) {
    if (!err || !prm || !state_io || !ev_out || !scratch || n_streams < 0 || n_streams >= ((int64_t)1 << 31) ||
        stream_len < 0 || prm->per_batch <= 0 || prm->per_batch > kMaxBatch) {
        ddm::set_error("ddm_scan_batches: invalid argument (per_batch must be 1..%d)", kMaxBatch);
        return DDM_E_ARG;
    }
    const int64_t nb = ddm::ceil_div(stream_len, prm->per_batch);
    const int64_t nbp = ddm::ceil_div(nb, 64) * 64;
    const int64_t n_items = n_streams * nb;
    if (n_streams == 0) return 0;
    const BatchScratch sc = batch_scratch(scratch, n_streams, nb);
    hipStream_t s = ddm::as_hip(stream);
    static const int refill = [] {
        const char* e = getenv("DDM_SCAN_FILL");
        return std::max(1, std::min(kSpecQ - 64, e ? atoi(e) : 64));
    }();
    static const int pop_min = [] {
        const char* e = getenv("DDM_SCAN_POP");
        return std::max(1, std::min(64, e ? atoi(e) : 16));
    }();
    static const int64_t waves_max = [] {
        const char* e = getenv("DDM_SCAN_WAVES");
        return e ? atoll(e) : 256 * 4 * 4;
    }();
    static const int64_t fix_blocks_max = [] {
        const char* e = getenv("DDM_FIX_BLOCKS");
        return e ? atoll(e) : 512;
    }();
    static const int fix_refill = [] {
        const char* e = getenv("DDM_FIX_REFILL");
        return e ? atoi(e) : 16;
    }();
    static const bool use_pre = [] {
        const char* e = getenv("DDM_SCAN_PRE");
        return e ? atoi(e) != 0 : true;
    }();
    static const bool use_pend = [] {
        const char* e = getenv("DDM_SCAN_PEND");
        return e ? atoi(e) != 0 : true;
    }();
    static const int fix_open = [] {
        const char* e = getenv("DDM_FIX_OPEN");
        return e ? atoi(e) : 16;
    }();
    if (ev_begin)
        if (int rc = ddm::hip_status(hipEventRecord(reinterpret_cast<hipEvent_t>(ev_begin), s), "event record")) return rc;
    if (int rc = ddm::hip_status(hipMemsetAsync(scratch, 0, (size_t)(256 + ((4 * n_streams + 255) & ~255)), s),
                                 "ddm_scan_batches: memset"))
        return rc;
    if (n_items > 0) {
        // ~8 waves per SIMD of resident work, each owning a contiguous range of items
        const int64_t waves = std::max<int64_t>(1, std::min<int64_t>(waves_max, ddm::ceil_div(n_items, 256)));
        const int64_t per_wave = ddm::ceil_div(n_items, waves);   // < 2^32 (queue entries hold an offset)
        if (per_wave >= ((int64_t)1 << 32)) {
            ddm::set_error("ddm_scan_batches: too many batches");
            return DDM_E_ARG;
        }
        const int64_t blocks = ddm::ceil_div(ddm::ceil_div(n_items, per_wave), kSpecThreads / 64);
        const bool pre = use_pre && prm->per_batch >= kPre;
        if (pre) {
            hipLaunchKernelGGL(k_scan_prefix_table, dim3(kPreN / 256), dim3(256), 0, s, *prm, sc.pst, sc.pinfo);
            if (int rc = ddm::launch_status("ddm_scan_batches/prefix")) return rc;
        }
        hipLaunchKernelGGL(perm_map ? k_scan_batches_spec<true> : k_scan_batches_spec<false>, dim3((unsigned)blocks),
                           dim3(kSpecThreads), 0, s, err, n_items,
                           stream_len, nb, nbp, *prm, reinterpret_cast<int2*>(ev_out), sc.flags, perm_map, per_wave,
                           refill, pop_min, sc.need, pre ? sc.pst : nullptr, pre ? sc.pinfo : nullptr,
                           use_pend ? sc.pend : nullptr);
        if (int rc = ddm::launch_status("ddm_scan_batches")) return rc;
    }
    hipLaunchKernelGGL(k_scan_batches_list, dim3((unsigned)ddm::ceil_div(n_streams, 256 * kListPer)), dim3(256), 0, s,
                       n_streams,
                       nb, state_io, sc.need, nev_out, sc.list, sc.ctr);
    const int64_t fix_blocks = std::max<int64_t>(1, std::min<int64_t>(fix_blocks_max, ddm::ceil_div(n_streams, kFixThreads)));
    hipLaunchKernelGGL(k_scan_batches_fix, dim3((unsigned)fix_blocks), dim3(kFixThreads), 0, s, err, stream_len, nb,
                       nbp, *prm, state_io, reinterpret_cast<int2*>(ev_out), sc.flags, nev_out, perm_map, sc.list,
                       sc.ctr, fix_refill, fix_open, use_pend ? sc.pend : nullptr);
    if (ev_end)
        if (int rc = ddm::hip_status(hipEventRecord(reinterpret_cast<hipEvent_t>(ev_end), s), "event record")) return rc;
    return ddm::launch_status("ddm_scan_batches");
}

extern "C" int ddm_scan_streams(const uint8_t* err, const int64_t* stream_off, int64_t n_streams,
                                const ddm_params* prm, ddm_state* state_io, const uint64_t* first_nz,
                                const int64_t* batch_base, int64_t n_batches_total, int32_t* ev_out,
                                int32_t* stop_out, int64_t* nev_out, int32_t mode, double* ps_out,
                                const uint8_t* perm_map, const int64_t* stream_end, ddm_stream_t stream,
                                ddm_event_t ev_begin, ddm_event_t ev_end) {
    if (!err || !stream_off || !prm || !state_io || !batch_base || !ev_out || n_streams < 0 ||
        n_batches_total < 0 || prm->per_batch <= 0 || (mode != 0 && mode != 1)) {
        ddm::set_error("ddm_scan_streams: invalid argument");
        return DDM_E_ARG;
    }
    if (n_streams == 0) return 0;
    hipStream_t s = ddm::as_hip(stream);
    if (int rc = ddm::hip_status(hipMemsetAsync(ev_out, 0xff, (size_t)n_batches_total * 2 * sizeof(int32_t), s),
                                 "ddm_scan_streams: memset"))
        return rc;
    const int threads = n_streams >= 256 ? 256 : 64;
    const int64_t blocks = ddm::ceil_div(n_streams, threads);
    if (ev_begin)
        if (int rc = ddm::hip_status(hipEventRecord(reinterpret_cast<hipEvent_t>(ev_begin), s), "event record")) return rc;
    if (ps_out) {                       // p/s trace: the reference-shaped exact kernel
        hipLaunchKernelGGL(k_scan_streams, dim3((unsigned)blocks), dim3(threads), 0, s, err, stream_off, n_streams,
                           *prm, state_io, first_nz, batch_base, ev_out, stop_out, nev_out, (int)mode, ps_out,
                           perm_map, stream_end);
    } else {
        // persistent lanes: one resident round of workgroups (the 32 KB reciprocal table
        // allows 5 per CU), each lane working through ~n_streams / (1280 * 256) streams
        const int64_t fast_blocks = std::max<int64_t>(1, std::min<int64_t>(ddm::ceil_div(n_streams, kFastThreads),
                                                                           256 * 5 * 4));
        hipLaunchKernelGGL(k_scan_fast, dim3((unsigned)fast_blocks), dim3(kFastThreads), 0, s, err, stream_off,
                           n_streams, *prm, state_io, first_nz, batch_base, ev_out, stop_out, nev_out, (int)mode,
                           perm_map, stream_end);
    }
    if (ev_end)
        if (int rc = ddm::hip_status(hipEventRecord(reinterpret_cast<hipEvent_t>(ev_end), s), "event record")) return rc;
    return ddm::launch_status("ddm_scan_streams");
}
