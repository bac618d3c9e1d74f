// The production one-lane DDM scan (k_scan_fast's worker), shared by ddm_scan.hip and the
// device-resident epoch's fused staging kernel (stage.hip), which runs it for its own
// partition's window (one kernel launch fewer per epoch).
#pragma once
#include "common.h"
#include "det.h"

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

constexpr int kFastThreads = 256;

__device__ __forceinline__ int byte_at(uint64_t lo, uint64_t hi, int k) {
    return (int)(((k < 8 ? lo >> (8 * k) : hi >> (8 * (k - 8)))) & 0xff);
}

// One lane = a persistent worker over streams sid, sid + nthreads, ...  The body is ONE
// flat loop whose iterations each do one step of one kind (start/finish a stream, two
// leading zeros, a zero run, a trivial-state change, or an exact row): no nested loops,
// so a lane that finishes a stream starts its next one at once instead of idling until
// the slowest lane of its wave is done with the same round.
// Event sink of k_scan_fast: the dense per-batch rows (ev), or, with a log (the device-
// resident runner, csrc/ctl.hip), one record (b0[sid] + b, warning, change) per batch
// with an event appended to the stream's own log (one lane owns a stream: no atomics).
struct EvSink {
    int32_t* ev;
    int32_t* const* logs;
    int64_t* log_n;
    int64_t log_stride;          // int64 words between the streams' counters
    const int64_t* b0;
    __device__ __forceinline__ void put(int64_t sid, int32_t* evs, int64_t b, int w, int c, int64_t& nlog) const {
        if (logs) {
            int32_t* r = logs[sid] + 3 * nlog;
            r[0] = (int32_t)(b0[sid] + b);
            r[1] = w;
            r[2] = c;
            ++nlog;
        } else {
            evs[2 * b] = w;
            evs[2 * b + 1] = c;
        }
    }
};

// The worker: lane sid0 takes streams sid0, sid0 + stride, ...; rcp: RN(1/k) for k < kRcpN
// (LDS).
__device__ __forceinline__ void scan_fast_worker(
    const uint8_t* __restrict__ err, const int64_t* __restrict__ off, int64_t n_streams, const ddm_params P,
    ddm_state* __restrict__ state, const uint64_t* __restrict__ first_nz, const int64_t* __restrict__ batch_base,
    const EvSink sink, int32_t* __restrict__ stop_out, int64_t* __restrict__ nev_out, int mode,
    const uint8_t* __restrict__ pmap, const int64_t* __restrict__ stream_end, int64_t sid0, int64_t nthreads,
    const double* __restrict__ rcp) {
    int32_t* const ev = sink.ev;
    int64_t nlog = 0;
    const int64_t pb = P.per_batch;
    const int min_inst = P.min_num_instances;
    const double wl = P.warning_level, cl = P.out_control_level;
    const bool shortcuts = min_inst == 3;   // the trivial-state shortcuts assume the reference gate

    int64_t sid = sid0 - nthreads;          // advanced on the first step
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
                if (sink.logs) sink.log_n[sid * sink.log_stride] = nlog;
            }
            sid += nthreads;
            if (sid >= n_streams) break;
            if (sink.logs) nlog = sink.log_n[sid * sink.log_stride];
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
            evs = ev ? ev + 2 * batch_base[sid] : nullptr;
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
            sink.put(sid, evs, b, (pmap && wpos >= 0) ? (int)pmap[bstart + wpos] : wpos,
                     pmap ? (int)pmap[bstart + cpos] : cpos, nlog);
            ++nev;
            if (mode == 0) {
                stop = (int32_t)b;
                i = hi;                     // finish this stream
                continue;
            }
            i = bend;                       // fresh detector from the next batch
        } else if (i >= bend && wpos >= 0) {
            if (sink.logs) sink.put(sid, evs, b, pmap ? (int)pmap[bstart + wpos] : wpos, -1, nlog);
            else evs[2 * b] = pmap ? (int)pmap[bstart + wpos] : wpos;
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


}  // namespace
