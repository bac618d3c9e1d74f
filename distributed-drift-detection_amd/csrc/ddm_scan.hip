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
#include "scan_fast.h"

namespace {

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
__global__ __launch_bounds__(kFastThreads) void k_scan_fast(
    const uint8_t* __restrict__ err, const int64_t* __restrict__ off, int64_t n_streams, ddm_params P,
    ddm_state* __restrict__ state, const uint64_t* __restrict__ first_nz, const int64_t* __restrict__ batch_base,
    EvSink sink, int32_t* __restrict__ stop_out, int64_t* __restrict__ nev_out, int mode,
    const uint8_t* __restrict__ pmap, const int64_t* __restrict__ stream_end) {
    __shared__ double rcp[kRcpN];
    for (int k = threadIdx.x; k < kRcpN; k += kFastThreads) rcp[k] = 1.0 / (double)(k > 0 ? k : 1);
    __syncthreads();
    scan_fast_worker(err, off, n_streams, P, state, first_nz, batch_base, sink, stop_out, nev_out, mode, pmap,
                     stream_end, (int64_t)blockIdx.x * kFastThreads + threadIdx.x, (int64_t)gridDim.x * kFastThreads,
                     rcp);
}

}  // namespace

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
                           n_streams, *prm, state_io, first_nz, batch_base, EvSink{ev_out, nullptr, nullptr, 0, nullptr},
                           stop_out, nev_out, (int)mode, perm_map, stream_end);
    }
    if (ev_end)
        if (int rc = ddm::hip_status(hipEventRecord(reinterpret_cast<hipEvent_t>(ev_end), s), "event record")) return rc;
    return ddm::launch_status("ddm_scan_streams");
}

extern "C" int ddm_scan_streams_log(const uint8_t* err, const int64_t* stream_off, int64_t n_streams,
                                    const ddm_params* prm, ddm_state* state_io, const uint64_t* first_nz,
                                    int32_t* const* logs, int64_t* log_n, int64_t log_n_stride, const int64_t* log_b0,
                                    int32_t* stop_out, int32_t mode, const uint8_t* perm_map,
                                    const int64_t* stream_end, ddm_stream_t stream) {
    if (!err || !stream_off || !prm || !state_io || !logs || !log_n || !log_b0 || log_n_stride <= 0 || n_streams < 0 ||
        prm->per_batch <= 0 || (mode != 0 && mode != 1)) {
        ddm::set_error("ddm_scan_streams_log: invalid argument");
        return DDM_E_ARG;
    }
    if (n_streams == 0) return 0;
    const int64_t fast_blocks =
        std::max<int64_t>(1, std::min<int64_t>(ddm::ceil_div(n_streams, kFastThreads), 256 * 5 * 4));
    hipLaunchKernelGGL(k_scan_fast, dim3((unsigned)fast_blocks), dim3(kFastThreads), 0, ddm::as_hip(stream), err,
                       stream_off, n_streams, *prm, state_io, first_nz, nullptr,
                       EvSink{nullptr, logs, log_n, log_n_stride, log_b0}, stop_out, nullptr, (int)mode, perm_map,
                       stream_end);
    return ddm::launch_status("ddm_scan_streams_log");
}
