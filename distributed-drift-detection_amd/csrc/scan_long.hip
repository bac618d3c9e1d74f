// Long carried DDM segments: run_DDM (DDM_Process.py:135-159) over streams whose
// detector carries across very many rows (DDM_Process.py:144-152, :202) — a window in
// which no change occurs for millions of rows while the detector is not in its trivial
// state (e.g. errors thinning out after a noisy start).  There the only exact form is
// the sequential recurrence p += (x - p) / n, and k_scan_fast runs it on ONE lane per
// stream: ~40 fp64 instructions per row at single-lane issue.
//
// Here one wave owns a chunk of 64 * per_batch rows (64 whole batches) and splits the
// row's work by dependency:
//   * the p chain (5 dependent fp64 operations per row: sub, Markstein division, add) is
//     the only sequential part; the wave runs it for a 64-row tile, lane k keeping p_k;
//   * everything else is lane-parallel over the tile: 1/n, s_k = sqrt(p_k(1-p_k)/n_k),
//     the running arg-min of p + s (a wave scan; ties go to the later row, the `<=` of
//     the reference), the change / warning tests against it, and ballots for the first
//     change and the first warning of each batch.
// Chunks are chained by a look-back on the carried detector: each chunk stages its bytes
// and 64-bit row masks in LDS as soon as it is dispatched, then waits for its
// predecessor's inclusive state (p, s, p_min, s_min, ps_min, n, flags, event count),
// scans, and publishes its own.  The carry is not associative (p is a rounded running
// mean), so the look-back is one step deep; what it buys is that loading and masking of
// every later chunk is done before the carry reaches it.  Chunks are taken in dispatch
// order from an atomic ticket, so a chunk only ever waits for one that is already
// running.
//
// Decisions and carried states are those of k_scan_streams bit for bit: the same
// recurrence (det.h: Markstein division by n with RN(1/n), sqrt_q), the same gate, the
// same `<=` arg-min and the same `elif` between change and warning.
#include "common.h"
#include "det.h"
#include "wave_det.h"

namespace {

constexpr int kLongMaxBatch = 256;
constexpr int kLongChunkMax = 64 * kLongMaxBatch;   // rows (= bytes) staged per chunk
constexpr int32_t kLongFailed = DDM_STOP_FAILED;    // stop of a stream whose look-back gave up
uint32_t g_spin_limit = 1u << 24;                  // look-back spins before giving up (~1 s)

struct Carry {                 // a chunk's inclusive state (look-back record)
    double p, s, pmin, smin, psmin;
    int64_t n;
    int32_t chg, warn;
    int64_t nev;               // batches with an event so far
    int64_t stop;              // batch of the (mode 0) change or -1
};

// Every block ends here: the last one to finish re-zeroes the dispatch ticket and the
// look-back flags, so the scratch is ready for the next call without a memset (the
// device-resident runner launches ddm_scan_long every epoch, mostly on empty windows).
__device__ __forceinline__ void long_block_done(uint32_t* ticket, int32_t* flag, int64_t n_flags, uint32_t grid) {
    __shared__ int s_last;
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        s_last = atomicAdd(ticket + 2, 1u) == grid - 1;
    }
    __syncthreads();
    if (s_last) {
        __threadfence();
        for (int64_t q = threadIdx.x; q < n_flags; q += blockDim.x) flag[q] = 0;
        if (threadIdx.x == 0) {
            ticket[0] = 0;
            ticket[2] = 0;
        }
    }
}

__global__ __launch_bounds__(64) void k_scan_long(
    const uint8_t* __restrict__ err, const int64_t* __restrict__ off, const int64_t* __restrict__ stream_end,
    int64_t n_streams, int64_t n_chunks, ddm_params P, ddm_state* __restrict__ state,
    const int64_t* __restrict__ batch_base, int32_t* __restrict__ ev, int32_t* __restrict__ stop_out,
    int64_t* __restrict__ nev_out, int mode, const uint8_t* __restrict__ pmap, uint32_t* __restrict__ ticket,
    int32_t* __restrict__ flag, Carry* __restrict__ carry, uint32_t spin_limit, const int32_t* __restrict__ only,
    const int32_t* __restrict__ any) {
    if (any && *any == 0) return;                              // (the certified scan's: nothing to rescan)
    __shared__ uint4 sbytes[kLongChunkMax / 16 + 1];
    __shared__ uint64_t smask[kLongChunkMax / 64];
    __shared__ int2 sev[64];
    __shared__ double s_tile[kTileScratch];
    __shared__ uint32_t stk;
    const int lane = threadIdx.x;
    if (lane == 0) stk = atomicAdd(ticket, 1u);
    __syncthreads();
    const int64_t t = stk;
    const int64_t c = t / n_streams, sid = t % n_streams;     // chunk-major: chunk c-1 holds an earlier ticket
    const uint32_t grid = gridDim.x;
    if (c >= n_chunks || (only && !only[sid])) {      // (only: the streams to scan, others untouched)
        long_block_done(ticket, flag, n_streams * n_chunks, grid);
        return;
    }
    const int64_t lo = off[sid], hi = stream_end ? stream_end[sid] : off[sid + 1];
    const int pb = P.per_batch;
    const int64_t C = 64 * (int64_t)pb;
    const int64_t c0 = lo + c * C;
    if (c0 >= hi) {                                            // no such chunk (empty streams: untouched)
        long_block_done(ticket, flag, n_streams * n_chunks, grid);
        return;
    }
    const int64_t c1 = min(c0 + C, hi);
    const int64_t last_chunk = (hi - lo - 1) / C;
    const int min_inst = P.min_num_instances;
    const double wl = P.warning_level, cl = P.out_control_level;
    int32_t* cflag = flag + sid * n_chunks;
    Carry* ccar = carry + sid * n_chunks;

    // ---- stage the chunk (independent of the carry): bytes, then one 64-bit mask per tile
    const int64_t a0 = c0 & ~(int64_t)15;
    const int shift = (int)(c0 - a0);
    const int nvec = (int)((c1 - a0 + 15) >> 4);
    for (int k = lane; k < nvec; k += 64) sbytes[k] = *reinterpret_cast<const uint4*>(err + a0 + 16 * (int64_t)k);
    if (lane < 64) sev[lane] = make_int2(-1, -1);
    __syncthreads();
    const int rows = (int)(c1 - c0);
    const int ntiles = (rows + 63) >> 6;
    const uint8_t* sb = reinterpret_cast<const uint8_t*>(sbytes) + shift;
    for (int tt = 0; tt < ntiles; ++tt) {
        const int r = tt * 64 + lane;
        const uint64_t m = __ballot(r < rows && sb[r] != 0);
        if (lane == 0) smask[tt] = m;
    }
    __syncthreads();

    // ---- the carry: the stream's state (chunk 0) or the predecessor's published state
    Carry in;
    if (c == 0) {
        const ddm_state st = state[sid];
        in.p = st.miss_prob;
        in.s = st.miss_std;
        in.pmin = st.miss_prob_min;
        in.smin = st.miss_sd_min;
        in.psmin = st.miss_prob_sd_min;
        in.n = st.sample_count;
        in.chg = st.in_concept_change;
        in.warn = st.in_warning_zone;
        in.nev = 0;
        in.stop = -1;
    } else {
        __shared__ Carry sin;
        if (lane == 0) {
            // bounded: the predecessor holds an earlier ticket, so it is running; a spin
            // past ~1 s marks the call failed (ticket[1]) instead of hanging the device, and
            // this chunk publishes a failed carry (stop = kLongFailed) rather than scanning
            // from a state that was never published
            uint32_t spins = 0;
            bool gave_up = false;
            while (__hip_atomic_load(cflag + c - 1, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == 0) {
                if (++spins > spin_limit) {
                    atomicOr(ticket + 1, 1u);
                    gave_up = true;
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
            sin = ccar[c - 1];
            if (gave_up) sin.stop = kLongFailed;
        }
        __syncthreads();
        in = sin;
    }
    const int64_t b0 = (c0 - lo) / pb;                         // first batch of the chunk
    const int nbc = (int)((rows + pb - 1) / pb);              // batches of the chunk
    Det d;
    d.p = in.p;
    d.s = in.s;
    d.pmin = in.pmin;
    d.smin = in.smin;
    d.psmin = in.psmin;
    d.n = in.n;
    d.chg = in.chg;
    d.warn = in.warn;
    int64_t stop = in.stop;
    const bool failed = stop == kLongFailed;                   // a predecessor's carry never came
    bool stopped = failed || (stop >= 0 && mode == 0);

    int pos = 0;                                               // next row of the chunk
    while (!stopped && pos < rows) {
        if (d.chg) det_reset(d);                               // DDM dropped / lazy reset
        const int cnt = min(64, rows - pos);
        const int tile = pos >> 6, sh = pos & 63;
        uint64_t m = smask[tile] >> sh;
        if (sh && tile + 1 < ntiles) m |= smask[tile + 1] << (64 - sh);
        if (cnt < 64) m &= (1ull << cnt) - 1;
        const TileOut to = wave_tile(d, m, cnt, min_inst, wl, cl, s_tile);
        const int kc = to.kc, last = to.last;
        const uint64_t W_ = to.warn;
        if (kc < 0 && W_ == 0) {                               // no event in the tile
            pos += cnt;
            continue;
        }
        // first warning of each batch the committed rows touch
        uint64_t wcommit = kc >= 0 ? (W_ & ((kc ? (~0ull >> (64 - kc)) : 0ull))) : W_;
        if (lane == 0) {
            int k = 0;
            while (k <= last) {
                const int64_t rr = c0 - lo + pos + k;                       // stream row
                const int bi = (int)(rr / pb - b0);
                const int kend = min(last + 1, k + (int)(pb - rr % pb));
                const uint64_t span = (kend - k >= 64 ? ~0ull : ((1ull << (kend - k)) - 1)) << k;
                const uint64_t wb = wcommit & span;
                if (wb && sev[bi].x < 0) sev[bi].x = (int)((rr + __builtin_ctzll(wb) - k) % pb);
                k = kend;
            }
            if (kc >= 0) {
                const int64_t rr = c0 - lo + pos + kc;
                sev[(int)(rr / pb - b0)].y = (int)(rr % pb);
            }
        }
        __syncthreads();
        if (kc >= 0) {
            const int64_t rr = c0 - lo + pos + kc;
            if (mode == 0) {
                stop = rr / pb;
                stopped = true;
                break;
            }
            // mode 1: rows after the change in its batch are never fed (DDM_Process.py:150-152);
            // a fresh DDM takes the next batch (:209, :136-139)
            pos = (int)((rr / pb + 1) * pb - (c0 - lo));
            det_reset(d);
            continue;
        }
        pos += cnt;
    }
    __syncthreads();
    // ---- publish the inclusive state, write this chunk's batch rows
    int nev_c = 0;
    for (int bi = 0; bi < nbc; ++bi) {
        const int2 e = sev[bi];
        nev_c += (e.x >= 0 || e.y >= 0) ? 1 : 0;
    }
    Carry outc;
    outc.p = d.p;
    outc.s = d.s;
    outc.pmin = d.pmin;
    outc.smin = d.smin;
    outc.psmin = d.psmin;
    outc.n = d.n;
    outc.chg = d.chg;
    outc.warn = d.warn;
    outc.nev = in.nev + nev_c;
    outc.stop = stop;
    const bool passthrough = mode == 0 && in.stop >= 0;     // a change before this chunk
    if (lane == 0) {
        ccar[c] = passthrough ? in : outc;
        __hip_atomic_store(cflag + c, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
    int32_t* evs = ev + 2 * (batch_base[sid] + b0);
    for (int bi = lane; bi < nbc; bi += 64) {
        int2 e = passthrough || failed ? make_int2(-1, -1) : sev[bi];
        if (pmap) {
            const int64_t bs = c0 + (int64_t)bi * pb;
            if (e.x >= 0) e.x = pmap[bs + e.x];
            if (e.y >= 0) e.y = pmap[bs + e.y];
        }
        evs[2 * bi] = e.x;
        evs[2 * bi + 1] = e.y;
    }
    // the stream's results: from its last chunk, or (mode 0) from the chunk of the change
    if (lane == 0 && !passthrough && (c == last_chunk || stopped)) {
        ddm_state st;
        st.miss_prob = outc.p;
        st.miss_std = outc.s;
        st.miss_prob_min = outc.pmin;
        st.miss_sd_min = outc.smin;
        st.miss_prob_sd_min = outc.psmin;
        st.sample_count = outc.n;
        st.in_concept_change = outc.chg;
        st.in_warning_zone = outc.warn;
        if (!failed) state[sid] = st;
        if (stop_out) stop_out[sid] = failed ? kLongFailed : (int32_t)outc.stop;
        if (nev_out) nev_out[sid] = failed ? 0 : outc.nev;
    }
    long_block_done(ticket, flag, n_streams * n_chunks, grid);
}

struct LongScratch {
    uint32_t* ticket;
    int32_t* flag;
    Carry* carry;
    int64_t flag_bytes, bytes;
};

LongScratch long_scratch(void* base, int64_t n_streams, int64_t n_chunks) {
    const auto up = [](int64_t x) { return (x + 255) & ~(int64_t)255; };
    const int64_t o_flag = 256, o_carry = o_flag + up(4 * n_streams * n_chunks);
    uint8_t* b = static_cast<uint8_t*>(base);
    return {reinterpret_cast<uint32_t*>(b), reinterpret_cast<int32_t*>(b + o_flag),
            reinterpret_cast<Carry*>(b + o_carry), o_carry, o_carry + (int64_t)sizeof(Carry) * n_streams * n_chunks};
}

}  // namespace

extern "C" int64_t ddm_scan_long_scratch_bytes(int64_t n_streams, int64_t max_rows, int32_t per_batch) {
    if (n_streams < 0 || max_rows < 0 || per_batch <= 0 || per_batch > kLongMaxBatch) return -1;
    return long_scratch(nullptr, n_streams, std::max<int64_t>(1, ddm::ceil_div(max_rows, 64 * (int64_t)per_batch)))
        .bytes;
}

static int scan_long_launch(const uint8_t* err, const int64_t* stream_off, const int64_t* stream_end,
                            int64_t n_streams, int64_t max_rows, const ddm_params* prm, ddm_state* state_io,
                            const int64_t* batch_base, int32_t* ev_out, int32_t* stop_out, int64_t* nev_out,
                            int32_t mode, const uint8_t* perm_map, void* scratch, ddm_stream_t stream,
                            ddm_event_t ev_begin, ddm_event_t ev_end, bool zero, const int32_t* only = nullptr,
                            const int32_t* any = nullptr) {
    if (!err || !stream_off || !prm || !state_io || !batch_base || !ev_out || !scratch || n_streams < 0 ||
        max_rows < 0 || prm->per_batch <= 0 || prm->per_batch > kLongMaxBatch || (mode != 0 && mode != 1)) {
        ddm::set_error("ddm_scan_long: invalid argument (per_batch must be 1..%d)", kLongMaxBatch);
        return DDM_E_ARG;
    }
    if (n_streams == 0 || max_rows == 0) return 0;
    const int64_t n_chunks = ddm::ceil_div(max_rows, 64 * (int64_t)prm->per_batch);
    const int64_t grid = n_streams * n_chunks;
    if (grid >= ((int64_t)1 << 31)) {
        ddm::set_error("ddm_scan_long: too many chunks");
        return DDM_E_ARG;
    }
    const LongScratch sc = long_scratch(scratch, n_streams, n_chunks);
    hipStream_t s = ddm::as_hip(stream);
    if (ev_begin)
        if (int rc = ddm::hip_status(hipEventRecord(reinterpret_cast<hipEvent_t>(ev_begin), s), "event record")) return rc;
    if (zero)
        if (int rc = ddm::hip_status(hipMemsetAsync(scratch, 0, (size_t)sc.flag_bytes, s), "ddm_scan_long: memset"))
            return rc;
    hipLaunchKernelGGL(k_scan_long, dim3((unsigned)grid), dim3(64), 0, s, err, stream_off, stream_end, n_streams,
                       n_chunks, *prm, state_io, batch_base, ev_out, stop_out, nev_out, (int)mode, perm_map,
                       sc.ticket, sc.flag, sc.carry, g_spin_limit, only, any);
    if (int rc = ddm::launch_status("ddm_scan_long")) return rc;
    if (ev_end)
        if (int rc = ddm::hip_status(hipEventRecord(reinterpret_cast<hipEvent_t>(ev_end), s), "event record")) return rc;
    return 0;
}

extern "C" int ddm_scan_long(const uint8_t* err, const int64_t* stream_off, const int64_t* stream_end,
                             int64_t n_streams, int64_t max_rows, const ddm_params* prm, ddm_state* state_io,
                             const int64_t* batch_base, int32_t* ev_out, int32_t* stop_out, int64_t* nev_out,
                             int32_t mode, const uint8_t* perm_map, void* scratch, ddm_stream_t stream,
                             ddm_event_t ev_begin, ddm_event_t ev_end) {
    return scan_long_launch(err, stream_off, stream_end, n_streams, max_rows, prm, state_io, batch_base, ev_out,
                            stop_out, nev_out, mode, perm_map, scratch, stream, ev_begin, ev_end, true);
}

// The device-resident runner's form (csrc/ctl.hip): the scratch was zeroed once when the
// runner entered device mode and every call leaves it zeroed (long_block_done).
extern "C" int ddm_scan_long_reuse(const uint8_t* err, const int64_t* stream_off, const int64_t* stream_end,
                                   int64_t n_streams, int64_t max_rows, const ddm_params* prm, ddm_state* state_io,
                                   const int64_t* batch_base, int32_t* ev_out, int32_t* stop_out, int64_t* nev_out,
                                   int32_t mode, const uint8_t* perm_map, void* scratch, const int32_t* any,
                                   ddm_stream_t stream) {
    return scan_long_launch(err, stream_off, stream_end, n_streams, max_rows, prm, state_io, batch_base, ev_out,
                            stop_out, nev_out, mode, perm_map, scratch, stream, nullptr, nullptr, false, nullptr, any);
}

// The certified scan's exact fallback (csrc/scan_cert.hip): only the streams with only[s] != 0,
// and nothing at all (every block returns at once) while *any == 0.  The caller zeroes the
// scratch's first ddm_scan_long_flag_bytes(...) bytes beforehand (no memset here).
extern "C" int ddm_scan_long_only(const uint8_t* err, const int64_t* stream_off, const int64_t* stream_end,
                                  int64_t n_streams, int64_t max_rows, const ddm_params* prm, ddm_state* state_io,
                                  const int64_t* batch_base, int32_t* ev_out, int32_t* stop_out, int64_t* nev_out,
                                  int32_t mode, const uint8_t* perm_map, void* scratch, const int32_t* only,
                                  const int32_t* any, ddm_stream_t stream) {
    return scan_long_launch(err, stream_off, stream_end, n_streams, max_rows, prm, state_io, batch_base, ev_out,
                            stop_out, nev_out, mode, perm_map, scratch, stream, nullptr, nullptr, false, only, any);
}

extern "C" int64_t ddm_scan_long_flag_bytes(int64_t n_streams, int64_t max_rows, int32_t per_batch) {
    if (n_streams < 0 || max_rows < 0 || per_batch <= 0 || per_batch > kLongMaxBatch) return 0;
    return long_scratch(nullptr, n_streams, std::max<int64_t>(1, ddm::ceil_div(max_rows, 64 * (int64_t)per_batch)))
        .flag_bytes;
}

extern "C" int ddm_scan_long_set_spin_limit(uint32_t spins) {
    g_spin_limit = spins;
    return 0;
}
