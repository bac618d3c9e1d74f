// Device-resident epoch controller: the per-epoch decisions of the BatchRunner
// (ddm_amd/controller.py: _epoch / _refit_prep / _epoch_after) for the partition loop of
// run_DDM_loop (DDM_Process.py:189-210), taken on the device so that epochs are enqueued
// ahead and no host round trip separates them.
//
// Per partition (one ddm_ctl_part), at the end of an epoch (k_ctl, after the staging):
//   * the scan stopped at a change in batch d (DDM_Process.py:150-152): the RNG position is
//     the draw after batch d's shuffle, batch d+1's shuffle and the refit's seeds were drawn
//     by the staging, the refit runs next on the device (:207-210, :194-196), the next
//     window starts at d+1 with a fresh DDM (:209, :136-139) and covers 9/8 of the concept
//     just closed;
//   * no change: the DDM state carries (:202), the RNG position is after the window's last
//     shuffle, the window doubles;
// then the next window's tables: the shuffle job (run on the side stream beside the
// refits), the predict segment (whose forest is the refit's when one ran: the predict reads
// its shape from the refit's result words), the scan range and carried state, the staging
// job.  Thread t owns partition t; thread 0 then splits the predict grid over the windows.
// The decisions are the host controller's, line for line: results do not depend on which
// side took them (tests/test_gpu_devctl.py runs both on the same partitions).
#include <algorithm>
#include <cstddef>

#include "common.h"

namespace {

constexpr int kCtlThreads = 256;
constexpr int64_t kChunk = 8192;

__device__ __forceinline__ bool st_fresh(const ddm_state& s) {
    return s.sample_count == 1 && s.miss_prob == 1.0 && s.miss_std == 0.0 && __builtin_isinf(s.miss_prob_sd_min);
}
__device__ __forceinline__ bool st_trivial(const ddm_state& s) {
    return s.miss_prob == 0.0 && s.miss_prob_sd_min == 0.0 && s.miss_prob_min == 0.0 && s.miss_sd_min == 0.0;
}
// controller.carried_exact: every next row of this detector needs the exact recurrence
__device__ __forceinline__ bool st_exact(const ddm_state& s) {
    return !s.in_concept_change && !(st_fresh(s) || st_trivial(s));
}
__device__ __forceinline__ ddm_state st_new() {
    ddm_state s;
    s.miss_prob = 1.0;
    s.miss_std = 0.0;
    s.miss_prob_min = __builtin_inf();
    s.miss_sd_min = __builtin_inf();
    s.miss_prob_sd_min = __builtin_inf();
    s.sample_count = 1;
    s.in_concept_change = 0;
    s.in_warning_zone = 0;
    return s;
}

// GpuShuffle.window_draws (rounded up, as the staging's plan): draws a window may need
__device__ __forceinline__ int64_t window_draws(int64_t W, int64_t dpb_x1024) {
    return (W * dpb_x1024 * 115 + 102399) / 102400 + 4 * kChunk;
}

__device__ __forceinline__ int64_t blen(const ddm_ctl_part& p, int64_t b) { return b == p.nb - 1 ? p.last_len : p.pb; }

// _epoch for one partition: refit bookkeeping (_refit_prep, device branch), the window
// (b_end, Wg) and everything the epoch's kernels read.  Leaves the partition idle (empty
// tables) when it is done, parked, stalled, or its stream words are not tabulated yet.
__device__ void plan(const ddm_ctl& c, ddm_ctl_part& p, int i) {
    const int64_t pb = p.pb;
    p.log_mark = p.n_log;                           // this epoch's scans append after it
    bool active = !(p.done || p.stall || p.park);
    const bool apply = active && p.retrain;
    const int64_t P_eff = apply ? p.P2 : p.P;
    const int64_t g0 = apply ? p.j + 1 : p.j;     // batch j was shuffled by the staging
    int64_t b_end = p.j, Wg = 0;
    bool exact = false;
    if (active) {
        b_end = min(p.nb, p.j + min(p.win, p.max_win));
        if (p.last_len != pb && b_end == p.nb && p.nb - 1 >= g0) {   // a short last batch not shuffled yet
            if (p.j == p.nb - 1) {
                p.park = 1;                                           // the host shuffles and scans it
                active = false;
            } else {
                b_end = p.nb - 1;
            }
        }
    }
    if (active) {
        exact = !apply && st_exact(p.state);
        if (exact) b_end = min(b_end, p.j + max((int64_t)1, p.long_cap_rows / pb));
        Wg = max((int64_t)0, min(b_end, p.n_full) - g0);
        // the window's shuffles and the staging's words must lie in the tabulated stream
        if (P_eff + window_draws(Wg, p.dpb_x1024) + p.n_words > p.avail) {
            const int64_t room = p.avail - P_eff - p.n_words - 4 * kChunk;
            const int64_t Wmax = room > 0 ? room * 102400 / (p.dpb_x1024 * 115) : -1;
            if (Wmax < 0 || (Wmax == 0 && g0 == p.j) || P_eff + p.n_words + 4 * kChunk > p.avail) {
                active = false;                                       // wait for the generator
            } else if (Wmax < Wg) {
                Wg = Wmax;
                b_end = g0 + Wg;
            }
        }
    }
    ddm_shuffle_job& jb = c.jobs[i];
    ddm_predict_segment& sg = c.segs[i];
    ddm_stage_job& st = c.stage[i];
    jb = p.job;
    sg = p.seg;
    st = p.stage;
    if (!active) {
        p.idle = 1;
        p.applied = 0;
        const int64_t at = p.base + p.j * pb;
        jb.W = 0;
        jb.pick_out = nullptr;
        sg.pos_begin = sg.pos_end = at;
        sg.nblocks = 0;
        c.seg_res[i] = nullptr;
        c.off[i] = c.end[i] = at;
        c.loff[i] = c.lend[i] = 0;
        c.state[i] = p.state;
        c.log_b0[i] = p.j;
        st.j = st.b_end = p.j;
        st.g0 = p.j;
        st.log = nullptr;                          // nothing to compact
        st.max_events = 0;
        st.p_after_first = st.p_tail_after = -1;
        return;
    }
    p.idle = 0;
    p.applied = apply ? 1 : 0;
    if (apply) {                                    // _refit_prep (device branch)
        p.P = P_eff;
        p.forest_dev = 1;
        p.retrain = 0;
        p.seg_start = p.j;
        p.state = st_new();                         // ddm = None -> a new DDM (:136-139)
        p.refits += 1;
    }
    p.g0 = g0;
    p.b_end = b_end;
    p.Wg = Wg;
    p.P_after_first = apply ? P_eff : -1;
    p.p0 = p.base + p.j * pb;
    p.p1 = p.base + (b_end - 1) * pb + blen(p, b_end - 1);
    // the window's shuffles (ddm_shuffle_window_batch) and the pick of the RNG position
    jb.avail = p.avail;
    jb.P = p.P;
    jb.W = Wg;
    jb.perm_out = const_cast<uint8_t*>(p.stage.perm) + p.base + g0 * pb;
    jb.pick_offset = g0 - p.j;
    jb.pick_last = b_end - 1 - p.j;
    // predict: positions [p0, p1); the forest of the last device refit or the host's
    sg.pos_begin = p.p0;
    sg.pos_end = p.p1;
    if (p.forest_dev) {
        sg.nodes = p.dnodes;
        sg.roots = p.droots;
        sg.leaf_value = p.dleaf;
        sg.classes = p.dclasses;
        sg.n_trees = p.dtrees;
        sg.cforest = p.dblob;
        c.seg_res[i] = p.res;
    } else {
        c.seg_res[i] = nullptr;
    }
    c.first[i] = ~0ull;                             // ddm_predict_segment flags: preset
    // scan: the carried state (fresh after a refit); exact carried windows go to ddm_scan_long
    c.state[i] = p.state;
    c.off[i] = p.p0;
    const bool longscan = exact && p.p1 - p.p0 >= p.long_min_rows;
    c.end[i] = longscan ? p.p0 : p.p1;
    c.loff[i] = longscan ? p.p0 : 0;
    c.lend[i] = longscan ? p.p1 : 0;
    // events: the one-lane scan appends them to the log itself; a long scan writes dense
    // rows, which the staging compacts into the log
    c.log_b0[i] = p.j;
    if (!longscan) {
        st.log = nullptr;
        st.max_events = 0;
    }
    // staging
    st.j = p.j;
    st.g0 = g0;
    st.b_end = b_end;
    st.p_after_first = p.P_after_first;
    st.p_tail_after = -1;
    st.tail = 0;
    st.p_now = p.P;
    st.win = p.win;
    st.seg_start = p.seg_start;
    st.next_avail = p.avail;
    st.plan_out = nullptr;
    st.next_job = nullptr;
}

// _epoch_after for one partition (after the scan, the pick and the staging of the epoch).
__device__ void commit(const ddm_ctl& c, ddm_ctl_part& p, int i) {
    if (p.idle || p.done || p.park) return;
    if (c.pstall[i]) {                              // the predict found the refit unusable
        // the predict wrote no errors for this window, so the scans read stale bytes: their
        // events are void (the host redoes the epoch)
        p.n_log = p.log_mark;
        p.stall = DDM_CTL_STALL_REFIT;
        if (p.applied) {                            // the host redoes the refit (_finish_pending)
            p.retrain = 1;
            p.applied = 0;
            p.refits -= 1;
        }
        return;
    }
    const int32_t stop = c.stop[i];
    p.epochs += 1;
    if (c.lend[i] > c.loff[i]) p.long_scans += 1;   // this epoch's window ran on ddm_scan_long
    const int64_t rows = p.p1 - p.p0;
    p.predicted_rows += rows;
    int64_t slots = p.host_slots;
    if (p.forest_dev && p.res) slots = p.res[DDM_DFIT_CF_SLOTS];
    p.predict_bytes += rows * (4 * slots + 6);
    if (stop == DDM_STOP_FAILED) {
        p.stall = DDM_CTL_STALL_SCAN;
        return;
    }
    if (stop >= 0) {
        const int64_t d = p.j + stop;
        const int64_t* info = p.stage.info_out;
        const int64_t P_at = info[0];               // the staging's: after batch d's shuffle
        p.P = P_at;
        const int64_t seg = d - p.seg_start + 1;
        p.win = max(p.min_win, seg + seg / 8);      // the next concept: 9/8 of this one
        p.j = d + 1;
        if (p.j >= p.nb) {
            p.done = 1;
        } else if (info[6] != 1) {
            p.stall = DDM_CTL_STALL_WORDS;          // the host draws batch j's shuffle and the seeds
            p.retrain = 1;
        } else {
            p.retrain = 1;                          // the device refit runs this epoch
            p.P1 = info[4];
            p.P2 = info[5];
        }
        return;
    }
    if (p.Wg > 0) p.P = c.pick[i] + 1;
    else if (p.P_after_first >= 0) p.P = p.P_after_first;
    p.state = c.state[i];
    p.j = p.b_end;
    p.win *= 2;
    if (p.j >= p.nb) p.done = 1;
}

// A wave per partition record: the 1 KB record comes into LDS by one coalesced load of the
// wave, lane 0 takes the decisions on the LDS copy, and the wave writes it back (holding
// the record in one thread's registers cost 208 VGPRs and 616 B of scratch: 31 us per call).
constexpr int kCtlWaves = kCtlThreads / 64;
constexpr int kPartVec = (int)(sizeof(ddm_ctl_part) / 16);
static_assert(sizeof(ddm_ctl_part) % 16 == 0, "ddm_ctl_part: 16-byte multiple");

__global__ __launch_bounds__(kCtlThreads) void k_ctl(const ddm_ctl c) {
    __shared__ ddm_ctl_part s_part[kCtlWaves];
    __shared__ int s_count[4];
    const int t = threadIdx.x;
    const int lane = t & 63, w = t >> 6;
    if (t < 4) s_count[t] = 0;
    __syncthreads();
    for (int i = w; i < c.n; i += kCtlWaves) {
        const uint4* src = reinterpret_cast<const uint4*>(c.parts + i);
        uint4* lds = reinterpret_cast<uint4*>(&s_part[w]);
        for (int k = lane; k < kPartVec; k += 64) lds[k] = src[k];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (lane == 0) {
            ddm_ctl_part& p = s_part[w];
            if (!c.entry) commit(c, p, i);
            plan(c, p, i);
            atomicAdd(&s_count[p.done ? 3 : p.stall ? 1 : p.park ? 2 : 0], 1);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        uint4* dst = reinterpret_cast<uint4*>(c.parts + i);
        for (int k = lane; k < kPartVec; k += 64) dst[k] = lds[k];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
    __threadfence();
    __syncthreads();
    // the predict grid, split over the windows in proportion to their rows (at least one
    // block per non-empty window)
    if (t == 0) {
        int64_t total = 0, nz = 0;
        for (int i = 0; i < c.n; ++i) {
            const int64_t r = c.segs[i].pos_end - c.segs[i].pos_begin;
            total += r;
            nz += r > 0;
        }
        int64_t b0 = 0;
        const int64_t spare = max((int64_t)0, c.predict_blocks - nz);
        for (int i = 0; i < c.n; ++i) {
            const int64_t r = c.segs[i].pos_end - c.segs[i].pos_begin;
            int64_t nbk = r > 0 ? 1 + (total > 0 ? spare * r / total : 0) : 0;
            nbk = min(nbk, max((int64_t)r > 0 ? 1 : 0, (r + 499) / 500));   // no more blocks than 500-row tiles
            c.segs[i].block0 = b0;
            c.segs[i].nblocks = nbk;
            b0 += nbk;
        }
        if (c.status) {
            for (int k = 0; k < 4; ++k) c.status[k] = s_count[k];
        }
    }
}

int launch_ctl(const ddm_ctl& c, int entry, hipStream_t s) {
    ddm_ctl cc = c;
    cc.entry = entry;
    hipLaunchKernelGGL(k_ctl, dim3(1), dim3(kCtlThreads), 0, s, cc);
    return ddm::launch_status("ddm_ctl");
}

// The window shuffles' grids: the replay and perms kernels stride over pieces and batches,
// so a device-planned window of any size is covered by a fixed grid; sizing it by the
// largest window the runner allows (65,536 batches) launched ~13k mostly idle blocks per
// epoch (C5: 64 us of every epoch).
constexpr int64_t kShufW = 64 * 256, kShufPieces = 256;

}  // namespace

extern "C" int ddm_scan_long_reuse(const uint8_t* err, const int64_t* stream_off, const int64_t* stream_end,
                                   int64_t n_streams, int64_t max_rows, const ddm_params* prm, ddm_state* state_io,
                                   const int64_t* batch_base, int32_t* ev_out, int32_t* stop_out, int64_t* nev_out,
                                   int32_t mode, const uint8_t* perm_map, void* scratch, ddm_stream_t stream);

namespace {

int rec(ddm_event_t e, hipStream_t s) {
    return e ? ddm::hip_status(hipEventRecord(reinterpret_cast<hipEvent_t>(e), s), "event record") : 0;
}

}  // namespace

static_assert(sizeof(ddm_ctl_part) % sizeof(int64_t) == 0, "ddm_ctl_part: int64 stride");

extern "C" int64_t ddm_ctl_part_bytes(void) { return (int64_t)sizeof(ddm_ctl_part); }
extern "C" int64_t ddm_ctl_epoch_bytes(void) { return (int64_t)sizeof(ddm_ctl_epoch); }

extern "C" int ddm_ctl_enter(const ddm_ctl_epoch* e) {
    if (!e || !e->ctl.parts || e->ctl.n <= 0 || e->ctl.n > 4096) {
        ddm::set_error("ddm_ctl_enter: invalid argument");
        return DDM_E_ARG;
    }
    hipStream_t s = ddm::as_hip(e->stream);
    if (e->long_max_rows > 0) {                     // zeroed once; every epoch's call leaves it zeroed
        const int64_t lb = ddm_scan_long_scratch_bytes(e->ctl.n, e->long_max_rows, e->per_batch);
        if (lb > 0)
            if (int rc = ddm::hip_status(hipMemsetAsync(e->long_scratch, 0, (size_t)lb, s), "ddm_ctl_enter: memset"))
                return rc;
    }
    if (int rc = launch_ctl(e->ctl, 1, s)) return rc;
    return ddm_shuffle_window_batch(e->ctl.jobs, e->ctl.n, std::min(e->max_W, kShufW),
                                    std::min(e->max_pieces, kShufPieces), e->per_batch, e->stream,
                                    nullptr, nullptr);
}

extern "C" int ddm_ctl_epochs(const ddm_ctl_epoch* e, int32_t n_epochs) {
    if (!e || !e->ctl.parts || e->ctl.n <= 0 || n_epochs < 0 || !e->side_stream || !e->fork_ev || !e->join_ev) {
        ddm::set_error("ddm_ctl_epochs: invalid argument");
        return DDM_E_ARG;
    }
    hipStream_t s = ddm::as_hip(e->stream);
    hipStream_t side = ddm::as_hip(e->side_stream);
    const ddm_ctl& c = e->ctl;
    for (int32_t k = 0; k < n_epochs; ++k) {
        if (int rc = rec(e->ev[0], s)) return rc;
        if (int rc = ddm_forest_predict_dev(c.segs, c.seg_res, c.n, e->per_batch, c.predict_blocks, c.pstall,
                                            e->stream, nullptr, nullptr))
            return rc;
        if (int rc = rec(e->ev[1], s)) return rc;
        if (int rc = rec(e->ev[2], s)) return rc;
        if (int rc = ddm_scan_streams_log(e->err, c.off, c.n, e->params, c.state, c.first, c.logs,
                                          reinterpret_cast<int64_t*>(reinterpret_cast<uint8_t*>(c.parts) +
                                                                     offsetof(ddm_ctl_part, n_log)),
                                          (int64_t)(sizeof(ddm_ctl_part) / sizeof(int64_t)), c.log_b0,
                                          const_cast<int32_t*>(c.stop), 0, e->perm_map, c.end, e->stream))
            return rc;
        if (e->long_max_rows > 0)
            if (int rc = ddm_scan_long_reuse(e->err, c.loff, c.lend, c.n, e->long_max_rows, e->params, c.state,
                                             e->batch_base, e->ev_out, const_cast<int32_t*>(c.stop), e->nev, 0,
                                             e->perm_map, e->long_scratch, e->stream))
                return rc;
        if (int rc = ddm_shuffle_pick_batch(c.jobs, c.n, e->stream)) return rc;
        if (int rc = rec(e->ev[3], s)) return rc;
        if (int rc = rec(e->ev[4], s)) return rc;
        if (int rc = ddm_epoch_stage(c.stage, c.n, e->stream)) return rc;
        if (int rc = launch_ctl(c, 0, s)) return rc;
        if (int rc = rec(e->ev[5], s)) return rc;
        // the next windows' shuffles beside the refits
        if (int rc = ddm::hip_status(hipEventRecord(reinterpret_cast<hipEvent_t>(e->fork_ev), s), "fork")) return rc;
        if (int rc = ddm::hip_status(hipStreamWaitEvent(side, reinterpret_cast<hipEvent_t>(e->fork_ev), 0), "fork"))
            return rc;
        if (int rc = rec(e->ev[10], side)) return rc;
        if (int rc = ddm_shuffle_window_batch(c.jobs, c.n, std::min(e->max_W, kShufW),
                                              std::min(e->max_pieces, kShufPieces), e->per_batch, e->side_stream,
                                              nullptr, nullptr))
            return rc;
        if (int rc = rec(e->ev[11], side)) return rc;
        if (int rc = ddm::hip_status(hipEventRecord(reinterpret_cast<hipEvent_t>(e->join_ev), side), "join"))
            return rc;
        if (e->n_dfit > 0) {
            if (int rc = rec(e->ev[6], s)) return rc;
            if (int rc = ddm_rf_fit_device_lf(e->dfit_jobs, e->n_dfit, e->max_trees, e->dfit_max_lf, e->stream)) return rc;
            if (int rc = rec(e->ev[7], s)) return rc;
        }
        if (int rc = ddm::hip_status(hipStreamWaitEvent(s, reinterpret_cast<hipEvent_t>(e->join_ev), 0), "join"))
            return rc;
    }
    return 0;
}
