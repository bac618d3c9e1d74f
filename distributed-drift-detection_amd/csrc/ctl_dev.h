// Device-side decisions of the device-resident epoch controller (the per-epoch decisions of
// the BatchRunner, ddm_amd/controller.py _epoch / _refit_prep / _epoch_after, for the
// partition loop of run_DDM_loop, DDM_Process.py:189-210): shared by k_ctl (csrc/ctl.hip)
// and the fused staging + decision kernel (csrc/stage.hip).
#pragma once
#include <algorithm>
#include <cstddef>

#include "common.h"

namespace {

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

// The window after a change (BatchRunner._epoch_after, DDMSettings.drift_window): the next
// concept likely lasts about as long as the one just closed (seg batches), so the window
// covers seg plus a margin of max(seg >> shift, pad) batches, at least min_win batches unless
// the concept was short (seg <= short: C5's concepts of 1.5-3 batches repeat, c2's short
// ones do not) (rule = shift | pad << 8 | short << 16); windows still double after a miss.
__device__ __forceinline__ int64_t drift_window(int64_t seg, int64_t min_win, int32_t rule) {
    const int64_t w = seg + max(seg >> (rule & 255), (int64_t)((rule >> 8) & 255));
    return seg <= (int64_t)(rule >> 16) ? w : max(min_win, w);
}

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
    // a window for ddm_scan_long when no long scan is enqueued: the host takes the partition
    // and enables the long scans for the rest of the run (their launch is skipped until then)
    if (active && exact && !c.long_ok &&
        p.base + (b_end - 1) * pb + blen(p, b_end - 1) - (p.base + p.j * pb) >= p.long_min_rows) {
        p.stall = DDM_CTL_STALL_LONG;
        active = false;
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

// The words commit reads from other kernels' outputs, fetched by the record's wave at once
// (ctl_record) instead of one dependent load after another by lane 0.
struct CommitPre {
    int64_t pstall, stop, lend, loff, slots, info0, info4, info5, info6, pick;
    ddm_state state;
};
constexpr int kPreWords = (int)(sizeof(CommitPre) / 8);
static_assert(sizeof(CommitPre) % 8 == 0 && kPreWords <= 64, "CommitPre: 64-bit words, one per lane");

// _epoch_after for one partition (after the scan, the pick and the staging of the epoch).
__device__ void commit(const ddm_ctl& c, ddm_ctl_part& p, int i, const CommitPre& q) {
    if (p.idle || p.done || p.park) return;
    if (q.pstall) {                                 // the predict found the refit unusable
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
    const int32_t stop = (int32_t)q.stop;
    p.epochs += 1;
    if (q.lend > q.loff) p.long_scans += 1;   // this epoch's window ran on ddm_scan_long
    const int64_t rows = p.p1 - p.p0;
    p.predicted_rows += rows;
    int64_t slots = p.host_slots;
    if (p.forest_dev && p.res) slots = q.slots;
    // algorithmic bytes of the predict kernel: the referenced feature columns and the label,
    // the error byte written, and (coupled epochs) the in-batch permutation byte read; a
    // decoupled epoch's permutation into DDM order is k_err_permute's (counted by its rows)
    p.predict_bytes += rows * (4 * slots + (c.decoupled ? 5 : 6));
    if (c.decoupled) p.permute_rows += rows;
    if (stop == DDM_STOP_FAILED) {
        p.stall = DDM_CTL_STALL_SCAN;
        return;
    }
    if (stop >= 0) {
        const int64_t d = p.j + stop;
        const int64_t P_at = q.info0;               // the staging's: after batch d's shuffle
        p.P = P_at;
        const int64_t seg = d - p.seg_start + 1;
        p.win = drift_window(seg, p.min_win, p.win_rule);   // the next concept, with a margin
        p.j = d + 1;
        if (p.j >= p.nb) {
            p.done = 1;
        } else if (q.info6 != 1) {
            p.stall = DDM_CTL_STALL_WORDS;          // the host draws batch j's shuffle and the seeds
            p.retrain = 1;
        } else {
            p.retrain = 1;                          // the device refit runs this epoch
            p.P1 = q.info4;
            p.P2 = q.info5;
        }
        return;
    }
    if (p.Wg > 0) p.P = q.pick + 1;
    else if (p.P_after_first >= 0) p.P = p.P_after_first;
    p.state = q.state;
    p.j = p.b_end;
    p.win *= 2;
    if (p.j >= p.nb) p.done = 1;
}

// A wave per partition record: the 1 KB record comes into LDS by one coalesced load of the
// wave, lane 0 takes the decisions on the LDS copy (commit unless entry, then plan), and the
// wave writes it back (holding the record in one thread's registers cost 208 VGPRs and
// 616 B of scratch: 31 us per call).  Returns the record's state for the status counts:
// 3 done, 1 stalled, 2 parked, 0 active (lane 0's value).
constexpr int kPartVec = (int)(sizeof(ddm_ctl_part) / 16);
static_assert(sizeof(ddm_ctl_part) % 16 == 0, "ddm_ctl_part: 16-byte multiple");

__device__ __forceinline__ int ctl_record(const ddm_ctl& c, int i, ddm_ctl_part* lds_part, int lane, int entry) {
    const uint4* src = reinterpret_cast<const uint4*>(c.parts + i);
    uint4* lds = reinterpret_cast<uint4*>(lds_part);
    for (int k = lane; k < kPartVec; k += 64) lds[k] = src[k];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // lane k fetches word k of CommitPre (the reads commit would make one after another)
    int64_t v = 0;
    if (!entry && lane < kPreWords) {
        const ddm_ctl_part& r = *lds_part;
        switch (lane) {
            case 0: v = c.pstall[i]; break;
            case 1: v = c.stop[i]; break;
            case 2: v = c.lend[i]; break;
            case 3: v = c.loff[i]; break;
            case 4: v = (r.forest_dev && r.res) ? r.res[DDM_DFIT_CF_SLOTS] : 0; break;
            case 5: v = r.stage.info_out ? r.stage.info_out[0] : 0; break;
            case 6: v = r.stage.info_out ? r.stage.info_out[4] : 0; break;
            case 7: v = r.stage.info_out ? r.stage.info_out[5] : 0; break;
            case 8: v = r.stage.info_out ? r.stage.info_out[6] : 0; break;
            case 9: v = c.pick ? c.pick[i] : 0; break;
            default: v = reinterpret_cast<const int64_t*>(c.state + i)[lane - 10]; break;
        }
    }
    CommitPre pre;
    int64_t* pw = reinterpret_cast<int64_t*>(&pre);
#pragma unroll
    for (int k = 0; k < kPreWords; ++k) pw[k] = __shfl(v, k, 64);
    int st = 0;
    if (lane == 0) {
        ddm_ctl_part& p = *lds_part;
        if (!entry) commit(c, p, i, pre);
        plan(c, p, i);
        st = p.done ? 3 : p.stall ? 1 : p.park ? 2 : 0;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    uint4* dst = reinterpret_cast<uint4*>(c.parts + i);
    for (int k = lane; k < kPartVec; k += 64) dst[k] = lds[k];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    return st;
}

// After every record: the predict grid split over the windows in proportion to their rows
// (at least one block per non-empty window), the status counts, and whether the next epoch
// has a long window (ddm_scan_long's blocks return at once when none has).  One wave, a
// partition per lane (64 at a time): the records' loads are issued together instead of one
// dependent load after another by one thread (10.8 -> ~2 us at the end of every epoch).
__device__ __forceinline__ int64_t wave_sum_i64(int64_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ void ctl_split(const ddm_ctl& c, int lane) {
    int64_t total = 0, nz = 0;
    bool any_long = false;
    int64_t cnt[4] = {0, 0, 0, 0};
    for (int b = 0; b < c.n; b += 64) {
        const int i = b + lane;
        int64_t r = 0;
        int cls = -1;
        if (i < c.n) {
            r = c.segs[i].pos_end - c.segs[i].pos_begin;
            any_long |= c.lend[i] > c.loff[i];
            if (c.status) {
                const ddm_ctl_part& p = c.parts[i];
                cls = p.done ? 3 : p.stall ? 1 : p.park ? 2 : 0;
            }
        }
        total += r;
        nz += r > 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) cnt[k] += __popcll(__ballot(cls == k));
    }
    total = wave_sum_i64(total);
    nz = wave_sum_i64(nz);
    const bool long_any = __ballot(any_long) != 0;
    int64_t b0 = 0;
    const int64_t spare = max((int64_t)0, c.predict_blocks - nz);
    for (int b = 0; b < c.n; b += 64) {
        const int i = b + lane;
        int64_t nbk = 0;
        if (i < c.n) {
            const int64_t r = c.segs[i].pos_end - c.segs[i].pos_begin;
            nbk = r > 0 ? 1 + (total > 0 ? spare * r / total : 0) : 0;
            nbk = min(nbk, max((int64_t)r > 0 ? 1 : 0, (r + 499) / 500));   // no more blocks than 500-row tiles
        }
        int64_t incl = nbk;                         // inclusive prefix over the lanes
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int64_t u = __shfl_up(incl, o, 64);
            if (lane >= o) incl += u;
        }
        if (i < c.n) {
            c.segs[i].block0 = b0 + incl - nbk;
            c.segs[i].nblocks = nbk;
        }
        b0 += __shfl(incl, 63, 64);
    }
    if (lane == 0) {
        if (c.sync) c.sync[1] = (uint32_t)long_any;
        if (c.status)
            for (int k = 0; k < 4; ++k) c.status[k] = cnt[k];
    }
}

}  // namespace
