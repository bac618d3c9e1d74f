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
#include "ctl_dev.h"

namespace {

constexpr int kCtlThreads = 256;
constexpr int kCtlWaves = kCtlThreads / 64;

// The decisions of every partition (a wave per record), then the grid split (one wave).
__global__ __launch_bounds__(kCtlThreads) void k_ctl(const ddm_ctl c) {
    __shared__ ddm_ctl_part s_part[kCtlWaves];
    const int t = threadIdx.x;
    const int lane = t & 63, w = t >> 6;
    for (int i = w; i < c.n; i += kCtlWaves) ctl_record(c, i, &s_part[w], lane, c.entry);
    __threadfence();
    __syncthreads();
    if (t < 64) ctl_split(c, t);
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
constexpr int32_t kPermBlocks = 256;            // ddm_err_permute_dev blocks per partition

// Cross-stream order without HIP events (ddm_ctl_epoch.sync_flags, common.h flag_publish /
// flag_poll): the producing stream stores a sequence number after its data (agent-scope
// release, then an sc1 store), the consuming stream polls it (sc1 loads, s_sleep between
// polls); the data are ordered by kernel boundaries (the consumer's kernels start after
// the poll).  The fork is stored by the last workgroup of k_stage_ctl itself and polled by
// a one-wave kernel at the head of the side stream; the side stream stores the join after
// its shuffles (a one-wave kernel), and in coupled epochs the refit's pack kernel polls it
// (one thread of workgroup 0, after its job), so the next predict starts right after the
// pack; decoupled epochs poll it by a one-wave kernel before the permutation.  A fork +
// join by one-wave kernels costs ~12 us against ~30 us with two events
// (profiles/r04/gap_bench.log).  Every poll is enqueued after the store it waits for, so
// even streams sharing one hardware queue cannot deadlock; a poll still gives up (a hang
// guard: after flags[3] ticks, 0 = 2 s) and counts it in flags[2], which voids the phase
// (ddm_amd/devctl.py raises FlagTimeout and the runner redoes the run with events).
__global__ __launch_bounds__(64) void k_flag_pub(uint32_t* flag, uint32_t v) {
    if (threadIdx.x == 0) ddm::flag_publish(flag, v);
}

__global__ __launch_bounds__(64) void k_flag_wait(const uint32_t* flag, uint32_t v, uint32_t* timeouts) {
    if (threadIdx.x == 0) ddm::flag_poll(flag, v, timeouts);
}

int flag_pub(uint32_t* flags, int k, uint32_t v, hipStream_t s) {
    hipLaunchKernelGGL(k_flag_pub, dim3(1), dim3(64), 0, s, flags + k, v);
    return ddm::launch_status("ddm_ctl_epochs/flag");
}

int flag_wait(uint32_t* flags, int k, uint32_t v, hipStream_t s) {
    hipLaunchKernelGGL(k_flag_wait, dim3(1), dim3(64), 0, s, flags + k, v, flags + 2);
    return ddm::launch_status("ddm_ctl_epochs/flag wait");
}

}  // namespace

extern "C" int ddm_scan_long_reuse(const uint8_t* err, const int64_t* stream_off, const int64_t* stream_end,
                                   int64_t n_streams, int64_t max_rows, const ddm_params* prm, ddm_state* state_io,
                                   const int64_t* batch_base, int32_t* ev_out, int32_t* stop_out, int64_t* nev_out,
                                   int32_t mode, const uint8_t* perm_map, void* scratch, const int32_t* any,
                                   ddm_stream_t stream);
extern "C" int ddm_forest_predict_dev_orig(const ddm_predict_segment* segs_dev, const int64_t* const* res_dev,
                                           int32_t n_segs, int32_t per_batch, int64_t grid, int32_t* stall,
                                           int64_t delta, uint64_t* clk, const uint32_t* join_flag,
                                           uint32_t join_v, uint32_t* timeouts, ddm_stream_t stream);
int forest_predict_dev_clk(const ddm_predict_segment* segs_dev, const int64_t* const* res_dev, int32_t n_segs,
                           int32_t per_batch, int64_t grid, int32_t* stall, uint64_t* clk, ddm_stream_t stream);
extern "C" int ddm_err_permute_dev(const ddm_predict_segment* segs_dev, int32_t n_segs, int32_t per_batch,
                                   int64_t delta, int32_t blocks_per_seg, ddm_stream_t stream);
extern "C" int ddm_epoch_stage_ctl(const ddm_stage_job* jobs_dev, const ddm_shuffle_job* shuffle_jobs,
                                   const ddm_ctl* ctl, const uint8_t* err, const ddm_params* prm,
                                   const uint8_t* perm_map, ddm_stream_t stream);
int epoch_stage_ctl_pub(const ddm_stage_job* jobs_dev, const ddm_shuffle_job* shuffle_jobs, const ddm_ctl* ctl,
                        const uint8_t* err, const ddm_params* prm, const uint8_t* perm_map, uint32_t* pub_flag,
                        uint32_t pub_v, ddm_stream_t stream);
int rf_fit_device_join(const ddm_dfit_job* jobs_dev, int32_t n_jobs, int32_t max_trees, int64_t max_lf,
                       const uint32_t* join_flag, uint32_t join_v, uint32_t* timeouts, ddm_stream_t stream);

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
    // ctl_split gives every non-empty window at least one block of the fixed predict grid:
    // more partitions than blocks would leave windows past the grid unpredicted
    if (e->ctl.n > e->ctl.predict_blocks) {
        ddm::set_error("ddm_ctl_enter: more partitions than predict blocks");
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

namespace {

// The epochs' launch sequence.  graph: the sequence is being captured into a graph that is
// replayed back to back on the stream, so the first epoch needs no join (the graph before
// it ended with one) and the last one ends with a join (a capture must end joined).
int ctl_epochs(const ddm_ctl_epoch* e, int32_t n_epochs, bool graph);

}  // namespace

extern "C" int ddm_ctl_epochs(const ddm_ctl_epoch* e, int32_t n_epochs) { return ctl_epochs(e, n_epochs, false); }

// Epoch groups as hipGraphs: the whole group (both streams, their fork / join edges) is
// captured once and replayed; every decision it needs is in device memory (k_ctl), so the
// same graph serves every group of a runner whose tables do not move.
extern "C" int ddm_ctl_graph_create(const ddm_ctl_epoch* e, int32_t n_epochs, void** exec_out) {
    if (!e || !exec_out || n_epochs <= 0 || e->predict_evs) {
        ddm::set_error("ddm_ctl_graph_create: invalid argument");
        return DDM_E_ARG;
    }
    for (int k = 0; k < 12; ++k)
        if (e->ev[k]) {
            ddm::set_error("ddm_ctl_graph_create: timing events are not captured");
            return DDM_E_ARG;
        }
    hipStream_t s = ddm::as_hip(e->stream);
    if (int rc = ddm::hip_status(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed), "graph capture")) return rc;
    const int rc_epochs = ctl_epochs(e, n_epochs, true);
    hipGraph_t g = nullptr;
    const int rc_end = ddm::hip_status(hipStreamEndCapture(s, &g), "graph capture end");
    if (rc_epochs || rc_end) {
        if (g) (void)hipGraphDestroy(g);
        return rc_epochs ? rc_epochs : rc_end;
    }
    hipGraphExec_t x = nullptr;
    const int rc = ddm::hip_status(hipGraphInstantiate(&x, g, nullptr, nullptr, 0), "graph instantiate");
    (void)hipGraphDestroy(g);
    if (rc) return rc;
    *exec_out = x;
    return 0;
}

extern "C" int ddm_ctl_graph_launch(void* exec, ddm_stream_t stream) {
    if (!exec) {
        ddm::set_error("ddm_ctl_graph_launch: invalid argument");
        return DDM_E_ARG;
    }
    return ddm::hip_status(hipGraphLaunch(reinterpret_cast<hipGraphExec_t>(exec), ddm::as_hip(stream)),
                           "graph launch");
}

extern "C" int ddm_ctl_graph_destroy(void* exec) {
    return exec ? ddm::hip_status(hipGraphExecDestroy(reinterpret_cast<hipGraphExec_t>(exec)), "graph destroy") : 0;
}

namespace {

int ctl_epochs(const ddm_ctl_epoch* e, int32_t n_epochs, bool graph) {
    if (!e || !e->ctl.parts || e->ctl.n <= 0 || n_epochs < 0 || !e->side_stream || !e->fork_ev || !e->join_ev) {
        ddm::set_error("ddm_ctl_epochs: invalid argument");
        return DDM_E_ARG;
    }
    hipStream_t s = ddm::as_hip(e->stream);
    hipStream_t side = ddm::as_hip(e->side_stream);
    const ddm_ctl& c = e->ctl;
    // decoupled epochs: the predict writes row-order errors (it needs the refit's forest, not
    // the window's shuffle) and waits for the shuffles only before the permutation into DDM
    // order, so the side stream's window shuffles overlap the refit AND the predict
    const bool dec = e->decouple && e->row_order_delta != 0 && c.sync;
    // fork / join by flags (not inside a graph: a replay would reuse the captured numbers)
    uint32_t* const flags = graph ? nullptr : e->sync_flags;
    uint32_t* const seq = e->sync_seq;
    if (flags && !seq) {
        ddm::set_error("ddm_ctl_epochs: sync_flags without sync_seq");
        return DDM_E_ARG;
    }
    // the predict's device-clock stamps are folded by k_stage_ctl: only with the fused tail
    uint64_t* const clk = c.sync ? c.predict_clock : nullptr;
    auto join = [&]() {
        if (flags) {
            if (seq[2] == seq[1]) return 0;           // a pack kernel held the last one already
            seq[2] = seq[1];
            return flag_wait(flags, 1, seq[1], s);
        }
        return ddm::hip_status(hipStreamWaitEvent(s, reinterpret_cast<hipEvent_t>(e->join_ev), 0), "join");
    };
    for (int32_t k = 0; k < n_epochs; ++k) {
        const bool first_in_graph = graph && k == 0;   // the graph before ended with the join
        if (!dec && !first_in_graph)
            if (int rc = join()) return rc;         // the last epoch's shuffles of this window
        const ddm_event_t pb0 = e->predict_evs ? e->predict_evs[2 * k] : e->ev[0];
        const ddm_event_t pb1 = e->predict_evs ? e->predict_evs[2 * k + 1] : e->ev[1];
        if (int rc = rec(pb0, s)) return rc;
        if (dec) {
            // the predict's first workgroup holds the join of this window's shuffles (the
            // permutation's input), unless it was held already
            const bool hold = flags && !first_in_graph && seq[2] != seq[1];
            if (int rc = ddm_forest_predict_dev_orig(c.segs, c.seg_res, c.n, e->per_batch, c.predict_blocks, c.pstall,
                                                     e->row_order_delta, clk, hold ? flags + 1 : nullptr,
                                                     hold ? seq[1] : 0u, flags ? flags + 2 : nullptr, e->stream))
                return rc;
            if (hold) seq[2] = seq[1];
        } else {
            if (int rc = forest_predict_dev_clk(c.segs, c.seg_res, c.n, e->per_batch, c.predict_blocks, c.pstall, clk,
                                                e->stream))
                return rc;
        }
        if (int rc = rec(pb1, s)) return rc;
        if (dec && !first_in_graph)
            if (int rc = join()) return rc;
        if (int rc = rec(e->ev[2], s)) return rc;
        if (dec)
            if (int rc = ddm_err_permute_dev(c.segs, c.n, e->per_batch, e->row_order_delta, kPermBlocks, e->stream))
                return rc;
        // fused tail (c.sync): the one-lane scan runs inside the staging kernel, after the
        // long scan of the windows it does not take
        if (!c.sync)
            if (int rc = ddm_scan_streams_log(e->err, c.off, c.n, e->params, c.state, c.first, c.logs,
                                              reinterpret_cast<int64_t*>(reinterpret_cast<uint8_t*>(c.parts) +
                                                                         offsetof(ddm_ctl_part, n_log)),
                                              (int64_t)(sizeof(ddm_ctl_part) / sizeof(int64_t)), c.log_b0,
                                              const_cast<int32_t*>(c.stop), 0, e->perm_map, c.end, e->stream))
                return rc;
        if (e->long_max_rows > 0)
            if (int rc = ddm_scan_long_reuse(e->err, c.loff, c.lend, c.n, e->long_max_rows, e->params, c.state,
                                             e->batch_base, e->ev_out, const_cast<int32_t*>(c.stop), e->nev, 0,
                                             e->perm_map, e->long_scratch,
                                             c.sync ? reinterpret_cast<const int32_t*>(c.sync + 1) : nullptr,
                                             e->stream))
                return rc;
        if (c.sync) {                               // scan + pick + staging + decisions: one launch
            if (int rc = rec(e->ev[3], s)) return rc;
            if (int rc = rec(e->ev[4], s)) return rc;
            ddm_ctl cd = c;
            cd.decoupled = dec ? 1 : 0;
            if (int rc = epoch_stage_ctl_pub(c.stage, c.jobs, &cd, e->err, e->params, e->perm_map,
                                             flags ? flags : nullptr, flags ? seq[0] + 1 : 0, e->stream))
                return rc;
        } else {
            if (int rc = ddm_shuffle_pick_batch(c.jobs, c.n, e->stream)) return rc;
            if (int rc = rec(e->ev[3], s)) return rc;
            if (int rc = rec(e->ev[4], s)) return rc;
            if (int rc = ddm_epoch_stage(c.stage, c.n, e->stream)) return rc;
            if (int rc = launch_ctl(c, 0, s)) return rc;
        }
        if (int rc = rec(e->ev[5], s)) return rc;
        // (starting them after the refit instead, beside the next predict, was measured on
        // C3: the refit's pack 53 -> 22 us, the predict 219 -> 256 us, the epoch 379 -> 388 us)
        auto side_work = [&]() -> int {
            // the next windows' shuffles beside the refits
            if (flags) {
                ++seq[0];
                if (!c.sync)                            // else k_stage_ctl stores it itself
                    if (int rc = flag_pub(flags, 0, seq[0], s)) return rc;
                if (int rc = flag_wait(flags, 0, seq[0], side)) return rc;
            } else {
                if (int rc = ddm::hip_status(hipEventRecord(reinterpret_cast<hipEvent_t>(e->fork_ev), s), "fork"))
                    return rc;
                if (int rc = ddm::hip_status(hipStreamWaitEvent(side, reinterpret_cast<hipEvent_t>(e->fork_ev), 0),
                                             "fork"))
                    return rc;
            }
            if (int rc = rec(e->ev[10], side)) return rc;
            if (int rc = ddm_shuffle_window_batch(c.jobs, c.n, std::min(e->max_W, kShufW),
                                                  std::min(e->max_pieces, kShufPieces), e->per_batch,
                                                  e->side_stream, nullptr, nullptr))
                return rc;
            if (int rc = rec(e->ev[11], side)) return rc;
            if (flags) {
                ++seq[1];
                return flag_pub(flags, 1, seq[1], side);
            }
            return ddm::hip_status(hipEventRecord(reinterpret_cast<hipEvent_t>(e->join_ev), side), "join");
        };
        auto refit = [&]() -> int {
            if (e->n_dfit <= 0) return 0;
            if (int rc = rec(e->ev[6], s)) return rc;
            // coupled epochs: the pack kernel holds the join, the next predict needs no poll
            const bool hold = flags && !dec;
            if (int rc = rf_fit_device_join(e->dfit_jobs, e->n_dfit, e->max_trees, e->dfit_max_lf,
                                            hold ? flags + 1 : nullptr, hold ? seq[1] : 0, flags ? flags + 2 : nullptr,
                                            e->stream))
                return rc;
            if (hold) seq[2] = seq[1];
            return rec(e->ev[7], s);
        };
        if (int rc = side_work()) return rc;
        if (int rc = refit()) return rc;
    }
    // the next call's first epoch waits for the last shuffles (the caller synchronises the
    // side stream before it reads anything they write); a captured group joins them itself
    if (graph && n_epochs > 0)
        if (int rc = join()) return rc;
    return 0;
}

}  // namespace
