// The epoch executor: one C call enqueues a whole speculative epoch of the BatchRunner
// (ddm_amd/controller.py) on its stream, in the order the controller needs:
//   control-block upload -> window shuffles -> forest predict -> DDM scan (one lane per
//   stream, plus ddm_scan_long for long carried windows) -> RNG pick -> staging ->
//   device refits -> control-block read-back.
// Nothing is decided here; the point is to replace ~10 separate binding calls and stream
// switches per epoch by one.  When the staging planned the next windows (next_jobs), their
// shuffles run on a side stream beside the device refits, so the next epoch can start
// with its forest predict.
#include "common.h"

extern "C" int ddm_epoch_launch(const ddm_epoch* e) {
    if (!e || !e->ctrl_d || !e->ctrl_h || e->upload_bytes < 0 || e->download_bytes < 0) {
        ddm::set_error("ddm_epoch_launch: invalid argument");
        return DDM_E_ARG;
    }
    hipStream_t s = ddm::as_hip(e->stream);
    if (e->upload_bytes)
        if (int rc = ddm::hip_status(hipMemcpyAsync(e->ctrl_d, e->ctrl_h, (size_t)e->upload_bytes,
                                                    hipMemcpyHostToDevice, s), "ddm_epoch_launch/upload"))
            return rc;
    if (e->n_shuffle > 0)
        if (int rc = ddm_shuffle_window_batch(e->shuffle_jobs, e->n_shuffle, e->max_W, e->max_pieces, e->per_batch,
                                              e->stream, e->ev[0], e->ev[1]))
            return rc;
    if (e->n_segs > 0)
        if (int rc = ddm_forest_predict_batch(e->segs_h, e->segs_d, e->n_segs, e->per_batch, e->stream, e->ev[2],
                                              e->ev[3]))
            return rc;
    if (int rc = ddm_scan_streams(e->err, e->offsets, e->n_streams, e->params, e->state, e->first_nz, e->batch_base,
                                  e->n_batches_total, e->ev_out, e->stop, e->nev, 0, nullptr, e->perm_map, e->ends,
                                  e->stream, e->ev[4], e->ev[5]))
        return rc;
    if (e->long_max_rows > 0)
        if (int rc = ddm_scan_long(e->err, e->long_off, e->long_end, e->n_streams, e->long_max_rows, e->params,
                                   e->state, e->batch_base, e->ev_out, e->stop, e->nev, 0, e->perm_map,
                                   e->long_scratch, e->stream, e->ev[6], e->ev[7]))
            return rc;
    if (e->n_pick > 0)
        if (int rc = ddm_shuffle_pick_batch(e->pick_jobs, e->n_pick, e->stream)) return rc;
    if (e->n_stage > 0)
        if (int rc = ddm_epoch_stage(e->stage_jobs, e->n_stage, e->stream)) return rc;
    const bool fork = e->n_next > 0 && e->next_jobs && e->side_stream && e->fork_ev && e->join_ev;
    const bool split = e->mid_ev != nullptr && e->download_bytes > 0;
    if (fork) {
        // the next windows' shuffles (planned by the staging) beside the refits
        hipStream_t side = ddm::as_hip(e->side_stream);
        if (int rc = ddm::hip_status(hipEventRecord(reinterpret_cast<hipEvent_t>(e->fork_ev), s), "fork")) return rc;
        if (int rc = ddm::hip_status(hipStreamWaitEvent(side, reinterpret_cast<hipEvent_t>(e->fork_ev), 0), "fork"))
            return rc;
        if (int rc = ddm_shuffle_window_batch(e->next_jobs, e->n_next, e->next_max_W, e->next_max_pieces, e->per_batch,
                                              e->side_stream, nullptr, nullptr))
            return rc;
        if (int rc = ddm::hip_status(hipEventRecord(reinterpret_cast<hipEvent_t>(e->join_ev), side), "join")) return rc;
    }
    if (split) {
        // everything but the refit results goes back now (mid_ev); the host works on it
        // while the refits and the next shuffles run
        if (int rc = ddm::hip_status(hipMemcpyAsync(e->ctrl_h, e->ctrl_d, (size_t)e->download_bytes,
                                                    hipMemcpyDeviceToHost, s), "ddm_epoch_launch/read-back"))
            return rc;
        if (int rc = ddm::hip_status(hipEventRecord(reinterpret_cast<hipEvent_t>(e->mid_ev), s), "mid")) return rc;
    }
    if (e->n_dfit > 0) {
        if (e->ev[8])
            if (int rc = ddm::hip_status(hipEventRecord(reinterpret_cast<hipEvent_t>(e->ev[8]), s), "event record"))
                return rc;
        if (int rc = ddm_rf_fit_device_lf(e->dfit_jobs, e->n_dfit, e->max_trees, e->dfit_max_lf, e->stream)) return rc;
        if (e->ev[9])
            if (int rc = ddm::hip_status(hipEventRecord(reinterpret_cast<hipEvent_t>(e->ev[9]), s), "event record"))
                return rc;
    }
    if (fork)
        if (int rc = ddm::hip_status(hipStreamWaitEvent(s, reinterpret_cast<hipEvent_t>(e->join_ev), 0), "join"))
            return rc;
    if (split) {
        if (e->tail_bytes > 0)
            if (int rc = ddm::hip_status(
                    hipMemcpyAsync(static_cast<uint8_t*>(e->ctrl_h) + e->tail_off,
                                   static_cast<const uint8_t*>(e->ctrl_d) + e->tail_off, (size_t)e->tail_bytes,
                                   hipMemcpyDeviceToHost, s),
                    "ddm_epoch_launch/refit read-back"))
                return rc;
    } else if (e->download_bytes) {
        if (int rc = ddm::hip_status(hipMemcpyAsync(e->ctrl_h, e->ctrl_d, (size_t)e->download_bytes,
                                                    hipMemcpyDeviceToHost, s), "ddm_epoch_launch/read-back"))
            return rc;
    }
    return 0;
}

extern "C" int64_t ddm_epoch_struct_bytes(void) { return (int64_t)sizeof(ddm_epoch); }
