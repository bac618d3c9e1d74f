"""Typed wrappers over the device entry points of the C-ABI (torch tensors in, no copies).

Every function is asynchronous on the given torch stream (default: current stream of
the tensor's device) and raises DdmError on a non-zero return code.
"""
import ctypes

import numpy as np
import torch

from ._capi import DdmParams, check, lib

STATE_DTYPE = np.dtype([("miss_prob", "<f8"), ("miss_std", "<f8"), ("miss_prob_min", "<f8"),
                        ("miss_sd_min", "<f8"), ("miss_prob_sd_min", "<f8"), ("sample_count", "<i8"),
                        ("in_concept_change", "<i4"), ("in_warning_zone", "<i4")])
assert STATE_DTYPE.itemsize == 56


# Batch tables (include/ddm_amd.h: ddm_predict_segment, ddm_shuffle_job, ddm_gen_job)
SEG_DTYPE = np.dtype([("X", "<u8"), ("ld", "<i8"), ("y", "<u8"), ("perm", "<u8"), ("err", "<u8"), ("pred", "<u8"),
                      ("first_err", "<u8"), ("pos_begin", "<i8"), ("pos_end", "<i8"), ("nodes", "<u8"),
                      ("roots", "<u8"), ("leaf_value", "<u8"), ("classes", "<u8"), ("n_trees", "<i4"),
                      ("n_classes", "<i4"), ("n_nodes", "<i4"), ("pure", "<i4"), ("row_base", "<i8"),
                      ("block0", "<i8"), ("nblocks", "<i8"), ("cforest", "<u8"), ("cf_slots", "<i4"),
                      ("cf_vote_regs", "<i4"), ("cf_leaves", "<i4"), ("flags", "<i4"),
                      ("cf_tab_words", "<i4"), ("pad", "<i4")])
SEG_FIRST_ERR_PRESET = 1
assert SEG_DTYPE.itemsize == 176
JOB_DTYPE = np.dtype([("R", "<u8"), ("Tpre", "<u8"), ("Tchunk", "<u8"), ("avail", "<i8"), ("P", "<i8"), ("W", "<i8"),
                      ("pieces", "<u8"), ("info", "<u8"), ("J", "<u8"), ("E", "<u8"), ("perm_out", "<u8"),
                      ("stop", "<u8"), ("pick_offset", "<i8"), ("pick_last", "<i8"), ("pick_out", "<u8"),
                      ("first", "<u8")])
assert JOB_DTYPE.itemsize == 128
GEN_DTYPE = np.dtype([("state", "<u8"), ("R", "<u8"), ("n", "<i8")])
TAB_DTYPE = np.dtype([("R", "<u8"), ("chunk0", "<i8"), ("nchunk", "<i8"), ("Tpre", "<u8"), ("Tchunk", "<u8")])
STAGE_DTYPE = np.dtype([("X", "<u8"), ("ld", "<i8"), ("y", "<u8"), ("perm", "<u8"), ("base", "<i8"), ("ev", "<u8"),
                        ("stop", "<u8"), ("pick", "<u8"), ("R", "<u8"), ("j", "<i8"), ("g0", "<i8"), ("nb", "<i8"),
                        ("b_end", "<i8"), ("p_after_first", "<i8"), ("p_tail_after", "<i8"), ("pb", "<i4"),
                        ("last_len", "<i4"), ("n_features", "<i4"), ("n_words", "<i4"), ("tail", "<i4"),
                        ("max_events", "<i4"), ("x_out", "<u8"), ("y_out", "<u8"), ("w_out", "<u8"),
                        ("info_out", "<u8"), ("ev_out", "<u8"), ("perm_w", "<u8"), ("seeds_out", "<u8"),
                        ("n_trees", "<i4"), ("win_rule", "<i4"), ("p_now", "<i8"), ("win", "<i8"), ("max_win", "<i8"),
                        ("seg_start", "<i8"), ("n_full", "<i8"), ("min_win", "<i8"), ("next_avail", "<i8"),
                        ("dpb_x1024", "<i8"), ("plan_out", "<u8"), ("next_job", "<u8")])
STAGE_DTYPE = np.dtype(STAGE_DTYPE.descr + [("log", "<u8"), ("log_n", "<u8"), ("log_cap", "<i8"), ("stall", "<u8")])
assert STAGE_DTYPE.itemsize == 320
# ddm_ctl_part (include/ddm_amd.h): one partition of the device-resident runner
CTL_PART_DTYPE = np.dtype([("job", JOB_DTYPE), ("seg", SEG_DTYPE), ("stage", STAGE_DTYPE), ("res", "<u8"),
                           ("dnodes", "<u8"), ("droots", "<u8"), ("dleaf", "<u8"), ("dclasses", "<u8"),
                           ("dblob", "<u8"), ("nb", "<i8"), ("n_full", "<i8"), ("base", "<i8"), ("max_win", "<i8"),
                           ("min_win", "<i8"), ("long_min_rows", "<i8"), ("long_cap_rows", "<i8"),
                           ("dpb_x1024", "<i8"), ("pb", "<i4"), ("last_len", "<i4"), ("n_words", "<i4"),
                           ("dtrees", "<i4"), ("host_slots", "<i4"), ("win_rule", "<i4"),
                           ("j", "<i8"), ("P", "<i8"), ("win", "<i8"), ("seg_start", "<i8"), ("P1", "<i8"),
                           ("P2", "<i8"), ("avail", "<i8"), ("retrain", "<i4"), ("done", "<i4"), ("stall", "<i4"),
                           ("park", "<i4"), ("forest_dev", "<i4"), ("applied", "<i4"), ("idle", "<i4"),
                           ("pad1", "<i4"), ("g0", "<i8"), ("b_end", "<i8"), ("Wg", "<i8"),
                           ("P_after_first", "<i8"), ("p0", "<i8"), ("p1", "<i8"), ("state", STATE_DTYPE),
                           ("n_log", "<i8"), ("predicted_rows", "<i8"), ("predict_bytes", "<i8"), ("epochs", "<i8"),
                           ("refits", "<i8"), ("log_mark", "<i8"), ("long_scans", "<i8"),
                           ("permute_rows", "<i8"), ("pad2", "<i8")])
CTL_STALL_REFIT, CTL_STALL_WORDS, CTL_STALL_SCAN, CTL_STALL_LONG = 1, 2, 3, 4


class PinnedTable:
    """A pinned host table of `dtype` records mirrored by a device buffer (its own, or
    byte views h / d of a larger pair of buffers that are copied as a whole)."""

    def __init__(self, dtype, n, device, h=None, d=None):
        self.dtype, self.n = dtype, int(n)
        nbytes = max(1, self.n) * dtype.itemsize
        self.h = torch.zeros(nbytes, dtype=torch.uint8, pin_memory=True) if h is None else h[:nbytes]
        # no fill on the device side: every table is uploaded before a kernel reads it, and a
        # fill kernel on the caller's stream would not be ordered with the stream that
        # uploads and reads the table
        self.d = torch.empty(nbytes, dtype=torch.uint8, device=device) if d is None else d[:nbytes]
        self.rec = self.h.numpy().view(dtype)

    def upload(self, count, stream):
        nb = int(count) * self.dtype.itemsize
        if nb:
            with torch.cuda.stream(stream):
                self.d[:nb].copy_(self.h[:nb], non_blocking=True)


def forest_predict_batch(table, n_segs, per_batch, stream, timer=None):
    """All segments of `table` (a PinnedTable of SEG_DTYPE) in one launch per kernel variant;
    the C-ABI assigns blocks and copies the table itself."""
    check(lib.ddm_forest_predict_batch(table.h.data_ptr(), table.d.data_ptr(), int(n_segs), int(per_batch),
                                       ctypes.c_void_p(stream.cuda_stream), *_evs(timer)), "ddm_forest_predict_batch")


def epoch_stage(table, n_jobs, stream, upload=True):
    """ddm_epoch_stage over the first n_jobs records of a PinnedTable of STAGE_DTYPE
    (upload=False: the caller already copied the table to the device)."""
    if upload:
        table.upload(n_jobs, stream)
    check(lib.ddm_epoch_stage(table.d.data_ptr(), int(n_jobs), ctypes.c_void_p(stream.cuda_stream)),
          "ddm_epoch_stage")


def shuffle_tables_batch(table, n_jobs, max_chunks, batch_len, stream):
    """Prefix tables of every job in a PinnedTable of TAB_DTYPE, one launch."""
    table.upload(n_jobs, stream)
    check(lib.ddm_shuffle_tables_batch(table.d.data_ptr(), int(n_jobs), int(max_chunks), int(batch_len),
                                       ctypes.c_void_p(stream.cuda_stream)), "ddm_shuffle_tables_batch")


def shuffle_generate_batch(table, n_jobs, stream):
    table.upload(n_jobs, stream)
    check(lib.ddm_shuffle_generate_batch(table.d.data_ptr(), int(n_jobs), ctypes.c_void_p(stream.cuda_stream)),
          "ddm_shuffle_generate_batch")


JUMP_DTYPE = np.dtype([("key", "<u8"), ("poly", "<u8"), ("out", "<u8"), ("scratch", "<u8")])
JUMP_SCRATCH_WORDS = 21216
POLY_WORDS = 312
_poly_cache = {}


def mt_jump_polys(jump, n, device):
    """Device tensor [n, POLY_WORDS] of x^((k+1)*jump) mod phi (MT19937 jump-ahead), cached
    per (device, jump) and grown on demand."""
    key = (str(device), int(jump))
    held = _poly_cache.setdefault(key, [])
    if not held or held[-1].shape[0] < n:
        m = max(int(n), 256, 2 * (held[-1].shape[0] if held else 0))
        host = np.zeros((m, POLY_WORDS), dtype=np.uint64)
        check(lib.ddm_mt_jump_polys(int(jump), m, host.ctypes.data), "ddm_mt_jump_polys")
        t = torch.from_numpy(host.view(np.int64)).to(device)
        torch.cuda.synchronize(device)      # readers run on other streams
        held.append(t)                      # earlier tables stay alive for in-flight jumps
    return held[-1]


def mt_jump(table, n_jobs, stream):
    """ddm_mt_jump over the first n_jobs records of a PinnedTable of JUMP_DTYPE."""
    table.upload(n_jobs, stream)
    check(lib.ddm_mt_jump(table.d.data_ptr(), int(n_jobs), ctypes.c_void_p(stream.cuda_stream)), "ddm_mt_jump")


def shuffle_window_batch(table, n_jobs, max_W, max_pieces, batch_len, stream, timer=None):
    """Window shuffles of every job in the (already uploaded) job table."""
    check(lib.ddm_shuffle_window_batch(table.d.data_ptr(), int(n_jobs), int(max_W), int(max_pieces), int(batch_len),
                                       ctypes.c_void_p(stream.cuda_stream), *_evs(timer)), "ddm_shuffle_window_batch")


def shuffle_pick_batch(table, n_jobs, stream):
    check(lib.ddm_shuffle_pick_batch(table.d.data_ptr(), int(n_jobs), ctypes.c_void_p(stream.cuda_stream)),
          "ddm_shuffle_pick_batch")


def fresh_states(n):
    """`DDM(...)` as constructed at DDM_Process.py:139 (skmultiflow reset())."""
    st = np.zeros(n, dtype=STATE_DTYPE)
    st["miss_prob"] = 1.0
    st["miss_prob_min"] = st["miss_sd_min"] = st["miss_prob_sd_min"] = np.inf
    st["sample_count"] = 1
    return st


def params_struct(min_num_instances=3, per_batch=100, warning_level=0.5, out_control_level=1.5):
    return DdmParams(int(min_num_instances), int(per_batch), float(warning_level), float(out_control_level))


def _stream(t, stream):
    s = stream if stream is not None else torch.cuda.current_stream(t.device)
    return ctypes.c_void_p(s.cuda_stream)


def _ptr(t):
    return None if t is None else t.data_ptr()


class LaunchTimer:
    """A (begin, end) HIP event pair recorded by the C-ABI around one kernel launch."""

    def __init__(self):
        self.ev = [ctypes.c_void_p(), ctypes.c_void_p()]
        for e in self.ev:
            check(lib.ddm_event_create(ctypes.byref(e)), "ddm_event_create")

    def elapsed_ms(self):
        ms = ctypes.c_float()
        check(lib.ddm_event_elapsed_ms(self.ev[0], self.ev[1], ctypes.byref(ms)), "ddm_event_elapsed_ms")
        return ms.value

    def __del__(self):
        if lib is None or getattr(lib, "ddm_event_destroy", None) is None:     # interpreter shutdown
            return
        for e in getattr(self, "ev", []):
            if e.value:
                lib.ddm_event_destroy(e)


def _evs(timer):
    return (None, None) if timer is None else (timer.ev[0], timer.ev[1])


def forest_predict(X, y, perm, pos_begin, pos_end, per_batch, forest, err, first_err=None, pred=None,
                   stream=None, timer=None):
    """X: float32 [F, ld] (columnar), y int32 [ld], perm/err uint8 indexed by DDM position."""
    assert X.dtype == torch.float32 and X.dim() == 2 and X.is_contiguous()
    assert y.dtype == torch.int32 and perm.dtype == torch.uint8 and err.dtype == torch.uint8
    assert pos_end <= perm.numel() and pos_end <= err.numel()
    F, ld = X.shape
    check(lib.ddm_forest_predict(X.data_ptr(), ld, F, y.data_ptr(), perm.data_ptr(), int(pos_begin), int(pos_end),
                                 int(per_batch), ctypes.byref(forest.desc), err.data_ptr(), _ptr(first_err),
                                 _ptr(pred), _stream(X, stream), *_evs(timer)), "ddm_forest_predict")


def scan_streams(err, offsets, params, state, batch_base, n_batches_total, ev, first_nz=None, stop=None, nev=None,
                 mode=0, ps=None, stream=None, timer=None, perm_map=None):
    """err uint8 (padded to a multiple of 16 past the last offset); offsets/batch_base int64;
    state: uint8 tensor holding n_streams ddm_state records; ev int32 [n_batches_total, 2]."""
    check(lib.ddm_scan_streams(err.data_ptr(), _ptr(offsets), offsets.numel() - 1, ctypes.byref(params),
                               _ptr(state), _ptr(first_nz), _ptr(batch_base), int(n_batches_total), _ptr(ev),
                               _ptr(stop), _ptr(nev), int(mode), _ptr(ps), _ptr(perm_map), None,
                               _stream(err, stream), *_evs(timer)), "ddm_scan_streams")


def scan_batches_scratch_size(n_streams, stream_len, per_batch=100):
    """Bytes of device scratch ddm_scan_batches needs."""
    return int(lib.ddm_scan_batches_scratch_bytes(int(n_streams), int(stream_len), int(per_batch)))


def scan_batches(err, n_streams, stream_len, params, state, ev, scratch, nev=None, perm_map=None, stream=None,
                 timer=None):
    """Mode-1 DDM over n_streams back-to-back streams of stream_len rows (batch-parallel kernels).
    ev int32 [n_streams*nb, 2]; scratch uint8 [scan_batches_scratch_size(...)]; state n_streams
    ddm_state records (updated in place)."""
    nb = -(-stream_len // params.per_batch)
    assert err.dtype == torch.uint8 and err.numel() >= ((n_streams * stream_len + 15) // 16) * 16
    assert ev.dtype == torch.int32 and ev.numel() >= 2 * n_streams * nb
    assert scratch.numel() >= scan_batches_scratch_size(n_streams, stream_len, params.per_batch)
    assert state.numel() >= 56 * n_streams
    check(lib.ddm_scan_batches(err.data_ptr(), int(n_streams), int(stream_len), ctypes.byref(params), _ptr(state),
                               _ptr(ev), _ptr(nev), _ptr(scratch), _ptr(perm_map), _stream(err, stream),
                               *_evs(timer)), "ddm_scan_batches")


def scan_long_scratch_size(n_streams, max_rows, per_batch=100):
    """Bytes of device scratch ddm_scan_long needs."""
    return int(lib.ddm_scan_long_scratch_bytes(int(n_streams), int(max_rows), int(per_batch)))


def scan_long(err, offsets, params, state, batch_base, ev, max_rows, scratch, ends=None, stop=None, nev=None, mode=0,
              perm_map=None, stream=None, timer=None):
    """ddm_scan_long over streams err[offsets[s]:ends[s]] (ends None: offsets[s+1]); the
    results of scan_streams for long carried segments (see include/ddm_amd.h)."""
    n = offsets.numel() - (0 if ends is not None else 1)
    assert scratch.numel() >= scan_long_scratch_size(n, max_rows, params.per_batch)
    check(lib.ddm_scan_long(err.data_ptr(), offsets.data_ptr(), _ptr(ends), int(n), int(max_rows),
                            ctypes.byref(params), state.data_ptr(), batch_base.data_ptr(), ev.data_ptr(), _ptr(stop),
                            _ptr(nev), int(mode), _ptr(perm_map), scratch.data_ptr(), _stream(err, stream),
                            *_evs(timer)), "ddm_scan_long")


def scan_certified_scratch_size(n_streams, max_rows, per_batch=100):
    """Bytes of device scratch ddm_scan_certified needs."""
    return int(lib.ddm_scan_certified_scratch_bytes(int(n_streams), int(max_rows), int(per_batch)))


def scan_certified(err, offsets, params, state, batch_base, ev, max_rows, scratch, ends=None, stop=None, nev=None,
                   mode=0, perm_map=None, bound=None, status=None, stream=None, timer=None):
    """ddm_scan_certified: ddm_scan_long's results with row-parallel certified decisions
    (include/ddm_amd.h); bound: float64 [n, 2] device tensor (in/out) or None; status:
    int32 [n] device tensor or None."""
    n = offsets.numel() - (0 if ends is not None else 1)
    assert scratch.numel() >= scan_certified_scratch_size(n, max_rows, params.per_batch)
    assert bound is None or (bound.dtype == torch.float64 and bound.numel() >= 2 * n)
    check(lib.ddm_scan_certified(err.data_ptr(), offsets.data_ptr(), _ptr(ends), int(n), int(max_rows),
                                 ctypes.byref(params), state.data_ptr(), _ptr(bound), batch_base.data_ptr(),
                                 ev.data_ptr(), _ptr(stop), _ptr(nev), int(mode), _ptr(perm_map), _ptr(status),
                                 scratch.data_ptr(), _stream(err, stream), *_evs(timer)), "ddm_scan_certified")


def scan_long_raw(err_ptr, off_ptr, end_ptr, n_streams, max_rows, params, state_ptr, batch_base_ptr, ev_ptr, stop_ptr,
                  nev_ptr, mode, perm_map_ptr, scratch_ptr, stream, timer=None):
    """Pointer-level ddm_scan_long (the controller's long carried windows)."""
    check(lib.ddm_scan_long(err_ptr, off_ptr, end_ptr, int(n_streams), int(max_rows), ctypes.byref(params), state_ptr,
                            batch_base_ptr, ev_ptr, stop_ptr, nev_ptr, int(mode), perm_map_ptr, scratch_ptr,
                            ctypes.c_void_p(stream.cuda_stream), *_evs(timer)), "ddm_scan_long")


def scan_streams_raw(err_ptr, offsets_ptr, n_streams, params, state_ptr, batch_base_ptr, n_batches_total, ev_ptr,
                     first_nz_ptr, stop_ptr, nev_ptr, mode, ps_ptr, stream, timer=None, perm_map_ptr=None,
                     end_ptr=None):
    """Pointer-level variant used by the controller (all pointers are device addresses)."""
    check(lib.ddm_scan_streams(err_ptr, offsets_ptr, n_streams, ctypes.byref(params), state_ptr, first_nz_ptr,
                               batch_base_ptr, n_batches_total, ev_ptr, stop_ptr, nev_ptr, mode, ps_ptr, perm_map_ptr,
                               end_ptr, ctypes.c_void_p(stream.cuda_stream), *_evs(timer)), "ddm_scan_streams")


def synth_block_labels(y, part, n_parts, block_rows, n_classes, stream=None):
    check(lib.ddm_synth_block_labels(y.data_ptr(), y.numel(), part, n_parts, block_rows, n_classes,
                                     _stream(y, stream)), "ddm_synth_block_labels")


def synth_jitter_labels(y, part, n_parts, period, jitter, n_classes, flip, seed, stream=None):
    check(lib.ddm_synth_jitter_labels(y.data_ptr(), y.numel(), part, n_parts, period, jitter, n_classes,
                                      float(flip), seed, _stream(y, stream)), "ddm_synth_jitter_labels")


def synth_features(X, y, row0, row_stride, seed, noise=0.04, stream=None):
    F, ld = X.shape
    check(lib.ddm_synth_features(X.data_ptr(), ld, F, y.data_ptr(), y.numel(), row0, row_stride, seed,
                                 ctypes.c_float(noise), _stream(X, stream)), "ddm_synth_features")


def synth_bernoulli_streams(err, n_streams, length, seed, stream=None):
    assert err.numel() >= n_streams * length
    check(lib.ddm_synth_bernoulli_streams(err.data_ptr(), n_streams, length, seed, _stream(err, stream)),
          "ddm_synth_bernoulli_streams")
