"""ctypes binding of libddm_amd.so (the C-ABI declared in include/ddm_amd.h).

torch is imported first so that the process holds torch's HIP runtime; the library's
`libamdhip64.so.7` dependency then resolves to that same runtime, and kernels launched
here run on torch streams against torch allocations.  There is no fallback: if the
library is missing this module raises at import time, and the product path fails.
"""
import ctypes
import os

import torch  # noqa: F401  (loads the HIP runtime the library binds to)

# DDM_AMD_LIB: an alternative build of the same library (e.g. an instrumented one)
LIB_PATH = os.environ.get("DDM_AMD_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libddm_amd.so")
ABI_VERSION = 24

DDM_E_ARG = 1001
DDM_E_FOREST = 1002
DDM_E_NAN = 1003
DDM_E_IMPURE = 1004
DDM_STOP_FAILED = -2      # ddm_scan_long: the stream's look-back gave up, its results are void
DDM_CERT_INEXACT = 3      # ddm_scan_certified: a decision was uncertified and the incoming state was
                          # inexact (a nonzero bound): every output void, redo from an exact carry


class DdmParams(ctypes.Structure):
    _fields_ = [("min_num_instances", ctypes.c_int32), ("per_batch", ctypes.c_int32),
                ("warning_level", ctypes.c_double), ("out_control_level", ctypes.c_double)]


class DdmState(ctypes.Structure):
    _fields_ = [("miss_prob", ctypes.c_double), ("miss_std", ctypes.c_double),
                ("miss_prob_min", ctypes.c_double), ("miss_sd_min", ctypes.c_double),
                ("miss_prob_sd_min", ctypes.c_double), ("sample_count", ctypes.c_int64),
                ("in_concept_change", ctypes.c_int32), ("in_warning_zone", ctypes.c_int32)]


class DdmForest(ctypes.Structure):
    _fields_ = [("nodes", ctypes.c_void_p), ("roots", ctypes.c_void_p), ("leaf_value", ctypes.c_void_p),
                ("classes", ctypes.c_void_p), ("n_trees", ctypes.c_int32), ("n_classes", ctypes.c_int32),
                ("n_nodes", ctypes.c_int32), ("pure", ctypes.c_int32), ("cforest", ctypes.c_void_p),
                ("cf_slots", ctypes.c_int32), ("cf_vote_regs", ctypes.c_int32), ("cf_leaves", ctypes.c_int32),
                ("cf_tab_words", ctypes.c_int32)]


assert ctypes.sizeof(DdmState) == 56 and ctypes.sizeof(DdmParams) == 24 and ctypes.sizeof(DdmForest) == 72

_vp, _i32, _i64, _u64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64


class DdmEpoch(ctypes.Structure):
    """ddm_epoch (include/ddm_amd.h): one BatchRunner epoch for ddm_epoch_launch."""
    _fields_ = [("stream", _vp), ("ctrl_d", _vp), ("ctrl_h", _vp), ("upload_bytes", _i64), ("download_bytes", _i64),
                ("shuffle_jobs", _vp), ("n_shuffle", _i32), ("per_batch", _i32), ("max_W", _i64),
                ("max_pieces", _i64), ("segs_h", _vp), ("segs_d", _vp), ("n_segs", _i32), ("n_stage", _i32),
                ("err", _vp), ("offsets", _vp), ("ends", _vp), ("n_streams", _i64), ("params", _vp),
                ("state", _vp), ("first_nz", _vp), ("batch_base", _vp), ("n_batches_total", _i64),
                ("ev_out", _vp), ("stop", _vp), ("nev", _vp), ("perm_map", _vp), ("long_off", _vp),
                ("long_end", _vp), ("long_max_rows", _i64), ("long_scratch", _vp), ("stage_jobs", _vp),
                ("dfit_jobs", _vp), ("n_dfit", _i32), ("max_trees", _i32), ("ev", _vp * 10),
                ("pick_jobs", _vp), ("n_pick", _i32), ("n_next", _i32), ("next_jobs", _vp), ("next_max_W", _i64),
                ("next_max_pieces", _i64), ("side_stream", _vp), ("fork_ev", _vp), ("join_ev", _vp),
                ("mid_ev", _vp), ("tail_off", _i64), ("tail_bytes", _i64), ("dfit_max_lf", _i64)]
_f32, _pi32 = ctypes.c_float, ctypes.POINTER(ctypes.c_int32)


class DdmCtl(ctypes.Structure):
    """ddm_ctl (include/ddm_amd.h): the device-resident runner's tables (device pointers)."""
    _fields_ = [("parts", _vp), ("n", _i32), ("entry", _i32), ("jobs", _vp), ("segs", _vp), ("seg_res", _vp),
                ("stage", _vp), ("off", _vp), ("end", _vp), ("state", _vp), ("first", _vp), ("stop", _vp),
                ("pick", _vp), ("loff", _vp), ("lend", _vp), ("pstall", _vp), ("predict_blocks", _i64),
                ("status", _vp), ("logs", _vp), ("log_b0", _vp), ("sync", _vp), ("decoupled", _i32),
                ("long_ok", _i32), ("predict_clock", _vp)]


class DdmCtlEpoch(ctypes.Structure):
    """ddm_ctl_epoch: ddm_ctl_enter / ddm_ctl_epochs."""
    _fields_ = [("stream", _vp), ("side_stream", _vp), ("fork_ev", _vp), ("join_ev", _vp), ("ctl", DdmCtl),
                ("ctl_d", _vp), ("n", _i32), ("per_batch", _i32), ("err", _vp), ("params", _vp),
                ("batch_base", _vp), ("n_batches_total", _i64), ("ev_out", _vp), ("nev", _vp), ("perm_map", _vp),
                ("long_max_rows", _i64), ("long_scratch", _vp), ("dfit_jobs", _vp), ("n_dfit", _i32),
                ("max_trees", _i32), ("max_W", _i64), ("max_pieces", _i64), ("dfit_max_lf", _i64),
                ("ev", _vp * 12), ("row_order_delta", _i64), ("decouple", _i32), ("pad_dc", _i32),
                ("predict_evs", _vp), ("sync_flags", _vp), ("sync_seq", _vp)]

# name -> (restype, argtypes); every symbol include/ddm_amd.h declares.
SIGNATURES = {
    "ddm_abi_version": (ctypes.c_int, []),
    "ddm_last_error": (ctypes.c_char_p, []),
    "ddm_forest_predict": (ctypes.c_int, [_vp, _i64, _i32, _vp, _vp, _i64, _i64, _i32, ctypes.POINTER(DdmForest),
                                          _vp, _vp, _vp, _vp, _vp, _vp]),
    "ddm_scan_streams": (ctypes.c_int, [_vp, _vp, _i64, ctypes.POINTER(DdmParams), _vp, _vp, _vp, _i64, _vp, _vp,
                                        _vp, _i32, _vp, _vp, _vp, _vp, _vp, _vp]),
    "ddm_scan_batches": (ctypes.c_int, [_vp, _i64, _i64, ctypes.POINTER(DdmParams), _vp, _vp, _vp, _vp, _vp, _vp,
                                        _vp, _vp]),
    "ddm_scan_batches_scratch_bytes": (_i64, [_i64, _i64, _i32]),
    "ddm_scan_long": (ctypes.c_int, [_vp, _vp, _vp, _i64, _i64, ctypes.POINTER(DdmParams), _vp, _vp, _vp, _vp, _vp,
                                     _i32, _vp, _vp, _vp, _vp, _vp]),
    "ddm_scan_long_scratch_bytes": (_i64, [_i64, _i64, _i32]),
    "ddm_scan_streams_log": (ctypes.c_int, [_vp, _vp, _i64, ctypes.POINTER(DdmParams), _vp, _vp, _vp, _vp, _i64, _vp,
                                            _vp, _i32, _vp, _vp, _vp]),
    "ddm_scan_long_set_spin_limit": (ctypes.c_int, [ctypes.c_uint32]),
    "ddm_scan_certified_scratch_bytes": (_i64, [_i64, _i64, _i32]),
    "ddm_scan_certified": (ctypes.c_int, [_vp, _vp, _vp, _i64, _i64, ctypes.POINTER(DdmParams), _vp, _vp, _vp, _vp,
                                          _vp, _vp, _i32, _vp, _vp, _vp, _vp, _vp, _vp]),
    "ddm_scan_certified_set_tol_scale": (ctypes.c_int, [ctypes.c_double]),
    "ddm_forest_predict_batch": (ctypes.c_int, [_vp, _vp, _i32, _i32, _vp, _vp, _vp]),
    "ddm_shuffle_generate_batch": (ctypes.c_int, [_vp, _i32, _vp]),
    "ddm_mt_charpoly": (ctypes.c_int, [_vp]),
    "ddm_mt_jump_polys": (ctypes.c_int, [_i64, _i32, _vp]),
    "ddm_mt_jump": (ctypes.c_int, [_vp, _i32, _vp]),
    "ddm_shuffle_window_batch": (ctypes.c_int, [_vp, _i32, _i64, _i64, _i32, _vp, _vp, _vp]),
    "ddm_shuffle_pick_batch": (ctypes.c_int, [_vp, _i32, _vp]),
    "ddm_shuffle_generate": (ctypes.c_int, [_vp, _vp, _i64, _vp]),
    "ddm_shuffle_tables": (ctypes.c_int, [_vp, _i64, _i64, _i32, _vp, _vp, _vp]),
    "ddm_shuffle_tables_batch": (ctypes.c_int, [_vp, _i32, _i64, _i32, _vp]),
    "ddm_epoch_launch": (ctypes.c_int, [_vp]),
    "ddm_ctl_part_bytes": (_i64, []),
    "ddm_ctl_epoch_bytes": (_i64, []),
    "ddm_ctl_enter": (ctypes.c_int, [_vp]),
    "ddm_ctl_epochs": (ctypes.c_int, [_vp, _i32]),
    "ddm_ctl_graph_create": (ctypes.c_int, [_vp, _i32, ctypes.POINTER(ctypes.c_void_p)]),
    "ddm_ctl_graph_launch": (ctypes.c_int, [_vp, _vp]),
    "ddm_ctl_graph_destroy": (ctypes.c_int, [_vp]),
    "ddm_forest_predict_dev": (ctypes.c_int, [_vp, _vp, _i32, _i32, _i64, _vp, _vp, _vp, _vp]),
    "ddm_epoch_struct_bytes": (_i64, []),
    "ddm_shuffle_window": (ctypes.c_int, [_vp, _vp, _vp, _i64, _i64, _i64, _i32, _vp, _i64, _vp, _vp, _vp, _vp, _vp,
                                          _vp, _vp, _vp]),
    "ddm_shuffle_pick": (ctypes.c_int, [_vp, _vp, _i64, _i64, _i64, _vp, _vp]),
    "ddm_event_create": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p)]),
    "ddm_event_create_sync": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p)]),
    "ddm_event_destroy": (ctypes.c_int, [_vp]),
    "ddm_event_elapsed_ms": (ctypes.c_int, [_vp, _vp, ctypes.POINTER(ctypes.c_float)]),
    "ddm_event_record": (ctypes.c_int, [_vp, _vp]),
    "ddm_stream_create_cu_stride": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, _vp, _pi32]),
    "ddm_forest_predict_dev_orig": (ctypes.c_int, [_vp, _vp, ctypes.c_int32, ctypes.c_int32, _i64, _vp, _i64, _vp,
                                                   _vp, ctypes.c_uint32, _vp, _vp]),
    "ddm_stream_cu_count": (ctypes.c_int, [_vp, _pi32]),
    "ddm_stream_destroy": (ctypes.c_int, [_vp]),
    "ddm_event_synchronize": (ctypes.c_int, [_vp]),
    "ddm_mt_perms": (ctypes.c_int, [_vp, _pi32, _vp, _i64, _vp, _vp]),
    "ddm_mt_randint31": (ctypes.c_int, [_vp, _pi32, _i64, _vp]),
    "ddm_mt_skip": (ctypes.c_int, [_vp, _pi32, _i64]),
    "ddm_mt_seed": (ctypes.c_int, [ctypes.c_uint32, _vp, _pi32]),
    "ddm_forest_compile": (ctypes.c_int, [_vp, _i32, _vp, _i32, _vp, _i32, _i32, _vp, _i64,
                                          ctypes.POINTER(ctypes.c_int64)]),
    "ddm_rf_fit_many": (ctypes.c_int, [_vp, _i32, _i32]),
    "ddm_epoch_stage": (ctypes.c_int, [_vp, _i32, _vp]),
    "ddm_rf_device_scratch_bytes": (_i64, [_i32, _i32, _i32, _i32]),
    "ddm_rf_fit_device": (ctypes.c_int, [_vp, _i32, _i32, _vp]),
    "ddm_rf_fit_device_lf": (ctypes.c_int, [_vp, _i32, _i32, _i64, _vp]),
    "ddm_words_perm_seeds": (ctypes.c_int, [_vp, _i64, _i32, _i32, _vp, _vp, _vp]),
    "ddm_rf_fit": (ctypes.c_int, [_vp, _i32, _i32, _vp, _i32, _vp, _i32, _i32, _vp, _i64, _vp, _vp, _i64, _vp]),
    "ddm_synth_block_labels": (ctypes.c_int, [_vp, _i64, _i64, _i64, _i64, _i32, _vp]),
    "ddm_synth_jitter_labels": (ctypes.c_int, [_vp, _i64, _i64, _i64, _i64, _i64, _i32, ctypes.c_double, _u64,
                                               _vp]),
    "ddm_synth_features": (ctypes.c_int, [_vp, _i64, _i32, _vp, _i64, _i64, _i64, _u64, _f32, _vp]),
    "ddm_synth_bernoulli_streams": (ctypes.c_int, [_vp, _i64, _i64, _u64, _vp]),
}


class DdmError(RuntimeError):
    pass


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is not built; run `python __graft_entry__.py` (build) or "
                          f"`make -C distributed-drift-detection_amd/csrc` first")
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype, fn.argtypes = res, args
    if lib.ddm_abi_version() != ABI_VERSION:
        raise ImportError(f"libddm_amd.so ABI {lib.ddm_abi_version()} != {ABI_VERSION}")
    if lib.ddm_epoch_struct_bytes() != ctypes.sizeof(DdmEpoch):
        raise ImportError("ddm_epoch layout differs from the ctypes binding")
    if lib.ddm_ctl_epoch_bytes() != ctypes.sizeof(DdmCtlEpoch):
        raise ImportError("ddm_ctl_epoch layout differs from the ctypes binding")
    return lib


lib = _load()


def check(rc, what):
    if rc != 0:
        msg = lib.ddm_last_error().decode(errors="replace")
        raise DdmError(f"{what} failed (code {rc}): {msg}")
