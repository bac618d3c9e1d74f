"""Partition controller — the MI355X drop-in for `run_DDM_loop` (DDM_Process.py:166-213).

Reference semantics (per partition, one global numpy MT19937):
  batches of PER_BATCH rows, last one short (:182-184); batch 0 shuffled -> training
  batch (:187); for every later batch: shuffle (:190), refit if flagged (:194-196),
  predict (:199), DDM with carried state (:202), record first warning / first change
  (:147-152, :204); on a change the shuffled batch becomes the training batch, the DDM
  is dropped, refit flagged (:207-210); `pd.concat` of the per-batch rows (:212).

MI355X execution: the partition lives in HBM (columnar float32 features, int32
labels) together with its MT19937 stream (shuffle.py: raw draws + interval-FSM tables).
Between two refits nothing the host does depends on the rows, so the controller
speculates: for the next W batches it generates the batch shuffles on the device
(ddm_shuffle_window), runs the forest-predict kernel over all W batches in DDM order
(writing the error bytes and the first error position) and the DDM-scan kernel over
them (stopping at the first change, reporting event rows through the shuffle), and
reads back one 128-byte control block.  No drift: the DDM state carries, W doubles.
Drift in batch d: events up to d are final, the RNG position becomes the draw after
batch d's shuffle (where the reference's next iteration continues), the next batch's
shuffle and the refit's 100 tree seeds are read from the stream on the host, the
forest is refit natively on batch d, and the next window starts at d+1.  Work past d
is discarded, so total predict work stays within ~2x the rows.
"""
import ctypes
import os
import time

import numpy as np
import pandas as pd
import torch

from . import dfit, kernels
from .devctl import FlagTimeout
from ._capi import DDM_STOP_FAILED, DdmEpoch, check, lib
from .forest import upload_forests
from .params import OUTPUT_COLUMNS, DDMSettings, infer_x_features
from .rng import MTStream
from .shuffle import (CHUNK, GEN_STATE_BYTES, JUMP_BYTES, GpuShuffle, expected_draws_per_batch, fy_from_words,
                      perm_seeds_from_words, table_bytes_per_chunk, untemper_keys)
from .trainer import BatchForestTrainer

# A window runs on ddm_scan_long when its carried detector is neither fresh nor trivial
# (every row of it is exact arithmetic) and it spans at least this many rows.
LONG_SCAN_MIN_ROWS = int(os.environ.get("DDM_LONG_SCAN_ROWS", 4 * 64 * 100))
# Device-resident epochs (devctl.py) by default; DDM_DEVICE_CTL=0 keeps every epoch on the host path.
# DDM_DEVICE_START=0: the first epoch (first fits on the host) stays host-planned.
DEVICE_CTL = os.environ.get("DDM_DEVICE_CTL", "1") not in ("", "0")
DEVICE_START = os.environ.get("DDM_DEVICE_START", "1") not in ("", "0")


def carried_exact(st):
    """A carried ddm_state whose next rows all need the exact recurrence: not fresh (or
    pending a reset) and not the trivial all-zero state (det.h det_fresh / det_trivial)."""
    if st["in_concept_change"]:
        return False
    fresh = (st["sample_count"] == 1 and st["miss_prob"] == 1.0 and st["miss_std"] == 0.0
             and np.isinf(st["miss_prob_sd_min"]))
    trivial = (st["miss_prob"] == 0.0 and st["miss_prob_sd_min"] == 0.0 and st["miss_prob_min"] == 0.0
               and st["miss_sd_min"] == 0.0)
    return not (fresh or trivial)


# Largest piece of a partition's MT19937 stream generated per side-stream launch: an epoch
# waits only for the piece holding the draws it reads, so the generator (one sequential
# recurrence per partition) runs ahead of the epochs instead of holding them to its end.
GEN_PIECE_MAX = int(os.environ.get("DDM_GEN_PIECE", 1 << 25))
# the smallest piece after the first: a piece's latency (jumps, one <= 2^20-draw segment per
# workgroup, its tables) hardly depends on its size, so the doubling starts at 8M draws
# (C3: the first ~25 epochs waited for pieces of 1M, 2M, 4M ... one after the other)
GEN_PIECE_MIN = int(os.environ.get("DDM_GEN_PIECE_MIN", 1 << 23))
# _enqueue_rest calls (two pieces each) right behind the first piece, before the host's
# run-start work (the head read-back, batch 0's shuffles, the device first fit, ~2.5 ms of
# host time with the GPU otherwise idle): C3 56.0 / 56.7 / 56.4 -> 54.9 / 54.8 / 55.1 ms
# per step (the same box, alternating)
EARLY_PIECES = int(os.environ.get("DDM_EARLY_PIECES", "1"))
# The side stream (the next windows' shuffles, beside the refits and the next predict) on
# every SIDE_CU_STRIDE-th CU only (ddm_stream_create_cu_stride; 1: all CUs): its fused replay
# holds ~17 KB of LDS per one-wave workgroup, so on every CU it left no room for the
# predict's workgroups, which then ran at 0.50 of HBM instead of 0.71.  Note for reading the
# A/B in profiles/r05/refit: a CU-masked stream (hipExtStreamCreateWithCUMask) is a blocking
# stream at normal priority, while the stream it replaces is a non-blocking torch stream at
# priority -1, so stride > 1 changes the mask, the priority and the null-stream sync at once.
# Round 6 (tools/cu_probe.hip): the MI355X pool's runtime does not apply the CU mask at all
# (a stride-2 / 4 / 8 stream's workgroups ran on all 256 CUs), so those A/Bs measured the
# priority and sync change only.
SIDE_CU_STRIDE = int(os.environ.get("DDM_SIDE_CU_STRIDE", "1"))


class _Done:
    """An already computed result with a Future's result() (the small-output fills)."""
    __slots__ = ("value",)

    def __init__(self, value):
        self.value = value

    def result(self):
        return self.value


def _round_up(n, m):
    return (n + m - 1) // m * m


def ps_feats(part):
    return part.X.shape[0]


def _int_labels(y):
    """Labels as int64, refusing what the device path cannot reproduce: non-integer values
    (the reference compares y_pred != y on the raw labels, DDM_Process.py:117) and values
    outside int32."""
    y = np.asarray(y)
    if y.dtype.kind == "f":
        if not np.isfinite(y).all() or not np.array_equal(y, np.floor(y)):
            raise ValueError("labels must be integers on the device path (non-integer or NaN targets)")
    elif y.dtype.kind not in "iub":
        raise ValueError(f"labels must be integers on the device path (dtype {y.dtype})")
    if y.size and (y.min() < np.iinfo(np.int32).min or y.max() > np.iinfo(np.int32).max):
        raise ValueError("labels must fit int32 on the device path")
    return y.astype(np.int64)


class DevicePartition:
    """One partition's rows resident in HBM: X float32 [F, ld] (column f contiguous), y int32."""

    def __init__(self, X, y, n_rows, host_X32=None, host_y=None):
        assert X.dtype == torch.float32 and y.dtype == torch.int32 and X.shape[1] == y.shape[0]
        self.X, self.y, self.n = X, y, int(n_rows)
        self.device = X.device
        self.host_X32, self.host_y = host_X32, host_y

    @classmethod
    def allocate(cls, n_rows, n_features, device):
        ld = max(64, _round_up(n_rows, 64))
        X = torch.empty((n_features, ld), dtype=torch.float32, device=device)
        y = torch.zeros(ld, dtype=torch.int32, device=device)
        return cls(X, y, n_rows)

    @classmethod
    def from_arrays(cls, X32, y, device, stream=None):
        """X32: [n, F] float32 host rows (the float32 cast sklearn applies), y: int labels."""
        X32 = np.ascontiguousarray(X32, dtype=np.float32)
        y = _int_labels(y)
        n, F = X32.shape
        part = cls.allocate(n, F, device)
        with torch.cuda.stream(stream or torch.cuda.current_stream(device)):
            if n:
                part.X[:, :n].copy_(torch.from_numpy(np.ascontiguousarray(X32.T)))
                part.y[:n].copy_(torch.from_numpy(y.astype(np.int32)))
        part.host_X32, part.host_y = X32, y.astype(np.int64)
        return part

    @classmethod
    def from_columns(cls, Xc, y, device, stream=None):
        """Xc: float32 [F, n] columnar host array (loader.PartitionArrays.X32), y: int labels."""
        Xc = np.asarray(Xc, dtype=np.float32)
        y = _int_labels(y)
        F, n = Xc.shape
        part = cls.allocate(n, F, device)
        with torch.cuda.stream(stream or torch.cuda.current_stream(device)):
            if n:
                part.X[:, :n].copy_(torch.from_numpy(np.ascontiguousarray(Xc)))
                part.y[:n].copy_(torch.from_numpy(y.astype(np.int32)))
        part.host_X32, part.host_y = np.ascontiguousarray(Xc.T), y.astype(np.int64)
        return part

    def rows(self, rows, stream):
        """Training rows (features float32 [k, F], labels int64) in the given order."""
        if self.host_X32 is not None:
            return self.host_X32[rows], self.host_y[rows]
        idx = torch.from_numpy(np.asarray(rows, dtype=np.int64)).to(self.device, non_blocking=False)
        with torch.cuda.stream(stream):
            xs = self.X.index_select(1, idx).t().contiguous().cpu().numpy()
            ys = self.y.index_select(0, idx).cpu().numpy().astype(np.int64)
        return xs, ys


def sklearn_refit(settings):
    """train_rf (DDM_Process.py:98-105) with sklearn itself: fit(X32, y, np_state) where
    np_state is numpy's global-RNG state at the refit (its 100 tree seeds come from it)."""
    from sklearn.ensemble import RandomForestClassifier

    from .treepack import pack_sklearn

    def refit(X32, y, np_state):
        rs = np.random.RandomState()
        rs.set_state(np_state)
        rf = RandomForestClassifier(n_estimators=settings.n_estimators, n_jobs=settings.cores, random_state=rs)
        rf.fit(X32, y)
        return pack_sklearn(rf)

    return refit


class RunStats:
    __slots__ = ("epochs", "refits", "predicted_rows", "refit_s", "gpu_s", "host_s", "predict_ms", "predict_bytes",
                 "scan_ms", "scan_rows", "shuffle_ms", "sklearn_refits", "refit_fit_s", "refit_readback_s",
                 "prep_s", "dfit_ms", "device_refits", "long_scans", "preshuffled", "device_epochs", "device_phases",
                 "permute_rows", "device_rows", "predict_dev_ms", "predict_dev_launches", "device_predict_bytes",
                 "flag_recoveries", "jump_ms", "jumps", "jump_bytes", "generate_ms", "generate_draws",
                 "generate_bytes", "tables_ms", "tables_chunks", "tables_bytes")

    def __init__(self):
        self.epochs = self.refits = self.predicted_rows = self.predict_bytes = self.scan_rows = 0
        self.sklearn_refits = self.device_refits = self.long_scans = self.preshuffled = 0
        self.device_epochs = self.device_phases = self.permute_rows = self.device_rows = 0
        self.flag_recoveries = 0       # runs redone with event-ordered fork / join (devctl.FlagTimeout)
        self.predict_dev_ms, self.predict_dev_launches, self.device_predict_bytes = 0.0, 0, 0
        self.refit_s = self.gpu_s = self.host_s = self.predict_ms = self.scan_ms = self.shuffle_ms = 0.0
        self.refit_fit_s = self.refit_readback_s = self.prep_s = self.dfit_ms = 0.0
        # the stream generation's batched launches (_ensure_all), HIP events around each on its
        # own stream while kernel timing is on: time, units, algorithmic bytes per kind
        self.jump_ms = self.generate_ms = self.tables_ms = 0.0
        self.jumps = self.jump_bytes = self.generate_draws = self.generate_bytes = 0
        self.tables_chunks = self.tables_bytes = 0

    def as_dict(self):
        return {k: getattr(self, k) for k in self.__slots__}


class _Part:
    """Host-side epoch state of one partition in a BatchRunner."""
    __slots__ = ("i", "nb", "last_len", "n_full", "max_win", "base", "ev_base", "j", "P", "retrain", "train_rows",
                 "state", "win", "forest", "out", "done", "P_after_first", "g0", "b_end", "Wg", "tail",
                 "P_tail_after", "seg_start", "pb", "staged", "rng_rows", "words0", "ev", "P_seeds")

    def blen(self, b):
        return self.last_len if b == self.nb - 1 else self.pb

    def b_end_is_tail(self, pb):
        """This epoch's window reaches a short last batch (shuffled on the host); g0 must
        already be this epoch's first GPU-shuffled batch."""
        b_end = min(self.nb, self.j + min(self.win, self.max_win))
        return b_end == self.nb and self.last_len != pb and self.nb - 1 >= self.g0


_HOST_TRACE = os.environ.get("DDM_HOST_TRACE", "") not in ("", "0")
_FRESH = kernels.fresh_states(1)[0]
_FRESH1 = kernels.fresh_states(1)


class BatchRunner:
    """Runs the speculative shuffle+predict+scan epochs of many partitions in lockstep on
    one HIP stream: each epoch is ONE batched shuffle launch (csrc/shuffle.hip job table),
    ONE batched forest-predict launch per kernel variant (segment table), ONE scan launch
    (a lane per partition) and ONE control-block read-back, whatever the partition count.
    Partitions are independent (DDM_Process.py:226 groups by device_id), so a partition
    that is done simply drops out of the tables.

    refit: "device" (ddm_rf_fit_device: the refit after a change runs on the GPU in the
    same epoch, on the rows, labels and seeds the staging kernel gathered; trees
    identical to the host trainer's), "native" (ddm_rf_fit_many, identical trees to
    sklearn 1.7.2, on host threads) or "sklearn".  A device refit that reports a status
    (NaN rows, more classes than its buffers hold) and the first fit of every partition
    go through "native"; NaN inputs go to sklearn itself.  The native refits of all
    partitions that drifted in an epoch are one call: every tree on a pool of
    `fit_threads` host threads."""

    def __init__(self, parts, settings=None, stream=None, refit="device", timing=False, fit_threads=8,
                 gen_stream=None, tab_stream=None, device_ctl=None):
        self.parts = list(parts)
        if not self.parts:
            raise ValueError("no partitions")
        dev = self.parts[0].device
        if any(p.device != dev for p in self.parts):
            raise ValueError("a BatchRunner drives the partitions of one device")
        self.device = dev
        self.s = settings or DDMSettings()
        self.stream = stream or torch.cuda.Stream(dev, priority=-1)   # epochs ahead of the generation
        self.refit_kind = refit
        self.fit_threads = max(1, int(fit_threads))
        pb = self.s.per_batch
        if not 2 <= pb <= 256:
            raise ValueError("per_batch must be in [2, 256] on the device path")
        self.batch_trainer = BatchForestTrainer(self.s.n_estimators, self.fit_threads)
        self.words_h = None
        self.sk_refit = sklearn_refit(self.s)
        self.timing = timing
        # HIP events recorded by the C-ABI right around each batched launch
        self.t_pred = kernels.LaunchTimer() if timing else None
        self.t_scan = kernels.LaunchTimer() if timing else None
        self.t_shuf = kernels.LaunchTimer() if timing else None
        # when a list: every predict launch's segment table is kept (replay_predict)
        self.predict_log = None
        self.params = kernels.params_struct(self.s.min_num_instances, pb, self.s.warning_level,
                                            self.s.out_control_level)
        n = len(self.parts)
        # partition p's DDM positions live at [base_p, base_p + n_p) of the shared perm/err
        # buffers (base_p a multiple of 16*pb, so batches and 16-byte scan chunks align)
        align = 16 * pb
        self.bases, self.ev_bases, self.max_wins, self.nbs = [], [], [], []
        pos = evp = 0
        for part in self.parts:
            nb = (part.n + pb - 1) // pb
            mw = max(1, min(self.s.max_window_batches, nb))
            self.bases.append(pos)
            self.ev_bases.append(evp)
            self.max_wins.append(mw)
            self.nbs.append(nb)
            pos = _round_up(pos + part.n, align) + align
            evp += mw + (mw & 1)                # even: every partition's event rows start 16-byte aligned
        self.perm_all = torch.zeros(pos + 256, dtype=torch.uint8, device=dev)
        self.err_all = torch.zeros(pos + 32, dtype=torch.uint8, device=dev)
        self.ev_total = evp
        self.ev_d = torch.empty((evp, 2), dtype=torch.int32, device=dev)
        self.ev_h = torch.empty((evp, 2), dtype=torch.int32, pin_memory=True)
        # control block, struct-of-arrays over partitions: outputs first, then inputs
        k = _round_up(n, 2)
        self.o_first, self.o_nev, self.o_stop, self.o_pick = 0, 8 * k, 16 * k, 20 * k
        self.o_off, self.o_end, self.o_bbase, self.o_state = 28 * k, 36 * k, 44 * k, 52 * k
        # one slab holds the control block, the shuffle-job and staging tables and the
        # staging outputs: an epoch is one host->device copy of [0, o_stage) and one
        # device->host copy of the whole slab
        F = max(p.X.shape[0] for p in self.parts)
        self.n_words = max(3 * pb + self.s.n_estimators + 64, 1024)   # >= the stage kernel's LDS words
        self.max_events = 64
        # ranges of the partitions routed to ddm_scan_long this epoch (empty for the others)
        self.o_loff, self.o_lend = 108 * k, 116 * k
        # shuffle-job tables: the epoch's windows (the pick reads them), a copy without the
        # windows the previous epoch shuffled already, and the next windows the staging
        # plans (one slot per partition, written by the device)
        jb = _round_up(n * kernels.JOB_DTYPE.itemsize, 256)
        self.o_jobs = _round_up(self.o_lend + 8 * k, 256)
        self.o_sjobs = self.o_jobs + jb
        self.o_njobs = self.o_sjobs + jb
        self.o_stage_tab = self.o_njobs + jb
        self.o_dfit_tab = self.o_stage_tab + _round_up(n * kernels.STAGE_DTYPE.itemsize, 256)
        self.o_stage = self.o_dfit_tab + _round_up(n * dfit.DFIT_DTYPE.itemsize, 256)
        sz = {"x": 4 * 256 * F, "y": 4 * 256, "w": 4 * self.n_words, "info": 64, "ev": 12 * self.max_events,
              "seeds": 8 * self.s.n_estimators, "dfit": 8 * dfit.RESULT_WORDS, "plan": 48}
        self.stage_off, self.stage_stride = {}, {}
        o = self.o_stage
        for key, nbytes in sz.items():
            self.stage_off[key] = o
            self.stage_stride[key] = _round_up(nbytes, 256)
            o += self.stage_stride[key] * n
        self.ctrl_bytes = o
        self.ctrl_h = torch.zeros(self.ctrl_bytes, dtype=torch.uint8, pin_memory=True)
        self._views = {}
        a = self.stage_off["info"]
        self._info_all = np.lib.stride_tricks.as_strided(      # every partition's staging info
            self.ctrl_h.numpy()[a:a + self.stage_stride["info"] * n].view(np.int64), shape=(n, 7),
            strides=(self.stage_stride["info"], 8), writeable=False)
        a = self.stage_off["plan"]
        self._plan_all = np.lib.stride_tricks.as_strided(      # every partition's next-window plan
            self.ctrl_h.numpy()[a:a + self.stage_stride["plan"] * n].view(np.int64), shape=(n, 6),
            strides=(self.stage_stride["plan"], 8), writeable=False)
        self.ctrl_d = torch.zeros(self.ctrl_bytes, dtype=torch.uint8, device=dev)
        c = self.ctrl_h.numpy()
        self.first_h = c[self.o_first:self.o_first + 8 * n].view(np.int64)
        self.nev_h = c[self.o_nev:self.o_nev + 8 * n].view(np.int64)
        self.stop_h = c[self.o_stop:self.o_stop + 4 * n].view(np.int32)
        self.pick_h = c[self.o_pick:self.o_pick + 8 * n].view(np.int64)
        self.off_h = c[self.o_off:self.o_off + 8 * n].view(np.int64)
        self.end_h = c[self.o_end:self.o_end + 8 * n].view(np.int64)
        self.bbase_h = c[self.o_bbase:self.o_bbase + 8 * n].view(np.int64)
        self.state_h = c[self.o_state:self.o_state + 56 * n].view(kernels.STATE_DTYPE)
        self.loff_h = c[self.o_loff:self.o_loff + 8 * n].view(np.int64)
        self.lend_h = c[self.o_lend:self.o_lend + 8 * n].view(np.int64)
        # long carried segments (a detector that is neither fresh nor trivial over a window
        # of >= LONG_SCAN_MIN_ROWS rows) run on ddm_scan_long instead of one lane
        self.long_max_rows = max(self.max_wins) * pb
        self.long_scratch = torch.empty(kernels.scan_long_scratch_size(n, self.long_max_rows, pb), dtype=torch.uint8,
                                        device=dev)
        self.t_long = kernels.LaunchTimer() if timing else None
        self.bbase_h[:] = self.ev_bases
        self.segs = kernels.PinnedTable(kernels.SEG_DTYPE, n, dev)
        self.jobs = kernels.PinnedTable(kernels.JOB_DTYPE, n, dev, self.ctrl_h[self.o_jobs:],
                                        self.ctrl_d[self.o_jobs:])
        self.sjobs = kernels.PinnedTable(kernels.JOB_DTYPE, n, dev, self.ctrl_h[self.o_sjobs:],
                                         self.ctrl_d[self.o_sjobs:])
        self.njobs = kernels.PinnedTable(kernels.JOB_DTYPE, n, dev, self.ctrl_h[self.o_njobs:],
                                         self.ctrl_d[self.o_njobs:])
        self.stage_jobs = kernels.PinnedTable(kernels.STAGE_DTYPE, n, dev, self.ctrl_h[self.o_stage_tab:],
                                              self.ctrl_d[self.o_stage_tab:])
        # device refits: per partition its output buffers and its (static) job record,
        # pointing at the partition's staging outputs; gated on a change with device seeds
        self.dfit_jobs = kernels.PinnedTable(dfit.DFIT_DTYPE, n, dev, self.ctrl_h[self.o_dfit_tab:],
                                             self.ctrl_d[self.o_dfit_tab:])
        self.dfit_bufs, self.dfit_rows = [], []
        if refit == "device":
            for i, part in enumerate(self.parts):
                b = dfit.RefitBuffers(pb, part.X.shape[0], self.s.n_estimators, 16, dev)
                info = self._sptr("info", i)
                self.dfit_bufs.append(b)
                self.dfit_rows.append(b.record(self._sptr("x", i), self._sptr("y", i), self._sptr("seeds", i),
                                               self._sptr("dfit", i), gate=info, gate2=info + 48))
        self.t_fit = kernels.LaunchTimer() if timing and refit == "device" else None
        # the partitions' MT19937 streams are generated and tabulated on a side stream, in
        # pieces, while the epochs run (GpuShuffle.wait_for orders the consumers)
        self.gen_stream = gen_stream or torch.cuda.Stream(dev)
        # tables on a stream of their own: the generator (8 workgroups, one sequential
        # recurrence per partition) never waits for a piece's tables before the next piece
        self.tab_stream = tab_stream or torch.cuda.Stream(dev)
        self.gen_tables = []
        # pinned staging per partition: [0] batch-j shuffle of a refit epoch, [1] short last
        # batch, [2] drift batch's shuffle read back
        self.small_h = [[torch.empty(256, dtype=torch.uint8, pin_memory=True) for _ in range(3)] for _ in self.parts]
        self.shuffles = []
        # stream capacity: the batch shuffles plus room for the refits' seeds (100 draws each;
        # a refit every 2.25 batches in C5 takes the stream to ~1.3x); device epochs need
        # every draw a window may ask for inside the buffers (they never regrow there)
        dev_ctl = (DEVICE_CTL if device_ctl is None else device_ctl) and refit == "device"
        # every partition's start-state rows (mt, seg0) in one device array, uploaded in one
        # copy per run from one pinned array (per-partition copies were ~20 us each)
        self.state_rows_d = torch.zeros((n, 2, 640), dtype=torch.int32, device=dev)
        self.state_rows_h = torch.zeros((n, 2, 640), dtype=torch.int32, pin_memory=True)
        for k, (part, nb, mw) in enumerate(zip(self.parts, self.nbs, self.max_wins)):
            cap = int(nb * expected_draws_per_batch(pb) * (1.45 if dev_ctl else 1.2)) + (128 if dev_ctl else 64) * 1024
            self.shuffles.append(GpuShuffle(dev, pb, cap, mw, self.stream, self.gen_stream, self.tab_stream,
                                            state_rows=self.state_rows_d[k]))
        self.stats = RunStats()
        self._gen_rest = None
        self._gen_evs = []            # (kind, begin, end, units, bytes) of timed generation launches
        self._forked = False          # the last epoch shuffled the next windows it planned
        self._pending_sync = False    # the last epoch's refit results are still on their way
        self._pending_forests = []
        self._E = self._epoch_desc()
        self.trace = [] if _HOST_TRACE else None     # (label, seconds since run start)
        # device-resident epochs (devctl.py): the epoch decisions on the device, epochs
        # enqueued ahead; the host path runs the first epoch and whatever the device hands back
        if device_ctl is None:
            device_ctl = DEVICE_CTL
        self.devctl = None
        if device_ctl and refit == "device":
            from .devctl import DeviceController
            self.devctl = DeviceController(self, LONG_SCAN_MIN_ROWS, min(4 * LONG_SCAN_MIN_ROWS, self.long_max_rows))

    def _mark(self, label):
        if self.trace is not None:
            self.trace.append((label, time.perf_counter() - self._t_run))

    # -- helpers
    def _dptr(self, off, i, size):
        return self.ctrl_d.data_ptr() + off + size * i

    def _sptr(self, key, i):
        return self.ctrl_d.data_ptr() + self.stage_off[key] + self.stage_stride[key] * i

    def _sview(self, key, i, dtype, count):
        """View of partition i's staging slot `key` in the pinned slab (memoised: the slab
        never moves)."""
        k = (key, i, dtype, count)
        v = self._views.get(k)
        if v is None:
            a = self.stage_off[key] + self.stage_stride[key] * i
            v = self._views[k] = self.ctrl_h.numpy()[a:a + np.dtype(dtype).itemsize * count].view(dtype)
        return v

    def _ensure_all(self, wants, wait=True):
        """wants: [(partition index, draws needed)].  Partitions whose enqueued stream falls
        short get one batched generate launch plus their tables on the side stream, closed
        by one event; then (wait=True) the epoch stream waits for what it will read."""
        reqs, tabs, jumps = [], [], []
        for i, upto in wants:
            sh = self.shuffles[i]
            if sh.chunks_for(upto) > sh.tab:
                req, need = sh.gen_request(upto, jumps)
                if len(req):
                    reqs.append(req)
                tabs.append((i, need))
        self._mark("requests")
        if jumps:
            # segment start states of every partition: one ddm_mt_jump launch
            rec = np.concatenate(jumps)
            jt = kernels.PinnedTable(kernels.JUMP_DTYPE, len(rec), self.device)
            jt.rec[:len(rec)] = rec
            e0 = self._gen_ev(self.gen_stream)
            kernels.mt_jump(jt, len(rec), self.gen_stream)
            self._gen_done(e0, "jump", self.gen_stream, len(rec), len(rec) * JUMP_BYTES)
            self.gen_tables.append(jt)
        self._mark("jumps")
        if reqs:
            reqs = np.concatenate(reqs)
            table = kernels.PinnedTable(kernels.GEN_DTYPE, len(reqs), self.device)   # read by the async copy
            table.rec[:len(reqs)] = reqs
            e0 = self._gen_ev(self.gen_stream)
            kernels.shuffle_generate_batch(table, len(reqs), self.gen_stream)
            draws = int(reqs["n"].sum())
            self._gen_done(e0, "generate", self.gen_stream, draws, 4 * draws + len(reqs) * GEN_STATE_BYTES)
            self.gen_tables.append(table)
        if tabs:
            g = torch.cuda.Event()
            g.record(self.gen_stream)
            self.tab_stream.wait_event(g)
            recs = []
            for i, need in tabs:
                self.shuffles[i].tables_to(need, recs)
            if recs:
                # every partition's new chunks: one ddm_shuffle_tables_batch launch
                tt = kernels.PinnedTable(kernels.TAB_DTYPE, len(recs), self.device)
                tt.rec[:len(recs)] = np.array(recs, dtype=kernels.TAB_DTYPE)
                e0 = self._gen_ev(self.tab_stream)
                kernels.shuffle_tables_batch(tt, len(recs), max(r[2] for r in recs), self.s.per_batch,
                                             self.tab_stream)
                chunks = sum(r[2] for r in recs)
                self._gen_done(e0, "tables", self.tab_stream, chunks, chunks * table_bytes_per_chunk(self.s.per_batch))
                self.gen_tables.append(tt)
            ev = torch.cuda.Event()
            ev.record(self.tab_stream)
            for i, _ in tabs:
                self.shuffles[i].mark_ready(ev)
        if wait:
            for i, upto in wants:
                self.shuffles[i].wait_for(upto)

    def _gen_ev(self, stream):
        """A timing event on `stream` ahead of a generation launch, while kernel timing is on."""
        if not self.timing or self.t_shuf is None:
            return None
        e = torch.cuda.Event(enable_timing=True)
        e.record(stream)
        return e

    def _gen_done(self, e0, kind, stream, units, nbytes):
        if e0 is None:
            return
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record(stream)
        self._gen_evs.append((kind, e0, e1, int(units), int(nbytes)))

    def _gen_collect(self):
        """Fold the drained generation launches' times and bytes into the stats."""
        st = self.stats
        for kind, e0, e1, units, nbytes in self._gen_evs:
            ms = e0.elapsed_time(e1)
            if kind == "jump":
                st.jump_ms += ms
                st.jumps += units
                st.jump_bytes += nbytes
            elif kind == "generate":
                st.generate_ms += ms
                st.generate_draws += units
                st.generate_bytes += nbytes
            else:
                st.tables_ms += ms
                st.tables_chunks += units
                st.tables_bytes += nbytes
        self._gen_evs = []

    def _upload_perm(self, i, b, perm, slot):
        pb = self.s.per_batch
        h = self.small_h[i][slot]
        h[:len(perm)].copy_(torch.from_numpy(perm))
        at = self.bases[i] + b * pb
        with torch.cuda.stream(self.stream):
            self.perm_all[at:at + len(perm)].copy_(h[:len(perm)], non_blocking=True)

    def _refit_prep(self, need):
        """Inputs of the refit of every partition in `need` on its drift batch (shuffled order).

        One read-back serves all of them: the stream words from each P (batch j's shuffle,
        then the T tree seeds, DDM_Process.py:190,:102) and the drift batches' rows; the
        native fits of all partitions run tree-parallel in one call (ddm_rf_fit_many) and
        the forests go back to HBM in one copy."""
        st, T, pb = self.stats, self.s.n_estimators, self.s.per_batch
        t0 = time.perf_counter()
        n_words = 3 * pb + T + 64
        if self.words_h is None or self.words_h.shape[0] < len(need):
            self.words_h = torch.empty((len(self.parts), n_words), dtype=torch.int32, pin_memory=True)
        rows_dev = []
        unstaged = [ps for ps in need if ps.staged is None]
        for ps in unstaged:
            if ps.words0 is None:
                self.shuffles[ps.i].ensure(ps.P + n_words)
        sync = False
        with torch.cuda.stream(self.stream):
            for k, ps in enumerate(need):
                if ps.staged is not None:           # everything came back with the epoch
                    rows_dev.append(None)
                    continue
                sh = self.shuffles[ps.i]
                if ps.words0 is None:
                    self.words_h[k].copy_(sh.R[ps.P:ps.P + n_words], non_blocking=True)
                    sync = True
                part = self.parts[ps.i]
                if part.host_X32 is None:
                    idx_h = torch.from_numpy(np.asarray(ps.train_rows, dtype=np.int64)).pin_memory()
                    idx = idx_h.to(self.device, non_blocking=True)
                    xh = torch.empty((len(idx_h), part.X.shape[0]), dtype=torch.float32, pin_memory=True)
                    yh = torch.empty(len(idx_h), dtype=torch.int32, pin_memory=True)
                    xh.copy_(part.X.t().index_select(0, idx), non_blocking=True)
                    yh.copy_(part.y.index_select(0, idx), non_blocking=True)
                    rows_dev.append((xh, yh, idx_h))
                    sync = True
                else:
                    rows_dev.append(None)
        self._enqueue_rest()                   # the first epoch: behind its refit inputs
        if sync:
            self.stream.synchronize()
        t1 = time.perf_counter()
        st.refit_readback_s += t1 - t0
        work = []
        for k, ps in enumerate(need):
            sh = self.shuffles[ps.i]
            if ps.staged is not None and isinstance(ps.staged[0], str):
                # refit on the GPU in the epoch that found the change (ddm_rf_fit_device)
                _, P1, P2, res = ps.staged
                ps.staged = None
                ps.P = P2
                ps.P_after_first = ps.P
                if res is None:                                 # the refit is still running
                    ps.forest = None
                    ps.P_seeds = P1
                    self._pending_forests.append(ps)
                else:
                    ps.forest = dfit.DeviceFitForest(self.dfit_bufs[ps.i], res)
                ps.retrain = False
                ps.state = kernels.fresh_states(1)              # ddm = None -> new DDM (:136-139)
                ps.g0 = ps.j + 1
                ps.seg_start = ps.j
                st.refits += 1
                st.device_refits += 1
                continue
            if ps.staged is not None and ps.staged[3] is not None:
                # batch j's shuffle is already in perm_all and the seeds came back staged
                seeds, P1, P2 = ps.staged[3], ps.staged[4], ps.staged[5]
            else:
                if ps.staged is not None:
                    words = ps.staged[2]
                elif ps.words0 is not None:
                    words, ps.words0 = ps.words0, None
                else:
                    words = self.words_h[k].numpy().view(np.uint32)
                L = ps.blen(ps.j)
                r = perm_seeds_from_words(words, L, T)
                if r is None:                                   # rejections ran past the read-back
                    permj, P1 = sh.host_perm(ps.P, L)
                    seeds, P2 = sh.host_seeds(P1, T)
                else:
                    permj, seeds = r[0], r[1]
                    P1 = ps.P + r[2]
                    P2 = P1 + r[3]
                self._upload_perm(ps.i, ps.j, permj, 0)         # batch_b.sample before the fit (:190, :194)
            P_seeds, ps.P = P1, P2                              # 100 tree seeds follow the shuffle
            ps.P_after_first = ps.P
            if ps.staged is not None:
                X32, y = ps.staged[0], ps.staged[1]
                ps.staged = None
            elif rows_dev[k] is None:
                X32, y = self.parts[ps.i].rows(ps.train_rows, self.stream)
            else:
                X32, y = rows_dev[k][0].numpy(), rows_dev[k][1].numpy().astype(np.int64)
            work.append((ps, X32, y, seeds, P_seeds))
            ps.g0 = ps.j + 1
            ps.seg_start = ps.j
        st.refit_s += time.perf_counter() - t0
        return work

    def _refit_fit(self, work):
        """The refits themselves (all partitions in one native call) and the forests' upload."""
        st = self.stats
        t0 = time.perf_counter()
        fits = [None] * len(work)
        if self.refit_kind in ("native", "device"):         # host refits of the device mode too
            t2 = time.perf_counter()
            fits = self.batch_trainer.fit_many([(X32, y, seeds) for _, X32, y, seeds, _ in work])
            st.refit_fit_s += time.perf_counter() - t2
        entries = []
        for (ps, X32, y, seeds, P_seeds), fit in zip(work, fits):
            if fit is None:                    # sklearn requested, or NaN in X (missing values)
                entries.append((self.sk_refit(X32, y, self.shuffles[ps.i].numpy_state(P_seeds)), None, None))
                st.sklearn_refits += 1
            else:
                entries.append(fit)
        forests = upload_forests(entries, self.device, self.stream)
        for (ps, *_), f in zip(work, forests):
            ps.forest = f
            ps.retrain = False
            ps.state = kernels.fresh_states(1)                  # ddm = None -> new DDM (:136-139)
        st.refits += len(work)
        st.refit_s += time.perf_counter() - t0

    def _pool(self):
        if getattr(self, "_executor", None) is None:
            from concurrent.futures import ThreadPoolExecutor
            self._executor = ThreadPoolExecutor(self.fit_threads)
        return self._executor

    def close(self):
        ex = getattr(self, "_executor", None)
        if ex is not None:
            ex.shutdown(wait=True)
            self._executor = None
        if getattr(self, "devctl", None) is not None:
            self.stream.synchronize()
            self.devctl.close()
        if getattr(self, "_side_raw", None) is not None:
            self.side_stream.synchronize()
            lib.ddm_stream_destroy(self._side_raw)
            self._side_raw = None

    # -- per-epoch tables: per-partition template records (the static fields), of which an
    #    epoch takes the live partitions' rows and sets the fields that move
    def _templates(self):
        if getattr(self, "_tmpl", None) is not None:
            return self._tmpl
        n, pb, T = len(self.parts), self.s.per_batch, self.s.n_estimators
        perm, err, ev = self.perm_all.data_ptr(), self.err_all.data_ptr(), self.ev_d.data_ptr()
        seg = np.zeros(n, dtype=kernels.SEG_DTYPE)
        stg = np.zeros(n, dtype=kernels.STAGE_DTYPE)
        job = np.zeros(n, dtype=kernels.JOB_DTYPE)
        for i, part in enumerate(self.parts):
            Xp, ld, yp, F = part.X.data_ptr(), part.X.shape[1], part.y.data_ptr(), part.X.shape[0]
            seg[i]["X"], seg[i]["ld"], seg[i]["y"], seg[i]["perm"], seg[i]["err"] = Xp, ld, yp, perm, err
            seg[i]["first_err"], seg[i]["row_base"] = self._dptr(self.o_first, i, 8), self.bases[i]
            seg[i]["flags"] = kernels.SEG_FIRST_ERR_PRESET
            r = stg[i]
            r["X"], r["ld"], r["y"], r["perm"], r["base"] = Xp, ld, yp, perm, self.bases[i]
            r["ev"], r["stop"], r["pick"] = ev + 8 * self.ev_bases[i], self._dptr(self.o_stop, i, 4), \
                self._dptr(self.o_pick, i, 8)
            r["nb"], r["pb"], r["last_len"], r["n_features"] = self.nbs[i], pb, part.n - (self.nbs[i] - 1) * pb, F
            r["n_words"], r["max_events"], r["n_trees"] = self.n_words, self.max_events, T
            r["win_rule"] = self.s.win_rule
            r["x_out"], r["y_out"], r["w_out"] = self._sptr("x", i), self._sptr("y", i), self._sptr("w", i)
            r["info_out"], r["ev_out"], r["perm_w"], r["seeds_out"] = self._sptr("info", i), self._sptr("ev", i), \
                perm, self._sptr("seeds", i)
            r["max_win"], r["n_full"], r["min_win"] = self.max_wins[i], self.nbs[i] - (1 if r["last_len"] != pb else 0), \
                self.s.min_window
            r["dpb_x1024"] = int(np.ceil(expected_draws_per_batch(pb) * 1024))
            r["plan_out"], r["next_job"] = self._sptr("plan", i), self.njobs.d.data_ptr() + i * kernels.JOB_DTYPE.itemsize
            sh = self.shuffles[i]
            q = job[i]
            q["pieces"], q["info"], q["J"], q["E"] = sh.pieces.data_ptr(), sh.info.data_ptr(), sh.J.data_ptr(), \
                sh.E.data_ptr()
            q["first"], q["pick_out"] = sh.first.data_ptr(), self._dptr(self.o_pick, i, 8)
            nj = self.njobs.rec[i]                       # the next-window slot (static fields)
            nj["pieces"], nj["info"], nj["J"], nj["E"], nj["first"] = q["pieces"], q["info"], q["J"], q["E"], q["first"]
            nj["W"] = 0
        self._tmpl = {"seg": seg, "stage": stg, "job": job, "forest": [None] * n, "ptrs": [None] * n,
                      "forest_view": seg[["nodes", "roots", "leaf_value", "classes", "n_trees", "n_classes", "n_nodes",
                                          "pure", "cforest", "cf_slots", "cf_vote_regs", "cf_leaves", "cf_tab_words"]],
                      "dfit": np.array(self.dfit_rows, dtype=dfit.DFIT_DTYPE) if self.dfit_rows else None,
                      "stop": np.array([self._dptr(self.o_stop, i, 4) for i in range(n)], dtype=np.uint64)}
        return self._tmpl

    def _stream_ptrs(self, live):
        """Refresh the R / table pointers of partitions whose stream buffers were regrown."""
        t = self._templates()
        for ps in live:
            p = self.shuffles[ps.i].ptrs
            if t["ptrs"][ps.i] is not p:
                t["ptrs"][ps.i] = p
                t["job"][ps.i]["R"], t["job"][ps.i]["Tpre"], t["job"][ps.i]["Tchunk"] = p
                t["stage"][ps.i]["R"] = p[0]
                nj = self.njobs.rec[ps.i]
                nj["R"], nj["Tpre"], nj["Tchunk"] = p
        return t

    def _segment_table(self, live):
        """ddm_predict_segment records (forest predict) of this epoch."""
        t = self._templates()
        seg = t["seg"]
        fv = t["forest_view"]
        for ps in live:
            if t["forest"][ps.i] is not ps.forest:          # a new forest: its descriptor fields
                t["forest"][ps.i] = ps.forest
                if isinstance(ps.forest, dfit.DeviceFitForest):
                    fv[ps.i] = ps.forest.seg_fields()
                else:
                    d = ps.forest.desc
                    fv[ps.i] = (d.nodes, d.roots, d.leaf_value or 0, d.classes, d.n_trees, d.n_classes, d.n_nodes,
                                d.pure, d.cforest or 0, d.cf_slots, d.cf_vote_regs, d.cf_leaves, d.cf_tab_words)
        idx = [ps.i for ps in live]
        rec = seg[idx]
        rec["pos_begin"] = [ps.rng_rows[0] for ps in live]
        rec["pos_end"] = [ps.rng_rows[1] for ps in live]
        self.segs.rec[:len(idx)] = rec

    def _stage_table(self, live):
        """ddm_stage_job records of this epoch (csrc/stage.hip)."""
        t = self._stream_ptrs(live)
        rec = t["stage"][[ps.i for ps in live]]
        rec["j"] = [ps.j for ps in live]
        rec["g0"] = [ps.g0 for ps in live]
        rec["b_end"] = [ps.b_end for ps in live]
        rec["p_after_first"] = [-1 if ps.P_after_first is None else ps.P_after_first for ps in live]
        rec["p_tail_after"] = [-1 if ps.P_tail_after is None else ps.P_tail_after for ps in live]
        rec["tail"] = [1 if ps.tail else 0 for ps in live]
        rec["p_now"] = [ps.P for ps in live]
        rec["win"] = [ps.win for ps in live]
        rec["seg_start"] = [ps.seg_start for ps in live]
        rec["next_avail"] = [self.shuffles[ps.i].waited * CHUNK for ps in live]
        self.stage_jobs.rec[:len(live)] = rec

    def _jobs_for(self, live, with_stop, upload=True):
        """Fill the job table for partitions with device shuffles this epoch."""
        t = self._stream_ptrs(live)
        pb = self.s.per_batch
        idx = [ps.i for ps in live]
        rec = t["job"][idx]
        rec["avail"] = [self.shuffles[ps.i].waited * CHUNK for ps in live]
        rec["P"] = [ps.P for ps in live]
        rec["W"] = [ps.Wg for ps in live]
        rec["perm_out"] = [self.perm_all.data_ptr() + self.bases[ps.i] + ps.g0 * pb for ps in live]
        if with_stop:
            rec["stop"] = t["stop"][idx]
            rec["pick_offset"] = [ps.g0 - ps.j for ps in live]
            rec["pick_last"] = [ps.b_end - 1 - ps.j for ps in live]
        else:                                # end of the window's GPU batches (tail epochs)
            rec["stop"] = 0
            rec["pick_offset"] = 0
            rec["pick_last"] = [ps.Wg - 1 for ps in live]
        self.jobs.rec[:len(idx)] = rec
        if upload:
            self.jobs.upload(len(live), self.stream)

    def replay_predict(self, repeats=1):
        """Launch the logged predict segment tables again back to back on the epoch stream
        (same inputs, same shapes), HIP events on that stream around all of them.  With the
        stream saturated the events time the kernels alone; in the epoch loop they also
        time the stream's idle gap before each launch.  Returns (ms per launch, launches)."""
        log = self.predict_log or []
        if not log:
            return 0.0, 0
        dev = [e for e in log if isinstance(e[0], str)]
        if dev:                                  # device-mode launches (devctl.py)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize(self.device)
            e0.record(self.stream)
            for _ in range(repeats):
                for e in dev:
                    self.devctl.replay(e, self.stream)
            e1.record(self.stream)
            e1.synchronize()
            n = repeats * len(dev)
            return e0.elapsed_time(e1) / n, n
        cap = max(k for _, k, _ in log)
        tabs = [kernels.PinnedTable(kernels.SEG_DTYPE, cap, self.device) for _ in log]
        for t, (rec, k, _) in zip(tabs, log):
            t.rec[:k] = rec
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(self.device)
        e0.record(self.stream)
        for _ in range(repeats):
            for t, (_, k, pb) in zip(tabs, log):
                kernels.forest_predict_batch(t, k, pb, self.stream)
        e1.record(self.stream)
        e1.synchronize()
        n = repeats * len(log)
        return e0.elapsed_time(e1) / n, n

    def run(self, rngs):
        """Returns, per partition, int64 [n_batches-1, 2]: partition rows of (first warning,
        change) per batch 1.. (-1 = none).  Consumes each `rngs[p]` (an MTStream, advanced
        in place) exactly as the reference consumes np.random in that partition's worker.

        A device phase whose cross-stream flag wait gave up (a hang guard, csrc/common.h
        flag_poll) is void: the run is redone from the callers' RNG states with the fork /
        join ordered by HIP events for the rest of the runner's life, so the results stay
        exact (stats.flag_recoveries counts it)."""
        if len(rngs) != len(self.parts):
            raise ValueError("one MT19937 stream per partition")
        snaps = [r.snapshot() for r in rngs]
        stats0 = {k: getattr(self.stats, k) for k in RunStats.__slots__}
        try:
            return self._run(rngs)
        except FlagTimeout as e:
            if self.devctl is None or not self.devctl.flags_ok:
                raise
            self._mark(f"flag timeout: {e}; run redone with event-ordered fork / join")
            for r, snap in zip(rngs, snaps):
                r.restore(snap)
            # the voided attempt's counts are dropped: the redo counts its own
            recoveries = self.stats.flag_recoveries + 1
            for k, v in stats0.items():
                setattr(self.stats, k, v)
            self.devctl.flags_off()
            self.stats.flag_recoveries = recoveries
            return self._run(rngs)

    def _run(self, rngs):
        s, st, pb = self.s, self.stats, self.s.per_batch
        self._t_run = time.perf_counter()
        self._gen_rest = None
        self._gen_evs = []
        self._forked = False
        self._pending_sync = False
        self._pending_forests = []
        if self.trace is not None:
            self.trace = []
        pss = []
        for i, part in enumerate(self.parts):
            ps = _Part()
            ps.pb = pb
            ps.words0 = None
            ps.i, ps.nb, ps.base, ps.ev_base, ps.max_win = i, self.nbs[i], self.bases[i], self.ev_bases[i], \
                self.max_wins[i]
            if ps.nb == 0:
                raise IndexError("list index out of range")       # batches[0] on an empty frame (:187)
            ps.last_len = part.n - (ps.nb - 1) * pb
            ps.n_full = ps.nb if ps.last_len == pb else ps.nb - 1
            pss.append(ps)
        # everything enqueued so far on the caller's stream (the partitions' rows, and the
        # fills of this runner's own zero-initialised buffers) happens before the runner's
        # streams touch them
        ready = torch.cuda.Event()
        ready.record(torch.cuda.current_stream(self.device))
        for s_ in (self.stream, self.gen_stream, self.tab_stream):
            s_.wait_event(ready)
        for s_ in (self.stream, self.gen_stream, self.tab_stream):   # nothing of the last run
            s_.synchronize()                                          # may still read the streams
        self._mark("streams idle")
        sr = self.state_rows_h.numpy().view(np.uint32)     # free: the streams are idle
        for ps, rng in zip(pss, rngs):
            self.shuffles[ps.i].reset(rng, synced=True, upload=False)
            sr[ps.i, :, :624] = rng.key
            sr[ps.i, :, 624] = int(rng.pos.value)
        with torch.cuda.stream(self.gen_stream):
            self.state_rows_d.copy_(self.state_rows_h, non_blocking=True)
        self._mark("MT states uploaded")
        started = []
        try:
            # each partition's whole stream up front (one batched generate + tables);
            # windows extend it if drifts (100 seed draws each) push it further
            # the whole stream of every partition, in growing pieces on the side stream: the
            # first epochs only wait for the first piece
            tp = time.perf_counter()
            self.gen_tables = []
            total = max(int(ps.nb * expected_draws_per_batch(pb) * 1.02) for ps in pss)
            upto = 1 << 19
            # the first words of every stream (batch 0's shuffle, then the first fit's seeds
            # and batch 1's shuffle) come back in ONE copy queued on the generation stream
            # right behind the first piece, ahead of the jumps and the later pieces
            n0 = max(64, 3 * pb) + 3 * pb + s.n_estimators + 64
            if getattr(self, "_head_h", None) is None or self._head_h.shape != (len(pss), n0):
                self._head_h = torch.empty((len(pss), n0), dtype=torch.int32, pin_memory=True)
            head_h = self._head_h            # free: the last run's copy into it has completed
            head_ev = None
            self._mark("head buffer")
            self._ensure_all([(ps.i, min(upto, int(ps.nb * expected_draws_per_batch(pb) * 1.02))) for ps in pss],
                             wait=False)
            with torch.cuda.stream(self.gen_stream):
                for k, ps in enumerate(pss):
                    head_h[k].copy_(self.shuffles[ps.i].R[:n0], non_blocking=True)
            head_ev = torch.cuda.Event()
            head_ev.record(self.gen_stream)
            # the rest of the streams (jumps, later pieces): the first pieces right away (the
            # GPU has nothing else to do while the host prepares the first epoch), the others
            # at the device phase's polls (_enqueue_rest)
            self._gen_rest = (upto, total, pss)
            for _ in range(EARLY_PIECES):
                self._enqueue_rest()
            if self.timing:
                st.prep_s += time.perf_counter() - tp
            self._mark("first piece + head copy enqueued")
            head_ev.synchronize()
            self._mark("head copy done")
            heads = head_h.numpy().view(np.uint32)
            for k, ps in enumerate(pss):
                # batches[0].sample (:187), natively (the Python loop took ~0.1 ms per partition
                # on the step's critical path)
                r = perm_seeds_from_words(heads[k, :n0 - (3 * pb + s.n_estimators + 64)], ps.blen(0), 0)
                ps.words0 = None
                if r is None:                                   # rejections ran past the read-back
                    perm0, ps.P = self.shuffles[ps.i].host_perm(0, ps.blen(0))
                else:
                    perm0, ps.P = r[0], r[2]
                    ps.words0 = heads[k, ps.P:ps.P + 3 * pb + s.n_estimators + 64].copy()
                started.append(ps)
                if ps.nb < 2:
                    raise ValueError("No objects to concatenate")  # pd.concat([]) (:212)
                ps.train_rows = perm0.astype(np.int64)
                ps.ev = []                       # (batch rows, column, positions) of every event
                ps.state = _FRESH1.copy()
                ps.forest, ps.retrain, ps.j, ps.done = None, True, 1, False
                ps.staged = None
                ps.win = max(1, s.window_batches)
                ps.seg_start = 1
            # the dense per-batch result (DDM_Process.py:212 concatenates one row per batch:
            # 1.25M rows per C3 partition) is filled with -1 on pool threads while the epochs
            # run (numpy releases the GIL for the fill); the events go in at the end
            # (small outputs are filled right here: a pool hand-off costs more than the fill)
            pool = self._pool()
            out_f = [pool.submit(np.full, (ps.nb - 1, 2), -1, np.int64) if ps.nb > 1 << 16 else
                     _Done(np.full((ps.nb - 1, 2), -1, np.int64)) for ps in pss]
            self._mark("batch-0 shuffles")
            host_epochs = 0
            if self.devctl is not None and DEVICE_START and self._device_start(pss):
                host_epochs = 1                  # straight into device epochs
                self._mark("device first fit enqueued")
            while True:
                live = [ps for ps in pss if not ps.done]
                if not live:
                    break
                if self.devctl is not None and host_epochs and self.devctl.eligible(live):
                    # device epochs until the partitions are done or need the host again
                    self.devctl.run_phase(live)
                    self._forked = False
                    host_epochs = 0
                    self._mark("device phase")
                    continue
                self._epoch(live)
                host_epochs += 1
            self._finish_pending()
            outs = []
            for ps, f in zip(pss, out_f):
                out = f.result()
                for r, c, v in ps.ev:
                    out[r, c] = v
                outs.append(out)
            self._mark("outputs")
            return outs
        finally:
            # every stream's numpy state after its last draw: one read-back for all
            plans = [(ps, self.shuffles[ps.i].state_plan(ps.P)) for ps in started]
            need = [(ps, start, pos) for ps, (start, pos) in plans if start is not None]
            states = {ps.i: pos for ps, (start, pos) in plans if start is None}
            if need:
                for ps, start, _ in need:
                    self.shuffles[ps.i].ensure(start + 624)
                if getattr(self, "_st_buf", None) is None or self._st_buf.shape[0] < len(need):
                    self._st_buf = torch.empty((len(self.parts), 624), dtype=torch.int32, pin_memory=True)
                buf = self._st_buf[:len(need)]     # free: the last run's copy into it has completed
                with torch.cuda.stream(self.stream):
                    # the windows of every stream gathered on the device: one copy back
                    buf.copy_(torch.stack([self.shuffles[ps.i].R[start:start + 624] for ps, start, _ in need]),
                              non_blocking=True)
                self.stream.synchronize()
                keys = untemper_keys(buf.numpy().view(np.uint32))
                for k, (ps, _, pos) in enumerate(need):
                    states[ps.i] = ("MT19937", keys[k], int(pos), 0, 0.0)
            for ps in started:
                ns = states[ps.i]
                rngs[ps.i].key[:] = ns[1]
                rngs[ps.i].pos.value = ns[2]
            self._mark("rng states")
            # pieces of the streams may still be generated / tabulated ahead on the side
            # streams: nothing may write into this runner's buffers once the caller can free them
            self.gen_stream.synchronize()
            self.tab_stream.synchronize()
            self._gen_collect()
            self._mark("side streams drained")

    def _device_start(self, pss):
        """The first fit of every partition on the device, so that the run starts in device
        epochs instead of a host-planned first epoch with host fits.  The reference draws
        batch 0's shuffle (DDM_Process.py:187, done on the host from the head words), batch
        1's shuffle and the first fit's 100 seeds (:190, :194-196, :102): exactly what the
        staging kernel draws after a change in a batch d, with d = 0 -- the training batch
        is batch 0 in shuffled order, batch d + 1 = 1 is shuffled, the seeds follow it.  So
        one ddm_epoch_stage launch with a change planted in batch 0 stages the rows, shuffle
        and seeds, the gated device refit runs on them, and every partition enters device
        mode with that refit pending (a refit that fails stalls to the host, which redoes it
        from the staged batch, as after any change).  False (nothing enqueued) when the host
        path must take the first epoch."""
        if not self.dfit_rows or len(pss) > len(self.parts):
            return False
        s, pb, T = self.s, self.s.per_batch, self.s.n_estimators
        plans = []
        for ps in pss:
            if ps.words0 is None or ps.nb < 2:
                return False
            r = perm_seeds_from_words(ps.words0, ps.blen(1), T)
            if r is None:                        # rejections ran past the head read-back
                return False
            plans.append((ps, ps.P + r[2], ps.P + r[2] + r[3]))
        self._mark("start: seeds drawn")
        n, stream = len(pss), self.stream
        t = self._stream_ptrs(pss)
        self._mark("start: stream pointers")
        rec = t["stage"][[ps.i for ps in pss]]
        rec["j"], rec["g0"], rec["b_end"] = 0, 1, 1
        rec["p_after_first"] = [ps.P for ps in pss]          # the draw after batch 0's shuffle
        rec["p_tail_after"], rec["tail"] = -1, 0
        rec["p_now"] = [ps.P for ps in pss]
        rec["win"] = [ps.win for ps in pss]
        rec["seg_start"] = 0
        rec["next_avail"] = [self.shuffles[ps.i].waited * CHUNK for ps in pss]
        rec["max_events"], rec["log"], rec["plan_out"], rec["next_job"] = 0, 0, 0, 0
        self.stage_jobs.rec[:n] = rec
        self.dfit_jobs.rec[:n] = self._templates()["dfit"][[ps.i for ps in pss]]
        self._mark("start: records")
        # batch 0's shuffle of every partition: one host->device copy and one scatter into
        # the partitions' perm arrays (eight separate copies took ~0.5 ms of the run start)
        key = tuple(ps.i for ps in pss)
        if getattr(self, "_p0", None) is None or self._p0[0] != key:
            idx = np.concatenate([self.bases[i] + np.arange(pb, dtype=np.int64) for i in key])
            self._p0 = (key, torch.empty((n, pb), dtype=torch.uint8, pin_memory=True),
                        torch.from_numpy(idx).to(self.device))
        _, p0_h, p0_idx = self._p0
        p0_h.numpy()[:] = np.stack([np.asarray(ps.train_rows, dtype=np.uint8) for ps in pss])
        self._mark("start: batch-0 perms staged")
        with torch.cuda.stream(stream):
            self.perm_all.index_copy_(0, p0_idx, p0_h.view(-1).to(self.device, non_blocking=True))
        self._mark("start: batch-0 perms uploaded")
        with torch.cuda.stream(stream):
            # the whole host half of the slab, as a host epoch uploads it: the device copy
            # must hold every static table field (the next-window jobs' stream pointers,
            # the batch bases, ...), since a device phase hands the slab back to the host
            # (ctrl_d -> ctrl_h) when it ends
            self.ctrl_d[:self.o_stage].copy_(self.ctrl_h[:self.o_stage], non_blocking=True)
            self.ctrl_d[self.o_stop:self.o_stop + 4 * len(self.parts)].zero_()   # a change in batch 0
        self._mark("start: slab uploaded")
        kernels.epoch_stage(self.stage_jobs, n, stream, upload=False)
        dfit.fit_device(self.dfit_jobs.d, n, T, stream, self._E.dfit_max_lf)
        for ps, P1, P2 in plans:
            ps.j, ps.seg_start, ps.retrain = 1, 1, True
            ps.staged = ("device", P1, P2, None)
            ps.words0 = None
        return True

    def _epoch_desc(self):
        """The ddm_epoch record of this runner (ddm_epoch_launch): the buffers never move, so
        every epoch only sets the counts and sizes."""
        E = DdmEpoch()
        base = self.ctrl_d.data_ptr()
        E.stream = self.stream.cuda_stream
        E.ctrl_d, E.ctrl_h = base, self.ctrl_h.data_ptr()
        E.upload_bytes, E.download_bytes = self.o_stage, self.ctrl_bytes
        E.shuffle_jobs, E.per_batch = self.jobs.d.data_ptr(), self.s.per_batch
        E.segs_h, E.segs_d = self.segs.h.data_ptr(), self.segs.d.data_ptr()
        E.err, E.offsets, E.ends = self.err_all.data_ptr(), base + self.o_off, base + self.o_end
        E.n_streams = len(self.parts)
        E.params = ctypes.addressof(self.params)
        E.state, E.first_nz, E.batch_base = base + self.o_state, base + self.o_first, base + self.o_bbase
        E.n_batches_total, E.ev_out = self.ev_total, self.ev_d.data_ptr()
        E.stop, E.nev, E.perm_map = base + self.o_stop, base + self.o_nev, self.perm_all.data_ptr()
        E.long_off, E.long_end, E.long_scratch = base + self.o_loff, base + self.o_lend, self.long_scratch.data_ptr()
        E.stage_jobs, E.dfit_jobs = self.stage_jobs.d.data_ptr(), self.dfit_jobs.d.data_ptr()
        E.max_trees = self.s.n_estimators
        E.next_jobs = self.njobs.d.data_ptr()
        self._side_raw = None
        if SIDE_CU_STRIDE > 1:
            raw, ncu = ctypes.c_void_p(), ctypes.c_int32()
            with torch.cuda.device(self.device):
                check(lib.ddm_stream_create_cu_stride(SIDE_CU_STRIDE, 0, ctypes.byref(raw), ctypes.byref(ncu)),
                      "ddm_stream_create_cu_stride")
            self._side_raw = raw
            self.side_cus = int(ncu.value)
            self.side_stream = torch.cuda.ExternalStream(raw.value, device=self.device)
        else:
            self.side_cus = None
            self.side_stream = torch.cuda.Stream(self.device, priority=-1)   # the next windows' shuffles
        E.side_stream = self.side_stream.cuda_stream
        self._fork_ev, self._join_ev = ctypes.c_void_p(), ctypes.c_void_p()
        check(lib.ddm_event_create_sync(ctypes.byref(self._fork_ev)), "ddm_event_create_sync")
        check(lib.ddm_event_create_sync(ctypes.byref(self._join_ev)), "ddm_event_create_sync")
        E.fork_ev, E.join_ev = self._fork_ev.value, self._join_ev.value
        if self.dfit_rows:
            # split read-back: the host works on the epoch while the refits run
            self._mid_ev = ctypes.c_void_p()
            check(lib.ddm_event_create(ctypes.byref(self._mid_ev)), "ddm_event_create")
            E.mid_ev = self._mid_ev.value
            E.dfit_max_lf = dfit.max_lf(self.s.per_batch, max(p.X.shape[0] for p in self.parts))
            E.tail_off = self.stage_off["dfit"]
            E.tail_bytes = self.stage_stride["dfit"] * len(self.parts)
        if self.timing:
            for k, t in enumerate((self.t_shuf, self.t_pred, self.t_scan, self.t_long, self.t_fit)):
                if t is not None:
                    E.ev[2 * k], E.ev[2 * k + 1] = t.ev[0].value, t.ev[1].value
        return E

    def set_kernel_timing(self, on):
        """HIP events around the epoch's launches (the kernel-time statistics) on or off.  Off,
        an epoch enqueues ten fewer HIP calls; the bench times its steps that way and takes
        the kernel times from an instrumented step of its own."""
        if not self.timing:
            return
        if not hasattr(self, "_timers"):
            self._timers = (self.t_shuf, self.t_pred, self.t_scan, self.t_long, self.t_fit)
        ts = self._timers if on else (None,) * 5
        self.t_shuf, self.t_pred, self.t_scan, self.t_long, self.t_fit = ts
        for k, t in enumerate(ts):
            self._E.ev[2 * k] = t.ev[0].value if t is not None else None
            self._E.ev[2 * k + 1] = t.ev[1].value if t is not None else None

    def set_predict_timing(self, on):
        """The device-clock span of every device-epoch predict launch (devctl.PredictTimer),
        read after each device phase into stats.predict_dev_ms / predict_dev_launches: the
        bench's in-step predict timing inside its timed region."""
        if self.devctl is None:
            return
        if on and self.devctl.pred_timer is None:
            from .devctl import PredictTimer
            self.devctl.pred_timer = PredictTimer(self.device)
        elif not on and self.devctl.pred_timer is not None:
            self.devctl.pred_timer.close()
            self.devctl.pred_timer = None

    def _next_bound(self, ps):
        """The largest window the epoch after this one can give partition ps (the policy of
        _epoch_after: 9/8 of the concept just closed after a change, twice the window
        otherwise)."""
        s = self.s
        lo = s.min_window
        return max(0, min(ps.max_win, ps.nb - ps.j,
                          max(lo, s.next_window(ps.b_end - ps.seg_start) + 1, 2 * ps.win)))

    def _enqueue_rest(self):
        """The partitions' whole streams, in growing pieces on the side streams (the first
        piece is enqueued by run())."""
        if self._gen_rest is None:
            return
        tp = time.perf_counter()
        upto, total, pss = self._gen_rest
        pb = self.s.per_batch
        # two pieces per epoch: the epochs' own coverage requests (_ensure_all with wait)
        # enqueue whatever a window needs first, so this only keeps generation ahead.
        # A piece's latency is one jump + one <= 2^20-draw segment per workgroup whatever its
        # size, so with fewer partitions on this GPU the pieces grow faster and larger (about
        # 256 segments per launch at most, the CUs' count): with one partition (N = 8) the
        # doubling from 1M left ~20 epochs waiting behind ~8 pieces one after the other
        # (profiles/r06/c3s8); with 8 (N = 1) the sizes are as before.
        grow = max(1, 8 // max(1, len(pss)))
        piece_max = max(GEN_PIECE_MAX, (256 << 20) // max(1, len(pss)))
        for _ in range(2):
            if upto >= total:
                break
            upto = min(total, upto + min(max(upto * grow, GEN_PIECE_MIN), piece_max))
            self._ensure_all([(ps.i, min(upto, int(ps.nb * expected_draws_per_batch(pb) * 1.02))) for ps in pss],
                             wait=False)
            self._mark(f"piece to {upto}")
        self._gen_rest = (upto, total, pss) if upto < total else None
        if self.timing:
            self.stats.prep_s += time.perf_counter() - tp

    def _epoch(self, live):
        s, st, pb, stream = self.s, self.stats, self.s.per_batch, self.stream
        t0 = time.perf_counter()
        refit_before = self.stats.refit_s
        need = [ps for ps in live if ps.retrain]
        for ps in live:
            ps.P_after_first = None
        self._mark("epoch")
        work = self._refit_prep(need) if need else []
        self._enqueue_rest()
        self._mark("refit prep")
        for ps in live:
            if ps not in need:
                ps.g0 = ps.j
        late_fit = bool(work) and not any(ps.b_end_is_tail(pb) for ps in live)
        if work and not late_fit:
            self._refit_fit(work)
        t1 = time.perf_counter()
        host = t1 - t0 - (self.stats.refit_s - refit_before)
        for ps in live:
            ps.b_end = min(ps.nb, ps.j + min(ps.win, ps.max_win))
            ps.Wg = max(0, min(ps.b_end, ps.n_full) - ps.g0)
            ps.tail = ps.b_end == ps.nb and ps.last_len != pb and ps.nb - 1 >= ps.g0
            ps.P_tail_after = None
        shuf = [ps for ps in live if ps.Wg]
        # windows the previous epoch shuffled already (the staging planned them on the
        # device and the executor ran them beside the refits): the plan must be this one
        pre = set()
        if self._forked and shuf:
            plans = self._plan_all.tolist()
            for ps in shuf:
                pl = plans[ps.i]
                if pl[5] == 1 and pl[0] == ps.P and pl[1] == ps.Wg and pl[2] == ps.g0:
                    pre.add(ps.i)
        # stream coverage: the window's shuffles, the words the staging reads after a change
        # (from at most the window's last draw), and the largest next window
        # (the next window's part stays inside the stream buffers: a window planned past
        # the tabulated draws is simply not pre-shuffled)
        nxt = {ps.i: self._next_bound(ps) for ps in live}
        wants = []
        for ps in live:
            sh = self.shuffles[ps.i]
            cur = ps.P + sh.window_draws(ps.Wg) + self.n_words
            wants.append((ps.i, max(cur, min(cur + sh.window_draws(nxt[ps.i]), sh.cap - 2 * CHUNK))))
        self._ensure_all(wants)
        rest = [ps for ps in shuf if ps.i not in pre]
        max_W = max_pieces = 0
        if rest:
            max_W = max(ps.Wg for ps in rest)
            max_pieces = max(2 + 64 + self.shuffles[ps.i].window_draws(ps.Wg) // 8192 for ps in rest)
        tails = [ps for ps in live if ps.tail]
        shuffled = False
        if tails:
            # the short last batch is shuffled on the host after the GPU batches before it
            if shuf:
                max_W = max(ps.Wg for ps in shuf)
                max_pieces = max(2 + 64 + self.shuffles[ps.i].window_draws(ps.Wg) // 8192 for ps in shuf)
                self._jobs_for(shuf, with_stop=False)
                kernels.shuffle_window_batch(self.jobs, len(shuf), max_W, max_pieces, pb, stream, self.t_shuf)
                kernels.shuffle_pick_batch(self.jobs, len(shuf), stream)
                with torch.cuda.stream(stream):
                    self.ctrl_h[self.o_pick:self.o_off].copy_(self.ctrl_d[self.o_pick:self.o_off], non_blocking=True)
                stream.synchronize()
                shuffled = True
            for ps in tails:
                P_tail = int(self.pick_h[ps.i]) + 1 if ps.Wg else ps.P
                permT, ps.P_tail_after = self.shuffles[ps.i].host_perm(P_tail, ps.last_len)
                self._upload_perm(ps.i, ps.nb - 1, permT, 1)
        # scan ranges and carried DDM states (the control block), segment table (predict)
        self.off_h[:] = 0
        self.end_h[:] = 0
        self.loff_h[:] = 0
        self.lend_h[:] = 0
        long_rows = 0
        for ps in live:
            p0 = ps.base + ps.j * pb
            p1 = ps.base + (ps.b_end - 1) * pb + ps.blen(ps.b_end - 1)
            ps.rng_rows = (p0, p1)
            self.off_h[ps.i], self.end_h[ps.i] = p0, p1
            # a refitting partition starts a fresh DDM (:136-139), whenever its fit runs
            self.state_h[ps.i] = _FRESH if ps.retrain else ps.state[0]
            if not ps.retrain and p1 - p0 >= LONG_SCAN_MIN_ROWS and carried_exact(ps.state[0]):
                self.loff_h[ps.i], self.lend_h[ps.i] = p0, p1
                self.end_h[ps.i] = p0            # nothing for the one-lane scan
                long_rows = max(long_rows, p1 - p0)
                st.long_scans += 1
        t2 = time.perf_counter()
        host += t2 - t1
        t1 = t2
        n = len(self.parts)
        base = self.ctrl_d.data_ptr()
        if shuf:
            self._jobs_for(shuf, with_stop=True, upload=False)
        self._stage_table(live)
        if self.dfit_rows:
            self.dfit_jobs.rec[:len(live)] = self._templates()["dfit"][[ps.i for ps in live]]
        self.first_h[:] = -1                    # the predict kernels' first-error slots
        native = not late_fit and not shuffled
        if native:
            # the whole epoch in one native call (csrc/epoch.hip)
            E = self._E
            E.pick_jobs, E.n_pick = self.jobs.d.data_ptr(), len(shuf)
            if pre and rest:                    # the shuffles skip the windows done already
                self.sjobs.rec[:len(shuf)] = self.jobs.rec[:len(shuf)]
                self.sjobs.rec["W"][[k for k, ps in enumerate(shuf) if ps.i in pre]] = 0
                E.shuffle_jobs = self.sjobs.d.data_ptr()
            else:
                E.shuffle_jobs = self.jobs.d.data_ptr()
            E.n_shuffle = len(shuf) if rest else 0
            E.max_W, E.max_pieces = max_W, max_pieces
            st.preshuffled += len(pre)
            # the next windows: planned by the staging, shuffled beside the refits
            live_ids = {ps.i for ps in live}
            self.njobs.rec["W"][[i for i in range(len(self.parts)) if i not in live_ids]] = 0
            E.n_next = len(self.parts)
            E.next_max_W = max(nxt.values())
            E.next_max_pieces = 2 + 64 + self.shuffles[live[0].i].window_draws(E.next_max_W) // 8192
            self._forked = True
        # the previous epoch's refits are needed from here on (their forests predict now)
        self._finish_pending()
        if not late_fit:
            self._segment_table(live)
        if native:
            E.n_segs = E.n_stage = len(live)
            E.long_max_rows = long_rows
            E.n_dfit = len(live) if self.dfit_rows else 0
            if self.predict_log is not None:
                self.predict_log.append((self.segs.rec[:len(live)].copy(), len(live), pb))
            self._mark("tables + upload")
            check(lib.ddm_epoch_launch(ctypes.byref(E)), "ddm_epoch_launch")
            self._mark("launched")
            if E.mid_ev:
                # everything but the refit results is back: the host goes on (this epoch's
                # events, the next epoch's tables) while the refits run
                check(lib.ddm_event_synchronize(E.mid_ev), "ddm_event_synchronize")
                self._mark("synchronized")
                self._pending_sync = True
                self._epoch_after(live, st, pb, E.n_shuffle > 0, long_rows, t1, host, deferred=True)
            else:
                stream.synchronize()
                self._mark("synchronized")
                self._epoch_after(live, st, pb, E.n_shuffle > 0, long_rows, t1, host)
            return
        self._forked = False
        with torch.cuda.stream(stream):
            self.ctrl_d[:self.o_stage].copy_(self.ctrl_h[:self.o_stage], non_blocking=True)
        if shuf and not shuffled:
            kernels.shuffle_window_batch(self.jobs, len(shuf), max_W, max_pieces, pb, stream, self.t_shuf)
        self._mark("tables + upload")
        if late_fit:
            # the window shuffles do not depend on the new forests: they run on the GPU
            # while the host fits them
            self._refit_fit(work)
            self._segment_table(live)
            self._mark("host fits")
        kernels.forest_predict_batch(self.segs, len(live), pb, stream, self.t_pred)
        if self.predict_log is not None:
            self.predict_log.append((self.segs.rec[:len(live)].copy(), len(live), pb))
        kernels.scan_streams_raw(self.err_all.data_ptr(), base + self.o_off, n, self.params, base + self.o_state,
                                 base + self.o_bbase, self.ev_total, self.ev_d.data_ptr(), base + self.o_first,
                                 base + self.o_stop, base + self.o_nev, 0, None, stream, self.t_scan,
                                 self.perm_all.data_ptr(), base + self.o_end)
        if long_rows:
            kernels.scan_long_raw(self.err_all.data_ptr(), base + self.o_loff, base + self.o_lend, n, long_rows,
                                  self.params, base + self.o_state, base + self.o_bbase, self.ev_d.data_ptr(),
                                  base + self.o_stop, base + self.o_nev, 0, self.perm_all.data_ptr(),
                                  self.long_scratch.data_ptr(), stream, self.t_long)
        if shuf:
            kernels.shuffle_pick_batch(self.jobs, len(shuf), stream)
        # stage what the host needs next, then one copy back and one synchronisation
        kernels.epoch_stage(self.stage_jobs, len(live), stream, upload=False)
        if self.dfit_rows:
            # the refits of the partitions that changed, on the rows the staging gathered
            if self.t_fit is not None:
                check(lib.ddm_event_record(self.t_fit.ev[0], ctypes.c_void_p(stream.cuda_stream)), "event record")
            dfit.fit_device(self.dfit_jobs.d, len(live), self.s.n_estimators, stream, self._E.dfit_max_lf)
            if self.t_fit is not None:
                check(lib.ddm_event_record(self.t_fit.ev[1], ctypes.c_void_p(stream.cuda_stream)), "event record")
        with torch.cuda.stream(stream):
            self.ctrl_h.copy_(self.ctrl_d, non_blocking=True)
        self._mark("launched")
        stream.synchronize()
        self._mark("synchronized")
        self._epoch_after(live, st, pb, bool(shuf), long_rows, t1, host)

    def _finish_pending(self):
        """The previous epoch's read-back of the refit results (split read-back): wait for
        it, then give the partitions whose refit ran on the device their forests (or, when
        a device refit reports a status, refit them on the host from the staged batch)."""
        if not self._pending_sync:
            return
        self.stream.synchronize()
        self._pending_sync = False
        self._mark("refits back")
        st = self.stats
        if self.timing and self.t_fit is not None:
            st.dfit_ms += self.t_fit.elapsed_ms()
        work = []
        for ps in self._pending_forests:
            res = self._sview("dfit", ps.i, np.int64, dfit.RESULT_WORDS)
            if int(res[0]) == 0:
                ps.forest = dfit.DeviceFitForest(self.dfit_bufs[ps.i], res.copy())
            else:                                   # refit on the host, same batch and seeds
                L = ps.blen(ps.j - 1)
                F_i = ps_feats(self.parts[ps.i])
                X32 = self._sview("x", ps.i, np.float32, L * F_i).reshape(L, -1).copy()
                y = self._sview("y", ps.i, np.int32, L).astype(np.int64)
                seeds = self._sview("seeds", ps.i, np.int64, self.s.n_estimators).copy()
                work.append((ps, X32, y, seeds, ps.P_seeds))
                st.refits -= 1
                st.device_refits -= 1
        self._pending_forests = []
        if work:
            self._refit_fit(work)

    def _epoch_after(self, live, st, pb, shuffled, long_rows, t1, host, deferred=False):
        """Everything after an epoch's read-back: timings, events, RNG positions, the next
        windows."""
        s, stream = self.s, self.stream
        if self.timing and self.t_pred is not None:
            st.predict_ms += self.t_pred.elapsed_ms()
            st.scan_ms += self.t_scan.elapsed_ms()
            if long_rows:
                st.scan_ms += self.t_long.elapsed_ms()
            if shuffled:
                st.shuffle_ms += self.t_shuf.elapsed_ms()
            if self.t_fit is not None and self.dfit_rows and not deferred:
                st.dfit_ms += self.t_fit.elapsed_ms()
        # the control block as Python ints, one conversion per array
        stops, nevs, picks = self.stop_h.tolist(), self.nev_h.tolist(), self.pick_h.tolist()
        if long_rows:
            bad = [ps.i for ps in live if stops[ps.i] == DDM_STOP_FAILED]
            if bad:
                raise RuntimeError(f"ddm_scan_long gave up waiting for a carried state (partitions {bad}): the "
                                   "epoch's results are void")
        infos = self._info_all.tolist()
        # read-backs beyond the staging (more events than it holds): rare
        pending = False
        for ps in live:
            stop, nev = stops[ps.i], nevs[ps.i]
            ps_last = ps.j + stop if stop >= 0 else ps.b_end - 1
            p0, p1 = ps.rng_rows
            st.predicted_rows += p1 - p0
            if self.timing:
                st.predict_bytes += (p1 - p0) * (4 * ps.forest.features_read + 6)
                st.scan_rows += min(p1, ps.base + (ps_last + 1) * pb) - p0
            if nev and infos[ps.i][2]:
                k, e0 = ps_last - ps.j + 1, ps.ev_base
                with torch.cuda.stream(stream):
                    self.ev_h[e0:e0 + k].copy_(self.ev_d[e0:e0 + k], non_blocking=True)
                pending = True
        if pending:
            stream.synchronize()
        t2 = time.perf_counter()
        st.gpu_s += t2 - t1
        st.epochs += 1
        for ps in live:
            stop, nev = stops[ps.i], nevs[ps.i]
            last = ps.j + stop if stop >= 0 else ps.b_end - 1
            info = infos[ps.i]
            if nev and info[2]:                     # overflowed the staging: full rows
                k, e0 = last - ps.j + 1, ps.ev_base
                ev = self.ev_h[e0:e0 + k].numpy()
                for c in range(2):
                    hit = np.nonzero(ev[:, c] >= 0)[0]
                    b = ps.j + hit
                    ps.ev.append((b - 1, c, b * pb + ev[hit, c].astype(np.int64)))
            elif nev:
                rec = self._sview("ev", ps.i, np.int32, 3 * self.max_events)[:3 * info[1]].tolist()
                for q in range(0, len(rec), 3):
                    b = ps.j + rec[q]
                    for c in range(2):
                        if rec[q + 1 + c] >= 0:
                            ps.ev.append((b - 1, c, b * pb + rec[q + 1 + c]))
            picked = picks[ps.i] if ps.Wg else -1
            # RNG position right after the last consumed batch shuffle
            if stop >= 0:
                d = ps.j + stop
                if d < ps.g0:
                    ps.P = ps.P_after_first              # drift in the refit batch: after its seeds
                elif ps.tail and d == ps.nb - 1:
                    ps.P = ps.P_tail_after
                else:
                    ps.P = picked + 1
                if info[0] != ps.P or info[3] != d:
                    raise RuntimeError(f"partition {ps.i}: staging disagrees (P {info[0]} vs {ps.P}, "
                                       f"batch {info[3]} vs {d})")
                L = ps.blen(d)
                drawn = info[6] == 1                # batch d+1's shuffle and the seeds, on the device
                res = self._sview("dfit", ps.i, np.int64, dfit.RESULT_WORDS) if self.dfit_rows else None
                if drawn and deferred and res is not None:
                    ps.staged = ("device", info[4], info[5], None)   # results after the next tables
                elif drawn and res is not None and int(res[0]) == 0:
                    ps.staged = ("device", info[4], info[5], res.copy())
                else:
                    F_i = ps_feats(self.parts[ps.i])
                    ps.staged = (self._sview("x", ps.i, np.float32, L * F_i).reshape(L, -1).copy(),
                                 self._sview("y", ps.i, np.int32, L).astype(np.int64),
                                 None if drawn else self._sview("w", ps.i, np.uint32, self.n_words).copy(),
                                 self._sview("seeds", ps.i, np.int64, self.s.n_estimators).copy() if drawn else None,
                                 info[4], info[5])
                ps.retrain = True
                # adaptive speculation: the next concept likely lasts about as long as this
                # one, so the next window covers it with a margin (one epoch per drift when
                # concepts repeat their length; windows still double after a miss)
                seg = d - ps.seg_start + 1
                ps.win = s.drift_window(seg)
                ps.j = d + 1
            else:
                if ps.tail:
                    ps.P = ps.P_tail_after
                elif ps.Wg:
                    ps.P = picked + 1
                elif ps.P_after_first is not None:
                    ps.P = ps.P_after_first
                ps.state = self.state_h[ps.i:ps.i + 1].copy()
                ps.j = ps.b_end
                ps.win *= 2
            if ps.j >= ps.nb:
                ps.done = True
        st.host_s += host + time.perf_counter() - t2


class GroupedRunner:
    """The partitions of one GPU in `groups` BatchRunners, each on its own epoch stream and
    driven by its own host thread, sharing the generation and table streams.  An epoch of
    one group is host work (refit inputs, window tables) and a chain of small kernels; with
    two groups the GPU runs one group's kernels while the host prepares the other's, and
    the two groups' small kernels run side by side.  Results are those of one BatchRunner
    over all partitions (partitions are independent, DDM_Process.py:226).

    Measured on one MI355X it does not pay where the GPU is the bottleneck: C3 141.6 ms
    (1 group) vs 147-171 ms (2), C5 at 8M rows 2.65 vs 1.97 M rows/s (each group runs as
    many epochs as the whole GPU did); the bench defaults to one group."""

    def __init__(self, parts, settings=None, groups=2, refit="device", timing=False, fit_threads=8):
        parts = list(parts)
        if not parts:
            raise ValueError("no partitions")
        dev = parts[0].device
        g = max(1, min(int(groups), len(parts)))
        # balance rows: partitions in decreasing size, each to the lightest group
        order = sorted(range(len(parts)), key=lambda k: -parts[k].n)
        self.members = [[] for _ in range(g)]
        load = [0] * g
        for k in order:
            t = load.index(min(load))
            self.members[t].append(k)
            load[t] += parts[k].n
        self.gen_stream, self.tab_stream = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
        self.runners = [BatchRunner([parts[k] for k in m], settings, torch.cuda.Stream(dev, priority=-1), refit,
                                    timing, max(1, fit_threads // g), self.gen_stream, self.tab_stream)
                        for m in self.members]
        from concurrent.futures import ThreadPoolExecutor
        self._pool = ThreadPoolExecutor(g) if g > 1 else None
        self.n = len(parts)

    def run(self, rngs):
        if len(rngs) != self.n:
            raise ValueError("one MT19937 stream per partition")
        jobs = [(r, [rngs[k] for k in m]) for r, m in zip(self.runners, self.members)]
        if self._pool is None:
            outs = [r.run(x) for r, x in jobs]
        else:
            outs = list(self._pool.map(lambda a: a[0].run(a[1]), jobs))
        res = [None] * self.n
        for m, o in zip(self.members, outs):
            for k, v in zip(m, o):
                res[k] = v
        return res

    @property
    def stats(self):
        agg = RunStats()
        for r in self.runners:
            for k in RunStats.__slots__:
                setattr(agg, k, getattr(agg, k) + getattr(r.stats, k))
        return agg

    def set_kernel_timing(self, on):
        for r in self.runners:
            r.set_kernel_timing(on)

    def set_predict_timing(self, on):
        for r in self.runners:
            r.set_predict_timing(on)

    @stats.setter
    def stats(self, value):
        for r in self.runners:
            r.stats = RunStats()

    @property
    def predict_log(self):
        logs = [r.predict_log for r in self.runners]
        return None if all(x is None for x in logs) else [e for x in logs if x for e in x]

    @predict_log.setter
    def predict_log(self, value):
        for r in self.runners:
            r.predict_log = None if value is None else []

    def replay_predict(self, repeats=1):
        tot, n = 0.0, 0
        for r in self.runners:
            ms, k = r.replay_predict(repeats)
            tot += ms * k
            n += k
        return (tot / n if n else 0.0), n

    def close(self):
        for r in self.runners:
            r.close()
        if self._pool is not None:
            self._pool.shutdown(wait=True)
            self._pool = None


class PartitionRunner(BatchRunner):
    """One partition (the reference's per-UDF-call unit) on one HIP stream."""

    def __init__(self, part, settings=None, stream=None, refit="device", timing=False, fit_threads=8):
        super().__init__([part], settings, stream, refit, timing, fit_threads=fit_threads)
        self.part = part

    def run(self, rng):
        return super().run([rng])[0]


def run_partition_frame(pdf, rng, settings=None, device=None, stream=None, refit="device", stats=None):
    """One partition frame through the GPU path with an explicit MT19937 stream `rng`
    (the RNG a Spark Python worker would hold).  Returns the reference's output frame:
    one row per batch after the first, columns warning_flag_local/global and
    change_flag_local/global (local = the frame's index label, global =
    full_df_row_number, -1 = no event), int64, index all 0 (the index=[0] rows that
    DDM_Process.py:154-159 builds, concatenated at :212)."""
    s = settings or DDMSettings()
    feats = s.x_features or infer_x_features(pdf.columns)
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device())
    X32 = pdf[feats].to_numpy(dtype=np.float64).astype(np.float32)
    y = pdf[s.target].to_numpy()
    part = DevicePartition.from_arrays(X32, y, device, stream)
    runner = PartitionRunner(part, s, stream, refit)
    rows = runner.run(rng)
    if stats is not None:
        stats.update(runner.stats.as_dict())
    return events_frame(rows, pdf.index.to_numpy(), pdf[s.row_number].to_numpy())


def run_partition_frames(frames, rngs, settings=None, device=None, stream=None, refit="device", stats=None):
    """Many partition frames of ONE device in lockstep (BatchRunner): the output frame of
    each, as run_partition_frame would return it, with rngs[k] consumed by frames[k]."""
    s = settings or DDMSettings()
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device())
    parts, labels = [], []
    for pdf in frames:
        feats = s.x_features or infer_x_features(pdf.columns)
        X32 = pdf[feats].to_numpy(dtype=np.float64).astype(np.float32)
        parts.append(DevicePartition.from_arrays(X32, pdf[s.target].to_numpy(), device, stream))
        labels.append((pdf.index.to_numpy(), pdf[s.row_number].to_numpy()))
    runner = BatchRunner(parts, s, stream, refit)
    try:
        rows = runner.run(rngs)
    finally:
        runner.close()
    if stats is not None:
        stats.update(runner.stats.as_dict())
    return [events_frame(r, *lab) for r, lab in zip(rows, labels)]


def run_partition_arrays(parts, rngs, settings=None, device=None, stream=None, refit="device", stats=None):
    """Columnar partitions of ONE device (loader.PartitionArrays: float32 [F, n], labels,
    full_df_row_number) in lockstep, without pandas on the way in: the output frame of
    each, as run_partition_frame would return it for parts[k].frame(...)."""
    s = settings or DDMSettings()
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device())
    dparts = [DevicePartition.from_columns(p.X32, p.target, device, stream) for p in parts]
    runner = BatchRunner(dparts, s, stream, refit)
    try:
        rows = runner.run(rngs)
    finally:
        runner.close()
    if stats is not None:
        stats.update(runner.stats.as_dict())
    return [events_frame(r, np.arange(len(p.target)), p.row_number) for r, p in zip(rows, parts)]


def events_frame(rows, local_labels, global_labels):
    res = np.full((rows.shape[0], 4), -1, dtype=np.int64)
    for c in range(2):
        hit = rows[:, c] >= 0
        res[hit, 2 * c] = local_labels[rows[hit, c]]
        res[hit, 2 * c + 1] = global_labels[rows[hit, c]]
    return pd.DataFrame(res, columns=OUTPUT_COLUMNS, index=np.zeros(len(res), dtype=np.int64))


def run_DDM_loop(pdf, settings=None, device=None, stream=None, refit="device", stats=None):
    """Drop-in for the grouped-map UDF `run_DDM_loop` (DDM_Process.py:166-213): same input
    frame, same output frame, and it draws from / advances numpy's global RandomState
    exactly as the reference does (so `np.random.seed(k)` before the call reproduces the
    reference's events bit for bit)."""
    rng = MTStream.from_global()
    try:
        return run_partition_frame(pdf, rng, settings, device, stream, refit, stats)
    finally:
        np.random.set_state(rng.numpy_state())
