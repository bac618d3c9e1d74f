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
import time

import numpy as np
import pandas as pd
import torch

from . import kernels
from .forest import DeviceForest
from .params import OUTPUT_COLUMNS, DDMSettings, infer_x_features
from .rng import MTStream
from .shuffle import GpuShuffle, expected_draws_per_batch
from .trainer import NativeForestTrainer

# control block layout (bytes) shared by host (pinned) and device
_FIRST_ERR, _NEV, _STOP, _OFF, _BASE, _PICK, _STATE, _CTRL_BYTES = 0, 8, 16, 24, 40, 48, 64, 128


def _round_up(n, m):
    return (n + m - 1) // m * m


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
        y = np.asarray(y)
        if y.size and (y.min() < np.iinfo(np.int32).min or y.max() > np.iinfo(np.int32).max):
            raise ValueError("labels must fit int32 on the device path")
        n, F = X32.shape
        part = cls.allocate(n, F, device)
        with torch.cuda.stream(stream or torch.cuda.current_stream(device)):
            if n:
                part.X[:, :n].copy_(torch.from_numpy(np.ascontiguousarray(X32.T)))
                part.y[:n].copy_(torch.from_numpy(y.astype(np.int32)))
        part.host_X32, part.host_y = X32, y.astype(np.int64)
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
                 "scan_ms", "scan_rows", "shuffle_ms", "sklearn_refits")

    def __init__(self):
        self.epochs = self.refits = self.predicted_rows = self.predict_bytes = self.scan_rows = 0
        self.sklearn_refits = 0
        self.refit_s = self.gpu_s = self.host_s = self.predict_ms = self.scan_ms = self.shuffle_ms = 0.0

    def as_dict(self):
        return {k: getattr(self, k) for k in self.__slots__}


class PartitionRunner:
    """Runs the speculative shuffle+predict+scan epochs of one partition on one HIP stream.

    refit: "native" (ddm_rf_fit, identical trees to sklearn 1.7.2; sklearn itself for NaN
    inputs) or "sklearn"."""

    def __init__(self, part, settings=None, stream=None, refit="native", timing=False):
        self.part = part
        self.s = settings or DDMSettings()
        self.stream = stream or torch.cuda.Stream(part.device)
        self.refit_kind = refit
        self.trainer = NativeForestTrainer(self.s.n_estimators)
        self.sk_refit = sklearn_refit(self.s)
        self.timing = timing
        # HIP events recorded by the C-ABI right around each launch on this runner's stream
        self.t_pred = kernels.LaunchTimer() if timing else None
        self.t_scan = kernels.LaunchTimer() if timing else None
        self.t_shuf = kernels.LaunchTimer() if timing else None
        self.params = kernels.params_struct(self.s.min_num_instances, self.s.per_batch, self.s.warning_level,
                                            self.s.out_control_level)
        n, dev, pb = part.n, part.device, self.s.per_batch
        if not 2 <= pb <= 256:
            raise ValueError("per_batch must be in [2, 256] on the device path")
        self.perm_d = torch.zeros(max(n, 1) + 256, dtype=torch.uint8, device=dev)
        self.err_d = torch.zeros(_round_up(max(n, 1), 16) + 16, dtype=torch.uint8, device=dev)
        self.ctrl_h = torch.zeros(_CTRL_BYTES, dtype=torch.uint8, pin_memory=True)
        self.ctrl_np = self.ctrl_h.numpy()
        self.ctrl_d = torch.zeros(_CTRL_BYTES, dtype=torch.uint8, device=dev)
        # pinned staging: [0] batch-j shuffle of a refit epoch, [1] short last batch, [2] D2H
        self.small_h = [torch.empty(256, dtype=torch.uint8, pin_memory=True) for _ in range(3)]
        self.neg1_d = torch.full((1,), -1, dtype=torch.int32, device=dev)
        nb = (n + pb - 1) // pb
        self.max_win = max(1, min(self.s.max_window_batches, nb))
        self.ev_d = torch.empty((self.max_win, 2), dtype=torch.int32, device=dev)
        self.ev_h = torch.empty((self.max_win, 2), dtype=torch.int32, pin_memory=True)
        cap = int(nb * expected_draws_per_batch(pb) * 1.2) + 64 * 1024
        self.shuffle = GpuShuffle(dev, pb, cap, self.max_win, self.stream)
        self.stats = RunStats()

    # -- host views of the control block
    def _ctrl(self, off, dtype, count=1):
        return self.ctrl_np[off:off + np.dtype(dtype).itemsize * count].view(dtype)

    def _fit(self, rows, P_seeds):
        """Refit on the rows of the drift batch (shuffled order); returns (forest, draws used)."""
        X32, y = self.part.rows(rows, self.stream)
        sh = self.shuffle
        t0 = time.perf_counter()
        seeds, P_after = sh.host_seeds(P_seeds, self.s.n_estimators)
        packed = None
        if self.refit_kind == "native":
            packed = self.trainer.fit(X32, y, seeds)
        if packed is None:                    # sklearn requested, or NaN in X (missing values)
            packed = self.sk_refit(X32, y, sh.numpy_state(P_seeds))
            self.stats.sklearn_refits += 1
        self.stats.refit_s += time.perf_counter() - t0
        self.stats.refits += 1
        return DeviceForest(packed, self.part.device), P_after

    def _upload_perm(self, b, perm, slot):
        pb = self.s.per_batch
        h = self.small_h[slot]
        h[:len(perm)].copy_(torch.from_numpy(perm))
        with torch.cuda.stream(self.stream):
            self.perm_d[b * pb:b * pb + len(perm)].copy_(h[:len(perm)], non_blocking=True)

    def _perm_rows(self, b, length):
        """Rows of batch b in its shuffled order (D2H of the batch's perm bytes)."""
        pb = self.s.per_batch
        h = self.small_h[2]
        with torch.cuda.stream(self.stream):
            h[:length].copy_(self.perm_d[b * pb:b * pb + length], non_blocking=True)
        self.stream.synchronize()
        return b * pb + h[:length].numpy().astype(np.int64)

    def run(self, rng):
        """Returns int64 [n_batches-1, 2]: partition rows of (first warning, change) per
        batch 1.. (-1 = none).  Consumes `rng` (advanced in place) exactly as the reference
        consumes np.random."""
        s, part, st = self.s, self.part, self.stats
        n, pb = part.n, s.per_batch
        nb = (n + pb - 1) // pb
        if nb == 0:
            raise IndexError("list index out of range")       # batches[0] on an empty frame (:187)
        last_len = n - (nb - 1) * pb
        n_full = nb if last_len == pb else nb - 1              # batches with exactly pb rows

        def blen(b):
            return pb if b < nb - 1 else last_len

        sh = self.shuffle
        sh.reset(rng)
        # the whole partition's stream up front (one generate + table pass); windows
        # extend it if drifts (100 seed draws each) push it further
        sh.ensure(int(nb * expected_draws_per_batch(pb) * 1.02))
        stream = self.stream
        base = self.ctrl_d.data_ptr()
        try:
            perm0, P = sh.host_perm(0, blen(0))                # batch_a = batches[0].sample (:187)
            if nb < 2:
                raise ValueError("No objects to concatenate")  # pd.concat([]) (:212)
            train_rows = perm0.astype(np.int64)
            out = np.full((nb - 1, 2), -1, dtype=np.int64)
            state = kernels.fresh_states(1)
            forest, retrain, j = None, True, 1
            win = max(1, s.window_batches)
            while j < nb:
                t0 = time.perf_counter()
                P_after_first = None
                if retrain:
                    permj, P = sh.host_perm(P, blen(j))        # batch_b.sample before the fit (:190, :194)
                    self._upload_perm(j, permj, 0)
                    forest, P = self._fit(train_rows, P)       # 100 tree seeds follow the shuffle
                    P_after_first = P
                    retrain = False
                    state = kernels.fresh_states(1)            # ddm = None -> new DDM (:136-139)
                    g0 = j + 1
                else:
                    g0 = j
                b_end = min(nb, j + min(win, self.max_win))
                gpu_end = min(b_end, n_full)
                Wg = max(0, gpu_end - g0)
                tail = b_end == nb and last_len != pb and nb - 1 >= g0
                P_tail_after = None
                if Wg:
                    sh.window(P, Wg, self.perm_d[g0 * pb:], timer=self.t_shuf)
                if tail:
                    if Wg:
                        sh.pick(self.neg1_d.data_ptr(), Wg, 0, Wg - 1, base + _PICK)   # end of the GPU batches
                        P_tail = int(self._read_pick_now()) + 1
                    else:
                        P_tail = P
                    permT, P_tail_after = sh.host_perm(P_tail, last_len)
                    self._upload_perm(nb - 1, permT, 1)
                p0, p1 = j * pb, (b_end - 1) * pb + blen(b_end - 1)
                self._ctrl(_OFF, np.int64, 2)[:] = (p0, p1)
                self._ctrl(_BASE, np.int64)[0] = 0
                self.ctrl_np[_STATE:_STATE + 56] = state.view(np.uint8)
                st.host_s += time.perf_counter() - t0
                t0 = time.perf_counter()
                with torch.cuda.stream(stream):
                    self.ctrl_d[_OFF:_CTRL_BYTES].copy_(self.ctrl_h[_OFF:_CTRL_BYTES], non_blocking=True)
                    kernels.forest_predict(part.X, part.y, self.perm_d, p0, p1, pb, forest, self.err_d,
                                           first_err=self.ctrl_d[_FIRST_ERR:_FIRST_ERR + 8].view(torch.int64),
                                           stream=stream, timer=self.t_pred)
                    kernels.scan_streams_raw(self.err_d.data_ptr(), base + _OFF, 1, self.params, base + _STATE,
                                             base + _BASE, b_end - j, self.ev_d.data_ptr(), base + _FIRST_ERR,
                                             base + _STOP, base + _NEV, 0, None, stream, self.t_scan,
                                             self.perm_d.data_ptr())
                    if Wg:
                        sh.pick(base + _STOP, Wg, g0 - j, b_end - 1 - j, base + _PICK)
                    self.ctrl_h.copy_(self.ctrl_d, non_blocking=True)
                stream.synchronize()
                stop = int(self._ctrl(_STOP, np.int32)[0])
                nev = int(self._ctrl(_NEV, np.int64)[0])
                picked = int(self._ctrl(_PICK, np.int64)[0]) if Wg else -1
                last = j + stop if stop >= 0 else b_end - 1
                if self.timing:
                    st.predict_ms += self.t_pred.elapsed_ms()
                    st.scan_ms += self.t_scan.elapsed_ms()
                    if Wg:
                        st.shuffle_ms += self.t_shuf.elapsed_ms()
                    st.predict_bytes += (p1 - p0) * (4 * forest.packed.features_used + 6)
                    st.scan_rows += min(p1, (last + 1) * pb) - p0
                if nev:
                    k = last - j + 1
                    with torch.cuda.stream(stream):
                        self.ev_h[:k].copy_(self.ev_d[:k], non_blocking=True)
                    stream.synchronize()
                    ev = self.ev_h[:k].numpy()
                    for c in range(2):
                        hit = np.nonzero(ev[:, c] >= 0)[0]
                        b = j + hit
                        out[b - 1, c] = b * pb + ev[hit, c].astype(np.int64)
                st.gpu_s += time.perf_counter() - t0
                st.epochs += 1
                st.predicted_rows += p1 - p0
                # RNG position right after the last consumed batch shuffle
                if stop >= 0:
                    d = j + stop
                    if d < g0:
                        P = P_after_first                      # drift in the refit batch: after its seeds
                    elif tail and d == nb - 1:
                        P = P_tail_after
                    else:
                        P = picked + 1
                    train_rows = self._perm_rows(d, blen(d))
                    retrain = True
                    j = d + 1
                    win = max(1, s.window_batches)
                else:
                    if tail:
                        P = P_tail_after
                    elif Wg:
                        P = picked + 1
                    elif P_after_first is not None:
                        P = P_after_first
                    state = self._ctrl(_STATE, np.uint8, 56).copy().view(kernels.STATE_DTYPE)
                    j = b_end
                    win *= 2
            return out
        finally:
            if "P" in locals():
                ns = sh.numpy_state(P)
                rng.key[:] = ns[1]
                rng.pos.value = ns[2]

    def _read_pick_now(self):
        with torch.cuda.stream(self.stream):
            self.ctrl_h[_PICK:_PICK + 8].copy_(self.ctrl_d[_PICK:_PICK + 8], non_blocking=True)
        self.stream.synchronize()
        return self._ctrl(_PICK, np.int64)[0]


def run_partition_frame(pdf, rng, settings=None, device=None, stream=None, refit="native", stats=None):
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


def events_frame(rows, local_labels, global_labels):
    res = np.full((rows.shape[0], 4), -1, dtype=np.int64)
    for c in range(2):
        hit = rows[:, c] >= 0
        res[hit, 2 * c] = local_labels[rows[hit, c]]
        res[hit, 2 * c + 1] = global_labels[rows[hit, c]]
    return pd.DataFrame(res, columns=OUTPUT_COLUMNS, index=np.zeros(len(res), dtype=np.int64))


def run_DDM_loop(pdf, settings=None, device=None, stream=None, refit="native", stats=None):
    """Drop-in for the grouped-map UDF `run_DDM_loop` (DDM_Process.py:166-213): same input
    frame, same output frame, and it draws from / advances numpy's global RandomState
    exactly as the reference does (so `np.random.seed(k)` before the call reproduces the
    reference's events bit for bit)."""
    rng = MTStream.from_global()
    try:
        return run_partition_frame(pdf, rng, settings, device, stream, refit, stats)
    finally:
        np.random.set_state(rng.numpy_state())
