"""Partition controller — the MI355X drop-in for `run_DDM_loop` (DDM_Process.py:166-213).

Reference semantics (per partition, one global numpy MT19937):
  batches of PER_BATCH rows, last one short (:182-184); batch 0 shuffled -> training
  batch (:187); for every later batch: shuffle (:190), refit if flagged (:194-196),
  predict (:199), DDM with carried state (:202), record first warning / first change
  (:147-152, :204); on a change the shuffled batch becomes the training batch, the DDM
  is dropped, refit flagged (:207-210); `pd.concat` of the per-batch rows (:212).

MI355X execution: the partition lives in HBM (columnar float32 features, int32
labels).  Between two refits nothing the host does depends on the rows, so the
controller speculates: it draws the next W batch shuffles (native MT19937), runs the
forest-predict kernel over all W batches in DDM order (writing the error bytes and the
first error position) and the DDM-scan kernel over them (stopping at the first
change), and reads back one small control block.  No drift: the DDM state carries, W
doubles.  Drift in batch d: events up to d are final, the RNG is re-positioned right
after batch d's shuffle (where the reference's next iteration continues), the host
refits on batch d and the next window starts at d+1.  Work past d is discarded, so
total predict work stays within ~2x the rows.
"""
import time

import numpy as np
import pandas as pd
import torch

from . import kernels
from .forest import DeviceForest, pack_sklearn
from .params import OUTPUT_COLUMNS, DDMSettings, infer_x_features
from .rng import MTStream
from .trainer import native_refit

# control block layout (bytes) shared by host (pinned) and device
_FIRST_ERR, _NEV, _STOP, _OFF, _BASE, _STATE, _CTRL_BYTES = 0, 8, 16, 24, 40, 64, 128


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
    """train_rf (DDM_Process.py:98-105) on the host, drawing its 100 tree seeds from the
    partition's MT19937 stream (== the reference's global RandomState)."""
    from sklearn.ensemble import RandomForestClassifier

    def refit(X32, y, rng):
        rs = rng.to_random_state()
        rf = RandomForestClassifier(n_estimators=settings.n_estimators, n_jobs=settings.cores, random_state=rs)
        rf.fit(X32, y)
        rng.load_random_state(rs)
        return pack_sklearn(rf)

    return refit


class RunStats:
    __slots__ = ("epochs", "refits", "predicted_rows", "refit_s", "gpu_s", "host_s", "predict_ms", "predict_bytes",
                 "scan_ms", "scan_rows")

    def __init__(self):
        self.epochs = self.refits = self.predicted_rows = self.predict_bytes = self.scan_rows = 0
        self.refit_s = self.gpu_s = self.host_s = self.predict_ms = self.scan_ms = 0.0

    def as_dict(self):
        return {k: getattr(self, k) for k in self.__slots__}


class PartitionRunner:
    """Runs the speculative predict+scan epochs of one partition on one HIP stream."""

    def __init__(self, part, settings=None, stream=None, refit=None, timing=False):
        self.part = part
        self.timing = timing
        # HIP events recorded by the C-ABI right around each launch on this runner's stream
        self.t_pred = kernels.LaunchTimer() if timing else None
        self.t_scan = kernels.LaunchTimer() if timing else None
        self.s = settings or DDMSettings()
        self.stream = stream or torch.cuda.Stream(part.device)
        self.refit = refit or native_refit(self.s)
        self.params = kernels.params_struct(self.s.min_num_instances, self.s.per_batch, self.s.warning_level,
                                            self.s.out_control_level)
        n, dev = part.n, part.device
        self.perm_h = torch.empty(max(n, 1), dtype=torch.uint8, pin_memory=True)
        self.perm_np = self.perm_h.numpy()
        self.perm_d = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
        self.err_d = torch.zeros(_round_up(max(n, 1), 16) + 16, dtype=torch.uint8, device=dev)
        self.ctrl_h = torch.zeros(_CTRL_BYTES, dtype=torch.uint8, pin_memory=True)
        self.ctrl_np = self.ctrl_h.numpy()
        self.ctrl_d = torch.zeros(_CTRL_BYTES, dtype=torch.uint8, device=dev)
        nb = (n + self.s.per_batch - 1) // self.s.per_batch
        self.max_win = max(1, min(self.s.max_window_batches, nb))
        self.ev_d = torch.empty((self.max_win, 2), dtype=torch.int32, device=dev)
        self.ev_h = torch.empty((self.max_win, 2), dtype=torch.int32, pin_memory=True)
        self.stats = RunStats()

    # -- host views of the control block
    def _ctrl(self, off, dtype, count=1):
        return self.ctrl_np[off:off + np.dtype(dtype).itemsize * count].view(dtype)

    def run(self, rng):
        """Returns int64 [n_batches-1, 2]: partition rows of (first warning, change) per
        batch 1.. (-1 = none).  Consumes `rng` exactly as the reference consumes np.random."""
        s, part, st = self.s, self.part, self.stats
        n, pb = part.n, s.per_batch
        nb = (n + pb - 1) // pb
        if nb == 0:
            raise IndexError("list index out of range")       # batches[0] on an empty frame (:187)
        blen = np.full(nb, pb, dtype=np.int32)
        blen[-1] = n - (nb - 1) * pb
        perm = self.perm_np

        def draw(b0, b1):
            if b1 > b0:
                rng.perms(blen[b0:b1], out=perm[b0 * pb:b0 * pb + int(blen[b0:b1].sum())])

        draw(0, 1)                                             # batch_a = batches[0].sample (:187)
        if nb < 2:
            raise ValueError("No objects to concatenate")      # pd.concat([]) (:212)
        train_rows = perm[:blen[0]].astype(np.int64)
        out = np.full((nb - 1, 2), -1, dtype=np.int64)
        state = kernels.fresh_states(1)
        forest = None
        retrain = True
        j = 1
        win = max(1, s.window_batches)
        stream = self.stream
        base = self.ctrl_d.data_ptr()
        while j < nb:
            t0 = time.perf_counter()
            if retrain:
                draw(j, j + 1)                                 # batch_b.sample before the fit (:190)
                X32, y = part.rows(train_rows, stream)
                t1 = time.perf_counter()
                forest = DeviceForest(self.refit(X32, y, rng), part.device)
                st.refit_s += time.perf_counter() - t1
                st.refits += 1
                retrain = False
                state = kernels.fresh_states(1)                # ddm = None -> new DDM (:136-139)
                gen_from = j + 1
            else:
                gen_from = j
            b_end = min(nb, j + min(win, self.max_win))
            snap = rng.snapshot()
            draw(gen_from, b_end)
            p0, p1 = j * pb, (b_end - 1) * pb + int(blen[b_end - 1])
            self._ctrl(_OFF, np.int64, 2)[:] = (p0, p1)
            self._ctrl(_BASE, np.int64)[0] = 0
            self.ctrl_np[_STATE:_STATE + 56] = state.view(np.uint8)
            st.host_s += time.perf_counter() - t0
            t0 = time.perf_counter()
            with torch.cuda.stream(stream):
                self.ctrl_d.copy_(self.ctrl_h, non_blocking=True)
                self.perm_d[p0:p1].copy_(self.perm_h[p0:p1], non_blocking=True)
                kernels.forest_predict(part.X, part.y, self.perm_d, p0, p1, pb, forest, self.err_d,
                                       first_err=self.ctrl_d[_FIRST_ERR:_FIRST_ERR + 8].view(torch.int64),
                                       stream=stream, timer=self.t_pred)
                kernels.scan_streams_raw(self.err_d.data_ptr(), base + _OFF, 1, self.params, base + _STATE,
                                         base + _BASE, b_end - j, self.ev_d.data_ptr(), base + _FIRST_ERR,
                                         base + _STOP, base + _NEV, 0, None, stream, self.t_scan)
                self.ctrl_h.copy_(self.ctrl_d, non_blocking=True)
            stream.synchronize()
            stop = int(self._ctrl(_STOP, np.int32)[0])
            nev = int(self._ctrl(_NEV, np.int64)[0])
            last = j + stop if stop >= 0 else b_end - 1
            if self.timing:
                st.predict_ms += self.t_pred.elapsed_ms()
                st.scan_ms += self.t_scan.elapsed_ms()
                st.predict_bytes += (p1 - p0) * (4 * forest.packed.features_used + 6)
                st.scan_rows += min(p1, (last + 1) * pb) - p0
            if nev:
                k = last - j + 1
                with torch.cuda.stream(stream):
                    self.ev_h[:k].copy_(self.ev_d[:k], non_blocking=True)
                stream.synchronize()
                ev = self.ev_h[:k].numpy()
                for c in range(2):
                    q = ev[:, c]
                    hit = np.nonzero(q >= 0)[0]
                    b = j + hit
                    out[b - 1, c] = b * pb + perm[b * pb + q[hit]].astype(np.int64)
            st.gpu_s += time.perf_counter() - t0
            st.epochs += 1
            st.predicted_rows += p1 - p0
            if stop >= 0:
                d = j + stop
                train_rows = d * pb + perm[d * pb:d * pb + blen[d]].astype(np.int64)
                retrain = True
                rng.restore(snap)                              # RNG right after batch d's shuffle
                draw(gen_from, d + 1)
                j = d + 1
                win = max(1, s.window_batches)
            else:
                state = self._ctrl(_STATE, np.uint8, 56).copy().view(kernels.STATE_DTYPE)
                j = b_end
                win *= 2
        return out


def run_partition_frame(pdf, rng, settings=None, device=None, stream=None, refit=None, stats=None):
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


def run_DDM_loop(pdf, settings=None, device=None, stream=None, refit=None, stats=None):
    """Drop-in for the grouped-map UDF `run_DDM_loop` (DDM_Process.py:166-213): same input
    frame, same output frame, and it draws from / advances numpy's global RandomState
    exactly as the reference does (so `np.random.seed(k)` before the call reproduces the
    reference's events bit for bit)."""
    rng = MTStream.from_global()
    try:
        return run_partition_frame(pdf, rng, settings, device, stream, refit, stats)
    finally:
        np.random.set_state(rng.numpy_state())
