"""Device forest refit (ddm_rf_fit_device).

train_rf (DDM_Process.py:98-105) on the GPU: the trees, the packed forest and the
compiled blob are the ones the host trainer (ddm_rf_fit_many) builds for the same rows,
labels and seeds.  The controller points the jobs at the rows, labels and seeds that
ddm_epoch_stage gathers after a change, gated on the change, so a refit never leaves the
device; the host reads back only the small result row of each job.
"""
import ctypes

import numpy as np
import torch

from ._capi import DdmForest, check, lib
from .treepack import NODE_DTYPE, PackedForest

DFIT_DTYPE = np.dtype([("X", "<u8"), ("y", "<u8"), ("seeds", "<u8"), ("gate", "<u8"), ("gate2", "<u8"),
                       ("L", "<i4"), ("F", "<i4"), ("n_trees", "<i4"), ("max_features", "<i4"),
                       ("k_cap", "<i4"), ("pad", "<i4"), ("scratch", "<u8"), ("nodes", "<u8"), ("roots", "<u8"),
                       ("leaf_value", "<u8"), ("classes", "<u8"), ("blob", "<u8"), ("blob_cap", "<i8"),
                       ("result", "<u8")])
assert DFIT_DTYPE.itemsize == 128

RESULT_WORDS = 12
STATUS, CLASSES, NODES, PURE, LEAF_ROWS, BLOB, CF_SLOTS, CF_VR, CF_LEAVES, CF_TAB = range(10)
BLOB_CAP = 1 << 20


def max_features_of(F):
    """max_features='sqrt' (sklearn: max(1, int(sqrt(F))))."""
    return max(1, int(np.sqrt(F)))


class RefitBuffers:
    """Device outputs of one partition's refits (reused: a refit overwrites the last)."""

    def __init__(self, L, F, n_trees, k_cap, device, blob_cap=BLOB_CAP):
        self.L, self.F, self.T, self.k_cap = int(L), int(F), int(n_trees), int(k_cap)
        nb = lib.ddm_rf_device_scratch_bytes(self.L, self.F, self.T, self.k_cap)
        if nb <= 0:
            raise ValueError("ddm_rf_device_scratch_bytes: bad shape")
        self.scratch = torch.empty(nb, dtype=torch.uint8, device=device)
        self.nodes = torch.empty(self.T * (2 * self.L - 1) * NODE_DTYPE.itemsize, dtype=torch.uint8, device=device)
        self.roots = torch.empty(self.T, dtype=torch.int32, device=device)
        self.leaf_value = torch.empty(self.T * self.L * self.k_cap, dtype=torch.float64, device=device)
        self.classes = torch.zeros(self.k_cap, dtype=torch.int32, device=device)
        self.blob = torch.empty(blob_cap, dtype=torch.uint8, device=device)

    def record(self, X, y, seeds, result, gate=0, gate2=0, L=None):
        """A DFIT_DTYPE row (tuple) for rows X [L][F] f32, labels y, seeds (device pointers)."""
        return (X, y, seeds, gate, gate2, self.L if L is None else int(L), self.F, self.T, max_features_of(self.F),
                self.k_cap, 0, self.scratch.data_ptr(), self.nodes.data_ptr(), self.roots.data_ptr(),
                self.leaf_value.data_ptr(), self.classes.data_ptr(), self.blob.data_ptr(), self.blob.numel(), result)

    def ptrs(self):
        """(nodes, roots, leaf_value, classes, blob) device addresses (the buffers never move)."""
        if getattr(self, "_ptrs", None) is None:
            self._ptrs = (self.nodes.data_ptr(), self.roots.data_ptr(), self.leaf_value.data_ptr(),
                          self.classes.data_ptr(), self.blob.data_ptr())
        return self._ptrs

    def descriptor(self, res):
        """ddm_forest of the refit whose result row is `res` (status 0)."""
        pure = int(res[PURE])
        blob = int(res[BLOB])
        return DdmForest(self.nodes.data_ptr(), self.roots.data_ptr(), 0 if pure else self.leaf_value.data_ptr(),
                         self.classes.data_ptr(), self.T, int(res[CLASSES]), int(res[NODES]), pure,
                         self.blob.data_ptr() if blob else 0, int(res[CF_SLOTS]) if blob else 0,
                         int(res[CF_VR]) if blob else 0, int(res[CF_LEAVES]) if blob else 0,
                         int(res[CF_TAB]) if blob else 0)


class DeviceFitForest:
    """The forest of a device refit, in a partition's RefitBuffers (the controller's
    counterpart of forest.DeviceForest)."""

    def __init__(self, bufs, res):
        self.bufs = bufs
        self.res = np.array(res, dtype=np.int64)
        self._desc = None

    @property
    def desc(self):
        if self._desc is None:
            self._desc = self.bufs.descriptor(self.res)
        return self._desc

    def seg_fields(self):
        """The forest fields of a ddm_predict_segment (kernels.SEG_DTYPE order: nodes, roots,
        leaf_value, classes, n_trees, n_classes, n_nodes, pure, cforest, cf_slots,
        cf_vote_regs, cf_leaves, cf_tab_words) without building the ctypes descriptor."""
        b, r = self.bufs, self.res.tolist()
        p = b.ptrs()
        pure, blob = r[PURE], r[BLOB]
        return (p[0], p[1], 0 if pure else p[2], p[3], b.T, r[CLASSES], r[NODES], pure, p[4] if blob else 0,
                r[CF_SLOTS] if blob else 0, r[CF_VR] if blob else 0, r[CF_LEAVES] if blob else 0,
                r[CF_TAB] if blob else 0)

    @property
    def compiled(self):
        return int(self.res[BLOB]) > 0

    @property
    def features_read(self):
        return int(self.res[CF_SLOTS]) if self.compiled else self.bufs.F


# Small batches can be gated, checked and presorted inside the tree kernel (every workgroup
# again) instead of by k_dfit_prep.  Measured on MI355X (tools/bench_refit.py, 8 refits of
# 100 x 27 batches): separable batches (C3's refits) 87 us with the prep kernel, 123 us
# fused; noisy batches 1.61 ms either way.  So the prep kernel stays.
FUSED_PREP = False


def max_lf(per_batch, n_features):
    """ddm_rf_fit_device_lf's max_lf for the controller's refits."""
    return int(per_batch) * int(n_features) if FUSED_PREP else -1


def fit_device(table_d, n_jobs, max_trees, stream, max_lf=-1):
    """ddm_rf_fit_device over a device table of DFIT_DTYPE records (max_lf >= every job's
    L*F: small batches are prepared inside the tree kernel)."""
    check(lib.ddm_rf_fit_device_lf(table_d.data_ptr(), int(n_jobs), int(max_trees), int(max_lf),
                                   ctypes.c_void_p(stream.cuda_stream)), "ddm_rf_fit_device")


class DeviceTrainer:
    """Stand-alone device refits of host batches (tests, tools): uploads the rows, runs the
    fit and reads back packed forests and blobs in the BatchForestTrainer.fit_many format."""

    def __init__(self, n_estimators=100, k_cap=16, device=None, fused=True):
        self.T, self.k_cap, self.fused = int(n_estimators), int(k_cap), bool(fused)
        self.device = device or torch.device("cuda", torch.cuda.current_device())

    def fit_many(self, batches, stream=None):
        stream = stream or torch.cuda.current_stream(self.device)
        dev = self.device
        recs, keep = [], []
        res_d = torch.full((len(batches), RESULT_WORDS), -7, dtype=torch.int64, device=dev)
        for k, (X32, y, seeds) in enumerate(batches):
            X32 = np.ascontiguousarray(X32, dtype=np.float32)
            L, F = X32.shape
            xd = torch.from_numpy(X32).to(dev)
            yd = torch.from_numpy(np.ascontiguousarray(y, dtype=np.int32)).to(dev)
            sd = torch.from_numpy(np.ascontiguousarray(seeds, dtype=np.int64)).to(dev)
            b = RefitBuffers(L, F, self.T, self.k_cap, dev)
            keep.append((xd, yd, sd, b))
            recs.append(b.record(xd.data_ptr(), yd.data_ptr(), sd.data_ptr(), res_d[k].data_ptr()))
        table = torch.from_numpy(np.array(recs, dtype=DFIT_DTYPE).view(np.uint8)).to(dev)
        torch.cuda.synchronize(dev)
        max_lf = max(np.asarray(X32).size for X32, _, _ in batches) if self.fused else -1
        fit_device(table, len(batches), self.T, stream, max_lf)
        stream.synchronize()
        res = res_d.cpu().numpy()
        out = []
        for k, (xd, yd, sd, b) in enumerate(keep):
            r = res[k]
            if r[STATUS] != 0:
                out.append((None, None, None, r))
                continue
            K, n_nodes, pure, rows = int(r[CLASSES]), int(r[NODES]), int(r[PURE]), int(r[LEAF_ROWS])
            nodes = b.nodes[:n_nodes * NODE_DTYPE.itemsize].cpu().numpy().view(NODE_DTYPE).copy()
            roots = b.roots.cpu().numpy().copy()
            classes = b.classes[:K].cpu().numpy().copy()
            lv = None if pure else b.leaf_value[:rows * K].cpu().numpy().reshape(rows, K).copy()
            pf = PackedForest(nodes, roots, lv, classes, bool(pure))
            blob = b.blob[:int(r[BLOB])].cpu().numpy().copy() if r[BLOB] else None
            head = ({"n_slots": int(r[CF_SLOTS]), "vote_regs": int(r[CF_VR]), "n_leaves": int(r[CF_LEAVES]),
                     "tab_words": int(r[CF_TAB])} if r[BLOB] else None)
            out.append((pf, blob, head, r))
        return out
