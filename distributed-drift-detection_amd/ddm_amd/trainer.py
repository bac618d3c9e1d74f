"""Native refit backend: train_rf (DDM_Process.py:98-105) via ddm_rf_fit (csrc/rf_fit.cpp),
an exact restatement of scikit-learn 1.7.2's RandomForestClassifier.fit.

The reference fits `RandomForestClassifier(n_jobs=CORES)` with random_state=None, i.e. it
draws the 100 per-tree seeds from numpy's global RandomState; the controller reads them
from the partition's MT19937 stream, then the trees are grown natively (the call releases
the GIL, so partition threads refit in parallel) and come back already packed for
ddm_forest_predict.  Inputs containing NaN (missing values) or more than FIT_MAX_CLASSES
(64) classes return None: the controller then refits with sklearn itself.
"""
import ctypes

import numpy as np

from ._capi import DDM_E_IMPURE, DDM_E_NAN, check, lib
from .treepack import FIT_MAX_CLASSES, NODE_DTYPE, PackedForest


class NativeForestTrainer:
    def __init__(self, n_estimators=100, max_rows=256):
        self.T = int(n_estimators)
        self._alloc(max_rows)
        self.leaf_value = None
        self.info = np.zeros(3, dtype=np.int64)
        self.sklearn_fallbacks = 0

    def _alloc(self, rows):
        self.max_rows = rows
        self.nodes = np.zeros(self.T * (2 * rows - 1), dtype=NODE_DTYPE)
        self.roots = np.zeros(self.T, dtype=np.int32)

    def fit(self, X32, y, seeds):
        """Packed forest for classes np.unique(y); seeds = the T randint(2**31-1) draws."""
        X32 = np.ascontiguousarray(X32, dtype=np.float32)
        n, F = X32.shape
        classes, yi = np.unique(np.asarray(y), return_inverse=True)
        if classes.size > FIT_MAX_CLASSES:
            return None                          # more classes than the native trainer takes: sklearn
        if n > self.max_rows:
            self._alloc(n)
        yi = np.ascontiguousarray(yi, dtype=np.int32)
        seeds = np.ascontiguousarray(seeds, dtype=np.int64)
        maxf = max(1, int(np.sqrt(F)))           # max_features="sqrt" (tree/_classes.py)
        for _ in range(2):
            lv = self.leaf_value
            rc = lib.ddm_rf_fit(X32.ctypes.data, n, F, yi.ctypes.data, classes.size, seeds.ctypes.data, self.T, maxf,
                                self.nodes.ctypes.data, self.nodes.size, self.roots.ctypes.data,
                                None if lv is None else lv.ctypes.data, 0 if lv is None else lv.shape[0],
                                self.info.ctypes.data)
            if rc == DDM_E_IMPURE:
                self.leaf_value = np.zeros((self.T * n, classes.size), dtype=np.float64)
                continue
            if rc == DDM_E_NAN:
                return None
            check(rc, "ddm_rf_fit")
            break
        n_nodes, pure, rows = (int(v) for v in self.info)
        leaf = None if pure else np.ascontiguousarray(self.leaf_value.reshape(-1)[:rows * classes.size]
                                                      .reshape(rows, classes.size)).copy()
        if self.leaf_value is not None and self.leaf_value.shape[1] != classes.size:
            self.leaf_value = None
        return PackedForest(self.nodes[:n_nodes].copy(), self.roots.copy(), leaf, classes.astype(np.int32),
                            bool(pure))



class FitJob(ctypes.Structure):
    """ddm_fit_job (include/ddm_amd.h)."""
    _fields_ = [("X", ctypes.c_void_p), ("y_idx", ctypes.c_void_p), ("seeds", ctypes.c_void_p),
                ("classes", ctypes.c_void_p), ("n", ctypes.c_int32), ("n_features", ctypes.c_int32),
                ("n_classes", ctypes.c_int32), ("n_trees", ctypes.c_int32), ("max_features", ctypes.c_int32),
                ("status", ctypes.c_int32), ("nodes", ctypes.c_void_p), ("nodes_cap", ctypes.c_int64),
                ("roots", ctypes.c_void_p), ("leaf_value", ctypes.c_void_p), ("leaf_rows_cap", ctypes.c_int64),
                ("info", ctypes.c_int64 * 3), ("blob", ctypes.c_void_p), ("blob_cap", ctypes.c_int64),
                ("blob_bytes", ctypes.c_int64), ("cf_slots", ctypes.c_int32), ("cf_vote_regs", ctypes.c_int32),
                ("cf_leaves", ctypes.c_int32), ("cf_tab_words", ctypes.c_int32)]


class BatchForestTrainer:
    """Many refits in one native call (ddm_rf_fit_many): every tree of every job on a pool
    of host threads, then per job the packed forest and its compiled blob."""

    BLOB_CAP = 1 << 20

    def __init__(self, n_estimators=100, n_threads=8, max_rows=256):
        self.T = int(n_estimators)
        self.n_threads = int(n_threads)
        self.max_rows = max_rows
        self._bufs = []

    def _buf(self, k, rows):
        while len(self._bufs) <= k:
            self._bufs.append(None)
        b = self._bufs[k]
        if b is None or b["rows"] < rows:
            b = {"rows": rows, "nodes": np.zeros(self.T * (2 * rows - 1), dtype=NODE_DTYPE),
                 "roots": np.zeros(self.T, dtype=np.int32), "blob": np.zeros(self.BLOB_CAP, dtype=np.uint8)}
            self._bufs[k] = b
        return b

    def fit_many(self, batches):
        """batches: [(X32 [n, F], y, seeds)] -> [(PackedForest, blob or None, head dict or None) or None
        (None: NaN in X or more than FIT_MAX_CLASSES classes, refit with sklearn)]."""
        jobs = (FitJob * len(batches))()
        keep = []
        for k, (X32, y, seeds) in enumerate(batches):
            X32 = np.ascontiguousarray(X32, dtype=np.float32)
            n, F = X32.shape
            classes, yi = np.unique(np.asarray(y), return_inverse=True)
            if classes.size > FIT_MAX_CLASSES:
                keep.append(None)                # more classes than the native trainer takes: sklearn
                continue
            yi = np.ascontiguousarray(yi, dtype=np.int32)
            seeds = np.ascontiguousarray(seeds, dtype=np.int64)
            cls32 = classes.astype(np.int32)
            b = self._buf(k, max(n, self.max_rows))
            leaf = np.zeros((self.T * n, classes.size), dtype=np.float64)
            keep.append((X32, yi, seeds, cls32, leaf, classes))
            j = jobs[k]
            j.X, j.y_idx, j.seeds, j.classes = X32.ctypes.data, yi.ctypes.data, seeds.ctypes.data, cls32.ctypes.data
            j.n, j.n_features, j.n_classes, j.n_trees = n, F, classes.size, self.T
            j.max_features = max(1, int(np.sqrt(F)))
            j.nodes, j.nodes_cap, j.roots = b["nodes"].ctypes.data, b["nodes"].size, b["roots"].ctypes.data
            j.leaf_value, j.leaf_rows_cap = leaf.ctypes.data, leaf.shape[0]
            j.blob, j.blob_cap = b["blob"].ctypes.data, b["blob"].size
        rc = lib.ddm_rf_fit_many(jobs, len(batches), self.n_threads)
        out = []
        for k, j in enumerate(jobs):
            if keep[k] is None or j.status == DDM_E_NAN:      # > FIT_MAX_CLASSES classes, or NaN
                out.append(None)
                continue
            check(j.status, "ddm_rf_fit_many")
            _, _, _, cls32, leaf, classes = keep[k]
            b = self._bufs[k]
            n_nodes, pure, rows = (int(v) for v in j.info)
            lv = None if pure else np.ascontiguousarray(leaf[:rows]).copy()
            pf = PackedForest(b["nodes"][:n_nodes].copy(), b["roots"].copy(), lv, cls32, bool(pure))
            if j.blob_bytes:
                blob = b["blob"][:j.blob_bytes].copy()
                head = {"n_slots": j.cf_slots, "vote_regs": j.cf_vote_regs, "n_leaves": j.cf_leaves,
                        "tab_words": j.cf_tab_words}
                out.append((pf, blob, head))
            else:
                out.append((pf, None, None))
        del rc
        return out
