"""Native refit backend: train_rf (DDM_Process.py:98-105) via ddm_rf_fit (csrc/rf_fit.cpp),
an exact restatement of scikit-learn 1.7.2's RandomForestClassifier.fit.

The reference fits `RandomForestClassifier(n_jobs=CORES)` with random_state=None, i.e. it
draws the 100 per-tree seeds from numpy's global RandomState; the controller reads them
from the partition's MT19937 stream, then the trees are grown natively (the call releases
the GIL, so partition threads refit in parallel) and come back already packed for
ddm_forest_predict.  Inputs containing NaN (missing values) return None: the controller
then refits with sklearn itself.
"""
import ctypes

import numpy as np

from ._capi import DDM_E_IMPURE, DDM_E_NAN, check, lib
from .treepack import MAX_CLASSES, NODE_DTYPE, PackedForest


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
        if classes.size > MAX_CLASSES:
            raise ValueError(f"{classes.size} classes > {MAX_CLASSES}")
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

