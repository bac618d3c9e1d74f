"""Host refit backends for train_rf (DDM_Process.py:98-105).  numpy + sklearn only: this
module is imported by spawn-started worker processes that never touch the GPU.

The reference fits `RandomForestClassifier(n_jobs=CORES)` on the shuffled drift batch with
random_state=None, i.e. numpy's global RandomState, which the partition's MT19937 stream
stands in for: the fit draws its 100 tree seeds from the stream (key, pos) and the new
(key, pos) is handed back so the next batch shuffle continues from the right position.
"""
import multiprocessing as mp

import numpy as np

from .treepack import pack_sklearn


def fit_packed(X32, y, key, pos, n_estimators=100, n_jobs=1):
    from sklearn.ensemble import RandomForestClassifier
    rs = np.random.RandomState()
    rs.set_state(("MT19937", np.asarray(key, dtype=np.uint32), int(pos), 0, 0.0))
    rf = RandomForestClassifier(n_estimators=n_estimators, n_jobs=n_jobs, random_state=rs)
    rf.fit(X32, y)
    st = rs.get_state()
    return pack_sklearn(rf), st[1], int(st[2])


def _warm(_):
    import sklearn.ensemble  # noqa: F401
    return 0


class RefitPool:
    """sklearn refits in P spawn-started processes (create it BEFORE the GPU is initialised).
    Partition threads block on their own refit while the others keep the GPU busy."""

    def __init__(self, processes, n_estimators=100, n_jobs=1):
        self.pool = mp.get_context("spawn").Pool(processes)
        self.pool.map(_warm, range(processes))
        self.n_estimators, self.n_jobs = n_estimators, n_jobs

    def __call__(self, X32, y, rng):
        packed, key, pos = self.pool.apply(fit_packed, (np.ascontiguousarray(X32), np.asarray(y), rng.key,
                                                        int(rng.pos.value), self.n_estimators, self.n_jobs))
        rng.key[:] = key
        rng.pos.value = pos
        return packed

    def close(self):
        self.pool.close()
        self.pool.join()
