"""Oracle RNG replay (test infrastructure only — see oracle/__init__.py).

ctypes front of oracle/mt_replay.c: the global MT19937 consumption of run_DDM_loop
(DDM_Process.py:187 and :190 one `permutation` per batch, :194-196 100 `randint(2**31-1)`
per refit, :207-210 a change makes the refit pending) replayed from the seed and the list
of change batches.  Used to pin configs[2]'s exact drift rows (the first new-class row of
the boundary batch IN SHUFFLED ORDER, DDM_Process.py:144-152) and the RNG position the
drop-in hands back, at sizes where re-running the whole oracle controller is too slow.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def _lib():
    global _LIB
    if _LIB is None:
        so = os.path.join(_HERE, "_build", "libddm_oracle.so")
        if not os.path.exists(so):
            subprocess.check_call(["make", "-C", _HERE])
        lib = ctypes.CDLL(so)
        vp = ctypes.c_void_p
        lib.oracle_mt_replay.restype = ctypes.c_int
        lib.oracle_mt_replay.argtypes = [ctypes.c_uint32, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                                         ctypes.c_int32, vp, ctypes.c_int64, vp, ctypes.c_int64, vp, vp, vp]
        _LIB = lib
    return _LIB


def mt_replay(seed, n_rows, changes, want=(), per_batch=100, n_estimators=100):
    """Replay one partition of n_rows rows whose DDM changed in the (batch index) list
    `changes`.  Returns ({batch: permutation int32 [len]} for each batch in `want`,
    key uint32 [624], pos) -- numpy's get_state()[1:3] after the partition."""
    nb = (int(n_rows) + per_batch - 1) // per_batch
    last = int(n_rows) - (nb - 1) * per_batch
    ch = np.ascontiguousarray(sorted(int(c) for c in changes), dtype=np.int64)
    wt = np.ascontiguousarray(sorted(int(w) for w in want), dtype=np.int64)
    perms = np.zeros((max(1, len(wt)), per_batch), dtype=np.int32)
    key = np.empty(624, dtype=np.uint32)
    pos = ctypes.c_int32()
    rc = _lib().oracle_mt_replay(int(seed) & 0xFFFFFFFF, nb, per_batch, last, n_estimators, ch.ctypes.data,
                                 len(ch), wt.ctypes.data, len(wt), perms.ctypes.data, key.ctypes.data,
                                 ctypes.byref(pos))
    if rc != 0:
        raise ValueError("oracle_mt_replay: bad arguments")
    out = {}
    for k, b in enumerate(wt):
        out[int(b)] = perms[k, :(last if b == nb - 1 else per_batch)].copy()
    return out, key, int(pos.value)
