"""Oracle DDM scan (test infrastructure only — see oracle/__init__.py).

ctypes front of oracle/ddm_scan.c (run_DDM, DDM_Process.py:135-159, with the reset of
:207-210 in mode 1), threaded over contiguous runs of equal-length streams so that a
whole configs[3] call (1M streams x 4096 rows, ~13 s on one core) is checked in a few
seconds.  Used by tests/test_gpu_scan_batches.py and by bench.py's post-timed c4 check.
"""
import ctypes
import os
import subprocess
from concurrent.futures import ThreadPoolExecutor

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
        lib.oracle_ddm_scan.restype = ctypes.c_int
        lib.oracle_ddm_scan.argtypes = [vp, vp, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_double,
                                        ctypes.c_double, ctypes.c_int32, vp, vp, vp, vp]
        _LIB = lib
    return _LIB


def scan_equal_streams(err, n_streams, L, per_batch=100, mode=1, min_inst=3, wl=0.5, cl=1.5, threads=8):
    """The C oracle over n_streams back-to-back streams of L rows (err uint8, at least
    n_streams * L bytes).  Returns (events int32 [n_streams * nb, 2], state float64
    [n_streams, 8]: p, s, p_min, s_min, ps_min, n, change, warn).  The streams are cut into
    `threads` contiguous runs scanned in parallel (ctypes drops the GIL)."""
    err = np.ascontiguousarray(err, dtype=np.uint8)
    assert err.size >= n_streams * L
    nb = (L + per_batch - 1) // per_batch
    ev = np.empty((n_streams * nb, 2), dtype=np.int32)
    st = np.empty((n_streams, 8), dtype=np.float64)
    stop = np.empty(n_streams, dtype=np.int32)
    lib = _lib()
    cuts = np.linspace(0, n_streams, max(1, int(threads)) + 1).astype(np.int64)

    def run(k):
        a, b = int(cuts[k]), int(cuts[k + 1])
        if b <= a:
            return 0
        off = np.arange(b - a + 1, dtype=np.int64) * L
        return lib.oracle_ddm_scan(err.ctypes.data + a * L, off.ctypes.data, b - a, per_batch, min_inst, wl, cl,
                                   mode, ev.ctypes.data + 8 * a * nb, stop.ctypes.data + 4 * a,
                                   st.ctypes.data + 64 * a, None)

    with ThreadPoolExecutor(max_workers=len(cuts) - 1) as pool:
        rcs = list(pool.map(run, range(len(cuts) - 1)))
    if any(rcs):
        raise ValueError("oracle_ddm_scan failed")
    return ev, st
