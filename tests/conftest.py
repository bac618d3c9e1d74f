import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_ROOT = os.path.join(ROOT, "distributed-drift-detection_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG_ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


# Tests that start other Python processes on the GPU run first, while this process has
# not initialised the GPU itself (a GPU-initialised process must not exec programs).
SPAWNING_MODULES = ("test_gpu_scaling.py", "test_gpu_dist.py::test_two_ranks")


def pytest_collection_modifyitems(config, items):
    items.sort(key=lambda it: 0 if any(m in it.nodeid for m in SPAWNING_MODULES) else 1)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running parity sweep")


@pytest.fixture(scope="session")
def oracle_lib():
    so = os.path.join(ROOT, "oracle", "_build", "libddm_oracle.so")
    if not os.path.exists(so):
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "oracle")])
    import ctypes
    lib = ctypes.CDLL(so)
    lib.oracle_ddm_scan.restype = ctypes.c_int
    vp = ctypes.c_void_p
    lib.oracle_ddm_scan.argtypes = [vp, vp, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_double,
                                    ctypes.c_double, ctypes.c_int32, vp, vp, vp, vp]
    return lib


def oracle_scan_c(lib, err, offsets, per_batch=100, mode=0, min_inst=3, wl=0.5, cl=1.5, trace=False):
    """Run oracle/ddm_scan.c; returns (events [nb_total,2] int32, stop [n] int32, state [n,8], ps)."""
    err = np.ascontiguousarray(err, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.int64)
    lens = np.diff(offsets)
    nb = (lens + per_batch - 1) // per_batch
    ev = np.empty((int(nb.sum()), 2), dtype=np.int32)
    stop = np.empty(len(lens), dtype=np.int32)
    st = np.empty((len(lens), 8), dtype=np.float64)
    ps = np.empty((len(err), 2), dtype=np.float64) if trace else None
    rc = lib.oracle_ddm_scan(err.ctypes.data, offsets.ctypes.data, len(lens), per_batch, min_inst, wl, cl, mode,
                             ev.ctypes.data, stop.ctypes.data, st.ctypes.data,
                             ps.ctypes.data if trace else None)
    assert rc == 0
    return ev, stop, st, ps


def load_npz(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def golden_configs():
    return [(m, i) for m in (1, 2, 4) for i in (1, 2, 4, 8, 16)]


def golden_partitions(mult, inst):
    """Rebuild the reference's partition frames (DDM_Process.py:220-226) from the fixtures."""
    import pandas as pd
    data = load_npz("outdoor.npz")
    cfg = load_npz(f"outdoor_cfg_m{mult}_i{inst}.npz")
    X, target = data["X"], data["target"]
    order = cfg["order"].astype(np.int64)
    F = X.shape[1]
    full = pd.DataFrame(X[order], columns=[str(i) for i in range(F)])
    full["target"] = target[order]
    full["full_df_row_number"] = order
    full["device_id"] = (order % inst).astype(np.int32)
    parts = []
    for d in range(inst):
        part = full[full["device_id"] == d].reset_index(drop=True)
        key = f"events/{d}"
        expect = cfg[key] if key in cfg.files else None
        parts.append((d, part, expect))
    return parts
