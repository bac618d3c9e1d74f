"""Microbenchmark of the predict kernels on one GPU (developer tool, not the bench).

Times ddm_forest_predict over N rows for a few forest shapes (single leaves, the C3
stump forest, a deeper rialto-like forest), compiled and node-walk, and prints GB/s of
algorithmic bytes (4*slots + 6 per row)."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-drift-detection_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
from sklearn.ensemble import RandomForestClassifier  # noqa: E402

from ddm_amd import kernels  # noqa: E402
from ddm_amd.forest import DeviceForest, pack_sklearn  # noqa: E402


def forests(F, rs):
    y = np.repeat([0, 1], 50)
    base = 0.05 + 0.1 * ((y[:, None] * 7 + np.arange(F) * 3) % 10)
    out = {}
    out["leaf"] = RandomForestClassifier(random_state=1).fit(base[:50], y[:50])
    out["stumps"] = RandomForestClassifier(random_state=1).fit(base + 0.04 * rs.rand(100, F), y)
    yk = np.sort(rs.randint(0, 10, 100))
    out["deep10"] = RandomForestClassifier(random_state=1).fit(rs.rand(100, F) + 0.3 * yk[:, None] / 10, yk)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=64_000_000)
    ap.add_argument("--features", type=int, default=27)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--only", default=None, help="forest name (leaf/stumps/deep10), compiled path only")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    rs = np.random.RandomState(0)
    n, F = a.rows, a.features
    X = torch.rand((F, n), device=dev, dtype=torch.float32)
    y = torch.randint(0, 2, (n,), device=dev, dtype=torch.int32)
    perm = torch.from_numpy(np.tile(rs.permutation(100).astype(np.uint8), n // 100 + 1)[:n]).to(dev)
    err = torch.empty(n + 16, dtype=torch.uint8, device=dev)
    first = torch.empty(1, dtype=torch.int64, device=dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for name, rf in forests(F, rs).items():
        if a.only and name != a.only:
            continue
        pf = pack_sklearn(rf)
        for compiled in ((True,) if a.only else (True, False)):
            f = DeviceForest(pf, dev, compiled=compiled)
            nbytes = n * (4 * f.features_read + 6)
            kernels.forest_predict(X, y, perm, 0, n, 100, f, err, first_err=first)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(a.reps):
                kernels.forest_predict(X, y, perm, 0, n, 100, f, err, first_err=first)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.reps
            print(f"{name:8s} compiled={compiled!s:5s} slots={f.features_read:2d} "
                  f"head={f.head and {k: f.head[k] for k in ('n_stumps', 'n_general', 'n_leaves')}} "
                  f"{ms:8.3f} ms  {n / ms / 1e6:8.2f} Mrows/ms  {nbytes / ms / 1e6:8.1f} GB/s", flush=True)
            if not compiled and name == "deep10":
                break


if __name__ == "__main__":
    t = time.time()
    main()
    print(f"total {time.time() - t:.1f} s")
