"""Time ddm_scan_certified (and ddm_scan_long once) on 10M-row carried thinning streams
(tests/test_gpu_scan_long.py's streams).  Run under rocprofv3 --kernel-trace --stats for the
per-kernel split:  python tools/bench_scan_cert.py [--reps 20] [--exact]"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "distributed-drift-detection_amd"))
from ddm_amd import kernels  # noqa: E402


def thinning_stream(n, a, jitter_seed=None):
    k = np.arange(int(n ** (1 / a)) + 2)
    pos = np.floor(k ** a).astype(np.int64)
    pos = pos[pos < n]
    e = np.zeros(n, np.uint8)
    e[pos] = 1
    if jitter_seed is not None:
        rs = np.random.RandomState(jitter_seed)
        mv = pos[(rs.rand(len(pos)) < 0.3) & (pos > 10) & (pos < n - 1)]
        e[mv] = 0
        e[mv + 1] = 1
    return e


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--streams", type=int, default=1)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--exact", action="store_true", help="also time ddm_scan_long once")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    n, S = a.rows, a.streams
    e = np.concatenate([thinning_stream(n, 1.5, jitter_seed=15 + s) for s in range(S)])
    pad = np.zeros(len(e) + 32, np.uint8)
    pad[:len(e)] = e
    err = torch.from_numpy(pad).to(dev)
    off = torch.arange(S + 1, dtype=torch.int64, device=dev) * n
    nb = (n + 99) // 100
    base = torch.arange(S, dtype=torch.int64, device=dev) * nb
    prm = kernels.params_struct(3, 100)
    st0 = torch.from_numpy(kernels.fresh_states(S).view(np.uint8).copy()).to(dev)
    ev = torch.empty((S * nb, 2), dtype=torch.int32, device=dev)
    stop = torch.empty(S, dtype=torch.int32, device=dev)
    nev = torch.empty(S, dtype=torch.int64, device=dev)
    status = torch.empty(S, dtype=torch.int32, device=dev)
    scratch = torch.empty(kernels.scan_certified_scratch_size(S, n, 100), dtype=torch.uint8, device=dev)
    ms = []
    for _ in range(a.reps):
        st = st0.clone()
        t = kernels.LaunchTimer()
        kernels.scan_certified(err, off, prm, st, base, ev, n, scratch, stop=stop, nev=nev, mode=0, status=status,
                               timer=t)
        torch.cuda.synchronize()
        ms.append(t.elapsed_ms())
    print(f"ddm_scan_certified {S} x {n} rows: median {np.median(ms):.3f} ms, min {min(ms):.3f} ms, "
          f"status {status.cpu().numpy().tolist()}")
    if a.exact:
        st = st0.clone()
        sc = torch.empty(kernels.scan_long_scratch_size(S, n, 100), dtype=torch.uint8, device=dev)
        t = kernels.LaunchTimer()
        kernels.scan_long(err, off, prm, st, base, ev, n, sc, stop=stop, nev=nev, mode=0, timer=t)
        torch.cuda.synchronize()
        print(f"ddm_scan_long {S} x {n} rows: {t.elapsed_ms():.1f} ms")


if __name__ == "__main__":
    main()
