"""Phase times of the device refit (instrumented build: tools/build_variant.sh dprof
rf_device.hip -DDDM_DFIT_PROFILE, then DDM_AMD_LIB=.../libddm_amd_dprof.so): a C3-like
drift batch (100 rows x 27 features, two classes), 8 jobs of 100 trees.  `stumps` as the
argument: every feature separates the classes (C3's trees: all stumps)."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, "distributed-drift-detection_amd")
from ddm_amd.dfit import DeviceTrainer  # noqa: E402

rng = np.random.default_rng(3)
batches = []
if "outdoor" in sys.argv:
    # c2-like: 16 partitions (row % 16) of the reference's outdoorStream rows, one 100-row
    # batch each (shuffled), ~9 classes per batch
    d = np.load("tests/golden/outdoor.npz", allow_pickle=False)
    Xo, yo = d["X"].astype(np.float32), d["target"].astype(np.int64)
    for k in range(16):
        rows = np.arange(k, len(yo), 16)[:100]
        rows = rows[rng.permutation(len(rows))]
        batches.append((Xo[rows], yo[rows], rng.integers(0, 2**31 - 1, 100)))
else:
    for k in range(8):
        y = np.where(np.arange(100) < 60, 3, 4)
        X = rng.random((100, 27), dtype=np.float32) + (y[:, None] == 4) * (10.0 if "stumps" in sys.argv else 0.5)
        batches.append((X.astype(np.float32), y, rng.integers(0, 2**31 - 1, 100)))
tr = DeviceTrainer(100, 64, torch.device("cuda", 0), fused="fused" in sys.argv)
for rep in range(3):
    t = time.perf_counter()
    out = tr.fit_many(batches)
    dt = time.perf_counter() - t
    r = out[0][3]
    a, p = int(r[10]), int(r[11])
    print(f"fit_many {dt*1e3:.2f} ms; tree 0: rng init {(a & 0xffff)/100:.1f} us, bootstrap {((a >> 16) & 0xffff)/100:.1f} us, "
          f"build {((a >> 32) & 0xffff)/100:.1f} us, init_genrand {(a >> 48)/100:.1f} us; pack: bfs {(p & 0xffff)/100:.1f} us, compile {((p >> 16) & 0xffff)/100:.1f} us "
          f"(A/B-C/zero/D {', '.join(str(((p >> (32 + 8 * i)) & 255) * 0.08)[:4] for i in range(4))} us); "
          f"nodes {int(r[2])}, blob {int(r[5])}")
    if "prep" in sys.argv:    # a DDM_PREP_PROFILE build: presort / boot timings of job 0
        a, b = int(r[10]) & ((1 << 64) - 1), int(r[11]) & ((1 << 64) - 1)
        f = [((b >> (16 * i)) & 0xffff) / 100 for i in range(4)]
        print(f"  presort: classes {((a >> 40) & 0xfff) / 100:.1f} us, end {(a >> 52) / 100:.1f} us; "
              f"boot tree 0: init done {f[0]:.1f}, twist done {f[1]:.1f}, draws done {f[2]:.1f}, end {f[3]:.1f} us")
