"""Debug aid: device-resident vs host epochs on one synthetic case; prints the first
differing batch of every partition and the runner statistics."""
import sys
import os
sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "..",
                                                                            "distributed-drift-detection_amd")]
import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
from test_gpu_devctl import _parts, _run  # noqa: E402

case = sys.argv[1] if len(sys.argv) > 1 else "jitter"
if case == "jitter":
    parts = _parts((24_000,) * 4, 27, 0, 5, jitter=True)
elif case == "noise":
    parts = _parts((30_000, 30_000), 27, 0, 7, flip=0.01, jitter=True)
else:
    parts = _parts((24_037, 17_055, 4_321, 9_999), 27, 6_007, 9)
seeds = [100 + k for k in range(len(parts))]
import ddm_amd.devctl as dc
if len(sys.argv) > 2:
    dc.GROUP = int(sys.argv[2])
d_out, d_rng, st = _run(parts, True, seeds)
h_out, h_rng, sh = _run(parts, False, seeds)
print("device stats", {k: getattr(st, k) for k in ("epochs", "device_epochs", "device_phases", "refits")})
print("host stats", {k: getattr(sh, k) for k in ("epochs", "refits")})
for k in range(len(parts)):
    a, b = d_out[k], h_out[k]
    bad = np.nonzero((a != b).any(axis=1))[0]
    if len(bad) == 0:
        print(k, "equal", (a[:, 1] >= 0).sum(), "drifts")
        continue
    f = bad[0]
    print(k, "first diff at out row", f, "of", len(a), "n diff", len(bad))
    print("  device", a[max(0, f - 4):f + 3].tolist())
    print("  host  ", b[max(0, f - 4):f + 3].tolist())
    print("  host drift rows before:", np.nonzero(b[:f, 1] >= 0)[0][-6:].tolist())
