"""Fixed cost of the device refit's launches (developer tool): 8 jobs of C3-like separable
100 x 27 batches, every job real or every job gated off (*gate < 0), timed back to back on
one stream; run under rocprofv3 --kernel-trace --stats for the per-kernel split.
    python tools/refit_overhead.py [--reps 200]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-drift-detection_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench_refit import batches  # noqa: E402
from ddm_amd.dfit import DFIT_DTYPE, RESULT_WORDS, RefitBuffers, fit_device  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    rs = np.random.RandomState(0)
    stream = torch.cuda.current_stream(dev)
    bs = batches("separable", 8, rs)
    keep, recs = [], []
    res = torch.zeros((8, RESULT_WORDS), dtype=torch.int64, device=dev)
    gate = torch.zeros(8, dtype=torch.int64, device=dev)
    for k, (X, y, seeds) in enumerate(bs):
        xd = torch.from_numpy(X).to(dev)
        yd = torch.from_numpy(y.astype(np.int32)).to(dev)
        sd = torch.from_numpy(seeds.astype(np.int64)).to(dev)
        b = RefitBuffers(100, 27, 100, 16, dev)
        keep.append((xd, yd, sd, b))
        recs.append(b.record(xd.data_ptr(), yd.data_ptr(), sd.data_ptr(), res[k].data_ptr(),
                             gate=gate.data_ptr() + 8 * k))
    table = torch.from_numpy(np.array(recs, dtype=DFIT_DTYPE).view(np.uint8)).to(dev)
    torch.cuda.synchronize()
    for label, g in (("real", 0), ("gated", -1), ("real", 0), ("gated", -1)):
        gate.fill_(g)
        for _ in range(5):
            fit_device(table, 8, 100, stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(a.reps):
            fit_device(table, 8, 100, stream)
        e1.record(stream)
        torch.cuda.synchronize()
        print(f"{label:6s} {e0.elapsed_time(e1) / a.reps * 1e3:8.1f} us per refit call (prep + trees + pack, 8 jobs)",
              flush=True)


if __name__ == "__main__":
    main()
