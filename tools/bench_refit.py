"""Refit microbenchmark (developer tool): 8 partitions' refits of C3-like batches on the
host trainer (ddm_rf_fit_many) and on the device (ddm_rf_fit_device)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-drift-detection_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from ddm_amd.dfit import DFIT_DTYPE, RESULT_WORDS, RefitBuffers, fit_device  # noqa: E402
from ddm_amd.trainer import BatchForestTrainer  # noqa: E402


def batches(kind, n, rs, L=100, F=27):
    out = []
    for k in range(n):
        if kind == "separable":
            y = np.repeat([k % 10, (k + 1) % 10], L // 2)
            X = 0.05 + 0.1 * ((y[:, None] * 7 + np.arange(F) * 3) % 10) + 0.04 * rs.rand(L, F)
        else:
            y = rs.randint(0, 10, L)
            X = rs.rand(L, F) + 0.3 * y[:, None] / 10
        out.append((X.astype(np.float32), y, rs.randint(0, 2**31 - 1, 100)))
    return out


def main():
    dev = torch.device("cuda", 0)
    rs = np.random.RandomState(0)
    stream = torch.cuda.current_stream(dev)
    for kind in ("separable", "noisy"):
        bs = batches(kind, 8, rs)
        tr = BatchForestTrainer(100, 16)
        tr.fit_many(bs)
        t = time.perf_counter()
        for _ in range(10):
            tr.fit_many(bs)
        host_ms = (time.perf_counter() - t) / 10 * 1e3
        res = torch.zeros((8, RESULT_WORDS), dtype=torch.int64, device=dev)
        keep, recs = [], []
        for k, (X, y, s) in enumerate(bs):
            xd, yd, sd = (torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (X, y.astype(np.int32), s))
            b = RefitBuffers(100, 27, 100, 16, dev)
            keep.append((xd, yd, sd, b))
            recs.append(b.record(xd.data_ptr(), yd.data_ptr(), sd.data_ptr(), res[k].data_ptr()))
        table = torch.from_numpy(np.array(recs, dtype=DFIT_DTYPE).view(np.uint8)).to(dev)
        torch.cuda.synchronize()
        for max_lf, label in ((-1, "prep+trees+pack"), (100 * 27, "fused prep")):
            fit_device(table, 8, 100, stream, max_lf)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                fit_device(table, 8, 100, stream, max_lf)
            e1.record()
            torch.cuda.synchronize()
            print(f"{kind:10s} host fit_many {host_ms:.3f} ms   device ({label}) {e0.elapsed_time(e1) / 10:.3f} ms   "
                  f"status {res[:, 0].tolist()} blob {res[:, 5].tolist()}", flush=True)


if __name__ == "__main__":
    main()
