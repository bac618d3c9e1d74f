"""Window-shuffle microbenchmark (developer tool): ddm_shuffle_window_batch for 8 partitions'
windows of W batches (C3's steady windows: W = 12,500), HIP events around the batched call,
and the per-kernel split from a rocprofv3 trace when run under it.
    python tools/bench_shuffle.py [W] [variant .so]"""
import os
import sys

if len(sys.argv) > 2:
    os.environ["DDM_AMD_LIB"] = os.path.abspath(sys.argv[2])
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-drift-detection_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from ddm_amd import kernels  # noqa: E402
from ddm_amd._capi import check, lib  # noqa: E402
from ddm_amd.rng import MTStream  # noqa: E402
from ddm_amd.shuffle import GpuShuffle  # noqa: E402

W = int(sys.argv[1]) if len(sys.argv) > 1 else 12_500
CAP = int(os.environ.get("SHUF_PIECE_CAP", 256))     # the replay grid's cap (ctl.hip kShufPieces)
L, n = 100, 8
dev = torch.device("cuda", 0)
stream = torch.cuda.current_stream(dev)
shs, perms = [], []
for k in range(n):
    sh = GpuShuffle(dev, L, int(W * 160 * 1.3), W, stream)
    sh.reset(MTStream.from_seed(100 + k))
    sh.ensure(sh.window_draws(W))
    shs.append(sh)
    perms.append(torch.empty(W * L, dtype=torch.uint8, device=dev))
torch.cuda.synchronize()
rec = np.zeros(n, dtype=kernels.JOB_DTYPE)
for k, sh in enumerate(shs):
    rec[k] = sh.job_tuple(1000 + 37 * k, W, perms[k].data_ptr())
jobs = torch.from_numpy(rec.view(np.uint8)).to(dev)
max_pieces = max(sh.max_pieces for sh in shs)
for it in range(3):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        check(lib.ddm_shuffle_window_batch(jobs.data_ptr(), n, W, min(max_pieces, CAP), L,
                                           torch.cuda.current_stream(dev).cuda_stream, None, None),
              "ddm_shuffle_window_batch")
    e1.record()
    torch.cuda.synchronize()
    print(f"W={W}: {e0.elapsed_time(e1) / 10 * 1e3:.1f} us per batched window shuffle (8 jobs)", flush=True)
# parity: each job's perms == the host Fisher-Yates from the same draws (production build)
for k, sh in enumerate(shs[:2] if len(sys.argv) <= 2 else []):
    host, _ = sh.host_perm(1000 + 37 * k, L)
    assert np.array_equal(perms[k][:L].cpu().numpy(), host), k
print("first batches == host perms")
