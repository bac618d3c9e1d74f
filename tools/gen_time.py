"""Time the stream generation's kernels alone (developer tool): ddm_mt_jump over n jobs of
2^20-draw segment jumps from random keys, and ddm_shuffle_tables (k_fsm_prefix) over random
words; HIP events around each launch; prints ms per launch and digests of the outputs
(equal across library builds when the kernels agree).
    [DDM_AMD_LIB=...] python tools/gen_time.py [n_jobs ...]"""
import ctypes
import hashlib
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "distributed-drift-detection_amd"))
from ddm_amd import kernels  # noqa: E402
from ddm_amd._capi import check, lib  # noqa: E402
from ddm_amd.shuffle import JUMP  # noqa: E402

dev = torch.device("cuda:0")
stream = torch.cuda.Stream(dev)
out = {"lib": os.environ.get("DDM_AMD_LIB", "default")}
for n in [int(a) for a in sys.argv[1:]] or [168, 256, 768, 1344]:
    rng = np.random.default_rng(n)
    keys = torch.from_numpy(rng.integers(0, 2**32, (n, 640), dtype=np.uint64).astype(np.uint32).view(np.int32)).to(dev)
    polys = kernels.mt_jump_polys(JUMP, n, dev)
    res = torch.zeros((n, 640), dtype=torch.int32, device=dev)
    tab = kernels.PinnedTable(kernels.JUMP_DTYPE, n, dev)
    idx = np.arange(n, dtype=np.uint64)
    tab.rec["key"] = keys.data_ptr() + idx * 640 * 4
    tab.rec["poly"] = polys.data_ptr() + idx * 8 * kernels.POLY_WORDS
    tab.rec["out"] = res.data_ptr() + idx * 640 * 4
    tab.rec["scratch"] = 0
    torch.cuda.synchronize()
    times = []
    for rep in range(6):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        kernels.mt_jump(tab, n, stream)
        e1.record(stream)
        e1.synchronize()
        times.append(e0.elapsed_time(e1))
    r = res.cpu().numpy()[:, :625].copy()
    r[:, 0] &= np.int32(-2**31)            # only the top bit of word 0 is state
    out[str(n)] = {"ms": round(float(np.median(times[1:])), 4), "sha1": hashlib.sha1(r.tobytes()).hexdigest()[:16]}
for nchunk in (256, 2048):
    L, S = 100, 99
    R = torch.from_numpy(np.random.default_rng(nchunk).integers(0, 2**32, nchunk * 8192, dtype=np.uint64)
                         .astype(np.uint32).view(np.int32)).to(dev)
    Tpre = torch.zeros(nchunk * 64 * S, dtype=torch.int32, device=dev)
    Tc = torch.zeros(nchunk * S + 4, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    times = []
    for rep in range(4):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        check(lib.ddm_shuffle_tables(R.data_ptr(), 0, nchunk, L, Tpre.data_ptr(), Tc.data_ptr(),
                                     ctypes.c_void_p(stream.cuda_stream)), "ddm_shuffle_tables")
        e1.record(stream)
        e1.synchronize()
        times.append(e0.elapsed_time(e1))
    ms = float(np.median(times[1:]))
    out[f"tables_{nchunk}"] = {"ms": round(ms, 4), "GB_per_s": round(nchunk * (8192 * 4 + 65 * S * 4) / ms / 1e6, 1),
                               "sha1": hashlib.sha1(Tpre.cpu().numpy().tobytes()).hexdigest()[:16]}
# the batched form the runner uses: 8 partitions' pieces of 1,024 chunks in one launch
nj, nchunk, L, S = 8, 1024, 100, 99
Rs = [torch.from_numpy(np.random.default_rng(100 + k).integers(0, 2**32, nchunk * 8192, dtype=np.uint64)
                       .astype(np.uint32).view(np.int32)).to(dev) for k in range(nj)]
Tps = [torch.zeros(nchunk * 64 * S, dtype=torch.int32, device=dev) for _ in range(nj)]
Tcs = [torch.zeros(nchunk * S + 4, dtype=torch.int32, device=dev) for _ in range(nj)]
tt = kernels.PinnedTable(kernels.TAB_DTYPE, nj, dev)
tt.rec[:nj] = np.array([(R.data_ptr(), 0, nchunk, Tp.data_ptr(), Tc.data_ptr()) for R, Tp, Tc in zip(Rs, Tps, Tcs)],
                       dtype=kernels.TAB_DTYPE)
torch.cuda.synchronize()
times = []
for rep in range(4):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    kernels.shuffle_tables_batch(tt, nj, nchunk, L, stream)
    e1.record(stream)
    e1.synchronize()
    times.append(e0.elapsed_time(e1))
ms = float(np.median(times[1:]))
h = hashlib.sha1()
for Tp in Tps:
    h.update(Tp.cpu().numpy().tobytes())
out["tables_batch_8x1024"] = {"ms": round(ms, 4), "GB_per_s": round(nj * nchunk * (8192 * 4 + 65 * S * 4) / ms / 1e6, 1),
                              "sha1": h.hexdigest()[:16]}
print(json.dumps(out))
