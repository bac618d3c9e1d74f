"""ddm_scan_batches bookkeeping on the C4 stream: listed streams, deferred streams, queue
lengths (scratch counters), for tuning.  Runs on the GPU box."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "distributed-drift-detection_amd"))
from ddm_amd import kernels  # noqa: E402

S, L = 1000000, 4096
dev = torch.device("cuda", 0)
err = torch.empty(S * L + 16, dtype=torch.uint8, device=dev)
kernels.synth_bernoulli_streams(err, S, L, 1234)
nb = (L + 99) // 100
ev = torch.empty((S * nb, 2), dtype=torch.int32, device=dev)
scratch = torch.empty(kernels.scan_batches_scratch_size(S, L), dtype=torch.uint8, device=dev)
state = torch.from_numpy(kernels.fresh_states(S).view(np.uint8)).to(dev)
kernels.scan_batches(err, S, L, kernels.params_struct(), state, ev, scratch)
torch.cuda.synchronize()
ctr = scratch[:16].cpu().numpy().view(np.uint32)
print("listed", ctr[0], "deferred", ctr[2], "changes", int((ev[:, 1] >= 0).sum().item()), "items", S * nb)
