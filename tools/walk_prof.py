"""Phase times of k_fsm_walk (instrumented build, DDM_AMD_LIB=.../libddm_amd_prof.so):
one C3-sized window on one partition's stream."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, "distributed-drift-detection_amd")
from ddm_amd.rng import MTStream  # noqa: E402
from ddm_amd.shuffle import GpuShuffle  # noqa: E402

dev = torch.device("cuda", 0)
sh = GpuShuffle(dev, 100, 4 << 20, 20000, torch.cuda.current_stream(dev))
sh.reset(MTStream.from_seed(7))
out = torch.zeros(20000 * 100, dtype=torch.uint8, device=dev)
for P, W in ((0, 14000), (1234567, 14000), (333, 256), (2000001, 14000)):
    sh.window(P if P < 100 else 0, W, out)      # P must be a batch boundary: windows from 0
    torch.cuda.synchronize()
    info = sh.info.cpu().numpy()
    print("W", W, "pieces", info[0], "batches", info[2], "t_phase0 %.1f us  t_phase1 %.1f us  first_load %.1f us  total %.1f us"
          % (info[3] / 100, info[4] / 100, info[6] / 100, info[5] / 100))
