"""C4 (configs[3]) ddm_scan_batches probe: time per call of the one-pass kernel and the
round-2 kernels on the same device-generated streams, events compared, and the one-pass
kernel's path counters (scratch words: replay anomalies, certified batches, uncertified
batches, end-state replays)."""
import os
import sys

import numpy as np
import torch

if len(sys.argv) > 2:                       # a variant library (tools/build_variant.sh)
    os.environ["DDM_AMD_LIB"] = os.path.abspath(sys.argv[2])
sys.path.insert(0, "distributed-drift-detection_amd")
from ddm_amd import kernels  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
L = 4096
dev = torch.device("cuda", 0)
err = torch.empty(S * L + 16, dtype=torch.uint8, device=dev)
kernels.synth_bernoulli_streams(err, S, L, 20261015)
nb = (L + 99) // 100
prm = kernels.params_struct()
st0 = torch.from_numpy(kernels.fresh_states(S).view(np.uint8)).to(dev)
out = {}
for v1 in ((False, True) if len(sys.argv) <= 3 else (False,)):
    ev = torch.empty((S * nb, 2), dtype=torch.int32, device=dev)
    st = st0.clone()
    sc = torch.zeros(kernels.scan_batches_scratch_size(S, L, v1=v1), dtype=torch.uint8, device=dev)
    times = []
    for k in range(4):
        st.copy_(st0)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        kernels.scan_batches(err, S, L, prm, st, ev, sc, v1=v1)
        e1.record()
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1))
    out[v1] = (ev.cpu().numpy(), st.cpu().numpy())
    cnt = sc[:16].cpu().numpy().view(np.uint32) if not v1 else None
    print(f"{'v1' if v1 else 'onepass'}: ms per call {['%.3f' % t for t in times]}; counters {cnt}")
if len(out) > 1:
    print("events equal:", np.array_equal(out[False][0], out[True][0]),
          "states equal:", np.array_equal(out[False][1], out[True][1]))
