"""One long mode-1 stream on the GPU: segments scanned by ddm_scan_batches and the carries
resolved (ddm_amd/longstream.py) == the C oracle's sequential scan of the whole stream:
events bit for bit; the end state bit for bit when its bound is 0 (exact rescans, p stuck at
0 or 1) and within 1e-12 relative otherwise (certified rescans, north_star)."""
import time

import numpy as np
import pytest
import torch

from conftest import oracle_scan_c
from test_gpu_scan_long import thinning_stream
from test_longstream import long_stream

pytestmark = pytest.mark.gpu


def _end_vec(end):
    return np.array([end["miss_prob"], end["miss_std"], end["miss_prob_min"], end["miss_sd_min"],
                     end["miss_prob_sd_min"], end["sample_count"], end["in_concept_change"], end["in_warning_zone"]],
                    dtype=np.float64)


def check_end(end, bound, want):
    got = _end_vec(end)
    assert np.array_equal(got[5:], want[5:])
    if not np.any(bound):
        np.testing.assert_array_equal(got, want)
        return
    fin = np.isfinite(want[:5])
    assert np.array_equal(np.isfinite(got[:5]), fin)
    assert np.all(np.abs(got[:5][fin] - want[:5][fin]) <= 1e-12 * np.abs(want[:5][fin]))
    assert abs(got[0] - want[0]) <= bound[0]


@pytest.mark.parametrize("n,seg_batches", [(2_000_000, 64), (1_234_567, 16)])
def test_device_segments_equal_oracle(oracle_lib, n, seg_batches):
    from ddm_amd import kernels
    from ddm_amd.longstream import DeviceScanner, scan_long_stream
    err = long_stream(n % 1000, n)
    dev = torch.device("cuda", 0)
    pad = np.zeros(((n + 15) // 16) * 16 + 16, np.uint8)
    pad[:n] = err
    e = torch.from_numpy(pad).to(dev)
    oev, _, ost, _ = oracle_scan_c(oracle_lib, err, np.array([0, n], dtype=np.int64), mode=1)
    hit = np.nonzero(oev[:, 1] >= 0)[0]
    for certified in (True, False):
        ev, end, first, bd = scan_long_stream(DeviceScanner(e, kernels.params_struct(), certified=certified), n, 100,
                                              seg_batches=seg_batches, with_bound=True)
        assert np.array_equal(ev, oev)
        check_end(end, bd, ost[0])
        assert first == (int(hit[0]) if len(hit) else -1)


def test_noisy_carried_stretch_certified(oracle_lib):
    """A stream whose middle is a 3M-row detector carried without a change (errors thinning
    out): the carried rescans are certified (no decision left inside its bound; runs with
    more than four changes are handed on by design) and much faster than the exact chain,
    with the same events."""
    from ddm_amd import kernels
    from ddm_amd.longstream import DeviceScanner, scan_long_stream
    rs = np.random.RandomState(4)
    head = (rs.rand(400_000) < 0.2).astype(np.uint8)               # reset-heavy
    mid = thinning_stream(3_000_000, 1.4, jitter_seed=8)           # carried, never changes
    tail = (rs.rand(600_000) < 0.3).astype(np.uint8)
    err = np.concatenate([head, mid, tail])
    n = len(err)
    dev = torch.device("cuda", 0)
    pad = np.zeros(((n + 15) // 16) * 16 + 16, np.uint8)
    pad[:n] = err
    e = torch.from_numpy(pad).to(dev)
    oev, _, ost, _ = oracle_scan_c(oracle_lib, err, np.array([0, n], dtype=np.int64), mode=1)
    walls = {}
    for certified in (True, False):
        sc = DeviceScanner(e, kernels.params_struct(), certified=certified)
        scan_long_stream(sc, n, 100, seg_batches=64)                 # warm-up
        t = time.perf_counter()
        ev, end, first, bd = scan_long_stream(sc, n, 100, seg_batches=64, with_bound=True)
        walls[certified] = time.perf_counter() - t
        assert np.array_equal(ev, oev)
        check_end(end, bd, ost[0])
        if certified:
            assert sc.status[1] == 0 and sc.status[0] > 0, sc.status
    print(f"4M-row stream with a 3M-row carried stretch: certified {walls[True] * 1e3:.1f} ms, "
          f"exact {walls[False] * 1e3:.1f} ms (wall, host resolution included)")
    assert walls[True] * 3 < walls[False]


def test_device_segments_under_rccl_world_one(oracle_lib):
    """The distributed path (carry all-gather, first-change all-reduce) under the `nccl`
    (RCCL) backend the driver's multi-GPU runs use: device tensors for the collectives."""
    import os
    import socket

    import torch.distributed as dist

    from ddm_amd import kernels
    from ddm_amd.longstream import DeviceScanner, scan_long_stream
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        n = 700_000
        err = long_stream(11, n)
        pad = np.zeros(((n + 15) // 16) * 16 + 16, np.uint8)
        pad[:n] = err
        e = torch.from_numpy(pad).to(dev)
        ev, end, first, bd = scan_long_stream(DeviceScanner(e, kernels.params_struct()), n, 100, seg_batches=16,
                                              distributed=True, with_bound=True)
        oev, _, ost, _ = oracle_scan_c(oracle_lib, err, np.array([0, n], dtype=np.int64), mode=1)
        assert np.array_equal(ev, oev)
        check_end(end, bd, ost[0])
        hit = np.nonzero(oev[:, 1] >= 0)[0]
        assert first == (int(hit[0]) if len(hit) else -1)
    finally:
        dist.destroy_process_group()
