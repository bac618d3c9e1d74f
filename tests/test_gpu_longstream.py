"""One long mode-1 stream on the GPU: segments scanned by ddm_scan_batches and the carries
resolved (ddm_amd/longstream.py) == the C oracle's sequential scan of the whole stream."""
import numpy as np
import pytest
import torch

from conftest import oracle_scan_c
from test_longstream import long_stream

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,seg_batches", [(2_000_000, 64), (1_234_567, 16)])
def test_device_segments_equal_oracle(oracle_lib, n, seg_batches):
    from ddm_amd import kernels
    from ddm_amd.longstream import DeviceScanner, scan_long_stream
    err = long_stream(n % 1000, n)
    dev = torch.device("cuda", 0)
    pad = np.zeros(((n + 15) // 16) * 16 + 16, np.uint8)
    pad[:n] = err
    e = torch.from_numpy(pad).to(dev)
    ev, end, first = scan_long_stream(DeviceScanner(e, kernels.params_struct()), n, 100, seg_batches=seg_batches)
    oev, _, ost, _ = oracle_scan_c(oracle_lib, err, np.array([0, n], dtype=np.int64), mode=1)
    assert np.array_equal(ev, oev)
    got = np.array([end["miss_prob"], end["miss_std"], end["miss_prob_min"], end["miss_sd_min"],
                    end["miss_prob_sd_min"], end["sample_count"], end["in_concept_change"], end["in_warning_zone"]],
                   dtype=np.float64)
    np.testing.assert_array_equal(got, ost[0])
    hit = np.nonzero(oev[:, 1] >= 0)[0]
    assert first == (int(hit[0]) if len(hit) else -1)


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
        ev, end, first = scan_long_stream(DeviceScanner(e, kernels.params_struct()), n, 100, seg_batches=16,
                                          distributed=True)
        oev, _, ost, _ = oracle_scan_c(oracle_lib, err, np.array([0, n], dtype=np.int64), mode=1)
        assert np.array_equal(ev, oev)
        hit = np.nonzero(oev[:, 1] >= 0)[0]
        assert first == (int(hit[0]) if len(hit) else -1)
    finally:
        dist.destroy_process_group()
