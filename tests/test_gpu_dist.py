"""The N>1 path on the GPU: two ranks (rehearsed on one GPU, gloo rendezvous) each run their
partitions (d % 2 == rank, DDM_Process.py:225-226) through the HIP hot path, then gather
every partition's events (DDM_Process.py:258) == the reference's fixtures; and the RCCL
ctypes binding (ddm_amd.rccl) that carries the gather on real multi-GPU runs, at world 1."""
import os
import socket

import numpy as np
import pytest
import torch

from conftest import golden_partitions

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, mult, inst, q):
    import sys
    from conftest import PKG_ROOT, ROOT
    for p in (ROOT, PKG_ROOT):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist

    from ddm_amd import dist as ddm_dist
    from ddm_amd.partition import run_partitions
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    parts = [(d, p) for d, p, _ in golden_partitions(mult, inst)]
    mine = [(d, p) for d, p in ddm_dist.local_partitions(parts, rank, world) if len(p) > 100]
    outs = run_partitions(mine, {d: 1000 + d for d, _ in mine}, devices=[torch.device("cuda", 0)])
    allev = ddm_dist.gather_events({d: o.to_numpy() for d, o in outs.items()})
    q.put((rank, {d: v.tolist() for d, v in allev.items()}))
    dist.barrier()
    dist.destroy_process_group()


def test_two_ranks_hip_path_gather_equals_reference():
    import torch.multiprocessing as mp
    assert not torch.cuda.is_initialized(), "must run before this process touches the GPU"
    mult, inst = 4, 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, mult, inst, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    expect = {d: e for d, _, e in golden_partitions(mult, inst) if e is not None}
    for rank, allev in res:
        assert sorted(allev) == sorted(expect)
        for d, e in expect.items():
            assert np.array_equal(np.array(allev[d], dtype=np.int64), e), (rank, d)


def test_rccl_ctypes_world1_gather():
    import torch.distributed as dist

    from ddm_amd.dist import RECORD, _gather_rccl, _records
    from ddm_amd.rccl import RcclComm
    dev = torch.device("cuda", 0)
    comm = RcclComm(0, 1, dev, dist.HashStore())
    try:
        x = torch.arange(10, dtype=torch.int64, device=dev)
        y = torch.empty(10, dtype=torch.int64, device=dev)
        comm.all_gather(x, y)
        torch.cuda.synchronize()
        assert torch.equal(x, y)
        outs = {3: np.array([[1, 2, -1, -1], [-1, -1, 5, 6], [-1, -1, -1, -1]])}
        rec = _records(outs, events_only=True)
        got = _gather_rccl(comm, rec)
        assert got.shape == (2, RECORD) and np.array_equal(got, rec)
    finally:
        comm.close()
