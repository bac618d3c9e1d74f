"""Multi-process path on CPU: world_size 2 with gloo.  Partitions go to rank d % world, each
rank runs its partitions (here with the oracle as the per-partition function — the GPU
function is exercised by the -m gpu tests) and one all_gather collects every event."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp

from conftest import golden_partitions


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
    from oracle.controller import run_partition
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    parts = [(d, p) for d, p, _ in golden_partitions(mult, inst)]
    mine = ddm_dist.local_partitions(parts, rank, world)
    assert all(d % world == rank for d, _ in mine)

    def oracle_fn(frame, rng, device, st):
        np.random.set_state(rng.numpy_state())
        return run_partition(frame[[str(i) for i in range(21)]].to_numpy(), frame["target"].to_numpy(),
                             frame.index.to_numpy(), frame["full_df_row_number"].to_numpy())

    outs = run_partitions(mine, {d: 1000 + d for d, _ in mine}, devices=[], max_workers=1, fn=oracle_fn)
    allev = ddm_dist.gather_events(outs)
    n_rows = {d: len(e) for d, _, e in golden_partitions(mult, inst)}
    compact = ddm_dist.gather_events(outs, n_rows=n_rows)
    assert sorted(compact) == sorted(allev)
    for d in allev:
        assert np.array_equal(compact[d], allev[d]), d
    q.put((rank, {d: v.tolist() for d, v in allev.items()}))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gather_equals_reference():
    mult, inst = 2, 4
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
    expect = {d: e for d, _, e in golden_partitions(mult, inst)}
    for rank, allev in res:
        assert sorted(allev) == sorted(expect)
        for d, e in expect.items():
            assert np.array_equal(np.array(allev[d], dtype=np.int64), e), (rank, d)


def test_records_roundtrip_single_process():
    from ddm_amd.dist import RECORD, _records
    outs = {3: np.array([[1, 2, -1, -1], [-1, -1, 5, 6]]), 1: np.zeros((0, 4), np.int64)}
    r = _records(outs)
    assert r.shape == (2, RECORD) and (r[:, 0] == 3).all() and list(r[:, 1]) == [0, 1]
    outs = {2: np.array([[-1, -1, -1, -1], [-1, -1, 5, 6], [-1, -1, -1, -1]])}
    r = _records(outs, events_only=True)
    assert r.shape == (1, RECORD) and list(r[0]) == [2, 1, -1, -1, 5, 6]
