"""One long mode-1 stream scanned as segments with carry resolution (ddm_amd/longstream.py,
SURVEY.md §8e single long stream): on CPU with the oracle as the segment scanner, in one
process and over two gloo ranks; the result must be the whole stream's sequential scan
(oracle/ddm.py scan_stream, mode "restart": DDM_Process.py:207-210) bit for bit."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def long_stream(seed, n):
    """Reset-heavy stretches, clean stretches (long carried trivial detectors), and all-error
    stretches (p = 1 forever: a detector carried through many segments, every carry
    rescanned)."""
    rs = np.random.RandomState(seed)
    out, pos = [], 0
    while pos < n:
        k = rs.randint(300, 6000)
        kind = rs.randint(4)
        if kind == 0:
            seg = rs.binomial(1, rs.uniform(0.05, 0.4), k)
        elif kind == 1:
            seg = rs.binomial(1, 0.003, k)
        elif kind == 2:
            seg = np.ones(k, np.int64)
        else:
            seg = rs.binomial(1, rs.uniform(0.01, 0.1), k)
        out.append(seg.astype(np.uint8))
        pos += k
    return np.concatenate(out)[:n]


class OracleScanner:
    """The segment scanner interface of longstream.DeviceScanner, on the CPU oracle."""

    def __init__(self, err, per_batch=100):
        self.err, self.pb = err, per_batch

    def scan(self, row0, n_segments, seg_len, states):
        from ddm_amd.kernels import STATE_DTYPE
        from oracle.ddm import OracleDDM, scan_stream
        evs = []
        fin = np.empty(n_segments, STATE_DTYPE)
        for k in range(n_segments):
            d = OracleDDM()
            st = states[k]
            d.miss_prob, d.miss_std = float(st["miss_prob"]), float(st["miss_std"])
            d.miss_prob_min, d.miss_sd_min = float(st["miss_prob_min"]), float(st["miss_sd_min"])
            d.miss_prob_sd_min, d.sample_count = float(st["miss_prob_sd_min"]), int(st["sample_count"])
            d.in_concept_change, d.in_warning_zone = bool(st["in_concept_change"]), bool(st["in_warning_zone"])
            lo = row0 + k * seg_len
            ev, _, d, _ = scan_stream(self.err[lo:lo + seg_len], per_batch=self.pb, mode="restart", ddm=d)
            evs.append(ev)
            fin[k] = d.state_tuple()
        return np.concatenate(evs), fin


@pytest.mark.parametrize("n,seg_batches", [(40_000, 16), (41_234, 32), (1_550, 16), (99, 16)])
def test_segments_equal_sequential_scan(n, seg_batches):
    from ddm_amd.longstream import scan_long_stream
    from oracle.ddm import scan_stream
    err = long_stream(n, n)
    ev, end, first = scan_long_stream(OracleScanner(err), n, 100, seg_batches=seg_batches)
    ref, _, dref, _ = scan_stream(err, per_batch=100, mode="restart")
    assert np.array_equal(ev, ref)
    assert tuple(end.tolist()) == tuple(dref.state_tuple())
    hit = np.nonzero(ref[:, 1] >= 0)[0]
    assert first == (int(hit[0]) if len(hit) else -1)


def test_chunk_bounds_cover_stream():
    from ddm_amd.longstream import chunk_bounds
    for n, w, s in [(10_000, 2, 1600), (10_000, 3, 1600), (1_000, 4, 1600), (16_000, 8, 1600)]:
        b = chunk_bounds(n, w, s)
        assert b[0][0] == 0 and b[-1][1] == n
        assert all(b[r][1] == b[r + 1][0] for r in range(w - 1))
        assert all(lo % s == 0 for lo, _ in b)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, q):
    import sys
    from conftest import PKG_ROOT, ROOT
    for p in (ROOT, PKG_ROOT):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist

    from ddm_amd.longstream import chunk_bounds, scan_long_stream
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    err = long_stream(7, n)
    lo, hi = chunk_bounds(n, world, 16 * 100)[rank]
    ev, end, first = scan_long_stream(OracleScanner(err[lo:hi]), hi - lo, 100, seg_batches=16, distributed=True,
                                      first_batch=lo // 100)
    q.put((rank, ev.tolist(), end.tolist(), first))
    dist.barrier()
    dist.destroy_process_group()


def test_two_ranks_equal_sequential_scan():
    from oracle.ddm import scan_stream
    n = 30_000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref, _, dref, _ = scan_stream(long_stream(7, n), per_batch=100, mode="restart")
    ev = np.concatenate([np.array(r[1], dtype=np.int32).reshape(-1, 2) for r in res])
    assert np.array_equal(ev, ref)
    assert tuple(res[-1][2]) == tuple(dref.state_tuple())
    hit = np.nonzero(ref[:, 1] >= 0)[0]
    assert res[0][3] == res[1][3] == (int(hit[0]) if len(hit) else -1)
