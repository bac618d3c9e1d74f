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


def _worker(rank, world, port, n, q, certifying=False):
    import sys
    from conftest import PKG_ROOT, ROOT
    for p in (ROOT, PKG_ROOT):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist

    from ddm_amd.longstream import chunk_bounds, scan_long_stream
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    err = _two_rank_stream(n, certifying)
    lo, hi = chunk_bounds(n, world, 16 * 100)[rank]
    from test_longstream import CertifyingScanner
    sc = (CertifyingScanner if certifying else OracleScanner)(err[lo:hi])
    ev, end, first = scan_long_stream(sc, hi - lo, 100, seg_batches=16, distributed=True, first_batch=lo // 100)
    q.put((rank, ev.tolist(), end.tolist(), first, getattr(sc, "calls", None)))
    dist.barrier()
    dist.destroy_process_group()


def _two_rank_stream(n, certifying):
    if not certifying:
        return long_stream(7, n)
    # a detector carried across the rank boundary (all errors around row n / 2): rank 1's
    # carry-in comes with a bound, its certified rescan is void, every rank redoes exactly
    rs = np.random.RandomState(5)
    a = n // 2 - 6_000
    return np.concatenate([rs.binomial(1, 0.3, a), np.ones(12_000, np.int64),
                           rs.binomial(1, 0.2, n - a - 12_000)]).astype(np.uint8)


@pytest.mark.parametrize("certifying", [False, True])
def test_two_ranks_equal_sequential_scan(certifying):
    from oracle.ddm import scan_stream
    n = 30_000 if not certifying else 32_000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n, q, certifying)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref, _, dref, _ = scan_stream(_two_rank_stream(n, certifying), per_batch=100, mode="restart")
    ev = np.concatenate([np.array(r[1], dtype=np.int32).reshape(-1, 2) for r in res])
    assert np.array_equal(ev, ref)
    assert tuple(res[-1][2]) == tuple(dref.state_tuple())
    hit = np.nonzero(ref[:, 1] >= 0)[0]
    assert res[0][3] == res[1][3] == (int(hit[0]) if len(hit) else -1)
    if certifying:                # rank 1's bounded carry-in was void: both ranks redid exactly
        assert res[1][4]["void"] >= 1 and res[0][4]["exact"] >= 1 and res[1][4]["exact"] >= 1, res


class CertifyingScanner(OracleScanner):
    """OracleScanner with the certified carried-scan interface: every carried call from a
    state with a nonzero bound reports a void result (ddm_scan_certified status 3, the
    near-tie case) unless it is asked for the exact kernel; a certified result's bound is
    nonzero.  Counts the calls by kind."""

    def __init__(self, err, per_batch=100):
        super().__init__(err, per_batch)
        self.certified = True
        self.calls = {"certified": 0, "void": 0, "exact": 0}

    def carried(self, row0, n_rows, state, bound=None, exact=False):
        from ddm_amd.kernels import STATE_DTYPE
        from ddm_amd.longstream import InexactCarry
        if not exact and self.certified and bound is not None and np.any(np.asarray(bound) != 0):
            self.calls["void"] += 1
            raise InexactCarry("near tie from an inexact carry")
        st = np.empty(1, STATE_DTYPE)
        st[0] = state
        ev, fin = self.scan(row0, 1, n_rows, st)
        if exact or not self.certified:
            self.calls["exact"] += 1
            return ev, fin[0], np.zeros(2)
        self.calls["certified"] += 1
        return ev, fin[0], np.array([1e-15, 1e-15])


def test_void_certified_rescan_redone_from_last_exact_carry():
    """a carried run whose certified rescan comes back void (status 3) is redone
    from the last exact carry on the exact kernel; the result is still the sequential scan."""
    from ddm_amd.longstream import scan_long_stream
    from oracle.ddm import scan_stream
    n = 60_000
    rs = np.random.RandomState(2)
    # a long all-error stretch: a detector carried through many segments (chained rescans)
    err = np.concatenate([rs.binomial(1, 0.3, 8_000), np.ones(30_000, np.int64), rs.binomial(1, 0.2, 22_000)])
    err = err.astype(np.uint8)
    sc = CertifyingScanner(err)
    ev, end, first = scan_long_stream(sc, n, 100, seg_batches=16)
    ref, _, dref, _ = scan_stream(err, per_batch=100, mode="restart")
    assert np.array_equal(ev, ref)
    assert tuple(end.tolist()) == tuple(dref.state_tuple())
    assert sc.calls["void"] >= 1 and sc.calls["exact"] >= 1, sc.calls
