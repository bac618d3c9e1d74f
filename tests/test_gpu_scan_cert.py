"""ddm_scan_certified (HIP, csrc/scan_cert.hip) vs the C oracle (oracle/ddm_scan.c): the
sequential run_DDM recurrence (DDM_Process.py:135-159, the DDM carried across batches at
:144-152, :202).

Events, stop batches, event counts, sample counts and the change / warning flags must be
the oracle's exactly (north_star: bit-exact drift and warning indices); p, s, p_min, s_min
and p_min + s_min are the certified kernel's running-mean values, which must lie within the
bound the kernel reports and within 1e-12 relative of the oracle's (north_star: p/s
statistics within 1e-12 relative).  Streams the kernel could not certify are rescanned by
ddm_scan_long and must then be bit-exact, state included (forced with the tolerance hook)."""
import time

import numpy as np
import pytest
import torch

from conftest import oracle_scan_c
from test_gpu_scan import _state_matrix, random_streams
from test_gpu_scan_long import gpu_scan_long, thinning_stream

pytestmark = pytest.mark.gpu

REL = 1e-12          # north_star: p/s statistics within 1e-12 relative


def _dev():
    return torch.device("cuda", 0)


def gpu_scan_cert(err, offsets, per_batch=100, mode=0, state=None, bound=None, perm_map=None, timed=False, reps=1):
    from ddm_amd import kernels
    dev = _dev()
    err = np.ascontiguousarray(err, dtype=np.uint8)
    offsets = np.asarray(offsets, dtype=np.int64)
    n = len(offsets) - 1
    lens = np.diff(offsets)
    nb = (lens + per_batch - 1) // per_batch
    base = np.concatenate([[0], np.cumsum(nb)[:-1]]).astype(np.int64) if n else np.zeros(0, np.int64)
    pad = np.zeros(((len(err) + 15) // 16) * 16 + 16, np.uint8)
    pad[:len(err)] = err
    e = torch.from_numpy(pad).to(dev)
    st_np = kernels.fresh_states(n) if state is None else state.copy()
    st0 = torch.from_numpy(st_np.view(np.uint8).copy()).to(dev)
    bd0 = torch.zeros((max(n, 1), 2), dtype=torch.float64, device=dev)
    if bound is not None:
        bd0[:n] = torch.from_numpy(np.asarray(bound, np.float64).reshape(n, 2)).to(dev)
    max_rows = int(lens.max()) if n else 0
    scratch = torch.empty(max(1, kernels.scan_certified_scratch_size(n, max_rows, per_batch)), dtype=torch.uint8,
                          device=dev)
    pm = None if perm_map is None else torch.from_numpy(np.ascontiguousarray(perm_map, np.uint8)).to(dev)
    prm = kernels.params_struct(3, per_batch)
    off_d = torch.from_numpy(offsets).to(dev)
    base_d = torch.from_numpy(base).to(dev)
    times = []
    for _ in range(reps):
        st = st0.clone()
        bd = bd0.clone()
        ev = torch.full((max(int(nb.sum()), 1), 2), -7, dtype=torch.int32, device=dev)
        stop = torch.full((max(n, 1),), -7, dtype=torch.int32, device=dev)
        nev = torch.full((max(n, 1),), -7, dtype=torch.int64, device=dev)
        status = torch.full((max(n, 1),), -7, dtype=torch.int32, device=dev)
        timer = kernels.LaunchTimer() if timed else None
        kernels.scan_certified(e, off_d, prm, st, base_d, ev, max_rows, scratch, stop=stop, nev=nev, mode=mode,
                               perm_map=pm, bound=bd, status=status, timer=timer)
        torch.cuda.synchronize()
        if timed:
            times.append(timer.elapsed_ms())
    out = dict(ev=ev.cpu().numpy()[:int(nb.sum())], stop=stop.cpu().numpy()[:n], nev=nev.cpu().numpy()[:n],
               st=st.cpu().numpy().view(kernels.STATE_DTYPE), bound=bd.cpu().numpy()[:n],
               status=status.cpu().numpy()[:n])
    if timed:
        out["ms"] = min(times)
    return out


def check_state(got_st, bound, want, rows=None, exact=None, status=None):
    """n and flags exact; p, s, p_min, s_min, p_min+s_min within REL of the oracle's and
    |p - p_ref| (|p_min - p_min_ref|) within the kernel's bound."""
    g_all = _state_matrix(got_st)
    rows = np.arange(len(g_all)) if rows is None else rows
    g, w, bd = g_all[rows], want[rows], bound[rows]
    bad = np.nonzero((g[:, 5:] != w[:, 5:]).any(axis=1))[0]
    assert len(bad) == 0, f"n/flags differ at {rows[bad][:5]}: got {g[bad[:3]]} want {w[bad[:3]]}" + (
        f" status {status[rows[bad[:5]]]}" if status is not None else "")
    fin = np.isfinite(w[:, :5])
    assert np.array_equal(np.isfinite(g[:, :5]), fin)
    scale = np.where(fin, np.abs(w[:, :5]), 1.0)
    rel = np.where(fin, np.abs(g[:, :5] - np.where(fin, w[:, :5], 0)), 0.0) / np.maximum(scale, 1e-300)
    assert (rel <= REL).all(), f"max rel {rel.max():.3g}"
    assert (np.abs(g[:, 0] - w[:, 0]) <= bd[:, 0]).all()
    minf = fin[:, 2]
    assert (np.abs(g[minf, 2] - w[minf, 2]) <= bd[minf, 1]).all()
    if exact is not None:                                   # rescanned exactly: bit for bit
        assert np.array_equal(g_all[exact], want[exact])
    return rel.max() if rel.size else 0.0


@pytest.mark.parametrize("a", [1.2, 1.5, 2.0])
def test_thinning_10m_rows_certified(oracle_lib, a):
    """The 10M-row carried segments ddm_scan_long takes ~0.5 s for: certified, no rescan."""
    n = 10_000_000
    e = thinning_stream(n, a, jitter_seed=int(a * 10))
    off = np.array([0, n])
    wev, wstop, wst, _ = oracle_scan_c(oracle_lib, e, off, mode=0)
    assert wstop[0] == -1 and wst[0, 5] == n + 1
    got = gpu_scan_cert(e, off, mode=0, timed=True, reps=3)
    assert np.array_equal(got["ev"], wev) and np.array_equal(got["stop"], wstop)
    assert got["nev"][0] == int((wev >= 0).any(axis=1).sum()) > 0
    assert got["status"][0] == 0                            # certified: no exact rescan
    rel = check_state(got["st"], got["bound"], wst)
    msg = f"10M-row carried segment (a={a}): ddm_scan_certified {got['ms']:.3f} ms, state max rel err {rel:.2e}"
    if a == 1.5:
        t = time.perf_counter()
        *_, ms_long = gpu_scan_long(e, off, mode=0, timed=True)
        msg += f"; ddm_scan_long {ms_long:.1f} ms ({ms_long / got['ms']:.0f}x)"
        assert got["ms"] * 10 <= ms_long
    print(msg)
    assert got["ms"] <= 50.0                                # <= 50 ms for 10M rows


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("per_batch", [100, 37, 64, 256, 1])
def test_random_streams_vs_oracle(oracle_lib, mode, per_batch):
    rs = np.random.RandomState(per_batch * 5 + mode)
    err, off = random_streams(rs, 60, max_len=30_000)
    got = gpu_scan_cert(err, off, per_batch, mode)
    wev, wstop, wst, _ = oracle_scan_c(oracle_lib, err, off, per_batch=per_batch, mode=mode)
    lens = np.diff(off)
    nonempty = lens > 0
    nb = (lens + per_batch - 1) // per_batch
    base = np.concatenate([[0], np.cumsum(nb)[:-1]])
    assert np.array_equal(got["ev"], wev)
    assert np.array_equal(got["stop"][nonempty], wstop[nonempty])
    want_nev = np.array([int(((wev[b:b + k] >= 0).any(axis=1)).sum()) for b, k in zip(base, nb)])
    assert np.array_equal(got["nev"][nonempty], want_nev[nonempty])
    check_state(got["st"], got["bound"], wst, rows=np.nonzero(nonempty)[0],
                exact=np.nonzero(nonempty & (got["status"] != 0))[0], status=got["status"])
    # empty streams are left untouched
    assert (got["stop"][~nonempty] == -7).all() and (got["nev"][~nonempty] == -7).all()
    assert (got["status"][~nonempty] == -7).all()


def test_carried_state_and_bound_chain(oracle_lib):
    """A stream cut at a batch boundary: the second half, started from the first half's
    CERTIFIED state and its bound, gives the uncut run's events; perm_map labels."""
    n, cut = 3_000_000, 1_234_500
    e = thinning_stream(n, 1.3, jitter_seed=3)
    wev, wstop, wst, _ = oracle_scan_c(oracle_lib, e, np.array([0, n]), mode=0)
    a = gpu_scan_cert(e[:cut], np.array([0, cut]), mode=0)
    assert a["status"][0] == 0 and a["bound"][0, 0] > 0
    b = gpu_scan_cert(e[cut:], np.array([0, n - cut]), mode=0, state=a["st"], bound=a["bound"])
    assert b["status"][0] == 0
    assert np.array_equal(b["ev"], wev[cut // 100:])
    check_state(b["st"], b["bound"], wst)
    assert b["bound"][0, 0] >= a["bound"][0, 0] * cut / n   # the incoming bound is carried (contracted)
    rs = np.random.RandomState(0)
    pmap = np.concatenate([rs.permutation(100) for _ in range(n // 100)]).astype(np.uint8)
    p = gpu_scan_cert(e, np.array([0, n]), mode=0, perm_map=pmap)
    want = wev.copy()
    for c in range(2):
        hit = want[:, c] >= 0
        bi = np.nonzero(hit)[0]
        want[hit, c] = pmap[bi * 100 + want[hit, c]]
    assert np.array_equal(p["ev"], want)


def test_state_from_the_exact_scan(oracle_lib):
    """The second half from ddm_scan_long's (exact) state, no bound: the incoming minimum is
    the reference's own."""
    n, cut = 2_000_000, 700_000
    e = thinning_stream(n, 1.6, jitter_seed=5)
    wev, _, wst, _ = oracle_scan_c(oracle_lib, e, np.array([0, n]), mode=0)
    _, _, _, st_a = gpu_scan_long(e[:cut], np.array([0, cut]), mode=0)
    b = gpu_scan_cert(e[cut:], np.array([0, n - cut]), mode=0, state=st_a)
    assert b["status"][0] == 0
    assert np.array_equal(b["ev"], wev[cut // 100:])
    check_state(b["st"], b["bound"], wst)


def test_forced_exact_rescan_is_bit_exact(oracle_lib):
    """With every bound scaled past any margin nothing certifies: every stream goes to
    ddm_scan_long and the results, state included, are the oracle's bit for bit."""
    from ddm_amd import _capi
    rs = np.random.RandomState(9)
    err, off = random_streams(rs, 40, max_len=20_000)
    lens = np.diff(off)
    nonempty = lens > 0
    try:
        assert _capi.lib.ddm_scan_certified_set_tol_scale(1e300) == 0
        for mode in (0, 1):
            got = gpu_scan_cert(err, off, 100, mode)
            wev, wstop, wst, _ = oracle_scan_c(oracle_lib, err, off, mode=mode)
            assert np.array_equal(got["ev"], wev)
            assert np.array_equal(got["stop"][nonempty], wstop[nonempty])
            np.testing.assert_array_equal(_state_matrix(got["st"])[nonempty], wst[nonempty])
            # streams that decide anything were rescanned (exact regimes certify alone)
            assert (got["status"][nonempty] != 0).sum() >= nonempty.sum() // 2
            assert (got["bound"][nonempty & (got["status"] != 0)] == 0).all()
    finally:
        _capi.lib.ddm_scan_certified_set_tol_scale(1.0)
    assert _capi.lib.ddm_scan_certified_set_tol_scale(0.5) != 0      # < 1 is refused


def test_inexact_carried_state_is_not_rescanned_exactly(oracle_lib):
    """a carried call whose incoming state is pa's (a nonzero incoming bound)
    and whose first round leaves a decision uncertified must not run the exact kernel from
    that state (its p is not the reference's) nor zero the bound: status 3, state and bound
    left as they came in, so the caller redoes the run from its last exact carry."""
    from ddm_amd import _capi
    n, cut = 1_000_000, 600_000
    e = thinning_stream(n, 1.3, jitter_seed=3)
    a = gpu_scan_cert(e[:cut], np.array([0, cut]), mode=0)
    assert a["status"][0] == 0 and a["bound"][0, 0] > 0
    try:
        assert _capi.lib.ddm_scan_certified_set_tol_scale(1e300) == 0
        for mode in (0, 1):
            b = gpu_scan_cert(e[cut:], np.array([0, n - cut]), mode=mode, state=a["st"], bound=a["bound"])
            assert b["status"][0] == 3, (mode, b["status"])
            np.testing.assert_array_equal(b["bound"], a["bound"])
            np.testing.assert_array_equal(_state_matrix(b["st"]), _state_matrix(a["st"]))
            # an exact incoming state (no bound) still takes the exact kernel: status 1
            c = gpu_scan_cert(e[cut:], np.array([0, n - cut]), mode=mode, state=a["st"])
            assert c["status"][0] in (1, 2) and (c["bound"] == 0).all()
    finally:
        _capi.lib.ddm_scan_certified_set_tol_scale(1.0)


def test_mode1_reset_heavy_long_stream(oracle_lib):
    """A change in almost every batch (20 % noise): four certified rounds, then the exact
    kernel from the fifth change on."""
    rs = np.random.RandomState(11)
    n = 2_000_000
    e = (rs.rand(n) < 0.2).astype(np.uint8)
    off = np.array([0, n])
    wev, wstop, wst, _ = oracle_scan_c(oracle_lib, e, off, mode=1)
    got = gpu_scan_cert(e, off, mode=1)
    assert np.array_equal(got["ev"], wev)
    assert got["nev"][0] == int((wev >= 0).any(axis=1).sum())
    assert got["status"][0] == 2
    np.testing.assert_array_equal(_state_matrix(got["st"]), wst)


def test_mode1_few_changes(oracle_lib):
    """Long carried segments separated by a few changes (mode 1): every round certified."""
    n = 3_000_000
    e = thinning_stream(n, 1.5, jitter_seed=2)
    for at in (400_000, 1_500_000):                       # bursts that force a change
        e[at:at + 400] = 1
    off = np.array([0, n])
    wev, _, wst, _ = oracle_scan_c(oracle_lib, e, off, mode=1)
    assert ((wev[:, 1] >= 0).sum()) >= 2
    got = gpu_scan_cert(e, off, mode=1)
    assert np.array_equal(got["ev"], wev)
    assert got["status"][0] in (0, 2)
    check_state(got["st"], got["bound"], wst, exact=np.nonzero(got["status"] != 0)[0])
