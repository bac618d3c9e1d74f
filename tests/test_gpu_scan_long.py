"""ddm_scan_long (HIP) vs the C oracle (oracle/ddm_scan.c): events, stop batch, event counts
and the carried detector must be bit-identical to run_DDM's sequential recurrence
(DDM_Process.py:135-159, the DDM carried across batches at :144-152, :202).

The long-segment streams are ones on which the detector never changes for 10M rows while
it is not in its trivial state: errors thinning out after a noisy start (an error at
every floor(k**a)), where k_scan_fast runs every row exactly on one lane."""
import time

import numpy as np
import pytest
import torch

from conftest import oracle_scan_c
from test_gpu_scan import _state_matrix, gpu_scan, random_streams

pytestmark = pytest.mark.gpu


def _dev():
    return torch.device("cuda", 0)


def gpu_scan_long(err, offsets, per_batch=100, mode=0, state=None, perm_map=None, timed=False):
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
    st = torch.from_numpy(st_np.view(np.uint8)).to(dev)
    ev = torch.full((max(int(nb.sum()), 1), 2), -7, dtype=torch.int32, device=dev)
    stop = torch.full((max(n, 1),), -7, dtype=torch.int32, device=dev)
    nev = torch.full((max(n, 1),), -7, dtype=torch.int64, device=dev)
    max_rows = int(lens.max()) if n else 0
    scratch = torch.empty(max(1, kernels.scan_long_scratch_size(n, max_rows, per_batch)), dtype=torch.uint8,
                          device=dev)
    pm = None if perm_map is None else torch.from_numpy(np.ascontiguousarray(perm_map, np.uint8)).to(dev)
    prm = kernels.params_struct(3, per_batch)
    timer = kernels.LaunchTimer() if timed else None
    kernels.scan_long(e, torch.from_numpy(offsets).to(dev), prm, st, torch.from_numpy(base).to(dev), ev, max_rows,
                      scratch, stop=stop, nev=nev, mode=mode, perm_map=pm, timer=timer)
    torch.cuda.synchronize()
    assert int(scratch[4:8].view(torch.int32).item()) == 0          # no chunk gave up on its predecessor
    out = (ev.cpu().numpy()[:int(nb.sum())], stop.cpu().numpy()[:n], nev.cpu().numpy()[:n],
           st.cpu().numpy().view(kernels.STATE_DTYPE))
    return out + ((timer.elapsed_ms(),) if timed else ())


def thinning_stream(n, a, jitter_seed=None):
    k = np.arange(int(n ** (1 / a)) + 2)
    pos = np.floor(k ** a).astype(np.int64)
    pos = pos[pos < n]
    e = np.zeros(n, np.uint8)
    e[pos] = 1
    if jitter_seed is not None:              # move some errors by one row: no periodic structure
        rs = np.random.RandomState(jitter_seed)
        mv = pos[(rs.rand(len(pos)) < 0.3) & (pos > 10) & (pos < n - 1)]
        e[mv] = 0
        e[mv + 1] = 1
    return e


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("per_batch", [100, 37, 64, 256, 1])
def test_random_streams_vs_oracle(oracle_lib, mode, per_batch):
    rs = np.random.RandomState(per_batch * 3 + mode)
    err, off = random_streams(rs, 60, max_len=30_000)
    got = gpu_scan_long(err, off, per_batch, mode)
    wev, wstop, wst, _ = oracle_scan_c(oracle_lib, err, off, per_batch=per_batch, mode=mode)
    ev, stop, nev, st = got
    lens = np.diff(off)
    nonempty = lens > 0
    nb = (lens + per_batch - 1) // per_batch
    base = np.concatenate([[0], np.cumsum(nb)[:-1]])
    assert np.array_equal(ev, wev)
    assert np.array_equal(stop[nonempty], wstop[nonempty])
    assert np.array_equal(_state_matrix(st)[nonempty], wst[nonempty])
    want_nev = np.array([int(((wev[b:b + k] >= 0).any(axis=1)).sum()) for b, k in zip(base, nb)])
    assert np.array_equal(nev[nonempty], want_nev[nonempty])
    # empty streams are left untouched
    assert (stop[~nonempty] == -7).all() and (nev[~nonempty] == -7).all()


@pytest.mark.parametrize("a", [1.2, 1.5, 2.0])
def test_thinning_10m_rows_vs_oracle_and_scan_streams(oracle_lib, a):
    n = 10_000_000
    e = thinning_stream(n, a, jitter_seed=int(a * 10))
    off = np.array([0, n])
    wev, wstop, wst, _ = oracle_scan_c(oracle_lib, e, off, mode=0)
    assert wstop[0] == -1 and wst[0, 5] == n + 1          # no change: a 10M-row carried segment
    t = time.perf_counter()
    ev, stop, nev, st, ms_long = gpu_scan_long(e, off, mode=0, timed=True)
    wall_long = (time.perf_counter() - t) * 1e3
    assert np.array_equal(ev, wev) and np.array_equal(stop, wstop)
    assert np.array_equal(_state_matrix(st), wst)
    assert nev[0] == int((wev >= 0).any(axis=1).sum()) > 0
    if a == 1.5:
        # the same stream through ddm_scan_streams (k_scan_fast: one lane runs every row)
        t = time.perf_counter()
        fev, fstop, _, fst, _ = gpu_scan(e, off, mode=0)
        ms_fast = (time.perf_counter() - t) * 1e3
        assert np.array_equal(fev, wev) and np.array_equal(_state_matrix(fst), wst)
        print(f"10M-row carried segment: ddm_scan_long {ms_long:.1f} ms kernel / {wall_long:.1f} ms wall, "
              f"ddm_scan_streams (k_scan_fast) {ms_fast:.1f} ms wall")
        assert wall_long < ms_fast


def test_carried_state_in_and_perm_map(oracle_lib):
    """A stream cut at a batch boundary: the second half, started from the first half's
    carried detector, gives the second half's events of the uncut run; perm_map labels."""
    n, cut = 3_000_000, 1_234_500
    e = thinning_stream(n, 1.3, jitter_seed=3)
    wev, wstop, wst, _ = oracle_scan_c(oracle_lib, e, np.array([0, n]), mode=0)
    _, _, _, st_a = gpu_scan_long(e[:cut], np.array([0, cut]), mode=0)
    ev_b, stop_b, _, st_b = gpu_scan_long(e[cut:], np.array([0, n - cut]), mode=0, state=st_a)
    assert np.array_equal(ev_b, wev[cut // 100:])
    assert np.array_equal(_state_matrix(st_b), wst)
    rs = np.random.RandomState(0)
    pmap = np.concatenate([rs.permutation(100) for _ in range(n // 100)]).astype(np.uint8)
    ev_p, _, _, _ = gpu_scan_long(e, np.array([0, n]), mode=0, perm_map=pmap)
    want = wev.copy()
    for c in range(2):
        hit = want[:, c] >= 0
        b = np.nonzero(hit)[0]
        want[hit, c] = pmap[b * 100 + want[hit, c]]
    assert np.array_equal(ev_p, want)


def test_mode1_reset_heavy_long_stream(oracle_lib):
    """A change in almost every batch (noise at 20%): chunks restart from fresh detectors."""
    rs = np.random.RandomState(11)
    n = 2_000_000
    e = (rs.rand(n) < 0.2).astype(np.uint8)
    off = np.array([0, n])
    wev, wstop, wst, _ = oracle_scan_c(oracle_lib, e, off, mode=1)
    ev, stop, nev, st = gpu_scan_long(e, off, mode=1)
    assert np.array_equal(ev, wev) and np.array_equal(_state_matrix(st), wst)
    assert nev[0] == int((wev >= 0).any(axis=1).sum())


@pytest.mark.parametrize("refit", ["device", "native"])
def test_controller_routes_long_carried_windows(refit):
    """A partition whose model is wrong on every row after batch 0 (class A in batch 0, class
    B after it): p = 1, s = 0, never a change (SURVEY.md finding 7), a carried detector that
    is neither fresh nor trivial, so the growing windows run on ddm_scan_long.  Events and
    RNG position == the oracle's."""
    from ddm_amd import synth
    from ddm_amd.controller import LONG_SCAN_MIN_ROWS, PartitionRunner
    from ddm_amd.params import DDMSettings
    from ddm_amd.rng import MTStream
    from oracle.controller import run_partition
    dev = _dev()
    n = 120_000
    part = synth.block_partition(n, 0, 1, 100, 5, dev)        # block 0 = class 0, then class 1 ...
    import torch as _t
    part.y[100:n].fill_(1)                                    # ... and class 1 for good
    _t.cuda.synchronize()
    X, y = synth.host_copy(part)
    assert (y[:100] == 0).all() and (y[100:] == 1).all()
    runner = PartitionRunner(part, DDMSettings(window_batches=64), refit=refit)
    rng = MTStream.from_seed(17)
    got = runner.run(rng)
    runner.close()
    np.random.seed(17)
    want = run_partition(X, y, np.arange(n), np.arange(n))
    assert np.array_equal(got[:, 0], want[:, 0]) and np.array_equal(got[:, 1], want[:, 2])
    assert (want[:, 2] < 0).all()
    after = np.random.get_state()
    assert np.array_equal(rng.key, after[1]) and rng.pos.value == after[2]
    assert runner.stats.long_scans >= 2 and n > 2 * LONG_SCAN_MIN_ROWS


def test_look_back_give_up_is_reported_not_silent():
    """With the look-back spin limit at 0 a chunk whose predecessor has not published gives
    up at once: that stream must come back as DDM_STOP_FAILED (events -1, state untouched),
    never as results scanned from a carry that was never published."""
    from ddm_amd import _capi, kernels
    dev = _dev()
    n = 1_000_000
    e = thinning_stream(n, 1.6)
    pad = np.zeros(n + 32, np.uint8)
    pad[:n] = e
    err = torch.from_numpy(pad).to(dev)
    prm = kernels.params_struct(3, 100)
    st0 = kernels.fresh_states(1)
    st = torch.from_numpy(st0.view(np.uint8).copy()).to(dev)
    ev = torch.full(((n + 99) // 100, 2), -7, dtype=torch.int32, device=dev)
    stop = torch.full((1,), -7, dtype=torch.int32, device=dev)
    nev = torch.full((1,), -7, dtype=torch.int64, device=dev)
    scratch = torch.empty(kernels.scan_long_scratch_size(1, n, 100), dtype=torch.uint8, device=dev)
    off = torch.tensor([0, n], dtype=torch.int64, device=dev)
    base = torch.zeros(1, dtype=torch.int64, device=dev)
    _capi.lib.ddm_scan_long_set_spin_limit(0)
    try:
        kernels.scan_long(err, off, prm, st, base, ev, n, scratch, stop=stop, nev=nev, mode=0)
        torch.cuda.synchronize()
    finally:
        _capi.lib.ddm_scan_long_set_spin_limit(1 << 24)
    gave_up = int(scratch[4:8].view(torch.int32).item())
    if gave_up:
        assert int(stop.item()) == _capi.DDM_STOP_FAILED and int(nev.item()) == 0
        assert np.array_equal(st.cpu().numpy().view(np.uint8), st0.view(np.uint8))
    else:       # every predecessor happened to publish in time: the results must be exact
        ref = gpu_scan_long(e, np.array([0, n]), mode=0)
        assert np.array_equal(ev.cpu().numpy(), ref[0])
