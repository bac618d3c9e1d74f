"""ddm_scan_batches (batch-parallel mode-1 scan for equal-length streams, configs[3]) vs
ddm_scan_streams in mode 1 and the C oracle: events, event counts and the carried state,
bit for bit."""
import numpy as np
import pytest
import torch

from conftest import oracle_scan_c
from test_gpu_scan import _state_matrix, gpu_scan

pytestmark = pytest.mark.gpu


def gpu_scan_batches(err, n_streams, L, per_batch=100, state=None, min_inst=3, wl=0.5, cl=1.5, pmap=None):
    from ddm_amd import kernels
    dev = torch.device("cuda", 0)
    err = np.ascontiguousarray(err, dtype=np.uint8)
    nb = -(-L // per_batch)
    pad = np.zeros(((n_streams * L + 15) // 16) * 16 + 16, np.uint8)
    pad[:n_streams * L] = err[:n_streams * L]
    e = torch.from_numpy(pad).to(dev)
    st_np = kernels.fresh_states(n_streams) if state is None else state.copy()
    st = torch.from_numpy(st_np.view(np.uint8)).to(dev)
    ev = torch.full((max(n_streams * nb, 1), 2), 7, dtype=torch.int32, device=dev)   # no memset needed
    flags = torch.empty(kernels.scan_batches_scratch_size(n_streams, L, per_batch), dtype=torch.uint8, device=dev)
    nev = torch.empty(max(n_streams, 1), dtype=torch.int64, device=dev)
    pm = None
    if pmap is not None:
        pp = np.zeros_like(pad)
        pp[:n_streams * L] = pmap
        pm = torch.from_numpy(pp).to(dev)
    prm = kernels.params_struct(min_inst, per_batch, wl, cl)
    kernels.scan_batches(e, n_streams, L, prm, st, ev, flags, nev=nev, perm_map=pm)
    torch.cuda.synchronize()
    return (ev.cpu().numpy()[:n_streams * nb], nev.cpu().numpy()[:n_streams],
            st.cpu().numpy().view(kernels.STATE_DTYPE))


def mixed_streams(rs, n, L):
    """Per-stream Bernoulli rates from clean (no error) to error-dense, plus all-ones and
    rate steps: trivial items, long exact items and unchanged batches all occur."""
    out = np.zeros((n, L), np.uint8)
    for k in range(n):
        kind = k % 6
        if kind == 0:
            out[k] = rs.binomial(1, rs.uniform(0.001, 0.05), L)
        elif kind == 1:
            out[k] = rs.binomial(1, rs.uniform(0.05, 0.5), L)
        elif kind == 2:
            tau = rs.randint(0, L + 1)
            out[k, tau:] = rs.binomial(1, 0.3, L - tau)
        elif kind == 3:
            out[k] = 1
        elif kind == 4:
            pass                       # all zeros: no event at all, carry through every batch
        else:
            out[k] = rs.binomial(1, 0.9, L) * rs.randint(1, 256)   # nonzero bytes other than 1
    return out.reshape(-1)


@pytest.mark.parametrize("per_batch,L", [(100, 4096), (100, 1000), (1, 37), (3, 301), (64, 640), (127, 1000),
                                         (128, 1031), (100, 1), (100, 100), (100, 199), (15, 300), (16, 400),
                                         (16, 1000), (17, 340), (50, 10000), (1, 100)])
@pytest.mark.parametrize("min_inst", [3, 5])
def test_scan_batches_equals_scan_streams(oracle_lib, per_batch, L, min_inst):
    rs = np.random.RandomState(per_batch * 7919 + L + min_inst)
    n = 600
    err = mixed_streams(rs, n, L)
    off = np.arange(n + 1, dtype=np.int64) * L
    ev, nev, st = gpu_scan_batches(err, n, L, per_batch=per_batch, min_inst=min_inst)
    ref_ev, _, ref_nev, ref_st, _ = gpu_scan(err, off, per_batch=per_batch, mode=1, min_inst=min_inst)
    assert np.array_equal(ev, ref_ev)
    assert np.array_equal(nev, ref_nev)
    np.testing.assert_array_equal(_state_matrix(st), _state_matrix(ref_st))
    if min_inst == 3:
        oev, _, ost, _ = oracle_scan_c(oracle_lib, err, off, per_batch=per_batch, mode=1)
        assert np.array_equal(ev, oev)
        np.testing.assert_array_equal(_state_matrix(st), ost)


def test_scan_batches_carried_state_and_perm_map(oracle_lib):
    """Non-fresh carry-in (batch 0 must be rescanned), a pending change (lazy reset) and
    events reported through perm_map labels."""
    from ddm_amd import kernels
    rs = np.random.RandomState(11)
    n, L, pb = 500, 1000, 100
    err = mixed_streams(rs, n, L)
    # carried states: run a prefix stream through the reference scan to get real DDM states
    pre = rs.binomial(1, 0.2, (n, 57)).astype(np.uint8).reshape(-1)
    _, _, _, st0, _ = gpu_scan(pre, np.arange(n + 1, dtype=np.int64) * 57, per_batch=1000, mode=1)
    st0 = st0.copy()
    st0["in_concept_change"][::7] = 1
    pmap = np.tile(rs.permutation(np.arange(L) % pb).astype(np.uint8), n)
    off = np.arange(n + 1, dtype=np.int64) * L
    ev, nev, st = gpu_scan_batches(err, n, L, per_batch=pb, state=st0, pmap=pmap)
    dev = torch.device("cuda", 0)
    nb = L // pb
    ref_ev = torch.empty((n * nb, 2), dtype=torch.int32, device=dev)
    ref_st = torch.from_numpy(st0.copy().view(np.uint8)).to(dev)
    ref_nev = torch.empty(n, dtype=torch.int64, device=dev)
    pad = np.zeros(n * L + 16, np.uint8)
    pad[:n * L] = err
    ppad = np.zeros_like(pad)
    ppad[:n * L] = pmap
    kernels.scan_streams(torch.from_numpy(pad).to(dev), torch.from_numpy(off).to(dev), kernels.params_struct(),
                         ref_st, torch.arange(n, dtype=torch.int64, device=dev) * nb, n * nb, ref_ev, nev=ref_nev,
                         mode=1, perm_map=torch.from_numpy(ppad).to(dev))
    torch.cuda.synchronize()
    assert np.array_equal(ev, ref_ev.cpu().numpy())
    assert np.array_equal(nev, ref_nev.cpu().numpy())
    np.testing.assert_array_equal(_state_matrix(st), _state_matrix(ref_st.cpu().numpy().view(kernels.STATE_DTYPE)))


def test_scan_batches_c4_shape(oracle_lib):
    """configs[3] shape generated on the device (20k streams x 4096 rows), against the C oracle."""
    from ddm_amd import kernels
    n, L = 20000, 4096
    dev = torch.device("cuda", 0)
    e = torch.empty(n * L + 16, dtype=torch.uint8, device=dev)
    kernels.synth_bernoulli_streams(e, n, L, seed=77)
    torch.cuda.synchronize()
    err = e[:n * L].cpu().numpy()
    ev, nev, st = gpu_scan_batches(err, n, L)
    oev, _, ost, _ = oracle_scan_c(oracle_lib, err, np.arange(n + 1, dtype=np.int64) * L, mode=1)
    assert np.array_equal(ev, oev)
    np.testing.assert_array_equal(_state_matrix(st), ost)
    assert (ev[:, 1] >= 0).mean() > 0.9     # reset-heavy: the speculation holds for most batches


def test_scan_batches_rejects_long_batches():
    from ddm_amd import kernels
    from ddm_amd._capi import DdmError
    dev = torch.device("cuda", 0)
    e = torch.zeros(512, dtype=torch.uint8, device=dev)
    st = torch.from_numpy(kernels.fresh_states(1).view(np.uint8)).to(dev)
    ev = torch.empty((2, 2), dtype=torch.int32, device=dev)
    fl = torch.empty(kernels.scan_batches_scratch_size(1, 258, 129), dtype=torch.uint8, device=dev)
    with pytest.raises(DdmError):
        kernels.scan_batches(e, 1, 258, kernels.params_struct(3, 129), st, ev, fl)


@pytest.mark.parametrize("per_batch,L", [(100, 100), (16, 16), (16, 32), (40, 80)])
def test_scan_batches_prefix_table_exhaustive(oracle_lib, per_batch, L):
    """Every 16-row error prefix (the spec kernel's prefix table, kPre = 16) opens a batch
    once, followed by random rows, against the C oracle: events and carried states."""
    rs = np.random.RandomState(per_batch + L)
    n = 1 << 16
    err = rs.binomial(1, 0.15, (n, L)).astype(np.uint8)
    bits = (np.arange(n)[:, None] >> np.arange(16)[None, :]) & 1
    err[:, :16] = bits
    err = err.reshape(-1)
    off = np.arange(n + 1, dtype=np.int64) * L
    ev, nev, st = gpu_scan_batches(err, n, L, per_batch=per_batch)
    oev, _, ost, _ = oracle_scan_c(oracle_lib, err, off, per_batch=per_batch, mode=1)
    assert np.array_equal(ev, oev)
    np.testing.assert_array_equal(_state_matrix(st), ost)


def test_scan_batches_c4_full_size():
    """configs[3] at FULL size, built exactly as `bench.py --workload c4` builds it (1M streams
    x 4096 rows, Bernoulli streams from the bench's seed): every event, event count and end
    state of ddm_scan_batches against the C oracle over all 1M streams (oracle/scan.py,
    DDM_Process.py:135-159 with the reset of :207-210) and against ddm_scan_streams in mode 1.
    Only at this size do the chain kernel's carried streams outnumber its waves (grid
    stride) and the classify pass run ~156 fills per wave."""
    import bench
    from ddm_amd import kernels
    from oracle.scan import scan_equal_streams
    from test_gpu_scan import _state_matrix
    S, L, pb = 1_000_000, 4096, 100
    nb = -(-L // pb)
    dev = torch.device("cuda", 0)
    err = torch.empty(S * L + 16, dtype=torch.uint8, device=dev)
    kernels.synth_bernoulli_streams(err, S, L, bench.SEED)
    ev = torch.full((S * nb, 2), 7, dtype=torch.int32, device=dev)
    scratch = torch.empty(kernels.scan_batches_scratch_size(S, L), dtype=torch.uint8, device=dev)
    st = torch.from_numpy(kernels.fresh_states(S).view(np.uint8)).to(dev)
    nev = torch.empty(S, dtype=torch.int64, device=dev)
    kernels.scan_batches(err, S, L, kernels.params_struct(), st, ev, scratch, nev=nev)
    # the oracle-pinned one-lane kernel on the same device bytes
    off = torch.arange(S + 1, dtype=torch.int64, device=dev) * L
    ref_ev = torch.full((S * nb, 2), 7, dtype=torch.int32, device=dev)
    ref_st = torch.from_numpy(kernels.fresh_states(S).view(np.uint8)).to(dev)
    ref_nev = torch.empty(S, dtype=torch.int64, device=dev)
    kernels.scan_streams(err, off, kernels.params_struct(), ref_st, torch.arange(S, dtype=torch.int64, device=dev) * nb,
                         S * nb, ref_ev, nev=ref_nev, mode=1)
    torch.cuda.synchronize()
    assert torch.equal(ev, ref_ev)
    assert torch.equal(nev, ref_nev)
    assert torch.equal(st, ref_st)
    evh = ev.cpu().numpy()
    sth = _state_matrix(st.cpu().numpy().view(kernels.STATE_DTYPE))
    del ref_ev, ref_st, scratch
    oev, ost = scan_equal_streams(err[:S * L].cpu().numpy(), S, L, per_batch=pb, mode=1, threads=16)
    assert np.array_equal(evh, oev)
    np.testing.assert_array_equal(sth, ost)
    o_nev = ((oev[:, 0] >= 0) | (oev[:, 1] >= 0)).reshape(S, nb).sum(axis=1)
    assert np.array_equal(nev.cpu().numpy(), o_nev)
    assert (oev[:, 1] >= 0).mean() > 0.9
