"""ddm_scan_streams (HIP) vs the oracle: events, stop batch, carried state and the p/s
trace must be bit-identical (the kernel runs the same fp64 recurrence, no FMA)."""
import numpy as np
import pytest
import torch

from conftest import load_npz, oracle_scan_c

pytestmark = pytest.mark.gpu


def _dev():
    return torch.device("cuda", 0)


def gpu_scan(err, offsets, per_batch=100, mode=0, hint=None, state=None, trace=False, min_inst=3, wl=0.5, cl=1.5):
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
    ev = torch.empty((max(int(nb.sum()), 1), 2), dtype=torch.int32, device=dev)
    stop = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    nev = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
    ps = torch.full((max(len(err), 1), 2), float("nan"), dtype=torch.float64, device=dev) if trace else None
    hint_t = torch.from_numpy(np.asarray(hint, dtype=np.uint64).view(np.int64)).to(dev) if hint is not None else None
    prm = kernels.params_struct(min_inst, per_batch, wl, cl)
    kernels.scan_streams(e, torch.from_numpy(offsets).to(dev), prm, st, torch.from_numpy(base).to(dev),
                         int(nb.sum()), ev, first_nz=hint_t, stop=stop, nev=nev, mode=mode, ps=ps)
    torch.cuda.synchronize()
    out_state = st.cpu().numpy().view(kernels.STATE_DTYPE)
    return (ev.cpu().numpy()[:int(nb.sum())], stop.cpu().numpy()[:n], nev.cpu().numpy()[:n], out_state,
            ps.cpu().numpy()[:len(err)] if trace else None)


def random_streams(rs, n, max_len=3000):
    streams = []
    for i in range(n):
        L = int(rs.choice([0, 1, 2, 3, 50, 99, 100, 101, 199, 200, 1000, max_len]))
        kind = i % 5
        if kind == 0:
            s = rs.binomial(1, rs.uniform(0.001, 0.5), L)
        elif kind == 1:      # clean prefix then noise: exercises the zero-run skip
            s = np.zeros(L, int)
            k = int(L * rs.uniform(0.3, 1.0))
            s[k:] = rs.binomial(1, 0.2, L - k)
        elif kind == 2:
            s = np.ones(L, int)
        elif kind == 3:
            s = np.zeros(L, int)
            if L > 5:
                s[rs.randint(0, L, 3)] = 1
        else:
            s = (np.arange(L) % 2).astype(int)
        streams.append(s.astype(np.uint8))
    err = np.concatenate(streams) if streams else np.zeros(0, np.uint8)
    off = np.concatenate([[0], np.cumsum([len(s) for s in streams])]).astype(np.int64)
    return err, off


def first_nonzero(err, off):
    out = np.empty(len(off) - 1, dtype=np.uint64)
    for i in range(len(off) - 1):
        nz = np.nonzero(err[off[i]:off[i + 1]])[0]
        out[i] = off[i] + nz[0] if len(nz) else np.iinfo(np.uint64).max
    return out


def _state_matrix(st):
    return np.stack([st["miss_prob"], st["miss_std"], st["miss_prob_min"], st["miss_sd_min"],
                     st["miss_prob_sd_min"], st["sample_count"].astype(np.float64),
                     st["in_concept_change"].astype(np.float64), st["in_warning_zone"].astype(np.float64)], axis=1)


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("use_hint", [False, True])
def test_scan_matches_oracle_random(oracle_lib, mode, use_hint):
    rs = np.random.RandomState(100 + mode)
    err, off = random_streams(rs, 400)
    hint = first_nonzero(err, off) if use_hint else None
    ev, stop, nev, st, ps = gpu_scan(err, off, mode=mode, hint=hint, trace=True)
    oev, ostop, ost, ops = oracle_scan_c(oracle_lib, err, off, mode=mode, trace=True)
    assert np.array_equal(ev, oev)
    if mode == 0:
        assert np.array_equal(stop, ostop)
    np.testing.assert_array_equal(_state_matrix(st), ost)
    np.testing.assert_array_equal(ps, ops)   # bit-exact p and s (tolerance 1e-12 rel not needed)
    lens = np.diff(off)
    nbs = (lens + 99) // 100
    base = np.concatenate([[0], np.cumsum(nbs)])
    for i in range(len(lens)):
        e = oev[base[i]:base[i + 1]]
        assert nev[i] == int(((e[:, 0] >= 0) | (e[:, 1] >= 0)).sum())


@pytest.mark.parametrize("per_batch", [1, 7, 64, 256])
def test_scan_batch_sizes(oracle_lib, per_batch):
    rs = np.random.RandomState(per_batch)
    err, off = random_streams(rs, 100, max_len=2000)
    for mode in (0, 1):
        ev, stop, _, st, _ = gpu_scan(err, off, per_batch=per_batch, mode=mode)
        oev, ostop, ost, _ = oracle_scan_c(oracle_lib, err, off, per_batch=per_batch, mode=mode)
        assert np.array_equal(ev, oev) and np.array_equal(stop, ostop)
        np.testing.assert_array_equal(_state_matrix(st), ost)


def test_scan_state_carry_across_calls(oracle_lib):
    """Splitting a stream at a batch boundary and carrying ddm_state == one call."""
    rs = np.random.RandomState(7)
    s = np.concatenate([np.zeros(5000, np.uint8), rs.binomial(1, 0.02, 3000).astype(np.uint8)])
    full_ev, full_stop, _, full_st, _ = gpu_scan(s, [0, len(s)], mode=1)
    cut = 4200
    ev1, _, _, st1, _ = gpu_scan(s[:cut], [0, cut], mode=1)
    ev2, _, _, st2, _ = gpu_scan(s[cut:], [0, len(s) - cut], mode=1, state=st1)
    assert np.array_equal(np.concatenate([ev1, ev2]), full_ev)
    np.testing.assert_array_equal(_state_matrix(st2), _state_matrix(full_st))


def test_scan_known_answers():
    kat = load_npz("ddm_kat.npz")
    for name in sorted({k.split("/")[0] for k in kat.files}):
        x = kat[name + "/x"]
        _, _, _, _, ps = gpu_scan(x, [0, len(x)], per_batch=256, mode=1, trace=True)
        n = len(x)
        ch = np.nonzero(kat[name + "/change"])[0]
        upto = (ch[0] + 1) if len(ch) else n
        np.testing.assert_array_equal(ps[:upto, 0], kat[name + "/p"][:upto])
        np.testing.assert_array_equal(ps[:upto, 1], kat[name + "/s"][:upto])


def test_scan_c4_shaped_synthetic(oracle_lib):
    """C4 shape (Bernoulli r0 -> r0+step streams of 4096 rows, fresh DDM after each change),
    generated on the device, 20k streams."""
    from ddm_amd import kernels
    n_streams, L = 20000, 4096
    dev = _dev()
    e = torch.empty(n_streams * L + 16, dtype=torch.uint8, device=dev)
    kernels.synth_bernoulli_streams(e, n_streams, L, seed=2024)
    torch.cuda.synchronize()
    err = e[:n_streams * L].cpu().numpy()
    assert 0.02 < err.mean() < 0.4
    off = np.arange(n_streams + 1, dtype=np.int64) * L
    ev, _, nev, st, _ = gpu_scan(err, off, mode=1)
    oev, _, ost, _ = oracle_scan_c(oracle_lib, err, off, mode=1)
    assert np.array_equal(ev, oev)
    np.testing.assert_array_equal(_state_matrix(st), ost)
    assert (oev[:, 1] >= 0).sum() > n_streams  # reset-heavy


def test_scan_lazy_reset_on_carried_change():
    """A carried detector with in_concept_change=1 resets on its next element (skmultiflow)."""
    from ddm_amd import kernels
    from oracle.ddm import OracleDDM
    st = kernels.fresh_states(1)
    st["in_concept_change"] = 1
    st["miss_prob"] = 0.3
    st["sample_count"] = 50
    x = np.array([0, 0, 1, 0, 0, 0, 1, 1], np.uint8)
    # per_batch=1: a fresh DDM at the next batch == skmultiflow's lazy reset at the next element
    _, _, _, out, ps = gpu_scan(x, [0, len(x)], per_batch=1, mode=1, state=st, trace=True)
    d = OracleDDM()
    d.in_concept_change = True
    for t, v in enumerate(x):
        d.add(int(v))
        assert ps[t, 0] == d.miss_prob and ps[t, 1] == d.miss_std


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("min_inst", [3, 5])
@pytest.mark.parametrize("per_batch", [3, 100])
def test_fast_scan_equals_trace_scan(oracle_lib, mode, min_inst, per_batch):
    """The production scan (Markstein division, fresh/trivial shortcuts, several streams per
    lane) against the reference-shaped trace kernel and the C oracle: events, stop batch,
    event counts and the carried state, bit for bit."""
    rs = np.random.RandomState(1000 + 10 * mode + min_inst + per_batch)
    err, off = random_streams(rs, 3000, max_len=5000)
    hint = first_nonzero(err, off)
    fast = gpu_scan(err, off, per_batch=per_batch, mode=mode, hint=hint, min_inst=min_inst)
    slow = gpu_scan(err, off, per_batch=per_batch, mode=mode, hint=hint, min_inst=min_inst, trace=True)
    for a, b in zip(fast[:3], slow[:3]):
        assert np.array_equal(a, b)
    np.testing.assert_array_equal(_state_matrix(fast[3]), _state_matrix(slow[3]))
    if min_inst == 3:
        oev, ostop, ost, _ = oracle_scan_c(oracle_lib, err, off, per_batch=per_batch, mode=mode)
        assert np.array_equal(fast[0], oev)
        np.testing.assert_array_equal(_state_matrix(fast[3]), ost)


def test_fast_scan_long_counts_use_ieee_reciprocal(oracle_lib):
    """Detectors past n = 4096 (reciprocal table) divide exactly as well."""
    rs = np.random.RandomState(5)
    s = np.concatenate([rs.binomial(1, 0.3, 20000), rs.binomial(1, 0.6, 20000)]).astype(np.uint8)
    off = np.array([0, len(s)], np.int64)
    for mode in (0, 1):
        fast = gpu_scan(s, off, per_batch=256, mode=mode)
        oev, ostop, ost, _ = oracle_scan_c(oracle_lib, s, off, per_batch=256, mode=mode)
        assert np.array_equal(fast[0], oev) and np.array_equal(fast[1], ostop)
        np.testing.assert_array_equal(_state_matrix(fast[3]), ost)
