"""GPU batch shuffles (csrc/shuffle.hip) == numpy's legacy permutation stream, draw for draw."""
import numpy as np
import pytest
import torch

from ddm_amd.rng import MTStream

pytestmark = pytest.mark.gpu


def _mk(L, cap=1 << 20, max_window=70000):
    from ddm_amd.shuffle import GpuShuffle
    dev = torch.device("cuda", 0)
    return GpuShuffle(dev, L, cap, max_window, torch.cuda.current_stream(dev))


def test_raw_stream_equals_numpy():
    sh = _mk(100)
    for seed, pre in ((1, 0), (2, 5), (3, 623), (4, 624 * 3 + 17)):
        mt = MTStream.from_seed(seed)
        mt.skip(pre)
        sh.reset(mt)
        got = sh.words(0, 50000).copy()
        rs = np.random.RandomState(seed)
        if pre:
            rs.randint(0, 2**32, pre, dtype=np.uint64)
        want = rs.randint(0, 2**32, 50000, dtype=np.uint64).astype(np.uint32)
        assert np.array_equal(got, want), (seed, pre)


@pytest.mark.parametrize("L", [100, 2, 7, 256])
def test_windows_equal_host_permutations(L):
    sh = _mk(L)
    for seed, pre in ((11, 0), (12, 333)):
        mt = MTStream.from_seed(seed)
        mt.skip(pre)
        host = mt.copy()
        sh.reset(mt)
        dev = torch.device("cuda", 0)
        P = 0
        for W in (1, 3, 64, 1000, 9000):
            out = torch.zeros(W * L, dtype=torch.uint8, device=dev)
            sh.window(P, W, out)
            torch.cuda.synchronize()
            draws = np.zeros(W, dtype=np.int64)
            want = host.perms(np.full(W, L, np.int32), draws=draws)
            assert np.array_equal(out.cpu().numpy(), want), (seed, W)
            E = sh.E[:W].cpu().numpy()
            assert np.array_equal(E, P + np.cumsum(draws) - 1)
            info = sh.info.cpu().numpy()
            assert info[2] >= W
            P = int(E[-1]) + 1
            ns = sh.numpy_state(P)
            assert np.array_equal(ns[1], host.key) and ns[2] == host.pos.value


def test_host_helpers_interleave_with_windows():
    """The controller's sequence: window, host perm, seeds, window — same as numpy."""
    sh = _mk(100)
    mt = MTStream.from_seed(99)
    sh.reset(mt)
    rs = np.random.RandomState(99)
    dev = torch.device("cuda", 0)
    out = torch.zeros(500 * 100, dtype=torch.uint8, device=dev)
    sh.window(0, 500, out)
    torch.cuda.synchronize()
    want = np.concatenate([rs.permutation(100) for _ in range(500)])
    assert np.array_equal(out.cpu().numpy(), want)
    P = int(sh.E[499].item()) + 1
    perm, P = sh.host_perm(P, 100)
    assert np.array_equal(perm, rs.permutation(100))
    seeds, P = sh.host_seeds(P, 100)
    assert np.array_equal(seeds, [rs.randint(2147483647) for _ in range(100)])
    perm, P = sh.host_perm(P, 37)
    assert np.array_equal(perm, rs.permutation(37))
    sh.window(P, 200, out)
    torch.cuda.synchronize()
    want = np.concatenate([rs.permutation(100) for _ in range(200)])
    assert np.array_equal(out[:20000].cpu().numpy(), want)
    P = int(sh.E[199].item()) + 1
    ns = sh.numpy_state(P)
    st = rs.get_state()
    assert np.array_equal(ns[1], st[1]) and ns[2] == st[2]


def test_stream_growth():
    """Capacity grows (R and tables copied) when a window needs more draws."""
    sh = _mk(100, cap=20000, max_window=5000)
    mt = MTStream.from_seed(5)
    host = mt.copy()
    sh.reset(mt)
    dev = torch.device("cuda", 0)
    out = torch.zeros(5000 * 100, dtype=torch.uint8, device=dev)
    sh.window(0, 5000, out)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), host.perms(np.full(5000, 100, np.int32)))


@pytest.mark.parametrize("jump", [5000, 1 << 13])
def test_raw_stream_across_jump_segments(monkeypatch, jump):
    """Segments after the first start from jumped states (ddm_mt_jump): the whole stream is
    still numpy's, draw for draw, whatever the start position inside a block."""
    from ddm_amd import shuffle
    monkeypatch.setattr(shuffle, "JUMP", jump)
    sh = _mk(100, cap=400000)
    for seed, pre in ((21, 0), (22, 5), (23, 623), (24, 624 * 2 + 300)):
        mt = MTStream.from_seed(seed)
        mt.skip(pre)
        sh.reset(mt)
        got = sh.words(0, 300000).copy()
        rs = np.random.RandomState(seed)
        if pre:
            rs.randint(0, 2**32, pre, dtype=np.uint64)
        want = rs.randint(0, 2**32, 300000, dtype=np.uint64).astype(np.uint32)
        assert np.array_equal(got, want), (seed, pre, int(np.argmax(got != want)))


def test_raw_stream_default_segments():
    """The production segment length (2^20 draws): a stream of 2.5M draws spans 3 segments."""
    sh = _mk(100, cap=3 << 20)
    mt = MTStream.from_seed(31)
    mt.skip(77)
    sh.reset(mt)
    n = 2_500_000
    got = sh.words(0, n).copy()
    rs = np.random.RandomState(31)
    rs.randint(0, 2**32, 77, dtype=np.uint64)
    want = rs.randint(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    assert np.array_equal(got, want), int(np.argmax(got != want))


def _host_prefix(words, L, chunks):
    """Tpre[c][k][s-1] by direct simulation: every start state through the chunk's draws."""
    S = L - 1
    masks = np.array([0] + [(1 << int(s).bit_length()) - 1 for s in range(1, S + 1)], dtype=np.uint64)
    out = np.zeros((chunks, 64, S), dtype=np.uint32)
    for c in range(chunks):
        st = np.arange(1, S + 1)
        done = np.zeros(S, dtype=np.int64)
        for k in range(64):
            for v in words[c * 8192 + k * 128: c * 8192 + (k + 1) * 128].astype(np.uint64):
                acc = (v & masks[st]) <= st
                wrap = acc & (st == 1)
                done += wrap
                st = np.where(wrap, S, np.where(acc, st - 1, st))
            out[c, k] = st | (done << 8)
    return out


@pytest.mark.parametrize("L", [100, 2, 37, 256])
def test_prefix_tables_equal_direct_simulation(L):
    """k_fsm_prefix (coupled trajectories merged) == every start state simulated alone."""
    sh = _mk(L, cap=1 << 17)
    mt = MTStream.from_seed(1234 + L)
    sh.reset(mt)
    chunks = 3
    sh.ensure(chunks * 8192)
    torch.cuda.synchronize()
    words = sh.words(0, chunks * 8192).copy()
    want = _host_prefix(words, L, chunks)
    got = sh.Tpre[:chunks * 64 * (L - 1)].cpu().numpy().view(np.uint32).reshape(chunks, 64, L - 1)
    assert np.array_equal(got, want)
    tc = sh.Tchunk[:chunks * (L - 1)].cpu().numpy().view(np.uint32).reshape(chunks, L - 1)
    assert np.array_equal(tc, want[:, 63])


@pytest.mark.parametrize("L", [100, 2, 7, 256])
def test_window_batch_small_and_large_windows(L):
    """ddm_shuffle_window_batch (the controller's batched window shuffles): short and long
    windows in one call, every one through the first / walk / replay / perms kernels; every
    partition's perm bytes and E equal numpy's permutation stream (DDM_Process.py:187,
    :190)."""
    import ctypes
    from ddm_amd import kernels
    from ddm_amd._capi import check, lib
    dev = torch.device("cuda", 0)
    Ws = [1, 5, 16, 17, 40, 3, 16, 300]
    shs, hosts, outs, recs = [], [], [], []
    for k, W in enumerate(Ws):
        sh = _mk(L, cap=1 << 19, max_window=1024)
        mt = MTStream.from_seed(500 + k)
        mt.skip(17 * k)
        host = mt.copy()
        sh.reset(mt)
        P = 0
        if k % 2:                     # a window that does not start at draw 0
            pre = np.zeros(3, dtype=np.int64)
            host.perms(np.full(3, L, np.int32), draws=pre)
            P = int(pre.sum())
        sh.ensure(P + sh.window_draws(W))
        out = torch.zeros(W * L, dtype=torch.uint8, device=dev)
        rec = np.zeros(1, kernels.JOB_DTYPE)
        sh.fill_job(rec[0], P, W, out.data_ptr())
        shs.append(sh)
        hosts.append((host, P))
        outs.append(out)
        recs.append(rec)
    table = torch.from_numpy(np.concatenate(recs).view(np.uint8)).to(dev)
    torch.cuda.synchronize()
    s = torch.cuda.current_stream(dev)
    check(lib.ddm_shuffle_window_batch(table.data_ptr(), len(Ws), max(Ws), 2 + 64 + 300 * L * 2 // 8192 + 2, L,
                                       ctypes.c_void_p(s.cuda_stream), None, None), "ddm_shuffle_window_batch")
    torch.cuda.synchronize()
    for k, W in enumerate(Ws):
        host, P = hosts[k]
        draws = np.zeros(W, dtype=np.int64)
        want = host.perms(np.full(W, L, np.int32), draws=draws)
        assert np.array_equal(outs[k].cpu().numpy(), want), (k, W)
        assert np.array_equal(shs[k].E[:W].cpu().numpy(), P + np.cumsum(draws) - 1), (k, W)
