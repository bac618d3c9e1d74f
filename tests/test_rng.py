"""Native MT19937 (ddm_mt_* in the C-ABI, host code) == numpy's legacy RandomState, the RNG
the reference shuffles batches (DDM_Process.py:187,190) and seeds forests (:102) with."""
import numpy as np
import pandas as pd
import pytest

from ddm_amd.rng import MTStream


@pytest.mark.parametrize("seed", [0, 1000, 1015, 2**31 - 1])
def test_perms_match_numpy_permutation(seed):
    rs = np.random.RandomState(seed)
    mt = MTStream.from_seed(seed)
    lens = np.array([100, 100, 37, 1, 2, 256, 100, 0, 5] * 40, dtype=np.int32)
    draws = np.zeros(len(lens), dtype=np.int64)
    got = mt.perms(lens, draws=draws)
    want = np.concatenate([rs.permutation(n) for n in lens]).astype(np.uint8)
    assert np.array_equal(got, want)
    st_np, st_mt = rs.get_state(), mt.numpy_state()
    assert np.array_equal(st_np[1], st_mt[1]) and st_np[2] == st_mt[2]
    assert (draws[lens > 1] >= lens[lens > 1] - 1).all()


def test_pandas_sample_is_permutation():
    np.random.seed(42)
    mt = MTStream.from_global()
    df = pd.DataFrame({"a": np.arange(100)})
    assert np.array_equal(df.sample(frac=1).index.to_numpy(), mt.perms([100]))


def test_randint31_matches_numpy():
    rs = np.random.RandomState(9)
    mt = MTStream.from_seed(9)
    want = [rs.randint(2147483647) for _ in range(1000)]
    assert np.array_equal(mt.randint31(1000), np.array(want))


def test_sklearn_forest_draws_100_seeds():
    """RandomForestClassifier.fit with random_state=None draws 100 randint(2**31-1) from the
    global RNG (sklearn ensemble/_base.py _set_random_states)."""
    from sklearn.ensemble import RandomForestClassifier
    np.random.seed(5)
    mt = MTStream.from_global()
    X = np.random.RandomState(0).rand(50, 3)
    y = np.arange(50) % 2
    RandomForestClassifier().fit(X, y)
    mt.randint31(100)
    a, b = np.random.get_state(), mt.numpy_state()
    assert np.array_equal(a[1], b[1]) and a[2] == b[2]


def test_skip_equals_draw():
    a, b = MTStream.from_seed(3), MTStream.from_seed(3)
    d = np.zeros(50, dtype=np.int64)
    a.perms(np.full(50, 100, np.int32), draws=d)
    b.skip(int(d.sum()))
    assert np.array_equal(a.key, b.key) and a.pos.value == b.pos.value
    b.skip(10_000)
    rs = a.to_random_state()
    for _ in range(10_000):
        rs.randint(0, 2**32, dtype=np.uint64)  # one 32-bit word each
    a.load_random_state(rs)
    assert np.array_equal(a.key, b.key) and a.pos.value == b.pos.value


def test_snapshot_restore_roundtrip():
    mt = MTStream.from_seed(11)
    snap = mt.snapshot()
    x = mt.perms([100, 100])
    mt.restore(snap)
    assert np.array_equal(mt.perms([100, 100]), x)


@pytest.mark.parametrize("seed", [0, 1, 123, 1000, 1015, 2**31 - 1, 2**32 - 1])
def test_from_seed_native_matches_numpy(seed):
    """ddm_mt_seed (ABI 24) == numpy's legacy RandomState(seed) state, and the draws after it."""
    st = MTStream.from_seed(seed)
    ref = np.random.RandomState(seed).get_state()
    assert np.array_equal(st.key, ref[1]) and st.pos.value == ref[2] and st.gauss == (ref[3], ref[4])
    rs = np.random.RandomState(seed)
    want = np.concatenate([rs.permutation(100) for _ in range(5)]).astype(np.uint8)
    assert np.array_equal(st.perms(np.full(5, 100, np.int32)), want)


def test_untemper_inverts_tempering():
    """shuffle.untemper_keys (uint32 closed forms, round 6) inverts MT19937's tempering."""
    from ddm_amd.shuffle import _temper, untemper_keys
    x = np.random.default_rng(5).integers(0, 2**32, 200_000, dtype=np.uint64).astype(np.uint32)
    x[:4] = [0, 1, 0xffffffff, 0x80000000]
    got = untemper_keys(_temper(x))
    assert got.dtype == np.uint32 and np.array_equal(got, x)
