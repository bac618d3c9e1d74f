"""ddm_rf_fit (native restatement of sklearn 1.7.2's RandomForestClassifier.fit) must grow
IDENTICAL trees: packed nodes, roots and leaf values equal, bit for bit — against sklearn
on varied data and against the reference's own refits (trace fixtures)."""
import numpy as np
import pytest
from sklearn.ensemble import RandomForestClassifier

from conftest import golden_partitions, load_npz
from ddm_amd.rng import MTStream
from ddm_amd.trainer import NativeForestTrainer
from ddm_amd.treepack import pack, pack_sklearn


def assert_same(a, b):
    assert a.pure == b.pure
    assert np.array_equal(a.roots, b.roots)
    assert a.nodes.shape == b.nodes.shape
    for f in ("threshold", "feature", "child"):
        assert np.array_equal(a.nodes[f], b.nodes[f]), f
    assert np.array_equal(a.classes, b.classes)
    if not a.pure:
        assert np.array_equal(a.leaf_value, b.leaf_value)


def native_vs_sklearn(X, y, seed, T=100):
    X32 = np.asarray(X, dtype=np.float32)
    rs = np.random.RandomState(seed)
    rf = RandomForestClassifier(n_estimators=T, random_state=rs).fit(X32.astype(np.float64), y)
    want = pack_sklearn(rf)
    seeds = MTStream.from_seed(seed).randint31(T)
    got = NativeForestTrainer(T).fit(X32, y, seeds)
    assert_same(got, want)
    return got


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("K,F", [(2, 27), (3, 21), (10, 27), (7, 1), (40, 21)])
def test_random_data(seed, K, F):
    rs = np.random.RandomState(seed * 100 + K)
    X = rs.rand(100, F)
    y = rs.randint(0, K, 100) * 3 + 1
    native_vs_sklearn(X, y, seed)


@pytest.mark.parametrize("seed", range(4))
def test_ties_constants_duplicates(seed):
    rs = np.random.RandomState(seed)
    X = np.round(rs.rand(100, 9) * 4) / 4          # many ties
    X[:, 2] = 0.5                                   # constant feature
    X[:, 5] = X[:, 1] + 5e-8                        # within FEATURE_THRESHOLD of another
    X[10:30] = X[0]                                 # duplicate rows ...
    y = rs.randint(0, 3, 100)                       # ... with different labels -> impure
    got = native_vs_sklearn(X, y, seed)
    assert not got.pure


def test_single_class_and_small_n():
    rs = np.random.RandomState(1)
    native_vs_sklearn(rs.rand(100, 5), np.full(100, 4), 3)
    native_vs_sklearn(rs.rand(7, 5), np.arange(7) % 2, 4)
    native_vs_sklearn(rs.rand(1, 3), np.array([2]), 5)


def test_nan_rejected_for_sklearn():
    X = np.random.RandomState(0).rand(100, 4).astype(np.float32)
    X[3, 1] = np.nan
    assert NativeForestTrainer(10).fit(X, np.arange(100) % 2, np.arange(10)) is None


@pytest.mark.parametrize("mult,inst", [(2, 1), (4, 16)])
def test_reference_refits(mult, inst):
    """The forests the reference itself fitted (train_rf, DDM_Process.py:98-105) on its
    shuffled drift batches, regrown natively from the same global-RNG seeds."""
    tr = load_npz(f"outdoor_trace_m{mult}_i{inst}.npz")
    checked = 0
    for d, part, _ in golden_partitions(mult, inst)[:4]:
        X32 = part[[str(i) for i in range(21)]].to_numpy().astype(np.float32)
        y = part["target"].to_numpy()
        # replay the partition's RNG to find each fit's seeds
        from oracle.controller import run_partition
        rec = []
        np.random.seed(1000 + d)
        seeds_at = []
        import sklearn.ensemble._forest as forest_mod
        orig = forest_mod.RandomForestClassifier.fit

        def spy(self, X, yy, *a, **k):
            st = np.random.get_state()
            seeds_at.append(MTStream.from_numpy_state(st).randint31(100))
            return orig(self, X, yy, *a, **k)
        forest_mod.RandomForestClassifier.fit = spy
        try:
            run_partition(part[[str(i) for i in range(21)]].to_numpy(), y, part.index.to_numpy(),
                          part["full_df_row_number"].to_numpy(), record=rec)
        finally:
            forest_mod.RandomForestClassifier.fit = orig
        k = 0
        while f"{d}/fit{k}/rows" in tr.files:
            if f"{d}/fit{k}/tree0/left" in tr.files:
                rows = tr[f"{d}/fit{k}/rows"]
                trees = [{key: tr[f"{d}/fit{k}/tree{t}/{key}"] for key in
                          ("left", "right", "feature", "threshold", "value", "missing_left")} for t in range(100)]
                want = pack(trees, tr[f"{d}/fit{k}/classes"])
                got = NativeForestTrainer(100).fit(X32[rows], y[rows], seeds_at[k])
                assert_same(got, want)
                checked += 1
            k += 1
    assert checked >= 3
