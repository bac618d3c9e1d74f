"""Forest export (host side of ddm_forest_predict): the BFS-renumbered 16-byte node layout
walked by a plain-Python emulation of the kernel's traversal equals sklearn's predict."""
import numpy as np
import pytest
from sklearn.ensemble import RandomForestClassifier

from ddm_amd.forest import MISSING_LEFT_BIT, pack, pack_sklearn, tree_arrays
from oracle import forest as oforest


def walk_packed(pf, X32):
    """What k_forest_predict computes, restated in numpy (test helper)."""
    n = len(X32)
    k = pf.n_classes
    votes = np.zeros((n, k), dtype=np.float64)
    for t in range(pf.n_trees):
        node = np.full(n, pf.roots[t], dtype=np.int64)
        while True:
            f = pf.nodes["feature"][node]
            inner = f >= 0
            if not inner.any():
                break
            r = np.nonzero(inner)[0]
            nd = node[r]
            fi = pf.nodes["feature"][nd] & (MISSING_LEFT_BIT - 1)
            xv = X32[r, fi].astype(np.float64)
            left = xv <= pf.nodes["threshold"][nd]
            nan = np.isnan(xv)
            left = np.where(nan, (pf.nodes["feature"][nd] & MISSING_LEFT_BIT) != 0, left)
            node[r] = pf.nodes["child"][nd] + np.where(left, 0, 1)
        leaf = pf.nodes["child"][node]
        if pf.pure:
            votes[np.arange(n), leaf] += 1.0
        else:
            votes += pf.leaf_value[leaf]
    if not pf.pure:
        votes /= pf.n_trees
    return pf.classes[np.argmax(votes, axis=1)]


@pytest.mark.parametrize("dup", [False, True])
def test_packed_walk_equals_sklearn(dup):
    rs = np.random.RandomState(4)
    X = rs.rand(100, 7)
    y = rs.randint(0, 5, 100) * 3 + 2
    if dup:  # identical rows with different labels -> impure leaves
        X[10:20] = X[0]
    rf = RandomForestClassifier(random_state=rs).fit(X, y)
    pf = pack_sklearn(rf)
    assert pf.pure == (not dup)
    Xt = rs.rand(500, 7).astype(np.float32)
    Xt[::17, 2] = np.nan
    assert np.array_equal(walk_packed(pf, Xt), rf.predict(Xt))


def test_trace_forests_pack_and_predict():
    from conftest import golden_partitions, load_npz
    tr = load_npz("outdoor_trace_m4_i16.npz")
    d, part, _ = golden_partitions(4, 16)[1]
    trees = [{key: tr[f"{d}/fit0/tree{t}/{key}"] for key in ("left", "right", "feature", "threshold", "value",
                                                                "missing_left")} for t in range(100)]
    pf = pack(trees, tr[f"{d}/fit0/classes"])
    X32 = part[[str(i) for i in range(21)]].to_numpy().astype(np.float32)
    assert np.array_equal(walk_packed(pf, X32), oforest.predict(trees, pf.classes, X32))


def test_class_limits():
    """ddm_forest_predict takes up to 256 classes (70 pack; a batch of <= 256 rows cannot
    hold more); more is refused.  The native trainer hands > 64 classes to sklearn."""
    from ddm_amd.trainer import BatchForestTrainer, NativeForestTrainer
    rs = np.random.RandomState(0)
    X = rs.rand(300, 3)
    y = np.arange(300) % 70
    rf = RandomForestClassifier(n_estimators=3, random_state=0).fit(X, y)
    pf = pack(tree_arrays(rf), rf.classes_)
    assert len(pf.classes) == 70
    y2 = np.arange(300) % 257
    rf2 = RandomForestClassifier(n_estimators=3, random_state=0).fit(X, y2)
    with pytest.raises(ValueError):
        pack(tree_arrays(rf2), rf2.classes_)
    X32 = X[:100].astype(np.float32)
    assert NativeForestTrainer(n_estimators=3).fit(X32, y[:100], np.arange(3)) is None
    out = BatchForestTrainer(n_estimators=3, n_threads=2).fit_many([(X32, y[:100], np.arange(3)),
                                                                    (X32, y[:100] % 5, np.arange(3))])
    assert out[0] is None and out[1] is not None

