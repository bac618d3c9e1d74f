"""Device forest refit (ddm_rf_fit_device) against the host trainer (ddm_rf_fit_many,
itself pinned to scikit-learn 1.7.2 by test_trainer.py): identical packed forests
(node for node, thresholds bit for bit), leaf values, classes and compiled blobs."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _host(batches):
    from ddm_amd.trainer import BatchForestTrainer
    return BatchForestTrainer(100, n_threads=4).fit_many(batches)


def _device(batches, k_cap=16, fused=True):
    from ddm_amd.dfit import DeviceTrainer
    return DeviceTrainer(100, k_cap=k_cap, fused=fused).fit_many(batches)


def _same(h, d):
    pf, blob, head = h
    dpf, dblob, dhead, res = d
    assert res[0] == 0
    assert dpf.pure == pf.pure
    assert np.array_equal(dpf.classes, pf.classes)
    assert np.array_equal(dpf.roots, pf.roots)
    assert dpf.nodes.shape == pf.nodes.shape
    assert np.array_equal(dpf.nodes["feature"], pf.nodes["feature"])
    assert np.array_equal(dpf.nodes["child"], pf.nodes["child"])
    assert np.array_equal(dpf.nodes["threshold"].view(np.uint64), pf.nodes["threshold"].view(np.uint64))
    if not pf.pure:
        assert np.array_equal(dpf.leaf_value, pf.leaf_value)
    assert (blob is None) == (dblob is None)
    if blob is not None:
        assert head == dhead
        assert np.array_equal(blob, dblob)


def _batch(rs, L, F, K, kind):
    if kind == "separable":                      # the C3 refit batch: two classes, stumps
        y = np.repeat([3, 7], [L // 2, L - L // 2])
        X = 0.05 + 0.1 * ((y[:, None] * 7 + np.arange(F) * 3) % 10) + 0.04 * rs.rand(L, F)
    elif kind == "noisy":                        # deep trees, general trees in the blob
        y = rs.randint(0, K, L) * 11 - 5
        X = rs.rand(L, F) + 0.3 * (y[:, None] % 7) / 7
    elif kind == "ties":                         # few distinct values, constant columns
        y = rs.randint(0, K, L)
        X = np.floor(rs.rand(L, F) * 3) / 3
        X[:, ::4] = 0.5
    elif kind == "impure":                       # duplicate rows with different labels
        y = rs.randint(0, K, L)
        X = np.repeat(rs.rand(L // 4 + 1, F), 4, axis=0)[:L]
    else:
        raise ValueError(kind)
    seeds = rs.randint(0, 2**31 - 1, 100)
    return X.astype(np.float32), y, seeds


@pytest.mark.parametrize("L,F,K,kind", [(100, 27, 2, "separable"), (100, 21, 10, "noisy"), (100, 12, 3, "ties"),
                                        (100, 9, 4, "impure"), (256, 5, 5, "noisy"), (7, 3, 2, "noisy"),
                                        (2, 4, 2, "noisy"), (150, 40, 16, "noisy"), (64, 6, 30, "noisy")])
@pytest.mark.parametrize("fused", [True, False])
def test_device_refit_matches_host(L, F, K, kind, fused):
    """fused: batches of <= 4096 values prepared inside the tree kernel; else k_dfit_prep."""
    rs = np.random.RandomState(L * 1000 + F * 10 + K)
    batches = [_batch(rs, L, F, K, kind) for _ in range(3)]
    host = _host(batches)
    dev = _device(batches, k_cap=64 if K > 16 else 16, fused=fused)
    for h, d in zip(host, dev):
        _same(h, d)


def test_device_refit_single_row():
    rs = np.random.RandomState(5)
    X = rs.rand(1, 4).astype(np.float32)
    batches = [(X, np.array([9]), rs.randint(0, 2**31 - 1, 100))]
    _same(_host(batches)[0], _device(batches)[0])


def test_device_refit_reports_nan_and_class_overflow():
    from ddm_amd._capi import DDM_E_FOREST, DDM_E_NAN
    rs = np.random.RandomState(6)
    X, y, seeds = _batch(rs, 50, 6, 3, "noisy")
    Xn = X.copy()
    Xn[3, 2] = np.nan
    yk = np.arange(50) % 20
    for fused in (True, False):
        out = _device([(Xn, y, seeds), (X, yk, seeds)], k_cap=16, fused=fused)
        assert out[0][3][0] == DDM_E_NAN
        assert out[1][3][0] == DDM_E_FOREST and out[1][3][1] == 20
