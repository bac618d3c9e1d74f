"""The synthetic configs of BASELINE.json on the host: the C1 rialto-shaped
table and its data prep, the C5 jittered-block labels, and the bench's C3 property check."""
import numpy as np
import pytest

from oracle import synth as hsynth


def test_c1_table_shape_and_determinism():
    from ddm_amd.synth import C1_FEATURES, C1_ROWS, rialto_partitions, rialto_table
    t = rialto_table()
    assert t.X32.shape == (C1_FEATURES, C1_ROWS) and t.X32.dtype == np.float32
    assert np.array_equal(np.bincount(t.target), np.full(10, C1_ROWS // 10))
    assert np.allclose(t.X32.sum(axis=0), 1.0, atol=1e-5)          # histograms
    t2 = rialto_table()
    assert np.array_equal(t.X32, t2.X32)
    _, order, parts = rialto_partitions(table=t)
    assert len(parts) == 1 and len(parts[0].target) == 2 * C1_ROWS
    # MULT=2 duplicates every csv row twice, then the stable sort by target (DDM_Process.py:44-51)
    assert np.array_equal(np.bincount(order, minlength=C1_ROWS), np.full(C1_ROWS, 2))
    assert (np.diff(parts[0].target) >= 0).all()
    assert np.array_equal(parts[0].row_number, order)


def test_c1_classes_separable_on_concentrated_bins():
    from ddm_amd.synth import rialto_table
    t = rialto_table(n_rows=2000)
    # class c's concentrated bin (f = c) carries the largest mean mass of its class
    for c in range(10):
        m = t.X32[:, t.target == c].mean(axis=1)
        assert int(np.argmax(m[:10])) == c


@pytest.mark.parametrize("part", [0, 3, 7])
def test_c5_jitter_blocks_are_150_to_300_partition_rows(part):
    y = hsynth.jitter_labels(100_000, part, 8, 1800, 300, 10, 0.0, 20261015)
    edges = np.nonzero(np.diff(y))[0] + 1
    lens = np.diff(edges)
    assert lens.min() >= 150 and lens.max() <= 300
    assert set(np.unique(y)) == set(range(10))
    # consecutive blocks differ by one class (block k has class k % 10)
    assert ((y[edges] - y[edges - 1]) % 10 == 1).all()


def test_c5_label_noise_rate():
    clean = hsynth.jitter_labels(200_000, 1, 8, 1800, 300, 10, 0.0, 5)
    noisy = hsynth.jitter_labels(200_000, 1, 8, 1800, 300, 10, 0.01, 5)
    rate = (clean != noisy).mean()
    assert 0.008 < rate < 0.012


def test_host_mirror_features_separable():
    y = hsynth.block_labels(1000, 2, 8, 1000, 10)
    X = hsynth.features(y, 2, 8, 7)
    assert X.dtype == np.float32 and X.shape == (1000, 27)
    for c in np.unique(y):
        rows = X[y == c]
        assert (rows.max(axis=0) - rows.min(axis=0) < 0.05).all()


def test_c3_property_check_accepts_the_analytic_answer_and_rejects_others():
    import bench
    n, P, block, pb = 50_000, 8, 100_037, 100
    res = {}
    for d in range(P):
        r = np.full(((n + pb - 1) // pb - 1, 2), -1, dtype=np.int64)
        k = 1
        while True:
            f = (k * block - d + P - 1) // P
            if f >= n:
                break
            if f >= pb:
                r[f // pb - 1, 1] = f + (3 if (f + 3) // pb == f // pb else 0)
            k += 1
        res[d] = r
    bench.c3_property_check(res, n, P, block)
    bad = {d: r.copy() for d, r in res.items()}
    bad[2][5, 1] = 600
    with pytest.raises(RuntimeError):
        bench.c3_property_check(bad, n, P, block)
    warn = {d: r.copy() for d, r in res.items()}
    warn[0][7, 0] = 800
    with pytest.raises(RuntimeError):
        bench.c3_property_check(warn, n, P, block)
