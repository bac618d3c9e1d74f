"""ddm_forest_predict (HIP) vs scikit-learn / the reference's own predictions: predicted
labels and error bytes must be identical."""
import numpy as np
import pytest
import torch
from sklearn.ensemble import RandomForestClassifier

from conftest import golden_partitions, load_npz

pytestmark = pytest.mark.gpu


def gpu_predict(packed, X32, y, perm, per_batch=100, pos=None, compiled=True, want_compiled=None):
    """X32 [n, F] rows in partition order; perm uint8 per DDM position.  compiled: use the
    compiled-forest kernels when the forest compiles (else the node walk)."""
    from ddm_amd import kernels
    from ddm_amd.forest import DeviceForest
    dev = torch.device("cuda", 0)
    n, F = X32.shape
    ld = ((n + 63) // 64) * 64
    Xd = torch.zeros((F, ld), dtype=torch.float32, device=dev)
    Xd[:, :n] = torch.from_numpy(np.ascontiguousarray(X32.T))
    yd = torch.zeros(ld, dtype=torch.int32, device=dev)
    yd[:n] = torch.from_numpy(np.asarray(y, np.int32))
    pd_ = torch.from_numpy(np.asarray(perm, np.uint8)).to(dev)
    err = torch.full((n + 16,), 7, dtype=torch.uint8, device=dev)
    pred = torch.full((n,), -99, dtype=torch.int32, device=dev)
    first = torch.zeros(1, dtype=torch.int64, device=dev)
    f = DeviceForest(packed, dev, compiled=compiled)
    if want_compiled is not None:
        assert f.compiled == want_compiled
    p0, p1 = pos if pos else (0, n)
    kernels.forest_predict(Xd, yd, pd_, p0, p1, per_batch, f, err, first_err=first, pred=pred)
    torch.cuda.synchronize()
    return err.cpu().numpy()[:n], pred.cpu().numpy(), int(first.cpu().numpy().view(np.uint64)[0])


def ddm_order_rows(n, perm, per_batch=100):
    g = np.arange(n)
    return (g // per_batch) * per_batch + perm.astype(np.int64)


def batch_perms(rs, n, per_batch=100):
    return np.concatenate([rs.permutation(min(per_batch, n - s)) for s in range(0, n, per_batch)]).astype(np.uint8)


@pytest.mark.parametrize("compiled", [True, False])
@pytest.mark.parametrize("n_classes,dup,nan", [(2, False, False), (5, False, True), (16, False, False),
                                              (40, False, False), (64, False, False), (3, True, False),
                                              (12, True, True), (33, True, False)])
def test_predict_matches_sklearn(n_classes, dup, nan, compiled):
    from ddm_amd.forest import pack_sklearn
    rs = np.random.RandomState(n_classes * 7 + dup)
    Xtr = rs.rand(300, 9)
    ytr = np.arange(300) % n_classes * 5 - 3
    if dup:
        Xtr[20:40] = Xtr[0]
    if nan:
        Xtr[rs.rand(300, 9) < 0.05] = np.nan
    rf = RandomForestClassifier(n_estimators=100, random_state=rs).fit(Xtr, ytr)
    pf = pack_sklearn(rf)
    assert pf.pure == (not dup)
    n = 5003
    X = rs.rand(n, 9)
    if nan:
        X[rs.rand(n, 9) < 0.05] = np.nan
    y = rs.choice(rf.classes_, n)
    perm = batch_perms(rs, n)
    rows = ddm_order_rows(n, perm)
    X32 = X.astype(np.float32)
    err, pred, first = gpu_predict(pf, X32, y, perm, compiled=compiled)
    want = rf.predict(X32[rows])
    assert np.array_equal(pred, want)
    assert np.array_equal(err, (want != y[rows]).astype(np.uint8))
    nz = np.nonzero(err)[0]
    assert first == (nz[0] if len(nz) else np.iinfo(np.uint64).max)


def test_predict_large_forest_global_path():
    """A forest whose nodes exceed the 64 KiB LDS budget walks nodes from global memory."""
    from ddm_amd.forest import pack_sklearn
    rs = np.random.RandomState(1)
    Xtr = rs.rand(3000, 6)
    ytr = rs.randint(0, 4, 3000)
    rf = RandomForestClassifier(n_estimators=60, random_state=0).fit(Xtr, ytr)
    pf = pack_sklearn(rf)
    assert pf.n_nodes * 16 > 64 * 1024
    n = 4000
    X32 = rs.rand(n, 6).astype(np.float32)
    y = rs.randint(0, 4, n)
    perm = batch_perms(rs, n)
    err, pred, _ = gpu_predict(pf, X32, y, perm)
    assert np.array_equal(pred, rf.predict(X32[ddm_order_rows(n, perm)]))


def test_predict_window_and_first_error():
    from ddm_amd.forest import pack_sklearn
    rs = np.random.RandomState(2)
    Xtr = rs.rand(100, 4)
    ytr = (Xtr[:, 0] > 0.5).astype(int)
    rf = RandomForestClassifier(random_state=0).fit(Xtr, ytr)
    n = 10_000
    X32 = rs.rand(n, 4).astype(np.float32)
    y = (X32[:, 0] > 0.5).astype(int)
    y[7777] = 1 - y[7777]
    perm = batch_perms(rs, n)
    err, _, first = gpu_predict(pack_sklearn(rf), X32, y, perm, pos=(7000, 9000))
    rows = ddm_order_rows(n, perm)
    want = (rf.predict(X32[rows[7000:9000]]) != y[rows[7000:9000]]).astype(np.uint8)
    assert np.array_equal(err[7000:9000], want)
    assert (err[:7000] == 7).all() and (err[9000:] == 7).all()
    nz = np.nonzero(want)[0]
    assert first == 7000 + nz[0]


@pytest.mark.parametrize("mult,inst", [(2, 1), (4, 16)])
def test_predict_reference_trace(mult, inst):
    """Exported forests of the reference's own refits reproduce its y_pred / error vectors."""
    from ddm_amd.forest import pack
    tr = load_npz(f"outdoor_trace_m{mult}_i{inst}.npz")
    checked = 0
    for d, part, _ in golden_partitions(mult, inst)[:4]:
        X32 = part[[str(i) for i in range(21)]].to_numpy().astype(np.float32)
        y = part["target"].to_numpy()
        n = len(part)
        k = 0
        while f"{d}/pred{k}/rows" in tr.files:
            fit = int(tr[f"{d}/pred{k}/fit_id"])
            if f"{d}/fit{fit}/tree0/left" in tr.files:
                trees = [{key: tr[f"{d}/fit{fit}/tree{t}/{key}"]
                          for key in ("left", "right", "feature", "threshold", "value", "missing_left")}
                         for t in range(100)]
                pf = pack(trees, tr[f"{d}/fit{fit}/classes"])
                rows = tr[f"{d}/pred{k}/rows"]
                b = rows[0] // 100
                perm = np.zeros(n, np.uint8)
                perm[b * 100:b * 100 + len(rows)] = rows - b * 100
                err, pred, _ = gpu_predict(pf, X32, y, perm, pos=(b * 100, b * 100 + len(rows)))
                assert np.array_equal(pred[b * 100:b * 100 + len(rows)], tr[f"{d}/pred{k}/y_pred"])
                assert np.array_equal(err[b * 100:b * 100 + len(rows)], tr[f"{d}/pred{k}/err"])
                checked += 1
            k += 1
    assert checked >= 5


@pytest.mark.parametrize("n_classes,nan,F,per_batch", [(1, False, 27, 100), (2, False, 27, 100), (2, True, 21, 100),
                                                       (4, False, 9, 100), (5, True, 21, 100), (8, False, 32, 100),
                                                       (10, False, 27, 64), (16, True, 12, 256), (3, False, 5, 7)])
def test_compiled_forest_batch_fits(n_classes, nan, F, per_batch):
    """Forests fit like the reference's (100-row batches, DDM_Process.py:98-105) compile
    (stumps, single leaves and QuickScorer trees) and predict exactly as sklearn."""
    from ddm_amd.forest import pack_sklearn
    rs = np.random.RandomState(n_classes * 31 + F)
    Xtr = rs.rand(100, F)
    ytr = np.sort(rs.randint(0, n_classes, 100)) * 3 + 1
    Xtr[:, 0] += ytr                                 # one separable feature -> many stumps
    if nan:
        Xtr[rs.rand(100, F) < 0.05] = np.nan
    rf = RandomForestClassifier(n_estimators=100, random_state=rs).fit(Xtr, ytr)
    pf = pack_sklearn(rf)
    n = 6007
    X = rs.rand(n, F)
    yy = rs.choice(rf.classes_, n)
    X[:, 0] += yy + rs.randint(-1, 2, n) * 3
    if nan:
        X[rs.rand(n, F) < 0.05] = np.nan
    perm = batch_perms(rs, n, per_batch)
    rows = ddm_order_rows(n, perm, per_batch)
    X32 = X.astype(np.float32)
    err, pred, first = gpu_predict(pf, X32, yy, perm, per_batch=per_batch, want_compiled=True)
    want = rf.predict(X32[rows])
    assert np.array_equal(pred, want)
    assert np.array_equal(err, (want != yy[rows]).astype(np.uint8))
    nz = np.nonzero(err)[0]
    assert first == (nz[0] if len(nz) else np.iinfo(np.uint64).max)


def test_compiled_thresholds_at_float32_ties():
    """x exactly at, just below and just above the float64 thresholds: the float32 image
    of every threshold must make the same decision as (double)x <= t."""
    from ddm_amd.forest import pack_sklearn
    rs = np.random.RandomState(9)
    Xtr = rs.rand(100, 3).astype(np.float32).astype(np.float64)
    ytr = (Xtr[:, 0] > 0.5).astype(int)
    rf = RandomForestClassifier(n_estimators=50, random_state=3).fit(Xtr, ytr)
    pf = pack_sklearn(rf)
    thr = pf.nodes["threshold"][pf.nodes["feature"] >= 0]
    t32 = thr.astype(np.float32)
    cand = np.concatenate([t32, np.nextafter(t32, np.float32(-1)), np.nextafter(t32, np.float32(2)),
                           Xtr[:, 0].astype(np.float32)])
    n = (len(cand) // 100 + 1) * 100
    X32 = rs.rand(n, 3).astype(np.float32)
    for f in range(3):
        X32[:len(cand), f] = cand
    y = rs.randint(0, 2, n)
    perm = batch_perms(rs, n)
    err, pred, _ = gpu_predict(pf, X32, y, perm, want_compiled=True)
    assert np.array_equal(pred, rf.predict(X32[ddm_order_rows(n, perm)]))


def test_compiled_unaligned_window_uses_walk():
    """A window that does not start on a batch boundary is served by the node walk."""
    from ddm_amd.forest import pack_sklearn
    rs = np.random.RandomState(4)
    Xtr = rs.rand(100, 4)
    ytr = (Xtr[:, 1] > 0.3).astype(int)
    rf = RandomForestClassifier(random_state=0).fit(Xtr, ytr)
    n = 3000
    X32 = rs.rand(n, 4).astype(np.float32)
    y = (X32[:, 1] > 0.3).astype(int)
    perm = batch_perms(rs, n)
    err, pred, _ = gpu_predict(pack_sklearn(rf), X32, y, perm, pos=(1234, 2900), want_compiled=True)
    rows = ddm_order_rows(n, perm)
    assert np.array_equal(pred[1234:2900], rf.predict(X32[rows[1234:2900]]))
