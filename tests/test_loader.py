"""Stream preparation, loader and post-loop record against the
reference's pinned stream order (tests/golden, generated from DDM_Process.py:44-51) and
against pandas itself (the reference's parser and sampler)."""
import os

import numpy as np
import pandas as pd
import pytest

from conftest import golden_partitions, load_npz


def _outdoor_csv(tmp_path):
    """outdoorStream as pandas parsed it, written back with round-trip float text."""
    d = load_npz("outdoor.npz")
    X, y = d["X"], d["target"]
    path = tmp_path / "outdoor.csv"
    with open(path, "w") as f:
        f.write(",".join([str(i) for i in range(X.shape[1])] + ["target"]) + "\n")
        for r in range(len(y)):
            f.write(",".join(repr(float(v)) for v in X[r]) + f",{int(y[r])}\n")
    return str(path), X, y


@pytest.mark.parametrize("mult", [1, 2, 4])
def test_order_matches_reference_fixture(mult):
    from ddm_amd import loader
    d = load_npz("outdoor.npz")
    cfg = load_npz(f"outdoor_cfg_m{mult}_i1.npz")
    order = loader.prepare_order(len(d["target"]), d["target"], mult, np.random.RandomState(123), "stable")
    assert np.array_equal(order, cfg["order"].astype(np.int64))


@pytest.mark.parametrize("mult,kind", [(0.5, "quicksort"), (0.37, "stable"), (3, "quicksort"), (1, "stable")])
def test_order_matches_pandas(mult, kind):
    """DDM_Process.py:44-51 run by pandas on a frame with many ties in target."""
    from ddm_amd import loader
    rs = np.random.RandomState(7)
    n = 997
    df = pd.DataFrame({"0": rs.rand(n), "target": rs.randint(0, 5, n)})
    np.random.seed(99)
    if mult < 1:
        want = df.sample(frac=mult)
    else:
        want = pd.concat([df] * int(mult)).sample(frac=1)
    want = want.sort_values(by="target", kind=kind).index.to_numpy()
    np.random.seed(99)
    got = loader.prepare_order(n, df["target"].to_numpy(), mult, None, kind)
    assert np.array_equal(got, want)
    # the global RNG is left where pandas leaves it
    np.random.seed(99)
    loader.prepare_order(n, df["target"].to_numpy(), mult, None, kind)
    a = np.random.rand()
    np.random.seed(99)
    (df.sample(frac=mult) if mult < 1 else pd.concat([df] * int(mult)).sample(frac=1))
    assert a == np.random.rand()


@pytest.mark.parametrize("engine", ["pyarrow", "pandas"])
def test_csv_columns_float32(tmp_path, engine):
    from ddm_amd import loader
    path, X, y = _outdoor_csv(tmp_path)
    t = loader.read_stream_csv(path, engine=engine)
    assert t.X32.dtype == np.float32 and t.X32.shape == (X.shape[1], len(y)) and t.X32.flags.c_contiguous
    assert np.array_equal(t.X32, X.T.astype(np.float32))
    assert np.array_equal(t.target, y)
    assert t.features == [str(i) for i in range(X.shape[1])]


@pytest.mark.skipif(not os.path.exists("/root/reference/outdoorStream.csv"), reason="reference csv not here")
def test_real_csv_float32_equals_pandas_parse():
    """pyarrow's correctly rounded parse, cast to float32, equals pandas' parse cast to
    float32 on the reference's own file (only float32 reaches the hot path)."""
    from ddm_amd import loader
    d = load_npz("outdoor.npz")
    t = loader.read_stream_csv("/root/reference/outdoorStream.csv")
    assert np.array_equal(t.X32, d["X"].T.astype(np.float32))
    assert np.array_equal(t.target, d["target"])


@pytest.mark.parametrize("mult,inst", [(2, 4), (4, 16), (1, 1)])
def test_partitions_match_reference_groups(mult, inst):
    from ddm_amd import loader
    d = load_npz("outdoor.npz")
    cfg = load_npz(f"outdoor_cfg_m{mult}_i{inst}.npz")
    table = loader.StreamTable(np.ascontiguousarray(d["X"].T.astype(np.float32)), d["target"],
                               [str(i) for i in range(d["X"].shape[1])])
    parts = loader.split_partitions(table, cfg["order"].astype(np.int64), inst)
    ref = golden_partitions(mult, inst)
    assert [p.device_id for p in parts] == [r[0] for r in ref if len(r[1])]
    for p, (dev, frame, _) in zip(parts, ref):
        assert np.array_equal(p.row_number, frame["full_df_row_number"].to_numpy())
        assert np.array_equal(p.target, frame["target"].to_numpy())
        assert np.array_equal(p.X32.T, frame[table.features].to_numpy().astype(np.float32))
        f = p.frame(table.features)
        assert list(f.columns) == list(frame.columns)
        assert np.array_equal(f["device_id"].to_numpy(), frame["device_id"].to_numpy())


def test_post_loop_record(tmp_path):
    """DDM_Process.py:250-273 on the reference's own events (outdoor MULT=2, INSTANCES=4)."""
    from ddm_amd import record
    from ddm_amd.params import OUTPUT_COLUMNS
    d = load_npz("outdoor.npz")
    cfg = load_npz("outdoor_cfg_m2_i4.npz")
    ev = pd.concat([pd.DataFrame(cfg[f"events/{k}"], columns=OUTPUT_COLUMNS, index=np.zeros(len(cfg[f"events/{k}"]),
                                                                                               dtype=np.int64))
                    for k in range(4)])
    dist = record.dist_between_changes(8000, d["target"])
    assert dist == 8000 // len(np.unique(d["target"]))
    out = record.change_distances(ev, dist)
    chg = ev["change_flag_global"].to_numpy()
    assert len(out) == (chg != -1).sum()
    assert np.array_equal(out["distance"].to_numpy(), (chg[chg != -1] % dist).astype(np.float64))
    assert out["distance"].dtype == np.float64
    row = record.results_row("outdoorStream.csv-x", "x", "local", 4, 2, "8g", 4, 1.5, out["distance"].mean())
    rd, wr = tmp_path / "ddm_cluster_runs.csv", tmp_path / "sparse_cluster_runs.csv"
    first = record.append_results(row, str(rd), str(wr))
    assert list(first.columns) == record.RESULT_COLUMNS and len(first) == 1
    os.replace(wr, rd)
    second = record.append_results(row, str(rd), str(wr))
    assert len(second) == 2 and second.iloc[0].tolist() == second.iloc[1].tolist()
