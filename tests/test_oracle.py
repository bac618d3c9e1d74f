"""Pin the oracle to the reference: every golden vector produced by executing the
reference's own function bodies (tests/golden/make_golden.py, DDM_Process.py:94-213)."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, golden_configs, golden_partitions, load_npz, oracle_scan_c
from oracle import forest as oforest
from oracle.controller import run_partition, run_partition_frames
from oracle.ddm import OracleDDM, scan_stream


def test_manifest_versions():
    man = json.load(open(os.path.join(GOLDEN, "manifest.json")))
    import sklearn
    assert man["sklearn"] == sklearn.__version__, "fixtures depend on sklearn's RF; regenerate"
    assert set(man["configs"]) == {f"m{m}_i{i}" for m, i in golden_configs()}


def test_ddm_known_answers():
    kat = load_npz("ddm_kat.npz")
    names = sorted({k.split("/")[0] for k in kat.files})
    assert len(names) == 8
    for name in names:
        ddm = OracleDDM()
        for t, x in enumerate(kat[name + "/x"]):
            ddm.add(int(x))
            assert ddm.miss_prob == kat[name + "/p"][t], (name, t)
            assert ddm.miss_std == kat[name + "/s"][t], (name, t)
            assert ddm.in_warning_zone == bool(kat[name + "/warn"][t]), (name, t)
            assert ddm.in_concept_change == bool(kat[name + "/change"][t]), (name, t)


def test_ddm_appendix_a_facts():
    # SURVEY.md Appendix A consequences
    ev, stop, _, _ = scan_stream([0, 0, 0, 0, 1], mode="stop")
    assert stop == 0 and tuple(ev[0]) == (-1, 4)
    ev, _, _, _ = scan_stream([1, 0, 0, 0, 0, 0])
    assert ev[0, 0] == 1
    ev, stop, _, _ = scan_stream([1] * 300)
    assert stop == -1 and (ev == -1).all()


@pytest.mark.parametrize("mult,inst", [(2, 1), (4, 16)])
def test_oracle_scan_matches_reference_trace(mult, inst):
    """The reference's own per-batch error vectors (predict_rf outputs in DDM order) fed
    through the oracle DDM reproduce the reference's per-batch events."""
    tr = load_npz(f"outdoor_trace_m{mult}_i{inst}.npz")
    for d, part, expect in golden_partitions(mult, inst):
        k = 0
        ddm = None
        rows = []
        while f"{d}/pred{k}/err" in tr.files:
            err = tr[f"{d}/pred{k}/err"]
            idx = tr[f"{d}/pred{k}/rows"]
            if ddm is None:
                ddm = OracleDDM()
            ev, stop, ddm, _ = scan_stream(err, per_batch=len(err), ddm=ddm)
            w, c = ev[0]
            glob = part["full_df_row_number"].to_numpy()
            rows.append((idx[w] if w >= 0 else -1, glob[idx[w]] if w >= 0 else -1,
                         idx[c] if c >= 0 else -1, glob[idx[c]] if c >= 0 else -1))
            if stop >= 0:
                ddm = None
            k += 1
        assert np.array_equal(np.array(rows, dtype=np.int64), expect), d


@pytest.mark.parametrize("mult,inst", [(2, 1), (4, 16)])
def test_oracle_forest_matches_sklearn_predictions(mult, inst):
    tr = load_npz(f"outdoor_trace_m{mult}_i{inst}.npz")
    checked = 0
    for d, part, _ in golden_partitions(mult, inst)[:4]:
        X = part[[str(i) for i in range(21)]].to_numpy()
        y = part["target"].to_numpy()
        k = 0
        while f"{d}/pred{k}/rows" in tr.files:
            fit = int(tr[f"{d}/pred{k}/fit_id"])
            if f"{d}/fit{fit}/tree0/left" in tr.files:
                trees = [{key: tr[f"{d}/fit{fit}/tree{t}/{key}"]
                          for key in ("left", "right", "feature", "threshold", "value", "missing_left")}
                         for t in range(100)]
                rows = tr[f"{d}/pred{k}/rows"]
                pred = oforest.predict(trees, tr[f"{d}/fit{fit}/classes"], X[rows])
                assert np.array_equal(pred, tr[f"{d}/pred{k}/y_pred"])
                assert np.array_equal((pred != y[rows]).astype(np.uint8), tr[f"{d}/pred{k}/err"])
                checked += 1
            k += 1
    assert checked >= 5


CPU_CONFIGS = [(1, 1), (1, 4), (1, 16), (2, 1), (2, 4), (2, 8), (4, 16)]


@pytest.mark.parametrize("mult,inst", CPU_CONFIGS)
def test_oracle_controller_matches_reference(mult, inst):
    for d, part, expect in golden_partitions(mult, inst):
        X = part[[str(i) for i in range(21)]].to_numpy()
        np.random.seed(1000 + d)
        got = run_partition(X, part["target"].to_numpy(), part.index.to_numpy(),
                            part["full_df_row_number"].to_numpy())
        assert np.array_equal(got, expect), (mult, inst, d)


def test_oracle_frames_variant_matches_reference():
    """The pandas/iterrows restatement (bench cpu_baseline) gives the same frames."""
    for d, part, expect in golden_partitions(1, 4):
        np.random.seed(1000 + d)
        got = run_partition_frames(part, [str(i) for i in range(21)])
        assert np.array_equal(got.to_numpy(), expect)
        assert list(got.index) == [0] * len(expect)


def test_small_partition_raises_like_reference():
    import pandas as pd
    part = pd.DataFrame({"0": np.arange(100.0), "target": np.zeros(100, int),
                         "full_df_row_number": np.arange(100)})
    with pytest.raises(ValueError, match="No objects to concatenate"):
        run_partition(part[["0"]].to_numpy(), part["target"].to_numpy(), part.index.to_numpy(),
                      part["full_df_row_number"].to_numpy())


def test_c_oracle_equals_python_oracle(oracle_lib):
    rs = np.random.RandomState(3)
    lens = [0, 1, 2, 99, 100, 101, 250, 777, 2000]
    streams = [rs.binomial(1, rs.uniform(0.0, 0.4), n).astype(np.uint8) for n in lens]
    streams.append(np.zeros(500, np.uint8))
    streams.append(np.ones(300, np.uint8))
    err = np.concatenate(streams)
    off = np.concatenate([[0], np.cumsum([len(s) for s in streams])])
    for mode in (0, 1):
        ev, stop, st, ps = oracle_scan_c(oracle_lib, err, off, mode=mode, trace=True)
        base = 0
        for i, s in enumerate(streams):
            pev, pstop, pddm, pps = scan_stream(s, mode="stop" if mode == 0 else "restart", trace=True)
            nb = len(pev)
            assert np.array_equal(ev[base:base + nb], pev), (mode, i)
            assert stop[i] == pstop
            np.testing.assert_array_equal(ps[off[i]:off[i + 1]], pps)
            assert st[i, 0] == pddm.miss_prob and st[i, 5] == pddm.sample_count
            base += nb
