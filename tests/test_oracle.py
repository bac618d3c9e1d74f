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
    # the small grid (make_golden.py) and the published cell (make_golden_cell.py)
    assert set(man["configs"]) == {f"m{m}_i{i}" for m, i in golden_configs()} | {"m512_i16"}


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


@pytest.mark.parametrize("mult,inst", [(2, 1), (4, 4), (1, 16)])
def test_chunked_oracle_matches_reference(mult, inst):
    """run_partition_chunked (many batches per predict, RNG rolled back after a change) ==
    the reference-executed fixtures, and leaves the global RNG where run_partition does."""
    from oracle.controller import run_partition_chunked
    for d, part, expect in golden_partitions(mult, inst):
        X = part[[str(i) for i in range(21)]].to_numpy()
        args = (X, part["target"].to_numpy(), part.index.to_numpy(), part["full_df_row_number"].to_numpy())
        np.random.seed(1000 + d)
        got = run_partition_chunked(*args)
        after = np.random.get_state()
        assert np.array_equal(got, expect), (mult, inst, d)
        np.random.seed(1000 + d)
        run_partition(*args)
        ref = np.random.get_state()
        assert np.array_equal(after[1], ref[1]) and after[2] == ref[2]


def test_chunked_oracle_long_concepts_with_noise():
    """Long concepts (the chunk doubles to its cap) with sparse label noise (changes
    anywhere in a chunk, including its last batch): == run_partition, RNG position too."""
    from oracle.controller import run_partition_chunked
    from oracle import synth
    n = 60_000
    y = synth.block_labels(n, 0, 8, 80_037, 10)
    rs = np.random.RandomState(11)
    flip = rs.rand(n) < 0.0007
    y = np.where(flip, (y + 3) % 10, y)
    X = synth.features(y, 0, 8, 5, 6).astype(np.float64)
    lab, glob = np.arange(n), np.arange(n) * 8
    np.random.seed(31)
    want = run_partition(X, y, lab, glob)
    st = np.random.get_state()
    np.random.seed(31)
    got = run_partition_chunked(X, y, lab, glob, max_chunk=64)
    st2 = np.random.get_state()
    assert np.array_equal(got, want)
    assert (want[:, 2] >= 0).sum() >= 8
    assert np.array_equal(st[1], st2[1]) and st[2] == st2[2]


def test_mt_replay_matches_numpy():
    """oracle/mt_replay.c: permutations and the generator state after a partition's
    draws (one permutation per batch, 100 randint(2**31-1) per refit) == numpy's."""
    from oracle.replay import mt_replay
    rs = np.random.RandomState(4)
    for n_rows, per_batch in ((1234, 100), (5000, 100), (777, 37), (256 * 9, 256)):
        nb = (n_rows + per_batch - 1) // per_batch
        changes = sorted(set(rs.randint(1, nb, size=nb // 3).tolist()))
        want = sorted(set([0, nb - 1] + rs.randint(0, nb, size=5).tolist()))
        perms, key, pos = mt_replay(2024 + n_rows, n_rows, changes, want, per_batch=per_batch)
        g = np.random.RandomState(2024 + n_rows)
        retrain = True
        for b in range(nb):
            p = g.permutation(min(per_batch, n_rows - b * per_batch))
            if b in perms:
                assert np.array_equal(perms[b], p), (n_rows, b)
            if b == 0:
                continue
            if retrain:
                g.randint(2 ** 31 - 1, size=100)
                retrain = False
            if b in changes:
                retrain = True
        st = g.get_state()
        assert np.array_equal(key, st[1]) and pos == st[2]


def test_mt_replay_matches_oracle_controller_rng():
    """Fed the changes the oracle controller found, the replay ends at the controller's RNG
    position (sklearn's own draws included)."""
    from oracle.replay import mt_replay
    for d, part, expect in golden_partitions(2, 4):
        X = part[[str(i) for i in range(21)]].to_numpy()
        np.random.seed(1000 + d)
        run_partition(X, part["target"].to_numpy(), part.index.to_numpy(), part["full_df_row_number"].to_numpy())
        st = np.random.get_state()
        changes = [k + 1 for k in np.nonzero(expect[:, 2] >= 0)[0]]
        _, key, pos = mt_replay(1000 + d, len(part), changes)
        assert np.array_equal(key, st[1]) and pos == st[2], d


def test_oracle_controller_matches_published_cell_partition():
    """The published cell (outdoorStream x512, 16 instances; tests/golden/make_golden_cell.py,
    the reference's own run_DDM_loop on every partition): the stream order the product's
    loader builds has the fixture's sha1, and the oracle controller reproduces partition 0's
    1,279 batch records (the GPU side compares all 16 through bench.py, test_gpu_scaling)."""
    import hashlib
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(GOLDEN), "..", "distributed-drift-detection_amd"))
    from ddm_amd import loader
    data = load_npz("outdoor.npz")
    cfg = load_npz("outdoor_cfg_m512_i16.npz")
    X, target = data["X"], data["target"].astype(np.int64)
    order = loader.prepare_order(len(target), target, 512, np.random.RandomState(123), "stable")
    assert hashlib.sha1(np.ascontiguousarray(order.astype(np.int32)).tobytes()).hexdigest() == str(cfg["order_sha1"])
    sel = order[order % 16 == 0]
    np.random.seed(1000)
    got = run_partition(X[sel], target[sel], np.arange(len(sel)), sel)
    assert np.array_equal(got, cfg["events/0"])
