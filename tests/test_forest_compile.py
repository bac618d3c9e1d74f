"""ddm_forest_compile (host C++, csrc/forest_compile.cpp): the compiled blob, evaluated here
by a numpy model of the compiled-forest kernel, must predict exactly what sklearn
predicts (no GPU needed).  The GPU kernel itself is checked in test_gpu_predict.py."""
import numpy as np
import pytest
from sklearn.ensemble import RandomForestClassifier

HEAD = np.dtype([("n_slots", "<i4"), ("n_classes", "<i4"), ("vote_regs", "<i4"), ("n_stumps", "<i4"),
                 ("n_general", "<i4"), ("n_leaves", "<i4"), ("total_bytes", "<i4"), ("any_nanleft", "<i4"),
                 ("stumps_off", "<i4"), ("stump_words", "<i4"), ("n_stumps_right", "<i4"), ("trees_off", "<i4"),
                 ("nodes_off", "<i4"), ("leafcls_off", "<i4"), ("pad0", "<i4"), ("pad1", "<i4"),
                 ("base_votes", "<u4", 4), ("cols", "<i4", 32),
                 ("classes", "<i4", 16), ("slots_off", "<i4"), ("xthr_off", "<i4"), ("rank_tab_off", "<i4"),
                 ("rank_tab_entries", "<i4")])
SLOT = np.dtype([("col", "<i4"), ("n4", "<i4"), ("tab", "<i4"), ("xthr", "<i4"), ("thr", "<f4", 4)])
TREE = np.dtype([("node_begin", "<i4"), ("n_nodes", "<i4"), ("leaf_begin", "<i4"), ("n_leaves", "<i4")])
NODE = np.dtype([("threshold", "<f4"), ("slot_nanleft", "<i4"), ("left_lo", "<u4"), ("left_hi", "<u4")])


def eval_blob(blob, X32, ranks=False):
    """Row-by-row model of k_cforest_predict's row phase: returns predicted labels.
    ranks=True evaluates the stumps through the per-slot rank tables (what the kernel
    does), False through the stump records."""
    h = blob[:HEAD.itemsize].view(HEAD)[0]
    U, K, vr = int(h["n_slots"]), int(h["n_classes"]), int(h["vote_regs"])
    S = int(h["n_stumps"])
    sw = int(h["stump_words"])
    recs = blob[h["stumps_off"]:h["stumps_off"] + 4 * S * sw].view(np.uint32).reshape(S, sw)[:, :2 + vr]
    thr = recs[:, 0].copy().view(np.float32)
    trees = blob[h["trees_off"]:h["trees_off"] + TREE.itemsize * h["n_general"]].view(TREE)
    n_nodes = int(trees["n_nodes"].sum()) if len(trees) else 0
    nodes = blob[h["nodes_off"]:h["nodes_off"] + NODE.itemsize * n_nodes].view(NODE)
    leafcls = blob[h["leafcls_off"]:h["leafcls_off"] + h["n_leaves"]]
    out = np.empty(len(X32), dtype=np.int64)
    with np.errstate(invalid="ignore"):
        for r, row in enumerate(X32):
            x = row[h["cols"][:U]]
            votes = h["base_votes"][:vr].astype(np.uint64)
            if ranks:
                slots = blob[h["slots_off"]:h["slots_off"] + SLOT.itemsize * U].view(SLOT)
                xthr = blob[h["xthr_off"]:h["rank_tab_off"]].view(np.float32)
                rtab = blob[h["rank_tab_off"]:h["rank_tab_off"] + 4 * vr * h["rank_tab_entries"]].view(
                    np.uint32).reshape(-1, vr)
                for sl, rs in enumerate(slots):
                    assert rs["col"] == h["cols"][sl]
                    if rs["n4"] == 0:
                        continue
                    t = np.concatenate([rs["thr"], xthr[4 * rs["xthr"]:4 * (rs["xthr"] + rs["n4"] - 1)]])
                    assert len(t) == 4 * rs["n4"] and np.isinf(t[-1])
                    rank = int((~(x[sl] <= t)).sum())          # NaN: every entry counts
                    votes = (votes + rtab[rs["tab"] + rank]) % (1 << 32)
            else:
                for k in range(S):
                    v = x[recs[k, 1]]
                    right = (not (v <= thr[k])) if k < h["n_stumps_right"] else (v > thr[k])
                    if right:
                        votes = (votes + recs[k, 2:]) % (1 << 32)
            for t in trees:
                m = (1 << 64) - 1
                for nd in nodes[t["node_begin"]:t["node_begin"] + t["n_nodes"]]:
                    v = x[nd["slot_nanleft"] & 0xff]
                    right = (v > nd["threshold"]) if (nd["slot_nanleft"] >> 8) else not (v <= nd["threshold"])
                    if right:
                        m &= ~((int(nd["left_hi"]) << 32) | int(nd["left_lo"]))
                leaf = (m & -m).bit_length() - 1
                c = int(leafcls[t["leaf_begin"] + leaf])
                votes[c >> 2] = (votes[c >> 2] + (1 << (8 * (c & 3)))) % (1 << 32)
            counts = [(int(votes[c >> 2]) >> (8 * (c & 3))) & 0xff for c in range(K)]
            out[r] = h["classes"][int(np.argmax(counts))]
    return out


@pytest.mark.parametrize("n_classes,nan,F", [(1, False, 5), (2, False, 27), (2, True, 21), (5, False, 9),
                                             (10, True, 21), (16, False, 12)])
def test_compiled_blob_predicts_like_sklearn(n_classes, nan, F):
    from ddm_amd.forest import compile_forest, pack_sklearn
    rs = np.random.RandomState(n_classes + 100 * F)
    Xtr = rs.rand(100, F)
    ytr = np.sort(rs.randint(0, n_classes, 100))
    Xtr[:, 0] += ytr
    if nan:
        Xtr[rs.rand(100, F) < 0.05] = np.nan
    rf = RandomForestClassifier(n_estimators=100, random_state=rs).fit(Xtr, ytr)
    blob, head = compile_forest(pack_sklearn(rf))
    assert blob is not None and head["n_classes"] == len(rf.classes_)
    X = rs.rand(400, F)
    X[:, 0] += rs.choice(rf.classes_, 400)
    if nan:
        X[rs.rand(400, F) < 0.05] = np.nan
    X32 = X.astype(np.float32)
    want = rf.predict(X32)
    assert np.array_equal(eval_blob(blob, X32), want)
    assert np.array_equal(eval_blob(blob, X32, ranks=True), want)


def test_compile_rejects_unsupported_forests():
    from ddm_amd.forest import compile_forest, pack_sklearn
    rs = np.random.RandomState(0)
    rf = RandomForestClassifier(n_estimators=10, random_state=0).fit(rs.rand(400, 4), rs.randint(0, 20, 400))
    assert compile_forest(pack_sklearn(rf)) == (None, None)        # 20 classes > 16
    Xd = rs.rand(100, 4)
    Xd[50:] = Xd[0]
    rf = RandomForestClassifier(n_estimators=10, random_state=0).fit(Xd, np.arange(100) % 2)
    assert not pack_sklearn(rf).pure
    assert compile_forest(pack_sklearn(rf)) == (None, None)        # impure leaves


def test_stump_forest_has_no_general_trees():
    """Separable 2-class batches (the C3 regime) compile to stumps and single leaves only."""
    from ddm_amd.forest import compile_forest, pack_sklearn
    rs = np.random.RandomState(3)
    y = np.repeat([0, 1], 50)
    X = 0.05 + 0.1 * ((y[:, None] * 7 + np.arange(27) * 3) % 10) + 0.04 * rs.rand(100, 27)
    rf = RandomForestClassifier(n_estimators=100, random_state=1).fit(X, y)
    blob, head = compile_forest(pack_sklearn(rf))
    assert head["n_general"] == 0 and head["n_stumps"] == 100
    Xt = (0.05 + 0.1 * ((np.array([0, 1])[:, None] * 7 + np.arange(27) * 3) % 10)).astype(np.float32)
    assert np.array_equal(eval_blob(blob, Xt), rf.predict(Xt))
    assert np.array_equal(eval_blob(blob, Xt, ranks=True), rf.predict(Xt))
