"""Oracle forest predict (test infrastructure only — see oracle/__init__.py).

Restates what `predict_rf` (DDM_Process.py:110-128) gets from scikit-learn 1.7.2:
  * X cast to float32 (`_validate_X_predict`), node test `(double)x <= threshold`,
    NaN routed by `missing_go_to_left` (sklearn tree/_tree.pyx `_apply_dense`);
  * per tree the leaf's class-fraction row `tree_.value[leaf, 0, :]`;
  * forest: `all_proba += proba_t` in tree order, `/= n_trees`, `argmax` first max,
    `classes_.take(...)` (sklearn ensemble/_forest.py:903-962);
  * `acc = y_pred != y` (DDM_Process.py:117).
Input: the raw per-tree arrays written by tests/golden/make_golden.py.
"""
import numpy as np


def apply_tree(tree, X32):
    left, right, feat, thr = tree["left"], tree["right"], tree["feature"], tree["threshold"]
    miss = tree.get("missing_left")
    node = np.zeros(len(X32), dtype=np.int64)
    rows = np.arange(len(X32))
    while True:
        active = left[node] != -1
        if not active.any():
            return node
        a = rows[active]
        nd = node[a]
        xv = X32[a, feat[nd]].astype(np.float64)
        go_left = xv <= thr[nd]
        if miss is not None:
            nan = np.isnan(xv)
            go_left = np.where(nan, miss[nd].astype(bool), go_left)
        node[a] = np.where(go_left, left[nd], right[nd])


def predict_proba(trees, X32):
    k = trees[0]["value"].shape[1]
    acc = np.zeros((len(X32), k), dtype=np.float64)
    for tree in trees:
        acc += tree["value"][apply_tree(tree, X32)]
    acc /= len(trees)
    return acc


def predict(trees, classes, X):
    X32 = np.asarray(X, dtype=np.float64).astype(np.float32)
    return np.asarray(classes).take(np.argmax(predict_proba(trees, X32), axis=1))


def errors(trees, classes, X, y):
    return (predict(trees, classes, X) != np.asarray(y)).astype(np.uint8)
