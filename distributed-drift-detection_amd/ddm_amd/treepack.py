"""Forest export (numpy only, importable without torch/HIP): a fitted RandomForestClassifier (train_rf, DDM_Process.py:98-105)
into the 16-byte node layout `ddm_forest_predict` walks (include/ddm_amd.h).

Layout in HBM (one forest per partition model):
  nodes  ddm_node[n_nodes]   {f64 threshold, i32 feature, i32 child}; the two children
                             of a node are adjacent (BFS renumbering), so a node is
                             one 16-byte load and a step is `child + (x > thr)`
  roots  i32[n_trees]
  leaf_value f64[n_leaf_rows, n_classes]  only for impure forests
  classes i32[n_classes]     `classes_` (DDM_Process.py:114's labels)
A forest is "pure" when every leaf row of `tree_.value` is one-hot, which fully grown
trees (max_depth=None, min_samples_leaf=1) give unless identical feature rows carry
different labels; then the leaf stores its class index and the kernel counts votes.
"""
import numpy as np

NODE_DTYPE = np.dtype([("threshold", "<f8"), ("feature", "<i4"), ("child", "<i4")])
MISSING_LEFT_BIT = 1 << 30
MAX_CLASSES = 256          # ddm_forest_predict's limit (a batch of <= 256 rows holds at most 256)
FIT_MAX_CLASSES = 64       # the native and device trainers' limit: more -> sklearn refit


def tree_arrays(rf):
    """Raw per-tree arrays of a fitted sklearn forest."""
    out = []
    for est in rf.estimators_:
        t = est.tree_
        out.append(dict(left=t.children_left, right=t.children_right, feature=t.feature,
                        threshold=t.threshold, value=t.value[:, 0, :],
                        missing_left=np.asarray(t.missing_go_to_left)))
    return out


class PackedForest:
    __slots__ = ("nodes", "roots", "leaf_value", "classes", "n_classes", "pure", "features_used")

    def __init__(self, nodes, roots, leaf_value, classes, pure):
        self.nodes, self.roots, self.leaf_value = nodes, roots, leaf_value
        self.classes, self.pure = classes, pure
        self.n_classes = len(classes)
        f = nodes["feature"]
        # distinct feature columns any node reads: the predict kernel's HBM bytes per row
        self.features_used = int(np.unique(f[f >= 0] & (MISSING_LEFT_BIT - 1)).size)

    @property
    def n_trees(self):
        return len(self.roots)

    @property
    def n_nodes(self):
        return len(self.nodes)


def pack(trees, classes):
    """BFS-renumber every tree so siblings are adjacent; detect purity."""
    classes = np.asarray(classes)
    if classes.size > MAX_CLASSES:
        raise ValueError(f"{classes.size} classes > {MAX_CLASSES} supported by ddm_forest_predict")
    if classes.min() < np.iinfo(np.int32).min or classes.max() > np.iinfo(np.int32).max:
        raise ValueError("class labels must fit int32")
    k = classes.size
    pure = len(trees) <= 255
    for t in trees:
        v = t["value"][t["left"] == -1]
        if not (np.all((v == 0.0) | (v == 1.0)) and np.all((v == 1.0).sum(axis=1) == 1)):
            pure = False
            break
    total = sum(len(t["left"]) for t in trees)
    nodes = np.zeros(total, dtype=NODE_DTYPE)
    roots = np.empty(len(trees), dtype=np.int32)
    leaf_rows = []
    base = 0
    for ti, t in enumerate(trees):
        left, right, feat, thr = t["left"], t["right"], t["feature"], t["threshold"]
        miss = t.get("missing_left")
        value = t["value"]
        n = len(left)
        new_id = np.empty(n, dtype=np.int64)
        new_id[0] = 0
        order = [0]
        nxt = 1
        qi = 0
        while qi < len(order):
            u = order[qi]
            qi += 1
            if left[u] != -1:
                new_id[left[u]], new_id[right[u]] = nxt, nxt + 1
                order.append(int(left[u]))
                order.append(int(right[u]))
                nxt += 2
        if nxt != n:
            raise ValueError("tree is not a full binary tree")
        roots[ti] = base
        internal = left != -1
        ids = base + new_id
        nodes["threshold"][ids] = np.where(internal, thr, 0.0)
        f = np.where(internal, feat, -1).astype(np.int64)
        if miss is not None:
            f = np.where(internal & (np.asarray(miss) != 0), f | MISSING_LEFT_BIT, f)
        nodes["feature"][ids] = f.astype(np.int32)
        child = np.where(internal, base + new_id[np.where(internal, left, 0)], 0)
        if pure:
            leaf_child = np.argmax(value, axis=1)
        else:
            leaf_idx = np.nonzero(~internal)[0]
            leaf_child = np.zeros(n, dtype=np.int64)
            leaf_child[leaf_idx] = len(leaf_rows) + np.arange(len(leaf_idx))
            leaf_rows.extend(value[leaf_idx])
        nodes["child"][ids] = np.where(internal, child, leaf_child).astype(np.int32)
        base += n
    leaf_value = None if pure else np.ascontiguousarray(np.array(leaf_rows, dtype=np.float64).reshape(-1, k))
    return PackedForest(nodes, roots, leaf_value, classes.astype(np.int32), pure)


def pack_sklearn(rf):
    return pack(tree_arrays(rf), rf.classes_)
