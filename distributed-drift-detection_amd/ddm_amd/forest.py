"""Device-resident forests for ddm_forest_predict (layout: treepack.py).

A pure forest is also compiled (ddm_forest_compile, csrc/forest_compile.cpp) into the
blob the fast predict kernels read; forests the compiler rejects (impure, > 64 leaves
in a tree, > 16 classes, > 32 feature columns) are predicted by the node-walk kernels.
"""
import ctypes

import numpy as np
import torch

from ._capi import DDM_E_FOREST, DdmForest, check, lib
from .treepack import MAX_CLASSES, MISSING_LEFT_BIT, NODE_DTYPE, PackedForest, pack, pack_sklearn, tree_arrays  # noqa: F401

# ddm_cforest_head (include/ddm_amd.h): the leading int32 fields
_HEAD_FIELDS = ("n_slots", "n_classes", "vote_regs", "n_stumps", "n_general", "n_leaves", "total_bytes",
                "any_nanleft")
_RANK_TAB_ENTRIES = 71          # int32 index of ddm_cforest_head.rank_tab_entries


def compile_forest(packed):
    """The compiled blob (uint8 numpy) and its header fields, or (None, None) when the
    forest is not compilable."""
    if not packed.pure:
        return None, None
    nodes = np.ascontiguousarray(packed.nodes)
    roots = np.ascontiguousarray(packed.roots, dtype=np.int32)
    classes = np.ascontiguousarray(packed.classes, dtype=np.int32)
    size = ctypes.c_int64()
    args = (nodes.ctypes.data, len(nodes), roots.ctypes.data, len(roots), classes.ctypes.data, len(classes), 1)
    rc = lib.ddm_forest_compile(*args, None, 0, ctypes.byref(size))
    if rc == DDM_E_FOREST:
        return None, None
    check(rc, "ddm_forest_compile")
    blob = np.zeros(size.value, dtype=np.uint8)
    check(lib.ddm_forest_compile(*args, blob.ctypes.data, blob.size, ctypes.byref(size)), "ddm_forest_compile")
    head = dict(zip(_HEAD_FIELDS, blob[:4 * len(_HEAD_FIELDS)].view(np.int32).tolist()))
    head["tab_words"] = int(blob[:4 * (_RANK_TAB_ENTRIES + 1)].view(np.int32)[_RANK_TAB_ENTRIES]) * head["vote_regs"]
    return blob, head


class DeviceForest:
    """A PackedForest resident in HBM plus the ddm_forest descriptor pointing at it.
    compiled=False keeps the node-walk kernels (tests compare both paths)."""

    def __init__(self, packed, device, compiled=True):
        self.packed = packed
        self.nodes = torch.from_numpy(packed.nodes.view('u1')).to(device, non_blocking=False)
        self.roots = torch.from_numpy(packed.roots).to(device)
        self.classes = torch.from_numpy(packed.classes).to(device)
        self.leaf_value = None if packed.pure else torch.from_numpy(packed.leaf_value).to(device)
        blob, head = compile_forest(packed) if compiled else (None, None)
        self.cforest = None if blob is None else torch.from_numpy(blob).to(device)
        self.head = head
        self.desc = DdmForest(self.nodes.data_ptr(), self.roots.data_ptr(),
                              0 if packed.pure else self.leaf_value.data_ptr(), self.classes.data_ptr(),
                              packed.n_trees, packed.n_classes, packed.n_nodes, 1 if packed.pure else 0,
                              0 if blob is None else self.cforest.data_ptr(),
                              head["n_slots"] if head else 0, head["vote_regs"] if head else 0,
                              head["n_leaves"] if head else 0, head["tab_words"] if head else 0)

    @classmethod
    def from_buffer(cls, packed, blob, head, dev, off, host_keepalive=None):
        """A forest whose arrays live in a shared device buffer at byte offsets `off`."""
        f = cls.__new__(cls)
        f.packed, f.head, f._buf, f._host = packed, head, dev, host_keepalive
        base = dev.data_ptr()
        f.nodes = f.roots = f.classes = f.leaf_value = None
        f.cforest = None if blob is None else dev[off["blob"]:off["blob"] + blob.size]
        f.desc = DdmForest(base + off["nodes"], base + off["roots"], 0 if packed.pure else base + off["leaf"],
                           base + off["classes"], packed.n_trees, packed.n_classes, packed.n_nodes,
                           1 if packed.pure else 0, 0 if blob is None else base + off["blob"],
                           head["n_slots"] if head else 0, head["vote_regs"] if head else 0,
                           head["n_leaves"] if head else 0, head["tab_words"] if head else 0)
        return f

    @property
    def compiled(self):
        return self.cforest is not None

    @property
    def features_read(self):
        """Feature columns one row loads: the compiled forest's slots, or every column a
        node of the walk reads."""
        return self.head["n_slots"] if self.head else self.packed.features_used


def upload_forests(entries, device, stream):
    """entries: [(PackedForest, blob or None, head or None)] -> [DeviceForest], all copied
    to HBM with ONE host->device transfer (a pinned staging buffer, 256-byte aligned
    pieces); the device buffer is shared by the returned forests."""
    pieces, layout = [], []
    off = 0

    def put(arr):
        nonlocal off
        b = np.ascontiguousarray(arr).view(np.uint8).reshape(-1)
        at = off
        pieces.append((at, b))
        off = (off + b.size + 255) & ~255
        return at

    for pf, blob, head in entries:
        o = {"nodes": put(pf.nodes), "roots": put(pf.roots), "classes": put(pf.classes)}
        o["leaf"] = None if pf.pure else put(pf.leaf_value)
        o["blob"] = None if blob is None else put(blob)
        layout.append(o)
    host = torch.empty(max(off, 256), dtype=torch.uint8, pin_memory=True)
    hn = host.numpy()
    for at, b in pieces:
        hn[at:at + b.size] = b
    with torch.cuda.stream(stream):
        dev = host.to(device, non_blocking=True)
    # keep the staging buffer alive until the copy has run (the caller's stream orders it)
    out = []
    for (pf, blob, head), o in zip(entries, layout):
        out.append(DeviceForest.from_buffer(pf, blob, head, dev, o, host))
    return out
