"""Device-resident forests for ddm_forest_predict (layout: treepack.py)."""
import torch

from ._capi import DdmForest
from .treepack import MAX_CLASSES, MISSING_LEFT_BIT, NODE_DTYPE, PackedForest, pack, pack_sklearn, tree_arrays  # noqa: F401


class DeviceForest:
    """A PackedForest resident in HBM plus the ddm_forest descriptor pointing at it."""

    def __init__(self, packed, device):
        self.packed = packed
        self.nodes = torch.from_numpy(packed.nodes.view('u1')).to(device, non_blocking=False)
        self.roots = torch.from_numpy(packed.roots).to(device)
        self.classes = torch.from_numpy(packed.classes).to(device)
        self.leaf_value = None if packed.pure else torch.from_numpy(packed.leaf_value).to(device)
        self.desc = DdmForest(self.nodes.data_ptr(), self.roots.data_ptr(),
                              0 if packed.pure else self.leaf_value.data_ptr(), self.classes.data_ptr(),
                              packed.n_trees, packed.n_classes, packed.n_nodes, 1 if packed.pure else 0)
