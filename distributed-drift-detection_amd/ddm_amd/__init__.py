"""ddm_amd — MI355X-native predict + DDM drift-detection hot path.

Drop-in for the reference's grouped-map partition function `run_DDM_loop`
(rcorizzo/distributed-drift-detection, DDM_Process.py:166-213): HIP kernels for gfx950
(forest predict, DDM scan) behind a C-ABI (include/ddm_amd.h) bound with ctypes;
PyTorch-ROCm provides device buffers, streams and torch.distributed (RCCL).

The package namespace is lazy: `ddm_amd.treepack` stays importable without torch; everything else loads libddm_amd.so through
`ddm_amd._capi`, which raises if the library is not built (there is no CPU fallback).
"""
import importlib

__version__ = "0.1.0"

_EXPORTS = {
    "run_DDM_loop": "controller", "run_partition_frame": "controller", "DevicePartition": "controller",
    "PartitionRunner": "controller", "DDMSettings": "params", "OUTPUT_COLUMNS": "params", "SCHEMA": "params",
    "MTStream": "rng", "DdmError": "_capi", "lib": "_capi",
}


def __getattr__(name):
    if name in _EXPORTS:
        return getattr(importlib.import_module(f".{_EXPORTS[name]}", __name__), name)
    raise AttributeError(name)
