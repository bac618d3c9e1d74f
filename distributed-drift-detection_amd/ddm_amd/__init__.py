"""ddm_amd — MI355X-native predict + DDM drift-detection hot path.

Drop-in for the reference's grouped-map partition function `run_DDM_loop`
(rcorizzo/distributed-drift-detection, DDM_Process.py:166-213): HIP kernels for gfx950
(forest predict, DDM scan) behind a C-ABI (include/ddm_amd.h) bound with ctypes;
PyTorch-ROCm provides device buffers, streams and torch.distributed (RCCL).

Importing the package loads libddm_amd.so and fails loudly if it is not built.
"""
from ._capi import DdmError, lib  # noqa: F401  (fails loudly without the HIP library)
from .controller import DevicePartition, PartitionRunner, run_DDM_loop, run_partition_frame  # noqa: F401
from .params import OUTPUT_COLUMNS, SCHEMA, DDMSettings  # noqa: F401
from .rng import MTStream  # noqa: F401

__version__ = "0.1.0"
