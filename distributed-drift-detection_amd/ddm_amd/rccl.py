"""Thin ctypes binding of RCCL (the collective library over xGMI) for the one exchange step
of the hot path: the collect of every partition's drift events (DDM_Process.py:258,
`.toPandas()`), SURVEY.md §5 / §8e.

PyTorch is only the buffer provider here: the communicator is RCCL's own
(ncclCommInitRank), its unique id travels through the torch.distributed rendezvous store,
and ncclAllGather runs on the caller's HIP stream over torch-allocated device buffers.
The library is the librccl.so that PyTorch-ROCm already loaded (torch/lib), so the
process holds one RCCL and one HIP runtime.
"""
import ctypes
import os

import torch

NCCL_UNIQUE_ID_BYTES = 128
NCCL_INT64 = 4          # ncclDataType_t (rccl.h)
_DTYPES = {torch.int64: NCCL_INT64, torch.int32: 2, torch.uint8: 1, torch.float64: 8}


class NcclUniqueId(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * NCCL_UNIQUE_ID_BYTES)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        path = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
        if not os.path.exists(path):
            path = "/opt/rocm/lib/librccl.so"
        L = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
        L.ncclGetUniqueId.argtypes = [ctypes.POINTER(NcclUniqueId)]
        L.ncclCommInitRank.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, NcclUniqueId, ctypes.c_int]
        L.ncclAllGather.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p,
                                    ctypes.c_void_p]
        L.ncclCommDestroy.argtypes = [ctypes.c_void_p]
        L.ncclGetErrorString.argtypes = [ctypes.c_int]
        L.ncclGetErrorString.restype = ctypes.c_char_p
        for f in ("ncclGetUniqueId", "ncclCommInitRank", "ncclAllGather", "ncclCommDestroy"):
            getattr(L, f).restype = ctypes.c_int
        _lib = L
    return _lib


class RcclError(RuntimeError):
    pass


def _check(rc, what):
    if rc != 0:
        raise RcclError(f"{what}: {lib().ncclGetErrorString(rc).decode(errors='replace')} ({rc})")


class RcclComm:
    """One rank's RCCL communicator over `world` ranks (one process per GPU).  `store` is a
    torch.distributed Store shared by the ranks (e.g. the default group's); rank 0 puts
    the unique id there under `key`."""

    def __init__(self, rank, world, device, store, key="ddm_amd_rccl_id"):
        self.rank, self.world, self.device = int(rank), int(world), device
        uid = NcclUniqueId()
        if self.rank == 0:
            _check(lib().ncclGetUniqueId(ctypes.byref(uid)), "ncclGetUniqueId")
            store.set(key, bytes(uid.internal))
        else:
            raw = store.get(key)
            ctypes.memmove(ctypes.byref(uid), raw, NCCL_UNIQUE_ID_BYTES)
        self.comm = ctypes.c_void_p()
        with torch.cuda.device(device):
            _check(lib().ncclCommInitRank(ctypes.byref(self.comm), self.world, uid, self.rank), "ncclCommInitRank")

    def all_gather(self, send, recv, stream=None):
        """recv[world * n] <- every rank's send[n] (device tensors, same dtype), on `stream`."""
        if send.dtype not in _DTYPES or recv.dtype != send.dtype or recv.numel() < self.world * send.numel():
            raise ValueError("all_gather: bad buffers")
        s = stream or torch.cuda.current_stream(self.device)
        _check(lib().ncclAllGather(send.data_ptr(), recv.data_ptr(), send.numel(), _DTYPES[send.dtype], self.comm,
                                   ctypes.c_void_p(s.cuda_stream)), "ncclAllGather")

    def close(self):
        if self.comm.value:
            lib().ncclCommDestroy(self.comm)
            self.comm = ctypes.c_void_p()

    @classmethod
    def from_default_group(cls, device):
        """The communicator of torch.distributed's default group's ranks (its store carries the id)."""
        import torch.distributed as dist
        from torch.distributed import distributed_c10d as c10d
        store = c10d._get_default_store()
        return cls(dist.get_rank(), dist.get_world_size(), device, store)
