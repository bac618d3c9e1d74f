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

    _serial = 0

    def __init__(self, rank, world, device, store, key=None, agree=None):
        """agree(ok: bool) -> bool: a collective AND over the ranks (None: no agreement
        step).  With it every rank learns whether all ranks got the unique id before any
        of them enters ncclCommInitRank (which blocks until all ranks join), and whether
        all of them initialised, so that the ranks fall back together."""
        self.rank, self.world, self.device = int(rank), int(world), device
        if key is None:             # one key per communicator: a second one never reads a stale id
            RcclComm._serial += 1
            key = f"ddm_amd_rccl_id/{RcclComm._serial}"
        self.comm = ctypes.c_void_p()
        uid = NcclUniqueId()
        err = None
        if self.rank == 0:
            try:
                _check(lib().ncclGetUniqueId(ctypes.byref(uid)), "ncclGetUniqueId")
                store.set(key, bytes(uid.internal))
            except Exception as e:  # noqa: BLE001  (the other ranks must not wait for the id)
                err = e
                store.set(key, b"")
        else:
            try:
                lib()
            except OSError as e:
                err = e
            raw = store.get(key)
            if len(raw) != NCCL_UNIQUE_ID_BYTES:
                err = err or RcclError("rank 0 could not create the RCCL unique id")
            else:
                ctypes.memmove(ctypes.byref(uid), raw, NCCL_UNIQUE_ID_BYTES)
        if agree is not None and not agree(err is None):
            raise err or RcclError("another rank could not set up RCCL")
        if err is not None:
            raise err
        try:
            with torch.cuda.device(device):
                _check(lib().ncclCommInitRank(ctypes.byref(self.comm), self.world, uid, self.rank),
                       "ncclCommInitRank")
        except Exception as e:      # noqa: BLE001
            err = e
        if agree is not None and not agree(err is None):
            self.close()
            raise err or RcclError("ncclCommInitRank failed on another rank")
        if err is not None:
            raise err

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
        on = device if dist.get_backend() == "nccl" else torch.device("cpu")

        def agree(ok):
            t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=on)
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
            return bool(t.item())

        return cls(dist.get_rank(), dist.get_world_size(), device, store, agree=agree)
