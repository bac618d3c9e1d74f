"""Multi-process (one process per GPU) partition execution and the event gather.

Replaces Spark's executor fan-out and the `.toPandas()` collect (DDM_Process.py:226,
258).  Partition d runs on rank d % world_size (no data moves between ranks: every
rank builds its partitions from the same stream description), then ONE exchange step
gathers the events: an all_gather of per-rank record counts followed by an all_gather of
the padded int64 records [device_id, batch, warn_local, warn_global, change_local,
change_global].  On GPUs the all-gathers run on RCCL directly (ddm_amd.rccl, ctypes on
librccl, HBM to HBM over xGMI); torch.distributed (gloo in the CPU tests) is the
fallback and the rendezvous.  The payload is tiny (<= 48 B per batch), so a
single padded all_gather beats anything ring-bandwidth-shaped.
"""
import numpy as np
import torch
import torch.distributed as dist

RECORD = 6


def local_partitions(parts, rank, world):
    return [(d, f) for d, f in parts if d % world == rank]


def _records(outputs, events_only=False):
    recs = []
    for d, ev in sorted(outputs.items()):
        ev = np.asarray(ev, dtype=np.int64).reshape(-1, 4)
        idx = np.nonzero((ev >= 0).any(axis=1))[0] if events_only else np.arange(len(ev))
        r = np.empty((len(idx), RECORD), dtype=np.int64)
        r[:, 0] = d
        r[:, 1] = idx
        r[:, 2:] = ev[idx]
        recs.append(r)
    return np.concatenate(recs) if recs else np.empty((0, RECORD), dtype=np.int64)


def _gather_rccl(comm, recs_np):
    """The two all-gathers on RCCL itself (ddm_amd.rccl, ctypes): counts, then the padded
    records, HBM to HBM on the current stream."""
    dev, world = comm.device, comm.world
    recs = torch.from_numpy(recs_np).to(dev)
    n = torch.tensor([recs.shape[0]], dtype=torch.int64, device=dev)
    counts_d = torch.empty(world, dtype=torch.int64, device=dev)
    comm.all_gather(n, counts_d)
    counts = [int(c) for c in counts_d.cpu().tolist()]
    cap = max(counts) if counts else 0
    if cap == 0:
        return np.empty((0, RECORD), dtype=np.int64)
    pad = torch.full((cap, RECORD), -1, dtype=torch.int64, device=dev)
    pad[:recs.shape[0]] = recs
    allbuf = torch.empty((world * cap, RECORD), dtype=torch.int64, device=dev)
    comm.all_gather(pad.view(-1), allbuf.view(-1))
    allh = allbuf.cpu().numpy().reshape(world, cap, RECORD)
    return np.concatenate([allh[r, :c] for r, c in enumerate(counts)])


def gather_events(outputs, group=None, device=None, n_rows=None, comm=None):
    """outputs: {device_id: int64 [n_batches-1, 4]} of this rank -> the same dict for ALL
    partitions of all ranks (on every rank).  n_rows ({device_id: output rows} of every
    partition, known to every rank from the stream description): only the batches with an
    event travel (the drift positions; a few KB instead of every batch row) and the
    full outputs are rebuilt with -1 elsewhere.  comm (an rccl.RcclComm): the all-gathers
    run on RCCL through ctypes instead of torch.distributed."""
    recs_np = _records(outputs, events_only=n_rows is not None)
    if comm is not None:
        allrec = _gather_rccl(comm, recs_np)
    else:
        world = dist.get_world_size(group)
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" \
                else torch.device("cpu")
        recs = torch.from_numpy(recs_np).to(device)
        n = torch.tensor([recs.shape[0]], dtype=torch.int64, device=device)
        counts = [torch.zeros_like(n) for _ in range(world)]
        dist.all_gather(counts, n, group=group)
        counts = [int(c.item()) for c in counts]
        cap = max(counts) if counts else 0
        pad = torch.full((cap, RECORD), -1, dtype=torch.int64, device=device)
        pad[:recs.shape[0]] = recs
        bufs = [torch.empty_like(pad) for _ in range(world)]
        dist.all_gather(bufs, pad, group=group)
        allrec = np.concatenate([b[:c].cpu().numpy() for b, c in zip(bufs, counts)]) if cap else \
            np.empty((0, RECORD), dtype=np.int64)
    out = {}
    if n_rows is not None:
        for d, n in n_rows.items():
            out[int(d)] = np.full((int(n), 4), -1, dtype=np.int64)
    for d in np.unique(allrec[:, 0]):
        r = allrec[allrec[:, 0] == d]
        r = r[np.argsort(r[:, 1])]
        if n_rows is not None:
            out[int(d)][r[:, 1]] = r[:, 2:]
        else:
            out[int(d)] = r[:, 2:].copy()
    return out
