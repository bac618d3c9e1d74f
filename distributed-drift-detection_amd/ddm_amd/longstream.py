"""One long DDM error stream in mode 1, scanned in parallel on one GPU and across GPUs
("single long stream").

run_DDM carries one detector from batch to batch (DDM_Process.py:144-152,202) and a change
drops it, so the next batch starts fresh (:207-210).  The stream is cut into segments of
whole batches (16*k batches, so every segment starts 16-byte aligned); all segments are
scanned at once, each speculatively from a fresh detector, by ddm_scan_batches (the
segments are its "streams").  The carries are then resolved in stream order: a segment
whose true carry-in is fresh (the batch before it changed) keeps its speculative result;
any other is rescanned from the carried detector, and the carry after it is the rescan's.
On reset-heavy streams almost every carry is fresh, so the resolution is a host loop over
the segments' end states plus a few one-segment rescans.

Across GPUs every rank owns a contiguous run of segments (chunk_bounds).  The ranks scan
their segments in parallel; the carry then hops once per rank boundary (one 56-byte state,
torch.distributed send/recv) while each rank resolves its own segments, and one
all-reduce(MIN) gives the first change of the whole stream.  Results equal one sequential
scan of the whole stream bit for bit, whatever the number of ranks.
"""
import numpy as np

from .kernels import STATE_DTYPE, fresh_states


def state_fresh(st):
    """A carry-in that behaves as a fresh detector: a pending change (skmultiflow resets on
    the next add) or the reset state itself (csrc/scan_batches.hip state_fresh)."""
    return bool(st["in_concept_change"]) or (
        int(st["sample_count"]) == 1 and float(st["miss_prob"]) == 1.0 and float(st["miss_std"]) == 0.0
        and np.isinf(st["miss_prob_min"]) and np.isinf(st["miss_sd_min"]) and np.isinf(st["miss_prob_sd_min"]))


def segment_rows(seg_batches, per_batch):
    if seg_batches <= 0 or seg_batches % 16:
        raise ValueError("seg_batches must be a positive multiple of 16")
    return seg_batches * per_batch


def chunk_bounds(n_rows, world, seg_rows):
    """Row ranges [lo, hi) of the ranks: contiguous runs of whole segments, the last rank
    taking the tail."""
    n_seg = n_rows // seg_rows
    cuts = [min(n_seg, (n_seg * r + world - 1) // world) * seg_rows for r in range(world)] + [n_rows]
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def resolve(carry, spec_final, n_segments, rescan):
    """The segments' true carries in stream order.  spec_final[k]: segment k's end state from
    a fresh carry-in; rescan(k, carry) -> (events of segment k, its end state) from `carry`.
    Returns (the end state after the last segment, {k: events} of the rescanned segments)."""
    redone = {}
    for k in range(n_segments):
        if state_fresh(carry):
            carry = spec_final[k]
        else:
            redone[k], carry = rescan(k, carry)
    return carry, redone


class DeviceScanner:
    """ddm_scan_batches over equal-length segments of a device error buffer (the product
    path; the CPU tests inject a scanner with the same interface)."""

    def __init__(self, err, params, stream=None):
        import torch
        self.err, self.params, self.stream = err, params, stream
        self.torch = torch

    def scan(self, row0, n_segments, seg_len, states):
        """(ev int32 [n_segments*nb, 2], end states) of segments err[row0 + k*seg_len, +seg_len)
        from the carry-in `states` (STATE_DTYPE [n_segments])."""
        from . import kernels
        torch = self.torch
        dev = self.err.device
        pb = self.params.per_batch
        nb = -(-seg_len // pb)
        st = torch.from_numpy(np.ascontiguousarray(states).view(np.uint8).copy()).to(dev)
        ev = torch.empty((max(1, n_segments * nb), 2), dtype=torch.int32, device=dev)
        scratch = torch.empty(kernels.scan_batches_scratch_size(n_segments, seg_len, pb), dtype=torch.uint8,
                              device=dev)
        kernels.scan_batches(self.err[row0:], n_segments, seg_len, self.params, st, ev, scratch, stream=self.stream)
        torch.cuda.synchronize(dev)
        return ev[:n_segments * nb].cpu().numpy(), st.cpu().numpy().view(STATE_DTYPE).copy()


def scan_long_stream(scanner, n_rows, per_batch, seg_batches=64, state_in=None, distributed=False, first_batch=0):
    """Mode-1 DDM over the rows [0, n_rows) the scanner holds, as ONE stream (the whole
    stream, or this rank's chunk of it when `distributed`: the ranks of the default
    torch.distributed group, chunks as chunk_bounds gives them, rank order = stream order).  Returns (ev int32
    [nb, 2] of this rank's batches, the stream's end state (on the last rank; the carry out
    of this rank's chunk elsewhere), the first change's global batch index or -1).
    first_batch: the global index of this chunk's first batch."""
    import torch
    import torch.distributed as dist
    seg_len = segment_rows(seg_batches, per_batch)
    n_full = n_rows // seg_len
    tail = n_rows - n_full * seg_len
    world = dist.get_world_size() if distributed else 1
    rank = dist.get_rank() if distributed else 0
    parts = []                                    # (row0, n_segments, length) per scan call
    if n_full:
        parts.append((0, n_full, seg_len))
    if tail:
        parts.append((n_full * seg_len, 1, tail))
    seg_rows0 = [k * seg_len for k in range(n_full)] + ([n_full * seg_len] if tail else [])
    seg_lens = [seg_len] * n_full + ([tail] if tail else [])
    ev_parts, finals = [], []
    for row0, n_seg, length in parts:             # speculation: every segment from a fresh detector
        e, f = scanner.scan(row0, n_seg, length, fresh_states(n_seg))
        ev_parts.append(e)
        finals.append(f)
    ev = np.concatenate(ev_parts) if ev_parts else np.empty((0, 2), np.int32)
    spec_final = np.concatenate(finals) if finals else np.empty(0, STATE_DTYPE)
    nbs = [-(-L // per_batch) for L in seg_lens]
    ev_off = np.concatenate([[0], np.cumsum(nbs)]).astype(np.int64)

    def rescan(k, carry):
        st = np.empty(1, STATE_DTYPE)
        st[0] = carry
        e, f = scanner.scan(seg_rows0[k], 1, seg_lens[k], st)
        return e, f[0]

    # the carry-in of this rank's chunk: the previous rank's carry-out (one hop)
    buf = torch.zeros(56, dtype=torch.uint8)
    carry = (fresh_states(1) if state_in is None else np.asarray(state_in, STATE_DTYPE).reshape(1))[0]
    if world > 1 and rank > 0:
        dist.recv(buf, src=rank - 1)
        carry = buf.numpy().view(STATE_DTYPE)[0].copy()
    end, redone = resolve(carry, spec_final, len(seg_lens), rescan)
    for k, e in redone.items():
        ev[ev_off[k]:ev_off[k + 1]] = e
    if world > 1 and rank < world - 1:
        out = np.array([end], dtype=STATE_DTYPE).view(np.uint8)
        buf = torch.from_numpy(out.copy())
        dist.send(buf, dst=rank + 1)
    hit = np.nonzero(ev[:, 1] >= 0)[0]
    first = int(first_batch + hit[0]) if len(hit) else -1
    if world > 1:
        t = torch.tensor([first if first >= 0 else np.iinfo(np.int64).max], dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        first = int(t.item()) if int(t.item()) != np.iinfo(np.int64).max else -1
    return ev, end, first
