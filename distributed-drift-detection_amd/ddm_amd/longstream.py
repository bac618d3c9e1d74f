"""One long DDM error stream in mode 1, scanned in parallel on one GPU and across GPUs
("single long stream").

run_DDM carries one detector from batch to batch (DDM_Process.py:144-152,202) and a change
drops it, so the next batch starts fresh (:207-210).  The stream is cut into segments of
whole batches (16*k batches, so every segment starts 16-byte aligned); all segments are
scanned at once, each speculatively from a fresh detector, by ddm_scan_batches (the
segments are its "streams").  The carries are then resolved in stream order: a segment
whose true carry-in is fresh (the batch before it changed) keeps its speculative result;
a run of segments entered with a carried detector is rescanned from it in ONE
ddm_scan_certified call (row-parallel, every decision certified against the reference's
rounded recurrence, csrc/scan_cert.hip; ddm_scan_long, the exact chained recurrence, with
certified=False), up to the first segment boundary whose carry is fresh again.  On
reset-heavy streams almost every carry is fresh, so the resolution is a host loop over the
segments' end states plus a few rescans.  A certified rescan hands back its detector with a
bound on |p - p_ref| (0 when it is exact, e.g. p stuck at 1); the bound travels with the
carry into the next rescan and across ranks.

Across GPUs every rank owns a contiguous run of segments (chunk_bounds).  The ranks scan
and resolve their segments in parallel as if their carry-in were fresh, then ONE
all-gather gives every rank every chunk's carry-out under that assumption: a rank whose
carry-in comes out fresh keeps its result without waiting for anyone.  Only a carried
(non-fresh) detector crossing a rank boundary costs another round (that rank resolves from
the true carry and the next all-gather publishes its carry-out).  One all-reduce(MIN) gives
the first change of the whole stream.  The collectives run on device tensors under the
`nccl` (RCCL) backend and on host tensors under gloo.  Results equal one sequential scan
of the whole stream bit for bit, whatever the number of ranks.
"""
import numpy as np

from .kernels import STATE_DTYPE, fresh_states

_FRESH = fresh_states(1)[0]
_I64_MAX = np.iinfo(np.int64).max


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


class Segments:
    """A chunk's segments: row offsets, lengths and the offsets of their batches' event rows."""

    def __init__(self, n_rows, seg_len, per_batch):
        n_full = n_rows // seg_len
        tail = n_rows - n_full * seg_len
        self.rows0 = [k * seg_len for k in range(n_full)] + ([n_full * seg_len] if tail else [])
        self.lens = [seg_len] * n_full + ([tail] if tail else [])
        nbs = [-(-L // per_batch) for L in self.lens]
        self.ev_off = np.concatenate([[0], np.cumsum(nbs)]).astype(np.int64)
        self.n = len(self.lens)


_NO_BOUND = np.zeros(2)


class InexactCarry(RuntimeError):
    """A certified carried scan met a decision inside its bound while its incoming state was
    itself inexact (ddm_scan_certified status 3): its results are void; the run must be
    redone from an exact carry."""


def _carried(scanner, row0, n_rows, state, bound, exact=False):
    """Mode-1 scan of rows [row0, row0 + n_rows) as one stream from `state` (whose p and
    p_min are within `bound` of the reference's); (events, end state, its bound).  exact:
    the exact kernel (the state must be the reference's)."""
    if hasattr(scanner, "carried"):
        out = scanner.carried(row0, n_rows, state, bound, exact=exact) if exact else \
            scanner.carried(row0, n_rows, state, bound)
        return out if len(out) == 3 else (out[0], out[1], _NO_BOUND)
    st = np.empty(1, STATE_DTYPE)
    st[0] = state
    e, f = scanner.scan(row0, 1, n_rows, st)
    return e, f[0], _NO_BOUND


def resolve(carry, spec_final, segs, ev, scanner, chain=4, bound=None):
    """The segments' true carries in stream order, from carry-in `carry` (p and p_min within
    `bound` of the reference's; None: exact).  spec_final[k]: segment k's end state from a
    fresh carry-in; ev: the speculative event rows, overwritten where a segment is rescanned.
    A run of segments entered with a carried detector is rescanned in one carried scan of up
    to `chain` segments (doubling while the run goes on), up to the first of them whose last
    batch changed (the carry after it is fresh again).  Returns (the end state after the last
    segment, segments rescanned, the end state's bound)."""
    k, redone = 0, 0
    n = segs.n
    bd = _NO_BOUND if bound is None else np.asarray(bound, np.float64)
    exact_at = (0, carry) if not np.any(bd) else None   # the last carry known to be the reference's
    force_exact = False
    while k < n:
        if state_fresh(carry):
            carry = spec_final[k]
            bd = _NO_BOUND                              # ddm_scan_batches: exact from a fresh carry
            k += 1
            exact_at = (k, carry)
            continue
        m = min(n, k + chain)
        rows = sum(segs.lens[k:m])
        try:
            e, f, fb = _carried(scanner, segs.rows0[k], rows, carry, bd, exact=force_exact)
        except InexactCarry:
            if exact_at is None:                        # inexact since this call's carry-in
                raise
            # back to the last exact carry, that run on the exact kernel
            k, carry = exact_at
            bd, force_exact = _NO_BOUND, True
            continue
        force_exact = False
        base = segs.ev_off[k]
        j_end = None
        for j in range(k, m - 1):                       # a change in segment j's last batch
            if e[segs.ev_off[j + 1] - 1 - base, 1] >= 0:
                j_end = j
                break
        if j_end is None:
            ev[base:segs.ev_off[m]] = e
            carry, bd = f, fb
            redone += m - k
            k = m
            chain *= 2
            if not np.any(bd):
                exact_at = (k, carry)
        else:
            ev[base:segs.ev_off[j_end + 1]] = e[:segs.ev_off[j_end + 1] - base]
            carry, bd = _FRESH, _NO_BOUND
            redone += j_end + 1 - k
            k = j_end + 1
            exact_at = (k, carry)
    return carry, redone, bd


class DeviceScanner:
    """ddm_scan_batches over equal-length segments of a device error buffer and
    ddm_scan_certified (certified=False: ddm_scan_long) for carried runs (the product path;
    the CPU tests inject a scanner with the same interface).  Scratch buffers are kept and
    reused across calls; `status` counts the certified calls by outcome: [certified, handed
    to the exact kernel for a decision inside its bound, (mode 1) handed over after four
    changes in the run, void (a decision inside the bound of an inexact carry-in: redone
    from the last exact carry by resolve)]."""

    def __init__(self, err, params, stream=None, certified=True):
        import torch
        self.err, self.params, self.stream = err, params, stream
        self.torch = torch
        self.certified = certified
        self.status = [0, 0, 0, 0]
        self._scratch = {}

    def _buf(self, key, nbytes):
        b = self._scratch.get(key)
        if b is None or b.numel() < nbytes:
            b = self.torch.empty(max(1, int(nbytes)), dtype=self.torch.uint8, device=self.err.device)
            self._scratch[key] = b
        return b

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
        scratch = self._buf("batches", kernels.scan_batches_scratch_size(n_segments, seg_len, pb))
        kernels.scan_batches(self.err[row0:], n_segments, seg_len, self.params, st, ev, scratch, stream=self.stream)
        torch.cuda.synchronize(dev)
        return ev[:n_segments * nb].cpu().numpy(), st.cpu().numpy().view(STATE_DTYPE).copy()

    def carried(self, row0, n_rows, state, bound=None, exact=False):
        """(ev int32 [nb, 2], end state, its bound) of rows [row0, row0 + n_rows) as ONE mode-1
        stream from `state` (p and p_min within `bound` of the reference's); exact: on
        ddm_scan_long whatever `certified` says.  Raises InexactCarry when the certified scan
        reports status 3."""
        from . import kernels
        from ._capi import DDM_CERT_INEXACT, DDM_STOP_FAILED
        torch = self.torch
        dev = self.err.device
        pb = self.params.per_batch
        nb = -(-n_rows // pb)
        st = torch.from_numpy(np.array([state], dtype=STATE_DTYPE).view(np.uint8).copy()).to(dev)
        ev = torch.empty((max(1, nb), 2), dtype=torch.int32, device=dev)
        stop = torch.empty(1, dtype=torch.int32, device=dev)
        off = torch.tensor([row0], dtype=torch.int64, device=dev)
        end = torch.tensor([row0 + n_rows], dtype=torch.int64, device=dev)
        base = torch.zeros(1, dtype=torch.int64, device=dev)
        if exact or not self.certified:
            if bound is not None and np.any(np.asarray(bound) != 0):
                raise ValueError("ddm_scan_long needs the reference's exact state (bound 0)")
            scratch = self._buf("long", kernels.scan_long_scratch_size(1, n_rows, pb))
            kernels.scan_long(self.err, off, self.params, st, base, ev, n_rows, scratch, ends=end, stop=stop, mode=1,
                              stream=self.stream)
            torch.cuda.synchronize(dev)
            if int(stop.item()) == DDM_STOP_FAILED:
                raise RuntimeError("ddm_scan_long gave up waiting for a carried state")
            return ev[:nb].cpu().numpy(), st.cpu().numpy().view(STATE_DTYPE)[0].copy(), _NO_BOUND
        bd = torch.from_numpy(np.asarray(_NO_BOUND if bound is None else bound, np.float64).reshape(2).copy()).to(dev)
        status = torch.empty(1, dtype=torch.int32, device=dev)
        scratch = self._buf("cert", kernels.scan_certified_scratch_size(1, n_rows, pb))
        kernels.scan_certified(self.err, off, self.params, st, base, ev, n_rows, scratch, ends=end, stop=stop, mode=1,
                               bound=bd, status=status, stream=self.stream)
        torch.cuda.synchronize(dev)
        code = int(status.item())
        self.status[code] += 1
        if code == DDM_CERT_INEXACT:
            raise InexactCarry(f"rows [{row0}, {row0 + n_rows}): uncertified decision from an inexact carry")
        if int(stop.item()) == DDM_STOP_FAILED:
            raise RuntimeError("ddm_scan_long gave up waiting for a carried state")
        return ev[:nb].cpu().numpy(), st.cpu().numpy().view(STATE_DTYPE)[0].copy(), bd.cpu().numpy()


def _coll_device():
    """Where the collectives' tensors live: HBM under RCCL ("nccl"), host memory under gloo."""
    import torch
    import torch.distributed as dist
    if dist.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def _all_gather_states(state, valid, bound=None):
    """Every rank's (valid, 56-byte state, its 16-byte bound) -> [(valid, state, bound)] in
    rank order (one all_gather of 80-byte records)."""
    import torch
    import torch.distributed as dist
    dev = _coll_device()
    rec = np.zeros(80, dtype=np.uint8)
    rec[:56] = np.array([state], dtype=STATE_DTYPE).view(np.uint8)
    rec[56] = 1 if valid else 0
    rec[64:80] = np.asarray(_NO_BOUND if bound is None else bound, np.float64).reshape(2).view(np.uint8)
    t = torch.from_numpy(rec).to(dev)
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    res = []
    for o in out:
        b = o.cpu().numpy()
        res.append((bool(b[56]), b[:56].view(STATE_DTYPE)[0].copy(), b[64:80].view(np.float64).copy()))
    return res


def scan_long_stream(scanner, n_rows, per_batch, seg_batches=64, state_in=None, distributed=False, first_batch=0,
                     with_bound=False):
    """Mode-1 DDM over the rows [0, n_rows) the scanner holds, as ONE stream (the whole
    stream, or this rank's chunk of it when `distributed`: the ranks of the default
    torch.distributed group, chunks as chunk_bounds gives them, rank order = stream order).
    Returns (ev int32 [nb, 2] of this rank's batches, the stream's end state (on the last
    rank; the carry out of this rank's chunk elsewhere), the first change's global batch
    index or -1), plus the end state's bound (p, p_min) when with_bound.  first_batch: the
    global index of this chunk's first batch."""
    import torch
    import torch.distributed as dist
    seg_len = segment_rows(seg_batches, per_batch)
    segs = Segments(n_rows, seg_len, per_batch)
    world = dist.get_world_size() if distributed else 1
    rank = dist.get_rank() if distributed else 0
    n_full = n_rows // seg_len
    ev_parts, finals = [], []
    calls = ([(0, n_full, seg_len)] if n_full else []) + ([(n_full * seg_len, 1, n_rows - n_full * seg_len)]
                                                           if n_rows > n_full * seg_len else [])
    for row0, n_seg, length in calls:             # speculation: every segment from a fresh detector
        e, f = scanner.scan(row0, n_seg, length, fresh_states(n_seg))
        ev_parts.append(e)
        finals.append(f)
    spec_ev = np.concatenate(ev_parts) if ev_parts else np.empty((0, 2), np.int32)
    spec_final = np.concatenate(finals) if finals else np.empty(0, STATE_DTYPE)
    carry0 = (fresh_states(1) if state_in is None else np.asarray(state_in, STATE_DTYPE).reshape(1))[0]

    failed = [False]

    def resolved(carry, bound):
        ev = spec_ev.copy()
        try:
            end, _, bd = resolve(carry, spec_final, segs, ev, scanner, bound=bound)
        except InexactCarry:
            # only a carry-in from another rank (with a bound) gets here: this rank's results
            # are void, the ranks agree on it below and redo the stream on the exact kernel
            failed[0] = True
            return ev, carry, _NO_BOUND
        return ev, end, bd

    if not distributed:
        ev, end, bd = resolved(carry0, None)
    else:
        # every rank resolves as if its carry-in were fresh; one all-gather of the carry-outs
        # tells each rank its true carry-in unless a carried detector crosses a rank boundary
        ev_f, end_f, bd_f = resolved(_FRESH, None)
        ends_f = [(s, b) for _, s, b in _all_gather_states(end_f, True, bd_f)]
        carry_in = [(carry0, None)] + [None] * (world - 1)
        true_end = {}
        mine = None
        while True:                       # every rank takes the same decisions (same data)
            for q in range(1, world):
                if carry_in[q] is None and carry_in[q - 1] is not None:
                    if state_fresh(carry_in[q - 1][0]):
                        carry_in[q] = ends_f[q - 1]
                    elif q - 1 in true_end:
                        carry_in[q] = true_end[q - 1]
            if all(c is not None for c in carry_in):
                break
            # a carried detector crosses a rank boundary: the ranks whose carry-in is known and
            # carried resolve from it and publish their true carry-out (at least one per round)
            new = None
            if carry_in[rank] is not None and not state_fresh(carry_in[rank][0]) and rank not in true_end:
                mine = resolved(*carry_in[rank])
                new = mine
            for q, (ok, st, b) in enumerate(_all_gather_states(new[1] if new is not None else _FRESH,
                                                               new is not None, new[2] if new is not None else None)):
                if ok:
                    true_end[q] = (st, b)
        if state_fresh(carry_in[rank][0]):
            ev, end, bd = ev_f, end_f, bd_f
        else:
            ev, end, bd = mine if mine is not None else resolved(*carry_in[rank])
    if distributed:
        t = torch.tensor([1 if failed[0] else 0], dtype=torch.int64, device=_coll_device())
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        if int(t.item()):
            cert = getattr(scanner, "certified", False)
            scanner.certified = False
            try:
                return scan_long_stream(scanner, n_rows, per_batch, seg_batches, state_in, distributed, first_batch,
                                        with_bound)
            finally:
                scanner.certified = cert
    hit = np.nonzero(ev[:, 1] >= 0)[0]
    first = int(first_batch + hit[0]) if len(hit) else -1
    if distributed:
        t = torch.tensor([first if first >= 0 else _I64_MAX], dtype=torch.int64, device=_coll_device())
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        first = int(t.item()) if int(t.item()) != _I64_MAX else -1
    return (ev, end, first, bd) if with_bound else (ev, end, first)
