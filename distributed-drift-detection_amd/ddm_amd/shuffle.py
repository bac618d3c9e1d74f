"""GPU batch shuffles: one partition's numpy MT19937 stream on the device (csrc/shuffle.hip).

The reference shuffles every 100-row batch with pandas `sample(frac=1)` (DDM_Process.py:187,
:190), i.e. legacy `RandomState.permutation` on numpy's global MT19937, and seeds every
refit with 100 `randint(2**31-1)` draws of the same stream (:102).  `GpuShuffle` keeps
that stream as raw tempered words R in HBM (draw 0 = the next draw of the state it was
reset from) and produces:
  * window(P, W, out)   shuffles of W full batches starting at draw P, on the device
  * host_perm(P, L)     one batch's shuffle on the host from a few words of R (the batch
                        before a refit, the short last batch)
  * host_seeds(P, T)    the T per-tree seeds of a refit
  * numpy_state(X)      numpy's exact (key, pos) after X draws (tempering is invertible)
"""
import ctypes
import functools

import numpy as np
import torch

from . import kernels
from ._capi import check, lib

SUB, CHUNK = 128, 8192
# Segment length of the parallel MT19937 generation: the stream of a partition is cut at
# draws D_0 = 0, D_s = (624 - pos0) + s * JUMP, and segment s >= 1 starts from the state
# T^(s * JUMP)(key0) (ddm_mt_jump), so all segments of a piece are generated at once.
JUMP = 1 << 20
# Algorithmic HBM bytes of the generation kernels (csrc/shuffle.hip), for the bench's
# stream-generation figures: a jump reads its key (624 words + pos) and its polynomial
# (312 u64) and writes the segment's start state; a generate job reads and writes its
# 625-word state and writes 4 B per draw; the tables read a chunk's 8192 draws and write
# 64 sub-chunk entries plus the chunk entry per interval state (S = L - 1, 4 B each).
JUMP_BYTES = 625 * 4 + 312 * 8 + 625 * 4
GEN_STATE_BYTES = 2 * 625 * 4


def table_bytes_per_chunk(L):
    return CHUNK * 4 + (CHUNK // SUB + 1) * (L - 1) * 4


@functools.lru_cache(maxsize=None)
def expected_draws_per_batch(L):
    """Mean 32-bit draws of `permutation(L)`: interval i takes (mask(i)+1)/(i+1) draws."""
    return sum(((1 << int(i).bit_length()) / (i + 1)) for i in range(1, L))


def _untemper(y):
    """MT19937's tempering inverted, in uint32 arithmetic (in place on a copy: ~2x fewer
    passes over the words than the uint64 form; the run's end untempers every partition's
    624 words)."""
    y = np.array(y, dtype=np.uint32)
    y ^= y >> np.uint32(18)
    y ^= (y << np.uint32(15)) & np.uint32(0xefc60000)
    t = y.copy()
    tmp = np.empty_like(y)
    for _ in range(4):                         # 7-bit steps cover the 32 bits
        np.left_shift(t, np.uint32(7), out=tmp)
        tmp &= np.uint32(0x9d2c5680)
        np.bitwise_xor(y, tmp, out=t)
    u = t ^ (t >> np.uint32(11))
    u ^= t >> np.uint32(22)                    # x ^ x >> 11 inverted: x ^ x >> 11 ^ x >> 22
    return u


def untemper_keys(words):
    """_untemper over rows of 624 tempered words at once ([n, 624] -> [n, 624] keys)."""
    return _untemper(np.asarray(words, dtype=np.uint32))


def untemper_state(words, pos):
    """numpy's ('MT19937', key, pos) from 624 tempered stream words."""
    return ("MT19937", _untemper(words), int(pos), 0, 0.0)


def _temper(y):
    y = y.astype(np.uint64)
    y ^= y >> 11
    y ^= (y << 7) & 0x9d2c5680
    y ^= (y << 15) & 0xefc60000
    y ^= y >> 18
    return (y & 0xffffffff).astype(np.uint32)


def fy_from_words(words, L):
    """Legacy permutation(L) from tempered draws -> (perm uint8, draws used) or None."""
    perm = np.arange(L, dtype=np.uint8)
    k = 0
    n = len(words)
    for i in range(L - 1, 0, -1):
        mask = (1 << int(i).bit_length()) - 1
        while True:
            if k >= n:
                return None
            v = int(words[k]) & mask
            k += 1
            if v <= i:
                break
        perm[i], perm[v] = perm[v], perm[i]
    return perm, k


def randint31_from_words(words, T):
    """T x randint(2**31-1) (mask 0x7fffffff, reject 0x7fffffff) -> (seeds, draws) or None."""
    out = np.empty(T, dtype=np.int64)
    k = 0
    for t in range(T):
        while True:
            if k >= len(words):
                return None
            v = int(words[k]) & 0x7fffffff
            k += 1
            if v <= 0x7ffffffe:
                break
        out[t] = v
    return out, k


def perm_seeds_from_words(words, L, T):
    """permutation(L) then T randint(2**31-1) seeds from tempered words (native) ->
    (perm uint8, seeds int64, draws used by the perm, draws used by the seeds) or None."""
    words = np.ascontiguousarray(words, dtype=np.uint32)
    perm = np.empty(max(L, 1), dtype=np.uint8)
    seeds = np.empty(max(T, 1), dtype=np.int64)
    used = np.zeros(2, dtype=np.int64)
    rc = lib.ddm_words_perm_seeds(words.ctypes.data, words.size, int(L), int(T), perm.ctypes.data, seeds.ctypes.data,
                                  used.ctypes.data)
    if rc != 0:
        return None
    return perm[:L], seeds[:T], int(used[0]), int(used[1])


class GpuShuffle:
    """One partition's MT19937 stream resident in HBM, with FSM tables for batch length L.

    R and the tables are produced on `gen_stream` (by default the consuming `stream`
    itself) in pieces, each closed by an event; consumers on `stream` wait on the event of
    the piece that covers what they read (`wait_for`), so generation overlaps the epochs."""

    def __init__(self, device, L, capacity_draws, max_window, stream, gen_stream=None, tab_stream=None,
                 state_rows=None):
        if not 2 <= L <= 256:
            raise ValueError("GPU shuffles need 2 <= batch length <= 256")
        self.device, self.L, self.S, self.stream = device, L, L - 1, stream
        self.gen_stream = gen_stream or stream
        self.tab_stream = tab_stream or self.gen_stream   # tables (after the words they read)
        self.max_window = int(max_window)
        # the stream's start state: `mt` is the key every jump reads, `seg0` segment 0's
        # generator state (it advances as segment 0 is generated); state_rows: two device
        # rows of >= 625 int32 the caller owns and uploads itself (a runner uploads every
        # partition's pair in one copy, reset(upload=False))
        if state_rows is None:
            state_rows = torch.zeros((2, 640), dtype=torch.int32, device=device)
        self.mt, self.seg0 = state_rows[0], state_rows[1]
        self._alloc(max(2 * CHUNK, int(capacity_draws)))
        # the window's first piece, the sub-chunks of the chunk holding its start, then chunks
        self.max_pieces = 4 + CHUNK // SUB + (self.max_window * L * 3) // CHUNK
        self.pieces = torch.empty(self.max_pieces * 16, dtype=torch.uint8, device=device)
        self.first = torch.empty((CHUNK // SUB) * self.S + 8, dtype=torch.int16, device=device)   # + 16-byte over-read
        self.info = torch.zeros(8, dtype=torch.int64, device=device)   # [3..7]: instrumented builds
        self.J = torch.zeros(self.max_window * L, dtype=torch.uint8, device=device)
        self.E = torch.zeros(self.max_window, dtype=torch.int64, device=device)
        self.words_h = torch.empty(4096, dtype=torch.int32, pin_memory=True)
        self.gen = self.tab = 0
        self.ready = []          # [(chunks covered by the tables, event)] in enqueue order
        self.waited = 0          # chunks the consuming stream has waited for
        self.init_key = None
        self.init_pos = 624
        self.seg = None
        self.n_seg = self.jumped = 0
        self._keep = []          # pinned job tables read by in-flight async copies

    def _alloc(self, cap):
        cap = (cap + CHUNK - 1) // CHUNK * CHUNK
        R = torch.empty(cap, dtype=torch.int32, device=self.device)
        Tp = torch.empty(cap // SUB * self.S, dtype=torch.int32, device=self.device)   # prefix tables [chunk][64][S]
        Tc = torch.empty(cap // CHUNK * self.S + 4, dtype=torch.int32, device=self.device)   # + 16-byte over-read
        if getattr(self, "R", None) is not None and self.gen:
            torch.cuda.synchronize(self.device)          # rare: growth past the initial estimate
            R[:self.gen].copy_(self.R[:self.gen])
            Tp[:self.tab * (CHUNK // SUB) * self.S].copy_(self.Tpre[:self.tab * (CHUNK // SUB) * self.S])
            Tc[:self.tab * self.S].copy_(self.Tchunk[:self.tab * self.S])
            torch.cuda.synchronize(self.device)
        self.R, self.Tpre, self.Tchunk, self.cap = R, Tp, Tc, cap
        self.ptrs = (R.data_ptr(), Tp.data_ptr(), Tc.data_ptr())    # changes only here

    def reset(self, rng, synced=False, upload=True):
        """Draw 0 of the device stream = the next draw of `rng` (an MTStream).  synced: the
        caller has synchronised this stream's three HIP streams already (a runner resets all
        its partitions after one synchronisation).  upload=False: the caller uploads the
        state rows (mt, seg0 = key[624], pos) itself, on gen_stream, before any generation."""
        self.init_key = rng.key.copy()
        self.init_pos = int(rng.pos.value)
        if not synced:
            self.stream.synchronize()
            self.gen_stream.synchronize()       # nothing of the previous run may still read R
            self.tab_stream.synchronize()
        self.n_seg = self._segments_for(self.cap)
        if getattr(self, "seg", None) is None or self.seg.shape[0] < self.n_seg:
            with torch.cuda.stream(self.gen_stream):   # allocated, filled and read on gen_stream
                self.seg = torch.zeros((self.n_seg, 640), dtype=torch.int32, device=self.device)
        if upload:
            with torch.cuda.stream(self.gen_stream):
                # from a pinned buffer of this stream's own (asynchronous copy; the previous
                # run's copy from it is done: gen_stream was synchronised)
                if getattr(self, "_st_h", None) is None:
                    self._st_h = torch.empty(625, dtype=torch.int32, pin_memory=True)
                st = self._st_h.numpy().view(np.uint32)
                st[:624] = self.init_key
                st[624] = self.init_pos
                self.mt[:625].copy_(self._st_h, non_blocking=True)
                self.seg0[:625].copy_(self.mt[:625])
        self.jumped = 1                     # segments whose start state exists
        self._keep = []
        self.gen = self.tab = self.waited = 0
        self.ready = []

    def _sp(self):
        return ctypes.c_void_p(self.stream.cuda_stream)

    def _gp(self):
        return ctypes.c_void_p(self.gen_stream.cuda_stream)

    def _tp(self):
        return ctypes.c_void_p(self.tab_stream.cuda_stream)

    def window_draws(self, W):
        """Draws a window of W batches may need (mean + 15% + slack; windows grow R on demand)."""
        return int(W * expected_draws_per_batch(self.L) * 1.15) + 4 * CHUNK

    @staticmethod
    def chunks_for(upto):
        return (int(upto) + CHUNK - 1) // CHUNK + 1

    def seg_start(self, s):
        return 0 if s == 0 else (624 - self.init_pos) + s * JUMP

    def _segments_for(self, draws):
        return max(1, (int(draws) - (624 - self.init_pos)) // JUMP + 1)

    def _jump_to(self, n_seg, out=None):
        """Start states of segments [jumped, n_seg) on gen_stream (ddm_mt_jump, one launch);
        with `out` (a list) the JUMP_DTYPE records are appended to it instead, for one
        launch over many partitions."""
        if n_seg <= self.jumped:
            return
        if n_seg > self.seg.shape[0]:
            torch.cuda.synchronize(self.device)
            with torch.cuda.stream(self.gen_stream):   # before the jumps and generation that read it
                seg = torch.zeros((2 * n_seg, 640), dtype=torch.int32, device=self.device)
                seg[:self.seg.shape[0]].copy_(self.seg)
            self.seg = seg
        nj = n_seg - self.jumped
        polys = kernels.mt_jump_polys(JUMP, n_seg - 1, self.device)
        segs = np.arange(self.jumped, n_seg, dtype=np.uint64)
        rec = np.empty(nj, dtype=kernels.JUMP_DTYPE)
        rec["key"] = self.mt.data_ptr()
        rec["poly"] = polys.data_ptr() + (segs - 1) * (8 * kernels.POLY_WORDS)
        rec["out"] = self.seg.data_ptr() + segs * (4 * self.seg.shape[1])
        rec["scratch"] = 0                  # the jump's word sequence lives in LDS
        self.jumped = n_seg
        if out is not None:
            out.append(rec)
            return
        tab = kernels.PinnedTable(kernels.JUMP_DTYPE, nj, self.device)
        tab.rec[:nj] = rec
        kernels.mt_jump(tab, nj, self.gen_stream)
        self._keep.append(tab)

    def gen_request(self, upto, jumps=None):
        """Grow R to cover draws [0, upto) plus one chunk; returns the (state, R, n) generate
        jobs still to launch on gen_stream (one per segment the new draws touch; every
        segment's state slot continues where its previous piece stopped) and the chunk count
        the tables must reach.  Segment start states still missing are jumped to on
        gen_stream first, or (jumps: a list) their records are appended for the caller's
        one launch, which must precede the generate jobs."""
        need_chunks = self.chunks_for(upto)
        target = need_chunks * CHUNK
        if target > self.cap:
            self._alloc(max(target, int(self.cap * 1.5)))
        reqs = np.empty(0, dtype=kernels.GEN_DTYPE)
        if target > self.gen:
            s_last = self._segments_for(target - 1) - 1
            if s_last >= 1:
                # the segments this piece reaches (all of the expected stream at once was one
                # ~4 ms launch of 1,952 jumps for C3 that held up the first pieces and the
                # first epochs beside it)
                self._jump_to(s_last + 1, jumps)
            s0 = self._segments_for(self.gen) - 1 if self.gen else 0
            seg = np.arange(s0, s_last + 1, dtype=np.int64)
            starts = np.where(seg == 0, 0, (624 - self.init_pos) + seg * JUMP)
            ends = (624 - self.init_pos) + (seg + 1) * JUMP
            lo, hi = np.maximum(self.gen, starts), np.minimum(target, ends)
            keep = lo < hi
            reqs = np.empty(int(keep.sum()), dtype=kernels.GEN_DTYPE)
            sk = seg[keep].astype(np.uint64)
            reqs["state"] = np.where(sk == 0, np.uint64(self.seg0.data_ptr()),
                                     np.uint64(self.seg.data_ptr()) + sk * np.uint64(4 * self.seg.shape[1]))
            reqs["R"] = self.R.data_ptr() + 4 * lo[keep].astype(np.uint64)
            reqs["n"] = hi[keep] - lo[keep]
            self.gen = target
        return reqs, need_chunks

    def tables_to(self, need_chunks, out=None):
        """Tabulate up to need_chunks on tab_stream (ordered after the words they read: the
        caller makes tab_stream wait for gen_stream when they differ); with `out` (a list)
        the TAB_DTYPE record is appended for the caller's one launch instead."""
        if need_chunks > self.tab:
            if out is not None:
                out.append((self.R.data_ptr(), self.tab, need_chunks - self.tab, self.Tpre.data_ptr(),
                            self.Tchunk.data_ptr()))
            else:
                check(lib.ddm_shuffle_tables(self.R.data_ptr(), self.tab, need_chunks - self.tab, self.L,
                                             self.Tpre.data_ptr(), self.Tchunk.data_ptr(), self._tp()),
                      "ddm_shuffle_tables")
            self.tab = need_chunks

    def mark_ready(self, event):
        """Everything enqueued on tab_stream (and so on gen_stream) so far is complete once
        `event` fires."""
        self.ready.append((self.tab, event))

    def wait_for(self, upto):
        """Make the consuming stream wait until draws [0, upto) and their tables exist."""
        need = self.chunks_for(upto)
        if need <= self.waited:
            return
        for cov, ev in self.ready:
            if cov >= need:
                if self.gen_stream is not self.stream:
                    self.stream.wait_event(ev)
                self.waited = cov
                return
        raise RuntimeError(f"draws up to {upto} were never enqueued (tables cover {self.tab} chunks)")

    def ensure(self, upto):
        """Generate R and tabulate chunks so that draws [0, upto) are covered and visible to
        the consuming stream."""
        if self.chunks_for(upto) > self.tab:
            reqs, need_chunks = self.gen_request(upto)
            if len(reqs):
                table = kernels.PinnedTable(kernels.GEN_DTYPE, len(reqs), self.device)
                table.rec[:len(reqs)] = reqs
                kernels.shuffle_generate_batch(table, len(reqs), self.gen_stream)
                self._keep.append(table)
            if self.tab_stream is not self.gen_stream:
                g = torch.cuda.Event()
                g.record(self.gen_stream)
                self.tab_stream.wait_event(g)
            self.tables_to(need_chunks)
            ev = torch.cuda.Event()
            ev.record(self.tab_stream)
            self.mark_ready(ev)
        self.wait_for(upto)

    def job_tuple(self, P, W, perm_out_ptr, stop_ptr=0, pick_offset=0, pick_last=0, pick_out_ptr=0):
        """fill_job's record as a tuple in kernels.JOB_DTYPE field order."""
        assert 0 <= W <= self.max_window
        return (self.R.data_ptr(), self.Tpre.data_ptr(), self.Tchunk.data_ptr(), self.waited * CHUNK, int(P), int(W),
                self.pieces.data_ptr(), self.info.data_ptr(), self.J.data_ptr(), self.E.data_ptr(), int(perm_out_ptr),
                int(stop_ptr), int(pick_offset), int(pick_last), int(pick_out_ptr), self.first.data_ptr())

    def fill_job(self, rec, P, W, perm_out_ptr, stop_ptr=0, pick_offset=0, pick_last=0, pick_out_ptr=0):
        """One ddm_shuffle_job record (kernels.JOB_DTYPE) for a window of W batches from draw P;
        R must already cover it (window_draws)."""
        assert 0 <= W <= self.max_window
        rec["R"], rec["Tpre"], rec["Tchunk"] = self.R.data_ptr(), self.Tpre.data_ptr(), self.Tchunk.data_ptr()
        rec["first"] = self.first.data_ptr()
        rec["avail"], rec["P"], rec["W"] = self.waited * CHUNK, int(P), int(W)
        rec["pieces"], rec["info"] = self.pieces.data_ptr(), self.info.data_ptr()
        rec["J"], rec["E"], rec["perm_out"] = self.J.data_ptr(), self.E.data_ptr(), int(perm_out_ptr)
        rec["stop"], rec["pick_offset"], rec["pick_last"] = int(stop_ptr), int(pick_offset), int(pick_last)
        rec["pick_out"] = int(pick_out_ptr)

    def window(self, P, W, perm_out, timer=None):
        """Shuffles of W batches from draw P into perm_out (device uint8, W*L bytes); E[b] =
        last draw of batch b (device)."""
        assert 0 < W <= self.max_window and perm_out.numel() >= W * self.L
        self.ensure(P + self.window_draws(W))
        ev = (None, None) if timer is None else (timer.ev[0], timer.ev[1])
        check(lib.ddm_shuffle_window(self.R.data_ptr(), self.Tpre.data_ptr(), self.Tchunk.data_ptr(),
                                     self.waited * CHUNK, int(P), int(W), self.L, self.pieces.data_ptr(),
                                     self.max_pieces, self.info.data_ptr(), self.J.data_ptr(), self.E.data_ptr(),
                                     perm_out.data_ptr(), self.first.data_ptr(), self._sp(), *ev),
              "ddm_shuffle_window")

    def pick(self, stop_ptr, W, offset, last, out_ptr):
        check(lib.ddm_shuffle_pick(stop_ptr, self.E.data_ptr(), int(W), int(offset), int(last), out_ptr, self._sp()),
              "ddm_shuffle_pick")

    def words(self, P, n):
        """Host copy of R[P:P+n] (synchronises the stream)."""
        self.ensure(P + n)
        if n > self.words_h.numel():
            self.words_h = torch.empty(n, dtype=torch.int32, pin_memory=True)
        with torch.cuda.stream(self.stream):
            self.words_h[:n].copy_(self.R[P:P + n], non_blocking=True)
        self.stream.synchronize()
        return self.words_h[:n].numpy().view(np.uint32)

    def host_perm(self, P, L):
        n = max(64, 3 * L)
        while True:
            r = fy_from_words(self.words(P, n), L)
            if r is not None:
                return r[0], P + r[1]
            n *= 2

    def host_seeds(self, P, T):
        n = T + 16
        while True:
            r = randint31_from_words(self.words(P, n), T)
            if r is not None:
                return r[0], P + r[1]
            n *= 2

    def state_plan(self, X):
        """(None, state) when numpy's state after X draws needs no stream words, else
        (start, pos): the state is the untempered words [start, start+624) at pos."""
        first = 624 - self.init_pos
        if X <= first:
            return None, ("MT19937", self.init_key.copy(), self.init_pos + int(X), 0, 0.0)
        r = int(X) - first
        q = (r - 1) // 624
        return first + q * 624, r - q * 624

    def numpy_state(self, X):
        """numpy's ('MT19937', key, pos) after X draws of this stream."""
        start, pos = self.state_plan(X)
        if start is None:
            return pos
        return ("MT19937", _untemper(self.words(start, 624)), pos, 0, 0.0)
