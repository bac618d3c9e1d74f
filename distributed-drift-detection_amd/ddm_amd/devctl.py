"""Device-resident epochs for the BatchRunner (csrc/ctl.hip).

The BatchRunner (controller.py) runs run_DDM_loop (DDM_Process.py:170-213) for many
partitions in lockstep epochs.  On the host path every epoch ends in a read-back: the host
learns where each partition's scan stopped, moves its RNG position, plans the next window
and builds the next epoch's tables.  Here those decisions (BatchRunner._refit_prep's device
branch, _epoch's window and _epoch_after) are taken by k_ctl on the device, so the host
enqueues groups of epochs ahead and only polls the partitions' records between groups:

    host:    enter (upload the records, plan + shuffle the first windows)
             [K epochs][K epochs] ... poll the records of the group before the last one
    device:  predict -> scan (+ long scan) -> [pick -> staging (events into a per-partition
             log, batch d+1's shuffle, the refit's seeds) -> decisions, next tables: one
             kernel, k_stage_ctl] -> next windows' shuffles (side stream) | device refits -> ...

A partition the device cannot carry on alone stalls (a refit that reported a status or did
not compile, stream words that ran out) or parks (a short last batch still to shuffle);
the phase ends, the host takes the records back into its own per-partition state and runs
one host epoch (which handles them exactly as before), then the runner re-enters device
mode.  The decisions are the host's, line for line, so results do not depend on the mode
(tests/test_gpu_devctl.py).
"""
import ctypes
import os
import time

import numpy as np
import torch

from . import dfit, kernels
from ._capi import DdmCtlEpoch, check, lib
from .shuffle import CHUNK, expected_draws_per_batch

CTL = kernels.CTL_PART_DTYPE
_OFF = {name: CTL.fields[name][1] for name in CTL.names}
PREDICT_BLOCKS = 2048
GROUP = 4                       # epochs per enqueued group
# Decoupled epochs (csrc/ctl.hip): when the partitions' windows average at least this many
# rows, the predict writes row-order errors without waiting for the window's shuffles (a
# serial chain of ~130 us at C3's 14k-batch windows, longer than the refit beside it) and a
# permutation kernel puts them into DDM order after it; small windows (C5, c2) keep the
# shuffles before the predict (they finish under the refit, and the permutation would be one
# launch more per epoch).
DECOUPLE_ROWS = int(os.environ.get("DDM_DECOUPLE_ROWS", 200_000))
# DDM_CTL_GRAPH=1: each group of epochs is one replayed hipGraph (ddm_ctl_graph_create) instead
# of ~20 launches and event operations per epoch enqueued from the host
CTL_GRAPH = os.environ.get("DDM_CTL_GRAPH", "0") not in ("", "0")
# the epochs' fork (main -> side stream) and join (side -> main) by flags in device memory
# (ddm_ctl_epoch.sync_flags: a one-wave store / poll kernel pair, ~12 us per epoch) instead
# of HIP events (~30 us); DDM_CTL_FLAGS=0: events
CTL_FLAGS = os.environ.get("DDM_CTL_FLAGS", "1") not in ("", "0")
# developer check: _write_records' column form against its per-partition loop form
CHECK_RECORDS = os.environ.get("DDM_CHECK_RECORDS", "0") not in ("", "0")


class FlagTimeout(RuntimeError):
    """A cross-stream flag wait of a device phase gave up (csrc/common.h flag_poll, a hang
    guard): a consumer may have read data its producer had not finished, so the phase's
    results are void.  BatchRunner.run redoes the run with event-ordered fork / join."""


class PredictTimer:
    """The span of every device-epoch predict launch of the timed runs on the 100 MHz device
    clock (ddm_ctl.predict_clock): the kernel stamps its workgroups' starts and ends into 8
    shards and the staging kernel after it adds max(end) - min(start) to word 16 and 1 to word
    17.  The kernel's own time, as a rocprofv3 kernel record measures it (HIP events around
    the launch added ~20 us of queue time to each, and ~7 us per event to the epoch), launches
    with no rows (the trailing epochs of a phase) included."""

    TICK_MS = 1e-5                   # 10-ns ticks

    def __init__(self, device):
        self.d = torch.zeros(18, dtype=torch.int64, device=device)
        self.d[:8] = -1              # min(start) shards: ~0
        self.h = torch.zeros(2, dtype=torch.int64, pin_memory=True)

    def ptr(self):
        return self.d.data_ptr()

    def take(self, stream):
        """(ms, launches) since the last take; the stream is synchronised."""
        with torch.cuda.stream(stream):
            self.h.copy_(self.d[16:18], non_blocking=True)
            self.d[16:18].zero_()
        stream.synchronize()
        return float(self.h[0]) * self.TICK_MS, int(self.h[1])

    def close(self):
        pass


class DeviceController:
    """The device-mode state of one BatchRunner (its buffers never move)."""

    def __init__(self, runner, long_min_rows, long_cap_rows):
        r = runner
        self.r = r
        n, dev = len(r.parts), r.device
        self.n = n
        self.parts_d = torch.zeros(n * CTL.itemsize, dtype=torch.uint8, device=dev)
        self.parts_h = torch.zeros(n * CTL.itemsize, dtype=torch.uint8, pin_memory=True)
        self.rec = self.parts_h.numpy().view(CTL)
        # two pinned copies of the records for the polls (one in flight, one read)
        self.poll_h = [torch.zeros(n * CTL.itemsize, dtype=torch.uint8, pin_memory=True) for _ in range(2)]
        self.res_ptrs = torch.zeros(n, dtype=torch.int64, device=dev)
        self.pstall = torch.zeros(n, dtype=torch.int32, device=dev)
        # [0] the fused staging + decision kernel's block ticket (it leaves it 0), [1] the next
        # epoch has a long window (ddm_scan_long's blocks return at once otherwise)
        self.sync = torch.zeros(2, dtype=torch.int32, device=dev)
        self.logs = [torch.empty(3 * max(1, nb), dtype=torch.int32, device=dev) for nb in r.nbs]
        self.log_off = np.concatenate([[0], np.cumsum([3 * max(1, nb) for nb in r.nbs])]).astype(np.int64)
        self.logs_h = torch.empty(int(self.log_off[-1]), dtype=torch.int32, pin_memory=True)   # read-back of all
        self.log_ptrs = torch.tensor([lg.data_ptr() for lg in self.logs], dtype=torch.int64, device=dev)
        self.log_b0 = torch.zeros(n, dtype=torch.int64, device=dev)
        self.avail_h = torch.zeros(64 * n, dtype=torch.int64, pin_memory=True)   # H2D sources (a ring)
        self._avail_k = 0
        self.long_min_rows, self.long_cap_rows = int(long_min_rows), int(long_cap_rows)
        # ddm_scan_long is enqueued in the epochs only once a window needed it (a partition
        # stalls with CTL_STALL_LONG the first time): until then every epoch is one launch
        # shorter (C5: ~6 us of each ~150-us epoch)
        self.long_ok = False
        # row-order errors of decoupled epochs: a buffer shaped like the runner's err
        self.err_rows = torch.empty_like(r.err_all)
        self.decouple_ok = True      # off after a decoupled predict found a forest it cannot take
        self.timers = []             # per-epoch HIP event pairs when the runner times kernels
        self.seg_log = None          # (segs, res) device copies per epoch when the runner logs predicts
        self.pred_timer = None       # a PredictTimer while the runner times the predict launches
        self.graphs = {}             # (decouple, long_ok) -> captured group of GROUP epochs
        # fork / join numbers: published on the device, enqueued so far on the host (both
        # monotonic for the runner's life), and the device's count of waits that gave up
        self.sync_flags = torch.zeros(4, dtype=torch.int32, device=dev)
        self.sync_seq = (ctypes.c_uint32 * 3)()
        self.sync_h = torch.zeros(4, dtype=torch.int32, pin_memory=True)
        self.flags_ok = True         # off for the runner's life after a FlagTimeout
        self._E = None

    # ---------------------------------------------------------------- eligibility
    def eligible(self, live):
        """Device epochs need device refits, compiled forests and no host-staged refit."""
        r = self.r
        if not r.dfit_rows or self.n > PREDICT_BLOCKS:    # a predict block per window at least
            return False
        for ps in live:
            if ps.retrain:
                if not (ps.staged is not None and isinstance(ps.staged[0], str)):
                    return False
                continue
            f = ps.forest
            if isinstance(f, dfit.DeviceFitForest):
                if not f.compiled:
                    return False
            elif f is None or not getattr(f, "compiled", False) or f.desc.cf_slots > 32:
                return False
        return True

    # ---------------------------------------------------------------- records
    def _epoch_struct(self):
        if self._E is not None:
            return self._E
        r = self.r
        E = DdmCtlEpoch()
        base = r.ctrl_d.data_ptr()
        E.stream, E.side_stream = r.stream.cuda_stream, r.side_stream.cuda_stream
        E.fork_ev, E.join_ev = r._fork_ev.value, r._join_ev.value
        c = E.ctl
        c.parts, c.n, c.entry = self.parts_d.data_ptr(), self.n, 0
        c.jobs, c.segs, c.seg_res, c.stage = r.jobs.d.data_ptr(), r.segs.d.data_ptr(), self.res_ptrs.data_ptr(), \
            r.stage_jobs.d.data_ptr()
        c.off, c.end, c.state, c.first = base + r.o_off, base + r.o_end, base + r.o_state, base + r.o_first
        c.stop, c.pick, c.loff, c.lend = base + r.o_stop, base + r.o_pick, base + r.o_loff, base + r.o_lend
        c.pstall, c.predict_blocks, c.status = self.pstall.data_ptr(), PREDICT_BLOCKS, None
        c.logs, c.log_b0 = self.log_ptrs.data_ptr(), self.log_b0.data_ptr()
        c.sync = self.sync.data_ptr()
        E.n, E.per_batch = self.n, r.s.per_batch
        E.err, E.params, E.batch_base = r.err_all.data_ptr(), ctypes.addressof(r.params), base + r.o_bbase
        E.n_batches_total, E.ev_out, E.nev, E.perm_map = r.ev_total, r.ev_d.data_ptr(), base + r.o_nev, \
            r.perm_all.data_ptr()
        E.long_max_rows, E.long_scratch = 0, r.long_scratch.data_ptr()
        E.dfit_jobs, E.n_dfit, E.max_trees = r.dfit_jobs.d.data_ptr(), self.n, r.s.n_estimators
        mw = max(r.max_wins)
        E.max_W = mw
        E.dfit_max_lf = dfit.max_lf(r.s.per_batch, max(p.X.shape[0] for p in r.parts))
        E.max_pieces = 2 + 64 + r.shuffles[0].window_draws(mw) // 8192
        E.row_order_delta = self.err_rows.data_ptr() - r.err_all.data_ptr()
        E.decouple = 0
        self._E = E
        return E

    def _static_records(self):
        """The record fields that never change over the runner's life (built once)."""
        if getattr(self, "_rec_static", None) is not None:
            return self._rec_static
        r = self.r
        pb = r.s.per_batch
        t = r._templates()
        st = np.zeros(self.n, CTL)
        base_d = self.parts_d.data_ptr()
        idx = np.arange(self.n, dtype=np.uint64)
        stg = st["stage"]
        stg["log"] = [lg.data_ptr() for lg in self.logs]
        stg["log_n"] = base_d + idx * np.uint64(CTL.itemsize) + np.uint64(_OFF["n_log"])
        stg["log_cap"] = [max(1, nb) for nb in r.nbs]
        stg["stall"] = self.pstall.data_ptr() + 4 * idx
        bp = [b.ptrs() for b in r.dfit_bufs]
        st["res"] = [r._sptr("dfit", i) for i in range(self.n)]
        for k, name in enumerate(("dnodes", "droots", "dleaf", "dclasses", "dblob")):
            st[name] = [p[k] for p in bp]
        st["dtrees"] = [b.T for b in r.dfit_bufs]
        st["nb"], st["n_full"], st["base"] = r.nbs, t["stage"]["n_full"], r.bases
        st["max_win"], st["min_win"] = r.max_wins, r.s.min_window
        st["win_rule"] = r.s.win_rule
        st["dpb_x1024"] = int(np.ceil(expected_draws_per_batch(pb) * 1024))
        st["pb"], st["n_words"] = pb, r.n_words
        st["last_len"] = [part.n - (nb - 1) * pb for part, nb in zip(r.parts, r.nbs)]
        st["done"] = 1
        self._rec_static = st
        return st

    def _write_records(self, live):
        """The records of every partition (static templates + the host state of the live ones),
        column by column (the per-partition loop of field stores, _write_records_loop, took
        ~18 us a partition of the phase entry's host time)."""
        r = self.r
        r._stream_ptrs(live)             # refreshes the R / table pointers of regrown stream buffers
        t = r._templates()
        rec = self.rec
        rec[:] = self._static_records()
        ptrs = np.array([sh.ptrs for sh in r.shuffles], dtype=np.uint64).reshape(self.n, 3)
        job = rec["job"]
        job[:] = t["job"]
        job["stop"] = t["stop"]
        job["R"], job["Tpre"], job["Tchunk"] = ptrs[:, 0], ptrs[:, 1], ptrs[:, 2]
        rec["seg"] = t["seg"]
        static_stage = self._static_records()["stage"]
        stg = rec["stage"]
        stg[:] = t["stage"]
        stg["plan_out"] = 0
        stg["next_job"] = 0
        stg["R"] = ptrs[:, 0]
        for name in ("log", "log_n", "log_cap", "stall"):
            stg[name] = static_stage[name]
        rec["long_min_rows"], rec["long_cap_rows"] = self.long_min_rows, self.long_cap_rows
        rec["avail"] = [sh.waited * CHUNK for sh in r.shuffles]
        if live:
            ix = np.array([ps.i for ps in live], dtype=np.int64)
            rec["done"][ix] = 0
            rec["j"][ix] = [ps.j for ps in live]
            rec["P"][ix] = [ps.P for ps in live]
            rec["win"][ix] = [ps.win for ps in live]
            rec["seg_start"][ix] = [ps.seg_start for ps in live]
            rec["state"][ix] = np.concatenate([ps.state[:1] for ps in live])
        for ps in live:
            if ps.retrain:                       # a device refit staged by the last epoch
                _, P1, P2, _ = ps.staged
                q = rec[ps.i]
                q["retrain"], q["P1"], q["P2"] = 1, P1, P2
                q["forest_dev"] = 1
            else:
                f = ps.forest
                if isinstance(f, dfit.DeviceFitForest):
                    rec[ps.i]["forest_dev"] = 1
                else:
                    q = rec[ps.i]
                    d = f.desc
                    s = q["seg"]
                    s["nodes"], s["roots"], s["leaf_value"], s["classes"] = d.nodes, d.roots, d.leaf_value or 0, \
                        d.classes
                    s["n_trees"], s["n_classes"], s["n_nodes"], s["pure"] = d.n_trees, d.n_classes, d.n_nodes, d.pure
                    s["cforest"], s["cf_slots"], s["cf_vote_regs"] = d.cforest or 0, d.cf_slots, d.cf_vote_regs
                    s["cf_leaves"], s["cf_tab_words"] = d.cf_leaves, d.cf_tab_words
                    q["host_slots"] = f.features_read
        if CHECK_RECORDS:
            got = rec.tobytes()
            self._write_records_loop(live)
            if rec.tobytes() != got:
                bad = [n for n in CTL.names if rec[n].tobytes() != np.frombuffer(got, CTL)[n].tobytes()]
                raise AssertionError(f"_write_records differs from the loop form in {bad}")
        # every partition's refit job (the slab's table is rewritten by host epochs)
        r.dfit_jobs.rec[:self.n] = r._templates()["dfit"]

    def _write_records_loop(self, live):
        """The per-partition loop form of _write_records' record fields (DDM_CHECK_RECORDS=1
        compares the two on every phase)."""
        r = self.r
        r._stream_ptrs(live)             # refreshes the R / table pointers of regrown stream buffers
        t = r._templates()
        pb, T = r.s.per_batch, r.s.n_estimators
        rec = self.rec
        rec[:] = np.zeros(1, CTL)
        base_d = self.parts_d.data_ptr()
        nlog = _OFF["n_log"]
        lo = r.s.min_window
        for i, part in enumerate(r.parts):
            q = rec[i]
            q["job"] = t["job"][i]
            q["job"]["stop"] = t["stop"][i]
            q["seg"] = t["seg"][i]
            q["stage"] = t["stage"][i]
            q["stage"]["plan_out"] = 0
            q["stage"]["next_job"] = 0
            q["stage"]["R"] = r.shuffles[i].ptrs[0]
            q["stage"]["log"] = self.logs[i].data_ptr()
            q["stage"]["log_n"] = base_d + i * CTL.itemsize + nlog
            q["stage"]["log_cap"] = max(1, r.nbs[i])
            q["stage"]["stall"] = self.pstall.data_ptr() + 4 * i
            R, Tp, Tc = r.shuffles[i].ptrs
            q["job"]["R"], q["job"]["Tpre"], q["job"]["Tchunk"] = R, Tp, Tc
            b = r.dfit_bufs[i]
            nodes, roots, leaf, classes, blob = b.ptrs()
            q["res"] = r._sptr("dfit", i)
            q["dnodes"], q["droots"], q["dleaf"], q["dclasses"], q["dblob"] = nodes, roots, leaf, classes, blob
            q["dtrees"] = b.T
            q["nb"], q["n_full"], q["base"] = r.nbs[i], t["stage"][i]["n_full"], r.bases[i]
            q["max_win"], q["min_win"] = r.max_wins[i], lo
            q["win_rule"] = r.s.win_rule
            q["long_min_rows"], q["long_cap_rows"] = self.long_min_rows, self.long_cap_rows
            q["dpb_x1024"] = int(np.ceil(expected_draws_per_batch(pb) * 1024))
            q["pb"], q["last_len"], q["n_words"] = pb, part.n - (r.nbs[i] - 1) * pb, r.n_words
            q["done"] = 1
            q["avail"] = r.shuffles[i].waited * CHUNK
        for ps in live:
            q = rec[ps.i]
            q["done"] = 0
            q["j"], q["P"], q["win"], q["seg_start"] = ps.j, ps.P, ps.win, ps.seg_start
            q["state"] = ps.state[0]
            if ps.retrain:                       # a device refit staged by the last epoch
                _, P1, P2, _ = ps.staged
                q["retrain"], q["P1"], q["P2"] = 1, P1, P2
                q["forest_dev"] = 1
            else:
                f = ps.forest
                if isinstance(f, dfit.DeviceFitForest):
                    q["forest_dev"] = 1
                else:
                    d = f.desc
                    s = q["seg"]
                    s["nodes"], s["roots"], s["leaf_value"], s["classes"] = d.nodes, d.roots, d.leaf_value or 0, \
                        d.classes
                    s["n_trees"], s["n_classes"], s["n_nodes"], s["pure"] = d.n_trees, d.n_classes, d.n_nodes, d.pure
                    s["cforest"], s["cf_slots"], s["cf_vote_regs"] = d.cforest or 0, d.cf_slots, d.cf_vote_regs
                    s["cf_leaves"], s["cf_tab_words"] = d.cf_leaves, d.cf_tab_words
                    q["host_slots"] = f.features_read

    def _publish_avail(self, polled=None, upload=True):
        """Stream coverage the generator finished since the last look: the epoch stream waits
        for it (free once done) and the records' avail fields are raised (upload=False: in
        the host records only, before the phase uploads them whole)."""
        r = self.r
        done = {}           # one query per event: a piece's event closes every partition's tables
        for i, sh in enumerate(r.shuffles):
            best = None
            # coverage grows in enqueue order and the events of one stream complete in order:
            # the newest completed event is the best, so look from the newest back
            for cov, ev in reversed(sh.ready):
                if cov <= sh.waited:
                    break
                ok = done.get(id(ev))
                if ok is None:
                    ok = done[id(ev)] = ev.query()
                if ok:
                    best = (cov, ev)
                    break
            if best is None:
                continue
            r.stream.wait_event(best[1])
            sh.waited = best[0]
            if not upload:
                continue
            k = self._avail_k % self.avail_h.numel()
            self._avail_k += 1
            self.avail_h[k] = sh.waited * CHUNK
            at = i * CTL.itemsize + _OFF["avail"]
            with torch.cuda.stream(r.stream):
                self.parts_d[at:at + 8].copy_(self.avail_h[k:k + 1].view(torch.uint8), non_blocking=True)

    def _extend(self, rec):
        """Enqueue generation for partitions whose position nears what is enqueued; False when
        one would outgrow its stream buffers (the host must regrow them outside device mode)."""
        r = self.r
        wants = []
        for i in range(self.n):
            if rec["done"][i] or rec["stall"][i] or rec["park"][i]:
                continue
            sh = r.shuffles[i]
            # the windows of the next groups, but never past the partition's last batch (the
            # draws beyond it would be generated at the end of the run and waited for)
            win = int(min(r.max_wins[i], max(1, int(rec["win"][i])) << (2 * GROUP),
                          max(1, r.nbs[i] - int(rec["j"][i]))))
            need = int(rec["P"][i]) + sh.window_draws(win) + r.n_words + 8 * CHUNK
            need = min(need, sh.cap - 2 * CHUNK)
            if int(rec["P"][i]) + sh.window_draws(1) + r.n_words + 4 * CHUNK > sh.cap - 2 * CHUNK:
                return False
            if sh.chunks_for(need) > sh.tab:
                wants.append((i, need))
        if wants:
            r._ensure_all(wants, wait=False)
        return True

    # ---------------------------------------------------------------- the phase
    def run_phase(self, live):
        """Device epochs until every live partition is done, parked or stalled; then the
        records back into the partitions' host state.  Returns the epochs run."""
        r, st = self.r, self.r.stats
        t0 = time.perf_counter()
        stream = r.stream
        # nothing of the host path may still be in flight: the last epoch's refits are read
        # by the device predict itself
        stream.synchronize()
        r._mark("phase: stream synchronised")
        r._pending_sync = False
        r._pending_forests = []
        E = self._epoch_struct()
        E.long_max_rows = self.long_cap_rows if self.long_ok else 0
        E.ctl.long_ok = 1 if self.long_ok else 0
        timing = r.t_pred is not None
        logging = r.predict_log is not None
        pt = self.pred_timer
        E.ctl.predict_clock = pt.ptr() if pt is not None else None
        # HIP cannot time events that a graph records (hipEventElapsedTime: invalid resource
        # handle), so timed predicts keep the launched form
        use_graph = CTL_GRAPH and pt is None and not (timing or logging)
        # the instrumented (timing / logging) epochs order the streams by HIP events: with
        # flags the joins sit inside the refit's pack and the predict's first workgroup, so
        # the event pairs around those kernels would time the wait for the side stream too
        flags = CTL_FLAGS and self.flags_ok and not use_graph and not (timing or logging)
        E.sync_flags = self.sync_flags.data_ptr() if flags else None
        E.sync_seq = ctypes.addressof(self.sync_seq) if flags else None
        if use_graph:
            # every launch sequence captured while both streams are idle (a capture joins the
            # side stream through the fork event)
            r.side_stream.synchronize()
            for dec in (0, 1):
                E.decouple = dec
                self._graph(E)
        # the rest of the streams in growing pieces, two more at every poll (all of it up
        # front kept the side streams busy past the last epoch: the run waited ~14 ms for
        # generation no epoch needed, C3); the first two only once the first group is
        # enqueued (~0.9 ms of host time the first epochs no longer wait for: their windows
        # are planned within the words already tabulated)
        # the coverage finished so far goes into the records before they go up (it was one
        # 8-byte copy per partition after the upload: ~15 us each at the phase's start)
        self._publish_avail(upload=False)
        self._write_records(live)
        r._mark("phase: records written")
        with torch.cuda.stream(stream):
            self.pstall.zero_()
            self.parts_d.copy_(self.parts_h, non_blocking=True)
            r.dfit_jobs.d[:self.n * dfit.DFIT_DTYPE.itemsize].copy_(
                r.dfit_jobs.h[:self.n * dfit.DFIT_DTYPE.itemsize], non_blocking=True)
        r._mark("phase: records uploaded")
        E.decouple = self._decouple([(ps.win, r.max_wins[ps.i]) for ps in live])
        check(lib.ddm_ctl_enter(ctypes.byref(E)), "ddm_ctl_enter")
        r._mark("device phase entered")
        pending, slot, epochs, group = None, 0, 0, 0
        while True:
            if timing or logging:
                for _ in range(GROUP):
                    self._one_epoch_instrumented(E, timing, logging)
            elif use_graph:
                check(lib.ddm_ctl_graph_launch(self._graph(E), stream.cuda_stream), "ddm_ctl_graph_launch")
            else:
                check(lib.ddm_ctl_epochs(ctypes.byref(E), GROUP), "ddm_ctl_epochs")
            epochs += GROUP
            group += 1
            if group == 1:
                r._enqueue_rest()
            with torch.cuda.stream(stream):
                self.poll_h[slot].copy_(self.parts_d, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(stream)
            if pending is not None:
                pev, pslot = pending
                pev.synchronize()
                rec = self.poll_h[pslot].numpy().view(CTL)
                active = (rec["done"] == 0) & (rec["stall"] == 0) & (rec["park"] == 0)
                if not active.any() or (rec["stall"] != 0).any():
                    r._mark(f"poll: {int(active.sum())} active, {int((rec['stall'] != 0).sum())} stalled")
                    break
                if not self._extend(rec):
                    r._mark("poll: stream buffers would overflow")
                    break
                E.decouple = self._decouple([(int(rec["win"][i]), r.max_wins[i]) for i in np.nonzero(active)[0]])
                r._enqueue_rest()
                self._publish_avail()
            pending = (ev, slot)
            slot ^= 1
        r._mark(f"device loop done ({epochs} epochs enqueued)")
        stream.synchronize()
        r.side_stream.synchronize()
        if pt is not None:
            ms, n = pt.take(stream)
            st.predict_dev_ms += ms
            st.predict_dev_launches += n
        r._mark("device epochs drained")
        st.gpu_s += time.perf_counter() - t0
        if timing:
            p_ms, s_ms, f_ms, sh_ms = self.kernel_times()
            st.predict_ms += p_ms
            st.scan_ms += s_ms
            st.dfit_ms += f_ms
            st.shuffle_ms += sh_ms
        out = self._take_back(live, flags)
        r._mark("records taken back")
        return out

    def _graph(self, E):
        """The captured group for the epochs' current launch sequence (decoupled or not, long
        scans enqueued or not); captured on first use, kept for the runner's life."""
        key = (int(E.decouple), int(E.ctl.long_ok), int(E.long_max_rows))
        g = self.graphs.get(key)
        if g is None:
            g = ctypes.c_void_p()
            E.predict_evs = None
            check(lib.ddm_ctl_graph_create(ctypes.byref(E), GROUP, ctypes.byref(g)), "ddm_ctl_graph_create")
            self.graphs[key] = g
        return g

    def set_flag_limit(self, ticks):
        """The join polls' give-up limit in 10-ns device-clock ticks (sync_flags[3]; 0: the
        default 2 s, which the fork wait always keeps).  Tests force a give-up with a tiny
        limit."""
        self.sync_flags[3] = int(ticks)
        torch.cuda.synchronize(self.r.device)

    def flags_off(self):
        """After a FlagTimeout: fork / join by HIP events from now on (the numbers and the
        give-up count start over should flags be turned back on).  Every stream is drained
        first: a fork poll still queued on the side stream must not see the zeroed numbers."""
        self.flags_ok = False
        torch.cuda.synchronize(self.r.device)
        self.sync_flags[:3].zero_()
        for k in range(3):
            self.sync_seq[k] = 0
        torch.cuda.synchronize(self.r.device)

    def close(self):
        for g in self.graphs.values():
            lib.ddm_ctl_graph_destroy(g)
        self.graphs = {}
        if self.pred_timer is not None:
            self.pred_timer.close()
            self.pred_timer = None

    def _decouple(self, wins):
        """1 when the active partitions' windows ((win, max_win) pairs) average at least
        DECOUPLE_ROWS rows."""
        w = [min(int(a), int(b)) for a, b in wins]
        if not w or not self.decouple_ok:
            return 0
        return int(sum(w) * self.r.s.per_batch >= DECOUPLE_ROWS * len(w))

    def _one_epoch_instrumented(self, E, timing, logging):
        r = self.r
        if timing:
            evs = [ctypes.c_void_p() for _ in range(8)]
            for e in evs:
                check(lib.ddm_event_create(ctypes.byref(e)), "ddm_event_create")
            E.ev[0], E.ev[1], E.ev[2], E.ev[3] = evs[0].value, evs[1].value, evs[2].value, evs[3].value
            E.ev[6], E.ev[7], E.ev[10], E.ev[11] = evs[4].value, evs[5].value, evs[6].value, evs[7].value
            self.timers.append(evs)
        if logging:
            k = len(r.predict_log)
            segs = torch.empty(self.n * kernels.SEG_DTYPE.itemsize, dtype=torch.uint8, device=r.device)
            res = torch.empty(self.n, dtype=torch.int64, device=r.device)
            with torch.cuda.stream(r.stream):
                segs.copy_(r.segs.d[:self.n * kernels.SEG_DTYPE.itemsize], non_blocking=True)
                res.copy_(self.res_ptrs, non_blocking=True)
            r.predict_log.append(("dev", segs, res, k, int(E.decouple)))
        check(lib.ddm_ctl_epochs(ctypes.byref(E), 1), "ddm_ctl_epochs")
        for k in range(12):
            E.ev[k] = None

    def kernel_times(self):
        """(predict, scan, refit, shuffle) ms summed over the timed epochs; clears them."""
        tot = [0.0, 0.0, 0.0, 0.0]
        ms = ctypes.c_float()
        for evs in self.timers:
            for k, (a, b) in enumerate(((0, 1), (2, 3), (4, 5), (6, 7))):
                if lib.ddm_event_elapsed_ms(evs[a], evs[b], ctypes.byref(ms)) == 0:
                    tot[k] += ms.value
            for e in evs:
                lib.ddm_event_destroy(e)
        self.timers = []
        return tot

    def replay(self, entry, stream):
        """One logged device-mode predict launch again, in the form the epoch ran it: row
        order into the decoupled epochs' second buffer, or DDM order through the shuffle (the
        bench's roofline replays)."""
        _, segs, res, _, dec = entry
        if dec:
            check(lib.ddm_forest_predict_dev_orig(segs.data_ptr(), res.data_ptr(), self.n, self.r.s.per_batch,
                                                  PREDICT_BLOCKS, self.pstall.data_ptr(),
                                                  self.err_rows.data_ptr() - self.r.err_all.data_ptr(), None, None, 0,
                                                  None, ctypes.c_void_p(stream.cuda_stream)),
                  "ddm_forest_predict_dev_orig")
        else:
            check(lib.ddm_forest_predict_dev(segs.data_ptr(), res.data_ptr(), self.n, self.r.s.per_batch,
                                             PREDICT_BLOCKS, self.pstall.data_ptr(),
                                             ctypes.c_void_p(stream.cuda_stream), None, None),
                  "ddm_forest_predict_dev")

    def _take_back(self, live, flags=True):
        """Device records -> the partitions' host state (and their events).  `flags`: the
        phase forked / joined by device flags, so their give-up count is read."""
        r, st, pb = self.r, self.r.stats, self.r.s.per_batch
        with torch.cuda.stream(r.stream):
            self.parts_h.copy_(self.parts_d, non_blocking=True)
            r._mark("records copy enqueued")
            r.ctrl_h.copy_(r.ctrl_d, non_blocking=True)        # staging slots and refit results
            r._mark("slab copy enqueued")
            self.sync_h.copy_(self.sync_flags, non_blocking=True)
            r._mark("flags copy enqueued")
        r.stream.synchronize()
        r._mark("records copied")
        if flags and int(self.sync_h[2]):
            raise FlagTimeout(f"{int(self.sync_h[2])} cross-stream flag waits of the device epochs gave up "
                              "(ddm_ctl_epoch.sync_flags): the phase's results are void")
        rec = self.rec
        epochs = int(rec["epochs"].max()) if len(rec) else 0
        # every partition's event log in one read-back
        with torch.cuda.stream(r.stream):
            for ps in live:
                n_log = int(rec[ps.i]["n_log"])
                if n_log:
                    o = int(self.log_off[ps.i])
                    self.logs_h[o:o + 3 * n_log].copy_(self.logs[ps.i][:3 * n_log], non_blocking=True)
        r.stream.synchronize()
        r._mark("logs copied")
        logs_np = self.logs_h.numpy()
        # the records' fields column by column (a field read of a structured scalar costs
        # ~1 us: ~25 of them a partition were ~0.4 ms of a 16-partition phase's end)
        ix = np.array([ps.i for ps in live], dtype=np.int64)
        sub = rec[ix]                    # one gather of the live records, then cheap field views
        col = {name: sub[name].tolist() for name in
               ("n_log", "applied", "done", "predicted_rows", "long_scans", "predict_bytes", "permute_rows",
                "refits", "stall", "j", "P", "win", "seg_start", "retrain", "P1", "P2", "forest_dev")}
        states = sub["state"]
        # every partition's event log parsed at once: (batch, warning pos, change pos) rows
        with_log = [(k, ps) for k, ps in enumerate(live) if col["n_log"][k]]
        if with_log:
            lens = [col["n_log"][k] for k, _ in with_log]
            lg = np.concatenate([logs_np[int(self.log_off[ps.i]):int(self.log_off[ps.i]) + 3 * n]
                                 for (k, ps), n in zip(with_log, lens)]).reshape(-1, 3).astype(np.int64)
            bounds = np.cumsum(lens)[:-1]
            for c in range(2):
                hit = lg[:, 1 + c] >= 0
                rows = np.split(lg[:, 0] - 1, bounds)
                vals = np.split(lg[:, 0] * pb + lg[:, 1 + c], bounds)
                hits = np.split(hit, bounds)
                for (k, ps), r_, v_, h_ in zip(with_log, rows, vals, hits):
                    ps.ev.append((r_[h_], c, v_[h_]))
        r._mark("take-back: events parsed")
        for k, ps in enumerate(live):
            # the last k_ctl may have applied a refit to the window it planned (P after the
            # seeds, batch j already shuffled, a fresh DDM): the host applies it itself in
            # _refit_prep, so it goes back as a pending refit
            applied = bool(col["applied"][k]) and not col["done"][k]
            retrain = col["retrain"][k]
            if applied:
                rec[ps.i]["retrain"] = 1
                retrain = 1
            st.predicted_rows += col["predicted_rows"][k]
            st.device_rows += col["predicted_rows"][k]
            st.long_scans += col["long_scans"][k]
            st.predict_bytes += col["predict_bytes"][k]
            st.device_predict_bytes += col["predict_bytes"][k]
            st.permute_rows += col["permute_rows"][k]
            st.refits += col["refits"][k] - applied
            st.device_refits += col["refits"][k] - applied
            stall = col["stall"][k]
            if stall == kernels.CTL_STALL_REFIT and self._E is not None and self._E.decouple:
                # the row-order predict's smaller LDS (csrc/forest_predict.hip) may be why
                self.decouple_ok = False
            if stall == kernels.CTL_STALL_LONG:          # the next phases enqueue the long scans
                self.long_ok = True
            if stall == kernels.CTL_STALL_SCAN:
                raise RuntimeError(f"ddm_scan_long gave up waiting for a carried state (partition {ps.i}): the "
                                   "epoch's results are void")
            ps.j, ps.P, ps.win, ps.seg_start = col["j"][k], col["P"][k], col["win"][k], col["seg_start"][k]
            ps.state = np.array(states[k:k + 1], dtype=kernels.STATE_DTYPE)
            ps.done = bool(col["done"][k])
            ps.staged = None
            if retrain:
                ps.retrain = True
                if stall == kernels.CTL_STALL_WORDS:
                    # the host path's own staging form: batch d's rows, the words after P
                    L = ps.blen(ps.j - 1)
                    F_i = r.parts[ps.i].X.shape[0]
                    info = r._info_all[ps.i]
                    ps.staged = (r._sview("x", ps.i, np.float32, L * F_i).reshape(L, -1).copy(),
                                 r._sview("y", ps.i, np.int32, L).astype(np.int64),
                                 r._sview("w", ps.i, np.uint32, r.n_words).copy(), None, int(info[4]), int(info[5]))
                else:
                    ps.staged = ("device", col["P1"][k], col["P2"][k], None)
                    r._pending_sync = True         # _finish_pending reads (or redoes) the refit
            else:
                ps.retrain = False
                if col["forest_dev"][k]:
                    res = r._sview("dfit", ps.i, np.int64, dfit.RESULT_WORDS).copy()
                    ps.forest = dfit.DeviceFitForest(r.dfit_bufs[ps.i], res)
            if ps.j >= ps.nb:
                ps.done = True
        r._mark("take-back: partitions")
        st.epochs += epochs
        st.device_epochs += epochs
        st.device_phases += 1
        self.rec["n_log"] = 0
        return epochs
