"""Oracle DDM (test infrastructure only — see oracle/__init__.py).

Restates scikit-multiflow's DDM as the reference instantiates it at
DDM_Process.py:139 (`DDM(min_num_instances=3, warning_level=0.5,
out_control_level=1.5)`, constants at DDM_Process.py:27-29), and the per-batch
event scan of `run_DDM` (DDM_Process.py:135-159).  Arithmetic is plain IEEE
double with no fused multiply-add, exactly what numpy scalar ops do.
"""
import math

import numpy as np

MIN_NUM_DDM_VALS = 3      # DDM_Process.py:27
WARNING_LEVEL = 0.5       # DDM_Process.py:28
CHANGE_LEVEL = 1.5        # DDM_Process.py:29
PER_BATCH = 100           # DDM_Process.py:25


class OracleDDM:
    """State machine of skmultiflow DDM (field names follow upstream)."""

    __slots__ = ("min_instances", "warning_level", "out_control_level", "sample_count", "miss_prob",
                 "miss_std", "miss_prob_sd_min", "miss_prob_min", "miss_sd_min", "in_concept_change",
                 "in_warning_zone")

    def __init__(self, min_instances=MIN_NUM_DDM_VALS, warning_level=WARNING_LEVEL,
                 out_control_level=CHANGE_LEVEL):
        self.min_instances = min_instances
        self.warning_level = float(warning_level)
        self.out_control_level = float(out_control_level)
        self.reset()

    def reset(self):
        self.sample_count = 1
        self.miss_prob = 1.0
        self.miss_std = 0.0
        self.miss_prob_sd_min = math.inf
        self.miss_prob_min = math.inf
        self.miss_sd_min = math.inf
        self.in_concept_change = False
        self.in_warning_zone = False

    def add(self, x):
        if self.in_concept_change:
            self.reset()
        n = float(self.sample_count)
        p = self.miss_prob + (float(x) - self.miss_prob) / n
        s = math.sqrt(p * (1.0 - p) / n)
        self.miss_prob, self.miss_std = p, s
        self.sample_count += 1
        self.in_concept_change = False
        self.in_warning_zone = False
        if self.sample_count < self.min_instances:
            return
        ps = p + s
        if ps <= self.miss_prob_sd_min:
            self.miss_prob_min, self.miss_sd_min, self.miss_prob_sd_min = p, s, ps
        if ps > self.miss_prob_min + self.out_control_level * self.miss_sd_min:
            self.in_concept_change = True
        elif ps > self.miss_prob_min + self.warning_level * self.miss_sd_min:
            self.in_warning_zone = True

    def state_tuple(self):
        return (self.miss_prob, self.miss_std, self.miss_prob_min, self.miss_sd_min,
                self.miss_prob_sd_min, self.sample_count, int(self.in_concept_change),
                int(self.in_warning_zone))


def scan_batch(err, ddm):
    """run_DDM on one batch (DDM_Process.py:141-152): first warning, first change + break.

    Returns (warn_pos, change_pos) as positions inside the batch (-1 = none)."""
    warn = -1
    for q, x in enumerate(err):
        ddm.add(int(x))
        if ddm.in_warning_zone and warn == -1:
            warn = q
        if ddm.in_concept_change:
            return warn, q
    return warn, -1


def scan_stream(err, per_batch=PER_BATCH, mode="stop", ddm=None, trace=False,
                min_instances=MIN_NUM_DDM_VALS, warning_level=WARNING_LEVEL,
                change_level=CHANGE_LEVEL):
    """DDM over consecutive batches of one error stream (the loop DDM_Process.py:189-210
    with the classifier factored out).

    mode "stop":    stop after the first batch with a change (controller mode: the model
                    is refit, so later errors change).
    mode "restart": drop the DDM after a change and start a fresh one at the next batch
                    (DDM_Process.py:207-210 with a fixed error stream).
    Returns events int32 [n_batches, 2] (-1 filled past a stop), stop batch (-1 if none),
    the final DDM and, if trace, p/s per processed row (NaN elsewhere)."""
    err = np.asarray(err, dtype=np.uint8)
    n = len(err)
    nb = (n + per_batch - 1) // per_batch
    ev = np.full((nb, 2), -1, dtype=np.int32)
    ps = np.full((n, 2), np.nan) if trace else None
    if ddm is None:
        ddm = OracleDDM(min_instances, warning_level, change_level)
    stop = -1
    for b in range(nb):
        lo, hi = b * per_batch, min(n, (b + 1) * per_batch)
        warn = chg = -1
        for q in range(hi - lo):
            ddm.add(int(err[lo + q]))
            if ps is not None:
                ps[lo + q] = (ddm.miss_prob, ddm.miss_std)
            if ddm.in_warning_zone and warn == -1:
                warn = q
            if ddm.in_concept_change:
                chg = q
                break
        ev[b] = (warn, chg)
        if chg >= 0:
            if mode == "stop":
                stop = b
                break
            ddm = OracleDDM(min_instances, warning_level, change_level)
    return ev, stop, ddm, ps
