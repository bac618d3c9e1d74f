"""Settings of the hot path, mirroring the reference's module constants
(DDM_Process.py:25-35).  Spark knobs (URL, INSTANCES, MEMORY) are not part of the
hot path; `cores` is RandomForestClassifier's n_jobs (DDM_Process.py:102), which
changes speed, not results."""
from dataclasses import dataclass, field
from typing import List, Optional


@dataclass
class DDMSettings:
    per_batch: int = 100                 # PER_BATCH            DDM_Process.py:25
    min_num_instances: int = 3           # MIN_NUM_DDM_VALS     DDM_Process.py:27
    warning_level: float = 0.5           # WARNING_LEVEL        DDM_Process.py:28
    out_control_level: float = 1.5       # CHANGE_LEVEL         DDM_Process.py:29
    n_estimators: int = 100              # RandomForestClassifier default (DDM_Process.py:102)
    cores: int = 1                       # CORES -> n_jobs      DDM_Process.py:8,102
    x_features: Optional[List[str]] = None   # X_features     DDM_Process.py:33-34 (None: '0','1',... present)
    target: str = "target"               # y_true               DDM_Process.py:35
    row_number: str = "full_df_row_number"   # DDM_Process.py:220
    window_batches: int = 256            # first speculative window (batches); doubles while no drift
    max_window_batches: int = 1 << 16
    drift_window_batches: int = 16       # least window after a drift (short concepts: an epoch costs more
                                         # than predicting a few batches past the next drift) ...
    drift_window_short: int = 0          # ... unless the concept was this short.  C5 (64M rows) with the
                                         # floor at 16 / 8 / 4 / 2 for every concept: 4,983 / 4,950 /
                                         # 4,707 / 4,708 ms per step, with short = 3: 4,826; but c2
                                         # 20.1 ms (short 0) / 21.4-21.8 (3) / 21.5 (floor 4): its short
                                         # concepts are followed by long ones, C5's by short ones
    # the window after a drift covers the concept just closed (seg batches) plus
    # max(seg >> drift_window_shift, drift_window_pad) batches: concepts that repeat their
    # length are found in one epoch each, with little predicted past them (a miss doubles)
    drift_window_shift: int = 5
    drift_window_pad: int = 4
    extra: dict = field(default_factory=dict)

    def next_window(self, seg):
        """The window after a change that closed a concept of seg batches, before the
        least-window floor."""
        return seg + max(seg >> self.drift_window_shift, self.drift_window_pad)

    @property
    def min_window(self):
        return max(1, min(self.window_batches, self.drift_window_batches))

    def drift_window(self, seg):
        """The window after a change that closed a concept of seg batches
        (csrc/ctl_dev.h drift_window)."""
        w = self.next_window(seg)
        return w if seg <= self.drift_window_short else max(self.min_window, w)

    @property
    def win_rule(self):
        """drift_window's parameters as the device records carry them."""
        if not (0 <= self.drift_window_shift < 64 and 0 <= self.drift_window_pad < 256
                and 0 <= self.drift_window_short < 32768):
            raise ValueError("drift_window_shift / _pad / _short out of range")
        return (int(self.drift_window_shift) | (int(self.drift_window_pad) << 8)
                | (int(self.drift_window_short) << 16))


SCHEMA = ("warning_flag_local int, warning_flag_global int, change_flag_local int, "
          "change_flag_global int")                                      # DDM_Process.py:167
OUTPUT_COLUMNS = ["warning_flag_local", "warning_flag_global", "change_flag_local", "change_flag_global"]


def infer_x_features(columns):
    """The reference's X_features are '0'..str(F-1) (DDM_Process.py:33-34)."""
    names = set(map(str, columns))
    out = []
    while str(len(out)) in names:
        out.append(str(len(out)))
    if not out:
        raise KeyError("no feature columns named '0', '1', ... (DDM_Process.py:34)")
    return out
