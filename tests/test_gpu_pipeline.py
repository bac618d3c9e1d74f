"""The whole job minus Spark (DDM_Process.py:38-55, :216-258) on the GPU: csv -> MULT
dup/shuffle -> sort -> partitions -> the hot path -> post-loop record, against the
reference's own events (tests/golden)."""
import numpy as np
import pandas as pd
import pytest

from conftest import load_npz
from test_loader import _outdoor_csv

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("mult,inst", [(2, 4), (4, 16), (2, 1)])
def test_stream_file_matches_reference(tmp_path, mult, inst):
    from ddm_amd.partition import run_stream_file
    path, X, y = _outdoor_csv(tmp_path)
    cfg = load_npz(f"outdoor_cfg_m{mult}_i{inst}.npz")
    events, rec = run_stream_file(path, mult, inst, base_seed=1000, data_seed=123, sort_kind="stable")
    want = np.concatenate([cfg[f"events/{d}"] for d in range(inst) if f"events/{d}" in cfg.files])
    assert np.array_equal(events.to_numpy(), want)
    chg = want[:, 3]
    assert rec["dist_between_changes"] == len(y) * mult // len(np.unique(y))
    assert np.array_equal(rec["distances"]["distance"].to_numpy(), chg[chg != -1] % rec["dist_between_changes"])
    assert rec["total_time"] > 0
