"""Intervals between consecutive epochs' predict launches in a rocprofv3 kernel trace, per
run (a gap > 1.5 ms between launches separates runs): where the first epochs wait for stream
pieces (round 6, the C3 share at N = 8).
    python tools/epoch_gaps.py gpurun_out/.../s8_kernel_trace.csv"""
import csv
import sys

import numpy as np

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
t = np.array([int(r["Start_Timestamp"]) for r in rows if "k_cforest_predict_dev" in r["Kernel_Name"]]) / 1e3
runs, cur = [], [t[0]]
for a, b in zip(t, t[1:]):
    if b - a > 1_500:
        runs.append(cur)
        cur = []
    cur.append(b)
runs.append(cur)
for k, r in enumerate(runs):
    d = np.diff(r)
    if len(d) < 10:
        continue
    head = d[:20]
    print(f"run {k}: {len(r)} epochs over {(r[-1] - r[0]) / 1e3:.2f} ms; first 20 gaps sum {head.sum() / 1e3:.2f} ms "
          f"(max {head.max():.0f} us); later gaps median {np.median(d[20:]):.0f} us")
