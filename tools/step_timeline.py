"""One run's first milliseconds: every kernel (queue, name, span) and the host marks of
bench.py's DDM_HOST_TRACE_OUT, on one clock (the kernel trace's ns and the marks'
CLOCK_MONOTONIC perf_counter) -- what the first epochs of a step wait for (round 6).
    python tools/step_timeline.py <kernel_trace.csv> <host trace file> [ms]"""
import csv
import json
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
ht = json.load(open(sys.argv[2]))
span_ms = float(sys.argv[3]) if len(sys.argv) > 3 else 20.0
t0 = ht["t_run"] * 1e9
ev = []
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if t0 <= s <= t0 + span_ms * 1e6:
        m = re.search(r"(k_[a-z_0-9]+|elementwise|copyBuffer|fillBuffer)", r["Kernel_Name"])
        ev.append(((s - t0) / 1e3, f"{(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  q{r['Queue_Id']:>2} "
                   f"{m.group(1) if m else r['Kernel_Name'][:30]}"))
for label, t in ht["marks"]:
    if t * 1e3 <= span_ms:
        ev.append((t * 1e6, f"{'':9} {'':8}  HOST {label}"))
for t, txt in sorted(ev):
    if "copyBuffer" in txt:
        continue
    print(f"{t:9.1f} {txt}")
