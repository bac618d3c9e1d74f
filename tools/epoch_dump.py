"""Every kernel of a few steady epochs of a device-resident run, in start order, from a
rocprofv3 kernel trace (developer tool):
    python tools/epoch_dump.py <kernel_trace.csv> [n_epochs]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
n_show = int(sys.argv[2]) if len(sys.argv) > 2 else 2
pred = [i for i, r in enumerate(rows) if "k_cforest_predict_dev" in r["Kernel_Name"]]
mid = len(pred) // 2
for a, b in zip(pred[mid:mid + n_show], pred[mid + 1:mid + 1 + n_show]):
    t0 = int(rows[a]["Start_Timestamp"])
    print(f"--- epoch at {t0}")
    for r in rows[a:b]:
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        q = r.get("Queue_Id") or r.get("Stream_Id") or ""
        print(f"{name[:40]:40s} q{q:>3s} {(int(r['Start_Timestamp']) - t0) / 1e3:9.1f} {(int(r['End_Timestamp']) - t0) / 1e3:9.1f}"
              f"  grid {r.get('Grid_Size', r.get('Grid_Size_X', ''))}")
