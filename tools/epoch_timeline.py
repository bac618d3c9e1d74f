"""Per-epoch kernel timeline of a device-resident run from a rocprofv3 kernel trace:
median start / end of each kernel relative to the epoch's predict launch (developer tool).
    python tools/epoch_timeline.py gpurun_out/prof_c3/c3_kernel_trace.csv"""
import csv
import statistics
import sys

KERNELS = ["k_cforest_predict_dev", "k_err_permute", "k_scan_fast", "k_scan_long", "k_pick_batch", "k_stage_ctl", "k_stage", "k_ctl",
           "k_fsm_first_batch", "k_fsm_walk_batch", "k_fsm_replay_batch", "k_fsm_perms_batch", "k_dfit_prep",
           "k_dfit_trees", "k_dfit_pack"]


def short(name):
    for k in KERNELS:
        if k in name:
            return k
    return None


rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
ev = [(short(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
ev = [e for e in ev if e[0]]
idx = [i for i, e in enumerate(ev) if e[0] == "k_cforest_predict_dev"]
# epochs: a predict followed by a scan (k_scan_fast, or the fused k_stage_ctl that runs it)
# before the next predict (the bench's back-to-back roofline replays are not epochs)
idx = [a for a, b in zip(idx, idx[1:] + [len(ev)]) if any(n in ("k_scan_fast", "k_stage_ctl") for n, _, _ in ev[a:b])]
lo, hi = len(idx) // 3, 2 * len(idx) // 3          # the middle third (steady epochs)
spans = []
for a, b in zip(idx[lo:hi], idx[lo + 1:hi + 1]):
    t0 = ev[a][1]
    d = {}
    for n, s, e in ev[a:b]:
        d.setdefault(n, (s - t0, e - t0))
    spans.append(d)
for k in KERNELS:
    st = [d[k][0] / 1e3 for d in spans if k in d]
    en = [d[k][1] / 1e3 for d in spans if k in d]
    if st:
        print(f"{k:24s} start {statistics.median(st):8.1f} us   end {statistics.median(en):8.1f} us")
per = [(ev[b][1] - ev[a][1]) / 1e3 for a, b in zip(idx[lo:hi], idx[lo + 1:hi + 1])]
print(f"epoch period: median {statistics.median(per):.1f} us over {len(per)} epochs")
