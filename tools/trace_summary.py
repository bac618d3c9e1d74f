"""Summarise a rocprofv3 kernel-trace CSV over the last K runs of a bench (a run starts at a
k_mt_jump burst): per-kernel time, per-stream busy time and the union of GPU-busy time."""
import csv
import sys
from collections import defaultdict


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0][:48]


def union(iv):
    iv.sort()
    tot, cur_s, cur_e = 0, None, None
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main(path, last=2, runs=3):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # one k_stage launch per epoch: the timed runs are the last `last` of `runs` equal runs
    # (warmup first), bounded by the end of the previous run's last k_stage
    st = [i for i, r in enumerate(rows) if "k_stage" in r["Kernel_Name"]]
    per_run = len(st) // runs
    a = st[per_run * (runs - last) - 1] if runs > last else -1
    b = st[-1]
    t0 = int(rows[a]["End_Timestamp"]) if a >= 0 else int(rows[0]["Start_Timestamp"])
    t1 = int(rows[b]["End_Timestamp"])
    sel = [r for r in rows if int(r["Start_Timestamp"]) >= t0 and int(r["End_Timestamp"]) <= t1]
    starts = [0] * runs
    per = defaultdict(lambda: [0, 0])
    streams = defaultdict(list)
    allv = []
    for r in sel:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        k = short(r["Kernel_Name"])
        per[k][0] += 1
        per[k][1] += e - s
        streams[r["Stream_Id"]].append((s, e))
        allv.append((s, e))
    span = (t1 - t0) / 1e6
    print(f"runs found {len(starts)}; last {last}: span {span:.1f} ms, GPU busy (union) {union(allv)/1e6:.1f} ms")
    for sid, iv in sorted(streams.items()):
        print(f"  stream {sid}: {len(iv)} kernels, busy {union(iv)/1e6:.1f} ms")
    for k, (c, t) in sorted(per.items(), key=lambda x: -x[1][1]):
        print(f"  {k:48s} {c:6d} {t/1e6/last:9.2f} ms/run {t/c/1e3:9.1f} us avg")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 2, int(sys.argv[3]) if len(sys.argv) > 3 else 3)
