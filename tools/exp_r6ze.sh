#!/bin/bash
# round 6: k_stage_ctl's phases (DDM_STAGE_PROFILE build: device-clock marks printed per
# launch) on a reduced C5 and on C3 -- the kernel on every epoch's critical path
set -o pipefail
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/r6ze && rm -rf gpurun_out/r6ze/*
export TMPDIR=/tmp
O=gpurun_out/r6ze
export DDM_AMD_LIB=$PWD/distributed-drift-detection_amd/ddm_amd/libddm_amd_stageprof.so
timeout -k 10 300 python -u bench.py --workload c5 --c5-rows 4000000 --steps 1 --warmup 0 --cpu-baseline 0 > $O/c5.out 2> $O/c5.err || { tail -5 $O/c5.err; exit 1; }
timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --cpu-baseline 0 --companion 0 > $O/c3.out 2> $O/c3.err || { tail -5 $O/c3.err; exit 1; }
python3 - <<'PY'
import re, statistics
for w in ("c5", "c3"):
    sp, sc = [], []
    for l in open(f"gpurun_out/r6ze/{w}.out"):
        m = re.match(r"stage-prof compact ([\d.]+) gather ([\d.]+) words ([\d.]+) shuffle ([\d.]+) seeds ([\d.]+) swaps ([\d.]+)", l)
        if m: sp.append([float(x) for x in m.groups()])
        m = re.match(r"stage-ctl block (\d+) scan\+pick ([\d.]+) stage ([\d.]+) record ([\d.]+) ticket ([\d.]+) split ([\d.]+)", l)
        if m: sc.append([float(x) for x in m.groups()[1:]])
    if sp:
        print(w, "stage_body (block 0) medians: compact gather words shuffle seeds swaps =", [round(statistics.median(c), 2) for c in zip(*sp)], len(sp))
    if sc:
        print(w, "stage_ctl medians: scan+pick stage record ticket split =", [round(statistics.median(c), 2) for c in zip(*sc)], len(sc))
        print(w, "stage_ctl p90:", [round(sorted(c)[int(0.9 * len(c))], 2) for c in zip(*sc)])
PY
echo done
