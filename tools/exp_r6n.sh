#!/bin/bash
# round 6: the stream generation / tables streams on every CU but every k-th
# (DDM_GEN_CU_EXCLUDE=k) so that the epochs beside them find free CUs: C3 (and C5, c2) A/B
set -o pipefail
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/r6n && rm -rf gpurun_out/r6n/*
export TMPDIR=/tmp
O=gpurun_out/r6n
for i in 1 2; do
  for k in 0 2 4 8; do
    DDM_GEN_CU_EXCLUDE=$k timeout -k 10 300 python -u bench.py --cpu-baseline 0 --companion 0 > $O/c3_x${k}_$i.json 2> $O/c3_x${k}_$i.err || { tail -5 $O/c3_x${k}_$i.err; exit 1; }
  done
done
for k in 0 4; do
  DDM_GEN_CU_EXCLUDE=$k timeout -k 10 300 python -u bench.py --workload c3 --solo-world 8 --cpu-baseline 0 --companion 0 > $O/c3s8_x$k.json 2> $O/c3s8_x$k.err || { tail -5 $O/c3s8_x$k.err; exit 1; }
  DDM_GEN_CU_EXCLUDE=$k timeout -k 10 300 python -u bench.py --workload c2 --cpu-baseline 0 > $O/c2_x$k.json 2> $O/c2_x$k.err || { tail -5 $O/c2_x$k.err; exit 1; }
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r6n/c*.json")):
    d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    b = d["breakdown"]
    print(f.split("/")[-1], round(d["ms_per_step"], 2), "frac", round(d["roofline"]["frac"], 3), b["checks"].get("events_sha1"))
PY
echo done
