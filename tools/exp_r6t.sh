#!/bin/bash
# round 6: pieces enqueued before the first epoch (DDM_EARLY_PIECES) on C3, with host marks
set -o pipefail
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/r6t && rm -rf gpurun_out/r6t/*
export TMPDIR=/tmp
O=gpurun_out/r6t
for i in 1 2; do
for e in 1 2 3 4; do
DDM_EARLY_PIECES=$e DDM_HOST_TRACE=1 DDM_HOST_TRACE_OUT=$O/ht_e${e}_$i timeout -k 10 300 python -u bench.py --cpu-baseline 0 --companion 0 > $O/c3_e${e}_$i.json 2> $O/c3_e${e}_$i.err || { tail -5 $O/c3_e${e}_$i.err; exit 1; }
done
done
python3 - <<'PY'
import json
for i in (1, 2):
    for e in (1, 2, 3, 4):
        d = json.loads([l for l in open(f"gpurun_out/r6t/c3_e{e}_{i}.json") if l.startswith("{")][-1])
        b = d["breakdown"]
        print(e, i, round(d["ms_per_step"], 2), round(d["roofline"]["frac"], 3), b["checks"].get("events_sha1"), b["timed_step_ms"])
PY
echo done
