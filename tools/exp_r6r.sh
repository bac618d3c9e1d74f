#!/bin/bash
# round 6: do CU-masked streams confine their workgroups (tools/cu_probe)? and the
# generation's piece sizes (DDM_GEN_PIECE) on C3
set -o pipefail
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/r6r && rm -rf gpurun_out/r6r/*
export TMPDIR=/tmp
O=gpurun_out/r6r
timeout -k 10 60 tools/cu_probe > $O/cu_probe.txt 2>&1 || { cat $O/cu_probe.txt; exit 1; }
cat $O/cu_probe.txt
for p in 25 23 24 22; do
DDM_GEN_PIECE=$((1 << p)) timeout -k 10 300 python -u bench.py --cpu-baseline 0 --companion 0 > $O/c3_p$p.json 2> $O/c3_p$p.err || { tail -5 $O/c3_p$p.err; exit 1; }
done
python3 - <<'PY'
import json
for p in (25, 23, 24, 22):
    d = json.loads([l for l in open(f"gpurun_out/r6r/c3_p{p}.json") if l.startswith("{")][-1])
    b = d["breakdown"]
    print(p, round(d["ms_per_step"], 2), round(d["roofline"]["frac"], 3), b["checks"].get("events_sha1"), b["timed_step_ms"])
PY
echo done
