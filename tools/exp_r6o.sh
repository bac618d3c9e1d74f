#!/bin/bash
# round 6: the stream generation's per-kind times and bytes in the C3 / C3 solo-8 breakdown
set -o pipefail
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/r6o && rm -rf gpurun_out/r6o/*
export TMPDIR=/tmp
O=gpurun_out/r6o
timeout -k 10 300 python -u bench.py --cpu-baseline 0 --companion 0 > $O/c3.json 2> $O/c3.err || { tail -5 $O/c3.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload c3 --solo-world 8 --cpu-baseline 0 --companion 0 > $O/c3s8.json 2> $O/c3s8.err || { tail -5 $O/c3s8.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload c5 --cpu-baseline 0 > $O/c5.json 2> $O/c5.err || { tail -5 $O/c5.err; exit 1; }
python3 - <<'PY'
import json
for f in ("c3", "c3s8", "c5"):
    d = json.loads([l for l in open(f"gpurun_out/r6o/{f}.json") if l.startswith("{")][-1])
    b = d["breakdown"]
    print(f, round(d["ms_per_step"], 2), b["checks"].get("events_sha1"), json.dumps(b["stream_generation"]))
PY
echo done
