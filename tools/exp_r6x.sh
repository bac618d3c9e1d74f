#!/bin/bash
# round 6: native per-partition seeding (ddm_mt_seed) and every partition's start state in
# one upload: the shuffle / device-epoch / scaling GPU tests, then c2 / C3 A/B against the
# committed tree (ab_head/)
set -o pipefail
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/r6x && rm -rf gpurun_out/r6x/*
export TMPDIR=/tmp
O=gpurun_out/r6x
cp distributed-drift-detection_amd/ddm_amd/libddm_amd.so ab_head/distributed-drift-detection_amd/ddm_amd/
mkdir -p ab_head/oracle/_build && cp oracle/_build/*.so ab_head/oracle/_build/
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_shuffle.py tests/test_gpu_devctl.py tests/test_gpu_scaling.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
timeout -k 10 300 python -u bench.py --workload c2 --cpu-baseline 0 > $O/c2_$i.json 2> $O/c2_$i.err || { tail -5 $O/c2_$i.err; exit 1; }
(cd ab_head && timeout -k 10 300 python -u bench.py --workload c2 --cpu-baseline 0 > ../$O/c2old_$i.json 2> ../$O/c2old_$i.err) || { tail -5 $O/c2old_$i.err; exit 1; }
timeout -k 10 300 python -u bench.py --cpu-baseline 0 --companion 0 > $O/c3_$i.json 2> $O/c3_$i.err || { tail -5 $O/c3_$i.err; exit 1; }
(cd ab_head && timeout -k 10 300 python -u bench.py --cpu-baseline 0 --companion 0 > ../$O/c3old_$i.json 2> ../$O/c3old_$i.err) || { tail -5 $O/c3old_$i.err; exit 1; }
done
python3 - <<'PY'
import json
for f in ("c2_1", "c2old_1", "c2_2", "c2old_2", "c3_1", "c3old_1", "c3_2", "c3old_2"):
    d = json.loads([l for l in open(f"gpurun_out/r6x/{f}.json") if l.startswith("{")][-1])
    b = d["breakdown"]
    print(f, round(d["ms_per_step"], 2), b["checks"].get("events_sha1"), b["timed_step_ms"], b["timed_step_run_ms"])
PY
echo done
