#!/bin/bash
# round 6: the run start's head words gathered on the device and copied once: controller /
# shuffle / device-epoch GPU tests, then c2 / C3 A/B against ab_head/
set -o pipefail
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/r6zj && rm -rf gpurun_out/r6zj/*
export TMPDIR=/tmp
O=gpurun_out/r6zj
mkdir -p ab_head/oracle/_build && cp oracle/_build/*.so ab_head/oracle/_build/
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_controller.py tests/test_gpu_shuffle.py tests/test_gpu_devctl.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do
timeout -k 10 300 python -u bench.py --workload c2 --cpu-baseline 0 > $O/c2_$i.json 2> $O/c2_$i.err || { tail -5 $O/c2_$i.err; exit 1; }
(cd ab_head && timeout -k 10 300 python -u bench.py --workload c2 --cpu-baseline 0 > ../$O/c2old_$i.json 2> ../$O/c2old_$i.err) || { tail -5 $O/c2old_$i.err; exit 1; }
done
timeout -k 10 300 python -u bench.py --cpu-baseline 0 --companion 0 > $O/c3.json 2> $O/c3.err || { tail -5 $O/c3.err; exit 1; }
python3 - <<'PY'
import json
for f in ("c2_1", "c2old_1", "c2_2", "c2old_2", "c2_3", "c2old_3", "c3"):
    d = json.loads([l for l in open(f"gpurun_out/r6zj/{f}.json") if l.startswith("{")][-1])
    b = d["breakdown"]
    print(f, round(d["ms_per_step"], 2), b["checks"].get("events_sha1"), b["timed_step_ms"])
PY
echo done
