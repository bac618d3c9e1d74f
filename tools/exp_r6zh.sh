#!/bin/bash
# round 6: MT untempering in uint32 arithmetic (the run end's numpy states): the controller,
# device-epoch, shuffle, config and scaling GPU tests, then c2 / C3 lines
set -o pipefail
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/r6zh && rm -rf gpurun_out/r6zh/*
export TMPDIR=/tmp
O=gpurun_out/r6zh
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_controller.py tests/test_gpu_devctl.py tests/test_gpu_shuffle.py tests/test_gpu_configs.py tests/test_gpu_scaling.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for w in c2 c3; do
timeout -k 10 300 python -u bench.py --workload $w --cpu-baseline 0 --companion 0 > $O/$w.json 2> $O/$w.err || { tail -5 $O/$w.err; exit 1; }
done
python3 - <<'PY'
import json
for f in ("c2", "c3"):
    d = json.loads([l for l in open(f"gpurun_out/r6zh/{f}.json") if l.startswith("{")][-1])
    b = d["breakdown"]
    print(f, round(d["ms_per_step"], 2), b["checks"].get("events_sha1"), b["timed_step_ms"])
PY
echo done
