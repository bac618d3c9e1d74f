#!/bin/bash
# round 6: stream pieces sized by the partitions on the GPU -- per-GPU shares of C3 / C5 at
# N = 2 / 4 / 8 (--solo-world) and N = 1, the N > 1 tests (events equal at every N)
set -o pipefail
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/r6k && rm -rf gpurun_out/r6k/*
export TMPDIR=/tmp
O=gpurun_out/r6k
for n in 8 4 2; do
  timeout -k 10 300 python -u bench.py --workload c3 --solo-world $n --cpu-baseline 0 --companion 0 > $O/c3_s$n.json 2> $O/c3_s$n.err || { tail -5 $O/c3_s$n.err; exit 1; }
done
timeout -k 10 300 python -u bench.py --workload c3 --cpu-baseline 0 --companion 0 > $O/c3_s1.json 2> $O/c3_s1.err || { tail -5 $O/c3_s1.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload c5 --solo-world 8 --cpu-baseline 0 --companion 0 > $O/c5_s8.json 2> $O/c5_s8.err || { tail -5 $O/c5_s8.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload c2 --solo-world 8 --cpu-baseline 0 --companion 0 > $O/c2_s8.json 2> $O/c2_s8.err || { tail -5 $O/c2_s8.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_s8 -o s8 -- python3 bench.py --workload c3 --solo-world 8 --cpu-baseline 0 --companion 0 --steps 2 --warmup 1 > $O/tr_s8_line.json 2> $O/tr_s8.err || exit 1
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r6k/c*_s*.json")):
    d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    b = d["breakdown"]
    print(f.split("/")[-1], round(d["ms_per_step"], 2), "epochs", b["epochs_per_step"],
          "shuffle", round(b["shuffle_kernels_ms_per_step"], 2), b["checks"].get("events_sha1"))
PY
timeout -k 10 900 python -u -m pytest tests/test_gpu_scaling.py tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
echo done
