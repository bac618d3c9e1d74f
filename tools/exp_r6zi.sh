#!/bin/bash
# round 6: the window perms kernel on a few strided workgroups per job (DDM_PERM_BLOCKS 8,
# variants 2 / 32) instead of W / 256 (1024 cap, "pbold"): shuffle / device-epoch tests,
# then C3 / C5 / c2 A/B on one box
set -o pipefail
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/r6zi && rm -rf gpurun_out/r6zi/*
export TMPDIR=/tmp
O=gpurun_out/r6zi
V=$PWD/distributed-drift-detection_amd/ddm_amd
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_shuffle.py tests/test_gpu_devctl.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() { # name lib workload extra
  DDM_AMD_LIB=$2 timeout -k 10 300 python -u bench.py --workload $3 --cpu-baseline 0 $4 > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
}
for i in 1 2; do
  run c3_pb8_$i $V/libddm_amd.so c3 "--companion 0"
  run c3_pbold_$i $V/libddm_amd_pbold.so c3 "--companion 0"
done
run c3_pb2 $V/libddm_amd_pb2.so c3 "--companion 0"
run c3_pb32 $V/libddm_amd_pb32.so c3 "--companion 0"
run c5_pb8 $V/libddm_amd.so c5 ""
run c5_pbold $V/libddm_amd_pbold.so c5 ""
for i in 1 2; do
  run c2_pb8_$i $V/libddm_amd.so c2 ""
  run c2_pbold_$i $V/libddm_amd_pbold.so c2 ""
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r6zi/c*.json")):
    d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    b = d["breakdown"]
    print(f.split("/")[-1], round(d["ms_per_step"], 2), round(d["roofline"]["frac"], 3), b["checks"].get("events_sha1"), b["timed_step_ms"])
PY
echo done
