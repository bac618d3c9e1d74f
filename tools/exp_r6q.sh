#!/bin/bash
# round 6: k_fsm_perms one wave per workgroup, J row staged in LDS by dword loads (vs the
# 256-thread byte-load kernel), with the full -m gpu suite on the new tree
set -o pipefail
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/r6q && rm -rf gpurun_out/r6q/*
export TMPDIR=/tmp
O=gpurun_out/r6q
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
OLD=$PWD/distributed-drift-detection_amd/ddm_amd/libddm_amd_oldperms.so
for i in 1 2; do
timeout -k 10 300 python -u bench.py --cpu-baseline 0 --companion 0 > $O/c3_$i.json 2> $O/c3_$i.err || { tail -5 $O/c3_$i.err; exit 1; }
DDM_AMD_LIB=$OLD timeout -k 10 300 python -u bench.py --cpu-baseline 0 --companion 0 > $O/c3old_$i.json 2> $O/c3old_$i.err || { tail -5 $O/c3old_$i.err; exit 1; }
done
timeout -k 10 300 python -u bench.py --workload c2 --cpu-baseline 0 > $O/c2.json 2> $O/c2.err || { tail -5 $O/c2.err; exit 1; }
DDM_AMD_LIB=$OLD timeout -k 10 300 python -u bench.py --workload c2 --cpu-baseline 0 > $O/c2old.json 2> $O/c2old.err || { tail -5 $O/c2old.err; exit 1; }
python3 - <<'PY'
import json
for f in ("c3_1", "c3old_1", "c3_2", "c3old_2", "c2", "c2old"):
    d = json.loads([l for l in open(f"gpurun_out/r6q/{f}.json") if l.startswith("{")][-1])
    b = d["breakdown"]
    print(f, round(d["ms_per_step"], 2), round(d["roofline"]["frac"], 3), b["checks"].get("events_sha1"), round(b["shuffle_kernels_ms_per_step"], 2))
PY
echo done
