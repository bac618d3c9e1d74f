#!/bin/bash
# round 6: prefix tables at 24 chunks per workgroup for large launches (vs the committed 8),
# then the pieces enqueued before the first epoch (DDM_EARLY_PIECES) on C3
set -o pipefail
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/r6u && rm -rf gpurun_out/r6u/*
export TMPDIR=/tmp
O=gpurun_out/r6u
OLD=$PWD/distributed-drift-detection_amd/ddm_amd/libddm_amd_head.so
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_shuffle.py > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
DDM_AMD_LIB=$OLD timeout -k 10 120 python -u tools/gen_time.py > $O/gen_old.json 2> $O/gen_old.err || { tail -5 $O/gen_old.err; exit 1; }
timeout -k 10 120 python -u tools/gen_time.py > $O/gen_new.json 2> $O/gen_new.err || { tail -5 $O/gen_new.err; exit 1; }
cat $O/gen_old.json $O/gen_new.json
for i in 1 2; do
timeout -k 10 300 python -u bench.py --cpu-baseline 0 --companion 0 > $O/c3_$i.json 2> $O/c3_$i.err || { tail -5 $O/c3_$i.err; exit 1; }
DDM_AMD_LIB=$OLD timeout -k 10 300 python -u bench.py --cpu-baseline 0 --companion 0 > $O/c3old_$i.json 2> $O/c3old_$i.err || { tail -5 $O/c3old_$i.err; exit 1; }
done
for e in 2 3; do
DDM_EARLY_PIECES=$e timeout -k 10 300 python -u bench.py --cpu-baseline 0 --companion 0 > $O/c3_e$e.json 2> $O/c3_e$e.err || { tail -5 $O/c3_e$e.err; exit 1; }
done
timeout -k 10 300 python -u bench.py --workload c3 --solo-world 8 --cpu-baseline 0 --companion 0 > $O/c3s8.json 2> $O/c3s8.err || { tail -5 $O/c3s8.err; exit 1; }
python3 - <<'PY'
import json
for f in ("c3_1", "c3old_1", "c3_2", "c3old_2", "c3_e2", "c3_e3", "c3s8"):
    d = json.loads([l for l in open(f"gpurun_out/r6u/{f}.json") if l.startswith("{")][-1])
    b = d["breakdown"]
    g = b["stream_generation"]
    print(f, round(d["ms_per_step"], 2), round(d["roofline"]["frac"], 3), b["checks"].get("events_sha1"), b["timed_step_ms"],
          "tables", g["tables"]["ms"], g["tables"]["GB_per_s"], "jump", g["jump"]["ms"], "gen", g["generate"]["ms"])
PY
echo done
