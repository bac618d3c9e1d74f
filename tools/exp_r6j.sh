#!/bin/bash
# round 6: the predict's slot rank over m + 1 compares (NaN aliased in the table) -- predict /
# refit parity, C3 A/B against the padded sweep (libddm_amd_fpold.so) with the isolated
# replay; where the C3 per-GPU share goes at N = 8 (--solo-world 8): bench line + kernel trace
set -o pipefail
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/r6j && rm -rf gpurun_out/r6j/*
export TMPDIR=/tmp
O=gpurun_out/r6j
L=$PWD/distributed-drift-detection_amd/ddm_amd
timeout -k 10 900 python -u -m pytest tests/test_gpu_predict.py tests/test_gpu_dfit.py tests/test_gpu_pipeline.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --cpu-baseline 0 --companion 0 > $O/c3_new_$i.json 2> $O/c3_new_$i.err || { tail -5 $O/c3_new_$i.err; exit 1; }
  DDM_AMD_LIB=$L/libddm_amd_fpold.so timeout -k 10 300 python -u bench.py --cpu-baseline 0 --companion 0 > $O/c3_old_$i.json 2> $O/c3_old_$i.err || { tail -5 $O/c3_old_$i.err; exit 1; }
done
timeout -k 10 300 python -u bench.py --workload c3 --solo-world 8 --cpu-baseline 0 --companion 0 > $O/c3_s8.json 2> $O/c3_s8.err || { tail -5 $O/c3_s8.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_s8 -o s8 -- python3 bench.py --workload c3 --solo-world 8 --cpu-baseline 0 --companion 0 --steps 2 --warmup 1 > $O/tr_s8_line.json 2> $O/tr_s8.err || exit 1
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r6j/c3_*.json")):
    d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    b = d["breakdown"]; r = d["roofline"]
    print(f.split("/")[-1], round(d["ms_per_step"], 2), "frac", round(r["frac"], 3),
          "iso", round((r.get("isolated_replay") or {}).get("frac") or 0, 3), "epochs", b["epochs_per_step"],
          "shuffle", round(b["shuffle_kernels_ms_per_step"], 2), "predict", round(b["predict_kernel_ms_per_step"], 2),
          "refit", round(b["device_refit_kernels_ms_per_step"], 2), b["checks"].get("events_sha1"))
PY
echo done
