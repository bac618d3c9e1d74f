#!/bin/bash
# Round 2: ddm_scan_long parity + timing, predict vec variant, regressions after the stage rewrite.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 250 --timeout-method thread > gpurun_out/pytest_dist.log 2>&1 || { tail -60 gpurun_out/pytest_dist.log; exit 1; }
tail -3 gpurun_out/pytest_dist.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_scan_long.py -x -v -s --timeout 200 --timeout-method thread > gpurun_out/pytest_long.log 2>&1 || { tail -80 gpurun_out/pytest_long.log; exit 1; }
grep -E "PASS|FAIL|carried segment" gpurun_out/pytest_long.log | tail -30
timeout -k 10 600 python -u -m pytest tests/test_gpu_predict.py tests/test_gpu_scan.py tests/test_gpu_scan_batches.py tests/test_gpu_controller.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_scan.log 2>&1 || { tail -40 gpurun_out/pytest_scan.log; exit 1; }
tail -2 gpurun_out/pytest_scan.log
for v in 1 0; do
DDM_PREDICT_VEC=$v timeout -k 10 200 python -u bench.py --oracle-check-rows 0 --cpu-baseline 0 > gpurun_out/c3_vec$v.json 2> gpurun_out/c3_vec$v.err || { tail -30 gpurun_out/c3_vec$v.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/c3_vec$v.json'));b=d['breakdown'];r=d['roofline'];print('vec$v', d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac'], r['avg_launch_ms_in_step'])"
done
timeout -k 10 200 python -u bench.py --solo-world 8 --oracle-check-rows 0 > gpurun_out/c3_solo8.json 2> gpurun_out/c3_solo8.err || { tail -30 gpurun_out/c3_solo8.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/c3_solo8.json'));b=d['breakdown'];print('solo8', d['value'], d['ms_per_step'], b['epochs_per_step'])"
