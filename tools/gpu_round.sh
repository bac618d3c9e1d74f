#!/bin/bash
# Scan + predict parity tests, C4 bench with/without the prefix table, C3 bench, rocprof stats of both.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_scan_batches.py tests/test_gpu_scan.py tests/test_gpu_predict.py tests/test_gpu_controller.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_round.log 2>&1 || { tail -40 gpurun_out/pytest_round.log; exit 1; }
tail -2 gpurun_out/pytest_round.log
for cfg in DDM_X=0 DDM_FIX_OPEN=8 DDM_FIX_OPEN=32 DDM_FIX_REFILL=8 DDM_FIX_REFILL=32 DDM_FIX_BLOCKS=256 DDM_SCAN_FILL=128; do
  env $cfg timeout -k 10 120 python -u bench.py --workload c4 --cpu-baseline 0 --steps 5 > gpurun_out/c4_sweep.json 2> gpurun_out/c4_sweep.err || { tail -20 gpurun_out/c4_sweep.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/c4_sweep.json'));print('$cfg', d['value'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
done
timeout -k 10 200 python -u bench.py --cpu-baseline 0 > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || { tail -30 gpurun_out/bench_c3.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_c3.json'));print(d['value'], d['ms_per_step'], d['roofline'])"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4 -o c4 -- python3 bench.py --workload c4 --cpu-baseline 0 > gpurun_out/prof_c4.log 2>&1 || { tail -30 gpurun_out/prof_c4.log; exit 1; }
find gpurun_out/prof_c4 -name '*kernel_stats.csv' -exec grep -h scan {} \;
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3 -o c3 -- python3 bench.py --cpu-baseline 0 > gpurun_out/prof_c3.log 2>&1 || { tail -30 gpurun_out/prof_c3.log; exit 1; }
find gpurun_out/prof_c3 -name '*kernel_stats.csv' -exec grep -h cforest {} \;
