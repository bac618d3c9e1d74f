#!/bin/bash
# Predict parity tests + one C3 bench line + rocprof kernel stats of the C3 bench.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_predict.py tests/test_gpu_controller.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_c3q.log 2>&1 || { tail -40 gpurun_out/pytest_c3q.log; exit 1; }
tail -2 gpurun_out/pytest_c3q.log
timeout -k 10 200 python -u bench.py --cpu-baseline 0 > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || { tail -30 gpurun_out/bench_c3.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_c3.json'));print(d['value'], d['ms_per_step'], d['roofline'])"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3 -o c3 -- python3 bench.py --cpu-baseline 0 > gpurun_out/prof_c3.log 2>&1 || { tail -30 gpurun_out/prof_c3.log; exit 1; }
find gpurun_out/prof_c3 -name '*kernel_stats.csv' -exec grep -h cforest {} \;
