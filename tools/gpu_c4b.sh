#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_scan_batches.py tests/test_gpu_scan.py -x -q --timeout 250 --timeout-method thread > gpurun_out/pytest_c4.log 2>&1 || { tail -30 gpurun_out/pytest_c4.log; exit 1; }
tail -1 gpurun_out/pytest_c4.log
run() { timeout -k 10 200 env "$@" python -u bench.py --workload c4 --steps 5 --warmup 2 --cpu-baseline 0 > gpurun_out/c4v.json 2> gpurun_out/c4v.err || { tail -5 gpurun_out/c4v.err; exit 1; }; python -c "import json;d=json.load(open('gpurun_out/c4v.json'));print('$*', round(d['roofline']['avg_launch_ms'],3), d['breakdown']['changes_per_step'])"; }
run X=1
run DDM_SCAN_WAVES=5120
run DDM_SCAN_WAVES=6144
run DDM_SCAN_WAVES=5120 DDM_FIX_BLOCKS=1024
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4 -o c4 -- python3 bench.py --workload c4 --steps 5 --warmup 2 --cpu-baseline 0 > gpurun_out/c4.json 2> gpurun_out/c4.err || { tail -20 gpurun_out/c4.err; exit 1; }
python -c "
import csv
for r in list(csv.DictReader(open('gpurun_out/prof_c4/c4_kernel_stats.csv')))[:5]: print(r['Name'][:50], r['Calls'], r['AverageNs'])"
