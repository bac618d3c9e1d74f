#!/bin/bash
# Scan parity tests + C4 bench sweep + rocprof kernel stats of the C4 bench.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_scan_batches.py tests/test_gpu_scan.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_scan.log 2>&1 || { tail -40 gpurun_out/pytest_scan.log; exit 1; }
tail -3 gpurun_out/pytest_scan.log
for cfg in DDM_SCAN_POP=8 DDM_SCAN_POP=1 DDM_SCAN_POP=16 DDM_SCAN_POP=24; do
  env $cfg timeout -k 10 120 python -u bench.py --workload c4 --cpu-baseline 0 --steps 5 > gpurun_out/c4_sweep.json 2> gpurun_out/c4_sweep.err || { tail -20 gpurun_out/c4_sweep.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/c4_sweep.json'));print('$cfg', d['value'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4 -o c4 -- python3 bench.py --workload c4 --cpu-baseline 0 > gpurun_out/prof_c4.log 2>&1 || { tail -30 gpurun_out/prof_c4.log; exit 1; }
find gpurun_out/prof_c4 -name '*kernel_stats.csv' -exec grep scan {} \;
