#!/bin/bash
# staging parity, then k_stage kernel times at N=1 for each DDM_STAGE_SPREAD value
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_controller.py tests/test_gpu_configs.py tests/test_gpu_pipeline.py tests/test_gpu_dfit.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pt_spread.log 2>&1 || { tail -30 gpurun_out/pt_spread.log; exit 1; }
tail -1 gpurun_out/pt_spread.log
for sp in "$@"; do
  rm -rf gpurun_out/prof_spread
  DDM_STAGE_SPREAD=$sp DDM_DFIT_SPREAD=$sp timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_spread -o c3 -- python3 bench.py --cpu-baseline 0 --steps 3 > gpurun_out/prof_spread.log 2>&1 || { tail -30 gpurun_out/prof_spread.log; exit 1; }
  python3 -c "
import csv, json
for r in csv.DictReader(open('gpurun_out/prof_spread/c3_kernel_stats.csv')):
    if 'k_stage' in r['Name'] or 'dfit' in r['Name']: print('spread $sp', r['Name'].split('(')[2][-14:], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us avg')
"
done
