#!/bin/bash
# predict parity, then the c3 bench line (roofline of the predict kernel) and its rocprof kernel stats
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_predict.py tests/test_gpu_controller.py tests/test_gpu_pipeline.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pt_pred.log 2>&1 || { tail -30 gpurun_out/pt_pred.log; exit 1; }
tail -1 gpurun_out/pt_pred.log
timeout -k 10 300 python -u bench.py --cpu-baseline 0 > gpurun_out/pred_c3.json 2> gpurun_out/pred_c3.err || { tail -30 gpurun_out/pred_c3.err; exit 1; }
python3 -c "
import json;d=json.loads(open('gpurun_out/pred_c3.json').read().strip().splitlines()[-1]);r=d['roofline']
print('c3', round(d['ms_per_step'],1), 'ms/step; predict', round(r['avg_launch_ms']*1e3,1), 'us/launch, frac', round(r['frac'],4), d['breakdown']['checks']['events_sha1'])"
rm -rf gpurun_out/prof_pred
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_pred -o c3 -- python3 bench.py --cpu-baseline 0 --steps 3 > gpurun_out/prof_pred.log 2>&1 || { tail -30 gpurun_out/prof_pred.log; exit 1; }
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/prof_pred/c3_kernel_stats.csv')):
    if 'cforest' in r['Name']: print(r['Name'][:50], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us avg', round(float(r['MinNs'])/1e3,1), 'min')"
