#!/bin/bash
# Parity (shuffle / controller / configs / dfit), the C3 host trace, then a C4 bench line and its kernel stats.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_shuffle.py tests/test_gpu_controller.py tests/test_gpu_configs.py tests/test_gpu_dfit.py -x -q --timeout 250 --timeout-method thread > gpurun_out/pytest_step.log 2>&1 || { tail -40 gpurun_out/pytest_step.log; exit 1; }
tail -1 gpurun_out/pytest_step.log
tools/gpu_htrace.sh > gpurun_out/ht.txt && tail -3 gpurun_out/ht.txt
python -c "
import json
d=json.load(open('gpurun_out/htrace_c3.json')); print('c3', round(d['value']/1e9,3), round(d['ms_per_step'],1), d['breakdown']['checks']['events_sha1'][:10])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4 -o c4 -- python3 bench.py --workload c4 --steps 5 --warmup 2 --cpu-baseline 0 > gpurun_out/c4.json 2> gpurun_out/c4.err || { tail -20 gpurun_out/c4.err; exit 1; }
python -c "
import json
d=json.load(open('gpurun_out/c4.json')); r=d['roofline']; print('c4', d['value'], round(d['ms_per_step'],3), r['frac'], r.get('avg_launch_ms'))"
python -c "
import csv
for r in list(csv.DictReader(open('gpurun_out/prof_c4/c4_kernel_stats.csv')))[:8]: print(r['Name'][:50], r['Calls'], r['AverageNs'])"
