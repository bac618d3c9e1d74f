#!/bin/bash
# C4: parity + fix-up timing.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_scan_batches.py tests/test_gpu_scan.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_c4.log 2>&1 || { tail -40 gpurun_out/pytest_c4.log; exit 1; }
tail -1 gpurun_out/pytest_c4.log
for cfg in DDM_X=0 DDM_FIX_OPEN=1; do
env $cfg timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fx -o fx -- python3 bench.py --workload c4 --cpu-baseline 0 --steps 3 > gpurun_out/prof_fx.log 2>&1 || { tail -30 gpurun_out/prof_fx.log; exit 1; }
python3 - "$cfg" <<'PY'
import csv, sys
out = []
for r in csv.DictReader(open('gpurun_out/prof_fx/fx_kernel_stats.csv')):
    if 'scan_batches' in r['Name']:
        out.append(f"{r['Name'].split('(')[0].split('_')[-1][:5]} {float(r['AverageNs'])/1e3:.0f}us")
print(sys.argv[1], *out)
PY
rm -rf gpurun_out/prof_fx
done
