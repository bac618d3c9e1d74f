#!/bin/bash
# C4 fix-up kernel sensitivity (blocks / refill / open thresholds).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in DDM_X=0 DDM_FIX_BLOCKS=128 DDM_FIX_BLOCKS=2048 DDM_FIX_BLOCKS=4096 DDM_FIX_REFILL=1 DDM_FIX_REFILL=48 DDM_FIX_OPEN=1 DDM_FIX_OPEN=48; do
env $cfg timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fx -o fx -- python3 bench.py --workload c4 --cpu-baseline 0 --steps 3 > gpurun_out/prof_fx.log 2>&1 || { tail -30 gpurun_out/prof_fx.log; exit 1; }
python3 - "$cfg" <<'PY'
import csv, sys
out = []
for r in csv.DictReader(open('gpurun_out/prof_fx/fx_kernel_stats.csv')):
    if 'fix' in r['Name'] or 'spec' in r['Name']:
        out.append(f"{'fix' if 'fix' in r['Name'] else 'spec'} {float(r['AverageNs'])/1e3:.0f}us")
print(sys.argv[1], *out)
PY
rm -rf gpurun_out/prof_fx
done
