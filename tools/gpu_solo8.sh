#!/bin/bash
# c3 at the N=8 per-GPU share (one partition per GPU) alone: bench line + kernel stats.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u bench.py --solo-world 8 --steps 3 --warmup 1 --cpu-baseline 0 > gpurun_out/solo8.json 2> gpurun_out/solo8.err || { tail -30 gpurun_out/solo8.err; exit 1; }
python3 -c "
import json;d=json.loads(open('gpurun_out/solo8.json').read().strip().splitlines()[-1]);b=d['breakdown']
print('ms/step', d['ms_per_step'], {k: b[k] for k in b if k.endswith('per_step')})"
rm -rf gpurun_out/prof_solo8
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_solo8 -o s8 -- python3 bench.py --solo-world 8 --steps 3 --warmup 1 --cpu-baseline 0 > gpurun_out/prof_solo8.log 2>&1 || { tail -30 gpurun_out/prof_solo8.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/prof_solo8/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    nm = r['Name'].replace('void ', '').replace('(anonymous namespace)::', '').split('(')[0][:50]
    print(f"{nm:50s} {r['Calls']:>6s} {float(r['AverageNs'])/1e3:8.1f}us {float(r['TotalDurationNs'])/1e6:8.2f}ms")
PY
