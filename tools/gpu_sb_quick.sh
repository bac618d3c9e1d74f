#!/bin/bash
# per-kernel times of the C4 bench (rocprofv3) for each configuration argument (env assignments)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in "$@"; do
  [ "$cfg" = "-" ] && cfg=DDM_X=0
  rm -rf gpurun_out/prof_q
  env $cfg timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_q -o q -- python3 bench.py --workload c4 --cpu-baseline 0 --steps 3 > gpurun_out/prof_q.json 2> gpurun_out/prof_q.err || { tail -30 gpurun_out/prof_q.err; exit 1; }
  python3 - "$cfg" <<'PY'
import csv, glob, sys
f = glob.glob('gpurun_out/prof_q/**/*kernel_stats.csv', recursive=True)[0]
out = []
for r in csv.DictReader(open(f)):
    if 'scan_batches' in r['Name'] or 'prefix_table' in r['Name']:
        nm = r['Name'].replace('void ', '').replace('(anonymous namespace)::', '').split('(')[0]
        out.append(f"{nm} {float(r['AverageNs'])/1e3:.1f}us")
print(sys.argv[1], '; '.join(out))
PY
done
