#!/bin/bash
# ddm_scan_batches: parity tests, then per-kernel times of the C4 bench (rocprofv3) for
# each configuration given as an argument (env assignments, "-" = defaults).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_scan_batches.py tests/test_gpu_scan_long.py tests/test_gpu_scan.py tests/test_gpu_longstream.py -x -q -s --timeout 200 --timeout-method thread > gpurun_out/pytest_sb.log 2>&1 || { tail -40 gpurun_out/pytest_sb.log; exit 1; }
tail -1 gpurun_out/pytest_sb.log
for cfg in "$@"; do
  [ "$cfg" = "-" ] && cfg=DDM_X=0
  env $cfg timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_sb -o sb -- python3 bench.py --workload c4 --cpu-baseline 0 --steps 3 > gpurun_out/prof_sb.json 2> gpurun_out/prof_sb.err || { tail -30 gpurun_out/prof_sb.err; exit 1; }
  python3 - "$cfg" <<'PY'
import csv, glob, json, sys
f = glob.glob('gpurun_out/prof_sb/**/*kernel_stats.csv', recursive=True)[0]
out, tot = [], 0.0
for r in csv.DictReader(open(f)):
    if 'scan_batches' in r['Name'] or 'prefix_table' in r['Name']:
        nm = r["Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
        out.append(f"{nm} {float(r['AverageNs'])/1e3:.1f}us")
        tot += float(r['AverageNs']) / 1e3
d = json.loads(open('gpurun_out/prof_sb.json').read().strip().splitlines()[-1])
print(sys.argv[1], f"sum {tot:.0f}us", 'bench', round(d['roofline']['avg_launch_ms'], 4), 'ms frac', round(d['roofline']['frac'], 3))
print('   ', '; '.join(out))
PY
  cp "$(ls gpurun_out/prof_sb/**/*kernel_stats.csv gpurun_out/prof_sb/*kernel_stats.csv 2>/dev/null | head -1)" "gpurun_out/sb_stats_${cfg//[^A-Za-z0-9]/_}.csv" 2>/dev/null
  rm -rf gpurun_out/prof_sb
done
