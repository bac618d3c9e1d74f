#!/bin/bash
# Round-2 evidence: default bench line (C3, with the CPU baseline), its rocprofv3 kernel
# stats, the C4 and C1 lines and C4 kernel stats; copied into profiles/ by the caller.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/final
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py > gpurun_out/final/bench_c3.json 2> gpurun_out/final/bench_c3.err || { tail -20 gpurun_out/final/bench_c3.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/final/bench_c3.json'));r=d['roofline'];print('c3', round(d['value']/1e9,3), round(d['ms_per_step'],1), round(r['avg_launch_ms'],4), round(r['frac'],3), d['cpu_baseline']['value'] if d['cpu_baseline'] else None)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final/prof_c3 -o c3 -- python3 bench.py --cpu-baseline 0 > gpurun_out/final/prof_c3.json 2> gpurun_out/final/prof_c3.err || { tail -20 gpurun_out/final/prof_c3.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload c4 > gpurun_out/final/bench_c4.json 2> gpurun_out/final/bench_c4.err || { tail -20 gpurun_out/final/bench_c4.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final/prof_c4 -o c4 -- python3 bench.py --workload c4 --cpu-baseline 0 > /dev/null 2> gpurun_out/final/prof_c4.err || { tail -20 gpurun_out/final/prof_c4.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload c1 > gpurun_out/final/bench_c1.json 2> gpurun_out/final/bench_c1.err || { tail -20 gpurun_out/final/bench_c1.err; exit 1; }
python -c "
import json, csv
for w in ('c4','c1'):
    d=json.load(open(f'gpurun_out/final/bench_{w}.json')); print(w, d['value'], round(d['ms_per_step'],3), d['roofline']['frac'])
for r in list(csv.DictReader(open('gpurun_out/final/prof_c3/c3_kernel_stats.csv')))[:6]: print(r['Name'][:48], r['Calls'], r['AverageNs'])"
