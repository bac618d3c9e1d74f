#!/bin/bash
# Full GPU test suite + smoke, then the C4 bench line with its rocprofv3 kernel stats.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_full.log 2>&1 || { tail -40 gpurun_out/pytest_full.log; exit 1; }
tail -2 gpurun_out/pytest_full.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 200 python -u bench.py --workload c4 --steps 5 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || { tail -30 gpurun_out/bench_c4.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/bench_c4.json').read().strip().splitlines()[-1]);print('c4', d['value'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
rm -rf gpurun_out/prof_c4
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4 -o c4 -- python3 bench.py --workload c4 --cpu-baseline 0 --steps 5 > gpurun_out/prof_c4.log 2>&1 || { tail -30 gpurun_out/prof_c4.log; exit 1; }
find gpurun_out/prof_c4 -name '*kernel_stats.csv' -exec grep -h "scan_batches\|prefix" {} \;
