#!/bin/bash
# End-of-round evidence: full GPU suite, smoke, default bench line (c3), c4 line, rocprofv3
# kernel stats of both benches.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_full.log 2>&1 || { tail -40 gpurun_out/pytest_full.log; exit 1; }
tail -1 gpurun_out/pytest_full.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/fin_c3.json 2> gpurun_out/fin_c3.err || { tail -30 gpurun_out/fin_c3.err; exit 1; }
timeout -k 10 200 python -u bench.py --workload c4 --steps 5 > gpurun_out/fin_c4.json 2> gpurun_out/fin_c4.err || { tail -30 gpurun_out/fin_c4.err; exit 1; }
for w in c3 c4; do python3 -c "
import json;d=json.loads(open('gpurun_out/fin_$w.json').read().strip().splitlines()[-1]);print('$w', d['value'], d['ms_per_step'], d['roofline']['frac'])"; done
rm -rf gpurun_out/prof_fc3 gpurun_out/prof_fc4
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fc3 -o c3 -- python3 bench.py --cpu-baseline 0 > gpurun_out/prof_fc3.log 2>&1 || { tail -30 gpurun_out/prof_fc3.log; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fc4 -o c4 -- python3 bench.py --workload c4 --cpu-baseline 0 --steps 5 > gpurun_out/prof_fc4.log 2>&1 || { tail -30 gpurun_out/prof_fc4.log; exit 1; }
echo profiles done
