#!/bin/bash
# Parity of the shuffle / controller / configs suites, then the host phase trace of C3.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_shuffle.py tests/test_gpu_controller.py tests/test_gpu_configs.py -x -q --timeout 250 --timeout-method thread > gpurun_out/pytest_step.log 2>&1 || { tail -40 gpurun_out/pytest_step.log; exit 1; }
tail -1 gpurun_out/pytest_step.log
tools/gpu_htrace.sh
python -c "
import json
d=json.load(open('gpurun_out/htrace_c3.json')); print('c3', round(d['value']/1e9,3), round(d['ms_per_step'],1), d['breakdown']['checks'])
t = json.load(open('gpurun_out/host_trace.json'))
ep=[x for l,x in t if l=='epoch']; sy=[x for l,x in t if l=='synchronized']; la=[x for l,x in t if l=='launched']
d=[b-a for a,b in zip(ep, ep[1:]+[t[-1][1]])]
print('start', round(ep[0]*1e3,2), 'epochs', len(d), [round(x*1e3,2) for x in d[:24]])
print('wait', round(sum(s-l for s,l in zip(sy,la))*1e3,1), 'total', round(t[-1][1]*1e3,1))
"
