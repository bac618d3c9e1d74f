#!/bin/bash
# Host phase trace of a steady C3 epoch at the N=8 share (one partition): marks 300-340.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp DDM_HOST_TRACE=1 DDM_HOST_TRACE_OUT=gpurun_out/host_trace.json
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --cpu-baseline 0 --oracle-check-rows 0 "$@" > gpurun_out/htrace_c3.json 2> gpurun_out/htrace_c3.err || { tail -30 gpurun_out/htrace_c3.err; exit 1; }
python -c "
import json
t = json.load(open('gpurun_out/host_trace.json'))
prev = t[299][1]
for l, x in t[300:345]:
    print(f'{x*1e3:9.3f} +{(x-prev)*1e6:8.1f}us {l}'); prev = x
print('...', len(t), 'marks, end', round(t[-1][1]*1e3, 2), 'ms')
"
