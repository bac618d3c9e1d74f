#!/bin/bash
# Host phase trace of the C3 bench's last run (DDM_HOST_TRACE).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp DDM_HOST_TRACE=1 DDM_HOST_TRACE_OUT=gpurun_out/host_trace.json
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --cpu-baseline 0 --oracle-check-rows 0 "$@" > gpurun_out/htrace_c3.json 2> gpurun_out/htrace_c3.err || { tail -30 gpurun_out/htrace_c3.err; exit 1; }
python -c "
import json
t = json.load(open('gpurun_out/host_trace.json'))
prev = 0.0
for k, (l, x) in enumerate(t[:60]):
    print(f'{x*1e3:9.2f} +{(x-prev)*1e3:7.2f} {l}'); prev = x
print('...', len(t), 'marks, end', round(t[-1][1]*1e3, 2), 'ms')
for l, x in t[-4:]: print(f'{x*1e3:9.2f} {l}')
"
