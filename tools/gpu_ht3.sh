#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp DDM_HOST_TRACE=1 DDM_HOST_TRACE_OUT=gpurun_out/host_trace.json
timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --oracle-check-rows 0 --cpu-baseline 0 > gpurun_out/c3.json 2> gpurun_out/c3.err || { tail -20 gpurun_out/c3.err; exit 1; }
python -c "
import json
t = json.load(open('gpurun_out/host_trace.json'))
prev=0
for l,x in t[:60]:
    print(f'{x*1e3:8.2f} +{(x-prev)*1e3:6.2f} {l}'); prev=x
"
