#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_controller.py tests/test_gpu_configs.py -x -q --timeout 250 --timeout-method thread > gpurun_out/pytest_step.log 2>&1 || { tail -40 gpurun_out/pytest_step.log; exit 1; }
tail -1 gpurun_out/pytest_step.log
export DDM_HOST_TRACE=1 DDM_HOST_TRACE_OUT=gpurun_out/host_trace_c1.json
timeout -k 10 200 python -u bench.py --workload c1 --cpu-baseline 0 > gpurun_out/c1.json 2> gpurun_out/c1.err || { tail -20 gpurun_out/c1.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/c1.json'));print('c1', round(d['value']/1e6,2), 'M rows/s', round(d['ms_per_step'],2), d['breakdown'].get('checks'))"
timeout -k 10 200 python -u bench.py --oracle-check-rows 0 --cpu-baseline 0 > gpurun_out/c3.json 2> gpurun_out/c3.err || { tail -20 gpurun_out/c3.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/c3.json'));print('c3', round(d['value']/1e9,3), round(d['ms_per_step'],1), d['breakdown']['checks']['events_sha1'][:10])"
