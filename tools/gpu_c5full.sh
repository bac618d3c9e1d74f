#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py --workload c5 --steps 1 --warmup 0 > gpurun_out/c5_full.json 2> gpurun_out/c5_full.err || { tail -20 gpurun_out/c5_full.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/c5_full.json'));b=d['breakdown'];print('c5', round(d['value']/1e6,2), 'M rows/s', round(d['ms_per_step'],1), b['epochs_per_step'], round(b['refits_per_s']), d.get('cpu_baseline'))"
