#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for cfg in "$@"; do
  env $cfg timeout -k 10 150 python -u bench.py --cpu-baseline 0 > gpurun_out/c3_sweep.json 2> gpurun_out/c3_sweep.err || { tail -20 gpurun_out/c3_sweep.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/c3_sweep.json'));b=d['breakdown'];print('$cfg', d['value'], d['ms_per_step'], b['gpu_wait_s_per_step'], b['epochs_per_step'])"
done
