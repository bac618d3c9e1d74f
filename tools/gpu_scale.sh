#!/bin/bash
# C3 per-GPU share at N = 8 / 4 / 2 (rank 0's partitions alone), C5 at 8M rows, C1.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for w in 8 4 2; do
timeout -k 10 200 python -u bench.py --solo-world $w --oracle-check-rows 0 --cpu-baseline 0 > gpurun_out/solo$w.json 2> gpurun_out/solo$w.err || { tail -20 gpurun_out/solo$w.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/solo$w.json'));print('solo$w', round(d['value']/1e9,3), round(d['ms_per_step'],1), d['breakdown']['epochs_per_step'])"
done
timeout -k 10 300 python -u bench.py --workload c5 --c5-rows 8000000 --steps 1 --warmup 0 --oracle-check-rows 0 --cpu-baseline 0 > gpurun_out/c5_8m.json 2> gpurun_out/c5_8m.err || { tail -20 gpurun_out/c5_8m.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/c5_8m.json'));b=d['breakdown'];print('c5 8M', round(d['value']/1e6,2), 'M rows/s', round(d['ms_per_step'],1), b['epochs_per_step'], round(b['refits_per_s']))"
timeout -k 10 200 python -u bench.py --workload c1 --cpu-baseline 0 > gpurun_out/c1.json 2> gpurun_out/c1.err || { tail -20 gpurun_out/c1.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/c1.json'));print('c1', round(d['value']/1e6,2), 'M rows/s', round(d['ms_per_step'],2), d['breakdown'].get('checks'))"
