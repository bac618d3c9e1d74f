#!/bin/bash
# GroupedRunner: parity (configs, scaling) and c3 / c5 / solo-4 timings with 1 and 2 groups.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_scaling.py tests/test_gpu_configs.py -x -q --timeout 250 --timeout-method thread > gpurun_out/pytest_grp.log 2>&1 || { tail -40 gpurun_out/pytest_grp.log; exit 1; }
tail -1 gpurun_out/pytest_grp.log
for g in 1 2 1 2; do
timeout -k 10 200 python -u bench.py --groups $g --oracle-check-rows 0 --cpu-baseline 0 > gpurun_out/c3_g$g.json 2> gpurun_out/c3_g$g.err || { tail -30 gpurun_out/c3_g$g.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/c3_g$g.json'));b=d['breakdown'];r=d['roofline'];print('c3 g$g', round(d['value']/1e9,3), round(d['ms_per_step'],1), round(r['avg_launch_ms'],4), round(r['frac'],3), b['epochs_per_step'], b['checks']['events_sha1'][:10])"
done
for g in 1 2; do
timeout -k 10 200 python -u bench.py --groups $g --solo-world 4 --oracle-check-rows 0 > gpurun_out/c3s4_g$g.json 2> gpurun_out/c3s4_g$g.err || { tail -30 gpurun_out/c3s4_g$g.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/c3s4_g$g.json'));print('solo4 g$g', round(d['value']/1e9,3), round(d['ms_per_step'],1))"
timeout -k 10 300 python -u bench.py --workload c5 --c5-rows 8000000 --steps 1 --warmup 0 --groups $g --oracle-check-rows 0 --cpu-baseline 0 > gpurun_out/c5_g$g.json 2> gpurun_out/c5_g$g.err || { tail -30 gpurun_out/c5_g$g.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/c5_g$g.json'));b=d['breakdown'];print('c5 8M g$g', round(d['value']/1e6,2), 'M rows/s', round(d['ms_per_step'],1), b['epochs_per_step'], round(b['refits_per_s']))"
done
