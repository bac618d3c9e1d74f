#!/bin/bash
# Round 2: per-GPU share of the strong-scaling c3 (solo 8 / 4 / 2), c5 full size, rocprof of c3 solo-8.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for w in 8 4 2; do
  timeout -k 10 200 python -u bench.py --solo-world $w --oracle-check-rows 0 > gpurun_out/c3_solo$w.json 2> gpurun_out/c3_solo$w.err || { tail -30 gpurun_out/c3_solo$w.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/c3_solo$w.json'));b=d['breakdown'];print('solo$w', d['value'], d['ms_per_step'], b['epochs_per_step'], b['predict_kernel_ms_per_step'], b['device_refit_kernels_ms_per_step'], b['shuffle_kernels_ms_per_step'], b['host_s_per_step'], b['gpu_wait_s_per_step'])"
done
timeout -k 10 500 python -u bench.py --workload c5 --steps 1 --warmup 0 --oracle-check-rows 20000 > gpurun_out/c5_full.json 2> gpurun_out/c5_full.err || { tail -30 gpurun_out/c5_full.err; exit 1; }
cat gpurun_out/c5_full.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_solo8 -o solo8 -- python3 bench.py --solo-world 8 --oracle-check-rows 0 > gpurun_out/prof_solo8.log 2>&1 || { tail -30 gpurun_out/prof_solo8.log; exit 1; }
find gpurun_out/prof_solo8 -name '*kernel_stats.csv' -exec cat {} \;
