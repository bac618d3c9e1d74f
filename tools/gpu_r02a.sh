#!/bin/bash
# Round 2, first GPU pass: config tests (C1/C5/C3 property), c5/c1/c3 bench lines, G-invariance.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_cfg.log 2>&1 || { tail -60 gpurun_out/pytest_cfg.log; exit 1; }
tail -8 gpurun_out/pytest_cfg.log
timeout -k 10 300 python -u bench.py --workload c5 --c5-rows 2000000 --steps 1 --warmup 0 --cpu-baseline 0 --oracle-check-rows 0 > gpurun_out/c5_small.json 2> gpurun_out/c5_small.err || { tail -30 gpurun_out/c5_small.err; exit 1; }
cat gpurun_out/c5_small.json
timeout -k 10 200 python -u bench.py --workload c1 --steps 3 --warmup 1 > gpurun_out/c1.json 2> gpurun_out/c1.err || { tail -30 gpurun_out/c1.err; exit 1; }
cat gpurun_out/c1.json
timeout -k 10 300 python -u bench.py > gpurun_out/c3.json 2> gpurun_out/c3.err || { tail -30 gpurun_out/c3.err; exit 1; }
cat gpurun_out/c3.json
timeout -k 10 400 python -u -m pytest tests/test_gpu_scaling.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_scale.log 2>&1 || { tail -60 gpurun_out/pytest_scale.log; exit 1; }
tail -5 gpurun_out/pytest_scale.log
