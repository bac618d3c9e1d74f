#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_shuffle.py tests/test_gpu_controller.py tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_c3.log 2>&1 || { tail -30 gpurun_out/pytest_c3.log; exit 1; }
tail -2 gpurun_out/pytest_c3.log
bash tools/gpu_c3sweep.sh "$@"
