#!/bin/bash
# Parity (shuffle / controller / configs), then host trace and kernel summary of C3.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_shuffle.py tests/test_gpu_controller.py tests/test_gpu_configs.py -x -q --timeout 250 --timeout-method thread > gpurun_out/pytest_step.log 2>&1 || { tail -40 gpurun_out/pytest_step.log; exit 1; }
tail -1 gpurun_out/pytest_step.log
tools/gpu_prof2.sh
