#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_shuffle.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_walk.log 2>&1 || { tail -30 gpurun_out/pytest_walk.log; exit 1; }
tail -1 gpurun_out/pytest_walk.log
DDM_AMD_LIB=$PWD/distributed-drift-detection_amd/ddm_amd/libddm_amd_prof.so timeout -k 10 120 python tools/walk_prof.py
