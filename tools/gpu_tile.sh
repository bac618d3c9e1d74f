#!/bin/bash
# wave_tile users: parity (scan_long, scan_batches, longstream) with the 10M-row timing line, then C4 kernel times
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_scan_long.py tests/test_gpu_scan_batches.py tests/test_gpu_longstream.py -x -q -s --timeout 300 --timeout-method thread > gpurun_out/pt_tile.log 2>&1 || { tail -30 gpurun_out/pt_tile.log; exit 1; }
grep "10M-row\|passed\|failed" gpurun_out/pt_tile.log
tools/gpu_sb_quick.sh - "DDM_FIX_BLOCKS=1024"
