#!/bin/bash
# scan_batches parity, then C4 per-kernel times for chain-kernel variants
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_scan_batches.py tests/test_gpu_longstream.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pt_chain.log 2>&1 || { tail -30 gpurun_out/pt_chain.log; exit 1; }
tail -1 gpurun_out/pt_chain.log
tools/gpu_sb_quick.sh "$@"
