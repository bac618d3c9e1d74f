#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/diag_c3prop3.py 0 > gpurun_out/diag_fresh.txt 2>&1
timeout -k 10 200 python -u tools/diag_c3prop3.py 1 > gpurun_out/diag_after.txt 2>&1
