#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3 -o c3 -- python3 bench.py --cpu-baseline 0 > gpurun_out/prof_c3.log 2>&1 || { tail -30 gpurun_out/prof_c3.log; exit 1; }
tail -1 gpurun_out/prof_c3.log | cut -c1-300
