#!/bin/bash
# rocprofv3 kernel trace + stats of the default C3 bench (timeline analysed on the host).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/prof_c3 -o c3 -- python3 bench.py --steps 2 --warmup 1 --cpu-baseline 0 --oracle-check-rows 0 > gpurun_out/prof_c3.json 2> gpurun_out/prof_c3.err || { tail -30 gpurun_out/prof_c3.err; exit 1; }
find gpurun_out/prof_c3 -name "*.csv" | head -20
