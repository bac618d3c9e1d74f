#!/bin/bash
# round 6: where a c2 (published cell) epoch goes now: kernel trace of the c2 command
set -o pipefail
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/r6zg && rm -rf gpurun_out/r6zg/*
export TMPDIR=/tmp
O=gpurun_out/r6zg
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c2 -- python3 bench.py --workload c2 --cpu-baseline 0 > $O/c2_line.json 2> $O/c2.err || { tail -5 $O/c2.err; exit 1; }
echo done
