#!/bin/bash
# round 6: a C5 epoch after the replay change (kernel trace of a reduced C5: 8M rows)
# host marks after the start-up changes
set -o pipefail
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/r6za && rm -rf gpurun_out/r6za/*
export TMPDIR=/tmp
O=gpurun_out/r6za
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c5 -- python3 bench.py --workload c5 --c5-rows 8000000 --steps 1 --warmup 1 --cpu-baseline 0 > $O/c5_line.json 2> $O/c5.err || { tail -5 $O/c5.err; exit 1; }
find $O -name "*.csv" | head
echo done
