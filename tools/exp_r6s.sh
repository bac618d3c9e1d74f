#!/bin/bash
# round 6: C3 kernel trace + host marks (aligned on CLOCK_MONOTONIC) on the current tree:
# what the first ~20 epochs of a step wait for
set -o pipefail
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/r6s && rm -rf gpurun_out/r6s/*
export TMPDIR=/tmp
O=gpurun_out/r6s
DDM_HOST_TRACE=1 DDM_HOST_TRACE_OUT=$O/ht timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o c3 -- python3 bench.py --steps 2 --warmup 1 --cpu-baseline 0 --companion 0 > $O/c3_line.json 2> $O/c3.err || { tail -5 $O/c3.err; exit 1; }
find $O -name "*kernel_trace.csv" | head -3
echo done
