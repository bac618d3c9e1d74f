#!/bin/bash
# Host-side cProfile of the C3 bench (where the epoch loop's host time goes).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m cProfile -o gpurun_out/c3.prof bench.py --steps 2 --warmup 1 --cpu-baseline 0 --oracle-check-rows 0 "$@" > gpurun_out/cprof_c3.json 2> gpurun_out/cprof_c3.err || { tail -30 gpurun_out/cprof_c3.err; exit 1; }
python -c "
import pstats
p = pstats.Stats('gpurun_out/c3.prof')
p.sort_stats('tottime').print_stats(45)
" > gpurun_out/cprof_c3.txt
head -c 300 gpurun_out/cprof_c3.json
