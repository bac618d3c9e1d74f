#!/bin/bash
# round 6: fp64 dependent latency on gfx950 (tools/lat_bench); the whole -m gpu suite with the
# round's changes (published-cell fixture, N>1 line); the c2 published cell bench line
set -o pipefail
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/r6c && rm -rf gpurun_out/r6c/*
export TMPDIR=/tmp
O=gpurun_out/r6c
timeout -k 10 60 tools/lat_bench > $O/lat.txt 2>&1 || { cat $O/lat.txt; exit 1; }
cat $O/lat.txt
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -u bench.py --workload c2 > $O/bench_c2.json 2> $O/bench_c2.err || { tail -20 $O/bench_c2.err; exit 1; }
echo done
