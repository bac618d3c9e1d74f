#!/bin/bash
# round 6: host time of a run (cProfile of the second run; host marks) for c2 and C3
set -o pipefail
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/r6v && rm -rf gpurun_out/r6v/*
export TMPDIR=/tmp
O=gpurun_out/r6v
DDM_HOST_TRACE=1 DDM_HOST_TRACE_OUT=$O/ht_c2 DDM_CPROFILE_OUT=$O/cprof_c2.txt timeout -k 10 300 python -u bench.py --workload c2 --cpu-baseline 0 > $O/c2.json 2> $O/c2.err || { tail -5 $O/c2.err; exit 1; }
DDM_HOST_TRACE=1 DDM_HOST_TRACE_OUT=$O/ht_c3 DDM_CPROFILE_OUT=$O/cprof_c3.txt timeout -k 10 300 python -u bench.py --cpu-baseline 0 --companion 0 > $O/c3.json 2> $O/c3.err || { tail -5 $O/c3.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload c2 --cpu-baseline 0 > $O/c2_plain.json 2> $O/c2_plain.err || { tail -5 $O/c2_plain.err; exit 1; }
head -50 $O/cprof_c2.txt
echo done
