#!/bin/bash
# round 6: C3 / c2 host marks on the last tree (where the run start still goes)
set -o pipefail
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/r6zd && rm -rf gpurun_out/r6zd/*
export TMPDIR=/tmp
O=gpurun_out/r6zd
DDM_HOST_TRACE=1 DDM_HOST_TRACE_OUT=$O/ht_c3 timeout -k 10 300 python -u bench.py --cpu-baseline 0 --companion 0 > $O/c3.json 2> $O/c3.err || { tail -5 $O/c3.err; exit 1; }
DDM_HOST_TRACE=1 DDM_HOST_TRACE_OUT=$O/ht_c2 timeout -k 10 300 python -u bench.py --workload c2 --cpu-baseline 0 > $O/c2.json 2> $O/c2.err || { tail -5 $O/c2.err; exit 1; }
echo done
