#!/bin/bash
# round 6: classify occupancy -- the LDS ring at 4 fills (DDM_RING), the LDS queue at 64
# (DDM_LQ), 5 / 6 waves per SIMD (DDM_CLS_WAVES): the C4 call and its digest per variant
set -o pipefail
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/r6f && rm -rf gpurun_out/r6f/*
export TMPDIR=/tmp
O=gpurun_out/r6f
L=$PWD/distributed-drift-detection_amd/ddm_amd
for i in 1 2; do
  timeout -k 10 300 python -u tools/c4_scan_time.py --reps 20 --label default >> $O/ab.jsonl 2>> $O/ab.err || exit 1
  for v in r4 r4w5 r4w5q64 r4w6q64; do
    DDM_AMD_LIB=$L/libddm_amd_$v.so timeout -k 10 300 python -u tools/c4_scan_time.py --reps 20 --label $v >> $O/ab.jsonl 2>> $O/ab.err || exit 1
  done
done
cat $O/ab.jsonl
echo done
