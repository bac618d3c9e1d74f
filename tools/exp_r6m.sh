#!/bin/bash
# round 6: spec-list slots per exact<1> wave (no same-address atomics) against one global
# counter (libddm_amd_spec.so): parity, C4, kernel trace
set -o pipefail
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/r6m && rm -rf gpurun_out/r6m/*
export TMPDIR=/tmp
O=gpurun_out/r6m
L=$PWD/distributed-drift-detection_amd/ddm_amd
timeout -k 10 900 python -u -m pytest tests/test_gpu_scan_batches.py tests/test_gpu_scan_long.py tests/test_gpu_longstream.py tests/test_gpu_scan_cert.py tests/test_gpu_scan.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  timeout -k 10 300 python -u tools/c4_scan_time.py --reps 20 --label specwave >> $O/ab.jsonl 2>> $O/ab.err || exit 1
  DDM_AMD_LIB=$L/libddm_amd_spec.so timeout -k 10 300 python -u tools/c4_scan_time.py --reps 20 --label spec >> $O/ab.jsonl 2>> $O/ab.err || exit 1
done
cat $O/ab.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o c4 -- python3 bench.py --workload c4 --cpu-baseline 0 > $O/trace_line.json 2> $O/trace.err || exit 1
echo done
