#!/bin/bash
# round 6: the carried runs after unchanged level-1 batches computed ahead, beside the walk
# (spec blocks of k_scan_batches_walk), the fix-up taking them (libddm_amd.so) against the tree
# without (libddm_amd_ldschain.so): parity, C4, the fix-up's profile, kernel trace
set -o pipefail
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/r6h && rm -rf gpurun_out/r6h/*
export TMPDIR=/tmp
O=gpurun_out/r6h
L=$PWD/distributed-drift-detection_amd/ddm_amd
timeout -k 10 900 python -u -m pytest tests/test_gpu_scan_batches.py tests/test_gpu_scan_long.py tests/test_gpu_longstream.py tests/test_gpu_scan_cert.py tests/test_gpu_scan.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  timeout -k 10 300 python -u tools/c4_scan_time.py --reps 20 --label spec >> $O/ab.jsonl 2>> $O/ab.err || exit 1
  DDM_AMD_LIB=$L/libddm_amd_ldschain.so timeout -k 10 300 python -u tools/c4_scan_time.py --reps 20 --label nospec >> $O/ab.jsonl 2>> $O/ab.err || exit 1
done
DDM_CHAIN_PROF=$O/chain_prof.json DDM_AMD_LIB=$L/libddm_amd_tune.so timeout -k 10 300 python -u tools/c4_scan_time.py --reps 3 --label chainprof >> $O/ab.jsonl 2>> $O/ab.err || exit 1
cat $O/ab.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o c4 -- python3 bench.py --workload c4 --cpu-baseline 0 > $O/trace_line.json 2> $O/trace.err || exit 1
echo done
