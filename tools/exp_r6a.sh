#!/bin/bash
# round 6: classify pass without the int64 division / item_stream on the exact-step path,
# buffer-descriptor fill loads, the flush without a recomputed geometry -- parity, A/B
# against the round-5 scan (libddm_amd_old.so), SQ_INSTS_VALU per call
set -o pipefail
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/r6a && rm -rf gpurun_out/r6a/*
export TMPDIR=/tmp
O=gpurun_out/r6a
timeout -k 10 600 python -u -m pytest tests/test_gpu_scan_batches.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
  timeout -k 10 300 python -u tools/c4_scan_time.py --reps 20 --label new >> $O/ab.jsonl 2>> $O/ab.err || exit 1
  DDM_AMD_LIB=$PWD/distributed-drift-detection_amd/ddm_amd/libddm_amd_old.so timeout -k 10 300 python -u tools/c4_scan_time.py --reps 20 --label old >> $O/ab.jsonl 2>> $O/ab.err || exit 1
done
cat $O/ab.jsonl
for v in new old; do
  if [ $v = old ]; then export DDM_AMD_LIB=$PWD/distributed-drift-detection_amd/ddm_amd/libddm_amd_old.so; else unset DDM_AMD_LIB; fi
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_INSTS_LDS --kernel-include-regex 'k_scan_batches' --output-format csv -d $O/sq_$v -o p -- python3 bench.py --workload c4 --steps 1 --warmup 0 --cpu-baseline 0 > $O/sq_$v.json 2> $O/sq_$v.err || { tail -5 $O/sq_$v.err; exit 1; }
done
unset DDM_AMD_LIB
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o c4 -- python3 bench.py --workload c4 --cpu-baseline 0 > $O/trace_line.json 2> $O/trace.err || exit 1
echo done
