#!/bin/bash
# round 6: the fix-up's lane pass (spec runs copied by one lane per stream, the wave pass only
# for what still needs rows) against the wave-per-stream fix-up (libddm_amd_spec.so):
# parity, C4, kernel trace, the scan's FETCH_SIZE / WRITE_SIZE passes
set -o pipefail
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/r6l && rm -rf gpurun_out/r6l/*
export TMPDIR=/tmp
O=gpurun_out/r6l
L=$PWD/distributed-drift-detection_amd/ddm_amd
timeout -k 10 900 python -u -m pytest tests/test_gpu_scan_batches.py tests/test_gpu_scan_long.py tests/test_gpu_longstream.py tests/test_gpu_scan_cert.py tests/test_gpu_scan.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  timeout -k 10 300 python -u tools/c4_scan_time.py --reps 20 --label fixlane >> $O/ab.jsonl 2>> $O/ab.err || exit 1
  DDM_AMD_LIB=$L/libddm_amd_spec.so timeout -k 10 300 python -u tools/c4_scan_time.py --reps 20 --label spec >> $O/ab.jsonl 2>> $O/ab.err || exit 1
done
cat $O/ab.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o c4 -- python3 bench.py --workload c4 --cpu-baseline 0 > $O/trace_line.json 2> $O/trace.err || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex 'k_scan_batches|k_scan_prefix' --output-format csv -d $O/pmc_$c -o p -- python3 bench.py --workload c4 --steps 1 --warmup 0 --cpu-baseline 0 --c4-check-stride 0 > $O/pmc_$c.txt 2>&1 || exit 1
done
timeout -k 10 600 python -u bench.py --workload c4 > $O/bench_c4.json 2> $O/bench_c4.err || { tail -5 $O/bench_c4.err; exit 1; }
echo done
