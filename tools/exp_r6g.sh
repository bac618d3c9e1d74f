#!/bin/bash
# round 6: wave_tile's chain with the next group's RN(1/n) prefetched from LDS, n stepped in a
# register and x from the tile's bits (libddm_amd.so) against the round-5 form
# (libddm_amd_ldschain.so): parity, C4, ddm_scan_long on 10M carried rows, the chain profile
set -o pipefail
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/r6g && rm -rf gpurun_out/r6g/*
export TMPDIR=/tmp
O=gpurun_out/r6g
L=$PWD/distributed-drift-detection_amd/ddm_amd
timeout -k 10 900 python -u -m pytest tests/test_gpu_scan_batches.py tests/test_gpu_scan_long.py tests/test_gpu_longstream.py tests/test_gpu_scan_cert.py tests/test_gpu_scan.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u tools/bench_scan_cert.py --reps 3 --exact > $O/long_new.txt 2>&1 || { tail -5 $O/long_new.txt; exit 1; }
DDM_AMD_LIB=$L/libddm_amd_ldschain.so timeout -k 10 300 python -u tools/bench_scan_cert.py --reps 3 --exact > $O/long_lds.txt 2>&1 || { tail -5 $O/long_lds.txt; exit 1; }
grep scan_long $O/long_new.txt $O/long_lds.txt
for i in 1 2; do
  timeout -k 10 300 python -u tools/c4_scan_time.py --reps 20 --label prefetch >> $O/ab.jsonl 2>> $O/ab.err || exit 1
  DDM_AMD_LIB=$L/libddm_amd_ldschain.so timeout -k 10 300 python -u tools/c4_scan_time.py --reps 20 --label r5tile >> $O/ab.jsonl 2>> $O/ab.err || exit 1
done
DDM_CHAIN_PROF=$O/chain_prof.json DDM_AMD_LIB=$L/libddm_amd_tune.so timeout -k 10 300 python -u tools/c4_scan_time.py --reps 3 --label chainprof >> $O/ab.jsonl 2>> $O/ab.err || exit 1
cat $O/ab.jsonl
echo done
