#!/bin/bash
# round 6: finish() once per fill (the exact steps are arithmetic only); A/B against the
# round-5 scan; the in-pass knobs re-swept (tuning build); the chain kernel's per-wave profile
set -o pipefail
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/r6b && rm -rf gpurun_out/r6b/*
export TMPDIR=/tmp
O=gpurun_out/r6b
L=$PWD/distributed-drift-detection_amd/ddm_amd
timeout -k 10 600 python -u -m pytest tests/test_gpu_scan_batches.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  timeout -k 10 300 python -u tools/c4_scan_time.py --reps 20 --label new >> $O/ab.jsonl 2>> $O/ab.err || exit 1
  DDM_AMD_LIB=$L/libddm_amd_old.so timeout -k 10 300 python -u tools/c4_scan_time.py --reps 20 --label old >> $O/ab.jsonl 2>> $O/ab.err || exit 1
done
DDM_AMD_LIB=$L/libddm_amd_tune.so timeout -k 10 600 python -u tools/c4_scan_time.py --reps 15 --sweep 'tune_default:' 'steps1:DDM_SCAN_STEPS=1' 'steps3:DDM_SCAN_STEPS=3' 'steps4:DDM_SCAN_STEPS=4' 'pop8:DDM_SCAN_POP=8' 'pop32:DDM_SCAN_POP=32' 'pop4:DDM_SCAN_POP=4' >> $O/ab.jsonl 2>> $O/ab.err || exit 1
DDM_CHAIN_PROF=$O/chain_prof.json DDM_AMD_LIB=$L/libddm_amd_tune.so timeout -k 10 300 python -u tools/c4_scan_time.py --reps 3 --label chainprof >> $O/ab.jsonl 2>> $O/ab.err || exit 1
cat $O/ab.jsonl
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_INSTS_LDS --kernel-include-regex 'k_scan_batches' --output-format csv -d $O/sq_new -o p -- python3 bench.py --workload c4 --steps 1 --warmup 0 --cpu-baseline 0 > $O/sq_new.json 2> $O/sq_new.err || { tail -5 $O/sq_new.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o c4 -- python3 bench.py --workload c4 --cpu-baseline 0 > $O/trace_line.json 2> $O/trace.err || exit 1
echo done
