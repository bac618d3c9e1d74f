#!/bin/bash
# round 6: launch sizes of the fix-up (DDM_FIX_BLOCKS) and of the spec workgroups
# (DDM_SPEC_BLOCKS) with the speculative carried runs; counts of both lists
set -o pipefail
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/r6i && rm -rf gpurun_out/r6i/*
export TMPDIR=/tmp
O=gpurun_out/r6i
L=$PWD/distributed-drift-detection_amd/ddm_amd
DDM_AMD_LIB=$L/libddm_amd_tune.so timeout -k 10 900 python -u tools/c4_scan_time.py --reps 15 --sweep 'default:' 'fix4096:DDM_FIX_BLOCKS=4096' 'fix8192:DDM_FIX_BLOCKS=8192' 'spec1024:DDM_SPEC_BLOCKS=1024' 'spec4096:DDM_SPEC_BLOCKS=4096' 'fix4096spec4096:DDM_FIX_BLOCKS=4096,DDM_SPEC_BLOCKS=4096' 'default2:' > $O/ab.jsonl 2> $O/ab.err || { tail -5 $O/ab.err; exit 1; }
cat $O/ab.jsonl
echo done
