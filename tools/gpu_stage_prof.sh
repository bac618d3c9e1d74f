#!/bin/bash
# refit parity, c3 kernel stats at N=1, then the staging kernel's phase clocks (profile build) at the N=8 share
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_dfit.py tests/test_gpu_controller.py tests/test_gpu_configs.py tests/test_gpu_pipeline.py tests/test_gpu_shuffle.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pt_sp.log 2>&1 || { tail -30 gpurun_out/pt_sp.log; exit 1; }
tail -1 gpurun_out/pt_sp.log
rm -rf gpurun_out/prof_sp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_sp -o c3 -- python3 bench.py --cpu-baseline 0 --steps 2 --warmup 1 > gpurun_out/prof_sp.log 2>&1 || { tail -30 gpurun_out/prof_sp.log; exit 1; }
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/prof_sp/c3_kernel_stats.csv')):
    if 'dfit' in r['Name'] or 'k_stage' in r['Name']: print(r['Name'].split('(')[0][-20:], r['Calls'], round(float(r['AverageNs'])/1e3, 1), 'us')"
DDM_AMD_LIB=distributed-drift-detection_amd/ddm_amd/libddm_amd_sprof.so timeout -k 10 300 python -u bench.py --solo-world 8 --cpu-baseline 0 --steps 1 --warmup 1 > gpurun_out/sp.json 2> gpurun_out/sp.err || { tail -30 gpurun_out/sp.err; exit 1; }
grep -h "stage-prof" gpurun_out/sp.json gpurun_out/sp.err > gpurun_out/sp_lines.txt || true
python3 -c "
import re, numpy as np
L=[list(map(float, re.findall(r'[0-9.]+', l)[-6:])) for l in open('gpurun_out/sp_lines.txt')]
a=np.array(L); print(len(L), 'launches; median us: compact/gather/words/shuffle/seeds/swaps', np.median(a, axis=0))"
