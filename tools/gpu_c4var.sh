#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
L=$PWD/distributed-drift-detection_amd/ddm_amd
run() { timeout -k 10 200 env "$@" python -u bench.py --workload c4 --steps 5 --warmup 2 --cpu-baseline 0 > gpurun_out/c4v.json 2> gpurun_out/c4v.err || { tail -5 gpurun_out/c4v.err; exit 1; }; python -c "import json;d=json.load(open('gpurun_out/c4v.json'));print('$*', round(d['roofline']['avg_launch_ms'],3))"; }
run X=1
run DDM_AMD_LIB=$L/libddm_amd_w5.so DDM_SCAN_WAVES=5120
run DDM_AMD_LIB=$L/libddm_amd_w5.so DDM_SCAN_WAVES=4096
run DDM_SCAN_WAVES=8192
run DDM_SCAN_FILL=32
run DDM_SCAN_FILL=128
run DDM_SCAN_POP=8
run DDM_SCAN_POP=32
run DDM_FIX_BLOCKS=1024
run DDM_FIX_BLOCKS=256
