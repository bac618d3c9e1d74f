#!/bin/bash
# staging parity, then per-block phase clocks of the staging kernel at N=1 (profile build)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_controller.py tests/test_gpu_configs.py tests/test_gpu_pipeline.py tests/test_gpu_shuffle.py tests/test_gpu_dfit.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pt_sb.log 2>&1 || { tail -30 gpurun_out/pt_sb.log; exit 1; }
tail -1 gpurun_out/pt_sb.log
DDM_AMD_LIB=distributed-drift-detection_amd/ddm_amd/libddm_amd_sprof.so timeout -k 10 300 python -u bench.py --cpu-baseline 0 --steps 1 --warmup 1 > gpurun_out/sp1.json 2> gpurun_out/sp1.err || { tail -30 gpurun_out/sp1.err; exit 1; }
grep -h "stage-" gpurun_out/sp1.json gpurun_out/sp1.err > gpurun_out/sp1_lines.txt || true
wc -l gpurun_out/sp1_lines.txt
