#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
DDM_AMD_LIB=$PWD/distributed-drift-detection_amd/ddm_amd/libddm_amd_dprof.so timeout -k 10 120 python tools/dfit_prof.py || exit 1
tools/gpu_final.sh
