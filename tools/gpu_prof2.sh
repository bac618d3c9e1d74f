#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
tools/gpu_htrace.sh > gpurun_out/ht.txt && tail -6 gpurun_out/ht.txt && tools/gpu_prof_c3.sh > /dev/null && python tools/trace_summary.py gpurun_out/prof_c3/c3_kernel_trace.csv 2 3
