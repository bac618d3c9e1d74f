#!/bin/bash
# End-of-session evidence: all GPU tests, both bench lines, rocprof stats, PMC traffic, SQ counters of the C4 scan.
set -o pipefail
cd "$(dirname "$0")/.."
bash tools/gpu_check.sh && bash tools/pmc_traffic.sh > gpurun_out/pmc_traffic.log 2>&1 && bash tools/pmc_c4.sh > gpurun_out/pmc_c4_summary.txt 2>&1
rc=$?
tail -5 gpurun_out/pmc_traffic.log
cat gpurun_out/pmc_c4_summary.txt | tail -40
exit $rc
