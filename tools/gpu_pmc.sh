#!/bin/bash
# HBM traffic of the predict kernel (C3 bench) and of ddm_scan_batches (C4 bench):
# FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes, summarised by tools/pmc_summary.py.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
C3="python3 bench.py --steps 1 --warmup 0 --cpu-baseline 0 --oracle-check-rows 0"
C4="python3 bench.py --workload c4 --steps 1 --warmup 0 --cpu-baseline 0"
for c in FETCH_SIZE WRITE_SIZE; do
timeout -k 10 300 rocprofv3 --pmc $c --kernel-include-regex "k_cforest_predict" --output-format csv -d gpurun_out/pmc_c3_$c -o p -- $C3 > gpurun_out/pmc_c3_$c.json 2> gpurun_out/pmc_c3_$c.err || { tail -5 gpurun_out/pmc_c3_$c.err; exit 1; }
timeout -k 10 300 rocprofv3 --pmc $c --kernel-include-regex "k_scan_batches|k_scan_prefix" --output-format csv -d gpurun_out/pmc_c4_$c -o p -- $C4 > gpurun_out/pmc_c4_$c.json 2> gpurun_out/pmc_c4_$c.err || { tail -5 gpurun_out/pmc_c4_$c.err; exit 1; }
done
python3 tools/pmc_summary.py
