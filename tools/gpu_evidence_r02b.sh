#!/bin/bash
# Round-2 evidence after the scan rework: default c3 line, c1, c5 (full), with kernel stats of c3.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py > gpurun_out/ev_c3.json 2> gpurun_out/ev_c3.err || { tail -30 gpurun_out/ev_c3.err; exit 1; }
tail -1 gpurun_out/ev_c3.json | cut -c1-300
timeout -k 10 200 python -u bench.py --workload c1 --steps 3 > gpurun_out/ev_c1.json 2> gpurun_out/ev_c1.err || { tail -30 gpurun_out/ev_c1.err; exit 1; }
tail -1 gpurun_out/ev_c1.json | cut -c1-200
timeout -k 10 400 python -u bench.py --workload c5 --steps 1 --warmup 0 > gpurun_out/ev_c5.json 2> gpurun_out/ev_c5.err || { tail -30 gpurun_out/ev_c5.err; exit 1; }
tail -1 gpurun_out/ev_c5.json | cut -c1-200
