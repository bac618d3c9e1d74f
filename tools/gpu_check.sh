#!/bin/bash
# One GPU call: parity tests, both bench lines, rocprof kernel stats of both benches.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 200 python -u bench.py > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || { tail -30 gpurun_out/bench_c3.err; exit 1; }
cat gpurun_out/bench_c3.json
timeout -k 10 120 python -u bench.py --workload c4 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || { tail -30 gpurun_out/bench_c4.err; exit 1; }
cat gpurun_out/bench_c4.json
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3 -o c3 -- python3 bench.py --cpu-baseline 0 > gpurun_out/prof_c3.log 2>&1 || { tail -30 gpurun_out/prof_c3.log; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4 -o c4 -- python3 bench.py --workload c4 --cpu-baseline 0 > gpurun_out/prof_c4.log 2>&1 || { tail -30 gpurun_out/prof_c4.log; exit 1; }
ls gpurun_out/prof_c3 gpurun_out/prof_c4
