#!/bin/bash
# The whole -m gpu suite (as the driver runs it), then smoke().
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_full.log 2>&1 || { grep -E "PASSED|FAILED|ERROR" gpurun_out/pytest_full.log | tail -5; tail -40 gpurun_out/pytest_full.log; exit 1; }
tail -1 gpurun_out/pytest_full.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
