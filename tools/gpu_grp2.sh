#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/tr
export TMPDIR=/tmp
DDM_BENCH_BACKEND=gloo timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29611 --log-dir gpurun_out/tr -r 3 bench.py --gpus 2 --workload c5 --c5-rows 160000 --steps 1 --warmup 0 --oracle-check-rows 0 --cpu-baseline 0 > gpurun_out/c5w2.json 2> gpurun_out/c5w2.err; echo "rc=$?"
find gpurun_out/tr -name "*.log" | while read f; do echo "== $f"; grep -v amdgpu.ids "$f" | tail -30; done
