#!/bin/bash
# Rehearsal of the N>1 bench path on a 1-GPU box: 2 ranks share cuda:0, gloo for the
# collectives (RCCL needs one GPU per rank; the driver's N>1 runs use it).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export DDM_BENCH_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 1 --warmup 1 --rows-per-part 20000000 --cpu-baseline 0 > gpurun_out/n2.json 2> gpurun_out/n2.err || { tail -30 gpurun_out/n2.err; exit 1; }
cat gpurun_out/n2.json | cut -c1-400
