#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
tools/gpu_htrace.sh > gpurun_out/ht.txt
head -16 gpurun_out/ht.txt
