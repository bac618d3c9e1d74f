#!/bin/bash
# SQ counters for the C4 scan kernels (one --pmc pass), summed per kernel.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU --kernel-include-regex 'scan_batches' --output-format csv -d gpurun_out/pmc_c4 -o sq -- python3 bench.py --workload c4 --cpu-baseline 0 --steps 1 --warmup 0 > gpurun_out/pmc_c4.log 2>&1 || { tail -20 gpurun_out/pmc_c4.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
f = glob.glob('gpurun_out/pmc_c4/**/*counter_collection.csv', recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f)):
    acc[r['Kernel_Name'][:60]][r['Counter_Name']] += float(r['Counter_Value'])
for k, v in acc.items():
    print(k)
    for c, x in sorted(v.items()):
        print(f"   {c:24s} {x:.4g}")
PY
