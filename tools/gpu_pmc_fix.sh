#!/bin/bash
# SQ counters of the C4 fix-up kernel.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --kernel-include-regex "scan_batches" --output-format csv -d gpurun_out/pmc_fix -o fx -- python3 bench.py --workload c4 --cpu-baseline 0 --steps 1 --warmup 0 > gpurun_out/pmc_fix.log 2>&1 || { tail -20 gpurun_out/pmc_fix.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
f = glob.glob('gpurun_out/pmc_fix/**/*counter_collection.csv', recursive=True)[0]
agg = collections.defaultdict(float)
for r in csv.DictReader(open(f)):
    k = r['Kernel_Name'].split('(')[0][-26:]
    agg[(k, r['Counter_Name'])] += float(r['Counter_Value'])
for (k, c), v in sorted(agg.items()):
    print(f"{k:28s} {c:22s} {v:.4g}")
PY
