#!/bin/bash
# SQ counters of the ddm_scan_batches kernels on the C4 bench (one rocprofv3 --pmc pass).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/pmc_sb
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --kernel-include-regex "scan_batches" --output-format csv -d gpurun_out/pmc_sb -o sb -- python3 bench.py --workload c4 --cpu-baseline 0 --steps 1 --warmup 0 > gpurun_out/pmc_sb.log 2>&1 || { tail -20 gpurun_out/pmc_sb.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
f = glob.glob('gpurun_out/pmc_sb/**/*counter_collection.csv', recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f)):
    nm = r['Kernel_Name'].replace('void ', '').replace('(anonymous namespace)::', '').split('(')[0]
    acc[nm][r['Counter_Name']] += float(r['Counter_Value'])
for nm, c in acc.items():
    print(nm, ' '.join(f"{k}={v:.3g}" for k, v in sorted(c.items())))
PY
