#!/bin/bash
# HBM traffic (FETCH_SIZE, WRITE_SIZE: separate passes) of the bench's dominant kernels.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/pmc_traffic
export TMPDIR=/tmp
run() {  # name counter regex bench-args...
  local name=$1 ctr=$2 rx=$3; shift 3
  timeout -s KILL 150 rocprofv3 --pmc $ctr --kernel-include-regex "$rx" --output-format csv -d gpurun_out/pmc_traffic/$name -o $name -- python3 bench.py --cpu-baseline 0 --steps 1 --warmup 0 "$@" > gpurun_out/pmc_traffic/$name.json 2> gpurun_out/pmc_traffic/$name.err || { tail -20 gpurun_out/pmc_traffic/$name.err; exit 1; }
}
run c3_fetch FETCH_SIZE cforest_predict && run c3_write WRITE_SIZE cforest_predict && \
run c4_fetch FETCH_SIZE scan_batches --workload c4 && run c4_write WRITE_SIZE scan_batches --workload c4 || exit 1
python3 - <<'PY'
import csv, glob, json, collections
out = {}
for name in ["c3_fetch", "c3_write", "c4_fetch", "c4_write"]:
    f = glob.glob(f"gpurun_out/pmc_traffic/{name}/**/*counter_collection.csv", recursive=True)[0]
    tot = collections.defaultdict(float); disp = collections.defaultdict(set)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        tot[k] += float(r["Counter_Value"]); disp[k].add(r["Dispatch_Id"])
    bench = json.loads(open(f"gpurun_out/pmc_traffic/{name}.json").read().strip().splitlines()[-1])
    out[name] = {"kb_by_kernel": dict(tot), "dispatches": {k: len(v) for k, v in disp.items()},
                 "roofline": bench["roofline"]}
json.dump(out, open("gpurun_out/pmc_traffic/summary.json", "w"), indent=1)
print(json.dumps(out, indent=1))
PY
