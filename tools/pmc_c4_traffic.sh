#!/bin/bash
# HBM traffic of one ddm_scan_batches call (C4 bench, one step): FETCH_SIZE and WRITE_SIZE in
# separate rocprofv3 --pmc passes; summary per row into gpurun_out/pmc_c4_traffic.json.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf gpurun_out/pmc_c4t_$c
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex "k_scan_batches|k_scan_prefix" --output-format csv -d gpurun_out/pmc_c4t_$c -o p -- python3 bench.py --workload c4 --cpu-baseline 0 --steps 1 --warmup 0 > gpurun_out/pmc_c4t_$c.json 2> gpurun_out/pmc_c4t_$c.err || { tail -20 gpurun_out/pmc_c4t_$c.err; exit 1; }
done
python3 - <<'PY'
import csv, glob, json, collections
rows = 4096 * 10 ** 6
out = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    per = collections.defaultdict(float)
    for path in glob.glob(f"gpurun_out/pmc_c4t_{c}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(path)):
            if r.get("Counter_Name") == c:
                per[r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]] += float(r["Counter_Value"])
    out[c] = dict(per)
f = sum(out["FETCH_SIZE"].values()); w = sum(out["WRITE_SIZE"].values())
out["summary"] = {"fetch_size_kb": f, "write_size_kb": w, "fetch_bytes_per_row": 2 * f * 1024 / rows,
                  "write_bytes_per_row": w * 1024 / rows, "hbm_bytes_per_row": (2 * f + w) * 1024 / rows}
json.dump(out, open("gpurun_out/pmc_c4_traffic.json", "w"), indent=1)
print(json.dumps(out["summary"]))
PY
