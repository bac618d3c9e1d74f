"""HBM traffic of the C3 epoch kernels from two rocprofv3 PMC passes (tools/gpu.sh `pmc c3 ...`
with `--steps 1 --warmup 0 --predict-replays 0`), as profiles/traffic.json entries.

    python tools/pmc_c3.py [NAME]      (reads gpurun_out/pmc_NAME_{FETCH_SIZE,WRITE_SIZE}/)

Counter unit KB (x1024); FETCH_SIZE doubled per MI355X_MICROARCH.md (gfx950 tallies 128-B
requests at 64 B).  Rows covered: the bench line's device-epoch rows per step (predict) and
permuted rows per step (k_err_permute), times the steps plus the instrumented step."""
import csv
import glob
import json
import sys

name = sys.argv[1] if len(sys.argv) > 1 else "c3"


def per_kernel(counter):
    tot, n = {}, {}
    for path in glob.glob(f"gpurun_out/pmc_{name}_{counter}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(path)):
            if r.get("Counter_Name") != counter:
                continue
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].strip()
            tot[k] = tot.get(k, 0.0) + float(r["Counter_Value"])
            n[k] = n.get(k, 0) + 1
    return tot, n


line = json.loads(open(f"gpurun_out/pmc_{name}_FETCH_SIZE.json").read().strip().splitlines()[-1])
steps = line["steps"] + 1                       # the timed steps + the instrumented one
bd = line["breakdown"]
rows = {"k_cforest_predict_dev": bd["device_predicted_rows_per_step"] * steps,
        "k_err_permute": bd["permute_rows_per_step"] * steps}
fetch, nf = per_kernel("FETCH_SIZE")
write, _ = per_kernel("WRITE_SIZE")
out = {}
for key, kern in (("ddm_forest_predict_dev_rows", "k_cforest_predict_dev"), ("ddm_err_permute", "k_err_permute")):
    kf = [k for k in fetch if k.endswith(kern)]
    if not kf:
        continue
    f, w = fetch[kf[0]], write.get(kf[0], 0.0)
    r = rows[kern]
    out[key] = {"kernel": kern + (" (row-order, decoupled epochs)" if kern.startswith("k_cf") else ""),
                "dispatches": nf[kf[0]], "rows_covered": r, "fetch_size_kb": f, "write_size_kb": w,
                "fetch_bytes_per_row_raw": f * 1024 / r, "fetch_bytes_per_row": 2 * f * 1024 / r,
                "write_bytes_per_row": w * 1024 / r, "hbm_bytes_per_row": (2 * f + w) * 1024 / r,
                "decoupled_row_fraction": line["roofline"].get("decoupled_row_fraction"),
                "command": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) --kernel-include-regex "
                           f"'k_cforest_predict_dev|k_err_permute' -- python3 bench.py --steps 1 --warmup 0 "
                           f"--cpu-baseline 0 --companion 0 --oracle-check-rows 0 --predict-replays 0"}
print(json.dumps(out, indent=1))
json.dump(out, open(f"gpurun_out/pmc_{name}_summary.json", "w"), indent=1)
