"""Summarise the PMC passes of tools/gpu_pmc.sh into bytes per row (profiles/traffic.json
entries): counter unit KB (x1024); FETCH_SIZE doubled on gfx950 (MI355X_MICROARCH.md: 128-B
requests tallied at 64 B for wide coalesced reads)."""
import csv
import glob
import json


def total(pattern, counter):
    n = 0
    tot = 0.0
    for path in glob.glob(pattern, recursive=True):
        for r in csv.DictReader(open(path)):
            if r.get("Counter_Name") == counter:
                tot += float(r["Counter_Value"])
                n += 1
    return tot, n


out = {}
c3 = json.load(open("gpurun_out/pmc_c3_FETCH_SIZE.json"))
pred_rows = c3["config"]["rows_per_step"] * c3["breakdown"]["speculation_overhead"] * 3   # step + 2 replays
for key, pat, rows, name in (("ddm_forest_predict", "gpurun_out/pmc_c3_{}/**/*counter_collection.csv", pred_rows,
                              "k_cforest_predict_arg<1,4>"),
                             ("ddm_scan_batches", "gpurun_out/pmc_c4_{}/**/*counter_collection.csv", 4096 * 10 ** 6,
                              "k_scan_prefix_table + k_scan_batches_spec/list/fix")):
    f, nf = total(pat.format("FETCH_SIZE"), "FETCH_SIZE")
    w, nw = total(pat.format("WRITE_SIZE"), "WRITE_SIZE")
    out[key] = {"kernel": name, "dispatches": nf, "rows_covered": rows, "fetch_size_kb": f, "write_size_kb": w,
                "fetch_bytes_per_row_raw": f * 1024 / rows, "fetch_bytes_per_row": 2 * f * 1024 / rows,
                "write_bytes_per_row": w * 1024 / rows, "hbm_bytes_per_row": (2 * f + w) * 1024 / rows}
print(json.dumps(out, indent=1))
json.dump(out, open("gpurun_out/pmc_summary.json", "w"), indent=1)
