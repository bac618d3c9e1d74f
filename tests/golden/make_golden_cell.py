"""Golden fixture of the published cell: outdoorStream x512, 16 instances (BASELINE.md,
`Plot Results.ipynb:572`; the only configuration with a published number).

Runs the REFERENCE's own partition function (`DDM_Process.py:170-213`, compiled from the
file's text by make_golden.load_reference_namespace, with the same two shims) on every one
of the 16 partitions, with the data prep of make_golden.prep_stream (data seed 123, stable
sort) and partition seeds 1000 + d -- the same stream bench.py --workload c2 builds.  Runs
only in the build container (it reads /root/reference); the partitions run in a pool of
worker processes forked after the namespace is compiled (outputs do not depend on it: each
partition seeds the global RandomState itself, DDM_Process.py:61-72 runs one worker per
partition too).

Output: tests/golden/outdoor_cfg_m512_i16.npz with every partition's events (int64
[batches - 1, 4], the reference's columns) and the sha1 of the stream order (int32
full_df_row_number order, 2,048,000 entries) instead of the order itself; manifest.json
gets the cell's entry.

Usage:  python tests/golden/make_golden_cell.py [--procs 8]
"""
import argparse
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np
import pandas as pd

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402

MULT, INSTANCES = 512, 16
_NS = None
_PARTS = None


def _run(d):
    part = _PARTS[d][1]
    np.random.seed(mg.BASE_SEED + d)
    t0 = time.time()
    out = _NS["run_DDM_loop"](part)
    ev = out[["warning_flag_local", "warning_flag_global", "change_flag_local",
              "change_flag_global"]].to_numpy().astype(np.int64)
    return d, ev, time.time() - t0


def main():
    global _NS, _PARTS
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=8)
    a = ap.parse_args()
    df = pd.read_csv(mg.CSV)
    n_feat = df.shape[1] - 1
    _NS = mg.load_reference_namespace(n_feat)
    order = mg.prep_stream(df, MULT, mg.DATA_SEED)
    _PARTS = mg.partitions(df, order, INSTANCES)
    blob = {"order_sha1": np.array(mg._sha1(order.astype(np.int32))), "order_len": np.int64(len(order)),
            "mult": MULT, "instances": INSTANCES}
    info = {"order_sha1": mg._sha1(order.astype(np.int32)), "rows": int(len(order))}
    t0 = time.time()
    with mp.get_context("fork").Pool(a.procs) as pool:
        for d, ev, dt in pool.imap_unordered(_run, range(INSTANCES)):
            blob[f"events/{d}"] = ev
            info[str(d)] = {"rows": int(len(ev)), "drifts": int((ev[:, 3] > -1).sum()),
                       "warnings": int((ev[:, 1] > -1).sum()), "sha1": mg._sha1(ev), "seconds": round(dt, 1)}
            print(f"partition {d}: {info[str(d)]}", flush=True)
    info["wall_seconds"] = round(time.time() - t0, 1)
    info["procs"] = a.procs
    np.savez_compressed(os.path.join(HERE, f"outdoor_cfg_m{MULT}_i{INSTANCES}.npz"), **blob)
    mpath = os.path.join(HERE, "manifest.json")
    manifest = json.load(open(mpath))
    manifest["configs"][f"m{MULT}_i{INSTANCES}"] = info
    with open(mpath, "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
