"""Time ddm_scan_batches on configs[3] (1M streams x 4096 rows, the bench's seed) and check
its events / states against the digest of the oracle-checked tree (bench.py c4_checks).

    python tools/c4_scan_time.py [--reps 10] [--label X]      (DDM_AMD_LIB picks a variant)
    python tools/c4_scan_time.py --sweep 'label:ENV=1,ENV2=3' 'label2:...'   (one child each)

Prints one JSON line per configuration: median / min ms per call, the fraction of 8 TB/s
at 1.08 algorithmic B/row, and whether the digest equals the expected one."""
import argparse
import hashlib
import json
import os
import subprocess
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
EXPECT_SHA1 = "e4dcddba8e279e6729f740ffa19da063b6cd39ac"     # round 5, C oracle on every 16th stream equal


def child(a):
    import numpy as np
    import torch
    sys.path.insert(0, os.path.join(ROOT, "distributed-drift-detection_amd"))
    sys.path.insert(0, ROOT)
    import bench
    from ddm_amd import kernels
    S, L = a.streams, 4096
    nb = (L + 99) // 100
    dev = torch.device("cuda", 0)
    err = torch.empty(S * L + 16, dtype=torch.uint8, device=dev)
    kernels.synth_bernoulli_streams(err, S, L, bench.SEED)
    ev = torch.empty((S * nb, 2), dtype=torch.int32, device=dev)
    scratch = torch.empty(kernels.scan_batches_scratch_size(S, L), dtype=torch.uint8, device=dev)
    st0 = torch.from_numpy(kernels.fresh_states(S).view(np.uint8)).to(dev)
    st = torch.empty_like(st0)
    prm = kernels.params_struct()
    s = torch.cuda.current_stream(dev)
    times = []
    for r in range(a.reps + 2):
        st.copy_(st0)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        kernels.scan_batches(err, S, L, prm, st, ev, scratch, stream=s)
        e1.record(s)
        torch.cuda.synchronize()
        if r >= 2:
            times.append(e0.elapsed_time(e1))
    if os.environ.get("DDM_CHAIN_PROF"):   # tuning build: the chain kernel's per-wave profile (last call)
        cp = scratch[-32 * 8192:].cpu().numpy().view(np.uint64).reshape(8192, 4).astype(np.int64)
        cp = cp[cp[:, 0] > 0]
        t0 = cp[:, 0].min()
        dur = (cp[:, 1] - cp[:, 0]) / 100.0          # us (100 MHz)
        order = np.argsort(-dur)
        prof_out = {"waves": int(len(cp)), "span_us": float((cp[:, 1].max() - t0) / 100.0),
                    "start_spread_us": float((cp[:, 0].max() - t0) / 100.0),
                    "dur_us_pct": {str(q): float(np.percentile(dur, q)) for q in (50, 90, 99, 99.9, 100)},
                    "rows_total": int(cp[:, 3].sum()), "streams_total": int(cp[:, 2].sum()),
                    "top": [{"dur_us": float(dur[i]), "start_us": float((cp[i, 0] - t0) / 100.0),
                             "streams": int(cp[i, 2]), "rows": int(cp[i, 3])} for i in order[:12]],
                    "hist_dur_us": np.histogram(dur, bins=[0, 5, 10, 20, 40, 60, 80, 100, 120, 160, 200, 400])[0].tolist()}
        with open(os.environ["DDM_CHAIN_PROF"], "w") as f:
            json.dump(prof_out, f, indent=1)
    ctr = scratch[:16].cpu().numpy().view(np.uint32)
    prof = scratch[64:128].cpu().numpy().view(np.uint64)
    h = hashlib.sha1()
    h.update(ev.cpu().numpy().tobytes())
    h.update(st.cpu().numpy().view(kernels.STATE_DTYPE)[:S].tobytes())
    med = float(np.median(times))
    alg = S * L * 1.08
    out = {"label": a.label, "median_ms": med, "min_ms": min(times), "frac_8TBs": alg / (med * 1e-3) / 8e12,
           "sha1_ok": h.hexdigest() == EXPECT_SHA1 if S == 1_000_000 else None, "sha1": h.hexdigest(),
           "fixup_streams": int(ctr[2]), "spec_runs": int(ctr[3])}
    if prof.any():      # a -DDDM_OP_PROFILE build: one-pass phase cycles summed over the waves (last call)
        names = ["load", "decide", "drain", "walk", "write", "tail", "-", "chunks"]
        tot = float(prof[:6].sum())
        out["phases"] = {n: round(float(v) / tot, 4) for n, v in zip(names[:6], prof[:6])}
        out["chunks"] = int(prof[7])
        out["wave_cycles_per_chunk"] = tot / max(1, int(prof[7]))
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--streams", type=int, default=1_000_000)
    ap.add_argument("--label", default="default")
    ap.add_argument("--sweep", nargs="*")
    a = ap.parse_args()
    if not a.sweep:
        return child(a)
    for spec in a.sweep:
        label, _, envs = spec.partition(":")
        env = dict(os.environ)
        for kv in filter(None, envs.split(",")):
            k, _, v = kv.partition("=")
            env[k] = v
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--reps", str(a.reps), "--streams",
                            str(a.streams), "--label", label], env=env, timeout=180)
        if r.returncode != 0:
            print(json.dumps({"label": label, "rc": r.returncode}), flush=True)
            return r.returncode
    return 0


if __name__ == "__main__":
    sys.exit(main())
