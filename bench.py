#!/usr/bin/env python
"""Benchmark: stream rows/s through predict + DDM (BASELINE.json `metric`).

Default workload = BASELINE.json configs[2] per GPU: a synthetic rialto-shaped stream
(27 float32 features, 10 classes in class blocks, noise-free separable classes ->
sparse abrupt drifts; rialto.csv is not shipped) partitioned `row % INSTANCES`
(DDM_Process.py:225) into 8 partitions of 125M rows = 1B rows per GPU, class blocks
of 10,000,037 global rows (~100 drifts per partition, block edges not batch aligned).
One step = every partition of this rank through the full reference hot path
(run_DDM_loop, DDM_Process.py:170-213): batch shuffles from the partition's MT19937,
forest predict + DDM scan on the GPU, refit on every drift (native exact RF refit).
Inputs are resident in HBM before the timed region.  Weak scaling: each rank owns its
own 8 partitions (global ids rank*8 + p, INSTANCES = 8 * world), no collective on the
data path; the per-rank event counts are all-reduced once for the self-check.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c3|c4]
"""
import argparse
import json
import os
import sys
import time

# one HIP stream per partition: give HIP enough hardware queues to run them concurrently
# (HIP's default is 4 per process; must be set before the runtime initialises)
os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "distributed-drift-detection_amd"))
sys.path.insert(0, ROOT)

PEAK_HBM_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s; 6.29 measured copy)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default="c3", choices=["c3", "c4"])
    ap.add_argument("--parts", type=int, default=8, help="partitions per GPU")
    ap.add_argument("--rows-per-part", type=int, default=125_000_000)
    ap.add_argument("--block-rows", type=int, default=10_000_037, help="global class-block length (C3)")
    ap.add_argument("--features", type=int, default=27)
    ap.add_argument("--refit", default="device", choices=["device", "native", "sklearn"],
                    help="device: ddm_rf_fit_device in the epoch that finds the change; native: "
                         "ddm_rf_fit_many on host threads (both identical trees to sklearn 1.7.2); "
                         "sklearn: host sklearn")
    ap.add_argument("--fit-threads", type=int, default=16, help="host threads for the tree-parallel native refits")
    ap.add_argument("--seed", type=int, default=20261015)
    ap.add_argument("--cpu-baseline", type=int, default=1)
    ap.add_argument("--cpu-sample-rows", type=int, default=150_000)
    ap.add_argument("--c4-streams", type=int, default=1_000_000)
    ap.add_argument("--c4-len", type=int, default=4096)
    return ap.parse_args()


def dist_env():
    return int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")), \
        int(os.environ.get("LOCAL_RANK", "0"))


def traffic_from_profile(name, rows_per_launch):
    """HBM bytes per launch from the committed PMC summary (profiles/), or None."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    if not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            d = json.load(f).get(name)
        return None if d is None else d["hbm_bytes_per_row"] * rows_per_launch
    except (OSError, ValueError, KeyError):
        return None


def cpu_baseline_c3(part, n_rows, seed):
    """The oracle's pandas/iterrows restatement of run_DDM_loop (kind "port") on the first
    n_rows of partition 0, one process, n_jobs=1."""
    import numpy as np
    import pandas as pd
    from oracle.controller import run_partition_frames
    n = min(n_rows, part.n)
    X = part.X[:, :n].t().contiguous().cpu().numpy().astype(np.float64)
    y = part.y[:n].cpu().numpy().astype(np.int64)
    feats = [str(i) for i in range(X.shape[1])]
    pdf = pd.DataFrame(X, columns=feats)
    pdf["target"] = y
    pdf["full_df_row_number"] = np.arange(n)
    np.random.seed(seed)
    t0 = time.perf_counter()
    run_partition_frames(pdf, feats, n_jobs=1)
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "rows/s", "cores": 1, "kind": "port",
            "sample": f"first {n} rows of partition 0 of the same workload, oracle/controller.py "
                      f"run_partition_frames (pandas sample + sklearn RF n_jobs=1 + iterrows DDM), "
                      f"{dt:.1f} s"}


def events_rows(out):
    """BatchRunner output (rows x [warning pos, change pos]) as the reference's 4 columns."""
    import numpy as np
    ev = np.full((len(out), 4), -1, dtype=np.int64)
    ev[:, 0] = ev[:, 1] = out[:, 0]
    ev[:, 2] = ev[:, 3] = out[:, 1]
    return ev


def run_c3(args, world, rank, dev, torch, dist):
    import numpy as np
    from ddm_amd import kernels
    from ddm_amd.controller import BatchRunner, DevicePartition
    from ddm_amd.params import DDMSettings
    from ddm_amd.rng import MTStream
    instances = args.parts * world
    block = args.block_rows if world == 1 else (args.block_rows // 8) * instances + 37
    n = args.rows_per_part
    parts = []
    settings = DDMSettings()
    for p in range(args.parts):
        gid = rank * args.parts + p
        part = DevicePartition.allocate(n, args.features, dev)
        kernels.synth_block_labels(part.y[:n], gid, instances, block, 10)
        kernels.synth_features(part.X, part.y[:n], gid, instances, args.seed, 0.04)
        parts.append((gid, part))
    # all partitions of this GPU in lockstep: one batched launch per kernel per epoch
    runner = BatchRunner([p for _, p in parts], settings, torch.cuda.Stream(dev, priority=-1), refit=args.refit, timing=True,
                         fit_threads=args.fit_threads)
    torch.cuda.synchronize()

    results = {}

    n_rows = {r * args.parts + p: (n + 99) // 100 - 1 for r in range(world) for p in range(args.parts)}

    def step():
        outs = runner.run([MTStream.from_seed(args.seed + gid) for gid, _ in parts])
        for (gid, _), o in zip(parts, outs):
            results[gid] = o
        if world > 1:
            # the collect of DDM_Process.py:258: drift/warning positions of every partition
            # on every rank, one RCCL all_gather of the batches with an event
            from ddm_amd.dist import gather_events
            allev = gather_events({gid: events_rows(results[gid]) for gid, _ in parts}, n_rows=n_rows)
            for gid, _ in parts:
                if not np.array_equal(allev[gid], events_rows(results[gid])):
                    raise RuntimeError(f"partition {gid}: gathered events differ")

    for _ in range(args.warmup):
        step()
    ref_events = {g: r.copy() for g, r in results.items()}
    from ddm_amd.controller import RunStats
    runner.stats = RunStats()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        results.clear()
        if k == args.steps - 1:
            runner.predict_log = []           # the last timed step's predict tables (replay below)
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    for g, r in results.items():          # every step reproduces the same events
        if args.warmup and not np.array_equal(r, ref_events[g]):
            raise RuntimeError(f"partition {g}: events differ between steps")
    st = [runner.stats]
    agg = {k: sum(getattr(s, k) for s in st) for k in ("epochs", "refits", "predicted_rows", "refit_s",
                                                        "predict_ms", "predict_bytes", "scan_ms", "scan_rows",
                                                        "shuffle_ms", "host_s", "gpu_s", "refit_fit_s",
                                                        "refit_readback_s", "prep_s", "dfit_ms",
                                                        "device_refits")}
    drifts = int(sum((r[:, 1] >= 0).sum() for r in results.values()))
    warns = int(sum((r[:, 0] >= 0).sum() for r in results.values()))
    rows_rank = n * args.parts * args.steps
    cpu = None
    if rank == 0 and world == 1 and args.cpu_baseline:
        cpu = cpu_baseline_c3(parts[0][1], args.cpu_sample_rows, args.seed)
    launches = max(1, agg["epochs"])
    rows_per_launch = agg["predicted_rows"] / launches
    avg_ms_step = agg["predict_ms"] / launches
    # the kernel's launch duration: the last timed step's launches again, back to back on
    # the epoch stream (HIP events around them).  In the epoch loop the events also time
    # the stream's idle wait for the host before each launch (avg_launch_ms_in_step).
    replay_ms, replay_n = runner.replay_predict(repeats=2)
    runner.predict_log = None
    avg_ms = replay_ms if replay_n else avg_ms_step
    achieved = (agg["predict_bytes"] / launches) / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    info = {
        "workload": f"configs[2]: synthetic rialto-shaped stream, {args.features} f32 features, 10 classes, "
                    f"class blocks of {block} global rows, INSTANCES={instances} (row % INSTANCES), "
                    f"{args.parts} partitions x {n} rows per GPU",
        "rows_per_gpu_step": n * args.parts, "partitions_per_gpu": args.parts,
        "refit": {"device": "ddm_rf_fit_device (sklearn 1.7.2 RandomForestClassifier restated, identical trees) "
                            "on the GPU, one wave per tree, in the epoch that finds the change; each partition's "
                            "first fit on the host",
                  "native": "native ddm_rf_fit_many (sklearn 1.7.2 RandomForestClassifier restated, identical "
                            f"trees), all trees of an epoch's refits on {args.fit_threads} host threads",
                  "sklearn": "host sklearn RandomForestClassifier(100 trees), in-process"}[args.refit],
        "shuffle": "batch shuffles generated on the GPU from the partition's MT19937 stream (ddm_shuffle_*)",
        "execution": "all partitions of the GPU in lockstep epochs: one batched shuffle, predict and scan "
                     "launch per epoch (BatchRunner)",
    }
    extra = {"drifts_per_step": drifts, "warnings_per_step": warns,
             "refits_per_step": agg["refits"] / args.steps, "epochs_per_step": agg["epochs"] / args.steps,
             "speculation_overhead": agg["predicted_rows"] / max(1, rows_rank),
             "refit_s_per_step_sum": agg["refit_s"] / args.steps,
             "predict_kernel_ms_per_step": agg["predict_ms"] / args.steps,
             "scan_kernel_ms_per_step": agg["scan_ms"] / args.steps,
             "shuffle_kernels_ms_per_step": agg["shuffle_ms"] / args.steps,
             "host_s_per_step": agg["host_s"] / args.steps, "gpu_wait_s_per_step": agg["gpu_s"] / args.steps,
             "refit_native_fit_s_per_step": agg["refit_fit_s"] / args.steps,
             "refit_readback_s_per_step": agg["refit_readback_s"] / args.steps,
             "stream_prep_s_per_step": agg["prep_s"] / args.steps,
             "device_refits_per_step": agg["device_refits"] / args.steps,
             "device_refit_kernels_ms_per_step": agg["dfit_ms"] / args.steps}
    roofline = {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": achieved / PEAK_HBM_GBS, "traffic": traffic_from_profile("ddm_forest_predict", rows_per_launch),
                "kernel": "ddm_forest_predict", "alg_bytes_per_row": "4*F_used + 6",
                "avg_launch_ms": avg_ms, "avg_rows_per_launch": rows_per_launch,
                "avg_launch_ms_in_step": avg_ms_step,
                "launch_timing": f"HIP events on the epoch stream around {replay_n} back-to-back launches of the last "
                                 "timed step's predict segment tables (2 passes)"}
    return rows_rank, elapsed, info, extra, roofline, cpu


def run_c4(args, world, rank, dev, torch, dist):
    """configs[3]: 1M independent error streams x 4096 rows, DDM only, fresh DDM after each change."""
    import numpy as np
    from ddm_amd import kernels
    S, L = args.c4_streams, args.c4_len
    err = torch.empty(S * L + 16, dtype=torch.uint8, device=dev)
    kernels.synth_bernoulli_streams(err, S, L, args.seed + rank)
    nb = (L + 99) // 100
    ev = torch.empty((S * nb, 2), dtype=torch.int32, device=dev)
    flags = torch.empty(kernels.scan_batches_scratch_size(S, L), dtype=torch.uint8, device=dev)
    state0 = torch.from_numpy(kernels.fresh_states(S).view(np.uint8)).to(dev)
    state = torch.empty_like(state0)
    prm = kernels.params_struct()
    stream = torch.cuda.current_stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def step(timed):
        state.copy_(state0)
        if timed:
            e0.record(stream)
        kernels.scan_batches(err, S, L, prm, state, ev, flags, stream=stream)
        if timed:
            e1.record(stream)

    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    kms = 0.0
    for _ in range(args.steps):
        step(True)
        torch.cuda.synchronize()
        kms += e0.elapsed_time(e1)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    changes = int((ev[:, 1] >= 0).sum().item())
    rows = S * L * args.steps
    avg_ms = kms / args.steps
    alg = S * L * 1.0 + S * nb * 8
    achieved = alg / (avg_ms * 1e-3) / 1e9
    cpu = None
    if rank == 0 and world == 1 and args.cpu_baseline:
        from oracle.ddm import scan_stream
        e = err[:2000 * L].cpu().numpy()
        t = time.perf_counter()
        k = 0
        while time.perf_counter() - t < 10 and k < 2000:
            scan_stream(e[k * L:(k + 1) * L], mode="restart")
            k += 1
        dt = time.perf_counter() - t
        cpu = {"value": k * L / dt, "unit": "rows/s", "cores": 1, "kind": "port",
               "sample": f"{k} streams x {L} rows, oracle/ddm.py scan_stream (pure-Python DDM, no iterrows)"}
    info = {"workload": f"configs[3]: {S} independent streams x {L} rows (Bernoulli r0~U(.01,.2) stepping "
                        f"by U(.05,.3)), DDM only, fresh DDM at the batch after each change"}
    extra = {"changes_per_step": changes, "scan_kernel_ms": avg_ms}
    roofline = {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": achieved / PEAK_HBM_GBS, "traffic": traffic_from_profile("ddm_scan_batches", S * L),
                "kernel": "ddm_scan_batches", "alg_bytes_per_row": "1 + 8/100",
                "avg_launch_ms": avg_ms,
                "note": "one ddm_scan_batches call: k_scan_prefix_table + k_scan_batches_spec (batch-parallel speculation) + k_scan_batches_list + k_scan_batches_fix (per-stream fix-up); HIP events around the call"}
    return rows, elapsed, info, extra, roofline, cpu


def main():
    args = parse()
    world, rank, local_rank = dist_env()
    import torch
    import torch.distributed as dist
    # DDM_BENCH_BACKEND=gloo with fewer GPUs than ranks rehearses the N>1 path on one box
    # (ranks share a GPU); the driver's runs use RCCL ("nccl"), one GPU per rank
    backend = os.environ.get("DDM_BENCH_BACKEND", "nccl")
    dev = torch.device("cuda", local_rank % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    fn = run_c3 if args.workload == "c3" else run_c4
    rows_rank, elapsed, info, extra, roofline, cpu = fn(args, world, rank, dev, torch, dist)
    if world > 1:
        rdev = dev if backend == "nccl" else torch.device("cpu")
        t = torch.tensor([elapsed], dtype=torch.float64, device=rdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        r = torch.tensor([rows_rank], dtype=torch.float64, device=rdev)
        dist.all_reduce(r)
        rows_total = float(r.item())
    else:
        rows_total = float(rows_rank)
    if rank == 0:
        out = {"metric": "stream rows/sec through predict+DDM (node, 1/2/4/8 GPU) + % HBM roofline",
               "value": rows_total / elapsed, "unit": "rows/s", "n_gpus": world, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
               "scaling": "weak", "vs_baseline": None, "dtype": "f64",
               "data": "synthetic (rialto.csv not shipped); generated in HBM by ddm_synth_*",
               "config": dict(info, parallelism=f"partitions over {world} GPU(s), no data-path collective"),
               "roofline": roofline, "cpu_baseline": cpu, "breakdown": extra}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
