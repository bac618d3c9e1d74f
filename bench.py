#!/usr/bin/env python
"""Benchmark: stream rows/s through predict + DDM (BASELINE.json `metric`).

Workloads (BASELINE.json configs; rialto.csv is not shipped, so every
rialto-shaped stream is synthetic and generated in HBM before the timed region):

  c3  (default) configs[2]: ONE 1B-row rialto-shaped stream (27 float32 features, 10
      noise-free separable classes in class blocks of 10,000,037 global rows -> sparse
      abrupt drifts), split row % 8 (DDM_Process.py:225) into 8 partitions of 125M rows.
      Partition d runs on GPU d % N: the SAME 8 partitions at every GPU
      count, so the events must not depend on N (strong scaling; `events_sha1` below).
  c3w weak-scaling variant: every GPU owns 8 partitions of its own (INSTANCES = 8N).
  c1  configs[0]: rialto-shaped table (82,250 x 27 Dirichlet histograms, 10 classes,
      PCG64 seed 20261015) through the reference's data prep at MULT=2 (164,500 rows,
      stable sort) as ONE partition (INSTANCES=1).
  c4  configs[3]: 1M independent streams x 4096 error bytes, DDM only (ddm_scan_batches).
  c5  configs[4]: 64M rows, class blocks of 150-300 partition rows -> a drift, hence a
      classifier refit, every one or two batches; 8 partitions on GPU d % N; reports
      refits/s and, at N > 1, the all-gather of the drift events.

One step = every partition of this rank through the full reference hot path
(run_DDM_loop, DDM_Process.py:170-213): batch shuffles from the partition's MT19937,
forest predict + DDM scan on the GPU, refit on every drift (device refit, trees
identical to sklearn 1.7.2).  The timed region is bracketed by a barrier and a device
synchronisation, the time is the max over ranks, and `value` = all rows of all ranks /
that time.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c3|c3w|c1|c4|c5]
"""
import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "distributed-drift-detection_amd"))
sys.path.insert(0, ROOT)

PEAK_HBM_GBS = 8000.0      # MI355X HBM3E (MI355X_MICROARCH.md: 8.0 TB/s; ~6.3 measured copy)
PEAK_FP64_VALU_TFLOPS = 78.6   # MI355X FP64 vector
BEST_PUBLISHED_ROWS_S = 25_722.0   # outdoorStream x512, 16 instances x 2 cores
C3_BLOCK = 10_000_037
C3_PARTS = 8
SEED = 20261015


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default="c3", choices=["c3", "c3w", "c1", "c4", "c5"])
    ap.add_argument("--parts", type=int, default=8, help="partitions (INSTANCES) of the c3/c5 stream")
    ap.add_argument("--rows-per-part", type=int, default=125_000_000, help="c3/c3w rows per partition")
    ap.add_argument("--block-rows", type=int, default=C3_BLOCK, help="global class-block length (c3)")
    ap.add_argument("--features", type=int, default=27)
    ap.add_argument("--refit", default="device", choices=["device", "native", "sklearn"])
    ap.add_argument("--fit-threads", type=int, default=16, help="host threads for native refits")
    ap.add_argument("--groups", type=int, default=1,
                    help="partition groups per GPU, each on its own epoch stream and host thread (pipelined)")
    ap.add_argument("--seed", type=int, default=SEED)
    ap.add_argument("--cpu-baseline", type=int, default=1)
    ap.add_argument("--cpu-procs", type=int, default=8, help="CPU baseline worker processes (P)")
    ap.add_argument("--cpu-cores", type=int, default=2, help="CPU baseline CORES = RF n_jobs per process")
    ap.add_argument("--cpu-sample-rows", type=int, default=30_000, help="rows per CPU baseline process")
    ap.add_argument("--oracle-check-rows", type=int, default=40_000,
                    help="rows of partition 0 re-run by the oracle after the timed region (0: off)")
    ap.add_argument("--c4-streams", type=int, default=1_000_000)
    ap.add_argument("--c4-len", type=int, default=4096)
    ap.add_argument("--c5-rows", type=int, default=64_000_000, help="c5 rows (all partitions)")
    ap.add_argument("--c5-flip", type=float, default=0.0, help="c5 label-noise rate")
    ap.add_argument("--solo-world", type=int, default=0,
                    help="measurement aid: run only rank 0's partitions of an N-GPU job (d % N == 0), one "
                         "process, no collective (the per-GPU share of the strong-scaling workloads)")
    return ap.parse_args()


def dist_env():
    return int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")), \
        int(os.environ.get("LOCAL_RANK", "0"))


def traffic_from_profile(name, rows_per_launch):
    """HBM bytes per launch from the committed PMC summary (profiles/traffic.json), or None."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    if not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            d = json.load(f).get(name)
        return None if d is None else d["hbm_bytes_per_row"] * rows_per_launch
    except (OSError, ValueError, KeyError):
        return None


# ---------------------------------------------------------------- CPU baseline (oracle)
# Samples are built from the host mirror of the generators (oracle/synth.py) inside the
# worker processes, which are forked before this process touches the GPU.

def _cpu_sample(spec):
    import numpy as np
    from oracle import synth
    kind, d, n_parts, r0, n, F, seed, extra = spec
    if kind == "c3":
        y = synth.block_labels(r0 + n, d, n_parts, extra, 10)[r0:]
    else:
        y = synth.jitter_labels(r0 + n, d, n_parts, extra[0], extra[1], 10, extra[2], seed)[r0:]
    X = synth.features(y, d + n_parts * r0, n_parts, seed, F)
    return X.astype(np.float64), y.astype(np.int64)


def _cpu_worker(spec_cores):
    """One Spark-task equivalent: the pandas/iterrows port of run_DDM_loop
    (oracle/controller.py run_partition_frames, sklearn RF n_jobs=CORES) on one sample."""
    import numpy as np
    import pandas as pd
    from oracle.controller import run_partition_frames
    spec, cores = spec_cores
    X, y = _cpu_sample(spec)
    feats = [str(i) for i in range(X.shape[1])]
    pdf = pd.DataFrame(X, columns=feats)
    pdf["target"] = y
    pdf["full_df_row_number"] = np.arange(len(y))
    np.random.seed(spec[1] + 1000)
    t0 = time.perf_counter()
    out = run_partition_frames(pdf, feats, n_jobs=cores)
    return len(y), int((out["change_flag_global"] >= 0).sum()), time.perf_counter() - t0


class CpuBaseline:
    """A pool of P worker processes forked at start-up (no HIP context inherited); the
    samples run after the GPU timed region, all P at once, timed from the first dispatch
    to the last result (DDM_Process.py:224-260 minus Spark)."""

    def __init__(self, procs, cores):
        import multiprocessing as mp
        self.procs, self.cores = procs, cores
        self.pool = mp.get_context("fork").Pool(procs)

    def run(self, specs, what):
        t0 = time.perf_counter()
        res = self.pool.map(_cpu_worker, [(s, self.cores) for s in specs], chunksize=1)
        wall = time.perf_counter() - t0
        self.pool.close()
        self.pool.join()
        rows = sum(r[0] for r in res)
        refits = sum(r[1] for r in res)
        return {"value": rows / wall, "unit": "rows/s", "cores": self.procs * self.cores, "kind": "port",
                "procs": self.procs, "CORES": self.cores, "os_cpu_count": os.cpu_count(),
                "refits_per_s": refits / wall, "sample": f"{what}; {len(specs)} samples on {self.procs} processes x "
                                                         f"n_jobs={self.cores}, {rows} rows, {refits} drifts+refits, "
                                                         f"{wall:.1f} s wall"}


def c3_cpu_specs(args, n_parts, block):
    """Per partition: a window of cpu_sample_rows rows centred on the partition's first
    class boundary (the predict, DDM, drift and refit work of the stream)."""
    half = args.cpu_sample_rows // 2
    specs = []
    for d in range(min(n_parts, args.cpu_procs)):
        b = (block - d + n_parts - 1) // n_parts
        specs.append(("c3", d, n_parts, max(0, b - half), args.cpu_sample_rows, args.features, args.seed, block))
    return specs


# ---------------------------------------------------------------- partition workloads

def events_rows(out):
    """BatchRunner output (rows x [warning pos, change pos]) as the reference's 4 columns."""
    import numpy as np
    ev = np.full((len(out), 4), -1, dtype=np.int64)
    ev[:, 0] = ev[:, 1] = out[:, 0]
    ev[:, 2] = ev[:, 3] = out[:, 1]
    return ev


def events_digest(results):
    h = hashlib.sha1()
    for g in sorted(results):
        h.update(str(g).encode())
        h.update(results[g].astype("<i8").tobytes())
    return h.hexdigest()


def c3_property_check(results, n_rows, n_parts, block, pb=100):
    """configs[2] has noise-free separable classes: exactly one drift per class boundary,
    in the batch holding the boundary, and no warning.  Partition d row r is global row
    r * n_parts + d; the first row of class block k in partition d is ceil((k*block - d) / n_parts)."""
    import numpy as np
    for d, r in results.items():
        kmax = (n_rows * n_parts + d) // block
        firsts = [(k * block - d + n_parts - 1) // n_parts for k in range(1, kmax + 1)]
        firsts = [f for f in firsts if pb <= f < n_rows]
        want = np.full(len(r), -1, dtype=np.int64)
        for f in firsts:
            want[f // pb - 1] = f // pb
        got = np.where(r[:, 1] >= 0, r[:, 1] // pb, -1)
        if not np.array_equal(got, want) or (r[:, 0] >= 0).any():
            bad = np.nonzero(got != want)[0][:8]
            raise RuntimeError(f"partition {d}: drifts are not one per class boundary (batches {bad.tolist()}: got "
                               f"{got[bad].tolist()} want {want[bad].tolist()}; warnings at "
                               f"{np.nonzero(r[:, 0] >= 0)[0][:8].tolist()})")
        # the drift row itself is one of the new class's rows of that batch
        for f in firsts:
            c = r[f // pb - 1, 1]
            if not (f <= c < (f // pb + 1) * pb):
                raise RuntimeError(f"partition {d}: drift row {c} before the boundary {f}")


def oracle_prefix_check(part, n, seed, got):
    """The oracle (oracle/controller.py) on the first n rows of a partition must give the
    same events for the batches those rows complete."""
    import numpy as np
    from ddm_amd.synth import host_copy
    from oracle.controller import run_partition
    n = min(n, part.n) // 100 * 100
    if n < 200:
        return None
    X, y = host_copy(part)
    np.random.seed(seed)
    want = run_partition(X[:n], y[:n], np.arange(n), np.arange(n))
    k = len(want)
    if not (np.array_equal(got[:k, 0], want[:, 0]) and np.array_equal(got[:k, 1], want[:, 2])):
        raise RuntimeError("events differ from the oracle on the checked prefix")
    return n


def run_partition_workload(args, world, rank, dev, torch, dist, kind, cpu):
    import numpy as np
    from ddm_amd import synth
    from ddm_amd.controller import BatchRunner, GroupedRunner, RunStats
    from ddm_amd.params import DDMSettings
    from ddm_amd.rng import MTStream
    P = args.parts
    # GPUs the partitions are placed on (solo_world: rank 0's share of an N-GPU job, alone)
    gpus = args.solo_world if args.solo_world > 1 and world == 1 else world
    if kind == "c3":
        instances, block, n = P, args.block_rows, args.rows_per_part
        mine = [d for d in range(instances) if d % gpus == rank]
    elif kind == "c3w":
        instances = P * gpus
        block = args.block_rows if gpus == 1 else (args.block_rows // 8) * instances + 37
        n = args.rows_per_part
        mine = [rank * P + p for p in range(P)]
    else:   # c5
        instances, block, n = P, None, args.c5_rows // P
        mine = [d for d in range(instances) if d % gpus == rank]
    parts = []
    for d in mine:
        if kind == "c5":
            part = synth.jitter_partition(n, d, instances, args.seed, dev, flip=args.c5_flip, n_features=args.features)
        else:
            part = synth.block_partition(n, d, instances, block, args.seed, dev, n_features=args.features)
        parts.append((d, part))
    results = {}
    n_rows = {d: (n + 99) // 100 - 1 for d in range(instances)}
    gather_s = [0.0]
    if not parts:
        raise RuntimeError(f"rank {rank} owns no partition ({instances} partitions over {world} GPUs)")
    if args.groups > 1 and len(parts) > 1:
        # partition groups pipelined on their own epoch streams and host threads
        runner = GroupedRunner([p for _, p in parts], DDMSettings(), groups=args.groups, refit=args.refit,
                               timing=True, fit_threads=args.fit_threads)
    else:
        runner = BatchRunner([p for _, p in parts], DDMSettings(), torch.cuda.Stream(dev, priority=-1),
                             refit=args.refit, timing=True, fit_threads=args.fit_threads)
    torch.cuda.synchronize()

    def step():
        outs = runner.run([MTStream.from_seed(args.seed + d) for d, _ in parts])
        for (d, _), o in zip(parts, outs):
            results[d] = o
        if getattr(runner, "trace", None) and os.environ.get("DDM_HOST_TRACE_OUT"):
            with open(os.environ["DDM_HOST_TRACE_OUT"], "w") as f:    # the last run's host phases
                json.dump(runner.trace, f)
        if world > 1:
            # the collect of DDM_Process.py:258: the drift/warning positions of every
            # partition on every rank, one all_gather of the batches with an event
            from ddm_amd.dist import gather_events
            tg = time.perf_counter()
            allev = gather_events({d: events_rows(results[d]) for d, _ in parts}, n_rows=n_rows, comm=args.comm)
            gather_s[0] += time.perf_counter() - tg
            for d, _ in parts:
                if not np.array_equal(allev[d], events_rows(results[d])):
                    raise RuntimeError(f"partition {d}: gathered events differ")
            step.all = allev

    for _ in range(args.warmup):
        step()
    ref_events = {g: r.copy() for g, r in results.items()}
    runner.stats = RunStats()
    gather_s[0] = 0.0
    # the timed steps enqueue no timing events; the kernel times come from one instrumented
    # step after them
    runner.set_kernel_timing(False)
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
    st_timed = runner.stats
    runner.stats = RunStats()
    runner.set_kernel_timing(True)
    log = runner.predict_log
    runner.predict_log = None
    step()                                # instrumented, not timed
    st_kern = runner.stats
    runner.stats = st_timed
    runner.predict_log = log
    for g, r in results.items():
        if not np.array_equal(r, ref_events.get(g, r)):
            raise RuntimeError(f"partition {g}: events differ in the instrumented step")
    checks = {}
    if kind == "c3":
        c3_property_check(results, n, instances, block)
        checks["property"] = "one drift per class boundary, in the batch holding it, no warning: ok"
    if args.oracle_check_rows and rank == 0:
        d0, p0 = parts[0]
        k = oracle_prefix_check(p0, args.oracle_check_rows, args.seed + d0, results[d0])
        if k:
            checks["oracle_prefix"] = f"partition {d0}: first {k} rows == oracle/controller.py"
    all_events = getattr(step, "all", None) if world > 1 else {d: events_rows(r) for d, r in results.items()}
    if all_events is not None:
        checks["events_sha1"] = events_digest(all_events)
    st = runner.stats
    agg = {k: getattr(st, k) for k in ("epochs", "refits", "predicted_rows", "predict_bytes", "host_s", "gpu_s",
                                       "device_refits", "prep_s")}
    # kernel times of one step (the instrumented one), scaled to the timed steps
    for k in ("predict_ms", "scan_ms", "shuffle_ms", "dfit_ms"):
        agg[k] = getattr(st_kern, k) * args.steps
    agg["predict_bytes"] = st_kern.predict_bytes * args.steps
    drifts = int(sum((r[:, 1] >= 0).sum() for r in results.values()))
    warns = int(sum((r[:, 0] >= 0).sum() for r in results.values()))
    rows_rank = n * len(parts) * args.steps
    launches = max(1, agg["epochs"])
    rows_per_launch = agg["predicted_rows"] / launches
    avg_ms_step = agg["predict_ms"] / launches
    replay_ms, replay_n = runner.replay_predict(repeats=2)
    runner.predict_log = None
    runner.close()
    avg_ms = replay_ms if replay_n else avg_ms_step
    achieved = (agg["predict_bytes"] / launches) / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    if kind == "c5":
        wl = (f"configs[4]: {args.c5_rows} rows, {args.features} f32 features, class blocks of 150-300 partition rows "
              f"(global boundaries every 1800 +- 300 rows), label noise {args.c5_flip}, INSTANCES={instances}")
    elif kind == "c3":
        wl = (f"configs[2]: one {n * instances}-row rialto-shaped stream, {args.features} f32 features, 10 classes, "
              f"class blocks of {block} global rows, INSTANCES={instances} (row % INSTANCES), partition d on GPU d % N")
    else:
        wl = (f"configs[2] weak-scaling variant: {P} partitions x {n} rows per GPU, INSTANCES={instances}, "
              f"class blocks of {block} global rows")
    info = {"workload": wl, "rows_per_step": n * instances if kind != "c3w" else n * P * gpus,
            "partitions": instances, "partitions_this_rank": len(parts),
            "solo_share_of_gpus": gpus if gpus != world else None,
            "refit": "ddm_rf_fit_device (sklearn 1.7.2 RandomForestClassifier restated, identical trees) on the GPU",
            "execution": (f"the GPU's partitions in {min(args.groups, len(parts))} groups (GroupedRunner), each in "
                          "lockstep epochs on its own stream and host thread: one batched shuffle, predict, scan, "
                          "stage and refit launch per group epoch" if min(args.groups, len(parts)) > 1 else
                          "all partitions of the GPU in lockstep epochs (BatchRunner): one batched shuffle, predict, "
                          "scan, stage and refit launch per epoch")}
    extra = {"drifts_per_step": drifts, "warnings_per_step": warns,
             "refits_per_step": agg["refits"] / args.steps, "epochs_per_step": agg["epochs"] / args.steps,
             "refits_per_s": agg["refits"] / elapsed,
             "speculation_overhead": agg["predicted_rows"] / max(1, rows_rank),
             "predict_kernel_ms_per_step": agg["predict_ms"] / args.steps,
             "scan_kernel_ms_per_step": agg["scan_ms"] / args.steps,
             "shuffle_kernels_ms_per_step": agg["shuffle_ms"] / args.steps,
             "device_refit_kernels_ms_per_step": agg["dfit_ms"] / args.steps,
             "host_s_per_step": agg["host_s"] / args.steps, "gpu_wait_s_per_step": agg["gpu_s"] / args.steps,
             "stream_prep_s_per_step": agg["prep_s"] / args.steps,
             "kernel_ms_from": "one instrumented step after the timed ones (HIP events around each launch)",
             "gather_ms_per_step": gather_s[0] / args.steps * 1e3 if world > 1 else None,
             "gather_backend": (None if world == 1 else "rccl (ctypes ncclAllGather, HBM to HBM)" if args.comm
                                else "torch.distributed all_gather"),
             "checks": checks}
    roofline = {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": achieved / PEAK_HBM_GBS, "traffic": traffic_from_profile("ddm_forest_predict", rows_per_launch),
                "kernel": "ddm_forest_predict", "alg_bytes_per_row": "4*F_used + 6",
                "avg_launch_ms": avg_ms, "avg_rows_per_launch": rows_per_launch,
                "avg_launch_ms_in_step": avg_ms_step,
                "launch_timing": f"HIP events on the epoch stream around {replay_n} back-to-back launches of the last "
                                 "timed step's predict segment tables (2 passes)"}
    cpu_res = None
    if cpu is not None:
        if kind == "c5":
            specs = [("c5", d, instances, 0, args.cpu_sample_rows, args.features, args.seed,
                      (synth.C5_PERIOD, synth.C5_JITTER, args.c5_flip)) for d in range(min(instances, cpu.procs))]
            cpu_res = cpu.run(specs, f"first {args.cpu_sample_rows} rows of each partition of the c5 stream")
        else:
            cpu_res = cpu.run(c3_cpu_specs(args, instances, block),
                              f"{args.cpu_sample_rows} rows around each partition's first class boundary "
                              f"(one drift + refit each) of the c3 stream")
    scaling = "weak" if kind == "c3w" else "strong"
    return rows_rank, elapsed, info, extra, roofline, cpu_res, scaling


def run_c1(args, world, rank, dev, torch, dist, cpu):
    """configs[0]: the rialto-shaped table through the data prep at MULT=2, INSTANCES=1."""
    import numpy as np
    from ddm_amd import synth
    from ddm_amd.controller import BatchRunner, DevicePartition, RunStats
    from ddm_amd.params import DDMSettings
    from ddm_amd.rng import MTStream
    table, order, parts = synth.rialto_partitions()
    pa = parts[0]
    part = DevicePartition.from_columns(pa.X32, pa.target, dev)
    runner = BatchRunner([part], DDMSettings(), torch.cuda.Stream(dev, priority=-1), refit=args.refit, timing=True,
                         fit_threads=args.fit_threads)
    torch.cuda.synchronize()
    out = [None]

    def step():
        out[0] = runner.run([MTStream.from_seed(args.seed)])[0]

    for _ in range(args.warmup):
        step()
    ref = None if out[0] is None else out[0].copy()
    runner.stats = RunStats()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if ref is not None and not np.array_equal(ref, out[0]):
        raise RuntimeError("c1: events differ between steps")
    runner.close()
    n = part.n
    checks = {"events_sha1": events_digest({0: events_rows(out[0])})}
    cpu_res = None
    t_or = None
    if cpu is not None or args.oracle_check_rows:
        from oracle.controller import run_partition
        np.random.seed(args.seed)
        t = time.perf_counter()
        want = run_partition(pa.X32.T.astype(np.float64), pa.target, np.arange(n), pa.row_number)
        t_or = time.perf_counter() - t
        if not (np.array_equal(out[0][:, 0], want[:, 0]) and np.array_equal(out[0][:, 1], want[:, 2])):
            raise RuntimeError("c1: events differ from the oracle")
        checks["oracle"] = f"all {n} rows == oracle/controller.py run_partition"
        if cpu is not None:
            cpu_res = {"value": n / t_or, "unit": "rows/s", "cores": 1, "kind": "port", "procs": 1, "CORES": 1,
                       "os_cpu_count": os.cpu_count(),
                       "sample": f"the whole c1 partition ({n} rows), oracle/controller.py run_partition (numpy "
                                 f"batches, sklearn RF n_jobs=1, DDM restated), {t_or:.1f} s"}
    st = runner.stats
    launches = max(1, st.epochs)
    info = {"workload": f"configs[0]: rialto-shaped table {synth.C1_ROWS} x {synth.C1_FEATURES} Dirichlet histograms "
                        f"(PCG64 seed {synth.C1_SEED}), MULT=2 -> {n} rows, stable sort by target, INSTANCES=1",
            "rows_per_step": n, "partitions": 1}
    extra = {"drifts_per_step": int((out[0][:, 1] >= 0).sum()), "warnings_per_step": int((out[0][:, 0] >= 0).sum()),
             "epochs_per_step": st.epochs / args.steps, "refits_per_step": st.refits / args.steps,
             "predict_kernel_ms_per_step": st.predict_ms / args.steps, "checks": checks}
    avg_ms = st.predict_ms / launches
    achieved = (st.predict_bytes / launches) / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    roofline = {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": achieved / PEAK_HBM_GBS, "traffic": None, "kernel": "ddm_forest_predict",
                "alg_bytes_per_row": "4*F_used + 6", "avg_launch_ms": avg_ms,
                "avg_rows_per_launch": st.predicted_rows / launches,
                "launch_timing": "HIP events around each in-step launch (includes idle stream gaps)"}
    return n * args.steps, elapsed, info, extra, roofline, cpu_res, "replicas"


def run_c4(args, world, rank, dev, torch, dist, cpu):
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
    cpu_res = None
    if rank == 0 and world == 1 and args.cpu_baseline:
        from oracle.ddm import scan_stream
        e = err[:2000 * L].cpu().numpy()
        t = time.perf_counter()
        k = 0
        while time.perf_counter() - t < 10 and k < 2000:
            scan_stream(e[k * L:(k + 1) * L], mode="restart")
            k += 1
        dt = time.perf_counter() - t
        cpu_res = {"value": k * L / dt, "unit": "rows/s", "cores": 1, "kind": "port",
                   "sample": f"{k} streams x {L} rows, oracle/ddm.py scan_stream (pure-Python DDM, no iterrows)"}
    info = {"workload": f"configs[3]: {S} independent streams x {L} rows (Bernoulli r0~U(.01,.2) stepping "
                        f"by U(.05,.3)), DDM only, fresh DDM at the batch after each change"}
    rows_s = S * L / (avg_ms * 1e-3)
    extra = {"changes_per_step": changes, "scan_kernel_ms": avg_ms}
    roofline = {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": achieved / PEAK_HBM_GBS, "traffic": traffic_from_profile("ddm_scan_batches", S * L),
                "kernel": "ddm_scan_batches", "alg_bytes_per_row": "1 + 8/100",
                "avg_launch_ms": avg_ms,
                "fp64_valu_roof": {"rows_per_s_at_roof": PEAK_FP64_VALU_TFLOPS * 1e12 / 2 / 45,
                                   "achieved_rows_per_s": rows_s,
                                   "note": "straightforward form ~45 fp64 VALU instructions per scanned row "
                                           "(SURVEY §8d); the batch-parallel form skips most rows"},
                "note": "one ddm_scan_batches call: k_scan_prefix_table + k_scan_batches_classify + "
                        "k_scan_batches_exact<0> + k_scan_batches_exact<1> + k_scan_batches_walk + "
                        "k_scan_batches_chain; HIP events around the call"}
    return rows, elapsed, info, extra, roofline, cpu_res, "weak"


def main():
    args = parse()
    world, rank, local_rank = dist_env()
    if args.solo_world > 1 and world == 1:
        args.cpu_baseline = 0
    cpu = None
    if args.cpu_baseline and rank == 0 and world == 1 and args.workload in ("c3", "c3w", "c5"):
        cpu = CpuBaseline(args.cpu_procs, args.cpu_cores)     # forked before any HIP call
    import torch
    import torch.distributed as dist
    # DDM_BENCH_BACKEND=gloo with fewer GPUs than ranks rehearses the N>1 path on one box
    # (ranks share a GPU); the driver's runs use RCCL ("nccl"), one GPU per rank
    backend = os.environ.get("DDM_BENCH_BACKEND", "nccl")
    dev = torch.device("cuda", local_rank % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    comm = None
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
            # the event collect runs on RCCL itself (ctypes), torch.distributed only for the
            # rendezvous, the barrier and the timing reduction
            try:
                from ddm_amd.rccl import RcclComm
                comm = RcclComm.from_default_group(dev)
            except Exception as e:      # noqa: BLE001  (reported in the JSON line)
                print(f"rank {rank}: RCCL ctypes communicator unavailable ({e}); gathering over torch.distributed",
                      file=sys.stderr)
        else:
            dist.init_process_group(backend)
    args.comm = comm
    if args.workload == "c1":
        res = run_c1(args, world, rank, dev, torch, dist, cpu if rank == 0 and args.cpu_baseline else None)
    elif args.workload == "c4":
        res = run_c4(args, world, rank, dev, torch, dist, cpu)
    else:
        res = run_partition_workload(args, world, rank, dev, torch, dist, args.workload, cpu)
    rows_rank, elapsed, info, extra, roofline, cpu_res, scaling = res
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
        value = rows_total / elapsed
        out = {"metric": "stream rows/sec through predict+DDM (node, 1/2/4/8 GPU) + % HBM roofline",
               "value": value, "unit": "rows/s", "n_gpus": world, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
               "scaling": scaling, "vs_baseline": value / BEST_PUBLISHED_ROWS_S,
               "vs_baseline_basis": "best published reference rows/s (BASELINE.md §1: outdoorStream x512, 16 Spark "
                                    "instances x 2 cores, 25,722 rows/s; different data and hardware)",
               "dtype": "f64",
               "data": "synthetic (rialto.csv not shipped), generated before the timed region",
               "config": dict(info, parallelism=f"partitions over {world} GPU(s), partition d on GPU d % {world}, "
                                                f"no data-path collective"),
               "roofline": roofline, "cpu_baseline": cpu_res, "breakdown": extra}
        print(json.dumps(out), flush=True)
    if comm is not None:
        comm.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
