#!/usr/bin/env python
"""Benchmark: stream rows/s through predict + DDM (BASELINE.json `metric`).

Workloads (BASELINE.json configs; rialto.csv is not shipped, so every
rialto-shaped stream is synthetic and generated in HBM before the timed region):

  c2  configs[1]: the reference's own outdoorStream (the parsed csv, tests/golden/outdoor.npz)
      through its data prep (DDM_Process.py:42-51: concat x MULT, shuffle, stable sort by
      target; data seed 123 as the fixtures) and row % INSTANCES (:220-226), partition d
      seeded 1000 + d.  Default MULT=512, INSTANCES=16: the published cell (BASELINE.md §1,
      79.6 s = 25,722 rows/s on 16 Spark instances x 2 cores) -> `vs_baseline`.  At MULT in
      {1,2,4} every partition's events are compared with the reference-executed fixtures.
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

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c2|c3|c3w|c1|c4|c5]

--gpus N > 1 without an external launcher starts N ranks itself (torch.distributed.run,
before this process touches the GPU) and exits with their status; under a launcher
WORLD_SIZE must equal N.
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
# published Final Time (s) of DDM_Process.py on outdoorStream, 8gb executors x
# 2 cores, per (MULT_DATA, INSTANCES) (Plot Results.ipynb:325-590)
PUBLISHED_S_2CORES = {
    (1, 4): 12.5, (1, 8): 12.5, (1, 16): 14.7,
    (2, 1): 19.1, (2, 2): 26.1, (2, 4): 15.3, (2, 8): 16.8, (2, 16): 18.6,
    (4, 1): 21.5, (4, 2): 27.7, (4, 4): 32.4, (4, 8): 26.5, (4, 16): 31.3,
    (8, 1): 26.2, (8, 2): 33.6, (8, 4): 61.1, (8, 8): 51.7, (8, 16): 50.0,
    (16, 1): 34.2, (16, 2): 26.8, (16, 4): 64.1, (16, 8): 102.2, (16, 16): 93.9,
    (32, 1): 48.2, (32, 2): 35.0, (32, 4): 55.7, (32, 8): 74.9, (32, 16): 158.2,
    (64, 1): 75.7, (64, 2): 50.0, (64, 4): 47.1, (64, 8): 56.3, (64, 16): 178.1,
    (128, 1): 131.8, (128, 2): 76.3, (128, 4): 74.1, (128, 8): 84.0, (128, 16): 115.3,
    (256, 1): 236.1, (256, 2): 133.2, (256, 4): 125.4, (256, 8): 75.8, (256, 16): 98.4,
    (512, 1): 456.7, (512, 2): 239.9, (512, 4): 222.5, (512, 8): 124.2, (512, 16): 79.6,
}
OUTDOOR_ROWS = 4000
C2_DATA_SEED, C2_BASE_SEED = 123, 1000      # tests/golden/make_golden.py (data seed, np.random.seed(base + d))
C3_BLOCK = 10_000_037
C3_PARTS = 8
SEED = 20261015


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="c3", choices=["c2", "c3", "c3w", "c1", "c4", "c5"])
    ap.add_argument("--c2-mult", type=int, default=512, help="c2 MULT_DATA")
    ap.add_argument("--c2-instances", type=int, default=16, help="c2 INSTANCES")
    ap.add_argument("--c2-cpu-rows", type=int, default=0,
                    help="c2 rows per CPU baseline process (0: the whole partition, i.e. the whole job over P = INSTANCES)")
    ap.add_argument("--companion", type=int, default=1,
                    help="c3 at N=1: also time the c2 published cell on the GPU (reported under 'companion')")
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
    ap.add_argument("--cpu-procs", type=int, default=16,
                    help="CPU baseline worker processes (P); P x CORES = 16 = the GPU box's CPU share per GPU")
    ap.add_argument("--cpu-cores", type=int, default=1,
                    help="CPU baseline CORES = RF n_jobs per process (> 1: joblib threading backend)")
    ap.add_argument("--cpu-sample-rows", type=int, default=90_000, help="rows per CPU baseline process (c5, c4)")
    ap.add_argument("--c3-cpu-rows", type=int, default=400_000,
                    help="rows per CPU baseline process, c3 / c3w (stratified windows of the stream)")
    ap.add_argument("--oracle-check-rows", type=int, default=40_000,
                    help="rows of partition 0 re-run by the oracle after the timed region (0: off)")
    ap.add_argument("--c4-streams", type=int, default=1_000_000)
    ap.add_argument("--c4-len", type=int, default=4096)
    ap.add_argument("--c4-check-stride", type=int, default=16,
                    help="c4: run the C oracle on every k-th stream after the timed calls (1: all, 0: off)")
    ap.add_argument("--c5-rows", type=int, default=64_000_000, help="c5 rows (all partitions)")
    ap.add_argument("--c5-flip", type=float, default=0.0, help="c5 label-noise rate")
    ap.add_argument("--drift-window", type=int, default=0,
                    help="least speculative window after a drift, in batches (0: DDMSettings' default)")
    ap.add_argument("--drift-short", type=int, default=-1,
                    help="concepts of at most this many batches skip that floor (-1: DDMSettings' default)")
    ap.add_argument("--predict-timing", type=int, default=-1,
                    help="device-clock stamps of every predict launch of the timed steps (the roofline's in-step "
                         "time: each launch's span from its first workgroup's start to its last one's end, folded "
                         "by the staging kernel after it); -1: on for c3/c3w, off for the latency-bound c2/c5 "
                         "epochs (a few us of each ~120-us C5 epoch), whose kernel times then come from an "
                         "instrumented step after the timed ones")
    ap.add_argument("--predict-replays", type=int, default=-1,
                    help="isolated back-to-back replays of the instrumented step's predict tables, reported as "
                         "roofline.isolated_replay next to the in-step frac (a side figure; 0 for PMC runs, whose "
                         "rows must be the steps' own); -1: 2 for c3 / c3w, 0 otherwise")
    ap.add_argument("--gc", default="on", choices=["on", "freeze", "off"],
                    help="Python's cyclic garbage collector during the timed steps: on, frozen after setup "
                         "(gc.freeze: the setup's objects leave the collected generations), or off")
    ap.add_argument("--solo-world", type=int, default=0,
                    help="measurement aid: run only rank 0's partitions of an N-GPU job (d %% N == 0), one "
                         "process, no collective (the per-GPU share of the strong-scaling workloads)")
    a = ap.parse_args()
    if a.predict_replays < 0:
        a.predict_replays = 2 if a.workload in ("c3", "c3w") else 0
    return a


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
        y = synth.block_labels(n, d, n_parts, extra, 10, start=r0)
    else:
        y = synth.jitter_labels(r0 + n, d, n_parts, extra[0], extra[1], 10, extra[2], seed)[r0:]
    X = synth.features(y, d + n_parts * r0, n_parts, seed, F)
    return X.astype(np.float64), y.astype(np.int64)


_C2 = {}


def outdoor_stream(mult, instances):
    """configs[1]: the reference's outdoorStream.csv (as pandas parsed it, tests/golden/
    outdoor.npz) through DDM_Process.py:44-51 (seeded, stable sort, as the fixtures) and
    :220-226.  Returns (loader.StreamTable, order, [loader.PartitionArrays]); memoised, and
    built in the parent before the CPU baseline's workers fork, which inherit it."""
    key = (int(mult), int(instances))
    if key not in _C2:
        import numpy as np
        from ddm_amd import loader
        d = np.load(os.path.join(ROOT, "tests", "golden", "outdoor.npz"), allow_pickle=False)
        X, tgt = d["X"], d["target"].astype(np.int64)
        table = loader.StreamTable(np.ascontiguousarray(X.T.astype(np.float32)), tgt,
                                   [str(i) for i in range(X.shape[1])])
        order = loader.prepare_order(table.n_rows, tgt, mult, np.random.RandomState(C2_DATA_SEED), "stable")
        _C2[key] = (table, order, loader.split_partitions(table, order, instances))
    return _C2[key]


def c1_stream():
    """configs[0]'s rialto-shaped table through the data prep (memoised like outdoor_stream)."""
    if "c1" not in _C2:
        from ddm_amd import synth
        _C2["c1"] = synth.rialto_partitions()
    return _C2["c1"]


def _cpu_frame(spec):
    """(frame, feature names, seed) of one CPU-baseline sample."""
    import numpy as np
    import pandas as pd
    if spec[0] == "c2":
        _, mult, inst, k, rows = spec
        table, _, parts = outdoor_stream(mult, inst)
        p = parts[k]
        f = p.frame(table.features)
        return (f.iloc[:rows] if rows else f), table.features, C2_BASE_SEED + p.device_id
    if spec[0] == "c1":
        _, rows, seed = spec
        table, _, parts = c1_stream()
        return parts[0].frame(table.features).iloc[:rows], table.features, seed
    X, y = _cpu_sample(spec)
    feats = [str(i) for i in range(X.shape[1])]
    pdf = pd.DataFrame(X, columns=feats)
    pdf["target"] = y
    pdf["full_df_row_number"] = np.arange(len(y))
    return pdf, feats, spec[1] + 1000


def _cpu_worker(spec_cores):
    """One Spark-task equivalent: the pandas/iterrows port of run_DDM_loop
    (oracle/controller.py run_partition_frames, sklearn RF n_jobs=CORES) on one sample."""
    import numpy as np
    from oracle.controller import run_partition_frames
    spec, cores = spec_cores
    pdf, feats, seed = _cpu_frame(spec)
    np.random.seed(seed)
    t0 = time.perf_counter()
    if cores > 1:
        # joblib's default (loky) backend is refused inside a multiprocessing worker (sklearn
        # then silently runs n_jobs=1): threads make n_jobs=CORES real
        from joblib import parallel_backend
        with parallel_backend("threading", n_jobs=cores):
            out = run_partition_frames(pdf, feats, n_jobs=cores)
    else:
        out = run_partition_frames(pdf, feats, n_jobs=cores)
    return len(pdf), int((out["change_flag_global"] >= 0).sum()), time.perf_counter() - t0


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
        try:
            avail = len(os.sched_getaffinity(0))
        except (AttributeError, OSError):
            avail = None
        busy = sum(r[2] for r in res)
        return {"value": rows / wall, "unit": "rows/s", "cores": self.procs * self.cores, "kind": "port",
                "procs": self.procs, "CORES": self.cores, "os_cpu_count": os.cpu_count(), "cpus_available": avail,
                "per_core_rows_per_s": rows / busy / self.cores if busy > 0 else None,
                "cores_note": (f"{self.procs} worker processes x n_jobs={self.cores} "
                               f"({'joblib threading backend' if self.cores > 1 else 'single-threaded sklearn'}) = "
                               f"{self.procs * self.cores} cores used; the GPU box allots 16 CPUs per GPU, so no "
                               f"whole-node (all {avail} CPUs) leg is run"),
                "refits_per_s": refits / wall, "sample": f"{what}; {len(specs)} samples on {self.procs} processes x "
                                                         f"n_jobs={self.cores}, {rows} rows, {refits} drifts+refits, "
                                                         f"{wall:.1f} s wall (from the first dispatch to the last "
                                                         f"result, sample building included)"}


def c3_cpu_specs(args, n_parts, block, n_rows):
    """One sample per worker process: partition k % n_parts, a window of c3_cpu_rows rows at
    a stratified position (sample j of the partition in the j-th of its equal strata, offset
    by the partition's phase), so that the samples hold class boundaries (drifts + refits) at
    the stream's own density instead of one each.  Each window still starts with the first
    fit, as every partition run does; at 400k rows that fit is ~1-2 % of the sample's time."""
    rows = min(args.c3_cpu_rows, n_rows)
    per = -(-args.cpu_procs // n_parts)              # samples per partition
    specs = []
    for k in range(args.cpu_procs):
        d, j = k % n_parts, k // n_parts
        r0 = int((j + (d + 0.5) / n_parts) / per * (n_rows - rows))
        specs.append(("c3", d, n_parts, r0, rows, args.features, args.seed, block))
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


def c3_property_check(results, n_rows, n_parts, block, pb=100, seeds=None, rng_after=None):
    """configs[2] has noise-free separable classes: exactly one drift per class boundary,
    in the batch holding the boundary, and no warning.  Partition d row r is global row
    r * n_parts + d; the first row of class block k in partition d is ceil((k*block - d) / n_parts).

    With `seeds` ({partition: seed}) the exact drift ROW is pinned too: the DDM carried
    through the old class's zero errors is trivial (p = s = p_min = s_min = 0), so the
    reference reports the first new-class row of the boundary batch IN SHUFFLED ORDER
    (DDM_Process.py:144-152); that order comes from replaying the partition's MT19937
    draws (oracle/mt_replay.c: a permutation per batch, 100 seeds per refit after the
    next batch's shuffle).  With `rng_after` ({partition: MTStream} after the run) the
    generator position handed back must be the replay's as well."""
    import numpy as np
    replays = {}
    if seeds is not None:
        # the replays (about 3 s of C per 125M-row partition) on threads, beside the checks
        from concurrent.futures import ThreadPoolExecutor
        from oracle.replay import mt_replay
        pool = ThreadPoolExecutor(max(1, min(8, len(results))))
        for d in results:
            kmax = (n_rows * n_parts + d) // block
            ch = [f // pb for f in ((k * block - d + n_parts - 1) // n_parts for k in range(1, kmax + 1))
                  if pb <= f < n_rows]
            replays[d] = pool.submit(mt_replay, seeds[d], n_rows, ch, ch, pb)
        pool.shutdown(wait=False)
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
        if seeds is None:
            continue
        changes = [f // pb for f in firsts]
        perms, key, pos = replays[d].result()
        prev = 0
        for f in firsts:
            b = f // pb
            if b - prev < 2:
                raise RuntimeError(f"partition {d}: class blocks too short for the trivial-detector argument")
            prev = b
            rows = b * pb + perms[b]
            exp = int(rows[np.argmax(rows >= f)])        # first new-class row in DDM order
            if r[b - 1, 1] != exp:
                raise RuntimeError(f"partition {d}: drift row {r[b - 1, 1]} in batch {b}, the first new-class row "
                                   f"in shuffled order is {exp}")
        if rng_after is not None:
            g = rng_after[d]
            if not (np.array_equal(g.key, key) and int(g.pos.value) == pos):
                raise RuntimeError(f"partition {d}: RNG position after the run differs from the replay")


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
    from ddm_amd.controller import BatchRunner, DevicePartition, GroupedRunner, RunStats
    from ddm_amd.params import DDMSettings
    from ddm_amd.rng import MTStream
    P = args.parts
    # GPUs the partitions are placed on (solo_world: rank 0's share of an N-GPU job, alone)
    gpus = args.solo_world if args.solo_world > 1 and world == 1 else world
    seed_base = args.seed
    c2parts = None
    if kind == "c2":
        table, _, allp = outdoor_stream(args.c2_mult, args.c2_instances)
        c2parts = {p.device_id: p for p in allp}
        instances, block, n = args.c2_instances, None, None
        mine = [d for d in sorted(c2parts) if d % gpus == rank]
        seed_base = C2_BASE_SEED
    elif kind == "c3":
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
        if kind == "c2":
            part = DevicePartition.from_columns(c2parts[d].X32, c2parts[d].target, dev)
        elif kind == "c5":
            part = synth.jitter_partition(n, d, instances, args.seed, dev, flip=args.c5_flip, n_features=args.features)
        else:
            part = synth.block_partition(n, d, instances, block, args.seed, dev, n_features=args.features)
        parts.append((d, part))
    results = {}
    if kind == "c2":
        n_rows = {d: (len(p.target) + 99) // 100 - 1 for d, p in c2parts.items()}
    else:
        n_rows = {d: (n + 99) // 100 - 1 for d in range(instances)}
    gather_s = [0.0]
    if not parts:
        raise RuntimeError(f"rank {rank} owns no partition ({instances} partitions over {world} GPUs)")
    settings = DDMSettings()
    if args.drift_window > 0:
        settings.drift_window_batches = args.drift_window
    if args.drift_short >= 0:
        settings.drift_window_short = args.drift_short
    if args.groups > 1 and len(parts) > 1:
        # partition groups pipelined on their own epoch streams and host threads
        runner = GroupedRunner([p for _, p in parts], settings, groups=args.groups, refit=args.refit,
                               timing=True, fit_threads=args.fit_threads)
    else:
        runner = BatchRunner([p for _, p in parts], settings, torch.cuda.Stream(dev, priority=-1),
                             refit=args.refit, timing=True, fit_threads=args.fit_threads)
    torch.cuda.synchronize()

    rngs = {}

    def step():
        streams = [MTStream.from_seed(seed_base + d) for d, _ in parts]
        step.calls = getattr(step, "calls", 0) + 1
        prof = None
        if os.environ.get("DDM_CPROFILE_OUT") and step.calls == 2:
            # developer knob: the second run under cProfile (host-time breakdown of a run)
            import cProfile
            prof = cProfile.Profile()
            prof.enable()
        tr = time.perf_counter()
        outs = runner.run(streams)
        tr = time.perf_counter() - tr
        if prof is not None:
            prof.disable()
            import pstats
            with open(os.environ["DDM_CPROFILE_OUT"], "w") as f:
                pstats.Stats(prof, stream=f).sort_stats("tottime").print_stats(60)
        for (d, _), o, g in zip(parts, outs, streams):
            results[d] = o
            rngs[d] = g
        step.run_ms = tr * 1e3
        if getattr(runner, "trace", None) and os.environ.get("DDM_HOST_TRACE_OUT"):
            step.n = getattr(step, "n", 0) + 1
            with open(f"{os.environ['DDM_HOST_TRACE_OUT']}.{step.n}", "w") as f:    # every run's host phases
                # t_run: the run's start on CLOCK_MONOTONIC (perf_counter), to align the marks
                # with a kernel trace's timestamps
                json.dump({"t_run": getattr(runner, "_t_run", None), "marks": runner.trace}, f)
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
    # the predict launches of the timed steps are timed on the device clock (devctl.PredictTimer:
    # each launch's first workgroups stamp their start and every workgroup its end, and the
    # staging kernel after it folds the span into a running sum); without it (c2 / c5 by
    # default) the instrumented step's HIP events around each predict are the fallback
    timed_predicts = args.predict_timing if args.predict_timing >= 0 else int(kind in ("c3", "c3w"))
    runner.set_predict_timing(bool(timed_predicts))
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    allocs0 = torch.cuda.memory_stats(dev).get("num_device_alloc", 0)
    import gc
    if args.gc != "on":
        gc.collect()
        gc.freeze()
        if args.gc == "off":
            gc.disable()
    step_ms, step_epochs, run_ms = [], [], []
    t0 = time.perf_counter()
    for k in range(args.steps):
        ts = time.perf_counter()
        results.clear()
        step()                            # returns with the run's outputs on the host
        step_ms.append((time.perf_counter() - ts) * 1e3)
        step_epochs.append(runner.stats.epochs)
        run_ms.append(step.run_ms)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    timed_allocs = torch.cuda.memory_stats(dev).get("num_device_alloc", 0) - allocs0
    if args.gc != "on":
        gc.enable()
        gc.unfreeze()
    runner.set_predict_timing(False)
    for g, r in results.items():          # every step reproduces the same events
        if args.warmup and not np.array_equal(r, ref_events[g]):
            raise RuntimeError(f"partition {g}: events differ between steps")
    st_timed = runner.stats
    runner.stats = RunStats()
    runner.set_kernel_timing(True)
    runner.predict_log = [] if args.predict_replays else None   # its predict tables (the replays below)
    step()                                # instrumented, not timed
    st_kern = runner.stats
    runner.stats = st_timed
    for g, r in results.items():
        if not np.array_equal(r, ref_events.get(g, r)):
            raise RuntimeError(f"partition {g}: events differ in the instrumented step")
    checks = {}
    fixture = None
    if kind == "c2":
        fixture = c2_fixture_check(args.c2_mult, instances, c2parts, results)
        if fixture:
            checks["fixtures"] = fixture
    if kind == "c3":
        c3_property_check(results, n, instances, block, seeds={d: seed_base + d for d, _ in parts}, rng_after=rngs)
        checks["property"] = ("one drift per class boundary, in the batch holding it, at the first new-class row in "
                              "shuffled order (oracle/mt_replay.c), no warning; RNG position == the replay: ok")
    if args.oracle_check_rows and rank == 0 and not fixture:
        d0, p0 = parts[0]
        k = oracle_prefix_check(p0, args.oracle_check_rows, seed_base + d0, results[d0])
        if k:
            checks["oracle_prefix"] = f"partition {d0}: first {k} rows == oracle/controller.py"
    all_events = getattr(step, "all", None) if world > 1 else {d: events_rows(r) for d, r in results.items()}
    if all_events is not None:
        checks["events_sha1"] = events_digest(all_events)
    st = runner.stats
    agg = {k: getattr(st, k) for k in ("epochs", "refits", "predicted_rows", "predict_bytes", "host_s", "gpu_s",
                                       "device_refits", "prep_s", "device_epochs", "device_phases", "permute_rows",
                                       "device_rows", "predict_dev_ms", "predict_dev_launches",
                                       "device_predict_bytes")}
    # kernel times of one step (the instrumented one), scaled to the timed steps
    for k in ("predict_ms", "scan_ms", "shuffle_ms", "dfit_ms"):
        agg[k] = getattr(st_kern, k) * args.steps
    agg["predict_bytes"] = st_kern.predict_bytes * args.steps
    drifts = int(sum((r[:, 1] >= 0).sum() for r in results.values()))
    warns = int(sum((r[:, 0] >= 0).sum() for r in results.values()))
    rows_rank = sum(p.n for _, p in parts) * args.steps
    if agg["predict_dev_launches"]:
        launches = agg["predict_dev_launches"]
        rows_per_launch = agg["device_rows"] / launches
        avg_ms_step = agg["predict_dev_ms"] / launches
        dev_bytes = agg["device_predict_bytes"]
    else:       # no predict timing in the timed steps (c2 / c5 by default, or host-planned epochs only):
        # the instrumented step's HIP events around each epoch's predict
        launches = max(1, agg["epochs"])
        rows_per_launch = agg["predicted_rows"] / launches
        avg_ms_step = agg["predict_ms"] / launches
        dev_bytes = agg["predict_bytes"]
    replay_ms, replay_n = runner.replay_predict(repeats=args.predict_replays) if args.predict_replays else (0.0, 0)
    runner.predict_log = None
    runner.close()
    # headline: the timed steps' own predict launches on the device clock (the side stream's
    # shuffles co-running), or the instrumented step's HIP events when that is off; the
    # isolated back-to-back replays of the same tables (in the form the epochs ran them) are a
    # side figure
    avg_ms = avg_ms_step
    bytes_launch = dev_bytes / launches
    achieved = bytes_launch / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    replay_gbs = bytes_launch / (replay_ms * 1e-3) / 1e9 if replay_n and replay_ms > 0 else None
    if kind == "c2":
        wl = (f"configs[1]: outdoorStream.csv (the reference's file, 4000 x 21) x MULT={args.c2_mult} "
              f"({OUTDOOR_ROWS * args.c2_mult} rows; concat, shuffle with data seed {C2_DATA_SEED}, stable sort by "
              f"target), INSTANCES={instances} (row % INSTANCES), partition d seeded {C2_BASE_SEED} + d, on GPU d % N")
    elif kind == "c5":
        wl = (f"configs[4]: {args.c5_rows} rows, {args.features} f32 features, class blocks of 150-300 partition rows "
              f"(global boundaries every 1800 +- 300 rows), label noise {args.c5_flip}, INSTANCES={instances}")
    elif kind == "c3":
        wl = (f"configs[2]: one {n * instances}-row rialto-shaped stream, {args.features} f32 features, 10 classes, "
              f"class blocks of {block} global rows, INSTANCES={instances} (row % INSTANCES), partition d on GPU d % N")
    else:
        wl = (f"configs[2] weak-scaling variant: {P} partitions x {n} rows per GPU, INSTANCES={instances}, "
              f"class blocks of {block} global rows")
    info = {"workload": wl, "rows_per_step": (OUTDOOR_ROWS * args.c2_mult if kind == "c2" else
                                              n * instances if kind != "c3w" else n * P * gpus),
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
             "device_epochs_per_step": agg["device_epochs"] / args.steps,
             "device_phases_per_step": agg["device_phases"] / args.steps,
             "refits_per_s": agg["refits"] / elapsed,
             "speculation_overhead": agg["predicted_rows"] / max(1, rows_rank),
             "device_predicted_rows_per_step": agg["device_rows"] / args.steps,
             "permute_rows_per_step": agg["permute_rows"] / args.steps,
             "predict_kernel_ms_per_step": agg["predict_dev_ms"] / args.steps if agg["predict_dev_launches"] else
             agg["predict_ms"] / args.steps,
             "scan_kernel_ms_per_step": agg["scan_ms"] / args.steps,
             "shuffle_kernels_ms_per_step": agg["shuffle_ms"] / args.steps,
             "stream_generation": stream_generation(st_kern),
             "device_refit_kernels_ms_per_step": agg["dfit_ms"] / args.steps,
             "host_s_per_step": agg["host_s"] / args.steps, "gpu_wait_s_per_step": agg["gpu_s"] / args.steps,
             "stream_prep_s_per_step": agg["prep_s"] / args.steps,
             "timed_step_ms": [round(v, 3) for v in step_ms],
             "timed_step_epochs": [b - a for a, b in zip([0] + step_epochs[:-1], step_epochs)],
             "timed_step_run_ms": [round(v, 3) for v in run_ms],
             "device_allocs_in_timed_steps": timed_allocs,
             "kernel_ms_from": "one instrumented step after the timed ones (HIP events around each launch)",
             "gather_ms_per_step": gather_s[0] / args.steps * 1e3 if world > 1 else None,
             "gather_backend": args.gather_backend,
             "checks": checks}
    dec_frac = agg["permute_rows"] / max(1, agg["device_rows"])
    kname = "k_cforest_predict_dev" if dec_frac < 0.5 else "k_cforest_predict_dev (row order)"
    tkey = "ddm_forest_predict_dev_rows" if dec_frac >= 0.5 else "ddm_forest_predict_dev"
    roofline = {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": achieved / PEAK_HBM_GBS, "traffic": traffic_from_profile(tkey, rows_per_launch),
                "traffic_key": tkey, "kernel": kname,
                "alg_bytes_per_row": "4*F_used + 4 (label) + 1 (error written) + 1 (permutation read, coupled epochs "
                                     "only; decoupled epochs leave the permutation to k_err_permute)",
                "alg_bytes_per_launch": bytes_launch, "avg_launch_ms": avg_ms, "avg_rows_per_launch": rows_per_launch,
                "launches": agg["predict_dev_launches"], "decoupled_row_fraction": dec_frac,
                "launch_timing": ("the device clock (100 MHz) over every device-epoch predict launch of the timed "
                                  "steps, from the launch's first workgroup start to its last workgroup end "
                                  "(ddm_ctl.predict_clock; launches with no rows -- epochs enqueued after a run's "
                                  "last active one -- included, as in a rocprofv3 average; the run's first, "
                                  "host-planned epoch is a different kernel and excluded)"
                                  if agg["predict_dev_launches"] else
                                  "HIP events around each epoch's predict in one instrumented step after the timed "
                                  "ones (no events in the timed steps: --predict-timing 0)"),
                "isolated_replay": {"avg_launch_ms": replay_ms if replay_n else None, "launches": replay_n,
                                    "achieved": replay_gbs,
                                    "frac": replay_gbs / PEAK_HBM_GBS if replay_gbs else None,
                                    "note": "the instrumented step's segment tables replayed back to back in the "
                                            "form each epoch ran them (row order for decoupled epochs, the "
                                            "permutation read for coupled ones), nothing co-running"},
                "k_err_permute": {"rows_per_step": agg["permute_rows"] / args.steps,
                                  "alg_bytes_per_row": "1 (error-free batches before the first error's batch: "
                                                       "zero-fill) to 3 (row-order error read, permutation read, "
                                                       "DDM-order error write)",
                                  "traffic": traffic_from_profile("ddm_err_permute", 1.0)}}
    cpu_res = None
    if cpu is not None:
        if kind == "c2":
            ids = sorted(c2parts)
            specs = [("c2", args.c2_mult, instances, k, args.c2_cpu_rows) for k in range(min(len(ids), cpu.procs))]
            what = f"the first {args.c2_cpu_rows} rows" if args.c2_cpu_rows else "all rows"
            cpu_res = cpu.run(specs, f"{what} of each of {len(specs)} partitions of the same stream (outdoorStream "
                                     f"x{args.c2_mult}, INSTANCES={instances})")
        elif kind == "c5":
            half = args.cpu_sample_rows
            specs = [("c5", k % instances, instances, (k // instances) * half, half, args.features, args.seed,
                      (synth.C5_PERIOD, synth.C5_JITTER, args.c5_flip)) for k in range(cpu.procs)]
            cpu_res = cpu.run(specs, f"{len(specs)} windows of {half} rows (partition k % {instances}, window k // "
                                     f"{instances}) of the c5 stream")
        else:
            cpu_res = cpu.run(c3_cpu_specs(args, instances, block, n),
                              f"windows of {min(args.c3_cpu_rows, n)} rows of the c3 stream at stratified positions "
                              f"(partition k % {instances}, sample k // {instances} in that stratum of the partition: "
                              f"class boundaries at the stream's own density, one per {block // instances} "
                              f"partition rows)")
    scaling = "weak" if kind == "c3w" else "strong"
    return rows_rank, elapsed, info, extra, roofline, cpu_res, scaling


def stream_generation(st):
    """Per step (the instrumented one): the MT19937 stream generation's batched launches on
    their own streams -- k_mt_jump, k_mt_generate_batch, k_fsm_prefix_batch -- with their
    algorithmic bytes (ddm_amd/shuffle.py JUMP_BYTES, GEN_STATE_BYTES, table_bytes_per_chunk)
    and the rate those bytes make over the launches' HIP-event spans, which run beside the
    epochs (so the rates are in-pipeline figures, not the kernels alone)."""
    out = {}
    for kind, units_key, unit in (("jump", "jumps", "jumps"), ("generate", "generate_draws", "draws"),
                                  ("tables", "tables_chunks", "chunks of 8192 draws")):
        ms, nb, units = getattr(st, kind + "_ms"), getattr(st, kind + "_bytes"), getattr(st, units_key)
        out[kind] = {"ms": round(ms, 3), unit: units, "alg_bytes": nb,
                     "GB_per_s": round(nb / (ms * 1e-3) / 1e9, 1) if ms > 0 else None}
    out["kernels"] = {"jump": "k_mt_jump", "generate": "k_mt_generate_batch", "tables": "k_fsm_prefix_batch"}
    return out


def c2_fixture_check(mult, instances, c2parts, results):
    """Every partition's events (reference columns: local = partition position, global =
    full_df_row_number) == the reference-executed fixture of this (MULT, INSTANCES), when
    tests/golden holds one; None otherwise."""
    import numpy as np
    path = os.path.join(ROOT, "tests", "golden", f"outdoor_cfg_m{mult}_i{instances}.npz")
    if not os.path.exists(path):
        return None
    cfg = np.load(path, allow_pickle=False)
    # the stream itself first: its row order (the fixture's order, or for the published
    # cell the sha1 of its 2,048,000 int32 entries) == the one this run built
    order = outdoor_stream(mult, instances)[1].astype(np.int32)
    if "order_sha1" in cfg.files:
        if hashlib.sha1(np.ascontiguousarray(order).tobytes()).hexdigest() != str(cfg["order_sha1"]):
            raise RuntimeError(f"c2 stream order differs from the reference fixture {os.path.basename(path)}")
    elif not np.array_equal(order, cfg["order"]):
        raise RuntimeError(f"c2 stream order differs from the reference fixture {os.path.basename(path)}")
    for d, r in results.items():
        rn = c2parts[d].row_number
        ev = np.full((len(r), 4), -1, dtype=np.int64)
        for c in range(2):
            hit = r[:, c] >= 0
            ev[hit, 2 * c] = r[hit, c]
            ev[hit, 2 * c + 1] = rn[r[hit, c]]
        want = cfg[f"events/{d}"]
        if not np.array_equal(ev, want):
            raise RuntimeError(f"c2 partition {d}: events differ from the reference fixture {os.path.basename(path)}")
    n_ev = sum(len(r) for r in results.values())
    return (f"all {len(results)} partitions ({n_ev} batch records, every event) and the stream order == "
            f"tests/golden/{os.path.basename(path)} (reference-executed)")


def run_c1(args, world, rank, dev, torch, dist, cpu):
    """configs[0]: the rialto-shaped table through the data prep at MULT=2, INSTANCES=1."""
    import numpy as np
    from ddm_amd import synth
    from ddm_amd.controller import BatchRunner, DevicePartition, RunStats
    from ddm_amd.params import DDMSettings
    from ddm_amd.rng import MTStream
    table, order, parts = c1_stream()
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
    if args.oracle_check_rows:
        from oracle.controller import run_partition
        np.random.seed(args.seed)
        want = run_partition(pa.X32.T.astype(np.float64), pa.target, np.arange(n), pa.row_number)
        if not (np.array_equal(out[0][:, 0], want[:, 0]) and np.array_equal(out[0][:, 1], want[:, 2])):
            raise RuntimeError("c1: events differ from the oracle")
        checks["oracle"] = f"all {n} rows == oracle/controller.py run_partition"
    if cpu is not None:
        rows_cpu = min(n, args.cpu_sample_rows // 2)
        cpu_res = cpu.run([("c1", rows_cpu, args.seed)],
                          f"the first {rows_cpu} rows of the c1 partition (configs[0]: one CPU worker)")
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


def c4_checks(args, err, ev, state, S, L, nb, rank):
    """After the timed calls: the digest of the last call's events and states, and the C
    oracle (oracle/scan.py, DDM_Process.py:135-159 with the reset of :207-210) on every
    `--c4-check-stride`-th stream (1: all of them), events and states bit for bit."""
    import numpy as np
    from ddm_amd import kernels
    from oracle.scan import scan_equal_streams
    evh = ev.cpu().numpy()
    sth = state.cpu().numpy().view(kernels.STATE_DTYPE)[:S]
    h = hashlib.sha1()
    h.update(evh.tobytes())
    h.update(sth.tobytes())
    k = max(1, int(args.c4_check_stride))
    sub = err[:S * L].view(S, L)[::k].contiguous().cpu().numpy()
    n = sub.shape[0]
    t = time.perf_counter()
    oev, ost = scan_equal_streams(sub.reshape(-1), n, L, mode=1, threads=16)
    dt = time.perf_counter() - t
    gev = evh.reshape(S, nb, 2)[::k].reshape(-1, 2)
    gst = np.stack([sth["miss_prob"], sth["miss_std"], sth["miss_prob_min"], sth["miss_sd_min"],
                    sth["miss_prob_sd_min"], sth["sample_count"].astype(np.float64),
                    sth["in_concept_change"].astype(np.float64), sth["in_warning_zone"].astype(np.float64)],
                   axis=1)[::k]
    ok_ev = bool(np.array_equal(gev, oev))
    ok_st = bool(np.array_equal(gst, ost))
    if not (ok_ev and ok_st):
        bad = np.nonzero((gev.reshape(n, nb, 2) != oev.reshape(n, nb, 2)).any(axis=(1, 2)))[0]
        print(f"[rank {rank}] c4 oracle check FAILED: {len(bad)} of {n} sampled streams differ "
              f"(first: stream {int(bad[0]) * k if len(bad) else -1}); states equal: {ok_st}", file=sys.stderr)
        raise SystemExit(3)
    return {"events_sha1": h.hexdigest(), "oracle_streams": n, "oracle_stride": k, "oracle_equal": True,
            "oracle_s": dt, "events_sha1_note": "sha1 of the last call's ev int32 [S*nb, 2] then its ddm_state "
                                                "records; oracle_*: oracle/ddm_scan.c on every oracle_stride-th "
                                                "stream, events and states bit for bit"}


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
    checks = c4_checks(args, err, ev, state, S, L, nb, rank) if args.c4_check_stride > 0 else {}
    # rows the DDM actually consumes: a batch is read up to its change (DDM_Process.py:150-152)
    blen = torch.full((nb,), 100, dtype=torch.int64, device=dev)
    blen[-1] = L - 100 * (nb - 1)
    chg = ev[:, 1].view(S, nb).to(torch.int64)
    scanned = int(torch.where(chg >= 0, chg + 1, blen.view(1, nb)).sum().item())
    rows = S * L * args.steps
    avg_ms = kms / args.steps
    alg = S * L * 1.0 + S * nb * 8
    achieved = alg / (avg_ms * 1e-3) / 1e9
    cpu_res = None
    if rank == 0 and args.cpu_baseline:
        # the whole workload on the host: the C restatement of run_DDM in mode 1 (oracle/ddm_scan.c,
        # DDM_Process.py:135-159 with the reset of :207-210) over all S streams, cut into
        # --cpu-procs contiguous runs scanned by as many threads (ctypes drops the GIL)
        from oracle.scan import scan_equal_streams
        eh = err[:S * L].cpu().numpy()
        t = time.perf_counter()
        scan_equal_streams(eh, S, L, per_batch=100, mode=1, threads=args.cpu_procs)
        dt = time.perf_counter() - t
        del eh
        cpu_res = {"value": S * L / dt, "unit": "rows/s", "cores": args.cpu_procs, "kind": "port",
                   "rows_scanned_per_s": scanned / dt,
                   "sample": f"all {S} streams x {L} rows of the workload, oracle/ddm_scan.c (C restatement, each "
                             f"batch up to its change as DDM_Process.py:150-152) on {args.cpu_procs} threads, "
                             f"{dt:.2f} s wall"}
    info = {"workload": f"configs[3]: {S} independent streams x {L} rows (Bernoulli r0~U(.01,.2) stepping "
                        f"by U(.05,.3)), DDM only, fresh DDM at the batch after each change"}
    rows_s = S * L / (avg_ms * 1e-3)
    extra = {"changes_per_step": changes, "scan_kernel_ms": avg_ms, "rows_scanned_per_call": scanned, "checks": checks,
             "rows_scanned_per_s": scanned / (avg_ms * 1e-3),
             "rows_note": "value counts every row of every stream (nominal); rows_scanned counts the rows the DDM "
                          "consumes (each batch up to its change), the same way on the CPU side"}
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


def launch_ranks(args):
    """--gpus N > 1 with no launcher around this process: start N ranks of this same
    command under torch.distributed.run (127.0.0.1, a free port) and return their exit
    status.  Runs before anything here touches the GPU (the children initialise their own)."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    return subprocess.run(cmd, env=env).returncode


def published_cell(workload, args):
    """(rows/s, basis) of the published reference number for this exact workload, or None."""
    if workload != "c2":
        return None
    sec = PUBLISHED_S_2CORES.get((args.c2_mult, args.c2_instances))
    if sec is None:
        return None
    rows = OUTDOOR_ROWS * args.c2_mult
    return rows / sec, (f"BASELINE.md §1 (Plot Results.ipynb:325-590): DDM_Process.py on outdoorStream x{args.c2_mult}, "
                        f"{args.c2_instances} Spark instances x 2 cores, 8gb: {sec} s = {rows / sec:,.0f} rows/s "
                        f"(unspecified CPU cluster)")


def companion_c2(args, rank, dev, torch, dist):
    """The published cell (c2, outdoorStream x512 / 16 instances) on this GPU, after the
    main measurement: GPU rows/s, its vs_baseline and checks, no CPU baseline."""
    import copy
    a = copy.copy(args)
    a.workload, a.steps, a.warmup, a.oracle_check_rows, a.groups = "c2", 3, 1, 12_800, 1
    rows, elapsed, info, extra, roofline, _, _ = run_partition_workload(a, 1, rank, dev, torch, dist, "c2", None)
    value = rows / elapsed
    pub = published_cell("c2", a)
    return {"workload": info["workload"], "value": value, "unit": "rows/s", "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": elapsed / a.steps * 1e3, "vs_baseline": value / pub[0] if pub else None,
            "vs_baseline_basis": pub[1] if pub else None, "epochs_per_step": extra["epochs_per_step"],
            "drifts_per_step": extra["drifts_per_step"], "checks": extra["checks"],
            "predict_roofline_frac": roofline["frac"]}


def keep_freed_outputs_in_heap():
    """glibc serves the runs' dense per-batch outputs (DDM_Process.py:212: one row per batch,
    20 MB per C3 partition) by mmap and, the first time such an array is freed, unmaps its
    pages and raises its dynamic mmap threshold; that one-off munmap of the previous step's
    ~160 MB (7-10 ms) landed in a timed step of most processes (round 4's "slow first step":
    run() itself took its usual time, profiles/r05/slowstep).  With the mmap and
    trim thresholds set up front, large arrays come from the heap and freed ones are reused,
    as they are after that first free anyway."""
    import ctypes
    try:
        libc = ctypes.CDLL("libc.so.6")
    except OSError:
        return False
    M_TRIM_THRESHOLD, M_MMAP_THRESHOLD = -1, -3
    ok = libc.mallopt(M_MMAP_THRESHOLD, 1 << 30) == 1
    return ok and libc.mallopt(M_TRIM_THRESHOLD, 1 << 30) == 1


def bench_line(args, world, rows_total, elapsed, info, extra, roofline, cpu_res, scaling):
    """The driver's JSON line (rank 0): whole-job rows/s over the max-over-ranks time.  At
    N > 1 it carries the same roofline (rank 0's own launches) and CPU baseline (rank 0's
    pool) as at N = 1 and names the collect's backend; a line missing one of them is refused."""
    value = rows_total / elapsed
    pub = published_cell(args.workload, args)
    out = {"metric": "stream rows/sec through predict+DDM (node, 1/2/4/8 GPU) + % HBM roofline",
           "value": value, "unit": "rows/s", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
           "scaling": scaling, "vs_baseline": value / pub[0] if pub else None,
           "vs_baseline_basis": pub[1] if pub else "no published reference number for this workload (the "
                                                   "reference publishes outdoorStream only: --workload c2)",
           "dtype": "f64",
           "data": ("the reference's outdoorStream.csv (parsed, tests/golden/outdoor.npz), resident in HBM "
                    "before the timed region" if args.workload == "c2" else
                    "synthetic (rialto.csv not shipped), generated before the timed region"),
           "config": dict(info, parallelism=f"partitions over {world} GPU(s), partition d on GPU d % {world}, "
                                            f"no data-path collective"),
           "roofline": roofline, "cpu_baseline": cpu_res, "breakdown": extra}
    if world > 1 and args.workload != "c4":
        out["gather_backend"] = extra.get("gather_backend")
    missing = [k for k in ("roofline", "cpu_baseline") if out[k] is None and (k != "cpu_baseline" or args.cpu_baseline)]
    if world > 1 and args.workload != "c4" and not out.get("gather_backend"):
        missing.append("gather_backend")
    if missing:
        raise RuntimeError(f"bench.py: the N={world} line lacks {missing}")
    return out


def main():
    args = parse()
    keep_freed_outputs_in_heap()
    world, rank, local_rank = dist_env()
    if "WORLD_SIZE" in os.environ:
        if args.gpus != world and args.solo_world == 0:
            raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    elif args.gpus > 1:
        sys.exit(launch_ranks(args))
    if args.solo_world > 1 and world == 1:
        args.cpu_baseline = 0
    if args.workload == "c2" or (args.workload == "c3" and args.companion and world == 1):
        outdoor_stream(args.c2_mult, args.c2_instances)      # host data, before the workers fork
    if args.workload == "c1":
        c1_stream()
    cpu = None
    # rank 0's CPU baseline at every N: its pool forks here, before any HIP call, and runs
    # after the timed region while the other ranks wait at the timing reduction
    if args.cpu_baseline and rank == 0 and args.workload in ("c1", "c2", "c3", "c3w", "c5"):
        procs = {"c1": 1, "c2": min(args.cpu_procs, args.c2_instances)}.get(args.workload, args.cpu_procs)
        cpu = CpuBaseline(procs, args.cpu_cores)              # forked before any HIP call
    import torch
    import torch.distributed as dist
    # DDM_BENCH_BACKEND=gloo with fewer GPUs than ranks rehearses the N>1 path on one box
    # (ranks share a GPU); the driver's runs use RCCL ("nccl"), one GPU per rank
    backend = os.environ.get("DDM_BENCH_BACKEND", "nccl")
    dev = torch.device("cuda", local_rank % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    comm = None
    args.gather_backend = None
    if world > 1:
        # ONE GPU communicator per rank: torch.distributed runs on gloo (host memory: the
        # rendezvous, the barriers and the max-over-ranks timing), and the event collect on
        # RCCL itself (ctypes ncclCommInitRank / ncclAllGather, its id through gloo's store)
        dist.init_process_group("gloo")
        if backend == "nccl":
            try:
                from ddm_amd.rccl import RcclComm
                comm = RcclComm.from_default_group(dev)
                args.gather_backend = "rccl (ctypes ncclAllGather, HBM to HBM over xGMI)"
            except Exception as e:      # noqa: BLE001  (reported in the JSON line, loudly)
                args.gather_backend = f"gloo (host all_gather): the RCCL communicator failed to initialise: {e}"
                print(f"rank {rank}: RCCL communicator failed ({e}); the events are gathered over gloo",
                      file=sys.stderr)
        else:
            args.gather_backend = f"{backend} (torch.distributed all_gather, host memory: a rehearsal)"
    args.comm = comm
    if args.workload == "c1":
        res = run_c1(args, world, rank, dev, torch, dist, cpu if rank == 0 and args.cpu_baseline else None)
    elif args.workload == "c4":
        res = run_c4(args, world, rank, dev, torch, dist, cpu)
    else:
        res = run_partition_workload(args, world, rank, dev, torch, dist, args.workload, cpu)
    rows_rank, elapsed, info, extra, roofline, cpu_res, scaling = res
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        r = torch.tensor([rows_rank], dtype=torch.float64)
        dist.all_reduce(r)
        rows_total = float(r.item())
    else:
        rows_total = float(rows_rank)
    if rank == 0:
        out = bench_line(args, world, rows_total, elapsed, info, extra, roofline, cpu_res, scaling)
        if args.workload == "c3" and args.companion and world == 1 and not args.solo_world:
            out["companion"] = {"c2_published_cell": companion_c2(args, rank, dev, torch, dist)}
        print(json.dumps(out), flush=True)
    if comm is not None:
        comm.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
