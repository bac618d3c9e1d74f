"""Partitioning and placement — the MI355X side of DDM_Process.py:220-226.

Reference: `full_df_row_number = df.index` (:220), `device_id = full_df_row_number %
INSTANCES` (:225, a row-at-a-time Python UDF), `repartition("device_id")
.groupby("device_id").apply(run_DDM_loop)` (:226): each group is handed to the UDF as a
pandas frame with a RangeIndex, and the UDF outputs are concatenated.

Here the groups are strided subsets computed with one vectorised modulo, each group's
rows go to HBM of GPU `device_id % n_gpus`, all partitions of one GPU run in lockstep in
one BatchRunner (one batched launch per kernel per epoch, controller.py), and the
per-partition outputs are concatenated in device_id order.  Partitions are
independent (the reference shares nothing between them), so there is no collective on
the data path; `dist.py` adds the one gather of events across processes.
"""
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pandas as pd
import torch

from .controller import run_partition_arrays, run_partition_frames
from .params import OUTPUT_COLUMNS, DDMSettings
from .rng import MTStream


def split_partitions(df, instances, row_number="full_df_row_number"):
    """[(device_id, frame)] in device_id order; frames keep the stream order and get a
    RangeIndex (grouped-map semantics) plus the full_df_row_number / device_id columns."""
    full = df.copy()
    full[row_number] = df.index.to_numpy()
    dev = (full[row_number].to_numpy() % int(instances)).astype(np.int32)
    full["device_id"] = dev
    order = np.argsort(dev, kind="stable")
    counts = np.bincount(dev, minlength=int(instances))
    out, start = [], 0
    for d in range(int(instances)):
        idx = order[start:start + counts[d]]
        start += counts[d]
        if counts[d]:
            out.append((d, full.iloc[idx].reset_index(drop=True)))
    return out


def placement(device_id, n_gpus):
    """GPU of a partition: device_id % n_gpus."""
    return int(device_id) % max(1, int(n_gpus))


def run_partitions(parts, seeds, settings=None, devices=None, max_workers=None, fn=None, stats=None):
    """Run [(device_id, frame)]: the partitions placed on each GPU run in lockstep in one
    BatchRunner, one host thread per GPU.

    seeds: device_id -> MT19937 seed, the RNG each partition's Spark worker would hold
    (`np.random.seed(base + device_id)` in the oracle).  fn(frame, rng, device, stats)
    replaces the GPU path with a per-partition function (tests only; run in a thread
    pool).  Returns {device_id: output frame}."""
    s = settings or DDMSettings()
    if devices is None:
        devices = [torch.device("cuda", i) for i in range(torch.cuda.device_count())]
    if fn is not None:
        def one(item):
            d, frame = item
            dev = devices[placement(d, len(devices))] if devices else None
            st = {}
            return d, fn(frame, MTStream.from_seed(seeds[d]), dev, st), st

        workers = max_workers or max(1, min(len(parts), 16))
        with ThreadPoolExecutor(workers) as ex:
            res = list(ex.map(one, parts))
        if stats is not None:
            for d, _, st in res:
                stats[d] = st
        return {d: out for d, out, _ in res}
    if not devices:
        raise RuntimeError("no GPU visible: the MI355X partition path needs a HIP device")
    groups = {}
    for d, frame in parts:
        groups.setdefault(placement(d, len(devices)), []).append((d, frame))

    def on_gpu(item):
        g, items = item
        dev = devices[g]
        st = {}
        outs = run_partition_frames([f for _, f in items], [MTStream.from_seed(seeds[d]) for d, _ in items], s,
                                    dev, torch.cuda.Stream(dev), stats=st)
        return [(d, o) for (d, _), o in zip(items, outs)], st

    with ThreadPoolExecutor(max(1, len(groups))) as ex:
        res = list(ex.map(on_gpu, sorted(groups.items())))
    out = {}
    for pairs, st in res:
        for d, o in pairs:
            out[d] = o
            if stats is not None:
                stats[d] = st
    return out


def apply_in_pandas(df, instances, base_seed, settings=None, devices=None, max_workers=None):
    """`df.groupby(device_id).apply(run_DDM_loop)` (DDM_Process.py:225-226) on the GPUs of
    this process: concatenated UDF outputs (schema DDM_Process.py:167) in device_id order."""
    parts = split_partitions(df, instances)
    outs = run_partitions(parts, {d: base_seed + d for d, _ in parts}, settings, devices, max_workers)
    frames = [outs[d] for d, _ in parts]
    return pd.concat(frames) if frames else pd.DataFrame(columns=OUTPUT_COLUMNS)


def run_stream_file(path, mult, instances, base_seed, data_seed=None, sort_kind="quicksort", settings=None,
                    devices=None, engine="pyarrow"):
    """The reference's whole job minus Spark (DDM_Process.py:38-55, :216-258): load and
    prepare the stream, split it into INSTANCES partitions, run every partition on the GPUs
    of this process (partition d on GPU d % n_gpus, seeded base_seed + d), and collect the
    output.  Returns (events frame in device_id order, post-loop record dict with the
    distances of DDM_Process.py:250-257, the total time of :224-258 and the mean distance)."""
    import time

    from . import loader, record
    table, order, parts = loader.load_partitions(path, mult, instances, data_seed, sort_kind, engine)
    s = settings or DDMSettings()
    if devices is None:
        devices = [torch.device("cuda", i) for i in range(torch.cuda.device_count())]
    if not devices:
        raise RuntimeError("no GPU visible: the MI355X partition path needs a HIP device")
    t0 = time.perf_counter()
    groups = {}
    for p in parts:
        groups.setdefault(placement(p.device_id, len(devices)), []).append(p)

    def on_gpu(item):
        g, items = item
        outs = run_partition_arrays(items, [MTStream.from_seed(base_seed + p.device_id) for p in items], s,
                                    devices[g], torch.cuda.Stream(devices[g]))
        return [(p.device_id, o) for p, o in zip(items, outs)]

    with ThreadPoolExecutor(max(1, len(groups))) as ex:
        res = dict(kv for pairs in ex.map(on_gpu, sorted(groups.items())) for kv in pairs)
    frames = [res[p.device_id] for p in parts]
    events = pd.concat(frames) if frames else pd.DataFrame(columns=OUTPUT_COLUMNS)
    dist = record.dist_between_changes(len(order), table.target[order])
    changes = record.change_distances(events, dist)
    total = time.perf_counter() - t0
    return events, {"distances": changes, "dist_between_changes": dist, "total_time": total,
                    "average_distance": float(changes["distance"].mean()) if len(changes) else float("nan")}
