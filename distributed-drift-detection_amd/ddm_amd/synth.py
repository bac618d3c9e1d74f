"""Synthetic stand-ins for the benchmark configs of BASELINE.json.

rialto.csv is not shipped (.MISSING_LARGE_BLOBS:1), so every rialto-shaped stream is
synthetic:

  C1 (configs[0])  `rialto_table`: an 82,250 x 27 table of Dirichlet histograms, 10
                   classes of 8,225 rows with class-specific concentrations (numpy PCG64,
                   seed 20261015), prepared like DDM_Process.py:38-55 (MULT=2: concat x2,
                   shuffle, sort by target) and run as ONE partition (INSTANCES=1).
  C3 (configs[2])  `block_partition`: noise-free separable class blocks of ~1e7 global
                   rows, partitioned row % 8, generated in HBM (ddm_synth_block_labels).
  C5 (configs[4])  `jitter_partition`: class blocks of 150-300 partition rows (global
                   boundaries every 1800 +- 300 rows over 8 partitions) and label noise: a drift,
                   hence a refit, every one or two batches (ddm_synth_jitter_labels).

C3/C5 rows come from a counter hash of the global row, so a partition regenerates the
same on any GPU and under any partition -> GPU placement.
"""
import numpy as np

C1_ROWS, C1_FEATURES, C1_CLASSES, C1_SEED = 82_250, 27, 10, 20261015
C5_PERIOD, C5_JITTER = 1800, 300


def rialto_table(n_rows=C1_ROWS, n_features=C1_FEATURES, n_classes=C1_CLASSES, seed=C1_SEED):
    """C1's stand-in for rialto.csv: a loader.StreamTable (X32 float32 [F, n], int64
    target) of Dirichlet histograms.  Class c concentrates on the bins f with f % 10 ==
    c (alpha 12 there, 1 elsewhere), so classes are separable; rows come class block by
    class block (ascending), as the reference's sort leaves them anyway."""
    from .loader import StreamTable
    rng = np.random.Generator(np.random.PCG64(seed))
    per = n_rows // n_classes
    target = np.repeat(np.arange(n_classes, dtype=np.int64), per)
    target = np.concatenate([target, np.full(n_rows - len(target), n_classes - 1, dtype=np.int64)])
    X = np.empty((n_rows, n_features), dtype=np.float64)
    for c in range(n_classes):
        alpha = np.ones(n_features)
        alpha[np.arange(n_features) % 10 == c % 10] = 12.0
        rows = target == c
        X[rows] = rng.dirichlet(alpha, size=int(rows.sum()))
    X32 = np.ascontiguousarray(X.T.astype(np.float32))
    return StreamTable(X32, target, [str(i) for i in range(n_features)])


def rialto_partitions(mult=2, instances=1, data_seed=C1_SEED, table=None):
    """C1: the table through DDM_Process.py:44-51 (concat x MULT, sample(frac=1) from a
    RandomState(data_seed), stable sort by target) and :220-226 (row % INSTANCES).
    Returns (table, order, [loader.PartitionArrays])."""
    from .loader import prepare_order, split_partitions
    table = table if table is not None else rialto_table()
    order = prepare_order(table.n_rows, table.target, mult, np.random.RandomState(data_seed), "stable")
    return table, order, split_partitions(table, order, instances)


def block_partition(n_rows, part, n_parts, block_rows, seed, device, n_features=27, n_classes=10, noise=0.04):
    """C3: partition `part` of a class-block stream (row % n_parts) in HBM."""
    from . import kernels
    from .controller import DevicePartition
    p = DevicePartition.allocate(n_rows, n_features, device)
    kernels.synth_block_labels(p.y[:n_rows], part, n_parts, block_rows, n_classes)
    kernels.synth_features(p.X, p.y[:n_rows], part, n_parts, seed, noise)
    return p


def jitter_partition(n_rows, part, n_parts, seed, device, period=C5_PERIOD, jitter=C5_JITTER, flip=0.0,
                     n_features=27, n_classes=10, noise=0.04):
    """C5: partition `part` (row % n_parts) of a stream with short jittered class blocks
    (and label noise `flip`) in HBM."""
    from . import kernels
    from .controller import DevicePartition
    p = DevicePartition.allocate(n_rows, n_features, device)
    kernels.synth_jitter_labels(p.y[:n_rows], part, n_parts, period, jitter, n_classes, flip, seed)
    kernels.synth_features(p.X, p.y[:n_rows], part, n_parts, seed, noise)
    return p


def host_copy(part):
    """(X float64 [n, F], y int64 [n]) of a device partition: the oracle's inputs."""
    import torch
    torch.cuda.synchronize(part.device)
    X = part.X[:, :part.n].t().contiguous().cpu().numpy().astype(np.float64)
    y = part.y[:part.n].cpu().numpy().astype(np.int64)
    return X, y
