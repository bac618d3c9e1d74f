"""Host (numpy) mirror of the synthetic stream generators in csrc/synth.hip.  TEST
INFRASTRUCTURE ONLY (see oracle/__init__.py): the tests check that the device generators
equal this mirror, and bench.py's cpu_baseline leg builds its partition samples with it
(before any GPU call, so its worker processes never inherit a HIP context).

The streams stand in for rialto.csv (absent, .MISSING_LARGE_BLOBS:1), partitioned as
DDM_Process.py:225 (`full_df_row_number % INSTANCES`): partition row r is global row
g = r * n_parts + part.
"""
import numpy as np

_M = np.uint64(0xFFFFFFFFFFFFFFFF)


def _mix64(z):
    with np.errstate(over="ignore"):
        z = (z + np.uint64(0x9e3779b97f4a7c15)) & _M
        z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xbf58476d1ce4e5b9)) & _M
        z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94d049bb133111eb)) & _M
    return z ^ (z >> np.uint64(31))


def unit(seed, a, b):
    """synth.hip unit(): U[0,1) double from a counter hash of (seed, a, b)."""
    a = np.asarray(a, dtype=np.uint64)
    b = np.asarray(b, dtype=np.uint64)
    with np.errstate(over="ignore"):
        inner = _mix64((a * np.uint64(0x2545f4914f6cdd1d) + b) & _M)
    h = _mix64(np.uint64(seed) ^ inner)
    return (h >> np.uint64(11)).astype(np.float64) * 2.0 ** -53


def block_labels(n, part, n_parts, block_rows, n_classes, start=0):
    """Labels of partition rows [start, start + n)."""
    g = np.arange(start, start + n, dtype=np.int64) * n_parts + part
    return ((g // block_rows) % n_classes).astype(np.int32)


def _boundary(seed, k, period, jitter):
    k = np.asarray(k, dtype=np.int64)
    if jitter == 0:
        return k * period
    j = (unit(seed, np.maximum(k, 0).astype(np.uint64), 0xb10c0001) * float(2 * jitter + 1)).astype(np.int64) - jitter
    return np.where(k <= 0, k * period, k * period + j)


def jitter_labels(n, part, n_parts, period, jitter, n_classes, flip, seed):
    g = np.arange(n, dtype=np.int64) * n_parts + part
    k = g // period
    k = np.where(g < _boundary(seed, k, period, jitter), k - 1, k)
    k = np.where(g >= _boundary(seed, k + 1, period, jitter), k + 1, k)
    c = k % n_classes
    if flip > 0 and n_classes > 1:
        s2 = np.uint64(seed) ^ np.uint64(0x7f4a7c15)
        hit = unit(s2, g.astype(np.uint64), 0xf119) < flip
        shift = 1 + (unit(s2, g.astype(np.uint64), 0xf11a) * (n_classes - 1)).astype(np.int64)
        c = np.where(hit, (c + shift) % n_classes, c)
    return c.astype(np.int32)


def features(y, row0, row_stride, seed, n_features=27, noise=0.04):
    """float32 [n, F] of synth.hip k_features (float32 arithmetic, no contraction)."""
    y = np.asarray(y, dtype=np.int64)
    g = (row0 + np.arange(len(y), dtype=np.int64) * row_stride).astype(np.uint64)
    X = np.empty((len(y), n_features), dtype=np.float32)
    for f in range(n_features):
        k = ((y * 7 + f * 3) % 10).astype(np.float32)
        base = np.float32(0.05) + np.float32(0.1) * k
        u = unit(seed, g, f).astype(np.float32)
        X[:, f] = base + np.float32(noise) * u
    return X
