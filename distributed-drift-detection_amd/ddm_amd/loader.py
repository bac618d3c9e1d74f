"""Stream preparation and loader: the data prep of DDM_Process.py:38-55
and the partition columns of :220-225, straight into columnar float32.

Reference, in order:
  * `df = pd.read_csv(FILENAME)` (:42);
  * MULT_DATA < 1: `df.sample(frac=MULT)`; else `pd.concat([df] * MULT).sample(frac=1)`
    (:44-49) -- both draw from numpy's global legacy RandomState: pandas' `sample` is
    `RandomState.choice(n, size, replace=False)` = `permutation(n)[:size]`;
  * `df.sort_values(by="target")` (:51, numpy quicksort: platform dependent for ties, so
    `sort_kind` selects it or a stable sort -- the fixtures pin the stable order);
  * `full_df_row_number = df.index` (:220): the ORIGINAL csv row, shared by all MULT copies;
  * `device_id = full_df_row_number % INSTANCES` (:225), one group per device_id in stream
    order (`groupby("device_id").apply`, :226).

Here the csv is parsed by pyarrow's multithreaded reader (correctly rounded; its float32
columns equal pandas' parse cast to float32 -- the only precision the hot path uses, since
sklearn casts X to float32 in fit and predict, DDM_Process.py:104,113), the permutation is
the same MT19937 draw (ddm_amd.rng, numpy's own generator), and every partition comes out
as columnar float32 [F, n] + int labels + row numbers, ready for one pinned host buffer
and one copy into HBM (controller.DevicePartition).
"""
from dataclasses import dataclass
from typing import List, Optional

import numpy as np

from .params import infer_x_features


@dataclass
class StreamTable:
    """A parsed stream: X32 float32 [F, n] (column f contiguous), target int64 [n]."""
    X32: np.ndarray
    target: np.ndarray
    features: List[str]

    @property
    def n_rows(self):
        return int(self.target.shape[0])


@dataclass
class PartitionArrays:
    """One device_id group (DDM_Process.py:226) in stream order."""
    device_id: int
    X32: np.ndarray          # float32 [F, n_d]
    target: np.ndarray       # int64 [n_d]
    row_number: np.ndarray   # int64 [n_d], full_df_row_number

    def frame(self, features):
        """The pandas frame the reference hands run_DDM_loop for this group: RangeIndex,
        float64 feature columns (the float32 values, exactly), target, row number, device_id."""
        import pandas as pd
        df = pd.DataFrame(self.X32.T.astype(np.float64), columns=list(features))
        df["target"] = self.target
        df["full_df_row_number"] = self.row_number
        df["device_id"] = np.full(len(self.target), self.device_id, dtype=np.int32)
        return df


def read_stream_csv(path, features: Optional[List[str]] = None, target="target", engine="pyarrow"):
    """DDM_Process.py:42 -> StreamTable.  engine="pandas" parses with pandas.read_csv
    (the reference's own parser) for bit-identical float64 text conversion."""
    if engine == "pyarrow":
        import pyarrow.csv as pacsv
        table = pacsv.read_csv(path)
        names = table.column_names
        feats = features or infer_x_features(names)
        X32 = np.empty((len(feats), table.num_rows), dtype=np.float32)
        for f, name in enumerate(feats):
            X32[f] = table.column(name).to_numpy().astype(np.float64, copy=False)
        y = table.column(target).to_numpy().astype(np.int64)
    elif engine == "pandas":
        import pandas as pd
        df = pd.read_csv(path)
        feats = features or infer_x_features(df.columns)
        X32 = np.ascontiguousarray(df[feats].to_numpy(dtype=np.float64).T.astype(np.float32))
        y = df[target].to_numpy().astype(np.int64)
    else:
        raise ValueError(f"unknown engine {engine!r}")
    return StreamTable(X32, y, list(feats))


def prepare_order(n_rows, target, mult, rng=None, sort_kind="quicksort"):
    """DDM_Process.py:44-51: the stream as original-row indices (= full_df_row_number,
    :220), drawing the shuffle from `rng` (a numpy RandomState; default: the global
    one, as the reference does)."""
    rs = np.random.mtrand._rand if rng is None else rng
    target = np.asarray(target)
    m = float(mult)
    if m < 1:
        size = int(round(m * n_rows))                   # pandas sample(frac=...)
        order = rs.permutation(n_rows)[:size]
    else:
        k = int(m)
        order = rs.permutation(n_rows * k) % n_rows     # concat([df] * k): position -> csv row
    idx = np.argsort(target[order], kind=sort_kind)    # sort_values(by="target")
    return order[idx].astype(np.int64)


def split_partitions(table: StreamTable, order, instances) -> List[PartitionArrays]:
    """device_id = full_df_row_number % INSTANCES (DDM_Process.py:225), groups in
    device_id order, rows in stream order (columnar gathers, no pandas)."""
    order = np.asarray(order, dtype=np.int64)
    dev = order % int(instances)
    sel = np.argsort(dev, kind="stable")
    counts = np.bincount(dev, minlength=int(instances))
    out, start = [], 0
    for d in range(int(instances)):
        rows = order[sel[start:start + counts[d]]]
        start += counts[d]
        if len(rows):
            out.append(PartitionArrays(d, np.ascontiguousarray(table.X32[:, rows]), table.target[rows], rows))
    return out


def load_partitions(path, mult, instances, data_seed=None, sort_kind="quicksort", engine="pyarrow"):
    """read_stream_csv + prepare_order + split_partitions.  data_seed: None draws from
    numpy's global RNG (the reference), an int seeds a private RandomState."""
    table = read_stream_csv(path, engine=engine)
    rng = None if data_seed is None else np.random.RandomState(data_seed)
    order = prepare_order(table.n_rows, table.target, mult, rng, sort_kind)
    return table, order, split_partitions(table, order, instances)


def pinned_columns(part: PartitionArrays):
    """Copy a partition's float32 columns and labels into page-locked host memory (one
    buffer each), the staging step before the single host-to-HBM copy."""
    import torch
    X = torch.empty(part.X32.shape, dtype=torch.float32, pin_memory=True)
    X.numpy()[...] = part.X32
    y = torch.empty(part.target.shape, dtype=torch.int32, pin_memory=True)
    y.numpy()[...] = part.target.astype(np.int32)
    return X, y
