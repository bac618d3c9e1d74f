"""Spark adaptor: the grouped-map hand-off of DDM_Process.py:226
(`repartition("device_id").groupby("device_id").apply(run_DDM_loop)`) on a GPU executor.

Spark hands a Python worker one group as Arrow record batches (grouped-map pandas UDFs
and `applyInPandas` convert them to a pandas frame; `mapInArrow` / Arrow-native UDFs pass
them as they are).  This module takes either form to the device path without a pandas
round trip for the feature columns:

  * `executor_device(device_id)`: the GPU of this task: the task's assigned GPU resource
    when Spark scheduled one (TaskContext resources "gpu"), else device_id % visible GPUs
    (SURVEY §8e placement);
  * `arrow_partition_columns(batches, features)`: the group's Arrow columns -> ONE
    page-locked float32 [F, n] staging buffer (each float64 Arrow column is read through
    a zero-copy numpy view and cast straight into its pinned row), plus labels and row
    numbers; `upload` then moves it to HBM with one asynchronous copy per buffer;
  * `run_arrow_group(batches, ...)`: the partition function on Arrow input, returning the
    reference's output frame (schema DDM_Process.py:167) or an Arrow table;
  * `grouped_map_udf(settings)`: the function to pass to `applyInPandas(fn, SCHEMA)`
    (the drop-in run_DDM_loop with executor device selection).

pyspark is not installed in this image; everything here takes plain pyarrow / pandas
objects, so it is exercised by the tests without Spark.
"""
import numpy as np

from .params import OUTPUT_COLUMNS, SCHEMA, DDMSettings, infer_x_features


def executor_device(device_id, n_gpus=None):
    """torch.device of this task's GPU (see module docstring)."""
    import torch
    n = torch.cuda.device_count() if n_gpus is None else int(n_gpus)
    if n <= 0:
        raise RuntimeError("no GPU visible to this executor: the MI355X partition path needs a HIP device")
    try:                                           # Spark 3 GPU scheduling: the task's own GPU
        from pyspark import TaskContext
        tc = TaskContext.get()
        if tc is not None and "gpu" in tc.resources():
            addr = tc.resources()["gpu"].addresses
            if addr:
                return torch.device("cuda", int(addr[0]) % n)
    except ImportError:
        pass
    return torch.device("cuda", int(device_id) % n)


class ArrowPartition:
    """One group's columns staged for the device: X32 float32 [F, n] (pinned when a GPU is
    present), labels int64, full_df_row_number int64."""

    def __init__(self, X32, target, row_number, device_id):
        self.X32, self.target, self.row_number, self.device_id = X32, target, row_number, device_id

    def upload(self, device, stream=None):
        """-> controller.DevicePartition: one host-to-HBM copy of the staged columns."""
        import torch

        from .controller import DevicePartition
        F, n = self.X32.shape
        part = DevicePartition.allocate(n, F, device)
        with torch.cuda.stream(stream or torch.cuda.current_stream(device)):
            if n:
                part.X[:, :n].copy_(torch.from_numpy(self.X32) if isinstance(self.X32, np.ndarray) else self.X32,
                                    non_blocking=True)
                part.y[:n].copy_(torch.from_numpy(self.target.astype(np.int32)), non_blocking=False)
        part.host_X32 = None
        part.host_y = self.target
        self._keep = self.X32                  # the pinned staging stays alive until the copy ran
        return part


def _concat_column(batches, name):
    cols = [b.column(b.schema.get_field_index(name)) for b in batches]
    return cols


def arrow_partition_columns(batches, features=None, target="target", row_number="full_df_row_number",
                            pinned=None):
    """Arrow record batches (or one pyarrow Table) of one group -> ArrowPartition.  Feature
    columns are float64 in the reference (pandas read_csv); each is read zero-copy and cast
    once into its row of the float32 staging buffer (the cast sklearn applies, exact)."""
    import pyarrow as pa
    if isinstance(batches, pa.Table):
        batches = batches.to_batches()
    batches = [b for b in batches if b.num_rows]
    names = batches[0].schema.names if batches else []
    feats = list(features) if features is not None else infer_x_features(names)
    n = sum(b.num_rows for b in batches)
    if pinned is None:
        try:
            import torch
            pinned = torch.cuda.is_available()
        except ImportError:
            pinned = False
    if pinned:
        import torch
        X = torch.empty((len(feats), n), dtype=torch.float32, pin_memory=True)
        Xn = X.numpy()
    else:
        X = Xn = np.empty((len(feats), n), dtype=np.float32)
    for f, name in enumerate(feats):
        o = 0
        for col in _concat_column(batches, name):
            k = len(col)
            if col.null_count:
                v = col.to_numpy(zero_copy_only=False)          # nulls -> NaN (sklearn sees NaN too)
            else:
                v = col.to_numpy(zero_copy_only=col.type in (pa.float64(), pa.float32()))
            Xn[f, o:o + k] = v
            o += k
    y = np.concatenate([c.to_numpy(zero_copy_only=False) for c in _concat_column(batches, target)]) if n else \
        np.zeros(0, np.int64)
    rn = np.concatenate([c.to_numpy(zero_copy_only=False) for c in _concat_column(batches, row_number)]) if n else \
        np.zeros(0, np.int64)
    dev_id = 0
    if n and "device_id" in names:
        dev_id = int(_concat_column(batches, "device_id")[0][0].as_py())
    return ArrowPartition(X, y, rn.astype(np.int64), dev_id)


def run_arrow_group(batches, rng=None, settings=None, device=None, as_arrow=False, refit="device"):
    """The partition function on one group's Arrow batches: the reference's output frame
    (local label = position in the group, DDM_Process.py:148,151 on a RangeIndex group), or
    the same as a pyarrow Table.  rng: an MTStream (default: numpy's global RandomState,
    advanced exactly as the reference advances it)."""
    import torch

    from .controller import PartitionRunner, _int_labels, events_frame
    from .rng import MTStream
    s = settings or DDMSettings()
    part = arrow_partition_columns(batches, s.x_features, s.target, s.row_number)
    part.target = _int_labels(part.target)
    dev = device or executor_device(part.device_id)
    stream = torch.cuda.Stream(dev)
    dpart = part.upload(dev, stream)
    own = rng is None
    rng = MTStream.from_global() if own else rng
    runner = PartitionRunner(dpart, s, stream, refit)
    try:
        rows = runner.run(rng)
    finally:
        runner.close()
        if own:
            np.random.set_state(rng.numpy_state())
    out = events_frame(rows, np.arange(len(part.target)), part.row_number)
    if as_arrow:
        import pyarrow as pa
        return pa.Table.from_pandas(out.astype(np.int32), preserve_index=False)
    return out


def grouped_map_udf(settings=None, refit="device"):
    """The function for `df.groupby("device_id").applyInPandas(fn, schema=SCHEMA)`
    (DDM_Process.py:226 in its modern form): the drop-in run_DDM_loop on the executor's GPU."""
    from .controller import run_DDM_loop
    s = settings or DDMSettings()

    def fn(pdf):
        dev = executor_device(int(pdf["device_id"].iloc[0]) if "device_id" in pdf and len(pdf) else 0)
        return run_DDM_loop(pdf, settings=s, device=dev, refit=refit)

    fn.schema = SCHEMA
    return fn


__all__ = ["executor_device", "arrow_partition_columns", "run_arrow_group", "grouped_map_udf", "ArrowPartition",
           "OUTPUT_COLUMNS", "SCHEMA"]
