"""Spark adaptor: Arrow group -> staged float32 columns, on the host; the
device run of Arrow groups is in tests/test_gpu_spark_adaptor.py."""
import numpy as np
import pyarrow as pa

from conftest import golden_partitions


def _arrow(pdf, chunks=3):
    t = pa.Table.from_pandas(pdf, preserve_index=False)
    n = t.num_rows
    cuts = np.linspace(0, n, chunks + 1).astype(int)
    return [t.slice(a, b - a).combine_chunks().to_batches()[0] for a, b in zip(cuts[:-1], cuts[1:]) if b > a]


def test_arrow_columns_equal_the_float32_cast_of_the_frame():
    from ddm_amd.spark import arrow_partition_columns
    d, part, _ = golden_partitions(2, 4)[1]
    feats = [str(i) for i in range(21)]
    ap = arrow_partition_columns(_arrow(part), feats, pinned=False)
    assert ap.X32.dtype == np.float32 and ap.X32.shape == (21, len(part))
    assert np.array_equal(ap.X32, part[feats].to_numpy(np.float64).astype(np.float32).T)
    assert np.array_equal(ap.target, part["target"].to_numpy())
    assert np.array_equal(ap.row_number, part["full_df_row_number"].to_numpy())
    assert ap.device_id == d


def test_arrow_nulls_become_nan_and_features_inferred():
    from ddm_amd.spark import arrow_partition_columns
    t = pa.table({"0": pa.array([0.5, None, 1.5]), "1": pa.array([1.0, 2.0, 3.0]),
                  "target": pa.array([0, 1, 0]), "full_df_row_number": pa.array([4, 5, 6])})
    ap = arrow_partition_columns(t, pinned=False)
    assert ap.X32.shape == (2, 3) and np.isnan(ap.X32[0, 1]) and ap.X32[1, 2] == 3.0


def test_grouped_map_udf_schema():
    from ddm_amd.params import SCHEMA
    from ddm_amd.spark import grouped_map_udf
    assert grouped_map_udf().schema == SCHEMA
