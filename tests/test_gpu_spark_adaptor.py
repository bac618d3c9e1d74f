"""Arrow groups (what Spark hands a Python worker, DDM_Process.py:226) through the device
path == the reference's fixtures; the applyInPandas function likewise."""
import numpy as np
import pytest

from conftest import golden_partitions
from test_spark_adaptor import _arrow

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("mult,inst", [(2, 1), (4, 4)])
def test_arrow_group_equals_reference(mult, inst):
    from ddm_amd.spark import run_arrow_group
    for d, part, expect in golden_partitions(mult, inst):
        if expect is None:
            continue
        np.random.seed(1000 + d)
        got = run_arrow_group(_arrow(part))
        assert np.array_equal(got.to_numpy(), expect), (mult, inst, d)
        np.random.seed(1000 + d)
        tab = run_arrow_group(_arrow(part, 1), as_arrow=True)
        assert tab.num_rows == len(expect) and np.array_equal(tab.to_pandas().to_numpy(), expect)


def test_apply_in_pandas_function():
    from ddm_amd.spark import grouped_map_udf
    fn = grouped_map_udf()
    for d, part, expect in golden_partitions(2, 4):
        np.random.seed(1000 + d)
        assert np.array_equal(fn(part).to_numpy(), expect)
