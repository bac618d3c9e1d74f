"""The driver's JSON line at N > 1 (bench.bench_line, host logic only): the same roofline and
CPU baseline as at N = 1, the collect's backend named, and a line missing any of them is
refused (DDM_Process.py:225-226, :258)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _args(workload, cpu=1):
    import bench
    old = sys.argv
    sys.argv = ["bench.py", "--workload", workload, "--cpu-baseline", str(cpu), "--gpus", "2"]
    try:
        return bench.parse()
    finally:
        sys.argv = old


ROOF = {"bound": "hbm", "achieved": 4000.0, "peak": 8000.0, "unit": "GB/s", "frac": 0.5, "traffic": None}
CPU = {"value": 5e5, "unit": "rows/s", "cores": 16, "kind": "port", "sample": "x"}


@pytest.mark.parametrize("workload", ["c3", "c2", "c5"])
def test_n2_line_carries_roofline_cpu_baseline_and_gather_backend(workload):
    import bench
    a = _args(workload)
    extra = {"gather_backend": "rccl (ctypes ncclAllGather, HBM to HBM over xGMI)", "checks": {}}
    out = bench.bench_line(a, 2, 2e9, 0.1, {"workload": workload}, extra, ROOF, CPU, "strong")
    assert out["n_gpus"] == 2 and out["value"] == pytest.approx(2e10)
    assert out["roofline"]["frac"] == 0.5 and out["cpu_baseline"]["cores"] == 16
    assert out["gather_backend"].startswith("rccl")
    if workload == "c2":
        assert out["vs_baseline"] is not None


def test_n2_line_refused_without_gather_backend_or_cpu_baseline():
    import bench
    a = _args("c3")
    with pytest.raises(RuntimeError, match="gather_backend"):
        bench.bench_line(a, 2, 2e9, 0.1, {}, {"gather_backend": None}, ROOF, CPU, "strong")
    with pytest.raises(RuntimeError, match="cpu_baseline"):
        bench.bench_line(a, 2, 2e9, 0.1, {}, {"gather_backend": "gloo"}, ROOF, None, "strong")
    # no CPU leg asked for: the line stands without it
    a0 = _args("c3", cpu=0)
    assert bench.bench_line(a0, 2, 2e9, 0.1, {}, {"gather_backend": "gloo"}, ROOF, None, "strong")["n_gpus"] == 2


def test_n1_line_has_no_gather_backend():
    import bench
    a = _args("c3")
    out = bench.bench_line(a, 1, 1e9, 0.1, {}, {"gather_backend": None}, ROOF, CPU, "strong")
    assert "gather_backend" not in out
