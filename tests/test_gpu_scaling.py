"""configs[2]/[4] at N > 1 as the driver runs them: the SAME partitions, partition d on rank
d % N (DDM_Process.py:225-226), must give the same events at every N.

Rehearsed on one GPU: `torch.distributed.run` starts 2 ranks of bench.py that share
cuda:0 and gather over gloo (DDM_BENCH_BACKEND=gloo); the digest of ALL partitions'
gathered events must equal the N=1 run's."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _bench(n, extra, self_launch=False):
    args = ["bench.py", "--gpus", str(n), "--steps", "1", "--warmup", "0", "--cpu-baseline", "0",
            "--oracle-check-rows", "0", "--companion", "0"] + extra
    env = dict(os.environ, DDM_BENCH_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    if n == 1 or self_launch:
        cmd = [sys.executable] + args
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
               "--master-addr", "127.0.0.1", "--master-port", str(_port())] + args
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")][-1]
    return json.loads(line)


@pytest.mark.parametrize("workload,extra", [
    ("c3", ["--rows-per-part", "2000000", "--block-rows", "1000037"]),
    ("c5", ["--c5-rows", "160000"]),
])
def test_events_do_not_depend_on_gpu_count(workload, extra):
    import torch
    assert not torch.cuda.is_initialized(), "must run before this process touches the GPU"
    one = _bench(1, ["--workload", workload] + extra)
    two = _bench(2, ["--workload", workload] + extra)
    d1, d2 = one["breakdown"]["checks"]["events_sha1"], two["breakdown"]["checks"]["events_sha1"]
    assert d1 == d2
    assert one["breakdown"]["drifts_per_step"] > 0
    assert two["config"]["partitions_this_rank"] == 4 and one["config"]["partitions_this_rank"] == 8
    assert one["scaling"] == two["scaling"] == "strong"
    assert two["gather_backend"] and "gather_backend" not in one
    assert two["roofline"]["frac"] > 0
    if workload == "c5":
        assert two["breakdown"]["gather_ms_per_step"] is not None


def test_bench_launches_its_own_ranks():
    """`bench.py --gpus 2` with no launcher starts 2 ranks itself (torch.distributed.run,
    before touching the GPU): n_gpus 2 and the events of the N=1 run."""
    import torch
    assert not torch.cuda.is_initialized()
    extra = ["--workload", "c3", "--rows-per-part", "1000000", "--block-rows", "500037"]
    one = _bench(1, extra)
    two = _bench(2, extra, self_launch=True)
    assert two["n_gpus"] == 2 and one["n_gpus"] == 1
    assert two["breakdown"]["checks"]["events_sha1"] == one["breakdown"]["checks"]["events_sha1"]


@pytest.mark.parametrize("mult,inst", [(2, 16), (2, 1), (4, 4), (512, 16)])
def test_bench_c2_matches_reference_fixtures(mult, inst):
    """configs[1] (outdoorStream) as the bench times it: every partition's events == the
    reference-executed fixture, and vs_baseline against the matching published cell.
    (512, 16) is the published cell itself (`Plot Results.ipynb:572`): all 16 partitions,
    20,464 batch records, against tests/golden/make_golden_cell.py's fixture, the stream
    order by its sha1."""
    import torch
    assert not torch.cuda.is_initialized()
    r = _bench(1, ["--workload", "c2", "--c2-mult", str(mult), "--c2-instances", str(inst)])
    assert "fixtures" in r["breakdown"]["checks"]
    assert "oracle_prefix" not in r["breakdown"]["checks"]
    assert r["config"]["rows_per_step"] == 4000 * mult
    assert r["vs_baseline"] is not None and r["vs_baseline"] > 1
    assert r["roofline"]["kernel"].startswith("k_cforest_predict_dev")
