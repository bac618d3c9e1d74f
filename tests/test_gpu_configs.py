"""BASELINE.json configs on the GPU vs the oracle:

  configs[0] C1  rialto-shaped table, MULT=2, INSTANCES=1: all 164,500 rows, events ==
                 oracle/controller.py run_partition (the restatement pinned to the
                 reference's own outputs by tests/test_oracle.py);
  configs[4] C5  short class blocks -> a refit every one or two batches: hundreds of
                 refits per partition, every event and the RNG position == the oracle;
  configs[2] C3  partition 0 through two class boundaries (2.6M rows) == the oracle
                 controller, every column and the RNG position; and the full 8 x 125M-row
                 configuration on the BatchRunner path the bench times: one drift per class
                 boundary at the first new-class row in shuffled order (the MT19937 draws
                 replayed by oracle/mt_replay.c), no warning, RNG positions == the replay;
  device generators == their host mirror (oracle/synth.py).
"""
import numpy as np
import pytest
import torch

from oracle import synth as hsynth

pytestmark = pytest.mark.gpu


def _dev():
    return torch.device("cuda", 0)


def test_device_generators_match_host_mirror():
    from ddm_amd import kernels, synth
    dev = _dev()
    n = 50_000
    p = synth.jitter_partition(n, 5, 8, 123, dev, flip=0.02)
    p3 = synth.block_partition(n, 2, 8, 10_037, 77, dev)
    X, y = synth.host_copy(p)
    assert np.array_equal(y, hsynth.jitter_labels(n, 5, 8, 1800, 300, 10, 0.02, 123))
    assert np.array_equal(X.astype(np.float32), hsynth.features(y, 5, 8, 123))
    X3, y3 = synth.host_copy(p3)
    assert np.array_equal(y3, hsynth.block_labels(n, 2, 8, 10_037, 10))
    assert np.array_equal(X3.astype(np.float32), hsynth.features(y3, 2, 8, 77))
    yk = torch.empty(1000, dtype=torch.int32, device=dev)
    with pytest.raises(Exception):
        kernels.synth_jitter_labels(yk, 0, 8, 1800, 900, 10, 0.0, 1)      # 2*jitter >= period


def test_c1_rialto_shaped_full_vs_oracle():
    from ddm_amd.controller import run_partition_arrays
    from ddm_amd.rng import MTStream
    from ddm_amd.synth import rialto_partitions
    from oracle.controller import run_partition
    _, _, parts = rialto_partitions()
    pa = parts[0]
    n = len(pa.target)
    assert n == 164_500
    rng = MTStream.from_seed(20261015)
    got = run_partition_arrays([pa], [rng], device=_dev())[0].to_numpy()
    np.random.seed(20261015)
    want = run_partition(pa.X32.T.astype(np.float64), pa.target, np.arange(n), pa.row_number)
    assert np.array_equal(got, want)
    after = np.random.get_state()
    assert np.array_equal(rng.key, after[1]) and rng.pos.value == after[2]
    assert (want[:, 2] >= 0).sum() >= 9


@pytest.mark.parametrize("flip,parts_run,groups", [(0.0, (0, 3), 1), (0.01, (6,), 1), (0.0, (1, 2, 5), 2)])
def test_c5_refit_heavy_vs_oracle(flip, parts_run, groups):
    """C5-shaped partitions (20k rows each of an 8-partition stream) in one BatchRunner, or
    in a GroupedRunner of two threads: a drift and a device refit every one or two batches."""
    from ddm_amd import synth
    from ddm_amd.controller import BatchRunner, GroupedRunner
    from ddm_amd.params import DDMSettings
    from ddm_amd.rng import MTStream
    from oracle.controller import run_partition
    dev = _dev()
    n = 20_000
    parts = [synth.jitter_partition(n, d, 8, 20261015, dev, flip=flip) for d in parts_run]
    host = [synth.host_copy(p) for p in parts]
    runner = BatchRunner(parts, DDMSettings()) if groups == 1 else GroupedRunner(parts, DDMSettings(), groups=groups)
    rngs = [MTStream.from_seed(9000 + d) for d in parts_run]
    got = runner.run(rngs)
    runner.close()
    for k, d in enumerate(parts_run):
        X, y = host[k]
        np.random.seed(9000 + d)
        want = run_partition(X, y, np.arange(n), np.arange(n))
        assert np.array_equal(got[k][:, 0], want[:, 0]) and np.array_equal(got[k][:, 1], want[:, 2]), d
        after = np.random.get_state()
        assert np.array_equal(rngs[k].key, after[1]) and rngs[k].pos.value == after[2]
        assert (want[:, 2] >= 0).sum() >= 60, d          # a refit every ~2-3 batches
    assert runner.stats.device_refits >= 100


def test_c3_partition0_through_class_boundaries_vs_oracle():
    """configs[2]'s partition 0 exactly as bench.py builds it (block_partition of the 1B-row
    stream: 27 features, class blocks of 10,000,037 global rows, row % 8), its first
    2.6M rows -- two class boundaries (partition rows 1,250,005 and 2,500,010), so two
    drifts, two device refits and a predict with a device-trained forest -- through the
    BatchRunner the bench times, against the oracle controller (run_partition_chunked,
    pinned to run_partition and the reference fixtures by tests/test_oracle.py): all four
    event columns (global row = partition row * 8 + 0) and the RNG position."""
    import bench
    from ddm_amd import synth
    from ddm_amd.controller import BatchRunner
    from ddm_amd.params import DDMSettings
    from ddm_amd.rng import MTStream
    from oracle.controller import run_partition_chunked
    dev = _dev()
    n, d, P = 2_600_000, 0, bench.C3_PARTS
    part = synth.block_partition(n, d, P, bench.C3_BLOCK, bench.SEED, dev)
    X, y = synth.host_copy(part)
    runner = BatchRunner([part], DDMSettings(), torch.cuda.Stream(dev, priority=-1), timing=True, fit_threads=16)
    rng = MTStream.from_seed(bench.SEED + d)
    got = runner.run([rng])[0]
    runner.close()
    np.random.seed(bench.SEED + d)
    want = run_partition_chunked(X, y, np.arange(n), np.arange(n) * P + d)
    after = np.random.get_state()
    ev = bench.events_rows(got)
    ev[:, 1] = np.where(ev[:, 1] >= 0, ev[:, 1] * P + d, -1)
    ev[:, 3] = np.where(ev[:, 3] >= 0, ev[:, 3] * P + d, -1)
    assert np.array_equal(ev, want)
    assert np.array_equal(rng.key, after[1]) and rng.pos.value == after[2]
    chg = np.nonzero(want[:, 2] >= 0)[0]
    assert len(chg) == 2 and list(chg + 1) == [12_500, 25_000], chg
    assert (want[:, 0] < 0).all()
    del part
    torch.cuda.empty_cache()


def test_c3_full_size_property_on_bench_path():
    """configs[2] at its full size -- 8 partitions x 125M rows of the 1B-row stream, global
    class blocks of 10,000,037 rows -- through the BatchRunner exactly as bench.py runs it:
    one drift per class boundary, in the batch holding it, AT the first new-class row of
    that batch in shuffled order (the MT19937 draws replayed by oracle/mt_replay.c), no
    warning, and every partition's RNG position == the replay's."""
    import bench
    from ddm_amd import synth
    from ddm_amd.controller import BatchRunner
    from ddm_amd.params import DDMSettings
    from ddm_amd.rng import MTStream
    dev = _dev()
    n, P, block = 125_000_000, bench.C3_PARTS, bench.C3_BLOCK
    parts = [synth.block_partition(n, d, P, block, bench.SEED, dev) for d in range(P)]
    runner = BatchRunner(parts, DDMSettings(), torch.cuda.Stream(dev, priority=-1), timing=True, fit_threads=16)
    rngs = [MTStream.from_seed(bench.SEED + d) for d in range(P)]
    outs = runner.run(rngs)
    runner.close()
    res = dict(enumerate(outs))
    bench.c3_property_check(res, n, P, block, seeds={d: bench.SEED + d for d in range(P)},
                            rng_after=dict(enumerate(rngs)))
    n_drifts = sum(int((r[:, 1] >= 0).sum()) for r in outs)
    assert n_drifts == sum(
        len([k for k in range(1, (n * P + d) // block + 1) if 100 <= (k * block - d + P - 1) // P < n])
        for d in range(P))
    assert n_drifts == 792
    del parts
    torch.cuda.empty_cache()
