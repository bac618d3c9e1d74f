"""The drop-in `run_DDM_loop` on the GPU vs the reference's own outputs (golden fixtures from
executing DDM_Process.py:94-213) — bit-exact events for every (MULT, INSTANCES) config."""
import numpy as np
import pandas as pd
import pytest
import torch

from conftest import golden_configs, golden_partitions

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("mult,inst", golden_configs())
def test_drop_in_matches_reference(mult, inst):
    import ddm_amd
    for d, part, expect in golden_partitions(mult, inst):
        np.random.seed(1000 + d)
        if expect is None:
            with pytest.raises(ValueError, match="No objects to concatenate"):
                ddm_amd.run_DDM_loop(part)
            continue
        got = ddm_amd.run_DDM_loop(part)
        assert list(got.columns) == ddm_amd.OUTPUT_COLUMNS
        assert list(got.index) == [0] * len(expect)
        assert np.array_equal(got.to_numpy(), expect), (mult, inst, d)


def test_global_rng_left_where_reference_leaves_it():
    import ddm_amd
    from oracle.controller import run_partition
    d, part, expect = golden_partitions(2, 4)[2]
    np.random.seed(5)
    np.random.standard_normal()          # leaves a cached Gaussian (has_gauss = 1)
    ddm_amd.run_DDM_loop(part)
    after_gpu = np.random.get_state()
    np.random.seed(5)
    np.random.standard_normal()
    run_partition(part[[str(i) for i in range(21)]].to_numpy(), part["target"].to_numpy(), part.index.to_numpy(),
                  part["full_df_row_number"].to_numpy())
    after_ref = np.random.get_state()
    assert np.array_equal(after_gpu[1], after_ref[1]) and after_gpu[2] == after_ref[2]
    assert after_ref[3] == 1 and after_gpu[3:] == after_ref[3:]


@pytest.mark.parametrize("win,maxwin", [(1, 1), (1, 4), (3, 1000), (10_000, 1 << 16)])
def test_window_schedule_does_not_change_results(win, maxwin):
    import ddm_amd
    for d, part, expect in golden_partitions(4, 4):
        np.random.seed(1000 + d)
        s = ddm_amd.DDMSettings(window_batches=win, max_window_batches=maxwin)
        got = ddm_amd.run_DDM_loop(part, settings=s)
        assert np.array_equal(got.to_numpy(), expect)


def test_edge_partitions():
    import ddm_amd
    part = pd.DataFrame({"0": np.arange(100.0), "target": np.zeros(100, int), "full_df_row_number": np.arange(100)})
    with pytest.raises(ValueError, match="No objects to concatenate"):
        ddm_amd.run_DDM_loop(part)
    with pytest.raises(IndexError):
        ddm_amd.run_DDM_loop(part.iloc[:0])
    one = ddm_amd.run_DDM_loop(pd.concat([part, part.iloc[:1]]).reset_index(drop=True))
    assert one.shape == (1, 4)


def test_concurrent_partitions_on_streams():
    """All partitions of a config at once, one stream + thread each (apply_in_pandas path)."""
    from ddm_amd.partition import run_partitions
    parts = golden_partitions(4, 16)
    outs = run_partitions([(d, p) for d, p, _ in parts], {d: 1000 + d for d, _, _ in parts})
    for d, _, expect in parts:
        assert np.array_equal(outs[d].to_numpy(), expect), d


def test_synthetic_rialto_stream_vs_oracle():
    """Device-generated rialto-shaped partition (27 features, class blocks not aligned to
    batches) through the GPU controller == the oracle on the same rows."""
    from ddm_amd import kernels
    from ddm_amd.controller import DevicePartition, PartitionRunner
    from ddm_amd.params import DDMSettings
    from ddm_amd.rng import MTStream
    from oracle.controller import run_partition
    dev = torch.device("cuda", 0)
    n, F, parts, block = 30_000, 27, 4, 10_037
    part = DevicePartition.allocate(n, F, dev)
    kernels.synth_block_labels(part.y[:n], part=1, n_parts=parts, block_rows=block, n_classes=10)
    kernels.synth_features(part.X, part.y[:n], row0=1, row_stride=parts, seed=99, noise=0.04)
    torch.cuda.synchronize()
    X = part.X[:, :n].t().contiguous().cpu().numpy()
    y = part.y[:n].cpu().numpy().astype(np.int64)
    runner = PartitionRunner(part, DDMSettings())
    got = runner.run(MTStream.from_seed(321))
    np.random.seed(321)
    want = run_partition(X.astype(np.float64), y, np.arange(n), np.arange(n))
    assert np.array_equal(got[:, 0], want[:, 0]) and np.array_equal(got[:, 1], want[:, 2])
    assert (want[:, 2] >= 0).sum() >= 3


@pytest.mark.parametrize("win,maxwin,refit", [(256, 1 << 16, "device"), (1, 8, "device"), (7, 64, "device"),
                                              (256, 1 << 16, "native"), (7, 64, "native")])
def test_lockstep_batch_of_unequal_partitions_vs_oracle(win, maxwin, refit):
    """Partitions of different lengths (short tails, one finishing epochs before the
    others) in ONE BatchRunner == the oracle run on each partition alone."""
    from ddm_amd import kernels
    from ddm_amd.controller import BatchRunner, DevicePartition
    from ddm_amd.params import DDMSettings
    from ddm_amd.rng import MTStream
    from oracle.controller import run_partition
    dev = torch.device("cuda", 0)
    sizes, F = (24_000, 17_055, 4_321, 250, 9_999), 27
    parts, host = [], []
    for k, n in enumerate(sizes):
        part = DevicePartition.allocate(n, F, dev)
        kernels.synth_block_labels(part.y[:n], part=k, n_parts=len(sizes), block_rows=6_007, n_classes=10)
        kernels.synth_features(part.X, part.y[:n], row0=k, row_stride=len(sizes), seed=7, noise=0.04)
        parts.append(part)
    torch.cuda.synchronize()
    for part in parts:
        host.append((part.X[:, :part.n].t().contiguous().cpu().numpy().astype(np.float64),
                     part.y[:part.n].cpu().numpy().astype(np.int64)))
    runner = BatchRunner(parts, DDMSettings(window_batches=win, max_window_batches=maxwin), refit=refit)
    rngs = [MTStream.from_seed(50 + k) for k in range(len(parts))]
    got = runner.run(rngs)
    runner.close()
    drifts = 0
    for k, (X, y) in enumerate(host):
        np.random.seed(50 + k)
        want = run_partition(X, y, np.arange(len(y)), np.arange(len(y)))
        assert np.array_equal(got[k][:, 0], want[:, 0]) and np.array_equal(got[k][:, 1], want[:, 2]), k
        after = np.random.get_state()
        assert np.array_equal(rngs[k].key, after[1]) and rngs[k].pos.value == after[2], k
        drifts += int((want[:, 2] >= 0).sum())
    assert drifts >= 5
    # every refit after a change ran on the device, the first one of each partition natively
    if refit == "device":
        assert runner.stats.device_refits > 0
        assert runner.stats.device_refits + len(parts) >= runner.stats.refits - 1
    else:
        assert runner.stats.device_refits == 0


def test_batches_with_more_than_64_classes_vs_oracle():
    """a training batch with more than 64 classes (the native / device
    trainers' limit) is refit by sklearn on the host and its forest predicted on the device
    by the wide node-walk variants (up to 256 classes), instead of raising; == the oracle,
    RNG position included."""
    from ddm_amd.controller import BatchRunner, DevicePartition
    from ddm_amd.params import DDMSettings
    from ddm_amd.rng import MTStream
    from oracle.controller import run_partition
    dev = torch.device("cuda", 0)
    rs = np.random.RandomState(12)
    n, F = 2_600, 5
    y = np.concatenate([np.arange(n // 2) % 90, 90 + np.arange(n - n // 2) % 80]).astype(np.int64)
    X = np.stack([y + 0.3 * rs.rand(n)] + [rs.rand(n) for _ in range(F - 1)], axis=1)
    part = DevicePartition.from_columns(np.ascontiguousarray(X.T.astype(np.float32)), y, dev)
    runner = BatchRunner([part], DDMSettings())
    rng = MTStream.from_seed(77)
    got = runner.run([rng])[0]
    runner.close()
    np.random.seed(77)
    want = run_partition(X.astype(np.float32).astype(np.float64), y, np.arange(n), np.arange(n))
    assert np.array_equal(got[:, 0], want[:, 0]) and np.array_equal(got[:, 1], want[:, 2])
    after = np.random.get_state()
    assert np.array_equal(rng.key, after[1]) and rng.pos.value == after[2]
    assert runner.stats.sklearn_refits >= 1
    assert (want[:, 2] >= 0).sum() + (want[:, 0] >= 0).sum() >= 1
