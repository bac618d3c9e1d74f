"""Device-resident epochs (csrc/ctl.hip, ddm_amd/devctl.py) == host-driven epochs == the
oracle: the epoch decisions of run_DDM_loop (DDM_Process.py:189-210) taken on the device
must give the same events and leave every partition's RNG where the reference leaves it."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _parts(sizes, F, block, seed, flip=0.0, jitter=False):
    from ddm_amd import kernels
    from ddm_amd.controller import DevicePartition
    dev = torch.device("cuda", 0)
    parts = []
    for k, n in enumerate(sizes):
        part = DevicePartition.allocate(n, F, dev)
        if jitter:
            kernels.synth_jitter_labels(part.y[:n], k, len(sizes), 1800, 300, 10, flip, seed)
        else:
            kernels.synth_block_labels(part.y[:n], part=k, n_parts=len(sizes), block_rows=block, n_classes=10)
        kernels.synth_features(part.X, part.y[:n], row0=k, row_stride=len(sizes), seed=seed, noise=0.04)
        parts.append(part)
    torch.cuda.synchronize()
    return parts


def _run(parts, device_ctl, seeds, win=256, maxwin=1 << 16):
    from ddm_amd.controller import BatchRunner
    from ddm_amd.params import DDMSettings
    from ddm_amd.rng import MTStream
    runner = BatchRunner(parts, DDMSettings(window_batches=win, max_window_batches=maxwin), device_ctl=device_ctl)
    rngs = [MTStream.from_seed(s) for s in seeds]
    out = runner.run(rngs)
    st = runner.stats
    runner.close()
    return out, [(r.key.copy(), r.pos.value) for r in rngs], st


@pytest.mark.parametrize("case", ["blocks", "jitter", "noise", "tails"])
def test_device_epochs_equal_host_epochs(case):
    if case == "blocks":
        parts = _parts((60_000,) * 4, 27, 20_011, 3)
    elif case == "jitter":
        parts = _parts((24_000,) * 4, 27, 0, 5, jitter=True)
    elif case == "noise":
        parts = _parts((30_000, 30_000), 27, 0, 7, flip=0.01, jitter=True)
    else:       # short last batches, one partition much shorter than the others
        parts = _parts((24_037, 17_055, 4_321, 9_999), 27, 6_007, 9)
    seeds = [100 + k for k in range(len(parts))]
    dev_out, dev_rng, st = _run(parts, True, seeds)
    host_out, host_rng, st_h = _run(parts, False, seeds)
    assert st.device_epochs > 0 and st_h.device_epochs == 0
    for k in range(len(parts)):
        assert np.array_equal(dev_out[k], host_out[k]), k
        assert np.array_equal(dev_rng[k][0], host_rng[k][0]) and dev_rng[k][1] == host_rng[k][1], k
    assert st.refits == st_h.refits


@pytest.mark.parametrize("case", ["blocks", "noise", "tails"])
def test_decoupled_epochs_equal_host_epochs(case, monkeypatch):
    """Decoupled device epochs (row-order predict, permutation into DDM order after the
    window's shuffles, csrc/ctl.hip) forced on for every group: the same events, RNG
    positions and refits as host epochs."""
    from ddm_amd import devctl
    monkeypatch.setattr(devctl, "DECOUPLE_ROWS", 0)
    if case == "blocks":
        parts = _parts((60_000,) * 4, 28, 20_011, 3)
    elif case == "noise":
        parts = _parts((30_000, 30_000), 27, 0, 7, flip=0.01, jitter=True)
    else:
        parts = _parts((24_037, 17_055, 4_321, 9_999), 27, 6_007, 9)
    seeds = [200 + k for k in range(len(parts))]
    dev_out, dev_rng, st = _run(parts, True, seeds)
    host_out, host_rng, st_h = _run(parts, False, seeds)
    assert st.device_epochs > 0 and st_h.device_epochs == 0
    for k in range(len(parts)):
        assert np.array_equal(dev_out[k], host_out[k]), k
        assert np.array_equal(dev_rng[k][0], host_rng[k][0]) and dev_rng[k][1] == host_rng[k][1], k
    assert st.refits == st_h.refits


@pytest.mark.parametrize("flags,device_start", [(True, True), (False, True), (True, False), (False, False)])
def test_device_epochs_vs_oracle(flags, device_start, monkeypatch):
    """Partitions with many refits, run with device epochs, == the oracle on each: fork / join
    by device flags or by HIP events (DDM_CTL_FLAGS=0), the first fit on the device or a
    host-planned first epoch (DDM_DEVICE_START=0)."""
    from ddm_amd import controller, devctl
    from oracle.controller import run_partition
    monkeypatch.setattr(devctl, "CTL_FLAGS", flags)
    monkeypatch.setattr(controller, "DEVICE_START", device_start)
    parts = _parts((12_000, 9_050, 15_100), 27, 0, 11, flip=0.005, jitter=True)
    seeds = [7, 8, 9]
    out, rng, st = _run(parts, True, seeds, win=7, maxwin=64)
    assert st.device_epochs > 0
    drifts = 0
    for k, part in enumerate(parts):
        X = part.X[:, :part.n].t().contiguous().cpu().numpy().astype(np.float64)
        y = part.y[:part.n].cpu().numpy().astype(np.int64)
        np.random.seed(seeds[k])
        want = run_partition(X, y, np.arange(part.n), np.arange(part.n))
        assert np.array_equal(out[k][:, 0], want[:, 0]) and np.array_equal(out[k][:, 1], want[:, 2]), k
        after = np.random.get_state()
        assert np.array_equal(rng[k][0], after[1]) and rng[k][1] == after[2], k
        drifts += int((want[:, 2] >= 0).sum())
    assert drifts >= 50


@pytest.mark.parametrize("case,decouple,timed", [("jitter", False, False), ("blocks", True, True),
                                                 ("tails", False, True), ("noise", True, False)])
def test_graph_epochs_equal_host_epochs(case, decouple, timed, monkeypatch):
    """Groups of device epochs captured once as hipGraphs and replayed (DDM_CTL_GRAPH,
    ddm_ctl_graph_create; with predict timing the launched form runs instead): the same
    events, RNG positions and refits as host epochs, over two runs of the same runner (the
    cached graphs replayed again)."""
    from ddm_amd import devctl
    from ddm_amd.controller import BatchRunner
    from ddm_amd.params import DDMSettings
    from ddm_amd.rng import MTStream
    monkeypatch.setattr(devctl, "CTL_GRAPH", True)
    if decouple:
        monkeypatch.setattr(devctl, "DECOUPLE_ROWS", 0)
    if case == "blocks":
        parts = _parts((60_000,) * 4, 27, 20_011, 3)
    elif case == "jitter":
        parts = _parts((24_000,) * 4, 27, 0, 5, jitter=True)
    elif case == "noise":
        parts = _parts((30_000, 30_000), 27, 0, 7, flip=0.01, jitter=True)
    else:
        parts = _parts((24_037, 17_055, 4_321, 9_999), 27, 6_007, 9)
    seeds = [300 + k for k in range(len(parts))]
    host_out, host_rng, st_h = _run(parts, False, seeds)
    runner = BatchRunner(parts, DDMSettings(), device_ctl=True)
    if timed:
        runner.set_predict_timing(True)
    for rep in range(2):
        rngs = [MTStream.from_seed(s) for s in seeds]
        out = runner.run(rngs)
        for k in range(len(parts)):
            assert np.array_equal(out[k], host_out[k]), (rep, k)
            assert np.array_equal(rngs[k].key, host_rng[k][0]) and rngs[k].pos.value == host_rng[k][1], (rep, k)
    st = runner.stats
    assert st.device_epochs > 0 and (timed or len(runner.devctl.graphs) > 0)
    if timed:
        assert st.predict_dev_launches > 0 and st.predict_dev_ms > 0
        runner.set_predict_timing(False)
    runner.close()


@pytest.mark.parametrize("decouple", [False, True])
def test_flag_timeout_voids_and_redoes_the_run(decouple, monkeypatch):
    """A cross-stream flag wait that gives up (csrc/common.h flag_poll, forced here by a
    1-tick limit in sync_flags[3]) voids the device phase: the runner redoes the run from
    the callers' RNG states with event-ordered fork / join, and the events, RNG positions
    and refits equal host epochs (DDM_Process.py:189-210)."""
    from ddm_amd import devctl
    from ddm_amd.controller import BatchRunner
    from ddm_amd.params import DDMSettings
    from ddm_amd.rng import MTStream
    if decouple:
        monkeypatch.setattr(devctl, "DECOUPLE_ROWS", 0)
    parts = _parts((30_000, 30_000), 27, 0, 7, flip=0.01, jitter=True)
    seeds = [400, 401]
    host_out, host_rng, st_h = _run(parts, False, seeds)
    runner = BatchRunner(parts, DDMSettings(), device_ctl=True)
    runner.devctl.set_flag_limit(1)
    rngs = [MTStream.from_seed(s) for s in seeds]
    out = runner.run(rngs)
    st = runner.stats
    assert st.flag_recoveries == 1 and not runner.devctl.flags_ok
    for k in range(len(parts)):
        assert np.array_equal(out[k], host_out[k]), k
        assert np.array_equal(rngs[k].key, host_rng[k][0]) and rngs[k].pos.value == host_rng[k][1], k
    # the runner stays usable (events from now on), and a second run gives the same
    rngs = [MTStream.from_seed(s) for s in seeds]
    out = runner.run(rngs)
    for k in range(len(parts)):
        assert np.array_equal(out[k], host_out[k]), k
    assert runner.stats.flag_recoveries == 1
    runner.close()
