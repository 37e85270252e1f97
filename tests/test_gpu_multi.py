"""The multi-GPU entry points on one MI355X: msim_run_multi (RCCL single-process communicator) and
distributed.run_sharded (one process per GPU, torch.distributed) at one device, against msim_run, bit for
bit. The reference's aggregation is main.cpp:205-217 (std::async runs, stats_total += stats)."""
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def msim(msim_lib_path):
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    torch.cuda.set_device(0)
    import miningsimulation_amd as m

    return m


def _rows(sums):
    return [[s.blocks_found, s.stale_blocks, s.share_hi, s.share_lo, s.rate_hi, s.rate_lo] for s in sums]


@pytest.mark.parametrize("preset,n", [("c2", 8192), ("c3", 4096), ("c1", 3001)])
def test_gpu_run_multi_one_device_equals_run(msim, preset, n):
    sim = msim.Simulation(msim.PRESETS[preset]())
    a = sim.run(n, 777, 1000, 0)
    b = sim.run_multi(n, 777, 1000, devices=[0])
    assert _rows(a.sums) == _rows(b.sums)
    for x, y in zip(a.stats_total, b.stats_total):
        assert (x.blocks_found, x.blocks_share, x.stale_rate) == (y.blocks_found, y.blocks_share, y.stale_rate)


def test_gpu_run_sharded_world1_equals_run(msim):
    import torch

    from miningsimulation_amd.distributed import run_sharded

    sim = msim.Simulation(msim.PRESETS["c2"]())
    n = 10_000
    got = run_sharded(sim, n, 1000, run_begin=50).cpu().tolist()
    assert got == _rows(sim.run(n, 50, 1000, 0).sums)
    torch.cuda.synchronize()


@pytest.mark.parametrize("preset", ["c2", "c3"])
def test_gpu_two_shards_sum_to_whole(msim, preset):
    """Two shard() halves launched separately and added (what the all-reduce computes) equal one launch."""
    from miningsimulation_amd.distributed import shard

    sim = msim.Simulation(msim.PRESETS[preset]())
    n = 6001
    whole = _rows(sim.run(n, 0, 1000, 0).sums)
    parts = []
    for r in range(2):
        b, c = shard(n, 2, r)
        parts.append(_rows(sim.run(c, b, 1000, 0).sums))
    added = [[x + y for x, y in zip(ra, rb)] for ra, rb in zip(*parts)]
    assert added == whole
    assert msim.sums_to_stats(added) == msim.sums_to_stats(whole)


def test_gpu_sweep_run_multi_one_device_equals_sweep_run(msim):
    """A 12-point slice of the configs[3] grid (selfish share x propagation) through msim_sweep_run_multi."""
    grid = msim.c4_grid()
    pts = [grid[i] for i in range(0, 360, 30)]
    sw = msim.Sweep(pts)
    a = sw.run(1024, 0, 1000, 0)
    b = sw.run_multi(1024, 0, 1000, devices=[0])
    for x, y in zip(a, b):
        assert _rows(x.sums) == _rows(y.sums)
        assert x.stats_total == y.stats_total


@pytest.mark.parametrize("preset", ["c2", "c3"])
def test_gpu_run_sharded_side_stream_many_chunks(msim, preset):
    """run_sharded on a non-current stream with several chunks reusing one output buffer: the adds and
    the reduction are ordered after each chunk's kernels, so the sums equal one msim_run."""
    import torch

    from miningsimulation_amd.distributed import run_sharded

    sim = msim.Simulation(msim.PRESETS[preset]())
    n = 5000
    st = torch.cuda.Stream()
    got = run_sharded(sim, n, 1000, run_begin=123, stream=st, max_chunk=1024).cpu().tolist()
    assert got == _rows(sim.run(n, 123, 1000, 0).sums)


def test_gpu_run_multi_shard_timing_and_release(msim):
    """msim_run_multi_timed reports each device's launch and all-reduce milliseconds (HIP events on its stream);
    msim_multi_release frees cached communicators (none exist for one device)."""
    from miningsimulation_amd._lib import lib

    sim = msim.Simulation(msim.PRESETS["c2"]())
    r = sim.run_multi(4096, 0, 1000, devices=[0])
    (launch_ms, reduce_ms), = r.extra["shard_ms"]
    assert launch_ms > 0.0 and reduce_ms >= 0.0
    assert lib.msim_multi_release() == 0
