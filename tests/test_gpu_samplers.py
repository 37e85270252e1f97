"""GPU-scale forms of test.cpp's samplers (msim_sample_picks / msim_sample_intervals):
bit-exact against the sequential oracle loops for the same seed, plus the reference's own expectations
at its full sample sizes (test.cpp:10-14: 10^8 picks over 100 x 1 % miners -> mean 10^6, std dev ~10^3;
test.cpp:188-190: 10^8 intervals -> mean ~ std dev ~ 600 000 ms); and the simulated configs[4] stale
rates against the analytical model (plot.py restated, model.py)."""
import numpy as np
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


def _sim(msim, weights, W=100):
    return msim.Simulation([msim.Miner(k, w, 0) for k, w in enumerate(weights)], total_weight=W)


@pytest.mark.parametrize("weights,W", [([1] * 100, 100), ([30, 29, 12, 11, 8, 5, 3, 1, 1], 100),
                                       ([12, 18, 20, 15, 35], 100), ([30720, 29696] + [41] * 1024, 102400)])
def test_gpu_pick_counts_exact(msim, oracle, weights, W):
    n = 3_000_017
    got = msim.sample_picks(_sim(msim, weights, W), 777, n)
    want = oracle.pick_counts(weights, W, 777, n)
    assert np.array_equal(got, want)
    assert int(got.sum()) == n


def test_gpu_interval_moments_exact(msim, oracle):
    n = 5_000_003
    got = msim.sample_intervals(4242, n)
    want = oracle.interval_moments(4242, n)
    assert (got["sum"], got["sumsq"], got["max"]) == (want["sum"], want["sumsq"], want["max"])


def test_gpu_miner_picker_sample_full_size(msim):
    """test.cpp:15-63 at its own size: 10^8 picks, 100 miners of 1 %."""
    c = msim.sample_picks(_sim(msim, [1] * 100), 12345, 100_000_000)
    assert c[-1] == 0
    counts = c[:-1].astype(np.float64)
    assert counts.mean() == 1_000_000
    assert 800 < counts.std() < 1200


def test_gpu_block_interval_sample_full_size(msim):
    """test.cpp:191-208 at its own size: 10^8 intervals, mean and std dev ~600 000 ms."""
    mo = msim.sample_intervals(99, 100_000_000)
    assert abs(mo["mean"] - 599_999.5) < 200
    assert abs(mo["std"] - 600_000) < 300


def test_gpu_c5_stale_rates_vs_model(msim):
    """configs[4] (1 026 miners, 1 s) simulated on the GPU vs the first-order model: pools within 10 %,
    the 1 024 small miners' mean within 25 % (the model's race term is cruder for tiny miners)."""
    w = [30720, 29696] + [41] * 1024
    sim = msim.Simulation([msim.Miner(k, x, 1000) for k, x in enumerate(w)], total_weight=102400)
    n = 16384
    res = sim.run(n, 0, 1000, 0)
    rate = np.array([s.stale_rate for s in res.stats_total]) / n
    mod = np.array(msim.model.stale_rates([x / 102400 for x in w], 1.0))
    assert np.all(np.abs(rate[:2] / mod[:2] - 1) < 0.10), (rate[:2], mod[:2])
    assert abs(rate[2:].mean() / mod[2:].mean() - 1) < 0.25, (rate[2:].mean(), mod[2:].mean())
