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


def test_gpu_miner_picker_small_big_full_size(msim):
    """test.cpp:68-119 MinerPickerSmallBig at its own size: 10^4 x 10^3 x 100 = 10^9 picks over miners
    {12, 18, 20, 15, 35} %. The reference prints the sample mean of blocks per 100; its expectation is
    100 * perc / 100 per miner (no skew with hashrate). Here: the total counts, within 5 sigma of a
    multinomial(10^9, perc)."""
    perc = [12, 18, 20, 15, 35]
    n = 1_000_000_000
    c = msim.sample_picks(_sim(msim, perc), 20240601, n)
    assert c[-1] == 0 and int(c.sum()) == n
    for k, pc in enumerate(perc):
        p = pc / 100
        mean_per_100 = float(c[k]) / n * 100  # the reference's "sample mean" (blocks per 100 picks)
        sigma = (p * (1 - p) / n) ** 0.5 * 100
        assert abs(mean_per_100 - pc) < 5 * sigma, (k, mean_per_100)


def test_gpu_simple_sim_full_size(msim, oracle):
    """test.cpp:122-187 SimpleSim at its own size: 100 samples x 100 runs of two weeks
    (BLOCK_INTERVAL * 144 * 14), miners {12, 18, 20, 15, 35} %, propagation 0. The reference steps time
    in 1 s increments and prints, per miner, the sample mean of BlocksFoundShare (expected: perc) and the
    std dev of the sample mean. Here the same network runs through the event-driven device path
    (msim_run; exact block times rather than 1 s steps, and without test.cpp's quirks of dropping the
    genesis block on chain.clear() and never resetting stale_blocks), so the check is statistical:
    sample means within 5 sigma of perc, the std dev of the sample means close to the binomial value,
    and no stale blocks beyond same-millisecond ties. The first 64 runs are bit-exact vs the oracle."""
    perc = [12, 18, 20, 15, 35]
    dur = 600_000 * 144 * 14
    sim = msim.Simulation([msim.Miner(k, w, 0) for k, w in enumerate(perc)], duration_ms=dur)
    n_samples, n_size = 100, 100
    res = sim.run(n_samples * n_size, 0, 1000, 0, per_run=True)
    f, st, _, _ = oracle.run_batch(perc, [0] * 5, [False] * 5, dur, 64, 0, 1000, threads=16)
    assert np.array_equal(res.found[:64].astype(np.int64), f)
    assert np.array_equal(res.stale[:64].astype(np.int64), st)
    share = res.found.astype(np.float64) / res.best_height.astype(np.float64)[:, None]
    means = share.reshape(n_samples, n_size, 5).mean(axis=1)  # [sample, miner]
    blocks = float(res.best_height.mean())
    assert abs(blocks - 2016) < 5 * (2016 ** 0.5) / (n_samples * n_size) ** 0.5
    for k, pc in enumerate(perc):
        p = pc / 100
        sm = means[:, k].mean()
        sd = means[:, k].std()
        sd_expect = (p * (1 - p) / (blocks * n_size)) ** 0.5
        assert abs(sm - p) < 5 * sd_expect / n_samples ** 0.5, (k, sm)
        assert 0.7 * sd_expect < sd < 1.3 * sd_expect, (k, sd, sd_expect)
    assert int(res.stale.sum()) <= 1e-4 * int(res.found.sum())
