"""Parity of the gfx950 large-network pipeline (msim_wide.h / msim_wide.hip, BASELINE configs[4]) through
libmsim's C ABI, against the CPU oracle (oracle/msim_oracle.c with the SURVEY Appendix C weights) and
against the narrow device path.

Bar: bit-exact per-run integer counters (found, stale, best height) for identical seeds. Networks with
W != 100 are not expressible in the reference (integer percentages, main.cpp:43): parity there is to the
oracle restatement only ("parity unpinned" by the reference); W = 100 networks forced onto the wide path
are pinned through the same golden vectors as the narrow path."""
import os
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

YEAR = 31_556_952_000
DAY = 86_400_000
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def msim(msim_lib_path):
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    torch.cuda.set_device(0)
    import miningsimulation_amd as m

    return m


def _wide(msim, weights, props, W, duration=YEAR):
    miners = [msim.Miner(k, weights[k], props[k]) for k in range(len(weights))]
    sim = msim.Simulation(miners, duration, total_weight=W)
    assert sim.wide
    return sim


def _vs_oracle(msim, oracle, weights, props, W, duration, n, begin=0, base=1000):
    res = _wide(msim, weights, props, W, duration).run(n, begin, base, 0, per_run=True)
    f, s, sh, r = oracle.run_batch(weights, props, [0] * len(weights), duration, n, begin, base, threads=16,
                                   total_weight=W)
    assert np.array_equal(res.found.astype(np.int64), f), np.argwhere(res.found != f)[:5]
    assert np.array_equal(res.stale.astype(np.int64), s), np.argwhere(res.stale != s)[:5]
    assert np.array_equal(res.best_height.astype(np.int64), f.sum(axis=1))
    return res, f, s, sh, r


def test_gpu_wide_picks(msim, oracle):
    """Weighted PickFinder on the device (bucket table + cumulative scan) vs the oracle's linear scan."""
    import ctypes

    import torch
    from miningsimulation_amd import _lib

    w = [30720, 29696] + [41] * 1024
    sim = _wide(msim, w, [1000] * len(w), 102400)
    words = np.array(oracle.rng_stream(11, 1 << 16), dtype=np.uint64)
    du = torch.from_numpy(words.view(np.int64)).cuda()
    dk = torch.empty(words.size, dtype=torch.int32, device="cuda")
    _lib.check(_lib.lib.msim_device_picks(sim.handle, ctypes.c_void_p(du.data_ptr()), ctypes.c_void_p(dk.data_ptr()),
                                          words.size, None))
    torch.cuda.synchronize()
    assert dk.cpu().tolist() == oracle.picks_w(w, 102400, 11, 1 << 16)


def test_gpu_wide_c5_year_vs_oracle(msim, oracle):
    """BASELINE configs[4] network, full year, run by run vs the oracle, plus the run-order f64 sums."""
    w = [30720, 29696] + [41] * 1024
    n = 48
    res, f, s, sh, r = _vs_oracle(msim, oracle, w, [1000] * len(w), 102400, YEAR, n, begin=1 << 20)
    assert s.sum() > 0
    for k in (0, 1, 2, 700, 1025):
        ref_share = 0.0
        ref_rate = 0.0
        for i in range(n):
            ref_share += sh[i, k]
            ref_rate += r[i, k]
        assert res.stats_total[k].blocks_found == int(f[:, k].sum())
        assert res.stats_total[k].blocks_share == ref_share
        assert res.stats_total[k].stale_rate == ref_rate


@pytest.mark.parametrize("duration", [0, 1, 600_000, 3 * DAY, 40 * DAY])
def test_gpu_wide_c5_short_vs_oracle(msim, oracle, duration):
    w = [30720, 29696] + [41] * 1024
    _vs_oracle(msim, oracle, w, [1000] * len(w), 102400, duration, 256)


@pytest.mark.parametrize("seed", range(4))
def test_gpu_wide_random_networks(msim, oracle, seed):
    """Heterogeneous weights (zeros included) and propagations (0 ms .. 20 s), 3..300 miners."""
    rnd = random.Random(100 + seed)
    m = rnd.choice([3, 17, 40, 300])
    w = [rnd.choice([0, 1, 2, 5, 40, 300]) for _ in range(m)]
    w[rnd.randrange(m)] += 500
    props = [rnd.choice([0, 1, 50, 700, 3000, 20_000]) for _ in range(m)]
    _vs_oracle(msim, oracle, w, props, sum(w), rnd.choice([20 * DAY, 120 * DAY, YEAR]), 64,
               base=rnd.randrange(1 << 32))


@pytest.mark.parametrize("name", ["c1_prop10s", "c2_prop100ms", "default_prop1s"])
def test_gpu_wide_golden_vectors(msim, name, monkeypatch):
    """W = 100 networks forced onto the wide path reproduce the golden vectors (pinned to the reference)."""
    monkeypatch.setenv("MSIM_FORCE_WIDE", "1")
    z = np.load(os.path.join(GOLD, "oracle_vectors.npz"))
    p, q, s = z[name + "_config"].tolist()
    miners = [msim.Miner(k, p[k], q[k], bool(s[k])) for k in range(len(p))]
    sim = msim.Simulation(miners, YEAR)
    assert sim.wide
    res = sim.run(64, 0, 1000, 0, per_run=True)
    assert np.array_equal(res.found.astype(np.int64), z[name + "_found"])
    assert np.array_equal(res.stale.astype(np.int64), z[name + "_stale"])
    assert np.array_equal(res.best_height.astype(np.int64), z[name + "_best_height"])


def test_gpu_wide_equals_narrow_pipeline(msim, monkeypatch):
    """Two independent device implementations of RunSimulation on 8192 runs of the default network."""
    miners = msim.PRESETS["default"]()
    narrow = msim.Simulation(miners).run(8192, 5000, 1000, 0, per_run=True)
    monkeypatch.setenv("MSIM_FORCE_WIDE", "1")
    sim = msim.Simulation(miners)
    assert sim.wide
    wide = sim.run(8192, 5000, 1000, 0, per_run=True)
    assert np.array_equal(narrow.found, wide.found)
    assert np.array_equal(narrow.stale, wide.stale)
    for k in range(9):
        a, b = narrow.sums[k], wide.sums[k]
        assert a.blocks_found == b.blocks_found and a.stale_blocks == b.stale_blocks
        assert (a.share_hi << 32) + a.share_lo == (b.share_hi << 32) + b.share_lo
        assert (a.rate_hi << 32) + a.rate_lo == (b.rate_hi << 32) + b.rate_lo
        # the reported f64 statistics are bit-identical (one rounding of the exact limb sum)
        x, y = narrow.stats_total[k], wide.stats_total[k]
        assert x.blocks_share == y.blocks_share and x.stale_rate == y.stale_rate


def test_gpu_wide_c5_full_slice_invariants(msim):
    """65536 full-year runs of configs[4] in one launch: no failed run, sum of found = best height per run,
    shares near the weights, honest stale rates near the 1 s first-order model (plot.py:22-77)."""
    w = [30720, 29696] + [41] * 1024
    sim = _wide(msim, w, [1000] * len(w), 102400)
    n = 65536
    res = sim.run(n, 0, 1000, 0, per_run=True)
    assert np.array_equal(res.found.sum(axis=1).astype(np.int64), res.best_height.astype(np.int64))
    share0 = res.stats_total[0].blocks_share / n
    share_small = sum(res.stats_total[k].blocks_share for k in range(2, 1026)) / n
    assert abs(share0 - 0.30) < 0.002
    assert abs(share_small - 0.41) < 0.002
    rate_small = np.mean([res.stats_total[k].stale_rate for k in range(2, 1026)]) / n
    assert 0.0005 < rate_small < 0.004


def test_gpu_wide_sharding_is_exact(msim):
    w = [30720, 29696] + [41] * 1024
    sim = _wide(msim, w, [1000] * len(w), 102400, 60 * DAY)
    n = 4096
    whole = sim.run(n, 0, 1000, 0)
    a = sim.run(n // 2, 0, 1000, 0)
    b = sim.run(n // 2, n // 2, 1000, 0)
    for k in range(len(w)):
        x, y, z = whole.sums[k], a.sums[k], b.sums[k]
        assert x.blocks_found == y.blocks_found + z.blocks_found
        assert x.stale_blocks == y.stale_blocks + z.stale_blocks
        assert (x.share_hi << 32) + x.share_lo == (y.share_hi << 32) + y.share_lo + (z.share_hi << 32) + z.share_lo
    # the two halves' limbs added as a caller (or an all-reduce) would, then converted: bit for bit equal
    rows = [[y.blocks_found + z.blocks_found, y.stale_blocks + z.stale_blocks, y.share_hi + z.share_hi,
             y.share_lo + z.share_lo, y.rate_hi + z.rate_hi, y.rate_lo + z.rate_lo]
            for y, z in zip(a.sums, b.sums)]
    for s_whole, s_halves in zip(whole.stats_total, msim.sums_to_stats(rows)):
        assert s_whole.blocks_share == s_halves.blocks_share
        assert s_whole.stale_rate == s_halves.stale_rate


@pytest.mark.parametrize("runs", ["", "1", "2", "8"])
def test_gpu_wide_max_network_any_runs_per_workgroup(msim, oracle, monkeypatch, runs):
    """MSIM_MAX_WIDE_MINERS (4 096) miners: W1's runs per workgroup come from the runtime occupancy (or an
    A/B override); every choice the library can make launches and gives the oracle's counters."""
    if runs:
        monkeypatch.setenv("MSIM_W1_RUNS", runs)
    rnd = random.Random(4096)
    w = [3000, 2000] + [rnd.randint(0, 3) for _ in range(4094)]
    _vs_oracle(msim, oracle, w, [1000] * len(w), sum(w), 5 * DAY, 32)
