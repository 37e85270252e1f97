"""The entity-engine path on the GPU (E1: the settled form msim_selm.h with in-lane draws and engine phases of
msim_sel.h -> E2 retries -> G), through the C ABI, against the oracle and the reference's own published
results.

Bit-exact per-run counters where the oracle can follow; at BASELINE sizes, size-independent properties
(sum of found = best height, no failed run, E1 == E2) and the reference's README results (README.md:56-63,
98-99), which pin whole selfish runs of the reference itself, within their Monte-Carlo error."""
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

D = 31_556_952_000


@pytest.fixture(scope="module")
def msim(msim_lib_path):
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    torch.cuda.set_device(0)
    import miningsimulation_amd as m

    return m


def _run(msim, p, q, s, n, begin=0, seed=1000, duration=D, W=100):
    miners = [msim.Miner(k, p[k], q[k], bool(s[k])) for k in range(len(p))]
    sim = msim.Simulation(miners, duration, total_weight=W)
    assert sim.pipeline_info(n)["uses_pipeline"] == 3  # E1 (its segment-parallel form is opt-in: test_gpu_selseg.py)
    return sim.run(n, begin, seed, 0, per_run=True)


def _rand_weights(m, rng, total=100):
    cuts = sorted(rng.sample(range(1, total), m - 1)) if m > 1 else []
    b = [0] + cuts + [total]
    return [b[i + 1] - b[i] for i in range(m)]


def test_gpu_two_to_four_selfish_vs_oracle(msim, oracle):
    """Several selfish miners (simulation.h:55 is per miner), heterogeneous delays, 64 runs each."""
    rng = random.Random(91)
    done = 0
    while done < 10:
        m = rng.randint(3, 12)
        p = _rand_weights(m, rng)
        ns = rng.randint(2, min(4, m - 1))
        sidx = set(rng.sample(range(m), ns))
        if sum(p[k] for k in sidx) > 45:  # keep clear of three-branch majority networks (flagged, not served)
            continue
        s = [k in sidx for k in range(m)]
        q = [rng.choice([0, 100, 1000, 10_000]) for _ in range(m)]
        dur = rng.choice([10**9, 10**10, D])
        seed = rng.randrange(2**32)
        res = _run(msim, p, q, s, 64, 0, seed, dur)
        f, st, _, _ = oracle.run_batch(p, q, s, dur, 64, 0, seed, threads=16)
        assert np.array_equal(res.found.astype(np.int64), f), (p, q, s, dur, seed)
        assert np.array_equal(res.stale.astype(np.int64), st), (p, q, s, dur, seed)
        done += 1


def test_gpu_weighted_selfish_vs_oracle(msim, oracle):
    """A selfish miner in networks with integer weights summing to W != 100."""
    rng = random.Random(17)
    for _ in range(6):
        m = rng.randint(3, 10)
        W = rng.choice([1000, 102_400, 2**20 + 3])
        p = _rand_weights(m, rng, W)
        sidx = rng.randrange(m)
        s = [k == sidx for k in range(m)]
        q = [rng.choice([100, 1000, 10_000])] * m
        seed = rng.randrange(2**31)
        res = _run(msim, p, q, s, 64, 0, seed, 10**10, W)
        f, st, _, _ = oracle.run_batch(p, q, s, 10**10, 64, 0, seed, threads=16, total_weight=W)
        assert np.array_equal(res.found.astype(np.int64), f), (p, W)
        assert np.array_equal(res.stale.astype(np.int64), st), (p, W)


@pytest.mark.parametrize("h,prop", [(40, 1000), (49, 30_000), (10, 100), (25, 10_000)])
def test_gpu_engine_equals_retry_kernel(msim, monkeypatch, h, prop):
    """E1 (in-lane fast draws, the settled form's four-find steps, fast engine capacities) and E2 (exact draws
    recomputed from the seeds, wide capacities) are two device paths through the engine: 2048 runs, identical
    per-run counters."""
    miners = msim.setup_miners(prop, selfish_perc=h)
    a = msim.Simulation(miners).run(2048, 31_000, 1000, 0, per_run=True)
    monkeypatch.setenv("MSIM_SEL_FORCE_RETRY", "1")
    b = msim.Simulation(miners).run(2048, 31_000, 1000, 0, per_run=True)
    assert np.array_equal(a.found, b.found)
    assert np.array_equal(a.stale, b.stale)
    assert np.array_equal(a.best_height, b.best_height)
    for x, y in zip(a.sums, b.sums):
        assert bytes(x) == bytes(y)


def _mc_close(per_run, ref_pct, n_ref):
    """|mean - ref| within 4.5 combined standard errors of ours and the reference's own sample."""
    x = np.asarray(per_run, dtype=np.float64) * 100.0
    se = x.std() * np.sqrt(1.0 / x.size + 1.0 / n_ref)
    return abs(x.mean() - ref_pct) <= 4.5 * se, x.mean(), se


def test_gpu_readme_selfish_pin(msim):
    """BASELINE configs[2] (40% selfish, gamma = 0; the README's propagation is the code default 1 s,
    SURVEY §6) at its per-GPU size, 131 072 runs: the reference's published result README.md:98-99
    (32 768 runs): miner 0 46.6844% of blocks / 27.4658% stale, miner 1 16.8889% / 67.4269%."""
    miners = msim.PRESETS["c3"]()
    n = 131_072
    res = msim.Simulation(miners).run(n, 0, 1000, 0, per_run=True)
    bh = res.best_height.astype(np.float64)
    assert np.array_equal(res.found.sum(axis=1), res.best_height)
    f = res.found.astype(np.float64)
    st = res.stale.astype(np.float64)
    share = f / bh[:, None]
    rate = np.where(f > 0, st / np.maximum(f, 1), 0.0)
    for k, sh_ref, rt_ref in ((0, 46.6844, 27.4658), (1, 16.8889, 67.4269)):
        ok, mean, se = _mc_close(share[:, k], sh_ref, 32768)
        assert ok, f"miner {k} share {mean:.4f}% vs README {sh_ref}% (se {se:.4f})"
        ok, mean, se = _mc_close(rate[:, k], rt_ref, 32768)
        assert ok, f"miner {k} stale {mean:.4f}% vs README {rt_ref}% (se {se:.4f})"
    # the reference's report divides the run-order f64 sums by SIM_RUNS (main.cpp:230-231)
    assert abs(res.stats_total[0].blocks_share * 100 / n - share[:, 0].mean() * 100) < 1e-9


def test_gpu_readme_honest_pin(msim):
    """configs[0]'s network (10 s propagation), 32 768 runs: README.md:56-63 (miner 0 30.0901% / 1.0092%,
    miner 7 0.993098% / 1.99286%). Runs on the event-skipping pipeline."""
    miners = msim.PRESETS["c1"]()
    n = 32_768
    res = msim.Simulation(miners).run(n, 0, 1000, 0, per_run=True)
    bh = res.best_height.astype(np.float64)
    f = res.found.astype(np.float64)
    share = f / bh[:, None]
    rate = np.where(f > 0, res.stale / np.maximum(f, 1), 0.0)
    for k, sh_ref, rt_ref in ((0, 30.0901, 1.0092), (7, 0.993098, 1.99286)):
        ok, mean, se = _mc_close(share[:, k], sh_ref, 32768)
        assert ok, f"miner {k} share {mean:.5f}% vs README {sh_ref}% (se {se:.5f})"
        ok, mean, se = _mc_close(rate[:, k], rt_ref, 32768)
        assert ok, f"miner {k} stale {mean:.5f}% vs README {rt_ref}% (se {se:.5f})"


def test_gpu_full_sweep_one_launch(msim, oracle):
    """The whole 360-point configs[3] grid in ONE sweep launch (256 runs per point): per-point invariants
    for every point (no failed run, sum of found = best height per run, shares sum to 1 per run), and 24
    sampled points against the oracle run by run."""
    grid = msim.c4_grid()
    n = 256
    sw = msim.Sweep(grid)
    out = sw.run(n, 0, 1000, 0, per_run=True)
    assert len(out) == 360
    for res in out:
        assert np.array_equal(res.found.sum(axis=1), res.best_height)
        tot = sum(s.blocks_share for s in res.stats_total)
        assert abs(tot - n) < 1e-6
    rng = random.Random(3)
    for i in rng.sample(range(360), 24):
        miners = grid[i]
        p = [m.perc for m in miners]
        q = [m.propagation_ms for m in miners]
        s = [m.is_selfish for m in miners]
        f, st, _, _ = oracle.run_batch(p, q, s, D, 32, 0, 1000, threads=16)
        assert np.array_equal(out[i].found[:32].astype(np.int64), f), (p[0], q[0])
        assert np.array_equal(out[i].stale[:32].astype(np.int64), st), (p[0], q[0])


def test_gpu_c3_status_and_retry_rate(msim):
    """configs[2] through the device-resident launch: status words say how many runs E2 recomputed (the
    fast capacities are sized so that this is rare at 1 s) and that none failed."""
    import torch

    miners = msim.PRESETS["c3"]()
    sim = msim.Simulation(miners)
    n = 32_768
    ws = torch.empty(sim.workspace_bytes(n), dtype=torch.uint8, device="cuda")
    sums = torch.zeros((9, 6), dtype=torch.int64, device="cuda")
    st = torch.zeros(2, dtype=torch.int32, device="cuda")
    sim.launch(n, 0, 1000, sums, ws, st)
    torch.cuda.synchronize()
    retried, failed = st.cpu().tolist()
    assert failed == 0
    assert retried < n * 0.05, retried
    one = sim.run(n, 0, 1000, 0)
    assert sums.cpu().numpy().tolist() == [[s.blocks_found, s.stale_blocks, s.share_hi, s.share_lo, s.rate_hi,
                                            s.rate_lo] for s in one.sums]


@pytest.mark.parametrize("xth,no_macro", [(1, False), (64, False), (16, True)])
def test_gpu_schedule_does_not_change_results(msim, monkeypatch, xth, no_macro):
    """The mixed schedule only decides which lanes of a wave advance together (msim_sel_kernels.hip): any
    engine-phase threshold, and the entity engine alone (no settled form), give the same per-run counters
    as the default schedule on configs[2] (4 096 runs, a full year)."""
    p, q, s = [40, 19, 12, 11, 8, 5, 3, 1, 1], [1000] * 9, [1] + [0] * 8
    base = _run(msim, p, q, s, 4096, begin=77)
    monkeypatch.setenv("MSIM_SEL_XTH", str(xth))
    if no_macro:
        monkeypatch.setenv("MSIM_SEL_NO_MACRO", "1")
    other = _run(msim, p, q, s, 4096, begin=77)
    assert np.array_equal(base.found, other.found) and np.array_equal(base.stale, other.stale)
    assert np.array_equal(base.best_height, other.best_height)


def test_gpu_selfish_eleven_miners_mixed_schedule(msim, oracle):
    """An 11-miner network with one selfish miner (E1's mixed schedule at another miner count): vs the oracle."""
    p = [30, 14, 12, 11, 8, 5, 5, 5, 4, 3, 3]
    q = [1000] * 11
    s = [1] + [0] * 10
    res = _run(msim, p, q, s, 512, begin=0)
    f, st, _, _ = oracle.run_batch(p, q, s, D, 512, 0, 1000, threads=16)
    assert np.array_equal(res.found.astype(np.int64), f)
    assert np.array_equal(res.stale.astype(np.int64), st)
