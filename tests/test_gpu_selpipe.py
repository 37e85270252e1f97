"""The selfish pipeline on the GPU (msim_selpipe.h: K1<NIB> draws every block, stores its finder nibble and
lists the candidates; S2 applies the settled-state transitions from the nibbles, the entity engine from the
candidates' stored RNG states), through the C ABI: run by run against the oracle, and against E1 (the entity
engine with in-lane draws, MSIM_NO_SELPIPE) at sizes the oracle cannot follow. The reference behaviour is
RunSimulation (main.cpp:128-192) with one selfish miner (simulation.h:55, 62-180); BASELINE configs[2]."""
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

YEAR = 31_556_952_000
DAY = 86_400_000
C3 = ([40, 19, 12, 11, 8, 5, 3, 1, 1], [1000] * 9, [1] + [0] * 8)


@pytest.fixture(autouse=True)
def _selpipe_on(monkeypatch):
    """The selfish pipeline is opt-in (msim_api.hip: E1 serves configs[2] by default)."""
    monkeypatch.setenv("MSIM_SELPIPE", "1")


@pytest.fixture(scope="module")
def msim(msim_lib_path):
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    torch.cuda.set_device(0)
    import miningsimulation_amd as m

    return m


def _sim(msim, p, q, s, duration=YEAR):
    return msim.Simulation([msim.Miner(k, p[k], q[k], bool(s[k])) for k in range(len(p))], duration)


def _same(a, b):
    assert np.array_equal(a.found, b.found)
    assert np.array_equal(a.stale, b.stale)
    assert np.array_equal(a.best_height, b.best_height)
    for x, y in zip(a.sums, b.sums):
        assert bytes(x) == bytes(y)


def test_gpu_selpipe_c3_vs_oracle(msim, oracle):
    """configs[2]'s network, 512 runs x 1 year on the selfish pipeline, identical to the oracle per run."""
    sim = _sim(msim, *C3)
    info = sim.pipeline_info(512)
    assert info["uses_pipeline"] == 5, info
    res = sim.run(512, 0, 1000, 0, per_run=True)
    f, st, _, _ = oracle.run_batch(*C3, YEAR, 512, 0, 1000, threads=16)
    assert np.array_equal(res.found.astype(np.int64), f)
    assert np.array_equal(res.stale.astype(np.int64), st)
    assert np.array_equal(res.best_height.astype(np.int64), f.sum(axis=1))


def test_gpu_selpipe_equals_e1(msim, monkeypatch):
    """16 384 configs[2] runs: the selfish pipeline and E1 (MSIM_NO_SELPIPE) agree per run and in the sums."""
    a = _sim(msim, *C3).run(16384, 5000, 1000, 0, per_run=True)
    monkeypatch.setenv("MSIM_NO_SELPIPE", "1")
    sim = _sim(msim, *C3)
    assert sim.pipeline_info(16384)["uses_pipeline"] == 3
    b = sim.run(16384, 5000, 1000, 0, per_run=True)
    _same(a, b)


@pytest.mark.parametrize("h,prop", [(10, 100), (25, 500), (33, 2000), (45, 5000), (49, 250)])
def test_gpu_selpipe_grid_points_vs_e1(msim, monkeypatch, h, prop):
    """Points of the configs[3] grid (selfish share h, miner 1 = 59 - h, every delay prop), 4 096 runs x 1 year."""
    p, q, s = [h, 59 - h, 12, 11, 8, 5, 3, 1, 1], [prop] * 9, [1] + [0] * 8
    sim = _sim(msim, p, q, s)
    assert sim.pipeline_info(4096)["uses_pipeline"] == 5
    a = sim.run(4096, 0, 1000, 0, per_run=True)
    monkeypatch.setenv("MSIM_NO_SELPIPE", "1")
    b = _sim(msim, p, q, s).run(4096, 0, 1000, 0, per_run=True)
    _same(a, b)


def test_gpu_selpipe_random_networks_vs_oracle(msim, oracle):
    """One selfish miner at any index, 2-15 miners, heterogeneous delays 1 ms - 20 s, 20-365 days, 96 runs."""
    rng = random.Random(2025)
    done = 0
    while done < 10:
        m = rng.randint(2, 15)
        cuts = sorted(rng.sample(range(1, 100), m - 1))
        b = [0] + cuts + [100]
        p = [b[i + 1] - b[i] for i in range(m)]
        q = [rng.choice([1, 7, 100, 900, 1000, 3000, 20000]) for _ in range(m)]
        s = [0] * m
        s[rng.randrange(m)] = 1
        dur = rng.randint(20, 365) * DAY
        sim = _sim(msim, p, q, s, dur)
        if sim.pipeline_info(96)["uses_pipeline"] != 5:
            continue
        seed = rng.randrange(2**32)
        res = sim.run(96, 0, seed, 0, per_run=True)
        f, st, _, _ = oracle.run_batch(p, q, s, dur, 96, 0, seed, threads=16)
        assert np.array_equal(res.found.astype(np.int64), f), (p, q, s, dur, seed)
        assert np.array_equal(res.stale.astype(np.int64), st), (p, q, s, dur, seed)
        done += 1


def test_gpu_selpipe_status_at_full_size(msim):
    """configs[2] at its per-GPU size (131 072 runs): no failed run, few runs recomputed by E2, and the
    size-independent invariant sum(found) = best height per run."""
    import torch

    sim = _sim(msim, *C3)
    n = 131_072
    ws = torch.empty(sim.workspace_bytes(n), dtype=torch.uint8, device="cuda")
    sums = torch.zeros((9, 6), dtype=torch.int64, device="cuda")
    st = torch.zeros(2, dtype=torch.int32, device="cuda")
    sim.launch(n, 0, 1000, sums, ws, st)
    torch.cuda.synchronize()
    retried, failed = st.cpu().tolist()
    assert failed == 0
    assert retried < n * 0.001, retried
    res = sim.run(8192, 0, 1000, 0, per_run=True)
    assert np.array_equal(res.found.sum(axis=1), res.best_height)
