"""The segment-parallel form of E1 on the GPU (msim_selseg.h: SW settled-form workers per (run, segment), ST stitching
each run with the entity engine; opt-in, MSIM_SELSEG=1), through the C ABI: run by run against the oracle, and
against E1 itself (the default) at sizes the oracle cannot follow. The reference behaviour is RunSimulation (main.cpp:128-192) with
one selfish miner (simulation.h:55, 62-180); BASELINE configs[2]. MSIM_SEG_NSEG forces many short segments so that
every segment boundary's coalescence walk runs many times per run."""
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

YEAR = 31_556_952_000
C3 = ([40, 19, 12, 11, 8, 5, 3, 1, 1], [1000] * 9, [1] + [0] * 8)


@pytest.fixture(autouse=True)
def _selseg(monkeypatch):
    monkeypatch.setenv("MSIM_SELSEG", "1")


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


@pytest.mark.parametrize("nseg", [None, "1", "23"])
def test_gpu_selseg_c3_vs_oracle(msim, oracle, monkeypatch, nseg):
    """configs[2]'s network, 512 runs x 1 year on SW + ST, identical to the oracle per run (the device's own segment
    count, one segment, and 23 short ones)."""
    if nseg:
        monkeypatch.setenv("MSIM_SEG_NSEG", nseg)
    sim = _sim(msim, *C3)
    info = sim.pipeline_info(512)
    assert info["uses_pipeline"] == 6, info
    if nseg:
        assert info["segments"] == int(nseg), info
    res = sim.run(512, 0, 1000, 0, per_run=True)
    f, st, _, _ = oracle.run_batch(*C3, YEAR, 512, 0, 1000, threads=16)
    assert np.array_equal(res.found.astype(np.int64), f)
    assert np.array_equal(res.stale.astype(np.int64), st)
    assert np.array_equal(res.best_height.astype(np.int64), f.sum(axis=1))


def test_gpu_selseg_equals_e1(msim, monkeypatch):
    """32 768 configs[2] runs: SW + ST and E1 (the default) agree per run and in the fixed-point sums."""
    a = _sim(msim, *C3).run(32768, 7000, 1000, 0, per_run=True)
    monkeypatch.delenv("MSIM_SELSEG")
    sim = _sim(msim, *C3)
    assert sim.pipeline_info(32768)["uses_pipeline"] == 3
    b = sim.run(32768, 7000, 1000, 0, per_run=True)
    _same(a, b)


@pytest.mark.parametrize("h,prop", [(10, 100), (25, 500), (33, 1000), (49, 250), (45, 1500)])
def test_gpu_selseg_grid_points_vs_e1(msim, monkeypatch, h, prop):
    """Points of the configs[3] grid the segment-parallel form serves (rare cuts), 4 096 runs x 1 year, against E1."""
    p, q, s = [h, 59 - h, 12, 11, 8, 5, 3, 1, 1], [prop] * 9, [1] + [0] * 8
    sim = _sim(msim, p, q, s)
    assert sim.pipeline_info(4096)["uses_pipeline"] == 6
    a = sim.run(4096, 0, 1000, 0, per_run=True)
    monkeypatch.delenv("MSIM_SELSEG")
    b = _sim(msim, p, q, s).run(4096, 0, 1000, 0, per_run=True)
    _same(a, b)


def test_gpu_selseg_random_networks_vs_oracle(msim, oracle):
    """Random one-selfish networks the form serves (2-15 miners, the selfish miner anywhere, mixed delays of
    1 ms - 2 s, 1-12 months): 64 runs each against the oracle."""
    rng = random.Random(66)
    done = 0
    while done < 6:
        m = rng.randint(2, 15)
        cuts = sorted(rng.sample(range(1, 100), m - 1))
        b = [0] + cuts + [100]
        w = [b[i + 1] - b[i] for i in range(m)]
        sid = rng.randrange(m)
        s = [1 if k == sid else 0 for k in range(m)]
        q = [rng.randint(1, 2000) for _ in range(m)]
        duration = YEAR * rng.randint(1, 12) // 12
        sim = _sim(msim, w, q, s, duration)
        if sim.pipeline_info(64)["uses_pipeline"] != 6:
            continue
        res = sim.run(64, 0, 4242, 0, per_run=True)
        f, st, _, _ = oracle.run_batch(w, q, s, duration, 64, 0, 4242, threads=16)
        assert np.array_equal(res.found.astype(np.int64), f), (w, q, s, duration)
        assert np.array_equal(res.stale.astype(np.int64), st), (w, q, s, duration)
        done += 1


def test_gpu_selseg_forced_retry(msim, monkeypatch):
    """Every run flagged by ST (MSIM_SEL_FORCE_RETRY) is recomputed by E2: the same results."""
    a = _sim(msim, *C3).run(2048, 0, 1000, 0, per_run=True)
    monkeypatch.setenv("MSIM_SEL_FORCE_RETRY", "1")
    b = _sim(msim, *C3).run(2048, 0, 1000, 0, per_run=True)
    _same(a, b)
