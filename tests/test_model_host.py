"""The product's compact state machine (miningsimulation_amd/csrc/msim_model.h), built for the host
(tests/native/model_host.cpp, test-only), against the oracle on random networks: per-run found and stale
counters and the best-chain height must be identical (bit-exact integer parity).

This checks the ALGORITHM on CPU-only machines; tests/test_gpu_parity.py checks the gfx950 build of the
same header against the same oracle."""
import ctypes
import random

import numpy as np
import pytest

D = 31_556_952_000


@pytest.fixture(scope="module")
def model(native_tests):
    lib = ctypes.CDLL(native_tests["model_host"])
    lib.model_run.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_int64),
                              ctypes.POINTER(ctypes.c_uint8), ctypes.c_int, ctypes.c_int64, ctypes.c_uint32,
                              ctypes.c_uint32, ctypes.c_int, ctypes.POINTER(ctypes.c_uint32),
                              ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32),
                              ctypes.POINTER(ctypes.c_uint32)]

    def run(percs, props, selfish, duration, si, sp, deep=0):
        m = len(percs)
        f = (ctypes.c_uint32 * m)()
        s = (ctypes.c_uint32 * m)()
        bh = ctypes.c_uint32()
        err = ctypes.c_uint32()
        rc = lib.model_run((ctypes.c_uint64 * m)(*percs), (ctypes.c_int64 * m)(*props),
                           (ctypes.c_uint8 * m)(*[1 if x else 0 for x in selfish]), m, duration, si, sp, deep, f, s,
                           ctypes.byref(bh), ctypes.byref(err))
        assert rc == 0
        return err.value, np.array([[f[k], s[k]] for k in range(m)], dtype=np.int64), bh.value

    return run


def _rand_percs(m, rng):
    cuts = sorted(rng.sample(range(1, 100), m - 1)) if m > 1 else []
    b = [0] + cuts + [100]
    return [b[i + 1] - b[i] for i in range(m)]


def _check(model, oracle, percs, props, selfish, duration, si, sp, deep=0):
    rc, ores, obh = oracle.run(percs, props, selfish, duration, si, sp)
    assert rc == 0
    err, mres, mbh = model(percs, props, selfish, duration, si, sp, deep)
    assert err == 0, f"capacity error {err} for {percs} {props} {selfish}"
    assert np.array_equal(ores, mres), (percs, props, selfish, duration, si, sp)
    assert obh == mbh


@pytest.mark.parametrize("seed", range(6))
def test_random_networks(model, oracle, seed):
    rng = random.Random(1234 + seed)
    for _ in range(40):
        m = rng.randint(1, 15)
        percs = _rand_percs(m, rng)
        if rng.random() < 0.3:
            props = [rng.choice([0, 1, 50, 100, 1000, 10_000, 30_000, 60_000]) for _ in range(m)]
        else:
            props = [rng.choice([100, 1000, 10_000, 30_000])] * m
        s = rng.randrange(m) if (m > 1 and rng.random() < 0.5) else -1
        selfish = [k == s for k in range(m)]
        duration = rng.choice([10**7, 10**8, 10**9])
        _check(model, oracle, percs, props, selfish, duration, rng.randrange(2**32), rng.randrange(2**32))


@pytest.mark.parametrize("h,prop", [(40, 1000), (49, 30_000), (45, 10_000), (25, 100), (10, 30_000)])
def test_selfish_full_year(model, oracle, h, prop):
    """SURVEY Q5's deepest forks: full-year selfish episodes (BASELINE configs[2], configs[3] corners)."""
    percs = [h, 59 - h, 12, 11, 8, 5, 3, 1, 1]
    for r in range(2):
        _check(model, oracle, percs, [prop] * 9, [True] + [False] * 8, D, 1000 + 2 * r, 1001 + 2 * r)


@pytest.mark.parametrize("prop", [100, 10_000])
def test_honest_full_year_presets(model, oracle, prop):
    for r in range(3):
        _check(model, oracle, [30, 29, 12, 11, 8, 5, 3, 1, 1], [prop] * 9, [False] * 9, D, 1000 + 2 * r, 1001 + 2 * r)


def test_deep_branches_honest(model, oracle):
    """The retry kernel's configuration (deep branches enabled) on honest networks with huge delays."""
    rng = random.Random(99)
    for _ in range(20):
        m = rng.randint(2, 9)
        percs = _rand_percs(m, rng)
        props = [rng.choice([60_000, 120_000, 300_000]) for _ in range(m)]
        si, sp = rng.randrange(2**32), rng.randrange(2**32)
        rc, ores, obh = oracle.run(percs, props, [False] * m, 10**9, si, sp)
        err, mres, mbh = model(percs, props, [False] * m, 10**9, si, sp, 1)
        if err == 0:
            assert np.array_equal(ores, mres) and obh == mbh


def test_edge_cases(model, oracle):
    # single miner holding 100%, zero propagation, zero duration, a 0% miner, selfish at the last index
    _check(model, oracle, [100], [0], [False], 10**9, 5, 6)
    _check(model, oracle, [100], [500], [False], 10**9, 5, 6)
    _check(model, oracle, [50, 50], [0, 0], [False, False], 10**9, 7, 8)
    _check(model, oracle, [60, 40], [0, 0], [True, False], 10**9, 7, 8)
    _check(model, oracle, [40, 60], [0, 0], [False, True], 10**9, 7, 8)
    _check(model, oracle, [30, 0, 70], [1000, 1000, 1000], [False, False, False], 10**9, 9, 10)
    _check(model, oracle, [30, 29, 12, 11, 8, 5, 3, 1, 1], [1000] * 9, [False] * 9, 0, 1, 2)
    _check(model, oracle, [30, 29, 12, 11, 8, 5, 3, 1, 1], [1000] * 9, [False] * 9, 1, 1, 2)
    _check(model, oracle, [10, 20, 30, 40], [1000] * 4, [False, False, False, True], 10**9, 11, 12)
