"""The product's entity engine (miningsimulation_amd/csrc/msim_sel.h), built for the host
(tests/native/sel_host.cpp, test-only), against the oracle: per-run found and stale counters and the
best-chain height must be identical (bit-exact integer parity).

Covers what the device's selfish path runs (BASELINE configs[2], configs[3]) and what the reference allows
beyond it: several selfish miners (simulation.h:55 is a per-miner flag), selfish miners at any index,
heterogeneous propagation, integer weights, honest networks, and the capacity error
paths. tests/test_gpu_selfish.py checks the gfx950 build of the same header against the same oracle."""
import ctypes
import random

import numpy as np
import pytest

D = 31_556_952_000


@pytest.fixture(scope="module")
def sel(native_tests):
    lib = ctypes.CDLL(native_tests["sel_host"])
    lib.sel_set_fold_every.argtypes = [ctypes.c_uint32]
    lib.sel_set_fold_every(0)
    run_fold = lib.sel_set_fold_every
    lib.sel_run.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_int64),
                            ctypes.POINTER(ctypes.c_uint8), ctypes.c_int, ctypes.c_uint64, ctypes.c_int64,
                            ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int, ctypes.POINTER(ctypes.c_uint32),
                            ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32),
                            ctypes.POINTER(ctypes.c_uint32)]

    def run(weights, props, selfish, duration, si, sp, caps=0, W=100):
        m = len(weights)
        f = (ctypes.c_uint32 * m)()
        s = (ctypes.c_uint32 * m)()
        bh = ctypes.c_uint32()
        err = ctypes.c_uint32()
        rc = lib.sel_run((ctypes.c_uint64 * m)(*weights), (ctypes.c_int64 * m)(*props),
                         (ctypes.c_uint8 * m)(*[1 if x else 0 for x in selfish]), m, W, duration, si, sp, caps, f, s,
                         ctypes.byref(bh), ctypes.byref(err))
        assert rc == 0
        return err.value, np.array([[f[k], s[k]] for k in range(m)], dtype=np.int64), bh.value

    run.fold_every = run_fold
    return run


def _rand_percs(m, rng, total=100):
    cuts = sorted(rng.sample(range(1, total), m - 1)) if m > 1 else []
    b = [0] + cuts + [total]
    return [b[i + 1] - b[i] for i in range(m)]


def _oracle(oracle, weights, props, selfish, duration, si, sp, W=100):
    if W == 100:
        rc, res, bh = oracle.run(weights, props, selfish, duration, si, sp)
        assert rc == 0
        return res, bh
    # weighted networks: one run through the batch API (run r = 0 uses seeds (base, base + 1))
    assert sp == si + 1
    f, s, _, _ = oracle.run_batch(weights, props, selfish, duration, 1, 0, si, threads=1, total_weight=W)
    return np.stack([f[0], s[0]], axis=1), int(f[0].sum())


def _check(sel, oracle, weights, props, selfish, duration, si, sp, caps=0, W=100, allow_err=False):
    ores, obh = _oracle(oracle, weights, props, selfish, duration, si, sp, W)
    err, mres, mbh = sel(weights, props, selfish, duration, si, sp, caps, W)
    if allow_err and err:
        return err
    assert err == 0, f"capacity error {err} for {weights} {props} {selfish} {duration} {si} {sp}"
    assert np.array_equal(ores, mres), (weights, props, selfish, duration, si, sp, ores.tolist(), mres.tolist())
    if W == 100:
        assert obh == mbh, (obh, mbh)
    return 0


@pytest.mark.parametrize("seed", range(8))
def test_random_networks(sel, oracle, seed):
    rng = random.Random(4321 + seed)
    for _ in range(40):
        m = rng.randint(1, 15)
        percs = _rand_percs(m, rng)
        if rng.random() < 0.3:
            props = [rng.choice([0, 1, 50, 100, 1000, 10_000, 30_000, 60_000]) for _ in range(m)]
        else:
            props = [rng.choice([100, 1000, 10_000, 30_000])] * m
        s = rng.randrange(m) if (m > 1 and rng.random() < 0.6) else -1
        selfish = [k == s for k in range(m)]
        duration = rng.choice([10**7, 10**8, 10**9])
        _check(sel, oracle, percs, props, selfish, duration, rng.randrange(2**32), rng.randrange(2**32), caps=1)


@pytest.mark.parametrize("seed", range(4))
def test_multiple_selfish(sel, oracle, seed):
    """Two to four selfish miners in one network (the reference's is_selfish is per miner). Every run is
    bit-exact or flagged; only networks whose selfish miners hold most of the hashrate (three long branches
    at once) may exceed the two deep branches of the window."""
    rng = random.Random(777 + seed)
    flagged = 0
    for _ in range(25):
        m = rng.randint(2, 12)
        percs = _rand_percs(m, rng)
        ns = rng.randint(2, min(4, m))
        sidx = set(rng.sample(range(m), ns))
        selfish = [k in sidx for k in range(m)]
        if rng.random() < 0.5:
            props = [rng.choice([0, 100, 1000, 10_000, 30_000]) for _ in range(m)]
        else:
            props = [rng.choice([100, 1000, 10_000])] * m
        duration = rng.choice([10**8, 10**9, 3 * 10**9])
        majority = sum(p for p, s in zip(percs, selfish) if s) > 50
        if _check(sel, oracle, percs, props, selfish, duration, rng.randrange(2**32), rng.randrange(2**32), caps=1,
                  allow_err=majority):
            flagged += 1
    assert flagged <= 3


@pytest.mark.parametrize("h,prop", [(40, 1000), (49, 30_000), (45, 10_000), (25, 100), (10, 30_000), (49, 100),
                                    (30, 5000)])
def test_selfish_full_year(sel, oracle, h, prop):
    """configs[2] and corners of the configs[3] grid, full year, with the fast kernel's capacities:
    anything they cannot hold must be flagged (never wrong), and the retry capacities must be exact."""
    percs = [h, 59 - h, 12, 11, 8, 5, 3, 1, 1]
    for r in range(2):
        si, sp = 1000 + 2 * r, 1001 + 2 * r
        if _check(sel, oracle, percs, [prop] * 9, [True] + [False] * 8, D, si, sp, caps=0, allow_err=True):
            _check(sel, oracle, percs, [prop] * 9, [True] + [False] * 8, D, si, sp, caps=1)


@pytest.mark.parametrize("prop", [100, 10_000])
def test_honest_full_year_presets(sel, oracle, prop):
    for r in range(2):
        _check(sel, oracle, [30, 29, 12, 11, 8, 5, 3, 1, 1], [prop] * 9, [False] * 9, D, 1000 + 2 * r, 1001 + 2 * r,
               caps=1)


def test_fast_capacities_flag_or_match(sel, oracle):
    """With no cold slots and one hot slot of everything, every run is either bit-exact or flagged."""
    rng = random.Random(5)
    flagged = 0
    for _ in range(60):
        m = rng.randint(2, 9)
        percs = _rand_percs(m, rng)
        props = [rng.choice([1000, 30_000, 120_000])] * m
        s = rng.randrange(m)
        selfish = [k == s for k in range(m)]
        flagged += bool(_check(sel, oracle, percs, props, selfish, 10**9, rng.randrange(2**32), rng.randrange(2**32),
                               caps=4, allow_err=True))
    assert flagged > 0  # the tiny capacities must actually be exceeded somewhere


@pytest.mark.parametrize("seed", range(4))
def test_cold_slots(sel, oracle, seed):
    """One hot active slot with a one-entry queue: extra active miners and deep queues live in the cold
    slots constantly (migration, cold finds, cold reorgs, cold folds), and every run stays bit-exact."""
    rng = random.Random(600 + seed)
    for _ in range(25):
        m = rng.randint(3, 12)
        percs = _rand_percs(m, rng)
        props = [rng.choice([1000, 10_000, 30_000, 60_000])] * m if rng.random() < 0.6 else \
            [rng.choice([0, 100, 1000, 10_000, 30_000]) for _ in range(m)]
        s = rng.randrange(m) if rng.random() < 0.8 else -1
        selfish = [k == s for k in range(m)]
        _check(sel, oracle, percs, props, selfish, rng.choice([10**9, 5 * 10**9]), rng.randrange(2**32),
               rng.randrange(2**32), caps=2)


def test_huge_delays(sel, oracle):
    rng = random.Random(99)
    for _ in range(15):
        m = rng.randint(2, 9)
        percs = _rand_percs(m, rng)
        props = [rng.choice([60_000, 120_000, 300_000]) for _ in range(m)]
        s = rng.randrange(m) if rng.random() < 0.5 else -1
        selfish = [k == s for k in range(m)]
        _check(sel, oracle, percs, props, selfish, 10**9, rng.randrange(2**32), rng.randrange(2**32), caps=1,
               allow_err=True)


def test_weighted_networks(sel, oracle):
    """Integer weights summing to W != 100, with selfish miners."""
    rng = random.Random(31)
    for _ in range(12):
        m = rng.randint(2, 10)
        W = rng.choice([17, 1000, 102_400, 2**20 + 3])
        w = _rand_percs(m, rng, W)
        s = rng.randrange(m)
        selfish = [k == s for k in range(m)]
        props = [rng.choice([100, 1000, 10_000])] * m
        si = rng.randrange(2**31)
        _check(sel, oracle, w, props, selfish, 10**9, si, si + 1, caps=1, W=W)


def test_edge_cases(sel, oracle):
    # one miner, zero propagation, zero/one-ms durations, a 0% miner, selfish first/last, all-selfish
    _check(sel, oracle, [100], [0], [False], 10**9, 5, 6)
    _check(sel, oracle, [100], [500], [True], 10**9, 5, 6)
    _check(sel, oracle, [50, 50], [0, 0], [False, False], 10**9, 7, 8)
    _check(sel, oracle, [60, 40], [0, 0], [True, False], 10**9, 7, 8)
    _check(sel, oracle, [40, 60], [0, 0], [False, True], 10**9, 7, 8)
    _check(sel, oracle, [50, 50], [0, 1000], [True, True], 10**9, 7, 8, caps=1)
    _check(sel, oracle, [30, 0, 70], [1000, 1000, 1000], [False, True, False], 10**9, 9, 10)
    _check(sel, oracle, [30, 29, 12, 11, 8, 5, 3, 1, 1], [1000] * 9, [True] + [False] * 8, 0, 1, 2)
    _check(sel, oracle, [30, 29, 12, 11, 8, 5, 3, 1, 1], [1000] * 9, [True] + [False] * 8, 1, 1, 2)
    _check(sel, oracle, [10, 20, 30, 40], [1000] * 4, [False, False, False, True], 10**9, 11, 12)


@pytest.mark.parametrize("every", [1, 3])
def test_early_folds(sel, oracle, every):
    """The device folds every lane of a wave when any lane is due (msim_sel.h step): folding before a lane
    is due must not change any result. Fold at every event / every third event on top of the due ones."""
    rng = random.Random(2024 + every)
    sel.fold_every(every)
    try:
        for _ in range(30):
            m = rng.randint(2, 12)
            percs = _rand_percs(m, rng)
            props = [rng.choice([100, 1000, 10_000, 30_000])] * m if rng.random() < 0.6 else \
                [rng.choice([0, 100, 1000, 10_000, 30_000]) for _ in range(m)]
            ns = rng.choice([0, 1, 1, 1, 2])
            sidx = set(rng.sample(range(m), min(ns, m - 1)))
            selfish = [k in sidx for k in range(m)]
            caps = rng.choice([0, 2])
            majority = sum(p for p, x in zip(percs, selfish) if x) > 50  # may exceed two deep branches
            _check(sel, oracle, percs, props, selfish, rng.choice([10**9, 5 * 10**9]), rng.randrange(2**32),
                   rng.randrange(2**32), caps=caps, allow_err=caps == 0 or (ns > 1 and majority))
        for h, prop in ((40, 1000), (49, 30_000)):
            _check(sel, oracle, [h, 59 - h, 12, 11, 8, 5, 3, 1, 1], [prop] * 9, [True] + [False] * 8, D, 1000, 1001,
                   caps=1)
    finally:
        sel.fold_every(0)


# ---------------------------------------------------------------- the settled-state form (msim_selm.h)
# caps 10 / 11: the device E1 schedule for one lane — the settled form while it applies, the entity engine
# (device capacities / one hot slot of everything) from a find that needs it until the run is settled again.

def _mix_stats(native_tests):
    lib = ctypes.CDLL(native_tests["sel_host"])
    out = (ctypes.c_uint64 * 3)()
    lib.sel_mix_stats(out)
    return list(out)


@pytest.mark.parametrize("seed", range(6))
def test_mixed_random_networks(sel, oracle, seed):
    """Random networks with one selfish miner at any index, uniform and heterogeneous delays (>= 1 ms, where
    the settled form applies), durations from 0 ms to a month: bit-exact with the oracle."""
    rng = random.Random(8080 + seed)
    for _ in range(30):
        m = rng.randint(1, 12)
        percs = _rand_percs(m, rng)
        s = rng.randrange(m)
        selfish = [k == s for k in range(m)]
        if rng.random() < 0.6:
            props = [rng.choice([1, 2, 100, 1000, 10_000, 30_000, 120_000])] * m
        else:
            props = [rng.choice([1, 5, 1000, 20_000, 60_000]) for _ in range(m)]
        duration = rng.choice([0, 1, 1000, 600_000, 86_400_000, D // 12])
        _check(sel, oracle, percs, props, selfish, duration, rng.randrange(2**32), rng.randrange(2**32),
               caps=rng.choice([10, 11]))


@pytest.mark.parametrize("h,prop", [(40, 1000), (49, 30_000), (49, 1000), (10, 100), (25, 5000), (45, 20_000)])
def test_mixed_full_year(sel, oracle, native_tests, h, prop):
    """configs[2] and corners of the configs[3] grid, a full year each: bit-exact, and the settled form
    carries most finds (the engine runs only around finds whose consequences overlap the next find)."""
    percs = [h, 59 - h, 12, 11, 8, 5, 3, 1, 1]
    _mix_stats(native_tests)
    for r in range(2):
        _check(sel, oracle, percs, [prop] * 9, [True] + [False] * 8, D, 1000 + 2 * r, 1001 + 2 * r, caps=10)
    macro, exact, entries = _mix_stats(native_tests)
    # a settled-form step carries up to four finds (SelMacro::step4), an engine step one event
    assert 4 * macro > 2 * exact and entries > 0


def test_mixed_edge_cases(sel, oracle):
    """Zero-length runs, a lone selfish miner, 0 % miners, the selfish miner last, 1 ms delays (the tightest
    settle condition), and a selfish majority (tie forks of hundreds of blocks)."""
    _check(sel, oracle, [100], [500], [True], 10**9, 5, 6, caps=10)
    _check(sel, oracle, [30, 0, 70], [1000, 1000, 1000], [False, True, False], 10**9, 9, 10, caps=10)
    _check(sel, oracle, [10, 20, 30, 40], [1000] * 4, [False, False, False, True], 10**9, 11, 12, caps=10)
    _check(sel, oracle, [40, 60], [1, 1], [True, False], 10**9, 13, 14, caps=10)
    _check(sel, oracle, [40, 60], [1, 2], [False, True], D, 13, 14, caps=11)
    _check(sel, oracle, [70, 30], [1000, 1000], [True, False], D // 4, 15, 16, caps=10)
    for dur in (0, 1, 2, 599_999, 600_000):
        _check(sel, oracle, [40, 19, 12, 11, 8, 5, 3, 1, 1], [1000] * 9, [True] + [False] * 8, dur, 1, 2, caps=10)


def test_mixed_equals_engine_alone(sel):
    """The schedule only changes which form advances a run: the engine alone (caps 0) and the mixed
    schedule give the same counters on 200 runs of configs[2]."""
    percs, props, selfish = [40, 19, 12, 11, 8, 5, 3, 1, 1], [1000] * 9, [True] + [False] * 8
    for r in range(200):
        a = sel(percs, props, selfish, D // 52, 5000 + 2 * r, 5001 + 2 * r, 0)
        b = sel(percs, props, selfish, D // 52, 5000 + 2 * r, 5001 + 2 * r, 10)
        assert a[0] == 0 and b[0] == 0
        assert np.array_equal(a[1], b[1]) and a[2] == b[2]
