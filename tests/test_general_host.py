"""The product's general engine (miningsimulation_amd/csrc/msim_general.h), built for the host
(tests/native/general_host.cpp, test-only), against the oracle: per-run found and stale counters and the
best-chain height must be identical (bit-exact integer parity).

The general engine serves what the fast engines cannot: selfish miners in networks of more
than 15 miners, more than 4 selfish miners, and runs whose withheld chains outgrow the entity engine's
window (a selfish majority). Its windows fold the common arrived prefix; small windows here force a fold
every few blocks, so the fold is exercised far more often than on the device."""
import ctypes
import random

import numpy as np
import pytest

DAY = 86_400_000
GERR_CAP = 1


@pytest.fixture(scope="module")
def gen(native_tests):
    lib = ctypes.CDLL(native_tests["general_host"])
    lib.gen_run.restype = ctypes.c_uint32
    lib.gen_run.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_int64),
                            ctypes.POINTER(ctypes.c_uint8), ctypes.POINTER(ctypes.c_uint32), ctypes.c_int,
                            ctypes.c_uint64, ctypes.c_int64,
                            ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32),
                            ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32),
                            ctypes.POINTER(ctypes.c_uint32)]

    def run(weights, props, selfish, duration, si, sp, cap, W=100, ids=None):
        m = len(weights)
        f = (ctypes.c_uint32 * m)()
        s = (ctypes.c_uint32 * m)()
        bh = ctypes.c_uint32()
        base = ctypes.c_uint32()
        idp = (ctypes.c_uint32 * m)(*ids) if ids is not None else None
        err = lib.gen_run((ctypes.c_uint64 * m)(*weights), (ctypes.c_int64 * m)(*props),
                          (ctypes.c_uint8 * m)(*[1 if x else 0 for x in selfish]), idp, m, W, duration, si, sp, cap,
                          f, s, ctypes.byref(bh), ctypes.byref(base))
        return err, np.array([[f[k], s[k]] for k in range(m)], dtype=np.int64), bh.value, base.value

    return run


def _rand_weights(m, rng, total=100):
    cuts = sorted(rng.sample(range(1, total), m - 1)) if m > 1 else []
    b = [0] + cuts + [total]
    return [b[i + 1] - b[i] for i in range(m)]


def _check_batch(gen, oracle, weights, props, selfish, duration, n_runs, seed_base, cap, W=100, allow_cap=False,
                 ids=None):
    """Runs 0..n-1 with the SURVEY seed convention (base + 2r, base + 2r + 1) vs the oracle's batch."""
    f, s, _, _ = oracle.run_batch(weights, props, selfish, duration, n_runs, 0, seed_base, threads=8, total_weight=W,
                                  ids=ids)
    folded = checked = 0
    for r in range(n_runs):
        si, sp = (seed_base + 2 * r) & 0xFFFFFFFF, (seed_base + 2 * r + 1) & 0xFFFFFFFF
        err, res, bh, base = gen(weights, props, selfish, duration, si, sp, cap, W, ids)
        if err == GERR_CAP and allow_cap:
            continue
        assert err == 0, (err, weights, props, selfish, duration, r)
        exp = np.stack([f[r], s[r]], axis=1)
        assert np.array_equal(exp, res), (weights, props, selfish, duration, r, exp.tolist(), res.tolist())
        if ids is None:
            assert bh == int(f[r].sum()), (bh, int(f[r].sum()))
        folded += base > 0
        checked += 1
    return folded, checked


@pytest.mark.parametrize("seed", range(6))
def test_random_networks_any_selfish(gen, oracle, seed):
    """1-15 miners, any number of selfish miners at any index, uniform or mixed delays (0 ms - 30 s)."""
    rng = random.Random(7100 + seed)
    folded = checked = 0
    for _ in range(12):
        m = rng.randint(1, 15)
        w = _rand_weights(m, rng)
        props = [rng.choice([0, 1, 100, 1000, 5000, 30000])] * m if rng.random() < 0.5 else \
            [rng.choice([0, 2, 50, 700, 2000, 12000]) for _ in range(m)]
        selfish = [rng.random() < 0.35 for _ in range(m)]
        # small windows: a run whose selfish miners hold a majority may outgrow one (flagged, never wrong)
        fo, ch = _check_batch(gen, oracle, w, props, selfish, rng.choice([DAY, 7 * DAY, 30 * DAY]), 4,
                              rng.randrange(1 << 32), cap=rng.choice([48, 64, 256]), allow_cap=True)
        folded += fo
        checked += ch
    assert folded > 8 and checked >= 24, (folded, checked)  # most runs checked, and the windows did fold


def test_selfish_majority_two_miners(gen, oracle):
    """Two selfish miners holding 70 % between them (the entity engine's window can overflow here)."""
    _check_batch(gen, oracle, [35, 35, 20, 10], [1000] * 4, [True, True, False, False], 30 * DAY, 6, 4242,
                 cap=4096)


def test_selfish_single_majority(gen, oracle):
    """One selfish miner with 60 %: its lead grows for the whole run, so the window must hold it."""
    _check_batch(gen, oracle, [60, 25, 15], [100, 100, 100], [True, False, False], 30 * DAY, 4, 99, cap=8192)
    # a window too small for that lead is flagged, never wrong
    err, _, _, _ = gen([60, 25, 15], [100] * 3, [True, False, False], 30 * DAY, 99, 100, 64)
    assert err == GERR_CAP


def test_many_selfish(gen, oracle):
    """Six selfish miners (the entity engine serves at most four)."""
    _check_batch(gen, oracle, [10] * 6 + [20, 20], [1000] * 8, [True] * 6 + [False] * 2, 30 * DAY, 6, 7, cap=512)


def test_large_network_one_selfish(gen, oracle):
    """100 miners (integer weights summing to W = 1000) with one selfish miner at 30 %."""
    rng = random.Random(5)
    w = [300] + _rand_weights(99, rng, 700)
    props = [1000] * 100
    selfish = [True] + [False] * 99
    _check_batch(gen, oracle, w, props, selfish, 7 * DAY, 3, 1000, cap=256, W=1000)


def test_zero_duration_and_zero_delay(gen, oracle):
    _check_batch(gen, oracle, [50, 30, 20], [0, 0, 0], [False, True, False], 0, 2, 3, cap=64)
    _check_batch(gen, oracle, [50, 30, 20], [0, 0, 0], [False, True, False], 10 * DAY, 3, 3, cap=64)
    _check_batch(gen, oracle, [100], [0], [True], 3 * DAY, 2, 11, cap=4096)


def test_shared_ids(gen, oracle):
    """Miners sharing an id share their blocks' identity (simulation.h:35-38), each other's stale counting
    (simulation.h:133) and found counts (main.cpp:24-26): the reference's values, not a rejection."""
    # two honest miners with id 3 and one selfish miner sharing id 3 with them; equal delays make equal
    # (id, arrival) blocks of different miners possible, and short windows force folds
    for props in ([1000] * 5, [0] * 5, [100, 100, 2000, 2000, 100]):
        _check_batch(gen, oracle, [30, 25, 20, 15, 10], props, [False] * 5, 30 * DAY, 6, 31, cap=64,
                     ids=[3, 3, 7, 3, 9])
        _check_batch(gen, oracle, [30, 25, 20, 15, 10], props, [True, False, False, False, False], 30 * DAY, 6, 77,
                     cap=4096, ids=[3, 3, 7, 3, 9])
    # every miner with one id
    _check_batch(gen, oracle, [40, 35, 25], [500] * 3, [False, True, False], 10 * DAY, 4, 5, cap=128, ids=[1, 1, 1])


def test_genesis_id(gen, oracle):
    """A miner whose id is UINT_MAX is Genesis's namesake (simulation.h:31-33): MinerStats counts Genesis
    among its blocks (main.cpp:24-26)."""
    U = 0xFFFFFFFF
    for ids in ([U, 1, 2, 3], [0, U, 2, U], [U, U, U, U]):
        _check_batch(gen, oracle, [40, 30, 20, 10], [1000] * 4, [False] * 4, 7 * DAY, 4, 123, cap=64, ids=ids)
        _check_batch(gen, oracle, [40, 30, 20, 10], [1000] * 4, [True, False, False, False], 7 * DAY, 4, 9, cap=4096,
                     ids=ids)
    # zero-duration run: the best chain is Genesis alone; the UINT_MAX miner has found one block
    f, _, _, _ = oracle.run_batch([50, 50], [0, 0], [False, False], 0, 1, 0, 1, ids=[U, 0])
    assert f[0].tolist() == [1, 0]
    _check_batch(gen, oracle, [50, 50], [0, 0], [False, False], 0, 2, 1, cap=64, ids=[U, 0])


def test_single_miner_zero_delay_fold(gen, oracle):
    """One miner, zero delay, tiny window: folds take blocks that arrived after the previous event's best
    chain was recorded (the window-relative best_chain_size goes below zero); ADVICE r3."""
    _check_batch(gen, oracle, [100], [0], [False], 10 * DAY, 4, 17, cap=16)
    # a lone selfish miner never publishes (its lead never drops), so nothing folds: the window holds the run
    _check_batch(gen, oracle, [100], [0], [True], 10 * DAY, 4, 17, cap=4096)


def test_selfish_strategy_kats_on_general_engine(native_tests):
    """The reference's only asserting test, test.cpp:213-367 TestSelfishStrategy, replayed on the PRODUCT's
    general engine (msim_general.h: FoundBlock, MaybeSelfishReveal, MaybeReorg on explicit chains), not only on
    the oracle: every case's resulting chain equals the reference's expected chain."""
    import json
    import os

    lib = ctypes.CDLL(native_tests["general_host"])
    u32p, i64p = ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_int64)
    lib.gen_kat.restype = ctypes.c_uint32
    lib.gen_kat.argtypes = [ctypes.c_uint32, ctypes.c_int64, ctypes.c_int, ctypes.c_int64, ctypes.c_uint32, u32p, i64p,
                            ctypes.c_uint32, u32p, i64p, ctypes.c_uint32, u32p, i64p, ctypes.c_uint32]
    doc = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "selfish_strategy_kats.json")))
    W = (1 << 63) - 1

    def chain(c):
        return [(0xFFFFFFFF, 0) if b == "G" else (b[0], W if b[1] == "W" else b[1]) for b in c]

    def arrays(c):
        n = max(len(c), 1)
        return (ctypes.c_uint32 * n)(*[b[0] for b in c]), (ctypes.c_int64 * n)(*[b[1] for b in c]), len(c)

    sm = doc["selfish_miner"]
    for case in doc["cases"]:
        own, arr, n = arrays(chain(case["chain"]))
        op = case["op"]
        if op[0] == "found":
            code, t, bcs, best = 0, op[1], op[2], []
        else:
            code, t, bcs, best = 1, op[2], 0, chain(op[1])
        bown, barr, bn = arrays(best)
        oo, oa = (ctypes.c_uint32 * 4096)(), (ctypes.c_int64 * 4096)()
        m = lib.gen_kat(sm["id"], sm["propagation_ms"], code, t, bcs, own, arr, n, bown, barr, bn, oo, oa, 4096)
        assert [(oo[i], oa[i]) for i in range(m)] == chain(case["expect"]), case["name"]
