"""The selfish pipeline (miningsimulation_amd/csrc/msim_selpipe.h: K1's nibble/candidate draw pass, then the
settled-state transitions from nibbles, the entity engine from stored RNG states, the drawn form at the end)
executed on the host from the same lane bodies (tests/native/selpipe_host.cpp, test-only), against the
oracle run by run: per-run found and stale counters and the best-chain height must be identical.

The reference behaviour is RunSimulation (main.cpp:128-192) with one selfish miner (simulation.h:55,
62-180); BASELINE configs[2] is the README example (README.md:89-107)."""
import ctypes
import random

import numpy as np
import pytest

YEAR = 31_556_952_000
DAY = 86_400_000


@pytest.fixture(scope="module")
def sp(native_tests):
    lib = ctypes.CDLL(native_tests["selpipe_host"])
    u32p = ctypes.POINTER(ctypes.c_uint32)
    lib.selpipe_run.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_int64),
                                ctypes.POINTER(ctypes.c_uint8), ctypes.c_int, ctypes.c_int64, ctypes.c_uint32,
                                ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, u32p, u32p, u32p,
                                u32p]
    lib.selpipe_stats.argtypes = [ctypes.POINTER(ctypes.c_uint64)]

    def run(percs, props, selfish, duration, n, run_begin=0, seed_base=1000, cap=0, slots=64):
        m = len(percs)
        f = np.zeros((n, m), dtype=np.uint32)
        s = np.zeros((n, m), dtype=np.uint32)
        bh = np.zeros(n, dtype=np.uint32)
        err = np.zeros(n, dtype=np.uint32)
        p = lambda a: a.ctypes.data_as(u32p)  # noqa: E731
        rc = lib.selpipe_run((ctypes.c_uint64 * m)(*percs), (ctypes.c_int64 * m)(*props),
                             (ctypes.c_uint8 * m)(*[1 if x else 0 for x in selfish]), m, duration, seed_base,
                             run_begin, n, cap, slots, p(f), p(s), p(bh), p(err))
        assert rc == 0, rc
        st = (ctypes.c_uint64 * 5)()
        lib.selpipe_stats(st)
        return f.astype(np.int64), s.astype(np.int64), bh, err, list(st)

    return run


def _check(sp, oracle, percs, props, selfish, duration, n, run_begin=0, seed_base=1000, cap=0, slots=64,
           max_err=0):
    f, s, bh, err, st = sp(percs, props, selfish, duration, n, run_begin, seed_base, cap, slots)
    of, os_, _, _ = oracle.run_batch(percs, props, selfish, duration, n, run_begin, seed_base, threads=8)
    ok = err == 0
    assert int((~ok).sum()) <= max_err, (int((~ok).sum()), err[~ok][:8])
    assert np.array_equal(f[ok], of[ok]), (percs, props, np.argwhere((f != of).any(axis=1))[:4].ravel())
    assert np.array_equal(s[ok], os_[ok])
    assert np.array_equal(bh[ok].astype(np.int64), of[ok].sum(axis=1))  # every best-chain block has a finder
    return st


def test_configs2_network(sp, oracle):
    """BASELINE configs[2]: the README's 40 % selfish miner at 1 s, a full year, run by run."""
    st = _check(sp, oracle, [40, 19, 12, 11, 8, 5, 3, 1, 1], [1000] * 9, [1] + [0] * 8, YEAR, 24)
    assert st[1] > 0  # engine episodes from candidates ran


def test_end_inside_the_last_window(sp, oracle):
    """Runs whose T_B falls inside [D - prop_k - prop_s, D): the engine finishes them from B. 30 s delays make
    that window 60 s wide (~10 % of runs), 20 days keep the oracle fast."""
    st = _check(sp, oracle, [40, 19, 12, 11, 8, 5, 3, 1, 1], [30000] * 9, [1] + [0] * 8, 20 * DAY, 40, run_begin=5)
    assert st[2] > 0


@pytest.mark.parametrize("h,prop", [(10, 100), (25, 500), (33, 2000), (45, 5000), (49, 250)])
def test_sweep_points(sp, oracle, h, prop):
    """Points of the configs[3] grid (selfish share h, miner 1 = 59 - h, all delays prop), 60 days."""
    percs = [h, 59 - h, 12, 11, 8, 5, 3, 1, 1]
    _check(sp, oracle, percs, [prop] * 9, [1] + [0] * 8, 60 * DAY, 16, run_begin=77)


@pytest.mark.parametrize("seed", range(6))
def test_random_networks(sp, oracle, seed):
    """Random percentages, one selfish miner at any index, heterogeneous delays 1 ms - 20 s, 20-120 days."""
    rng = random.Random(9000 + seed)
    for _ in range(4):
        m = rng.randint(2, 15)
        cuts = sorted(rng.sample(range(1, 100), m - 1))
        b = [0] + cuts + [100]
        percs = [b[i + 1] - b[i] for i in range(m)]
        props = [rng.choice([1, 7, 100, 900, 1000, 3000, 20000]) for _ in range(m)]
        sel = [0] * m
        sel[rng.randrange(m)] = 1
        _check(sp, oracle, percs, props, sel, rng.randint(20, 120) * DAY, 6, run_begin=rng.randrange(10**6))


def test_many_segments_and_short_slices(sp, oracle):
    """Many K1 workers per run (small wave-slot count: long jump chains, several band segments)."""
    _check(sp, oracle, [40, 19, 12, 11, 8, 5, 3, 1, 1], [1000] * 9, [1] + [0] * 8, 90 * DAY, 8, slots=4)


def test_capacity_overflow_is_flagged(sp, oracle):
    """Candidate slots of 1 per segment: runs that outgrow them are flagged (E2 recomputes them), never wrong."""
    f, s, bh, err, _ = sp([40, 19, 12, 11, 8, 5, 3, 1, 1], [1000] * 9, [1] + [0] * 8, 60 * DAY, 8, cap=1)
    assert (err != 0).any()
    _check(sp, oracle, [40, 19, 12, 11, 8, 5, 3, 1, 1], [1000] * 9, [1] + [0] * 8, 60 * DAY, 8, cap=1, max_err=8)
