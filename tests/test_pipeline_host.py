"""The event-skipping pipeline (miningsimulation_amd/csrc/msim_pipeline.h) executed on the host from the
SAME lane bodies the gfx950 kernels run (tests/native/pipeline_host.cpp, test-only), against the oracle.

It checks the decomposition itself — jump-ahead states vs sequential stepping, fast/slow blocks, episodes
from quiet states, the end-of-run search and the last-block correction — bit-exactly on CPU-only hosts;
tests/test_gpu_parity.py checks the device build of the same code against the same oracle."""
import ctypes
import random

import numpy as np
import pytest

D = 31_556_952_000
H = [30, 29, 12, 11, 8, 5, 3, 1, 1]


@pytest.fixture(scope="module")
def pipe(native_tests):
    lib = ctypes.CDLL(native_tests["pipeline_host"])

    def run(percs, props, duration, n, base=1000, begin=0, cap=0, slots=8192):
        m = len(percs)
        f = (ctypes.c_uint32 * (n * m))()
        s = (ctypes.c_uint32 * (n * m))()
        ok = (ctypes.c_uint8 * n)()
        ne = ctypes.c_uint32()
        rc = lib.pipeline_run((ctypes.c_uint64 * m)(*percs), (ctypes.c_int64 * m)(*props), (ctypes.c_uint8 * m)(),
                              m, ctypes.c_int64(duration), ctypes.c_uint32(base), ctypes.c_uint64(begin),
                              ctypes.c_uint32(n), ctypes.c_uint32(cap), ctypes.c_uint32(slots), f, s, ok, ctypes.byref(ne))
        assert rc == 0, f"pipeline_run rc={rc} (-100: jump-ahead state differs from sequential stepping)"
        return (np.array(f, dtype=np.int64).reshape(n, m), np.array(s, dtype=np.int64).reshape(n, m),
                np.array(ok, dtype=bool), ne.value)

    return run


def _check(pipe, oracle, percs, props, duration, n, base=1000, begin=0, cap=0, need_all_ok=True, slots=8192):
    f, s, ok, ne = pipe(percs, props, duration, n, base, begin, cap, slots)
    of, os_, _, _ = oracle.run_batch(percs, props, [0] * len(percs), duration, n, begin, base, threads=8)
    if need_all_ok:
        assert ok.all(), f"{(~ok).sum()} runs flagged for retry"
    assert np.array_equal(f[ok], of[ok]), (percs, props, duration)
    assert np.array_equal(s[ok], os_[ok]), (percs, props, duration)
    return ok, ne


@pytest.mark.parametrize("prop", [0, 1, 100, 1000, 10_000, 30_000])
def test_presets_full_year(pipe, oracle, prop):
    _check(pipe, oracle, H, [prop] * 9, D, 12)


@pytest.mark.parametrize("slots", [1, 64, 5000, 10**6])
def test_worker_geometries(pipe, oracle, slots):
    """Segment lengths from one worker per run (no jump) to the shortest allowed workers."""
    _check(pipe, oracle, H, [1000] * 9, D, 8, slots=slots)


def _rand_percs(m, rng):
    cuts = sorted(rng.sample(range(1, 100), m - 1)) if m > 1 else []
    b = [0] + cuts + [100]
    return [b[i + 1] - b[i] for i in range(m)]


@pytest.mark.parametrize("seed", range(4))
def test_random_networks(pipe, oracle, seed):
    """Heterogeneous propagation (incl. 0 ms), zero-percent miners, 1..15 miners, random run ranges."""
    rng = random.Random(77 + seed)
    for _ in range(6):
        m = rng.randint(1, 15)
        percs = _rand_percs(m, rng)
        if m > 2 and rng.random() < 0.3:
            percs[rng.randrange(m)] += percs[0]
            percs[0] = 0
        props = [rng.choice([0, 1, 7, 250, 2000, 12_000, 45_000]) for _ in range(m)]
        dur = rng.choice([D, D // 3, 86_400_000 * 30])
        _check(pipe, oracle, percs, props, dur, 4, base=rng.randrange(2**32), begin=rng.randrange(10**9))


@pytest.mark.parametrize("dur", [0, 1, 599_999, 600_000, 3_600_000, 25_000_000, 250_000_000])
def test_short_durations(pipe, oracle, dur):
    """Runs that end before the first block, inside the first segment, or after a handful of blocks."""
    _check(pipe, oracle, H, [10_000] * 9, dur, 64)


def test_capacity_overflow_is_flagged(pipe, oracle):
    """With one slot per segment, runs with more slow blocks must be flagged, never mis-counted."""
    ok, _ = _check(pipe, oracle, H, [10_000] * 9, D, 8, cap=1, need_all_ok=False)
    assert not ok.all()
