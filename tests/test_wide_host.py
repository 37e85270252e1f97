"""The large-network pipeline (miningsimulation_amd/csrc/msim_wide.h, BASELINE configs[4]) executed on
the host from the SAME lane bodies the gfx950 kernels run (tests/native/wide_host.cpp, test-only), run by
run against the oracle (oracle/msim_oracle.c with the SURVEY Appendix C weight generalisation).

Parity for W != 100 is against the oracle's restatement only ("parity unpinned" by the reference, which
cannot express such networks: integer percentages summing to 100, simulation.h:45, main.cpp:43); for
W = 100 the same engine is pinned to the reference through the oracle's golden vectors."""
import ctypes
import random

import numpy as np
import pytest

YEAR = 31_556_952_000
DAY = 86_400_000
H9 = [30, 29, 12, 11, 8, 5, 3, 1, 1]


def c5_network():
    """W = 102400; pools 30% and 29%; 1024 small miners of weight 41; prop 1 s."""
    w = [30720, 29696] + [41] * 1024
    return w, [1000] * len(w), 102400


@pytest.fixture(scope="module")
def wide(native_tests):
    lib = ctypes.CDLL(native_tests["wide_host"])

    def run(weights, props, W, duration, n, base=1000, begin=0):
        m = len(weights)
        f = (ctypes.c_uint32 * (n * m))()
        s = (ctypes.c_uint32 * (n * m))()
        e = (ctypes.c_uint32 * n)()
        ne = ctypes.c_uint32()
        rc = lib.wide_host_run((ctypes.c_uint64 * m)(*weights), (ctypes.c_int64 * m)(*props), ctypes.c_uint32(m),
                               ctypes.c_uint64(W), ctypes.c_int64(duration), ctypes.c_uint32(base),
                               ctypes.c_uint64(begin), ctypes.c_uint32(n), f, s, e, ctypes.byref(ne))
        assert rc == 0
        return (np.array(f, dtype=np.int64).reshape(n, m), np.array(s, dtype=np.int64).reshape(n, m),
                np.array(e, dtype=np.uint32), ne.value)

    return run


def _check(wide, oracle, weights, props, W, duration, n, base=1000, begin=0):
    f, s, err, neps = wide(weights, props, W, duration, n, base, begin)
    assert (err == 0).all(), err
    of, os_, _, _ = oracle.run_batch(weights, props, [0] * len(weights), duration, n, begin, base, threads=8,
                                     total_weight=W)
    assert np.array_equal(f, of), (np.argwhere(f != of)[:5], props[:3], duration)
    assert np.array_equal(s, os_), (np.argwhere(s != os_)[:5], props[:3], duration)
    return f, s, neps


@pytest.mark.parametrize("prop", [0, 100, 1000, 10_000, 30_000])
def test_default_network_year(wide, oracle, prop):
    """W = 100: the same networks the narrow path runs, through the large-network engine."""
    _, s, neps = _check(wide, oracle, H9, [prop] * 9, 100, YEAR, 8)
    if prop >= 1000:
        assert neps & 0xFFFFFF > 0 and s.sum() > 0


def test_c5_network_month(wide, oracle):
    w, p, W = c5_network()
    f, s, neps = _check(wide, oracle, w, p, W, 30 * DAY, 6)
    assert neps & 0xFFFFFF > 0


def test_c5_network_year(wide, oracle):
    w, p, W = c5_network()
    f, s, _ = _check(wide, oracle, w, p, W, YEAR, 2, begin=77)
    assert s.sum() > 0


@pytest.mark.parametrize("seed", range(6))
def test_random_weighted_networks(wide, oracle, seed):
    """Heterogeneous weights (including zero weights) and propagations, 3..300 miners."""
    rnd = random.Random(seed)
    m = rnd.choice([3, 17, 40, 300])
    w = [rnd.choice([0, 1, 2, 5, 40, 300]) for _ in range(m)]
    w[rnd.randrange(m)] += 500
    W = sum(w)
    props = [rnd.choice([0, 1, 50, 700, 3000, 20_000]) for _ in range(m)]
    _check(wide, oracle, w, props, W, rnd.choice([DAY, 20 * DAY, 90 * DAY]), 6, base=rnd.randrange(1 << 32))


def test_retry_capacities_exercised(wide, oracle):
    """Long propagation (30 s) forks often enough that some episodes outgrow the first pass's capacities
    (WE_FAST blocks / WA_FAST miners) and take the retry instantiation; results stay exact."""
    w = [5] * 20
    _, _, neps = _check(wide, oracle, w, [30_000] * 20, 100, YEAR, 8)
    assert neps >> 24 > 0, "no episode needed the retry capacities"


@pytest.mark.parametrize("duration", [0, 1, 599_999, 600_000, 3 * DAY])
def test_short_durations(wide, oracle, duration):
    w, p, W = c5_network()
    _check(wide, oracle, w, p, W, duration, 16)


def test_weighted_pick_matches_oracle(native_tests, oracle):
    lib = ctypes.CDLL(native_tests["wide_host"])
    for weights, W in (([30720, 29696] + [41] * 1024, 102400), (H9, 100), ([1, 0, 2, 0, 7], 10)):
        seed = 4242
        expect = oracle.picks_w(weights, W, seed, 20000)
        u = np.array(oracle.rng_stream(seed, 20000), dtype=np.uint64)
        # adversarial uniforms: bucket edges and the pick-table boundaries
        mult = 0xFFFFFFFFFFFFFFFF // W
        cum = np.cumsum(weights)
        edges = []
        for c in cum[:50]:
            for d in (-1, 0, 1):
                x = int(c) * mult + d
                if 0 <= x < 1 << 64:
                    edges.append(x)
        edges += [(b << 52) + d for b in range(4096) for d in (-1, 0, 1) if 0 <= (b << 52) + d < (1 << 64)] + [(1 << 64) - 1]
        uu = np.concatenate([u, np.array(edges, dtype=np.uint64)])
        out = (ctypes.c_int32 * len(uu))()
        lib.wide_host_pick((ctypes.c_uint64 * len(weights))(*weights), ctypes.c_uint32(len(weights)), ctypes.c_uint64(W),
                           uu.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), out, ctypes.c_uint64(len(uu)))
        got = np.array(out[:], dtype=np.int64)
        assert list(got[:20000]) == expect
        # reference PickFinder on the edges: first k with cum_k * mult > u
        thr = [int(c) * mult for c in cum]
        for x, g in zip(edges, got[20000:]):
            k = next((i for i, t in enumerate(thr) if t > x), -1)
            assert g == k, (x, g, k)
