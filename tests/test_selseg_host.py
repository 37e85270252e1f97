"""The segment-parallel selfish path's lane bodies (miningsimulation_amd/csrc/msim_selseg.h: SW workers from the
quiet state per segment, ST stitching the true run through them with the entity engine inline), built for the host
(tests/native/selseg_host.cpp, test-only), against the oracle: per-run found and stale counters and the best-chain
height identical to the reference's loop (RunSimulation, main.cpp:128-192; simulation.h:62-180).

The segment count is a free parameter of the decomposition: one segment (only cuts), the device's few, and many
short segments (every boundary a coalescence walk) must all give the oracle's run. tests/test_gpu_selseg.py checks
the gfx950 build of the same header."""
import ctypes
import random

import numpy as np
import pytest

D = 31_556_952_000


@pytest.fixture(scope="module")
def seg(native_tests):
    lib = ctypes.CDLL(native_tests["selseg_host"])
    lib.selseg_run.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_int64),
                               ctypes.POINTER(ctypes.c_uint8), ctypes.c_int, ctypes.c_uint64, ctypes.c_int64,
                               ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                               ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32),
                               ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32)]
    lib.selseg_stats.argtypes = [ctypes.POINTER(ctypes.c_uint64)]
    lib.selseg_qcap.argtypes = [ctypes.c_uint32]

    def run(weights, props, selfish, duration, si, sp, nseg, cap=1 << 20, W=100):
        m = len(weights)
        mu = duration / 600000.0
        need = int(mu + 8 * max(mu, 1.0) ** 0.5 + 64)
        segb = max(1, (need + nseg - 1) // nseg)
        f = (ctypes.c_uint32 * m)()
        s = (ctypes.c_uint32 * m)()
        bh = ctypes.c_uint32()
        err = ctypes.c_uint32()
        rc = lib.selseg_run((ctypes.c_uint64 * m)(*weights), (ctypes.c_int64 * m)(*props),
                            (ctypes.c_uint8 * m)(*[1 if x else 0 for x in selfish]), m, W, duration, si, sp, nseg, segb,
                            cap, f, s, ctypes.byref(bh), ctypes.byref(err))
        return rc, np.array([[f[k], s[k]] for k in range(m)], dtype=np.int64), bh.value

    def stats():
        out = (ctypes.c_uint64 * 7)()
        lib.selseg_stats(out)
        return dict(zip(("subs", "cuts", "jumps", "walk_steps", "engine_entries", "end_steps", "checkpoints"),
                        list(out)))

    run.stats = stats
    run.qcap = lib.selseg_qcap
    return run


def _check(seg, oracle, w, p, s, duration, si, nseg):
    rc0, ores, obh = oracle.run(w, p, s, duration, si, si + 1)
    assert rc0 == 0
    rc, mres, mbh = seg(w, p, s, duration, si, si + 1, nseg)
    assert rc == 0, (w, p, s, duration, si, nseg, rc)
    assert np.array_equal(ores, mres), (w, p, s, duration, si, nseg, ores.tolist(), mres.tolist())
    assert obh == mbh, (obh, mbh)


@pytest.mark.parametrize("nseg", [1, 5, 24])
def test_configs2_full_year(seg, oracle, nseg):
    """BASELINE configs[2] (40 % selfish, 1 s): full-year runs, one to many segments."""
    w, p, s = [40, 19, 12, 11, 8, 5, 3, 1, 1], [1000] * 9, [1] + [0] * 8
    seg.stats()
    for r in range(3):
        _check(seg, oracle, w, p, s, D, 1000 + 2 * r, nseg)
    st = seg.stats()
    assert st["cuts"] > 100 and st["jumps"] > 100 and st["engine_entries"] > 100, st


@pytest.mark.parametrize("h,prop", [(10, 100), (25, 500), (33, 2000), (49, 250), (45, 5000)])
def test_grid_points_quarter_year(seg, oracle, h, prop):
    """configs[3] grid points (selfish share h, miner 1 = 59 - h), a quarter of a year, several segment counts."""
    w, p, s = [h, 59 - h, 12, 11, 8, 5, 3, 1, 1], [prop] * 9, [1] + [0] * 8
    for nseg in (1, 3, 9):
        _check(seg, oracle, w, p, s, D // 4, 77 + h, nseg)


@pytest.mark.parametrize("seed", range(4))
def test_random_networks(seg, oracle, seed):
    """Random networks: 2-12 miners, the selfish miner at any index, uniform or mixed delays from 1 ms to 30 s,
    durations from zero to a month, 1 / 3 / 7 segments."""
    rng = random.Random(seed)
    for _ in range(12):
        m = rng.randint(2, 12)
        cuts = sorted(rng.sample(range(1, 100), m - 1))
        b = [0] + cuts + [100]
        w = [b[i + 1] - b[i] for i in range(m)]
        sid = rng.randrange(m)
        s = [1 if k == sid else 0 for k in range(m)]
        base = rng.choice([1, 50, 500, 1000, 3000, 10000, 30000])
        p = [base] * m if rng.random() < 0.5 else [max(1, int(base * rng.uniform(0.2, 3))) for _ in range(m)]
        duration = rng.choice([0, 1000, 600000 * 5, 600000 * 300, 86_400_000 * 30])
        si = rng.randrange(1 << 31)
        for nseg in (1, 3, 7):
            _check(seg, oracle, w, p, s, duration, si, nseg)


def test_overflow_is_reported(seg):
    """A segment that outgrows its sub capacity is reported (the device hands the run to E2), never dropped."""
    w, p, s = [40, 19, 12, 11, 8, 5, 3, 1, 1], [30000] * 9, [1] + [0] * 8
    rc, _, _ = seg(w, p, s, D // 12, 5, 6, 2, cap=4)
    assert rc == 1


@pytest.mark.parametrize("qcap", [0 + 1, 7, 40])
def test_checkpoint_room_runs_out(seg, oracle, qcap):
    """Workers whose checkpoint room fills up store no more checkpoints (the device's seg_qcap bound): the stitch
    walks further and the run is still the oracle's."""
    w, p, s = [40, 19, 12, 11, 8, 5, 3, 1, 1], [1000] * 9, [1] + [0] * 8
    seg.qcap(qcap)
    try:
        seg.stats()
        for nseg in (1, 4):
            _check(seg, oracle, w, p, s, D // 6, 31 + qcap, nseg)
        st = seg.stats()
        assert st["checkpoints"] <= 4 * qcap + qcap, st
    finally:
        seg.qcap(0)
