"""Parity of the gfx950 path (libmsim.so through its C ABI) against the CPU oracle and golden vectors.

Bar: bit-exact per-run integer counters (found, stale, best-chain height) for identical seeds; f64
aggregates from per-run records bit-exact against the oracle's run-order sums (main.cpp:211-217);
fixed-point device sums within 1e-9 relative of those; sizes where the oracle cannot follow are checked
through size-independent invariants."""
import os
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

D = 31_556_952_000
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def msim(msim_lib_path):
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    torch.cuda.set_device(0)
    import miningsimulation_amd as m

    return m


def _sim(msim, percs, props, selfish, duration=D):
    miners = [msim.Miner(k, percs[k], props[k], bool(selfish[k])) for k in range(len(percs))]
    return msim.Simulation(miners, duration)


def test_gpu_log1p_and_intervals(msim, oracle):
    """glibc log1p and NextBlockInterval on the device, bit for bit (xoroshiro128++.h:19, simulation.h:205-210)."""
    import ctypes

    import torch
    from miningsimulation_amd import _lib

    rng = np.random.default_rng(5)
    n = 1 << 22
    u = rng.integers(0, 2**64 - 1, size=n, dtype=np.uint64, endpoint=True)
    # plus both ends of the domain and the branch thresholds of the fdlibm algorithm
    edge = np.concatenate([np.arange(4096, dtype=np.uint64) << np.uint64(11),
                           ((np.uint64(2**53 - 1) - np.arange(4096, dtype=np.uint64)) << np.uint64(11))])
    # and inputs whose 6e11*E + 0.5 lies within +-4 ns of a millisecond boundary: the domain of the
    # draw kernel's exact fallback (msim_fastdraw.h)
    q = rng.integers(1, 22_000_000, size=200_000).astype(np.float64)
    y = q * 1e6 - 0.5 + rng.uniform(-4.0, 4.0, size=q.size)
    m = ((1.0 - np.exp(-y / 6e11)) * 2.0**53).astype(np.uint64)
    near = np.concatenate([m + np.uint64(d) for d in (0, 1, 2)]) << np.uint64(11)
    u = np.concatenate([u, edge, near])
    x = (u >> np.uint64(11)).astype(np.float64) * -(2.0**-53)
    du = torch.from_numpy(u.view(np.int64)).cuda()
    dx = torch.from_numpy(x).cuda()
    dl = torch.empty_like(dx)
    di = torch.empty(u.size, dtype=torch.int64, device="cuda")
    _lib.check(_lib.lib.msim_device_log1p(ctypes.c_void_p(dx.data_ptr()), ctypes.c_void_p(dl.data_ptr()), u.size, None))
    _lib.check(_lib.lib.msim_device_intervals(ctypes.c_void_p(du.data_ptr()), ctypes.c_void_p(di.data_ptr()), u.size, None))
    torch.cuda.synchronize()
    ref_l = oracle.log1p_array(x)
    ref_i = oracle.interval_of_array(u)
    assert np.array_equal(dl.cpu().numpy().view(np.uint64), ref_l.view(np.uint64))
    assert np.array_equal(di.cpu().numpy(), ref_i)


def test_gpu_picks(msim, oracle):
    import ctypes

    import torch
    from miningsimulation_amd import _lib

    percs = [30, 29, 12, 11, 8, 5, 3, 1, 1]
    sim = _sim(msim, percs, [1000] * 9, [0] * 9)
    words = np.array(oracle.rng_stream(7, 4096), dtype=np.uint64)
    du = torch.from_numpy(words.view(np.int64)).cuda()
    dk = torch.empty(words.size, dtype=torch.int32, device="cuda")
    _lib.check(_lib.lib.msim_device_picks(sim.handle, ctypes.c_void_p(du.data_ptr()), ctypes.c_void_p(dk.data_ptr()),
                                          words.size, None))
    torch.cuda.synchronize()
    assert dk.cpu().tolist() == oracle.picks(percs, 7, 4096)


@pytest.mark.parametrize("name", ["c1_prop10s", "c2_prop100ms", "default_prop1s", "c3_selfish40_prop1s",
                                  "c4_selfish49_prop30s", "c4_selfish10_prop100ms"])
def test_gpu_golden_vectors(msim, name):
    """64 full-year runs per configuration, per-run counters identical to tests/golden/oracle_vectors.npz."""
    z = np.load(os.path.join(GOLD, "oracle_vectors.npz"))
    p, q, s = z[name + "_config"].tolist()
    res = _sim(msim, p, q, s).run(64, 0, 1000, 0, per_run=True)
    assert np.array_equal(res.found.astype(np.int64), z[name + "_found"])
    assert np.array_equal(res.stale.astype(np.int64), z[name + "_stale"])
    assert np.array_equal(res.best_height.astype(np.int64), z[name + "_best_height"])


@pytest.mark.parametrize("preset", ["c1", "c2", "c3", "default"])
def test_gpu_presets_vs_oracle(msim, oracle, preset):
    """512 runs of each BASELINE configuration vs the oracle, run by run, plus the f64 aggregate."""
    miners = msim.PRESETS[preset]()
    p = [m.perc for m in miners]
    q = [m.propagation_ms for m in miners]
    s = [m.is_selfish for m in miners]
    n, begin = 512, 4096
    res = _sim(msim, p, q, s).run(n, begin, 1000, 0, per_run=True)
    f, st, sh, r = oracle.run_batch(p, q, s, D, n, begin, 1000, threads=16)
    assert np.array_equal(res.found.astype(np.int64), f)
    assert np.array_equal(res.stale.astype(np.int64), st)
    for k in range(len(p)):
        # exact run-order sums (main.cpp:211-217)
        ref_share = 0.0
        ref_rate = 0.0
        for i in range(n):
            ref_share += sh[i, k]
            ref_rate += r[i, k]
        assert res.stats_total[k].blocks_found == int(f[:, k].sum())
        assert res.stats_total[k].blocks_share == ref_share
        assert res.stats_total[k].stale_rate == ref_rate
        # fixed-point device sums
        fx = msim.sums_to_stats([[res.sums[k].blocks_found, res.sums[k].stale_blocks, res.sums[k].share_hi,
                                  res.sums[k].share_lo, res.sums[k].rate_hi, res.sums[k].rate_lo]])[0]
        assert abs(fx.blocks_share - ref_share) <= 1e-9 * max(1.0, ref_share)
        assert abs(fx.stale_rate - ref_rate) <= 1e-9 * max(1.0, ref_rate) + n * 2.0**-32


def test_gpu_random_networks(msim, oracle):
    """Random networks (1-15 miners, mixed delays incl. 0 ms, honest or one selfish), 64 runs each."""
    rng = random.Random(2024)
    for _ in range(24):
        m = rng.randint(1, 15)
        cuts = sorted(rng.sample(range(1, 100), m - 1)) if m > 1 else []
        b = [0] + cuts + [100]
        p = [b[i + 1] - b[i] for i in range(m)]
        q = [rng.choice([0, 1, 100, 1000, 10_000, 30_000]) for _ in range(m)]
        sidx = rng.randrange(m) if (m > 1 and rng.random() < 0.5) else -1
        s = [k == sidx for k in range(m)]
        dur = rng.choice([10**8, 10**9, 10**10])
        seed = rng.randrange(2**32)
        res = _sim(msim, p, q, s, dur).run(64, 0, seed, 0, per_run=True)
        f, st, _, _ = oracle.run_batch(p, q, s, dur, 64, 0, seed, threads=16)
        assert np.array_equal(res.found.astype(np.int64), f), (p, q, s, dur, seed)
        assert np.array_equal(res.stale.astype(np.int64), st), (p, q, s, dur, seed)


def test_gpu_c4_grid_sample(msim, oracle):
    """A sample of the 360-point sweep (BASELINE configs[3]) at full length, 32 runs per point."""
    rng = random.Random(7)
    grid = msim.c4_grid()
    for miners in rng.sample(grid, 10):
        p = [m.perc for m in miners]
        q = [m.propagation_ms for m in miners]
        s = [m.is_selfish for m in miners]
        res = _sim(msim, p, q, s).run(32, 0, 1000, 0, per_run=True)
        f, st, _, _ = oracle.run_batch(p, q, s, D, 32, 0, 1000, threads=16)
        assert np.array_equal(res.found.astype(np.int64), f), (p, q)
        assert np.array_equal(res.stale.astype(np.int64), st), (p, q)


def test_gpu_sweep_vs_oracle(msim, oracle):
    """One sweep launch over 12 grid points (BASELINE configs[3]) against the oracle run by run: every
    point sees the seeds of runs [run_begin, run_begin + n), like msim_run(cfg_p, run_begin, n)."""
    rng = random.Random(11)
    pts = rng.sample(msim.c4_grid(), 12)
    n, begin = 48, 5000
    out = msim.Sweep(pts).run(n, begin, 1000, 0, per_run=True)
    for miners, res in zip(pts, out):
        p = [m.perc for m in miners]
        q = [m.propagation_ms for m in miners]
        s = [m.is_selfish for m in miners]
        f, st, _, _ = oracle.run_batch(p, q, s, D, n, begin, 1000, threads=16)
        assert np.array_equal(res.found.astype(np.int64), f), (p, q)
        assert np.array_equal(res.stale.astype(np.int64), st), (p, q)
        assert np.array_equal(res.found.sum(axis=1), res.best_height)


def test_gpu_sweep_equals_single_runs(msim):
    """Mixed sweep (honest networks through the selfish instantiation, runs per point not a multiple of
    the workgroup) == msim_run per point: same fixed-point sums, same per-run counters. For the honest
    points msim_run takes the event-skipping pipeline, so this also cross-checks two device paths."""
    pts = [msim.setup_miners(1000, selfish_perc=25), msim.setup_miners(100), msim.setup_miners(30000, selfish_perc=45),
           msim.setup_miners(10000)]
    n = 1000
    out = msim.Sweep(pts).run(n, 123, 1000, 0, per_run=True)
    for miners, res in zip(pts, out):
        one = msim.Simulation(miners).run(n, 123, 1000, 0, per_run=True)
        assert np.array_equal(res.found, one.found)
        assert np.array_equal(res.stale, one.stale)
        assert np.array_equal(res.best_height, one.best_height)
        no_rec = msim.Simulation(miners).run(n, 123, 1000, 0)
        for a, b in zip(res.sums, no_rec.sums):
            assert bytes(a) == bytes(b)


def test_gpu_retry_path_huge_delays(msim, oracle):
    """Delays of minutes overflow the fast kernel's in-flight capacity; the retry kernel must take those
    runs and still match the oracle."""
    p = [30, 29, 12, 11, 8, 5, 3, 1, 1]
    q = [300_000] * 9
    s = [False] * 9
    res = _sim(msim, p, q, s, 10**10).run(128, 0, 1000, 0, per_run=True)
    f, st, _, _ = oracle.run_batch(p, q, s, 10**10, 128, 0, 1000, threads=16)
    assert np.array_equal(res.found.astype(np.int64), f)
    assert np.array_equal(res.stale.astype(np.int64), st)


def test_gpu_sharding_is_exact(msim):
    """Integer sums are partition-independent: [0,N) == [0,N/2) + [N/2,N), bit for bit (what makes the
    1/2/4/8-GPU all-reduce results identical)."""
    sim = _sim(msim, [40, 19, 12, 11, 8, 5, 3, 1, 1], [1000] * 9, [1] + [0] * 8)
    n = 8192
    whole = sim.run(n, 0, 1000, 0)
    a = sim.run(n // 2, 0, 1000, 0)
    b = sim.run(n // 2, n // 2, 1000, 0)
    for k in range(9):
        for fld in ("blocks_found", "stale_blocks", "share_hi", "share_lo", "rate_hi", "rate_lo"):
            assert getattr(whole.sums[k], fld) == getattr(a.sums[k], fld) + getattr(b.sums[k], fld)


@pytest.mark.parametrize("preset", ["c1", "c2"])
def test_gpu_pipeline_equals_per_lane_kernel(msim, preset, monkeypatch):
    """The event-skipping pipeline (honest networks) and the per-lane kernel are two independent device
    implementations of RunSimulation: 4096 runs, per-run counters must be identical."""
    miners = msim.PRESETS[preset]()
    fast = msim.Simulation(miners).run(4096, 77_000, 1000, 0, per_run=True)
    monkeypatch.setenv("MSIM_NO_PIPELINE", "1")
    slow = msim.Simulation(miners).run(4096, 77_000, 1000, 0, per_run=True)
    assert np.array_equal(fast.found, slow.found)
    assert np.array_equal(fast.stale, slow.stale)
    assert np.array_equal(fast.best_height, slow.best_height)


def test_gpu_invariants_full_scale(msim):
    """BASELINE configs[1] at full size (32768 runs x 365 d, one launch): no failed run; per-run
    sum of found = best height (the genesis block has no owner, main.cpp:27-28); the aggregate matches
    README.md:72,80 within Monte-Carlo error."""
    miners = msim.PRESETS["c2"]()
    res = msim.Simulation(miners).run(32768, 0, 1000, 0, per_run=True)
    assert np.array_equal(res.found.sum(axis=1).astype(np.int64), res.best_height.astype(np.int64))
    n = 32768
    share0 = res.stats_total[0].blocks_share * 100 / n
    rate0 = res.stats_total[0].stale_rate * 100 / n
    assert abs(share0 - 30.0008) < 0.02
    assert abs(rate0 - 0.0101929) < 0.0015


def test_host_dropin_driver(msim):
    """host/msim_main (the C++ drop-in for main.cpp) prints main.cpp:224-234's report; its numbers equal
    the Python host path's fixed-point sums for the same runs."""
    import subprocess

    exe = os.path.join(os.path.dirname(GOLD), "..", "host", "msim_main")
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", os.path.join(os.path.dirname(GOLD), "..", "host")], check=True)
    # split on "\n" only: the progress line starts with "\r" like the reference's (main.cpp:219)
    # (bytes, then decode: text mode's universal newlines would turn that "\r" into "\n")
    raw = subprocess.run([exe, "1", "1000"], capture_output=True, check=True).stdout
    out = raw.decode().rstrip("\n").split("\n")
    assert out[0] == "Running 32768 simulations in parallel using 1 threads."  # main.cpp:201's format
    assert out[1] == "\r100% progress.."
    assert out[2] == "After running 32768 simulations for 365d each, on average:"
    miners = msim.setup_miners(1000)
    res = msim.Simulation(miners).run(32768, 0, 1000, 0)
    rows = [[s.blocks_found, s.stale_blocks, s.share_hi, s.share_lo, s.rate_hi, s.rate_lo] for s in res.sums]
    want = msim.report(miners, msim.sums_to_stats(rows), 32768).splitlines()
    assert out[2:] == want


def test_host_dropin_driver_large_network(msim):
    """host/msim_main c5: BASELINE configs[4] through the C++ drop-in (msim_config_create_weighted)."""
    import subprocess

    exe = os.path.join(os.path.dirname(GOLD), "..", "host", "msim_main")
    raw = subprocess.run([exe, "1", "1000", "c5"], capture_output=True, check=True).stdout
    out = raw.decode().rstrip("\n").split("\n")
    assert out[2] == "After running 32768 simulations for 365d each, on average:"
    assert len(out) == 3 + 1026
    assert out[3].startswith("  - Miner 0 (30% of network hashrate) found ")
    assert out[5].startswith("  - Miner 2 (0.0400391% of network hashrate) found ")


def test_host_dropin_driver_sweep(msim, tmp_path):
    """host/msim_main's sweep surface: a 3-point JSON network list (one sweep launch, msim_sweep_run_multi)
    printed as JSON lines, and a 3-point --grid printed as main.cpp:224-234 reports, both equal to the
    Python Sweep path's fixed-point sums for the same runs."""
    import json
    import subprocess

    exe = os.path.join(os.path.dirname(GOLD), "..", "host", "msim_main")
    pts = [msim.setup_miners(1000, selfish_perc=40), msim.setup_miners(10_000, selfish_perc=25),
           msim.setup_miners(100)]
    spec = {"runs": 1024, "seed_base": 1000,
            "points": [{"miners": [{"id": m.id, "perc": m.perc, "propagation_ms": m.propagation_ms,
                                    "selfish": m.is_selfish} for m in p]} for p in pts]}
    f = tmp_path / "sweep.json"
    f.write_text(json.dumps(spec))
    raw = subprocess.run([exe, "--sweep", str(f), "--json"], capture_output=True, check=True).stdout.decode()
    lines = [json.loads(x) for x in raw.strip().split("\n")]
    assert len(lines) == 3
    want = msim.Sweep(pts).run(1024, 0, 1000, 0)
    for p, (line, res) in enumerate(zip(lines, want)):
        assert line["point"] == p and line["runs"] == 1024
        for m, w in zip(line["miners"], res.stats_total):
            assert m["blocks_share"] == w.blocks_share / 1024
            assert m["stale_rate"] == w.stale_rate / 1024
            assert m["blocks_found"] == w.blocks_found / 1024
    # the grid form: selfish share x propagation over SetupMiners, text reports
    raw = subprocess.run([exe, "--grid", "10,45:1000", "--runs", "512"], capture_output=True, check=True).stdout
    out = raw.decode().rstrip("\n").split("\n")
    grid = [msim.setup_miners(1000, selfish_perc=10), msim.setup_miners(1000, selfish_perc=45)]
    res = msim.Sweep(grid).run(512, 0, 1000, 0)
    want = []
    for p, (g, r) in enumerate(zip(grid, res)):
        want.append(f"Point {p + 1} of 2:")
        rows = [[s.blocks_found, s.stale_blocks, s.share_hi, s.share_lo, s.rate_hi, s.rate_lo] for s in r.sums]
        want += msim.report(g, msim.sums_to_stats(rows), 512).splitlines()
    assert out == want


@pytest.mark.parametrize("preset", ["c2", "c3"])
def test_gpu_overlapped_streams_equal_serial(msim, preset):
    """bench.py overlaps consecutive steps on two HIP streams (each with its own workspace): launches in
    flight together give exactly the sums of the same launches run one after the other."""
    import torch

    sim = msim.Simulation(msim.PRESETS[preset]())
    m = len(sim.miners)
    n = 8192
    dev = torch.device("cuda", 0)
    lanes = [(torch.cuda.Stream(dev), torch.empty(sim.workspace_bytes(n), dtype=torch.uint8, device=dev),
              torch.zeros((m, 6), dtype=torch.int64, device=dev), torch.zeros(2, dtype=torch.int32, device=dev),
              torch.zeros((m, 6), dtype=torch.int64, device=dev)) for _ in range(2)]
    torch.cuda.synchronize()
    for i in range(4):  # steps i and i+1 are in flight together
        st, ws, sums, status, acc = lanes[i % 2]
        with torch.cuda.stream(st):
            sim.launch(n, i * n, 1000, sums, ws, status, stream=st)
            acc.add_(sums)  # ordered on st after its own launch
    torch.cuda.synchronize()
    got = lanes[0][4] + lanes[1][4]
    assert int(lanes[0][3][1]) == 0 and int(lanes[1][3][1]) == 0
    want = torch.zeros((m, 6), dtype=torch.int64, device=dev)
    ws = torch.empty(sim.workspace_bytes(n), dtype=torch.uint8, device=dev)
    sums = torch.zeros((m, 6), dtype=torch.int64, device=dev)
    status = torch.zeros(2, dtype=torch.int32, device=dev)
    for i in range(4):
        sim.launch(n, i * n, 1000, sums, ws, status)
        want.add_(sums)
        assert int(status[1]) == 0
    torch.cuda.synchronize()
    assert torch.equal(got, want)


@pytest.mark.parametrize("preset", ["c1", "c2"])
def test_gpu_dirty_workspace_equals_clean(msim, preset):
    """A launch must not depend on what its workspace held before (the driver's torch.empty buffers are
    reused across launches). K1 reserves episode-list slots a wave chunk at a time and marks the unused tail
    of every chunk; with c1's 10 s delays a chunk is 256 slots, longer than a wave, so the whole tail must be
    marked. Filled with 0xFF bytes, the workspace's unmarked slots would send K2 to run and
    segment indices far out of range."""
    import torch

    sim = msim.Simulation(msim.PRESETS[preset]())
    m = len(sim.miners)
    n = 8192
    dev = torch.device("cuda", 0)
    out = []
    for fill in (0x00, 0xFF, 0x00):
        ws = torch.full((sim.workspace_bytes(n),), fill, dtype=torch.uint8, device=dev)
        sums = torch.zeros((m, 6), dtype=torch.int64, device=dev)
        status = torch.zeros(2, dtype=torch.int32, device=dev)
        rec = torch.zeros((n, m, 2), dtype=torch.int32, device=dev)
        bh = torch.zeros(n, dtype=torch.int32, device=dev)
        sim.launch(n, 0, 1000, sums, ws, status, d_per_run=rec, d_best_height=bh)
        torch.cuda.synchronize()
        assert int(status[1]) == 0
        out.append((sums.cpu(), rec.cpu(), bh.cpu()))
        del ws
    for a, b in zip(out[0], out[1]):
        assert torch.equal(a, b)
    for a, b in zip(out[0], out[2]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("preset", ["c1", "c2"])
def test_gpu_concurrent_launch_plans_agree(msim, preset):
    """msim_config_set_concurrent_launches only re-plans K1's grid (three rounds of shorter segments for one launch
    in flight, one round for two): every run's counters and the sums are the same for 1, 2 and 4."""
    import torch

    n = 8192
    dev = torch.device("cuda", 0)
    out = []
    for jobs in (1, 2, 4):
        sim = msim.Simulation(msim.PRESETS[preset]())
        sim.set_concurrent_launches(jobs)
        m = len(sim.miners)
        ws = torch.empty((sim.workspace_bytes(n),), dtype=torch.uint8, device=dev)
        sums = torch.zeros((m, 6), dtype=torch.int64, device=dev)
        status = torch.zeros(2, dtype=torch.int32, device=dev)
        rec = torch.zeros((n, m, 2), dtype=torch.int32, device=dev)
        bh = torch.zeros(n, dtype=torch.int32, device=dev)
        sim.launch(n, 4096, 1000, sums, ws, status, d_per_run=rec, d_best_height=bh)
        torch.cuda.synchronize()
        assert int(status[1]) == 0
        out.append((sim.pipeline_info(n)["segments"], sums.cpu(), rec.cpu(), bh.cpu()))
        del ws
    assert out[0][0] > out[1][0], [o[0] for o in out]  # one launch in flight: more, shorter segments
    for o in out[1:]:
        for a, b in zip(out[0][1:], o[1:]):
            assert torch.equal(a, b)
