"""Host-side mirror of the reference's configuration and driver surface, over libmsim's C ABI.

Reference surface (/root/reference/main.cpp):
  SIM_DURATION  main.cpp:7    months{12} = 31 556 952 000 ms
  SIM_RUNS      main.cpp:10   16 * 2048
  SetupMiners   main.cpp:44-65
  MinerStats    main.cpp:13-41 (blocks_found, blocks_share, stale_rate; operator+=)
  main          main.cpp:195-235 (batch driver + report)
and Miner(id, perc, propagation, selfish=false) from simulation.h:57-59.

Simulation.run() is the GPU replacement for main()'s std::async loop; report() prints main.cpp:224-234's
lines so outputs can be diffed against the reference's stdout.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import Iterable, List, Optional, Sequence

import numpy as np

from . import _lib
from ._lib import MsimMiner, MsimRunRecord, MsimStats, MsimSums, MsimTiming, check, lib

SIM_DURATION_MS = 31_556_952_000  # main.cpp:7 std::chrono::months{12}
SIM_RUNS = 16 * 2048              # main.cpp:10
BLOCK_INTERVAL_MS = 600_000       # simulation.h:16
DEFAULT_SEED_BASE = 1000          # SURVEY §8d seed convention


@dataclass(frozen=True)
class Miner:
    """Miner(unsigned id, uint64_t perc, milliseconds prop, bool selfish) — simulation.h:57-59."""

    id: int
    perc: int
    propagation_ms: int
    is_selfish: bool = False


def setup_miners(propagation_ms: int = 1000, selfish_perc: Optional[int] = None) -> List[Miner]:
    """SetupMiners() (main.cpp:44-65): the 2025 hashrate approximation, homogeneous propagation.

    With ``selfish_perc`` = h, miner 0 is selfish with h% and miner 1 gets 59-h% (README.md:85-107 uses
    h = 40; SURVEY §8d C4 sweeps h over 10..49)."""
    percs = [30, 29, 12, 11, 8, 5, 3, 1, 1]
    selfish = False
    if selfish_perc is not None:
        percs[0], percs[1] = selfish_perc, 59 - selfish_perc
        selfish = True
    return [Miner(k, p, propagation_ms, selfish and k == 0) for k, p in enumerate(percs)]


# BASELINE.json configs: C1 plumbing, C2 single-GPU bench, C3 selfish 40%.
PRESETS = {
    "c1": lambda: setup_miners(10_000),
    "c2": lambda: setup_miners(100),
    "c3": lambda: setup_miners(1_000, selfish_perc=40),
    "default": lambda: setup_miners(1_000),
}
C5_TOTAL_WEIGHT = 102_400


def c5_network(propagation_ms: int = 1000) -> List[Miner]:
    """BASELINE.json configs[4]: 2 pools + 1024 small miners, integer weights summing to
    W = 102400 (pool 0 30%, pool 1 29%, 1024 x 41 = 41%), all honest. Not expressible in the reference
    (integer percentages summing to 100, main.cpp:43); run with Simulation(..., total_weight=C5_TOTAL_WEIGHT)."""
    w = [30720, 29696] + [41] * 1024
    return [Miner(k, x, propagation_ms) for k, x in enumerate(w)]


PRESET_WEIGHTS = {"c5": C5_TOTAL_WEIGHT}
PRESETS["c5"] = c5_network
C4_SELFISH_PERCS = list(range(10, 50))
C4_PROPAGATIONS_MS = [100, 250, 500, 1000, 2000, 5000, 10000, 20000, 30000]


def c4_grid() -> List[List[Miner]]:
    """The 360-point sweep of BASELINE.json configs[3]: h in 10..49 x propagation 0.1..30 s."""
    return [setup_miners(p, selfish_perc=h) for h in C4_SELFISH_PERCS for p in C4_PROPAGATIONS_MS]


@dataclass
class MinerStats:
    """MinerStats (main.cpp:13-41)."""

    blocks_found: int = 0
    blocks_share: float = 0.0
    stale_rate: float = 0.0

    def __iadd__(self, other: "MinerStats") -> "MinerStats":  # main.cpp:34-40
        self.blocks_found += other.blocks_found
        self.blocks_share += other.blocks_share
        self.stale_rate += other.stale_rate
        return self


@dataclass
class SimulationResult:
    stats_total: List[MinerStats]              # like main.cpp:199 stats_total (sums over runs)
    sums: List[MsimSums]                        # fixed-point device sums
    found: Optional[np.ndarray] = None          # [n_runs, M] uint32, per-run blocks_found
    stale: Optional[np.ndarray] = None          # [n_runs, M] uint32, per-run stale_blocks
    best_height: Optional[np.ndarray] = None    # [n_runs] uint32, |best chain| - 1
    n_runs: int = 0
    extra: dict = field(default_factory=dict)


def _miners_struct(miners: Sequence[Miner]):
    arr = (MsimMiner * len(miners))()
    for i, m in enumerate(miners):
        arr[i] = MsimMiner(m.id, m.perc, m.propagation_ms, 1 if m.is_selfish else 0)
    return arr


class Simulation:
    """A network description bound to the device library (msim_config)."""

    def __init__(self, miners: Sequence[Miner], duration_ms: int = SIM_DURATION_MS, total_weight: int = 100):
        """total_weight = 100: Miner.perc are the reference's integer percentages (SetupMiners, main.cpp:43).
        Otherwise Miner.perc are integer weights summing to total_weight."""
        self.miners = list(miners)
        self.duration_ms = int(duration_ms)
        self.total_weight = int(total_weight)
        handle = ctypes.c_void_p()
        if self.total_weight == 100:
            check(lib.msim_config_create(_miners_struct(self.miners), len(self.miners), self.duration_ms,
                                         ctypes.byref(handle)), "msim_config_create")
        else:
            check(lib.msim_config_create_weighted(_miners_struct(self.miners), len(self.miners), self.duration_ms,
                                                  self.total_weight, ctypes.byref(handle)), "msim_config_create_weighted")
        self._h = handle

    @property
    def wide(self) -> bool:
        """True when the network runs on the large-network pipeline (msim_wide.h)."""
        return bool(lib.msim_config_is_wide(self._h))

    @property
    def handle(self) -> ctypes.c_void_p:
        return self._h

    def set_concurrent_launches(self, n: int) -> None:
        """msim_config_set_concurrent_launches: how many launches of this config the caller keeps in flight
        (e.g. steps alternating over n HIP streams). A grid-planning hint, no effect on results; it changes
        workspace_bytes, so call it before sizing the workspace."""
        check(lib.msim_config_set_concurrent_launches(self._h, int(n)), "msim_config_set_concurrent_launches")

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            lib.msim_config_destroy(h)
            self._h = None

    def run(self, n_runs: int, run_begin: int = 0, seed_base: int = DEFAULT_SEED_BASE, device: int = 0,
            per_run: bool = False) -> SimulationResult:
        m = len(self.miners)
        stats = (MsimStats * m)()
        sums = (MsimSums * m)()
        rec = (MsimRunRecord * (n_runs * m))() if per_run else None
        bh = (ctypes.c_uint32 * n_runs)() if per_run else None
        check(lib.msim_run(self._h, run_begin, n_runs, seed_base & 0xFFFFFFFF, device, stats, sums, rec, bh), "msim_run")
        res = SimulationResult(
            stats_total=[MinerStats(s.blocks_found, s.blocks_share, s.stale_rate) for s in stats],
            sums=list(sums),
            n_runs=n_runs,
        )
        if per_run:
            a = np.ctypeslib.as_array(ctypes.cast(rec, ctypes.POINTER(ctypes.c_uint32)), shape=(n_runs, m, 2)).copy()
            res.found = a[:, :, 0]
            res.stale = a[:, :, 1]
            res.best_height = np.ctypeslib.as_array(bh).copy()
        return res

    def run_multi(self, n_runs: int, run_begin: int = 0, seed_base: int = DEFAULT_SEED_BASE,
                  devices: Sequence[int] = (0,)) -> SimulationResult:
        """msim_run_multi: the runs sharded over `devices` (one host thread each) and combined with one RCCL
        all-reduce of the integer sums; bit-identical to run() for any device list."""
        m = len(self.miners)
        stats = (MsimStats * m)()
        sums = (MsimSums * m)()
        devs = (ctypes.c_int * len(devices))(*devices)
        shard_ms = (ctypes.c_double * (2 * len(devices)))()
        check(lib.msim_run_multi_timed(self._h, run_begin, n_runs, seed_base & 0xFFFFFFFF, devs, len(devices), stats,
                                       sums, shard_ms), "msim_run_multi_timed")
        return SimulationResult(
            stats_total=[MinerStats(s.blocks_found, s.blocks_share, s.stale_rate) for s in stats],
            sums=list(sums),
            n_runs=n_runs,
            # per device: [launches ms, all-reduce ms] (msim_run_multi_timed)
            extra={"shard_ms": [(shard_ms[2 * g], shard_ms[2 * g + 1]) for g in range(len(devices))]},
        )

    def pipeline_info(self, n_runs: int) -> dict:
        """How msim_launch executes n_runs on the current device (msim_pipeline_info)."""
        pl = _lib.MsimPipelineLayout()
        check(lib.msim_pipeline_info(self._h, n_runs, ctypes.byref(pl)), "msim_pipeline_info")
        return {f: getattr(pl, f) for f, _ in pl._fields_}

    # ---- device-resident form (torch tensors as HBM buffers; used by bench.py and the RCCL path)
    def workspace_bytes(self, n_runs: int) -> int:
        return int(lib.msim_workspace_bytes(self._h, n_runs))

    def launch(self, n_runs: int, run_begin: int, seed_base: int, d_sums, d_workspace, d_status,
               d_per_run=None, d_best_height=None, stream=None) -> None:
        """Asynchronous launch on the current device: all buffers are torch CUDA (HIP) tensors.

        d_sums: int64 [M, 6] (msim_sums); d_status: int32 [2]; d_workspace: uint8 [workspace_bytes]."""
        ptr = (lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None)
        sh = ctypes.c_void_p(stream.cuda_stream) if stream is not None else None
        check(lib.msim_launch(self._h, run_begin, n_runs, seed_base & 0xFFFFFFFF, ptr(d_sums), ptr(d_per_run),
                              ptr(d_best_height), ptr(d_status), ptr(d_workspace), d_workspace.numel(), sh),
              "msim_launch")


def sample_picks(sim: "Simulation", seed: int, n: int, device: int = 0) -> np.ndarray:
    """test.cpp:15-63 MinerPickerSample on the GPU: per-miner counts of n PickFinder draws of RNG{seed}
    (the last entry counts draws where the reference would assert), identical to the sequential loop."""
    m = len(sim.miners)
    out = (ctypes.c_uint64 * (m + 1))()
    check(lib.msim_sample_picks(sim.handle, seed, n, out, device), "msim_sample_picks")
    return np.array(out[:], dtype=np.uint64)


def sample_intervals(seed: int, n: int, device: int = 0) -> dict:
    """test.cpp:191-208 BlockIntervalSample on the GPU: exact integer moments of n NextBlockInterval draws
    of RNG{seed}, plus the mean and standard deviation the reference prints."""
    mo = _lib.MsimIntervalMoments()
    check(lib.msim_sample_intervals(seed, n, ctypes.byref(mo), device), "msim_sample_intervals")
    sumsq = (int(mo.sumsq_hi) << 64) | int(mo.sumsq_lo)
    mean = mo.sum / n if n else 0.0
    var = sumsq / n - mean * mean if n else 0.0
    return {"n": int(mo.n), "sum": int(mo.sum), "sumsq": sumsq, "max": int(mo.max), "mean": mean,
            "std": var ** 0.5 if var > 0 else 0.0}


class Sweep:
    """A grid of networks run in ONE device launch (BASELINE configs[3]; msim_sweep_* in include/msim.h).

    The reference covers a grid by editing SetupMiners (main.cpp:44-65) and rebuilding per point
    (README.md:21-27). Point p, run r of a sweep is bit-identical to Simulation(points[p]).run for run
    run_begin + r: every point sees the same seeds."""

    def __init__(self, points: Sequence[Sequence[Miner]], duration_ms: int = SIM_DURATION_MS):
        self.sims = [Simulation(p, duration_ms) for p in points]
        self.m = len(self.sims[0].miners)
        handles = (ctypes.c_void_p * len(self.sims))(*[s.handle.value for s in self.sims])
        h = ctypes.c_void_p()
        check(lib.msim_sweep_create(handles, len(self.sims), ctypes.byref(h)), "msim_sweep_create")
        self._h = h

    def __len__(self) -> int:
        return len(self.sims)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            lib.msim_sweep_destroy(h)
            self._h = None

    def run_multi(self, runs_per_point: int, run_begin: int = 0, seed_base: int = DEFAULT_SEED_BASE,
                  devices: Sequence[int] = (0,)) -> List[SimulationResult]:
        """msim_sweep_run_multi: every device runs every point on its shard of the runs, one RCCL all-reduce;
        bit-identical to run()'s sums for any device list."""
        n, m = len(self.sims), self.m
        stats = (MsimStats * (n * m))()
        sums = (MsimSums * (n * m))()
        devs = (ctypes.c_int * len(devices))(*devices)
        check(lib.msim_sweep_run_multi(self._h, run_begin, runs_per_point, seed_base & 0xFFFFFFFF, devs, len(devices),
                                       stats, sums), "msim_sweep_run_multi")
        return [SimulationResult(
            stats_total=[MinerStats(s.blocks_found, s.blocks_share, s.stale_rate) for s in stats[p * m:(p + 1) * m]],
            sums=list(sums[p * m:(p + 1) * m]),
            n_runs=runs_per_point,
        ) for p in range(n)]

    def run(self, runs_per_point: int, run_begin: int = 0, seed_base: int = DEFAULT_SEED_BASE, device: int = 0,
            per_run: bool = False) -> List[SimulationResult]:
        n, m = len(self.sims), self.m
        stats = (MsimStats * (n * m))()
        sums = (MsimSums * (n * m))()
        rec = (MsimRunRecord * (n * runs_per_point * m))() if per_run else None
        bh = (ctypes.c_uint32 * (n * runs_per_point))() if per_run else None
        check(lib.msim_sweep_run(self._h, run_begin, runs_per_point, seed_base & 0xFFFFFFFF, device, stats, sums, rec, bh),
              "msim_sweep_run")
        out = []
        for p in range(n):
            res = SimulationResult(
                stats_total=[MinerStats(s.blocks_found, s.blocks_share, s.stale_rate) for s in stats[p * m:(p + 1) * m]],
                sums=list(sums[p * m:(p + 1) * m]),
                n_runs=runs_per_point,
            )
            if per_run:
                a = np.ctypeslib.as_array(ctypes.cast(rec, ctypes.POINTER(ctypes.c_uint32)),
                                          shape=(n, runs_per_point, m, 2))
                res.found = a[p, :, :, 0].copy()
                res.stale = a[p, :, :, 1].copy()
                res.best_height = np.ctypeslib.as_array(bh).reshape(n, runs_per_point)[p].copy()
            out.append(res)
        return out

    def workspace_bytes(self, runs_per_point: int) -> int:
        return int(lib.msim_sweep_workspace_bytes(self._h, runs_per_point))

    def launch(self, runs_per_point: int, run_begin: int, seed_base: int, d_sums, d_workspace, d_status,
               d_per_run=None, d_best_height=None, stream=None) -> None:
        """Asynchronous launch on the current device; d_sums: int64 [n_points, M, 6]."""
        ptr = (lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None)
        sh = ctypes.c_void_p(stream.cuda_stream) if stream is not None else None
        check(lib.msim_sweep_launch(self._h, run_begin, runs_per_point, seed_base & 0xFFFFFFFF, ptr(d_sums),
                                    ptr(d_per_run), ptr(d_best_height), ptr(d_status), ptr(d_workspace),
                                    d_workspace.numel(), sh), "msim_sweep_launch")


def timing_enable(on: bool = True) -> None:
    """Start (or stop) stage timing: HIP events on the launch stream around every msim_launch and every
    draw kernel (K1) it issues (msim_timing_enable)."""
    check(lib.msim_timing_enable(1 if on else 0), "msim_timing_enable")


def timing_read() -> dict:
    """Summed draw-kernel / entity-engine / whole-launch milliseconds and the launch count since the last
    enable/read (synchronises). draws_ms: K1 / W1 (honest pipelines; 0 for selfish networks); engine_ms: E1.
    *_busy_ms: the union of those intervals over every stream (msim_timing_read_all): the stage's share of the
    wall clock when launches overlap on several streams."""
    t = MsimTiming()
    check(lib.msim_timing_read_all(ctypes.byref(t)), "msim_timing_read_all")
    return {k: getattr(t, k) for k, _ in MsimTiming._fields_}


def sums_to_stats(sums_rows: Iterable[Sequence[int]]) -> List[MinerStats]:
    """Fixed-point msim_sums rows ([found, stale, share_hi, share_lo, rate_hi, rate_lo]) -> MinerStats.

    Each Q32.32 sum is converted with one rounding of its exact value (hi << 32) + lo (as
    msim_sums_to_stats), so the result is the same for every split of the runs into launches or ranks."""
    out = []
    for r in sums_rows:
        found, _stale, sh, sl, rh, rl = (int(x) for x in r)
        out.append(MinerStats(found, float((sh << 32) + sl) * 2.0 ** -32, float((rh << 32) + rl) * 2.0 ** -32))
    return out


def exact_stats_total(found: np.ndarray, stale: np.ndarray, best_height: np.ndarray) -> List[MinerStats]:
    """MinerStats per run (main.cpp:22-30) summed in run order (main.cpp:211-217), bit-exact."""
    n, m = found.shape
    tot = [MinerStats() for _ in range(m)]
    for r in range(n):
        L = float(best_height[r])
        for k in range(m):
            f = int(found[r, k])
            share = 0.0 if f == 0 else f / L
            rate = 0.0 if f == 0 else int(stale[r, k]) / f
            tot[k] += MinerStats(f, share, rate)
    return tot


def report(miners: Sequence[Miner], stats_total: Sequence[MinerStats], sim_runs: int,
           duration_ms: int = SIM_DURATION_MS) -> str:
    """The report lines of main.cpp:224-234 (iostream default float format = %g, 6 digits)."""
    days = duration_ms // 86_400_000
    lines = [f"After running {sim_runs} simulations for {days}d each, on average:"]
    for m, s in zip(miners, stats_total):
        line = (f"  - Miner {m.id} ({m.perc}% of network hashrate) found {int(s.blocks_found) // sim_runs} blocks i.e. "
                f"{s.blocks_share * 100 / sim_runs:.6g}% of blocks. Stale rate: {s.stale_rate * 100 / sim_runs:.6g}%.")
        if m.is_selfish:
            line += " ('selfish mining' strategy)"
        lines.append(line)
    return "\n".join(lines)
