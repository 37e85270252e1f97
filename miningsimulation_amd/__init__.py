"""miningsimulation_amd — MI355X-native engine for darosior/miningsimulation's per-run simulation loop.

One simulation run per GPU lane (hand-written gfx950 HIP, libmsim.so behind the C ABI in
include/msim.h); runs shard across GPUs with one RCCL all-reduce of integer sums (bench.py,
miningsimulation_amd.distributed). See DESIGN.md.
"""
from ._lib import MsimError, LIB_PATH  # noqa: F401  (raises ImportError when libmsim.so is missing)
from .simulation import (  # noqa: F401
    C4_PROPAGATIONS_MS,
    C4_SELFISH_PERCS,
    C5_TOTAL_WEIGHT,
    PRESET_WEIGHTS,
    DEFAULT_SEED_BASE,
    PRESETS,
    SIM_DURATION_MS,
    SIM_RUNS,
    Miner,
    MinerStats,
    Simulation,
    SimulationResult,
    Sweep,
    c4_grid,
    c5_network,
    exact_stats_total,
    report,
    sample_intervals,
    sample_picks,
    setup_miners,
    sums_to_stats,
    timing_enable,
    timing_read,
)

from . import model  # noqa: F401,E402  (first-order analytical stale-rate model, plot.py restated)

__version__ = "0.1.0"
