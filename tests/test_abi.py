"""The C-ABI library loads and exports every symbol include/msim.h declares (no GPU calls), and the
ctypes structs match the header's layouts."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    with open(os.path.join(ROOT, "include", "msim.h")) as f:
        src = f.read()
    return sorted(set(re.findall(r"\b(msim_[a-z0-9_]+)\s*\(", src)))


def test_exports_every_declared_symbol(msim_lib_path):
    lib = ctypes.CDLL(msim_lib_path)
    declared = _declared()
    assert len(declared) >= 12
    for name in declared:
        assert hasattr(lib, name), name


def test_python_binding_covers_header(msim_lib_path):
    from miningsimulation_amd import _lib

    assert sorted(_lib.EXPORTED) == _declared()


def test_struct_layouts(msim_lib_path):
    from miningsimulation_amd import _lib

    assert ctypes.sizeof(_lib.MsimStats) == 24  # MinerStats: long, double, double (main.cpp:13-20)
    assert ctypes.sizeof(_lib.MsimSums) == 48
    assert ctypes.sizeof(_lib.MsimRunRecord) == 8
    assert ctypes.sizeof(_lib.MsimMiner) == 32


def test_config_validation_without_gpu(msim_lib_path):
    """Config creation is host-only: the reference's asserted preconditions become error codes."""
    from miningsimulation_amd import Miner, MsimError, Simulation, setup_miners
    from miningsimulation_amd import _lib

    Simulation(setup_miners())  # valid
    bad = [
        ([Miner(0, 60, 1000), Miner(1, 30, 1000)], _lib.MSIM_E_WEIGHTS),            # sums to 90
        ([Miner(0, 60, 1000), Miner(1, 50, 1000)], _lib.MSIM_E_WEIGHTS),            # sums to 110
        # a selfish network whose one G lane (every block of every miner's chain) exceeds 96 GiB
        ([Miner(k, 1 if k < 100 else 0, 1000, k == 0) for k in range(160000)], _lib.MSIM_E_MINERS),
        ([Miner(0, 50, -1), Miner(1, 50, 1000)], _lib.MSIM_E_INVALID),
    ]
    for miners, code in bad:
        try:
            Simulation(miners)
        except MsimError as e:
            assert e.code == code, (miners, e)
        else:
            raise AssertionError(f"accepted invalid network {miners}")
    # several selfish miners, and selfish miners in weighted networks, run on the entity engine (msim_sel.h)
    for miners, W in (([Miner(0, 50, 1000, True), Miner(1, 50, 1000, True)], 100),
                      ([Miner(k, 25, 1000, k < 4) for k in range(4)], 100),
                      ([Miner(0, 7, 1000, True), Miner(1, 3, 1000)], 10)):
        sim = Simulation(miners, total_weight=W)
        assert not sim.wide and sim.pipeline_info(1024)["uses_pipeline"] == 3
    # every other network with selfish miners runs on the general engine (msim_general.h): more than
    # MSIM_MAX_SELFISH selfish miners, or selfish miners in networks of more than 15 miners, any W
    for miners, W in (([Miner(k, 20, 1000, True) for k in range(5)], 100),
                      ([Miner(k, 7 if k < 10 else 5, 1000, k == 0) for k in range(16)], 100),
                      ([Miner(k, 1, 1000, k == 0) for k in range(16)], 16)):
        assert Simulation(miners, total_weight=W).pipeline_info(1024)["uses_pipeline"] == 4
    # the reference's id semantics (shared / Genesis ids, simulation.h:31-38, main.cpp:24-26) and honest
    # networks beyond the large-network pipeline run on the general engine too
    for miners in ([Miner(0, 50, 1000), Miner(0, 50, 1000)],
                   [Miner(0xFFFFFFFF, 30, 1000)] + [Miner(k, 10, 1000) for k in range(7)],
                   [Miner(k, 1 if k < 100 else 0, 1000) for k in range(4097)]):
        sim = Simulation(miners)
        assert sim.pipeline_info(1024)["uses_pipeline"] == 4
    # G's windows follow its byte budget (one lane of the last window at least): a 1 026-miner network with a
    # selfish miner, and the fallback G reserves behind every entity-engine launch, stay bounded
    big = Simulation([Miner(k, w, 1000, k == 0) for k, w in enumerate([30720, 29696] + [41] * 1024)],
                     total_weight=102400)
    assert big.pipeline_info(1024)["uses_pipeline"] == 4
    assert big.workspace_bytes(65536) < 3 * 2**30, big.workspace_bytes(65536)
    # configs[2] at its per-GPU size: E1 stays under 1 GiB; the opt-in segment-parallel form (msim_selseg.h,
    # MSIM_SELSEG) keeps every run's worker subs and checkpoints within its 24 GiB slice budget
    import os
    e1 = Simulation(setup_miners(1000, selfish_perc=40))
    assert e1.pipeline_info(131072)["uses_pipeline"] == 3
    assert e1.workspace_bytes(131072) < 2**30
    os.environ["MSIM_SELSEG"] = "1"
    try:
        c3 = Simulation(setup_miners(1000, selfish_perc=40))
        info = c3.pipeline_info(131072)
        assert info["uses_pipeline"] == 6 and info["segments"] >= 2, info
        assert c3.workspace_bytes(131072) < 26 * 2**30, c3.workspace_bytes(131072)
    finally:
        del os.environ["MSIM_SELSEG"]
    # the large-network path (msim_wide.h): more than 15 honest miners, or integer weights
    assert Simulation([Miner(k, 7 if k < 10 else 5, 1000) for k in range(16)]).wide
    assert not Simulation(setup_miners()).wide
    # an honest network on G sizes its windows to 4 096 blocks (honest forks fold far inside it):
    # 20 000 miners fit, and the workspace stays at the 2 GiB window budget
    huge = Simulation([Miner(k, 1 if k < 100 else 0, 1000) for k in range(20000)])
    assert huge.pipeline_info(1024)["uses_pipeline"] == 4
    assert huge.workspace_bytes(65536) < 3 * 2**30, huge.workspace_bytes(65536)
    c5 = [Miner(k, w, 1000) for k, w in enumerate([30720, 29696] + [41] * 1024)]
    assert Simulation(c5, total_weight=102400).wide
    for miners, W, code in (
        (c5, 102401, _lib.MSIM_E_WEIGHTS),                                      # weights sum to 102400
        ([Miner(0, 1 << 31, 1000)], 1 << 31, _lib.MSIM_E_WEIGHTS),              # W >= 2^31
    ):
        try:
            Simulation(miners, total_weight=W)
        except MsimError as e:
            assert e.code == code, (W, e)
        else:
            raise AssertionError(f"accepted invalid weighted network (W={W})")


def test_concurrent_launches_hint(msim_lib_path):
    """msim_config_set_concurrent_launches: 1..64 accepted, anything else MSIM_E_INVALID; it may change the
    workspace the pipeline asks for (K1's grid), never the config's validity."""
    from miningsimulation_amd import MsimError, Simulation, setup_miners

    sim = Simulation(setup_miners(100))
    for bad in (0, 65):
        with pytest.raises(MsimError):
            sim.set_concurrent_launches(bad)
    for ok in (1, 2, 64):
        sim.set_concurrent_launches(ok)
        assert sim.workspace_bytes(32768) > 0


def test_report_format():
    from miningsimulation_amd import MinerStats, report, setup_miners

    miners = setup_miners(10_000)
    # README.md:55-56 first line, from its printed averages
    st = [MinerStats(15621 * 32768, 0.300901 * 32768, 0.010092 * 32768)] + [MinerStats()] * 8
    out = report(miners, st, 32768).splitlines()
    assert out[0] == "After running 32768 simulations for 365d each, on average:"
    assert out[1] == "  - Miner 0 (30% of network hashrate) found 15621 blocks i.e. 30.0901% of blocks. Stale rate: 1.0092%."


def test_general_engine_keeps_full_window_for_long_delays():
    """G (msim_general_launch.h) drops its full-chain last window tier for honest networks, whose forks fold
    within 4 096 blocks, but keeps it when the largest propagation delay could span a quarter of that window
    (a honest network with delays of days would otherwise fail with MSIM_E_CAPACITY). Host-only:
    msim_pipeline_info reports G's tier count as `segments`."""
    from miningsimulation_amd import Miner, Simulation

    def tiers(prop_ms, selfish=False):
        miners = [Miner(k, 1 if k < 100 else 0, prop_ms, selfish and k == 0) for k in range(5000)]
        info = Simulation(miners).pipeline_info(64)
        assert info["uses_pipeline"] == 4, info
        return info["segments"]

    assert tiers(1000) == 2                 # 1 s: forks fold within a few blocks
    assert tiers(6 * 3600 * 1000) == 2      # 6 h: ~36 blocks per delay
    assert tiers(5 * 86400 * 1000) == 3     # 5 days: ~720 blocks per delay + 10 sigma + 64 > 1 024
    assert tiers(1000, selfish=True) == 3   # a selfish miner can withhold every block
