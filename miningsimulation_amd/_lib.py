"""ctypes binding of libmsim.so (include/msim.h).

The library is GPU-only: there is no CPU fallback anywhere in the product path. Importing this module
without a built ``libmsim.so`` raises immediately; calling into it without a HIP device returns
MSIM_E_HIP, which the wrappers turn into :class:`MsimError`.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MSIM_LIB", os.path.join(_HERE, "libmsim.so"))

MSIM_OK = 0
MSIM_E_INVALID = -1
MSIM_E_WEIGHTS = -2
MSIM_E_SELFISH = -3
MSIM_E_MINERS = -4
MSIM_E_HIP = -5
MSIM_E_CAPACITY = -6
MSIM_E_PICK = -7
MSIM_MAX_MINERS = 15
MSIM_MAX_SELFISH = 4

# Every symbol include/msim.h declares (checked by tests/test_abi.py).
EXPORTED = (
    "msim_config_create",
    "msim_config_create_weighted",
    "msim_config_is_wide",
    "msim_config_set_concurrent_launches",
    "msim_config_destroy",
    "msim_config_miner_count",
    "msim_run",
    "msim_run_multi",
    "msim_run_multi_timed",
    "msim_multi_release",
    "msim_sweep_run_multi",
    "msim_sweep_point_count",
    "msim_sweep_miner_count",
    "msim_workspace_bytes",
    "msim_launch",
    "msim_device_log1p",
    "msim_device_intervals",
    "msim_device_picks",
    "msim_sums_to_stats",
    "msim_timing_enable",
    "msim_timing_read",
    "msim_timing_read_stages",
    "msim_timing_read_all",
    "msim_pipeline_info",
    "msim_sweep_create",
    "msim_sweep_destroy",
    "msim_sweep_workspace_bytes",
    "msim_sweep_launch",
    "msim_sweep_run",
    "msim_strerror",
    "msim_version",
    "msim_sample_picks",
    "msim_sample_intervals",
)


class MsimTiming(ctypes.Structure):
    _fields_ = [("draws_ms", ctypes.c_double), ("engine_ms", ctypes.c_double), ("launch_ms", ctypes.c_double),
                ("draws_busy_ms", ctypes.c_double), ("engine_busy_ms", ctypes.c_double),
                ("launch_busy_ms", ctypes.c_double), ("launches", ctypes.c_uint32)]


class MsimMiner(ctypes.Structure):
    _fields_ = [
        ("id", ctypes.c_uint32),
        ("perc", ctypes.c_uint64),
        ("propagation_ms", ctypes.c_int64),
        ("is_selfish", ctypes.c_uint8),
    ]


class MsimStats(ctypes.Structure):
    _fields_ = [("blocks_found", ctypes.c_int64), ("blocks_share", ctypes.c_double), ("stale_rate", ctypes.c_double)]


class MsimSums(ctypes.Structure):
    _fields_ = [
        ("blocks_found", ctypes.c_int64),
        ("stale_blocks", ctypes.c_int64),
        ("share_hi", ctypes.c_uint64),
        ("share_lo", ctypes.c_uint64),
        ("rate_hi", ctypes.c_uint64),
        ("rate_lo", ctypes.c_uint64),
    ]


class MsimRunRecord(ctypes.Structure):
    _fields_ = [("found", ctypes.c_uint32), ("stale", ctypes.c_uint32)]


class MsimPipelineLayout(ctypes.Structure):
    _fields_ = [
        ("uses_pipeline", ctypes.c_uint32),
        ("slice_runs", ctypes.c_uint32),
        ("segment_blocks", ctypes.c_uint32),
        ("segments", ctypes.c_uint32),
        ("blocks_per_run", ctypes.c_uint64),
        ("workspace_bytes", ctypes.c_uint64),
        ("rho", ctypes.c_double),
    ]


class MsimError(RuntimeError):
    def __init__(self, code: int, what: str = ""):
        self.code = code
        super().__init__(f"{what}: {strerror(code)} ({code})" if what else f"{strerror(code)} ({code})")


class MsimIntervalMoments(ctypes.Structure):
    _fields_ = [("n", ctypes.c_uint64), ("sum", ctypes.c_uint64), ("sumsq_lo", ctypes.c_uint64),
                ("sumsq_hi", ctypes.c_uint64), ("max", ctypes.c_uint64)]


def _load() -> ctypes.CDLL:
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libmsim.so not found at {LIB_PATH}: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(the simulation path is HIP-only; there is no CPU fallback)"
        )
    lib = ctypes.CDLL(LIB_PATH)
    vp, u32, u64, i64, sz = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int64, ctypes.c_size_t
    lib.msim_config_create.argtypes = [ctypes.POINTER(MsimMiner), u32, i64, ctypes.POINTER(vp)]
    lib.msim_config_create.restype = ctypes.c_int
    lib.msim_config_create_weighted.argtypes = [ctypes.POINTER(MsimMiner), u32, i64, u64, ctypes.POINTER(vp)]
    lib.msim_config_create_weighted.restype = ctypes.c_int
    lib.msim_config_is_wide.argtypes = [vp]
    lib.msim_config_is_wide.restype = ctypes.c_int
    lib.msim_config_set_concurrent_launches.argtypes = [vp, u32]
    lib.msim_config_set_concurrent_launches.restype = ctypes.c_int
    lib.msim_config_destroy.argtypes = [vp]
    lib.msim_config_destroy.restype = None
    lib.msim_config_miner_count.argtypes = [vp]
    lib.msim_config_miner_count.restype = u32
    lib.msim_run.argtypes = [vp, u64, u64, u32, ctypes.c_int, ctypes.POINTER(MsimStats), ctypes.POINTER(MsimSums),
                             ctypes.POINTER(MsimRunRecord), ctypes.POINTER(u32)]
    lib.msim_run.restype = ctypes.c_int
    lib.msim_run_multi.argtypes = [vp, u64, u64, u32, ctypes.POINTER(ctypes.c_int), u32, ctypes.POINTER(MsimStats),
                                   ctypes.POINTER(MsimSums)]
    lib.msim_run_multi.restype = ctypes.c_int
    lib.msim_run_multi_timed.argtypes = [vp, u64, u64, u32, ctypes.POINTER(ctypes.c_int), u32,
                                         ctypes.POINTER(MsimStats), ctypes.POINTER(MsimSums),
                                         ctypes.POINTER(ctypes.c_double)]
    lib.msim_run_multi_timed.restype = ctypes.c_int
    lib.msim_multi_release.argtypes = []
    lib.msim_multi_release.restype = ctypes.c_int
    lib.msim_sweep_run_multi.argtypes = [vp, u64, u64, u32, ctypes.POINTER(ctypes.c_int), u32,
                                         ctypes.POINTER(MsimStats), ctypes.POINTER(MsimSums)]
    lib.msim_sweep_run_multi.restype = ctypes.c_int
    lib.msim_sweep_point_count.argtypes = [vp]
    lib.msim_sweep_point_count.restype = u32
    lib.msim_sweep_miner_count.argtypes = [vp]
    lib.msim_sweep_miner_count.restype = u32
    lib.msim_workspace_bytes.argtypes = [vp, u64]
    lib.msim_workspace_bytes.restype = sz
    lib.msim_launch.argtypes = [vp, u64, u64, u32, vp, vp, vp, vp, vp, sz, vp]
    lib.msim_launch.restype = ctypes.c_int
    lib.msim_device_log1p.argtypes = [vp, vp, u64, vp]
    lib.msim_device_log1p.restype = ctypes.c_int
    lib.msim_device_intervals.argtypes = [vp, vp, u64, vp]
    lib.msim_device_intervals.restype = ctypes.c_int
    lib.msim_device_picks.argtypes = [vp, vp, vp, u64, vp]
    lib.msim_device_picks.restype = ctypes.c_int
    lib.msim_sums_to_stats.argtypes = [ctypes.POINTER(MsimSums), u32, ctypes.POINTER(MsimStats)]
    lib.msim_sums_to_stats.restype = None
    lib.msim_timing_enable.argtypes = [ctypes.c_int]
    lib.msim_timing_enable.restype = ctypes.c_int
    lib.msim_timing_read.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                     ctypes.POINTER(u32)]
    lib.msim_timing_read.restype = ctypes.c_int
    lib.msim_timing_read_stages.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                            ctypes.POINTER(ctypes.c_double), ctypes.POINTER(u32)]
    lib.msim_timing_read_stages.restype = ctypes.c_int
    lib.msim_timing_read_all.argtypes = [ctypes.POINTER(MsimTiming)]
    lib.msim_timing_read_all.restype = ctypes.c_int
    lib.msim_pipeline_info.argtypes = [vp, u64, ctypes.POINTER(MsimPipelineLayout)]
    lib.msim_pipeline_info.restype = ctypes.c_int
    lib.msim_sweep_create.argtypes = [ctypes.POINTER(vp), u32, ctypes.POINTER(vp)]
    lib.msim_sweep_create.restype = ctypes.c_int
    lib.msim_sweep_destroy.argtypes = [vp]
    lib.msim_sweep_destroy.restype = None
    lib.msim_sweep_workspace_bytes.argtypes = [vp, u64]
    lib.msim_sweep_workspace_bytes.restype = sz
    lib.msim_sweep_launch.argtypes = [vp, u64, u64, u32, vp, vp, vp, vp, vp, sz, vp]
    lib.msim_sweep_launch.restype = ctypes.c_int
    lib.msim_sweep_run.argtypes = [vp, u64, u64, u32, ctypes.c_int, ctypes.POINTER(MsimStats),
                                   ctypes.POINTER(MsimSums), ctypes.POINTER(MsimRunRecord), ctypes.POINTER(u32)]
    lib.msim_sweep_run.restype = ctypes.c_int
    lib.msim_strerror.argtypes = [ctypes.c_int]
    lib.msim_strerror.restype = ctypes.c_char_p
    lib.msim_sample_picks.argtypes = [vp, u64, u64, ctypes.POINTER(u64), ctypes.c_int]
    lib.msim_sample_picks.restype = ctypes.c_int
    lib.msim_sample_intervals.argtypes = [u64, u64, ctypes.POINTER(MsimIntervalMoments), ctypes.c_int]
    lib.msim_sample_intervals.restype = ctypes.c_int
    lib.msim_version.argtypes = []
    lib.msim_version.restype = ctypes.c_char_p
    return lib


lib = _load()


def strerror(code: int) -> str:
    return lib.msim_strerror(code).decode()


def check(code: int, what: str = "") -> None:
    if code != MSIM_OK:
        raise MsimError(code, what)
