"""ctypes wrapper of the CPU oracle (oracle/msim_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg,
and only as the checker / the timed CPU baseline. The product path (miningsimulation_amd) never loads it.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import List, Optional, Sequence, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "liboracle.so")
CLI = os.path.join(HERE, "build", "oracle_cli")


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


class OMiner(ctypes.Structure):
    _fields_ = [("id", ctypes.c_uint32), ("perc", ctypes.c_uint64), ("propagation_ms", ctypes.c_int64),
                ("is_selfish", ctypes.c_int32)]


class ORunStats(ctypes.Structure):
    _fields_ = [("blocks_found", ctypes.c_int64), ("stale_blocks", ctypes.c_int64),
                ("blocks_share", ctypes.c_double), ("stale_rate", ctypes.c_double)]


class OSum(ctypes.Structure):
    _fields_ = [("blocks_found", ctypes.c_int64), ("blocks_share", ctypes.c_double), ("stale_rate", ctypes.c_double)]


class ORng(ctypes.Structure):
    _fields_ = [("s0", ctypes.c_uint64), ("s1", ctypes.c_uint64)]


class OTrace(ctypes.Structure):
    _fields_ = [("events", ctypes.c_uint64), ("finds", ctypes.c_uint64), ("best_len", ctypes.c_uint64)]


_lib: Optional[ctypes.CDLL] = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        L.oracle_run.argtypes = [ctypes.POINTER(OMiner), ctypes.c_int, ctypes.c_int64, ctypes.c_uint32, ctypes.c_uint32,
                                 ctypes.POINTER(ORunStats), ctypes.POINTER(OTrace)]
        L.oracle_run_batch.argtypes = [ctypes.POINTER(OMiner), ctypes.c_int, ctypes.c_int64, ctypes.c_uint64,
                                       ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int, ctypes.POINTER(ORunStats),
                                       ctypes.POINTER(OSum)]
        L.oracle_run_batch_w.argtypes = [ctypes.POINTER(OMiner), ctypes.c_int, ctypes.c_int64, ctypes.c_uint64,
                                         ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int,
                                         ctypes.POINTER(ORunStats), ctypes.POINTER(OSum)]
        L.oracle_pick_finder_w.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int, ctypes.c_uint64,
                                           ctypes.POINTER(ORng)]
        L.oracle_pick_counts_w.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int, ctypes.c_uint64,
                                           ctypes.c_uint64, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]
        L.oracle_interval_moments.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]
        L.oracle_rng_seed.argtypes = [ctypes.POINTER(ORng), ctypes.c_uint64]
        L.oracle_rng_rand64.argtypes = [ctypes.POINTER(ORng)]
        L.oracle_rng_rand64.restype = ctypes.c_uint64
        L.oracle_next_block_interval.argtypes = [ctypes.POINTER(ORng)]
        L.oracle_next_block_interval.restype = ctypes.c_int64
        L.oracle_pick_finder.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int, ctypes.POINTER(ORng)]
        L.oracle_state_new.argtypes = [ctypes.POINTER(OMiner)]
        L.oracle_state_new.restype = ctypes.c_void_p
        L.oracle_state_free.argtypes = [ctypes.c_void_p]
        L.oracle_state_set_chain.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32),
                                             ctypes.POINTER(ctypes.c_int64), ctypes.c_size_t]
        L.oracle_state_get_chain.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32),
                                             ctypes.POINTER(ctypes.c_int64), ctypes.c_size_t]
        L.oracle_state_get_chain.restype = ctypes.c_size_t
        L.oracle_state_stale.argtypes = [ctypes.c_void_p]
        L.oracle_state_found_block.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_size_t]
        L.oracle_state_notify.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32),
                                          ctypes.POINTER(ctypes.c_int64), ctypes.c_size_t, ctypes.c_int64]
        L.oracle_selfish_arrival.restype = ctypes.c_int64
        L.oracle_log1p_array.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
        L.oracle_interval_of_array.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
        L.oracle_genesis_id.restype = ctypes.c_uint32
        _lib = L
    return _lib


def _miners(percs: Sequence[int], props: Sequence[int], selfish: Sequence[bool], ids: Optional[Sequence[int]] = None):
    m = len(percs)
    arr = (OMiner * m)()
    for k in range(m):
        arr[k] = OMiner(ids[k] if ids is not None else k, percs[k], props[k], 1 if selfish[k] else 0)
    return arr


def run(percs, props, selfish, duration_ms: int, seed_interval: int, seed_picker: int) -> Tuple[int, np.ndarray]:
    """One RunSimulation: returns (rc, array [M, 2] of (blocks_found, stale_blocks)) plus best length via trace."""
    m = len(percs)
    out = (ORunStats * m)()
    tr = OTrace()
    rc = lib().oracle_run(_miners(percs, props, selfish), m, duration_ms, seed_interval & 0xFFFFFFFF,
                          seed_picker & 0xFFFFFFFF, out, ctypes.byref(tr))
    res = np.array([[out[k].blocks_found, out[k].stale_blocks] for k in range(m)], dtype=np.int64)
    return rc, res, int(tr.best_len) - 1


def run_batch(percs, props, selfish, duration_ms: int, n_runs: int, run_begin: int = 0, seed_base: int = 1000,
              threads: int = 8, total_weight: int = 100, ids: Optional[Sequence[int]] = None):
    """Per-run stats for runs [run_begin, run_begin+n) with the SURVEY seed convention.

    total_weight != 100: `percs` are integer weights summing to it (SURVEY Appendix C generalisation).
    ids: Miner::id per miner (default: the index).
    Returns (found [n, M] int64, stale [n, M] int64, share [n, M] f64, rate [n, M] f64)."""
    m = len(percs)
    out = (ORunStats * (n_runs * m))()
    rc = lib().oracle_run_batch_w(_miners(percs, props, selfish, ids), m, duration_ms, total_weight, run_begin, n_runs,
                                  seed_base & 0xFFFFFFFF, threads, out, None)
    if rc:
        raise RuntimeError(f"oracle_run_batch rc={rc}")
    a = np.ctypeslib.as_array(ctypes.cast(out, ctypes.POINTER(ctypes.c_uint8)), shape=(n_runs * m * 32,))
    rec = np.frombuffer(a.tobytes(), dtype=np.dtype([("f", "<i8"), ("s", "<i8"), ("sh", "<f8"), ("r", "<f8")]))
    rec = rec.reshape(n_runs, m)
    return rec["f"].copy(), rec["s"].copy(), rec["sh"].copy(), rec["r"].copy()


def rng_stream(seed: int, n: int) -> List[int]:
    r = ORng()
    lib().oracle_rng_seed(ctypes.byref(r), seed)
    return [lib().oracle_rng_rand64(ctypes.byref(r)) for _ in range(n)]


def intervals(seed: int, n: int) -> List[int]:
    r = ORng()
    lib().oracle_rng_seed(ctypes.byref(r), seed)
    return [lib().oracle_next_block_interval(ctypes.byref(r)) for _ in range(n)]


def picks(percs: Sequence[int], seed: int, n: int) -> List[int]:
    r = ORng()
    lib().oracle_rng_seed(ctypes.byref(r), seed)
    P = (ctypes.c_uint64 * len(percs))(*percs)
    return [lib().oracle_pick_finder(P, len(percs), ctypes.byref(r)) for _ in range(n)]


def picks_w(weights: Sequence[int], total_weight: int, seed: int, n: int) -> List[int]:
    """PickFinder with the Appendix C weight generalisation (multiplier UINT64_MAX // W)."""
    r = ORng()
    lib().oracle_rng_seed(ctypes.byref(r), seed)
    P = (ctypes.c_uint64 * len(weights))(*weights)
    mult = 0xFFFFFFFFFFFFFFFF // total_weight
    return [lib().oracle_pick_finder_w(P, len(weights), mult, ctypes.byref(r)) for _ in range(n)]


def pick_counts(weights: Sequence[int], total_weight: int, seed: int, n: int) -> np.ndarray:
    """test.cpp:15-63 MinerPickerSample, sequential: counts per miner (+ fall-throughs last)."""
    m = len(weights)
    out = (ctypes.c_uint64 * (m + 1))()
    lib().oracle_pick_counts_w((ctypes.c_uint64 * m)(*weights), m, total_weight, seed, n, out)
    return np.array(out[:], dtype=np.uint64)


def interval_moments(seed: int, n: int) -> dict:
    """test.cpp:191-208 BlockIntervalSample, sequential: exact integer moments."""
    out = (ctypes.c_uint64 * 4)()
    lib().oracle_interval_moments(seed, n, out)
    return {"sum": int(out[0]), "sumsq": (int(out[2]) << 64) | int(out[1]), "max": int(out[3])}


def log1p_array(x: np.ndarray) -> np.ndarray:
    """glibc log1p elementwise (what the reference calls, xoroshiro128++.h:19)."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    out = np.empty_like(x)
    lib().oracle_log1p_array(x.ctypes.data, out.ctypes.data, x.size)
    return out


def interval_of_array(u: np.ndarray) -> np.ndarray:
    """NextBlockInterval (simulation.h:205-210) of given uniform u64 draws, in ms."""
    u = np.ascontiguousarray(u, dtype=np.uint64)
    out = np.empty(u.shape, dtype=np.int64)
    lib().oracle_interval_of_array(u.ctypes.data, out.ctypes.data, u.size)
    return out


class MinerState:
    """An explicit-chain Miner (simulation.h:41-202) for replaying test.cpp's TestSelfishStrategy."""

    def __init__(self, id: int, perc: int, prop_ms: int, selfish: bool):
        self._h = lib().oracle_state_new(_miners([perc], [prop_ms], [selfish], [id]))

    def __del__(self):
        if getattr(self, "_h", None):
            lib().oracle_state_free(self._h)
            self._h = None

    @staticmethod
    def _arrays(chain):
        n = len(chain)
        ids = (ctypes.c_uint32 * max(n, 1))(*[b[0] for b in chain])
        arr = (ctypes.c_int64 * max(n, 1))(*[b[1] for b in chain])
        return ids, arr, n

    def set_chain(self, chain):
        ids, arr, n = self._arrays(chain)
        lib().oracle_state_set_chain(self._h, ids, arr, n)

    def chain(self):
        ids = (ctypes.c_uint32 * 4096)()
        arr = (ctypes.c_int64 * 4096)()
        n = lib().oracle_state_get_chain(self._h, ids, arr, 4096)
        return [(int(ids[i]), int(arr[i])) for i in range(n)]

    def found_block(self, t: int, best_chain_size: int):
        lib().oracle_state_found_block(self._h, t, best_chain_size)

    def notify(self, best_chain, t: int):
        ids, arr, n = self._arrays(best_chain)
        lib().oracle_state_notify(self._h, ids, arr, n, t)

    @property
    def stale(self) -> int:
        return lib().oracle_state_stale(self._h)


SELFISH_ARRIVAL = (1 << 63) - 1
GENESIS_ID = 0xFFFFFFFF
