"""Multi-GPU sharding of runs: one process per GPU, one all-reduce of integer sums.

The reference's only parallelism is one std::async thread per run (main.cpp:205-220), with the per-miner
MinerStats summed on the main thread. Runs are independent and their seeds are a pure function of the run
index, so here rank r of W takes a contiguous run range and the ranks combine their per-miner sums with a
single all-reduce (backend "nccl" = RCCL over xGMI on MI355X; "gloo" in CPU tests). The sums are integers
(msim_sums: found, stale and Q32.32 fixed-point share/stale-rate limbs), so the result is bit-identical
for every W and every partition.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Tuple

FIXED_ONE = 4294967296.0  # 2^32: per-run share / stale_rate are summed as round(x * 2^32)


def shard(n_total: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous partition of runs [0, n_total): rank r gets [begin, begin + n)."""
    base, rem = divmod(n_total, world)
    begin = rank * base + min(rank, rem)
    return begin, base + (1 if rank < rem else 0)


def fixed_point(x: float) -> Tuple[int, int]:
    """The device's per-run conversion (msim_kernels.hip): v = (uint64)(x * 2^32 + 0.5) -> (v >> 32, v & 0xffffffff)."""
    v = int(x * FIXED_ONE + 0.5)
    return v >> 32, v & 0xFFFFFFFF


def sums_rows_from_runs(found, stale, share, rate) -> List[List[int]]:
    """msim_sums rows [found, stale, share_hi, share_lo, rate_hi, rate_lo] from per-run values [n, M]."""
    n, m = found.shape
    rows = [[0] * 6 for _ in range(m)]
    for r in range(n):
        for k in range(m):
            sh, sl = fixed_point(float(share[r, k]))
            rh, rl = fixed_point(float(rate[r, k]))
            row = rows[k]
            row[0] += int(found[r, k])
            row[1] += int(stale[r, k])
            row[2] += sh
            row[3] += sl
            row[4] += rh
            row[5] += rl
    return rows


def allreduce_sums(local_rows, device=None):
    """SUM all-reduce of the [M, 6] int64 sums over the default process group; returns the global rows."""
    import torch
    import torch.distributed as dist

    t = torch.as_tensor(local_rows, dtype=torch.int64, device=device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t)
    return t.cpu().tolist()


MAX_LAUNCH_RUNS = 1 << 26  # msim_launch's per-call limit (msim_api.hip); larger shards run in chunks


def run_sharded(sim, n_total: int, seed_base: int, run_begin: int = 0, stream=None,
                launch: Optional[Callable] = None, device=None, max_chunk: int = MAX_LAUNCH_RUNS):
    """This rank's shard through msim_launch on the current device, then one all-reduce (RCCL on GPUs) of the
    sums with the status words packed behind them.

    Returns the global [M, 6] int64 sums as a tensor on `device` (identical on every rank). `launch`
    replaces sim.launch (same signature, workspace None) so that the partition, chunking, status check and
    all-reduce can be exercised on CPU ranks with a gloo group (tests/test_distributed.py)."""
    import contextlib

    import torch
    import torch.distributed as dist

    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    begin, n = shard(n_total, world, rank)
    m = len(sim.miners)
    dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    # the sums and the two status words in one buffer: ONE all-reduce per job
    buf = torch.zeros(6 * m + 2, dtype=torch.int64, device=dev)
    sums = buf[: 6 * m].view(m, 6)
    status = buf[6 * m:]
    part = torch.zeros((m, 6), dtype=torch.int64, device=dev)
    pst = torch.zeros(2, dtype=torch.int32, device=dev)
    chunk = min(n, max_chunk)
    ws = None
    if n and launch is None:
        ws = torch.empty(sim.workspace_bytes(chunk), dtype=torch.uint8, device=dev)
    # Everything that touches the launch's outputs runs on the launch stream: the adds read `part` / `pst`
    # after the kernels that wrote them, the next chunk's launch overwrites them only after the adds, and
    # the all-reduce (RCCL enqueues on the current stream) sees the final sums.
    # The buffers above were zeroed on the caller's current stream: the launch stream waits for that first.
    ctx = torch.cuda.stream(stream) if (stream is not None and dev.type == "cuda") else contextlib.nullcontext()
    if stream is not None and dev.type == "cuda":
        stream.wait_stream(torch.cuda.current_stream(dev))
    with ctx:
        for off in range(0, n, max(chunk, 1)):
            cn = min(chunk, n - off)
            (launch or sim.launch)(cn, run_begin + begin + off, seed_base, part, ws, pst, stream=stream)
            sums += part
            status += pst
        if world > 1:
            dist.all_reduce(buf)
    if stream is not None and dev.type == "cuda":
        torch.cuda.current_stream(dev).wait_stream(stream)  # the caller's stream sees the result
    if int(status[1].item()) != 0:
        raise RuntimeError(f"{int(status[1].item())} runs exceeded the compact state capacity")
    return sums
