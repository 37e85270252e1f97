"""Sweep throughput (BASELINE configs[3]): the 360-point grid (selfish share 10..49 % x propagation
0.1..30 s) in ONE device launch per step, run-years/s of the whole job.

    python scripts/bench_sweep.py [--runs-per-point 2048] [--steps 2] [--warmup 1]
    torchrun --nproc-per-node N scripts/bench_sweep.py ...   (runs of every point sharded over ranks)

configs[3] is 2^16 runs per point over 8 GPUs (8192 per GPU per point); the default here is a bounded
2048 per point so one step stays ~10 s on one GPU. Prints one JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs-per-point", type=int, default=2048, help="per GPU per step")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--seed-base", type=int, default=1000)
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from miningsimulation_amd import Sweep, c4_grid

    grid = c4_grid()
    sw = Sweep(grid)
    m, npts, rpp = sw.m, len(sw), args.runs_per_point
    dev = torch.device("cuda", local)
    ws = torch.empty(sw.workspace_bytes(rpp), dtype=torch.uint8, device=dev)
    sums = torch.zeros((npts, m, 6), dtype=torch.int64, device=dev)
    total = torch.zeros_like(sums)
    status = torch.zeros(2, dtype=torch.int32, device=dev)
    fails = torch.zeros(1, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev)

    def step(i: int, ev=None):
        begin = (i * world + rank) * rpp  # disjoint run ranges per step and rank
        if ev is not None:
            ev[0].record(stream)
        sw.launch(rpp, begin, args.seed_base, sums, ws, status, stream=stream)
        if ev is not None:
            ev[1].record(stream)
        fails.add_(status[1:2].to(torch.int64))
        if world > 1:
            dist.all_reduce(sums)  # per-(point, miner) integer sums: the sweep's only exchange
        total.add_(sums)

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    total.zero_()
    fails.zero_()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i, evs[i])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = sum(a.elapsed_time(b) for a, b in evs) / args.steps
    t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(fails)
    elapsed, kern_ms = float(t[0]), float(t[1])
    if int(fails.item()) != 0:
        raise SystemExit(f"{int(fails.item())} runs exceeded the compact state capacity")
    runs_total = args.steps * rpp * npts * world
    tot = total.cpu()
    # sanity: the selfish miner's average block share at h = 40 %, 1 s (README.md:89-107 example)
    i40 = [k for k, g in enumerate(grid) if g[0].perc == 40 and g[0].propagation_ms == 1000][0]
    share40 = (float(tot[i40, 0, 2]) + float(tot[i40, 0, 3]) * 2.0**-32) / (args.steps * rpp * world) * 100
    if rank == 0:
        print(json.dumps({
            "metric": "simulated run-years/sec (whole node), 360-point sweep",
            "value": round(runs_total / elapsed, 1),
            "unit": "run-years/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "kernel_ms": round(kern_ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "dtype": "int64+fp64",
            "data": "synthetic (seeded runs)",
            "config": {"workload": "c4: BASELINE configs[3] (40 selfish shares x 9 propagations)",
                       "points": npts, "runs_per_point_per_gpu": rpp,
                       "selfish40_1s_share_pct": round(share40, 4)},
        }), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
