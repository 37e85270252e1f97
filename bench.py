"""Throughput benchmark: simulated run-years/s of darosior/miningsimulation's per-run loop on MI355X.

One step = one batch of `--runs` (default 32768 = SIM_RUNS, main.cpp:10) independent runs of
RunSimulation(months{12}) per GPU on BASELINE.json configs[1] (9-miner 2025 network, 100 ms propagation),
followed by the single exchange step of the path: an RCCL all-reduce of the per-miner integer sums.
Weak scaling: per-GPU work is fixed; each step and rank takes a fresh, disjoint run range (fresh seeds).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2] [--runs 32768]
    torchrun --nproc-per-node N bench.py --gpus N ...      (one process per GPU, RCCL over xGMI)

With --gpus N > 1 and no WORLD_SIZE in the environment, bench.py starts the N ranks itself (one child
process per GPU, 127.0.0.1 rendezvous) before anything touches HIP, relays rank 0's JSON line and exits
non-zero if any rank fails: the reference's own driver fans out over every hardware thread the same way
(main.cpp:198-209).

Rank 0 prints ONE JSON line (driver contract) with a live VALU roofline (HIP events around every launch
on the launch stream) and, at N=1, the CPU baseline: the oracle (explicit-chain C port of the reference
loop, oracle/msim_oracle.c) timed on a bounded sample on the host's cores.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# MI355X VALU peak (MI355X_MICROARCH.md: 256 CUs, 4 SIMD-32 per CU, 2.4 GHz): 256*4*32*2.4e9 lane-ops/s.
VALU_PEAK_LANE_OPS = 256 * 4 * 32 * 2.4e9
BLOCKS_PER_RUN_YEAR = 31_556_952_000 / 600_000  # SIM_DURATION / BLOCK_INTERVAL = 52594.92


# PMC constants of the dominant kernel per launch at the default run counts, from rocprofv3 --pmc passes of
# `bench.py --config C --steps 2 --warmup 0 --streams 1` (scripts/gpu_pmc_r05.sh: FETCH_SIZE, WRITE_SIZE and the SQ
# set in separate passes; the files hold values summed over the 2 launches, KB). PMC counters cannot be collected
# inside the timed process: these are the recorded values of the same kernel, and every field computed from them
# names its file.
#   traffic = FETCH_SIZE x 2 (gfx950: FETCH_SIZE counts half the bytes of wide reads, MI355X_MICROARCH.md §HBM)
#             + WRITE_SIZE, bytes per launch;
#   valu    = SQ_INSTS_VALU (wave instructions) per launch: the counter-based VALU issue fraction is
#             valu x 64 lanes / the kernel's time / peak.
PMC_DIR = "profiles/r05/final/pmc"
PMC = {
    ("c2", 32768): {"kernel": "K1 msim_draws_kernel", "file": "pmc_c2.txt"},
    ("c3", 131072): {"kernel": "E1 msim_sel_kernel<9,1,1,4,1,4,true>", "file": "pmc_c3.txt"},
    ("c5", 65536): {"kernel": "W1 msim_wide_draws_kernel<4>", "file": "pmc_c5.txt"},
}
# rocprofv3 --kernel-trace --stats summaries (scripts/rocprof_summary.py) of the exact bench commands: the default
# two streams (_s0) and --streams 1 (_s1). Their "busy ms/call" column is the union of the kernel's dispatch
# intervals per call, the file-backed counterpart of the live dominant_ms; the serial file's average is the
# kernel alone.
ROCPROF_DIR = "profiles/r05/final"
KERNEL_SUBSTR = {"c1": "msim_draws_kernel", "c2": "msim_draws_kernel", "c3": "msim_sel_kernel<",
                 "c5": "msim_wide_draws_kernel"}


def pmc_constants(config: str, n: int) -> dict | None:
    """{kernel, src, fetch_kb, write_kb, valu} per launch from the committed PMC file (None if absent)."""
    ent = PMC.get((config, n))
    if not ent:
        return None
    path = os.path.join(PMC_DIR, ent["file"])
    try:
        txt = open(os.path.join(ROOT, path)).read()
    except OSError:
        return None
    # scripts/pmc_csv.py format: a header "<kernel>  dispatches=D  mean_ms=..." (D over the three passes), then
    # "    <COUNTER>  <value summed over the launches of its pass>" lines
    vals, cur, launches = {}, False, 2
    for ln in txt.splitlines():
        if not ln.startswith(" "):
            cur = KERNEL_SUBSTR[config] in ln and not vals
            if cur:
                for tok in ln.split():
                    if tok.startswith("dispatches=") and int(tok.split("=")[1]) % 3 == 0:
                        launches = max(1, int(tok.split("=")[1]) // 3)
            continue
        parts = ln.split()
        if cur and len(parts) == 2:
            vals[parts[0]] = float(parts[1])
    vals = {k: v / launches for k, v in vals.items()}
    need = ("FETCH_SIZE", "WRITE_SIZE", "SQ_INSTS_VALU")
    if not all(k in vals for k in need):
        return None
    return {"kernel": ent["kernel"], "src": path, "fetch_kb": vals["FETCH_SIZE"], "write_kb": vals["WRITE_SIZE"],
            "valu": vals["SQ_INSTS_VALU"]}


def rocprof_kernel_ms(config: str, streams: int) -> dict | None:
    """{file, avg_ms, busy_ms} of the dominant kernel in the committed rocprof summary of this command."""
    path = os.path.join(ROCPROF_DIR, f"rocprof_{config}_s{0 if streams == 2 else 1}.md")
    try:
        rows = open(os.path.join(ROOT, path)).read().splitlines()
    except OSError:
        return None
    for ln in rows:
        cells = [c.strip() for c in ln.strip().strip("|").split("|")]
        if len(cells) >= 6 and KERNEL_SUBSTR.get(config, "?") in cells[0]:
            try:
                return {"file": path, "avg_ms": float(cells[3]), "busy_ms": float(cells[5])}
            except ValueError:
                return None
    return None


def w_blk(m: int) -> int:
    """SURVEY §8(d) fixed accounting convention: algorithmic VALU lane-ops per simulated block."""
    import math

    return 140 + 4 * math.ceil(math.log2(max(m, 2)))


# SURVEY §8(d) calibration of the oracle port against the reference binary: both at 8 threads in the
# same 8-vCPU build container (Intel Xeon @ 2.1 GHz), c2 at 32 768 runs: the unmodified reference
# measured 609 run-years/s; the port measured 352.1 run-years/s (oracle_cli time c2
# 32768 8, 93.08 s). A port figure divided by this ratio estimates the reference binary on the same cores.
PORT_TO_REFERENCE = round(352.056 / 609.0, 4)


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform

    return platform.processor() or "unknown"


def host_threads() -> tuple[int, int, str]:
    """(threads to use, visible CPUs, note). The GPU box exports OMP_NUM_THREADS = the CPU share one GPU
    job may use (its nproc shows the whole machine); the harness asks worker pools to stay within that
    share, so the timed sample uses it and the all-cores figure is extrapolated from it (cpu_baseline)."""
    cpus = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    share = os.environ.get("OMP_NUM_THREADS")
    if share and share.isdigit() and 0 < int(share) < cpus:
        return int(share), cpus, f"{share} of {cpus} visible CPUs (the job's CPU share, OMP_NUM_THREADS)"
    return cpus, cpus, f"all {cpus} visible CPUs"


def cgroup_cpu_quota() -> str | None:
    """cgroup v2 cpu.max of this process (quota period), if readable."""
    try:
        with open("/proc/self/cgroup") as f:
            rel = f.read().strip().split("::")[-1]
        with open(os.path.join("/sys/fs/cgroup", rel.lstrip("/"), "cpu.max")) as f:
            return f.read().strip()
    except OSError:
        return None


def cpu_baseline(preset: str, sample_runs: int, threads: int, visible: int, target_s: float = 15.0) -> dict:
    """The oracle port (explicit chains like the reference) timed on `threads` host threads, plus a
    one-thread sample (the per-core rate) and the all-visible-CPUs extrapolation of the threaded rate."""
    from oracle import pyoracle

    pyoracle.build()

    def timed(runs: int, th: int) -> dict:
        out = subprocess.run([pyoracle.CLI, "time", preset, str(runs), str(th)], capture_output=True,
                             text=True, check=True)
        return json.loads(out.stdout.splitlines()[0])

    per = 1 if preset == "c5" else 16  # c5: ~1 run-year/s per core (explicit chains, 1026 miners)
    if not sample_runs:  # calibrate on a small sample, then size the real sample to ~target_s seconds
        probe = timed(threads * per, threads)
        sample_runs = max(threads * per, int(probe["run_years_per_s"] * target_s) // threads * threads)
    rec = timed(sample_runs, threads)
    one = timed(max(1, per // 2), 1)  # per-core rate (a few seconds)
    per_thread = rec["run_years_per_s"] / threads
    return {
        "value": round(rec["run_years_per_s"], 2),
        "unit": "run-years/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{sample_runs} runs x 365.2425 d of preset {preset} (oracle/msim_oracle.c, explicit chains as "
                  f"in the reference, {threads} pthreads), {rec['seconds']:.1f} s wall",
        "cpu_model": cpu_model(),
        "visible_cpus": visible,
        "cgroup_cpu_max": cgroup_cpu_quota(),
        "one_thread_value": round(one["run_years_per_s"], 3),
        "all_visible_cpus_extrapolated": round(per_thread * visible, 1),
        "all_cpus_note": f"{threads}-thread rate / {threads} x {visible} visible CPUs: the job may use only its "
                         f"CPU share, so the whole-host figure is extrapolated (linear, an upper bound)",
        "port_to_reference_ratio": PORT_TO_REFERENCE,
        "reference_equivalent": round(rec["run_years_per_s"] / PORT_TO_REFERENCE, 2),
        "reference_equivalent_all_visible_cpus": round(per_thread * visible / PORT_TO_REFERENCE, 1),
        "calibration": "port 352.1 vs reference binary 609 run-years/s, c2, 32768 runs, 8 threads, same container "
                       "(BASELINE.md §2); reference_equivalent = value / ratio",
    }


def free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def spawn_ranks(n: int, argv: list[str], timeout_s: float = 1800.0) -> int:
    """Start ranks 0..n-1 of this script (one process per GPU) and relay rank 0's stdout. The parent never
    imports torch or touches HIP: each child initialises its own device. Every rank is polled: the first
    rank to fail (or the overall time limit) ends the job, and the remaining ranks, rank 0 included, are
    killed, so a rank stuck in a collective whose peer died cannot hang the parent."""
    import tempfile

    port = free_port()
    procs = []
    out0 = tempfile.TemporaryFile(mode="w+")  # rank 0's stdout (a file: no pipe to drain while polling)
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env,
                                      stdout=out0 if r == 0 else subprocess.DEVNULL, text=True))
    t_end = time.monotonic() + timeout_s
    failed = None
    while True:
        codes = [p.poll() for p in procs]
        bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
        if bad:
            failed = f"rank {bad[0][0]} exited with {bad[0][1]}"
            break
        if all(c == 0 for c in codes):
            break
        if time.monotonic() > t_end:
            failed = f"time limit {timeout_s:.0f} s"
            break
        time.sleep(0.2)
    if failed:
        for p in procs:
            if p.poll() is None:
                p.kill()
        codes = [p.wait() for p in procs]
        print(f"bench.py: {failed}; rank exit codes {codes}", file=sys.stderr)
        return 1
    out0.seek(0)
    for ln in out0.read().splitlines():  # the JSON line to stdout; library chatter (gloo/RCCL banners) to stderr
        print(ln, file=sys.stdout if ln.startswith("{") else sys.stderr, flush=True)
    return 0


class _StubSim:
    """--stub (tests only): a CPU stand-in for Simulation that fills deterministic integer sums, so the
    rank spawn / gloo reduction / JSON path of this script runs without a GPU. Never used for a number."""

    def __init__(self, m: int):
        self.m, self.wide = m, False

    def pipeline_info(self, n):
        return {"uses_pipeline": 1, "stub": 1}

    def workspace_bytes(self, n):
        return 8

    def launch(self, n, begin, seed_base, sums, ws, status, stream=None):
        import torch

        sums.copy_(torch.arange(sums.numel(), dtype=torch.int64).reshape(sums.shape) + n)
        status.zero_()


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--config", default="c2", choices=["c1", "c2", "c3", "c5", "default"])
    ap.add_argument("--runs", type=int, default=0,
                    help="runs per GPU per step (0: 32768 = SIM_RUNS; c3: 131072 = configs[2]'s 1M runs / 8 GPUs; c5: 65536)")
    ap.add_argument("--seed-base", type=int, default=1000)
    ap.add_argument("--streams", type=int, default=0,
                    help="HIP streams the steps alternate over (1: serial; 0 = 2: an honest step's latency-bound "
                         "tail kernels, and a selfish launch's last engine waves, overlap the next step)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-runs", type=int, default=0, help="0 = auto (~15 s of CPU work)")
    ap.add_argument("--stub", action="store_true", help=argparse.SUPPRESS)  # tests: CPU stand-in, gloo
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        raise SystemExit(spawn_ranks(args.gpus, sys.argv[1:]))

    import contextlib

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.stub:
        dev = torch.device("cpu")
        if world > 1:
            dist.init_process_group("gloo")
        if os.environ.get("MSIM_BENCH_STUB_FAIL_RANK") == str(rank):  # tests: a rank dying mid-job
            raise SystemExit(3)
    else:
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
        if world > 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("nccl", device_id=dev)

    from miningsimulation_amd import PRESETS
    from miningsimulation_amd.simulation import PRESET_WEIGHTS

    miners = PRESETS[args.config]()
    m = len(miners)
    if args.stub:
        sim = _StubSim(m)
        stub_t = {"on": False, "t0": 0.0}

        def timing_enable(on):
            stub_t["on"] = on
            stub_t["t0"] = time.perf_counter()

        def timing_read():  # stand-in kernel spans: half of the wall clock since enable
            ms = 0.5 * (time.perf_counter() - stub_t["t0"]) * 1e3
            return {"launches": args.steps, "launch_ms": ms, "draws_ms": ms, "engine_ms": 0.0, "draws_busy_ms": ms,
                    "engine_busy_ms": 0.0, "launch_busy_ms": ms}

        def sync():
            pass

        def on_stream(st):
            return contextlib.nullcontext()
    else:
        from miningsimulation_amd import Simulation, timing_enable, timing_read

        sim = Simulation(miners, total_weight=PRESET_WEIGHTS.get(args.config, 100))

        def sync():
            torch.cuda.synchronize()

        def on_stream(st):
            return torch.cuda.stream(st)
    n = args.runs or {"c3": 131072, "c5": 65536}.get(args.config, 32768)
    # Consecutive steps are independent batches: they alternate over `--streams` HIP streams, each with its
    # own workspace and sums, so one step's latency-bound tail kernels (episodes, combine, finalize) and
    # all-reduce overlap the next step's draw kernel. Every step still runs to completion inside the timed
    # region (both sides bracketed by barrier + synchronize).
    # Two streams for every network (measured on MI355X: c2 7.4 -> 8.7 M in round 2; c3 2.29 -> 2.36 M in round 3,
    # profiles/r03/e1ab/c3_s*.json: the last waves of one E1 launch overlap the first of the next).
    ns = args.streams if args.streams > 0 else 2
    lanes = []
    for j in range(ns):
        st = None if args.stub else (torch.cuda.current_stream(dev) if ns == 1 else torch.cuda.Stream(dev))
        lanes.append({
            "stream": st,
            "ws": torch.empty(sim.workspace_bytes(n), dtype=torch.uint8, device=dev),
            "sums": torch.zeros((m, 6), dtype=torch.int64, device=dev),
            "total": torch.zeros((m, 6), dtype=torch.int64, device=dev),
            "status": torch.zeros(2, dtype=torch.int32, device=dev),
            "fails": torch.zeros(1, dtype=torch.int64, device=dev),
            "local": torch.zeros((m, 6), dtype=torch.int64, device=dev),  # this rank's own sums (before reduce)
        })
    sync()

    def step(i: int):
        begin = (i * world + rank) * n  # disjoint run ranges per step and rank -> fresh seeds
        ln = lanes[i % ns]
        with on_stream(ln["stream"]):
            sim.launch(n, begin, args.seed_base, ln["sums"], ln["ws"], ln["status"], stream=ln["stream"])
            ln["fails"].add_(ln["status"][1:2].to(torch.int64))
            if world > 1:
                ln["local"].add_(ln["sums"])
                dist.all_reduce(ln["sums"])  # the path's only exchange: per-miner integer sums (RCCL over xGMI)
            ln["total"].add_(ln["sums"])

    for i in range(args.warmup):
        step(i)
    sync()
    for ln in lanes:
        ln["total"].zero_()
        ln["fails"].zero_()
        ln["local"].zero_()
    timing_enable(True)  # HIP events on the launch stream around every launch and every K1
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i)
    sync()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    tm = timing_read()
    timing_enable(False)
    assert tm["launches"] == args.steps, tm
    kern_ms = tm["launch_ms"] / args.steps  # all kernels of one msim_launch (K1+K2+K3+finalize), per launch
    k1_ms = tm["draws_ms"] / args.steps     # K1 / W1 per launch (span of each launch's draw kernel)
    e1_ms = tm.get("engine_ms", 0.0) / args.steps  # E1 kernels (selfish networks)
    # busy = union of those spans over both streams / steps: the stage's share of each step's wall clock
    k1_busy = tm.get("draws_busy_ms", 0.0) / args.steps
    e1_busy = tm.get("engine_busy_ms", 0.0) / args.steps
    kern_busy = tm.get("launch_busy_ms", 0.0) / args.steps  # every kernel of a launch, union over the streams
    total = sum(ln["total"] for ln in lanes)
    fails = sum(ln["fails"] for ln in lanes)
    t = torch.tensor([elapsed, kern_ms, k1_ms, e1_ms, k1_busy, e1_busy, kern_busy], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(fails)
    elapsed, kern_ms, k1_ms, e1_ms, k1_busy, e1_busy, kern_busy = (float(x) for x in t)
    if int(fails.item()) != 0:
        raise SystemExit(f"{int(fails.item())} runs exceeded the compact state capacity")
    rccl = None
    if world > 1:
        # The exchange step, checked once outside the timed region: every rank's own (pre-reduce) found counts,
        # gathered, must add up to the all-reduced total each rank holds.
        local_found = sum(ln["local"] for ln in lanes)[:, 0].sum().reshape(1)
        gathered = [torch.zeros_like(local_found) for _ in range(world)]
        dist.all_gather(gathered, local_found)
        per_rank = [int(g.item()) for g in gathered]
        reduced = int(total[:, 0].sum().item())
        rccl = {"rccl_world": dist.get_world_size(), "backend": dist.get_backend(),
                "found_allreduced": reduced, "found_per_rank": per_rank, "ok": reduced == sum(per_rank)}
        if not rccl["ok"]:
            raise SystemExit(f"all-reduce check failed: {rccl}")

    pipe = sim.pipeline_info(n)
    ms_step = elapsed / args.steps * 1e3
    # Roofline of the dominant kernel: the draw kernel for honest networks (K1 / W1: it does every fast block's
    # whole work), E1 for selfish ones. Its time, dominant_ms, is its BUSY time per step: the union of its
    # launches' HIP-event spans over both streams in the timed region, divided by the steps (two launches in
    # flight on two streams count their overlap once), so it never exceeds ms_per_step. The same union per
    # call is in the committed rocprofv3 summary of this command (rocprof_<config>_s<0|1>.md, busy ms/call).
    # (A single launch's span is not reported: under two-stream overlap it exceeds ms_per_step.)
    honest = pipe.get("uses_pipeline") in (1, 2)
    if honest and k1_ms > 0:
        dom_ms = k1_busy
    elif e1_ms > 0:
        dom_ms = e1_busy
    else:
        dom_ms = min(kern_busy if kern_busy > 0 else kern_ms, ms_step)
    pmc = None if args.stub else pmc_constants(args.config, n)
    rp_here = rocprof_kernel_ms(args.config, ns)  # this command's summary (default streams or --streams 1)
    rp_serial = rocprof_kernel_ms(args.config, 1)
    peak = VALU_PEAK_LANE_OPS
    work = n * BLOCKS_PER_RUN_YEAR * w_blk(m)  # SURVEY 8(d) convention, lane-ops per launch
    roof = {
        "bound": "valu",
        "unit": "T lane-op/s",
        "peak": round(peak / 1e12, 2),
        "peak_source": "MI355X_MICROARCH.md: 256 CU x 4 SIMD-32 x 2.4 GHz (a wave64 VALU op issues over 2 cycles)",
        "kernel": ("W1 msim_wide_draws_kernel" if sim.wide else "K1 msim_draws_kernel" if honest else
                   "E1 msim_sel_kernel (settled form + entity engine)"),
        "dominant_ms": round(dom_ms, 4),
        "dominant_ms_how": "busy time per step: union of the kernel's HIP-event spans over the streams / steps",
        "dominant_ms_file": rp_here["file"] if rp_here else None,
        "dominant_ms_file_busy": rp_here["busy_ms"] if rp_here else None,
    }
    if pmc and dom_ms > 0:
        # headline: the counter-based VALU issue fraction, SQ_INSTS_VALU x 64 lanes over the kernel's busy time
        achieved = pmc["valu"] * 64 / (dom_ms / 1e3)
        roof.update({
            "achieved": round(achieved / 1e12, 4),
            "frac": round(achieved / peak, 4),
            "frac_how": f"SQ_INSTS_VALU {pmc['valu']:.5g} per launch ({pmc['src']}) x 64 / dominant_ms / peak",
            "traffic": round(pmc["fetch_kb"] * 1024 * 2 + pmc["write_kb"] * 1024),
            "traffic_source": f"rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE of {pmc['kernel']} per launch ({pmc['src']})",
            "valu_per_block": round(pmc["valu"] * 64 / (n * BLOCKS_PER_RUN_YEAR), 2),
        })
        if rp_serial:
            roof.update({
                "frac_serial": round(pmc["valu"] * 64 / (rp_serial["avg_ms"] / 1e3) / peak, 4),
                "frac_serial_how": f"same counter over the kernel alone: avg ms in {rp_serial['file']} (--streams 1)",
            })
    else:
        roof.update({"achieved": None, "frac": None, "traffic": None,
                     "frac_how": "no PMC file for this config / run count (profiles/r05/final/pmc)"})
    # SURVEY 8(d)'s fixed accounting (156 lane-ops per block at M = 9): saturated, because K1 skips the state
    # machine for >99.9 % of blocks; kept for continuity, never the headline.
    roof["frac_convention_per_step"] = round(work / (ms_step / 1e3) / peak, 4)
    roof["saturated"] = roof["frac_convention_per_step"] >= 0.95
    if rp_serial:
        roof["frac_convention_serial"] = round(work / (rp_serial["avg_ms"] / 1e3) / peak, 4)
    roof["accounting"] = f"SURVEY 8(d): W_blk({m}) = {w_blk(m)} lane-ops/block x 52594.92 blocks/run-year"
    roof["kernels_busy_ms"] = round(kern_busy, 4)  # all kernels of a step, union over the streams (<= ms_per_step)
    roof["pipeline"] = pipe
    runs_total = args.steps * n * world
    value = runs_total / elapsed
    # sanity: aggregate share of miner 0 (integer sums, exact across ranks)
    tot = total.cpu().tolist()
    share0 = (tot[0][2] + tot[0][3] * 2.0**-32) / (runs_total) * 100

    if rank == 0:
        line = {
            "metric": "simulated run-years/sec (whole node) at 1/2/4/8 MI355X; % of VALU peak",
            "value": round(value, 1),
            "unit": "run-years/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int64+fp64",
            "data": "synthetic (seeded runs; run r uses rd()-equivalents (base+2r, base+2r+1))",
            "config": {
                "workload": {"c1": "c1: BASELINE configs[0] (10 s propagation)", "c2": "c2: BASELINE configs[1]",
                             "c3": "c3: BASELINE configs[2]",
                             "c5": "c5: BASELINE configs[4] (SURVEY Appendix C weights, W=102400)"}.get(args.config, args.config),
                "network": ([[mm.id, mm.perc, mm.propagation_ms, int(mm.is_selfish)] for mm in miners] if m <= 16 else
                            f"{m} miners: weights 30720, 29696, 1024 x 41 (W=102400), all honest, prop 1000 ms"),
                "runs_per_gpu_per_step": n,
                "duration": "months{12} = 31556952000 ms",
                "parallelism": f"runs sharded over {world} GPU(s), RCCL all-reduce of per-miner integer sums; "
                               f"steps alternate over {ns} HIP stream(s)",
                "miner0_share_pct": round(share0, 5),
            },
            "roofline": roof,
        }
        if rccl:
            line["rccl"] = rccl
        if args.stub:
            line["data"] = "STUB (--stub: CPU stand-in for the launch, tests of the rank/JSON plumbing only)"
        if world == 1 and not args.no_cpu_baseline and not args.stub:
            threads, visible, how = host_threads()
            line["cpu_baseline"] = cpu_baseline(args.config, args.cpu_sample_runs, threads, visible)
            line["cpu_baseline"]["cores_note"] = how
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
