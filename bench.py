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
# `bench.py --config C --steps 2 --warmup 0 --streams 1` (scripts/gpu_pmc_r06.sh: FETCH_SIZE, WRITE_SIZE, the SQ
# issue/stall set, the VALU instruction mix and the VALU busy/lane set in separate passes; scripts/pmc_csv.py writes
# every counter as its mean per dispatch). PMC counters cannot be collected inside the timed process: these are the
# recorded values of the same kernel, and every field computed from them names its file.
#   traffic = FETCH_SIZE x 2 (gfx950: FETCH_SIZE counts half the bytes of wide reads, MI355X_MICROARCH.md §HBM)
#             + WRITE_SIZE, bytes per launch;
#   valu    = SQ_INSTS_VALU (wave instructions) per launch: the counter-based VALU issue fraction is
#             valu x 64 lanes / the kernel's time / peak (every instruction priced at one full-rate issue slot);
#   cycles  = the same instructions priced by class: FP64 FMA/MUL/ADD and f64 conversions at half rate (the MI355X
#             FP64 vector peak, 78.6 TF, is half the FP32 one), 64-bit integer at half rate, FP64 transcendentals at
#             1/8, everything else full rate (2 cycles per wave64 instruction on a SIMD-32): frac_cycles is the share
#             of the SIMDs' cycles those issue costs fill;
#   lanes   = SQ_THREAD_CYCLES_VALU / (SQ_ACTIVE_INST_VALU x 64): the active share of a VALU instruction's 64 lanes
#             (rocprof's VALUUtilization; below 1 = divergence).
PMC_DIR = "profiles/r06/final/pmc"
PMC = {
    ("c1", 32768): {"kernel": "K1 msim_draws_kernel", "file": "pmc_c1.txt", "substr": "msim_draws_kernel"},
    ("c2", 32768): {"kernel": "K1 msim_draws_kernel", "file": "pmc_c2.txt", "substr": "msim_draws_kernel"},
    ("c3", 131072): {"kernel": "E1 msim_sel_kernel<9,1,1,4,1,4,true>", "file": "pmc_c3.txt", "substr": "msim_sel_kernel<"},
    ("c5", 65536): {"kernel": "W1 msim_wide_draws_kernel<4>", "file": "pmc_c5.txt", "substr": "msim_wide_draws_kernel"},
}
# issue cycles of one wave64 instruction per class on a SIMD-32 (see `cycles` above)
CYC_FULL, CYC_HALF, CYC_TRANS64 = 2.0, 4.0, 16.0
N_SIMD = 256 * 4
CLOCK_HZ = 2.4e9
# rocprofv3 --kernel-trace --stats summaries (scripts/rocprof_summary.py) of the exact bench commands: the default
# two streams (_s0) and --streams 1 (_s1). Their "busy ms/call" column is the union of the kernel's dispatch
# intervals per call, the file-backed counterpart of the live dominant_ms; the serial file's average is the
# kernel alone.
ROCPROF_DIR = "profiles/r06/final"
KERNEL_SUBSTR = {"c1": "msim_draws_kernel", "c2": "msim_draws_kernel", "c3": "msim_sel_kernel<",
                 "c5": "msim_wide_draws_kernel"}


# Second kernels worth reporting beside the dominant one (same files): c1's episode kernel K2, which takes about
# as long as K1 at configs[0]'s 1.7 % fork rate.
PMC_EXTRA = {
    ("c1", 32768): {"kernel": "K2 msim_episode_kernel<9,1>", "file": "pmc_c1.txt", "substr": "msim_episode_kernel<"},
}


def pmc_constants(config: str, n: int, table: dict | None = None) -> dict | None:
    """Per-launch PMC values of the config's profiled kernel from the committed file (None if absent)."""
    ent = (table or PMC).get((config, n))
    if not ent:
        return None
    path = os.path.join(PMC_DIR, ent["file"])
    try:
        txt = open(os.path.join(ROOT, path)).read()
    except OSError:
        return None
    # scripts/pmc_csv.py format: "<kernel>  dispatches=D  mean_ms=X  vgpr=..." then "    <COUNTER>  <per dispatch>"
    vals, cur, head = {}, False, ""
    for ln in txt.splitlines():
        if ln.startswith("#"):
            continue
        if not ln.startswith(" "):
            cur = ent["substr"] in ln and not vals
            if cur:
                head = ln
            continue
        parts = ln.split()
        if cur and len(parts) == 2:
            vals[parts[0]] = float(parts[1])
    need = ("FETCH_SIZE", "WRITE_SIZE", "SQ_INSTS_VALU")
    if not all(k in vals for k in need):
        return None
    out = {"kernel": ent["kernel"], "src": path, "fetch_kb": vals["FETCH_SIZE"], "write_kb": vals["WRITE_SIZE"],
           "valu": vals["SQ_INSTS_VALU"], "counters": vals}
    for tok in head.split():
        if tok.startswith("mean_ms="):
            out["profiled_mean_ms"] = float(tok.split("=")[1])
    mix = ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_CVT",
           "SQ_INSTS_VALU_INT64", "SQ_INSTS_VALU_TRANS_F64")
    if all(k in vals for k in mix):
        half = sum(vals[k] for k in mix[:5])
        tr = vals["SQ_INSTS_VALU_TRANS_F64"]
        full = max(vals["SQ_INSTS_VALU"] - half - tr, 0.0)
        out["issue_cycles"] = (full * CYC_FULL + half * CYC_HALF + tr * CYC_TRANS64) / N_SIMD  # per SIMD per launch
        out["half_rate_share"] = (half + tr) / vals["SQ_INSTS_VALU"]
    if vals.get("SQ_ACTIVE_INST_VALU"):
        if "SQ_THREAD_CYCLES_VALU" in vals:
            out["valu_utilization"] = vals["SQ_THREAD_CYCLES_VALU"] / (vals["SQ_ACTIVE_INST_VALU"] * 64)
    if vals.get("GRBM_GUI_ACTIVE") and out.get("profiled_mean_ms"):
        out["profiled_clock_ghz"] = vals["GRBM_GUI_ACTIVE"] / 8 / (out["profiled_mean_ms"] * 1e-3) / 1e9
    if vals.get("SQ_WAVE_CYCLES") and vals.get("SQ_WAIT_INST_ANY") is not None:
        out["wait_inst_share"] = vals["SQ_WAIT_INST_ANY"] / vals["SQ_WAVE_CYCLES"]
        out["wait_any_share"] = vals.get("SQ_WAIT_ANY", 0.0) / vals["SQ_WAVE_CYCLES"]
    return out


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


# Calibration of the oracle port against the reference binary (port run-years/s / reference run-years/s on the
# same cores and config). The reference cannot be built in this image without a stand-in for a library feature
# libstdc++ 11 lacks (C++20 chrono operator<<), which this project's build rules exclude, so it is
# never built or timed here; the two measurements on record are:
#   8 threads: the survey container (8-vCPU Intel Xeon @ 2.1 GHz), c2 at 32 768 runs: reference 609 run-years/s
#              (BASELINE.md §2), port 352.1 (oracle_cli time c2 32768 8, 93.08 s) -> 0.578;
#   1 thread:  the round-5 review (Missing #2), c2: reference 65.4 vs port 42.2 -> 0.645.
# reference_equivalent = port / ratio; the job's threaded sample uses the 8-thread ratio, and the line carries
# the 1-thread ratio's figure beside it as the spread.
PORT_TO_REFERENCE = round(352.056 / 609.0, 4)
PORT_TO_REFERENCE_1T = round(42.2 / 65.4, 4)


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
        "port_to_reference_ratio_1thread": PORT_TO_REFERENCE_1T,
        "reference_equivalent": round(rec["run_years_per_s"] / PORT_TO_REFERENCE, 2),
        "reference_equivalent_spread": [round(rec["run_years_per_s"] / PORT_TO_REFERENCE_1T, 2),
                                        round(rec["run_years_per_s"] / PORT_TO_REFERENCE, 2)],
        "reference_equivalent_all_visible_cpus": round(per_thread * visible / PORT_TO_REFERENCE, 1),
        "calibration": "port/reference on c2: 0.578 at 8 threads (survey container, port 352.1 vs reference 609 "
                       "run-years/s, BASELINE.md §2) and 0.645 at 1 thread (round-5 review, port 42.2 vs reference "
                       "65.4); reference_equivalent = value / the 8-thread ratio, spread = value / each ratio. The "
                       "reference binary is not built here (DESIGN.md §5)",
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

    def set_concurrent_launches(self, n):
        pass

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
    sim.set_concurrent_launches(ns)  # the pipeline plans K1's grid for ns launches in flight (msim.h)
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

    def step(i: int, ln=None, s=None):
        begin = (i * world + rank) * n  # disjoint run ranges per step and rank -> fresh seeds
        ln = ln or lanes[i % ns]
        s = s or sim
        with on_stream(ln["stream"]):
            s.launch(n, begin, args.seed_base, ln["sums"], ln["ws"], ln["status"], stream=ln["stream"])
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

    # The single-job rate beside the headline: the same steps on ONE stream, each launch waiting for the previous
    # one (nothing overlaps), timed separately after the headline region with the same barrier + synchronize.
    serial = None
    if ns > 1:
        # the same job as a caller with one launch in flight runs it: a config planned for one launch
        # (msim_config_set_concurrent_launches(1), the library's default), its own workspace, one stream
        sim1 = sim if args.stub else Simulation(miners, total_weight=PRESET_WEIGHTS.get(args.config, 100))
        ln1 = dict(lanes[0])
        ln1["ws"] = torch.empty(sim1.workspace_bytes(n), dtype=torch.uint8, device=dev)
        ks = min(args.steps, 20)
        step(args.warmup + args.steps, ln1, sim1)  # untimed: uploads the config's tables
        sync()
        for ln in lanes:
            ln["fails"].zero_()
        if world > 1:
            dist.barrier()
        sync()
        t1 = time.perf_counter()
        for i in range(ks):
            step(args.warmup + args.steps + 1 + i, ln1, sim1)
        sync()
        if world > 1:
            dist.barrier()
        ts = torch.tensor([time.perf_counter() - t1], dtype=torch.float64, device=dev)
        sfails = lanes[0]["fails"].clone()
        if world > 1:
            dist.all_reduce(ts, op=dist.ReduceOp.MAX)
            dist.all_reduce(sfails)
        if int(sfails.item()) != 0:
            raise SystemExit(f"{int(sfails.item())} runs exceeded the compact state capacity (serial steps)")
        serial = {"value": round(ks * n * world / float(ts.item()), 1), "steps": ks,
                  "ms_per_step": round(float(ts.item()) / ks * 1e3, 3),
                  "how": "the same workload, one HIP stream, one step in flight at a time, the config planned for one "
                         "launch in flight (timed after the headline)"}

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
        if "issue_cycles" in pmc:
            roof.update({
                "frac_cycles": round(pmc["issue_cycles"] / (dom_ms / 1e3 * CLOCK_HZ), 4),
                "frac_cycles_how": f"SQ_INSTS_VALU by class ({pmc['src']}): FP64 FMA/MUL/ADD, CVT, INT64 at "
                                   f"{CYC_HALF:g} cycles, FP64 TRANS at {CYC_TRANS64:g}, the rest at {CYC_FULL:g} "
                                   f"per wave instruction, / {N_SIMD} SIMDs / (dominant_ms x 2.4 GHz)",
                "half_rate_share": round(pmc["half_rate_share"], 4),
            })
        for key in ("valu_utilization", "profiled_clock_ghz", "wait_inst_share", "wait_any_share"):
            if key in pmc:
                roof[key] = round(pmc[key], 4)
        if rp_serial:
            roof.update({
                "frac_serial": round(pmc["valu"] * 64 / (rp_serial["avg_ms"] / 1e3) / peak, 4),
                "frac_serial_how": f"same counter over the kernel alone: avg ms in {rp_serial['file']} (--streams 1)",
            })
            if "issue_cycles" in pmc:
                roof["frac_cycles_serial"] = round(pmc["issue_cycles"] / (rp_serial["avg_ms"] / 1e3 * CLOCK_HZ), 4)
    else:
        roof.update({"achieved": None, "frac": None, "traffic": None,
                     "frac_how": f"no PMC file for this config / run count / kernel ({PMC_DIR})"})
    extra = None if args.stub else pmc_constants(args.config, n, PMC_EXTRA)
    if extra:  # recorded, not timed live: its profiled mean duration and counters
        roof["second_kernel"] = {
            "kernel": extra["kernel"], "src": extra["src"], "profiled_mean_ms": extra.get("profiled_mean_ms"),
            "valu_utilization": round(extra.get("valu_utilization", 0.0), 4),
            "traffic": round(extra["fetch_kb"] * 1024 * 2 + extra["write_kb"] * 1024),
            "frac_cycles_profiled": (round(extra["issue_cycles"] / (extra["profiled_mean_ms"] / 1e3 * CLOCK_HZ), 4)
                                     if "issue_cycles" in extra and extra.get("profiled_mean_ms") else None)}
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
        if serial:
            line["serial_single_job"] = serial
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
