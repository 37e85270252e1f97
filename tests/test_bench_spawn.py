"""bench.py --gpus N starts its own N ranks (one process per GPU, 127.0.0.1 rendezvous) when no launcher
set WORLD_SIZE, and rank 0 prints the single JSON line of the whole job. Driven on CPU with --stub (gloo
stand-in for the launch; the real path uses RCCL): the spawn, barrier, max-over-ranks and reduction
plumbing is the same code."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--stub", "--no-cpu-baseline", *args],
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_spawn_two_ranks_one_line():
    d = _bench("--gpus", "2", "--steps", "3", "--warmup", "1")
    assert d["n_gpus"] == 2
    assert d["steps"] == 3
    assert d["scaling"] == "weak"
    assert d["value"] > 0
    assert d["data"].startswith("STUB")
    # whole-job aggregate: 2 ranks x 3 steps x 32768 runs over the max-over-ranks time
    assert abs(d["value"] * d["ms_per_step"] * 3 / 1e3 - 2 * 3 * 32768) < 1e-3 * 2 * 3 * 32768
    _check_rccl(d, 2)


def _check_rccl(d, n):
    """The line shows the collective saw every rank: world size, and the all-reduced found count equals the
    sum of each rank's own counts gathered once outside the timed region."""
    r = d["rccl"]
    assert r["rccl_world"] == n
    assert r["ok"] is True
    assert len(r["found_per_rank"]) == n
    assert r["found_allreduced"] == sum(r["found_per_rank"])
    assert all(v > 0 for v in r["found_per_rank"])


def test_single_rank_unchanged():
    d = _bench("--gpus", "1", "--steps", "2", "--warmup", "0")
    assert d["n_gpus"] == 1
    assert "cpu_baseline" not in d
    assert "rccl" not in d
    # no time in the roofline exceeds the step (the dominant kernel's busy time is a share of the step)
    roof = d["roofline"]
    assert roof["dominant_ms"] <= d["ms_per_step"] + 1e-9
    assert roof["kernels_busy_ms"] <= d["ms_per_step"] + 1e-9
    assert not any(k.endswith("span_ms") for k in roof)


def test_spawn_eight_ranks():
    """The driver's 8-GPU node: eight ranks, one JSON line, the aggregate over all of them."""
    d = _bench("--gpus", "8", "--steps", "2", "--warmup", "1")
    assert d["n_gpus"] == 8
    assert abs(d["value"] * d["ms_per_step"] * 2 / 1e3 - 8 * 2 * 32768) < 1e-3 * 8 * 2 * 32768
    _check_rccl(d, 8)


def test_spawn_failing_rank_ends_job():
    """A rank that dies (here: rank 1 of 4, before its collectives) ends the job quickly with a non-zero exit
    and no JSON line, instead of leaving rank 0 waiting in a collective."""
    import time

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["MSIM_BENCH_STUB_FAIL_RANK"] = "1"
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--stub", "--no-cpu-baseline", "--gpus", "4",
                        "--steps", "2", "--warmup", "0"], capture_output=True, text=True, timeout=240, env=env,
                       cwd=ROOT)
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert "rank 1 exited" in r.stderr, r.stderr[-2000:]
    assert time.monotonic() - t0 < 120
