"""The N>1 path on CPU: world-size-2 gloo process group, runs sharded by index, one SUM all-reduce of the
integer sums. The ranks drive the product's multi-GPU entry point, distributed.run_sharded (partition,
chunked launches, status reduction, all-reduce), with the device launch replaced by one that computes the
shard's per-run values with the oracle (there is no GPU here); the sharded + all-reduced sums must equal
the single-process sums bit for bit, for even and ragged partitions."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

D = 10**9
PERCS = [40, 19, 12, 11, 8, 5, 3, 1, 1]
PROPS = [1000] * 9
SELF = [True] + [False] * 8


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _OracleSim:
    """Stands in for Simulation on a CPU rank: miners + a launch with msim_launch's signature whose sums
    come from the oracle (per-run values -> fixed-point rows, as the device kernels sum them)."""

    miners = PERCS

    def __init__(self, fail_rank=None):
        self.fail_rank = fail_rank

    def launch(self, n, begin, seed_base, sums, ws, status, stream=None):
        import torch
        import torch.distributed as dist

        from miningsimulation_amd.distributed import sums_rows_from_runs
        from oracle import pyoracle

        assert ws is None
        f, s, sh, r = pyoracle.run_batch(PERCS, PROPS, SELF, D, n, begin, seed_base, threads=2)
        sums.copy_(torch.tensor(sums_rows_from_runs(f, s, sh, r), dtype=torch.int64))
        status.zero_()
        if self.fail_rank is not None and dist.get_rank() == self.fail_rank:
            status[1] = 1  # a run that failed even on the retry kernel


def _worker(rank, world, port, n_total, out_q, fail_rank=None):
    import torch
    import torch.distributed as dist

    from miningsimulation_amd.distributed import run_sharded

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sim = _OracleSim(fail_rank)
    try:
        glob = run_sharded(sim, n_total, 1000, launch=sim.launch, device=torch.device("cpu")).tolist()
    except RuntimeError as e:
        glob = str(e)
    out_q.put((rank, glob))
    dist.destroy_process_group()


def _spawn(n_total, fail_rank=None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n_total, q, fail_rank)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def test_shard_partition():
    from miningsimulation_amd.distributed import shard

    for n in (0, 1, 7, 64, 1000):
        for w in (1, 2, 3, 8):
            parts = [shard(n, w, r) for r in range(w)]
            assert sum(c for _, c in parts) == n
            pos = 0
            for b, c in parts:
                assert b == pos
                pos += c


@pytest.mark.parametrize("n_total", [24, 13, 1])
def test_gloo_world2_run_sharded_matches_single_process(oracle, n_total):
    from miningsimulation_amd.distributed import sums_rows_from_runs

    res = _spawn(n_total)
    f, s, sh, r = oracle.run_batch(PERCS, PROPS, SELF, D, n_total, 0, 1000, threads=4)
    want = sums_rows_from_runs(f, s, sh, r)
    assert res[0] == want and res[1] == want
    # and the fixed-point means agree with the f64 run-order means (main.cpp:211-217) to 1e-9
    for k in range(len(PERCS)):
        share = want[k][2] + want[k][3] * 2.0**-32
        assert abs(share - float(np.sum(sh[:, k]))) < 1e-9 * max(1.0, share) + n_total * 2.0**-33


def test_gloo_world2_failed_run_is_reported_on_every_rank():
    """A run that failed on one rank (status[1]) is all-reduced, so every rank raises, not just that one."""
    res = _spawn(8, fail_rank=1)
    assert all(isinstance(v, str) and "exceeded" in v for v in res.values()), res
