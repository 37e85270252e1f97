"""The N>1 path on CPU: world-size-2 gloo process group, runs sharded by index, one SUM all-reduce of the
integer sums. The per-run values come from the oracle (CPU); the test checks that sharded + all-reduced
sums equal the single-process sums bit for bit, for even and ragged partitions."""
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


def _worker(rank, world, port, n_total, out_q):
    import torch.distributed as dist

    from miningsimulation_amd.distributed import allreduce_sums, shard, sums_rows_from_runs
    from oracle import pyoracle

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    begin, n = shard(n_total, world, rank)
    if n:
        f, s, sh, r = pyoracle.run_batch(PERCS, PROPS, SELF, D, n, begin, 1000, threads=2)
        rows = sums_rows_from_runs(f, s, sh, r)
    else:
        rows = [[0] * 6 for _ in PERCS]
    glob = allreduce_sums(rows)
    out_q.put((rank, glob))
    dist.destroy_process_group()


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


@pytest.mark.parametrize("n_total", [24, 13])
def test_gloo_world2_allreduce_matches_single_process(oracle, n_total):
    from miningsimulation_amd.distributed import sums_rows_from_runs

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n_total, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    f, s, sh, r = oracle.run_batch(PERCS, PROPS, SELF, D, n_total, 0, 1000, threads=4)
    want = sums_rows_from_runs(f, s, sh, r)
    assert res[0] == want and res[1] == want
    # and the fixed-point means agree with the f64 run-order means (main.cpp:211-217) to 1e-9
    for k in range(len(PERCS)):
        share = want[k][2] + want[k][3] * 2.0**-32
        assert abs(share - float(np.sum(sh[:, k]))) < 1e-9 * max(1.0, share) + n_total * 2.0**-33
