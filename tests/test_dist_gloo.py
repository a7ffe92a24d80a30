"""bench.py's multi-GPU harness on CPU: world_size 2 over gloo (127.0.0.1).

Each rank owns independent streams (no data-path collective); ranks share only a barrier and a
max-reduction of the elapsed time. Here each rank's "step" is the CPU oracle over its own stream,
so the harness logic (barriers, max over ranks, per-rank seeds, aggregate bytes) is exercised
without a GPU.
"""
import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import time
    import bench
    from bs_amd.synth import splitmix_array
    from oracle import oracle as O
    w, r, local = bench.dist_setup()
    assert (w, r) == (world, rank)
    table = O.buzhash32_table(1)
    data = splitmix_array(bench.BASE_SEED + r, 1 << 20)  # rank r's own stream
    out = {}

    def step():
        if r == 1:
            time.sleep(0.05)  # make rank 1 the slow one: the max must reflect it
        out["chunks"] = O.split(table, data)

    elapsed = bench.timed_steps(step, lambda: None, w, steps=2, warmup=1)
    q.put((r, elapsed, len(out["chunks"]), int(out["chunks"]["len"].sum())))
    import torch.distributed as dist
    dist.destroy_process_group()


def test_two_rank_harness():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, e0, c0, b0), (r1, e1, c1, b1) = res
    assert e0 == pytest.approx(e1)          # both ranks report the max over ranks
    assert e0 >= 0.1                        # >= rank 1's two sleeps
    assert b0 == b1 == 1 << 20              # each rank split its whole stream
    assert c0 > 0 and c1 > 0
