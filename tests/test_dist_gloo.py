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
    bench.check_world(world, w)                 # --gpus N == WORLD_SIZE passes
    try:
        bench.check_world(world + 1, w)         # a mismatch must stop the bench
        raise AssertionError("check_world accepted a wrong --gpus")
    except SystemExit:
        pass
    lib = bench.build_once(w, local)            # rank 0 builds (if stale), the others wait
    assert os.path.exists(lib)
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


def _racer(out, q):
    import sys
    import time
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    from bs_amd import build

    def compile_to(tmp):
        time.sleep(0.3)  # a slow compiler: the racers overlap
        with open(tmp, "w") as f:
            f.write(f"built by {os.getpid()}")

    q.put(build.build_locked(out, lambda: not os.path.exists(out), compile_to))


def test_concurrent_builders_compile_once(tmp_path):
    """Four processes start a build of the same stale library at once: exactly one compiles,
    the rest wait on the lock and find the finished file; no temporary file is left behind."""
    out = str(tmp_path / "lib.so")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_racer, args=(out, q)) for _ in range(4)]
    for p in procs:
        p.start()
    compiled = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert compiled.count(True) == 1
    assert open(out).read().startswith("built by ")
    assert sorted(os.listdir(tmp_path)) == ["lib.so", "lib.so.lock"]


def test_bench_refuses_wrong_gpu_count():
    """`python bench.py --gpus 2` without torch.distributed.run exits non-zero at once (before
    any GPU call), instead of timing one GPU and reporting it as the 2-GPU number."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2"],
                       capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode != 0
    assert "WORLD_SIZE=1" in r.stderr
