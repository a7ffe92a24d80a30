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
    # the bench's per-rank parity check and its reduction over ranks: both ranks see rank 1's
    # tampered record
    ok = bench.records_match(out["chunks"], None, O.split(table, data), 1, True)
    all_ok = bench.max_over_ranks(0.0 if ok else 1.0, w) == 0.0
    bad = out["chunks"].copy()
    if r == 1:
        bad["ref"][len(bad) // 2, 0] ^= 1
    ok_bad = bench.records_match(bad, None, O.split(table, data), 1, True)
    all_bad = bench.max_over_ranks(0.0 if ok_bad else 1.0, w) == 0.0
    assert ok and all_ok and not all_bad
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


def test_records_match_prefix_and_batch():
    """bench.records_match, the check behind the bench line's oracle_check: a single stream
    checked on a prefix (the oracle's forced last chunk is not compared), and a batch whose
    first k streams the oracle split whole."""
    import sys
    import numpy as np
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    from bs_amd.synth import splitmix_array
    from oracle import oracle as O
    table = O.buzhash32_table(1)
    d = splitmix_array(5, 3 << 20)
    full = O.split(table, d)
    assert bench.records_match(full, None, full, 1, True)
    pre = O.split(table, d[: 1 << 20])          # a prefix: its last chunk is forced
    assert bench.records_match(full, None, pre, 1, False)
    assert not bench.records_match(full, None, pre, 1, True)
    streams = [splitmix_array(9 + i, 300_000 + 7 * i) for i in range(4)]
    lens = [len(a) for a in streams]
    base = np.concatenate(streams)
    off = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    dev, counts = O.split_streams(table, base, off, lens, threads=2)
    ref, _ = O.split_streams(table, base[: int(off[2])], off[:2], lens[:2], threads=2)
    assert bench.records_match(dev, counts, ref, 4, True)
    dev2 = dev.copy()
    dev2["level"][1] += 1
    assert not bench.records_match(dev2, counts, ref, 4, True)
