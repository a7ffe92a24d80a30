#!/usr/bin/env python3
"""bench.py — BASELINE.json metric: "GiB/s device-resident split+ref-hash; chunk/ref bit-parity
vs Go ref".

Workload (BASELINE.json configs[1], and configs[3] when launched on 8 GPUs): one 1 GiB random
byte stream per GPU (SplitMix64 counter stream generated in HBM, seed 0xB5B52026 + rank),
split.NewWriter defaults (Bits 16, MinSize 1024). A step = one full pass of the hot path over
that stream: rolling-hash scan -> MinSize boundary selection -> SHA-256 of every chunk, with the
(offset, len, level, ref) records left in HBM. Streams are independent: no collectives on the
data path (weak scaling); torch.distributed is used only for the barrier and the max-over-ranks
timing.

The default N=1 run then times configs[2] (256 x 64 MiB streams on the same GPU: the many-blob
path, the largest single-GPU config) the same way, after freeing the configs[1] buffers, and
reports it as the nested "configs2" record of the same JSON line (its own value, ms_per_step,
stage times, roofline and 16-thread CPU baseline). The headline value stays configs[1].

  python bench.py [--gpus N] [--steps K] [--warmup W]
  (N>1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
METRIC = "GiB/s device-resident split+ref-hash; chunk/ref bit-parity vs Go ref"
BASE_SEED = 0xB5B52026


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--stream-mib", type=int, default=1024, help="bytes per stream (MiB)")
    ap.add_argument("--streams", type=int, default=1, help="independent streams per GPU")
    ap.add_argument("--bits", type=int, default=16)
    ap.add_argument("--min-size", type=int, default=1024)
    ap.add_argument("--cpu-sample-mib", type=int, default=1024,
                    help="bytes the CPU oracle baseline splits+hashes: a prefix of stream 0 for "
                         "one stream, else whole streams (at least one per thread) (0: skip)")
    ap.add_argument("--e2e-mib", type=int, default=1024,
                    help="bytes of host-memory stream for the PCIe-inclusive streaming rate "
                         "(bsg_write -> records in host memory; 0: skip)")
    ap.add_argument("--no-writer-e2e", dest="writer_e2e", action="store_false",
                    help="skip the split.Writer -> store/mem leg (same host stream as --e2e-mib)")
    ap.add_argument("--configs2-steps", type=int, default=None,
                    help="timed steps of the nested configs[2] record (256 x 64 MiB on the same "
                         "GPU, N=1 default run only; default: --steps, 0: skip)")
    ap.add_argument("--check", action="store_true",
                    help="also verify the records against the oracle on bytes generated on the "
                         "host (checks the device fill too); the default run already checks them "
                         "against the oracle on the device bytes (the CPU baseline's sample)")
    a = ap.parse_args()
    if a.configs2_steps is None:
        a.configs2_steps = a.steps
    return a


def dist_setup():
    """One process per GPU. Ranks only exchange a barrier and one float (max elapsed time), so
    the process group is gloo over 127.0.0.1: the data path has no collective, and torch's own
    (bundled) HIP runtime is never initialised next to libbsgpu's."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("BSG_BENCH_SHARE_GPU") == "1":
        # rehearsal of the N>1 path on a one-GPU box: every rank drives device 0 (never for
        # reported numbers; the driver launches one rank per GPU)
        local = 0
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(backend="gloo")
    return world, rank, local


def check_world(gpus: int, world: int) -> None:
    """--gpus N must match the launch: N ranks under torch.distributed.run, one per GPU.
    A plain `python bench.py --gpus 8` would otherwise time one GPU and report it as n_gpus 1."""
    if gpus != world:
        raise SystemExit(
            f"bench.py: --gpus {gpus} but WORLD_SIZE={world}; launch one rank per GPU: "
            f"python -m torch.distributed.run --nnodes=1 --nproc-per-node {gpus} "
            f"--master-addr 127.0.0.1 --master-port P bench.py --gpus {gpus} ...")


def build_once(world: int, local: int) -> str:
    """Local rank 0 builds libbsgpu.so if it is stale (normally a no-op: the tree ships the
    built library), the other ranks wait at a barrier and then only load it. The build itself
    is also flock-serialised (bs_amd/build.py), so even concurrent builders compile once."""
    from bs_amd import build
    if local == 0:
        build.build()
    barrier(world)
    return build.build()  # fresh after the barrier: returns the path without compiling


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def max_over_ranks(x: float, world: int) -> float:
    if world == 1:
        return x
    import torch
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def timed_steps(step, sync, world: int, steps: int, warmup: int) -> float:
    """W untimed warmups, then exactly K steps between barrier+sync brackets; max over ranks."""
    for _ in range(warmup):
        step()
    sync()
    barrier(world)
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    barrier(world)
    t1 = time.perf_counter()
    return max_over_ranks(t1 - t0, world)


def cpu_threads() -> int:
    """Host threads for the multi-stream CPU baseline: the GPU box's CPU share (16 per GPU,
    OMP_NUM_THREADS), not os.cpu_count(), which shows the whole machine there."""
    return max(1, min(int(os.environ.get("OMP_NUM_THREADS", "16")), os.cpu_count() or 1))


def cpu_baseline(host_streams: list, bits: int, min_size: int, sample: str, base=None):
    """The C oracle ("port" of the reference's per-stream Splitter + sha256: literal per-byte
    buzhash32 loop, SHA-256 with the x86 SHA extensions when the host has them, as Go's amd64
    crypto/sha256 does) over a bounded sample of the same bytes on this host. One stream per
    thread, as the reference runs one goroutine per stream: 1 thread for a single stream,
    cpu_threads() for a batch. It is NOT Go's split.Writer: the per-byte loop is a tight C
    register loop (oracle/bsoracle.c), likely faster than hashsplit's append + Roll per byte, so
    the stated CPU rate is an optimistic stand-in for the reference (Go is absent here and on
    the GPU box). Returns (baseline record, the oracle's chunks of the sample): the chunks are
    the parity check of the device records on the same bytes."""
    if not host_streams:
        return None, None
    import numpy as np
    from oracle import oracle as O  # checker / baseline only
    table = O.buzhash32_table(1)
    impl = O.sha256_use(True)
    n = sum(len(a) for a in host_streams)
    if len(host_streams) == 1:
        threads = 1
        t0 = time.perf_counter()
        ch = O.split(table, host_streams[0], bits=bits, min_size=min_size)
        dt = time.perf_counter() - t0
        nch = len(ch)
    else:
        threads = min(cpu_threads(), len(host_streams))
        lens = [len(a) for a in host_streams]
        if base is None:
            base = np.concatenate(host_streams)
            off = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
        else:  # the streams are views of `base`
            off = np.array([a.ctypes.data - base.ctypes.data for a in host_streams], np.uint64)
        t0 = time.perf_counter()
        ch, _ = O.split_streams(table, base, off, lens, bits=bits, min_size=min_size,
                                threads=threads)
        dt = time.perf_counter() - t0
        nch = len(ch)
    full = cpu_full_writer(O, table, host_streams, bits, min_size, threads)
    return ({"value": round(n / dt / 2**30, 4), "unit": "GiB/s", "cores": threads, "kind": "port",
             "sample": f"{sample} (same bytes/params), C oracle split + sha256 ({impl}), "
                       f"{threads} thread(s), one stream per thread, {nch} chunks in {dt:.2f}s",
             "loop": "tight C restatement of hashsplit's per-byte loop, not Go's Splitter",
             "full_writer": full}, ch)


def cpu_full_writer(O, table, host_streams: list, bits: int, min_size: int, threads: int) -> dict:
    """SURVEY §8(d)'s "full" CPU variant: split.Writer end to end (oracle bso_writer_root:
    Splitter + sha256 + TreeBuilder + PutProto of every node, each blob copied as store/mem's
    Put keeps Go's appended chunk) over the same sample, one stream per thread (ctypes drops the
    GIL, so the threads run the C code in parallel)."""
    from concurrent.futures import ThreadPoolExecutor
    n = sum(len(a) for a in host_streams)
    t0 = time.perf_counter()
    with ThreadPoolExecutor(max_workers=threads) as ex:
        res = list(ex.map(lambda a: O.writer_root(table, a, bits=bits, min_size=min_size,
                                                  fanout=8, keep_copies=True), host_streams))
    dt = time.perf_counter() - t0
    return {"value": round(n / dt / 2**30, 4), "unit": "GiB/s", "cores": threads,
            "kind": "port", "puts": sum(p for _, p in res),
            "sample": f"same sample, split.Writer -> store/mem restated in C, Fanout 8, "
                      f"{dt:.2f}s"}


def chain_roofline(diag: dict) -> dict | None:
    """k_sha's real bound: the longest chunk's serial SHA-256 chain, run by a skewed octet on an
    early chain (k_early, sha256_oct_solo_loop.inc). Its loop issues 557 instructions per 64-round
    block (66 iterations of 8 VALU: 64 rounds + the skew's fill and drain; 16 ds_read_b128 of
    K+W; 4 cndmask, 4 feed-forward adds, 2 waits, 3 loop control), and a lone wave issues one
    every 4.0 cycles (tools/ubench/oct_pmc under rocprofv3: SQ_ACTIVE_INST_ANY per counted
    instruction, profiles/r06_oct_pmc.json). Floors: that issue count x 4 (the loop as built),
    and 64 rounds x 8 VALU x 4 (the octet formulation with no fill, drain or K+W reads).
    achieved = the in-kernel s_memtime cycles per block of the longest job."""
    try:
        cyc = float(diag["long"]["cycles_per_block"])
    except (KeyError, TypeError, ValueError):
        return None
    if cyc <= 0:
        return None
    loop = 557
    floor = loop * 4.0
    formulation = 64 * 8 * 4.0
    return {"bound": "issue (serial chain, lone wave: 4 cycles per instruction)",
            "kernel": "k_early / k_sha wave mode (skewed octet)",
            "loop_instructions_per_block": loop, "floor_cycles_per_block": floor,
            "formulation_floor_cycles_per_block": formulation,
            "achieved_cycles_per_block": round(cyc, 1), "frac": round(floor / cyc, 4),
            "frac_of_formulation": round(formulation / cyc, 4),
            "pmc_src": "profiles/r06_oct_pmc.json", "blocks": diag["long"].get("blocks")}


def host_placement() -> dict:
    """The process's CPU placement on the host: the CPUs it may run on and their NUMA nodes
    (the GPU's node and the pinned stages' nodes come from bsg_stream_stats)."""
    import glob
    cpus = sorted(os.sched_getaffinity(0))
    node_of = {}
    for d in glob.glob("/sys/devices/system/node/node[0-9]*"):
        try:
            text = open(os.path.join(d, "cpulist")).read().strip()
        except OSError:
            continue
        k = int(os.path.basename(d)[4:])
        for part in filter(None, text.split(",")):
            lo, _, hi = part.partition("-")
            for c in range(int(lo), int(hi or lo) + 1):
                node_of[c] = k
    by_node = {}
    for c in cpus:
        by_node[node_of.get(c, -1)] = by_node.get(node_of.get(c, -1), 0) + 1
    return {"cpus_allowed": len(cpus), "cpus_by_node": {str(k): v for k, v in sorted(by_node.items())},
            "nodes": len(set(node_of.values())) or None}


def end_to_end(mib: int, bits: int, min_size: int, device: int) -> dict | None:
    """The streaming path from host memory: bsg_write of 32 MiB pieces (copy into a ring of
    pinned stages, each copied H2D into its 256 MiB device tile as it fills, three tiles in
    flight) -> split + SHA-256 -> records D2H -> bsg_drain. Best of 3 after one warm-up on the
    same context (bsg_reset). Every rep records where its time went (bsg_stream_stats: the host
    copies into pinned staging, the H2D copies timed by HIP events on the copy stream, the NUMA
    nodes of the GPU, the stages, the source and the copying threads)."""
    if mib <= 0:
        return None
    from bs_amd import bsgpu
    from bs_amd.synth import splitmix_array
    n = mib << 20
    data = splitmix_array(BASE_SEED, n)
    mv = memoryview(data)
    piece = 32 << 20
    w = bsgpu.StreamingSplitter(bits=bits, min_size=min_size, device=device)
    best, nch, recs, reps, rep_stats = None, 0, [], [], []
    import gc
    gc.collect()
    gc.disable()  # no cyclic-GC pass inside a timed rep (host-side noise, not the library's)
    try:
        for rep in range(4):  # rep 0 grows the pinned staging; best of the other three
            w.reset()
            recs = []
            t0 = time.perf_counter()
            for i in range(0, n, piece):
                w.write(mv[i:i + piece])
                recs.append(w.drain())
            tw = time.perf_counter() - t0
            w.close()
            recs.append(w.drain())
            dt = time.perf_counter() - t0
            reps.append([round(dt * 1e3, 2), round(tw * 1e3, 2)])
            rep_stats.append(w.stats())  # after the timed region
            if rep and (best is None or dt < best):
                best = dt
    finally:
        gc.enable()
    w.free()
    import numpy as np
    last = np.concatenate(recs)  # the last rep's records: checked against the oracle in main()
    nch = len(last)
    return {"value": round(n / best / 2**30, 3), "unit": "GiB/s", "bytes": n, "chunks": nch,
            "records": last,
            "reps_ms": reps,  # [whole rep, of which the Write calls] per rep, rep 0 = warm-up
            "reps_breakdown": rep_stats,
            "host": host_placement(),
            "path": "host memory -> bsg_write (ring of 4 x 64 MiB pinned stages, each copied "
                    "H2D as it fills, on a copy stream into 4 device data slots) -> split + "
                    "SHA-256 on 3 engines -> records in host memory; tile 256 MiB"}


def writer_e2e(mib: int, bits: int, min_size: int, device: int) -> dict | None:
    """The drop-in surface itself (split/split.go:44-126 -> store/mem/mem.go:62-76): the C++
    split::Writer -> MemStore over the same host-memory stream in 32 MiB Writes; every chunk Put
    (aliasing the Write pieces, as store/mem keeps the caller's slice), the tree built with its
    nodes hashed on the GPU and Put, Root computed. A fresh store per rep, the Writer's context
    from the process pool (a server ingesting many files); rep 0 is the warm-up, best of the
    other three. The Root is checked against the C oracle's split.Writer restatement after
    timing (main())."""
    if mib <= 0:
        return None
    from bs_amd import bsgpu
    from bs_amd.synth import splitmix_array
    n = mib << 20
    data = splitmix_array(BASE_SEED, n)
    mv = memoryview(data)
    piece = 32 << 20
    best, reps, roots, blobs = None, [], set(), 0
    import gc
    gc.collect()
    gc.disable()
    try:
        for rep in range(4):
            st = bsgpu.MemStore(device)
            t0 = time.perf_counter()
            w = bsgpu.Writer(st, bits=bits, min_size=min_size, fanout=8, device=device)
            for i in range(0, n, piece):
                w.write(mv[i:i + piece])
            tw = time.perf_counter() - t0
            w.close()
            dt = time.perf_counter() - t0
            roots.add(w.root)
            tm = w.timings()
            blobs = len(st)
            w.free()
            st.free()  # outside the timed region
            reps.append({"ms": round(dt * 1e3, 2), "write_ms": round(tw * 1e3, 2), **tm})
            if rep and (best is None or dt < best):
                best = dt
    finally:
        gc.enable()
    return {"value": round(n / best / 2**30, 3), "unit": "GiB/s", "bytes": n, "blobs": blobs,
            "root": roots.pop().hex() if len(roots) == 1 else None, "data": data,
            "reps": reps,  # rep 0 = warm-up; times in ms (bsg_writer_timings)
            "path": "host memory -> C++ split::Writer (32 MiB Writes) -> chunks Put into "
                    "store/mem, tree nodes hashed on the GPU and Put, Root"}


# rocprofv3 names of each stage's kernels (k_sha: two instantiations launched back to back, one of
# which returns at once; the stage's bytes are their sum)
KERNEL_NAMES = {"k_scan": ("void bsg::k_scan<true>(bsg::ScanArgs)",
                           "void bsg::k_scan<false>(bsg::ScanArgs)"),
                "k_sha": ("void bsg::k_sha<true>(bsg::ShaArgs)",
                          "void bsg::k_sha<false>(bsg::ShaArgs)",
                          "bsg::k_sha(bsg::ShaArgs)")}  # (one kernel before the split)


def same_workload(doc_w: str, workload: str) -> bool:
    """A PMC summary belongs to this line's workload: the same BASELINE config ("configs[k]"
    before the colon), or the same name exactly. Empty or generic names never match."""
    if not doc_w or not workload:
        return False
    if doc_w.startswith("configs[") and workload.startswith("configs["):
        return doc_w.split(":", 1)[0] == workload.split(":", 1)[0]
    return doc_w == workload


def pmc_traffic(kernel: str, workload: str):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary for this workload
    (profiles/rNN_pmc.json, written by tools/pmc_summary.py from rocprofv3 FETCH_SIZE and
    WRITE_SIZE passes, gfx950 correction applied there). None if no summary matches."""
    import glob
    names = KERNEL_NAMES.get(kernel, ())
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc.json")), reverse=True):
        if path.endswith("_valu_pmc.json"):  # SQ counter summaries (work_roofline), no bytes
            continue
        try:
            with open(path) as f:
                doc = json.load(f)
        except (OSError, ValueError):
            continue
        if not same_workload(doc.get("workload") or "", workload):
            continue
        ks = [doc.get("kernels", {}).get(n) for n in names]
        ks = [k for k in ks if k and "hbm_bytes_per_launch" in k]
        if ks:
            return int(sum(k["hbm_bytes_per_launch"] for k in ks)), os.path.relpath(path, ROOT)
    return None, None


CONFIGS1 = "configs[1]: 1 GiB random stream per GPU, default split params"
CONFIGS2 = "configs[2]: 256 x 64 MiB streams per GPU"
STAGES = ["k_scan", "k_compact+k_select+k_chunks+prefix", "k_sha"]
STAGE_SRC = ("HIP events on the engine's stream: k_sha (the roofline's kernel) over the timed "
             "steps; k_scan and selection over the warmup steps after the first (their two "
             "extra events per step are left out of the timed region)")


def workload_name(ns: int, nbytes: int, bits: int, min_size: int) -> str:
    if bits == 16 and min_size == 1024 and ns == 1 and nbytes == 1 << 30:
        return CONFIGS1
    if bits == 16 and min_size == 1024 and ns == 256 and nbytes == 64 << 20:
        return CONFIGS2
    return f"{ns} x {nbytes >> 20} MiB streams per GPU"


def device_leg(ns: int, nbytes: int, bits: int, min_size: int, steps: int, warmup: int,
               world: int, rank: int, local: int, cpu_sample: int, check: bool) -> dict:
    """One device-resident workload: ns streams of nbytes generated in HBM, W warmups, K timed
    steps (each a full scan -> select -> SHA-256 pass, records left in HBM), then the CPU
    baseline over a bounded sample of the same bytes. Frees its device memory before returning."""
    from bs_amd import bsgpu
    stride = (nbytes + 15) & ~15
    buf = bsgpu.DeviceBuffer(stride * ns, device=local)
    eng = bsgpu.Engine(device=local)
    offs = [i * stride for i in range(ns)]
    lens = [nbytes] * ns
    for i in range(ns):  # stream s of rank r uses seed BASE + r*ns + s
        bsgpu.fill_splitmix(buf.ptr + offs[i], nbytes, BASE_SEED + rank * ns + i,
                            stream=eng.stream, device=local)
    # Stage times come from HIP events on the engine's stream, and every event costs the step
    # time (≈ 0.05 ms for four on configs[1], tools/profile_cost.py): the warmup steps time all
    # three stages, the timed steps only the SHA-256 stage (the dominant kernel, two events).
    stage_sum = [0.0, 0.0, 0.0]
    nsteps = [0, 0]  # warmup steps with all stages timed (the first, cold, left out), timed steps

    def step(warm=False):
        eng.run(buf.ptr, offs, lens, bits=bits, min_size=min_size)
        eng.finish()  # waits on the engine's stream; records stay in HBM
        ms = eng.stage_ms()
        if warm:
            for i in range(2):
                stage_sum[i] += ms[i]
            nsteps[0] += 1
        else:
            stage_sum[2] += ms[2]
            nsteps[1] += 1

    def sync():
        bsgpu.synchronize(local)

    # Between two steps the GPU idles while the host wakes from finish() and enqueues the next
    # run (tools/step_gaps.py, profiles/r05_step_gaps.txt): finish() polls its stream by the
    # library's default (BSG_KNOB_POLL), and the Python GC stays off for the steps (harness
    # noise: a GC pass in the step loop, not library work).
    import gc
    gc.collect()
    gc.disable()
    try:
        eng.profile(1)
        for w in range(warmup):
            step(warm=w > 0 or warmup == 1)
        eng.profile(2)
        elapsed = timed_steps(step, sync, world, steps, 0)
    finally:
        gc.enable()
    stage_avg = [stage_sum[0] / max(nsteps[0], 1), stage_sum[1] / max(nsteps[0], 1),
                 stage_sum[2] / max(nsteps[1], 1)]
    if nsteps[0] == 0:  # no warmup: the scan and selection stages were not timed
        stage_avg[0] = stage_avg[1] = 0.0
    diag = eng.diag()
    chunks = int(eng.nchunks)
    # the last timed step's records, copied to the host after timing: checked below against
    # the oracle on the same device bytes (the metric's "chunk/ref bit-parity" half)
    dev_ch = eng.chunks()
    dev_counts = eng.counts() if ns > 1 else None
    gen_ok = None
    if check and rank == 0:  # --check: also against bytes generated on the host (checks the fill)
        from bs_amd.synth import splitmix_array
        from oracle import oracle as O  # checker only, after timing
        ref = O.split(O.buzhash32_table(1), splitmix_array(BASE_SEED, nbytes), bits=bits,
                      min_size=min_size)
        got = dev_ch[: len(ref)] if ns == 1 else dev_ch[: int(dev_counts[0])]
        gen_ok = bool(len(got) == len(ref) and (got["ref"] == ref["ref"]).all()
                      and (got["offset"] == ref["offset"]).all())
    # the CPU baseline's sample: the same device bytes, copied back after timing. A batch is
    # copied back whole: the baseline is timed on its first streams, the parity check below
    # covers every stream of it.
    host_streams, sample, full_prefix, host_all = [], "", True, None
    if rank == 0 and world == 1 and cpu_sample > 0:
        want = cpu_sample << 20
        if ns == 1:
            host_streams = [buf.to_host(0, min(nbytes, want))]
            full_prefix = len(host_streams[0]) == nbytes
            sample = f"first {len(host_streams[0]) >> 20} MiB of stream 0"
        else:
            k = min(ns, max(4 * cpu_threads(), -(-want // nbytes)))
            host_all = buf.to_host(0, offs[-1] + nbytes)
            host_streams = [host_all[offs[i]:offs[i] + nbytes] for i in range(k)]
            sample = f"streams 0..{k - 1} of {ns} ({k} x {nbytes >> 20} MiB)"
    check_streams = []
    if world > 1 and ns == 1:  # N>1: every rank checks its own stream (no CPU baseline there)
        check_streams = [buf.to_host(0, nbytes)]
    # the engine and its input are done with: free them before the next leg
    eng.close()
    buf.free()
    cpu, ref_ch = cpu_baseline(host_streams, bits, min_size, sample,
                               base=host_all[:offs[len(host_streams) - 1] + nbytes]
                               if host_all is not None else None)
    del host_streams
    ok, checked = None, ""
    if host_all is not None:  # every stream of the batch against the oracle, 16 threads
        from oracle import oracle as O  # checker only, after timing
        t0 = time.perf_counter()
        ref_all, _ = O.split_streams(O.buzhash32_table(1), host_all, offs, lens, bits=bits,
                                     min_size=min_size, threads=cpu_threads())
        ok = records_match(dev_ch, dev_counts, ref_all, ns, True)
        checked = (f"streams 0..{ns - 1} of {ns} ({ns} x {nbytes >> 20} MiB), "
                   f"{len(ref_all)} records, oracle {time.perf_counter() - t0:.1f}s")
        del ref_all
        host_all = None
    elif ref_ch is not None:
        ok = records_match(dev_ch, dev_counts, ref_ch, ns, full_prefix)
        checked = sample
    elif check_streams:
        from oracle import oracle as O  # checker only, after timing
        ref_ch = O.split(O.buzhash32_table(1), check_streams[0], bits=bits, min_size=min_size)
        ok = records_match(dev_ch, None, ref_ch, 1, True)
        checked = f"rank {rank}'s whole stream"
    del check_streams
    if world > 1 and ok is not None:  # all ranks' checks
        ok = max_over_ranks(0.0 if ok else 1.0, world) == 0.0
        checked = "every rank's whole stream"
    if gen_ok is not None:
        ok = gen_ok if ok is None else (ok and gen_ok)
    return {"elapsed": elapsed, "stage_avg": stage_avg, "diag": diag, "chunks": chunks,
            "check": ok, "checked": checked, "cpu": cpu,
            "ref": ref_ch if (ns == 1 and full_prefix) else None}


def records_match(dev, dev_counts, ref, ns: int, full: bool) -> bool:
    """Device records == the oracle's, bit for bit (offset, len, level, stream, ref). ns == 1:
    the oracle split a prefix of the stream (full: the whole stream; else its last chunk is the
    prefix's forced final one and is not compared). ns > 1: the oracle split whole streams
    0..k-1, which are the first counts[0..k) device records."""
    import numpy as np
    if ns == 1:
        n = len(ref) if full else len(ref) - 1
        if (full and len(dev) != n) or len(dev) < n:
            return False
        d, r = dev[:n], ref[:n]
    else:
        k = len(np.unique(ref["stream"])) if len(ref) else 0
        n = int(dev_counts[:k].sum())
        if n != len(ref):
            return False
        d, r = dev[:n], ref
    return all(bool((d[f] == r[f]).all()) for f in ("offset", "len", "level", "stream", "ref"))


def pmc_valu(workload: str):
    """Per-launch SQ counters of the SHA-256 stage's kernels from the newest committed VALU PMC
    summary for this workload (profiles/rNN*_valu_pmc.json, tools/valu_pmc.py)."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_valu_pmc.json")), reverse=True):
        try:
            with open(path) as f:
                doc = json.load(f)
        except (OSError, ValueError):
            continue
        if same_workload(doc.get("workload") or "", workload):
            return doc.get("kernels", {}), os.path.relpath(path, ROOT)
    return None, None


def work_roofline(workload: str, sha_ms: float, diag: dict) -> dict | None:
    """The SHA-256 stage's second bound: its VALU work. achieved = the
    VALU wave-instructions one run of the stage issues (SQ_INSTS_VALU of k_sha<false>, k_sha<true>
    and k_early, from the committed PMC summary) / the stage's event-timed duration; peak = the
    chip's VALU issue rate, 256 CUs x 4 SIMDs x clock / 2 cycles per wave64 instruction
    (MI355X_MICROARCH.md: SIMD-32, a wave64 VALU op over 2 cycles) at the per-lane jobs' measured
    clock; beside it the rate this kernel's 3-input integer ops were measured to reach on one
    SIMD whatever the occupancy (4 cycles per wave instruction)."""
    ks, src = pmc_valu(workload)
    if not ks or sha_ms <= 0:
        return None
    names = ("void bsg::k_sha<false>(bsg::ShaArgs)", "void bsg::k_sha<true>(bsg::ShaArgs)",
             "bsg::k_early(bsg::ShaArgs, unsigned int)")
    insts = sum(float(ks[n]["SQ_INSTS_VALU"]) for n in names if n in ks)
    if insts <= 0:
        return None
    clk = float((diag.get("lane") or {}).get("clock_ghz") or 2.4)
    rate = insts / (sha_ms * 1e-3)
    peak = 256 * 4 * clk * 1e9 / 2
    peak4 = 256 * 4 * clk * 1e9 / 4
    return {"bound": "VALU issue (per-lane SHA-256 work)", "kernel": "k_sha + k_early",
            "valu_wave_insts_per_run": insts, "achieved": round(rate / 1e12, 4),
            "peak": round(peak / 1e12, 4), "unit": "T wave-instructions/s",
            "frac": round(rate / peak, 4), "clock_ghz": clk,
            "peak_3input_measured": round(peak4 / 1e12, 4),
            "frac_of_3input_measured": round(rate / peak4, 4), "src": src}


def roofline(workload: str, per_launch_bytes: int, stage_avg: list, bound: str = "hbm") -> dict:
    """The dominant kernel's algorithmic bytes per launch / its event-timed duration, against
    the 8 TB/s HBM peak; k_scan beside it. traffic = HBM bytes per launch from the newest
    committed PMC summary of the same workload (profiles/rNN*_pmc.json)."""
    dom = max(range(3), key=lambda i: stage_avg[i])
    achieved = per_launch_bytes / (stage_avg[dom] * 1e-3) / 1e9 if stage_avg[dom] > 0 else 0.0
    scan_gbs = per_launch_bytes / (stage_avg[0] * 1e-3) / 1e9 if stage_avg[0] > 0 else 0.0
    traffic, traffic_src = pmc_traffic(STAGES[dom], workload)
    scan_traffic, _ = pmc_traffic("k_scan", workload)
    # the SHA-256 stage runs from k_sha's launch to the end of k_early_fix, which waits for the
    # early chains (k_early, second stream, started during selection)
    kernel = "k_sha (+ the early chains' tail)" if STAGES[dom] == "k_sha" else STAGES[dom]
    return {"bound": bound, "roof": "hbm", "kernel": kernel,
            "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
            "traffic_unit": "bytes/launch", "traffic_src": traffic_src,
            "algorithmic_bytes": per_launch_bytes,
            "limiter": "longest chunk's serial SHA-256 chain (issue latency)",
            "k_scan": {"achieved": round(scan_gbs, 1), "frac": round(scan_gbs / HBM_PEAK_GBS, 4),
                       "traffic": scan_traffic}}


def main():
    args = parse()
    world, rank, local = dist_setup()
    check_world(args.gpus, world)
    from bs_amd import bsgpu

    build_once(world, local)
    assert bsgpu.device_count() > local, "bench.py needs a GPU (the HIP path is the product)"
    # bsg_init up front, as a server does at start-up (include/bsgpu.h): the device, the pooled
    # streams and the pinned stage ring are set up before the legs' own large host allocations.
    # Without it the host-memory legs varied from rep to rep (the final tile 8.3-12.8 ms, the
    # Writer's copies 24 against 17 ms per GiB; profiles/r06_c4_legs_*.log). BSG_BENCH_INIT=0
    # skips it (A/B).
    init = os.environ.get("BSG_BENCH_INIT", "1") != "0"
    if init:
        bsgpu.init(local)
    nbytes = args.stream_mib << 20
    ns = args.streams
    leg = device_leg(ns, nbytes, args.bits, args.min_size, args.steps, args.warmup, world, rank,
                     local, args.cpu_sample_mib, args.check)
    elapsed, stage_avg = leg["elapsed"], leg["stage_avg"]
    total_bytes = world * ns * nbytes * args.steps
    value = total_bytes / elapsed / 2**30
    workload = workload_name(ns, nbytes, args.bits, args.min_size)
    # configs[2] (the largest single-GPU config, the many-blob path) on the same GPU, timed the
    # same way, as a nested record; the headline stays configs[1]
    c2 = None
    if (rank == 0 and world == 1 and workload == CONFIGS1 and args.configs2_steps > 0):
        n2, ns2 = 64 << 20, 256
        leg2 = device_leg(ns2, n2, 16, 1024, args.configs2_steps, args.warmup, 1, 0, local,
                          args.cpu_sample_mib, False)
        c2 = {"workload": CONFIGS2,
              "oracle_check": leg2["check"], "oracle_checked": leg2["checked"],
              "value": round(ns2 * n2 * args.configs2_steps / leg2["elapsed"] / 2**30, 3),
              "unit": "GiB/s", "steps": args.configs2_steps, "warmup": args.warmup,
              "ms_per_step": round(leg2["elapsed"] * 1e3 / args.configs2_steps, 3),
              "stage_ms": {n: round(v, 4) for n, v in zip(STAGES, leg2["stage_avg"])},
              "stage_ms_src": STAGE_SRC,
              "chunks_per_step": leg2["chunks"],
              "roofline": roofline(CONFIGS2, ns2 * n2, leg2["stage_avg"],
                                   "serial SHA-256 chain + per-lane VALU work (HBM frac reported)"),
              "work_roofline": work_roofline(CONFIGS2, leg2["stage_avg"][2], leg2["diag"]),
              "cpu_baseline": leg2["cpu"], "sha_path": leg2["diag"],
              "chain_roofline": chain_roofline(leg2["diag"])}
    e2e = end_to_end(args.e2e_mib, args.bits, args.min_size, local) \
        if (rank == 0 and world == 1) else None
    wr = writer_e2e(args.e2e_mib, args.bits, args.min_size, local) \
        if (rank == 0 and world == 1 and args.writer_e2e) else None
    if wr is not None:  # Root against the C oracle's split.Writer restatement, after timing
        from oracle import oracle as O  # checker only
        data = wr.pop("data")
        ref_root, _ = O.writer_root(O.buzhash32_table(1), data, bits=args.bits,
                                    min_size=args.min_size, fanout=8)
        del data
        wr["root_check"] = wr["root"] == ref_root.hex()
        wr["bsg_init"] = init
    if e2e is not None:
        # the e2e stream is the same SplitMix64 stream as configs[1]'s (seed BASE_SEED): when the
        # device leg's oracle split covered that whole stream, the host-path records are checked
        # against it too (bsg_write -> records in host memory, bit for bit)
        e2e["bsg_init"] = init
        recs, ref = e2e.pop("records"), leg.get("ref")
        if ref is not None and e2e["bytes"] == nbytes:
            e2e["oracle_check"] = records_match(recs, None, ref, 1, True)
    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed * 1e3 / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic: SplitMix64 counter stream in HBM, seed 0xB5B52026+stream",
            "config": {"workload": workload,
                       "stream_bytes": nbytes, "streams_per_gpu": ns,
                       "split_bits": args.bits, "min_size": args.min_size, "fanout": 8,
                       "parallelism": "independent streams, one set per GPU, no collectives"},
            "roofline": roofline(workload, ns * nbytes, stage_avg,
                                 "serial SHA-256 chain (HBM frac reported)"),
            "cpu_baseline": leg["cpu"],
            "end_to_end": e2e,
            "writer_e2e": wr,
            "stage_ms": {n: round(v, 4) for n, v in zip(STAGES, stage_avg)},
            "stage_ms_src": STAGE_SRC,
            "chunks_per_step": leg["chunks"],
            "sha_path": leg["diag"],
            "chain_roofline": chain_roofline(leg["diag"]),
            "configs2": c2,
            # how the timed region was run: the library's defaults (no knob set by the bench),
            # bsg_init first unless BSG_BENCH_INIT=0, Python's cyclic GC off inside timed loops
            "host_settings": {"library_knobs": "defaults", "bsg_init": init,
                              "python_gc_in_timed_loops": "off"},
        }
        line["oracle_check"] = leg["check"]
        line["oracle_checked"] = leg["checked"]
        print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
