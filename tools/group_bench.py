"""Experiment: a many-stream batch (configs[2]: 256 x 64 MiB) split into G groups, each group
on its own engine (HIP stream), all enqueued before any is waited on, so the scan/select of
later groups overlaps the SHA-256 of earlier ones. Prints GiB/s per G."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bs_amd import bsgpu  # noqa: E402

ns, mib = int(os.environ.get("NS", "256")), int(os.environ.get("MIB", "64"))
nbytes = mib << 20
stride = (nbytes + 15) & ~15
buf = bsgpu.DeviceBuffer(stride * ns)
offs = [i * stride for i in range(ns)]
lens = [nbytes] * ns
engs = [bsgpu.Engine() for _ in range(4)]
for i in range(ns):
    bsgpu.fill_splitmix(buf.ptr + offs[i], nbytes, 0xB5B52026 + i, stream=engs[0].stream)
bsgpu.synchronize(0)
for G in [int(x) for x in os.environ.get("GROUPS", "1,2,3,4").split(",")]:
    bounds = [round(ns * g / G) for g in range(G + 1)]
    def step():
        for g in range(G):
            a, b = bounds[g], bounds[g + 1]
            engs[g].run(buf.ptr, offs[a:b], lens[a:b])
        tot = 0
        for g in range(G):
            tot += engs[g].finish()
        return tot
    for _ in range(2):
        step()
    bsgpu.synchronize(0)
    t0 = time.perf_counter()
    K = 5
    for _ in range(K):
        n = step()
    bsgpu.synchronize(0)
    dt = (time.perf_counter() - t0) / K
    print(json.dumps({"groups": G, "ms_per_step": round(dt * 1e3, 3), "chunks": n,
                      "gib_per_s": round(ns * nbytes / dt / 2**30, 1)}), flush=True)
