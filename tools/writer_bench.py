"""The drop-in Writer surface vs the raw streaming C ABI, from host memory (PCIe-inclusive).

  raw     bsg_write of 32 MiB pieces + bsg_drain (records only; the caller keeps the bytes)
  writer  the C++ split.Writer (bs_split.hpp) -> store/mem, same pieces: every chunk stored,
          the tree built and its nodes stored, Root computed (split/split.go:44-126)

One SplitMix64 stream (default 4 GiB, WRITER_MIB), default params. The Writer's streaming
context comes from the process pool after the first ("cold") run, as in a server ingesting
many files. Prints one JSON line per variant/run.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bs_amd import bsgpu  # noqa: E402
from bs_amd.synth import splitmix_array  # noqa: E402


def thp() -> str:
    try:
        return open("/sys/kernel/mm/transparent_hugepage/enabled").read().strip()
    except OSError:
        return "n/a"


def main():
    n = int(os.environ.get("WRITER_MIB", "4096")) << 20
    piece = 32 << 20
    data = splitmix_array(0xB5B52026, n)
    mv = memoryview(data)
    print(json.dumps({"thp": thp(), "bytes": n, "piece": piece}), flush=True)
    w = bsgpu.StreamingSplitter()
    best = None
    for rep in range(3):
        w.reset()
        t0 = time.perf_counter()
        nch = 0
        for i in range(0, n, piece):
            w.write(mv[i:i + piece])
            nch += len(w.drain())
        w.close()
        nch += len(w.drain())
        dt = time.perf_counter() - t0
        if rep and (best is None or dt < best):
            best = dt
    w.free()
    raw = n / best / 2**30
    print(json.dumps({"variant": "raw bsg_write/bsg_drain", "chunks": nch,
                      "gib_per_s": round(raw, 3)}), flush=True)
    roots = set()
    for run in ("cold", "warm", "warm"):
        st = bsgpu.MemStore()
        t0 = time.perf_counter()
        wr = bsgpu.Writer(st)
        for i in range(0, n, piece):
            wr.write(mv[i:i + piece])
        wr.close()
        dt = time.perf_counter() - t0
        roots.add(wr.root)
        nblobs = len(st)
        wr.free()
        t1 = time.perf_counter()
        st.free()
        tfree = time.perf_counter() - t1
        print(json.dumps({"variant": "C++ split.Writer -> store/mem", "run": run, "blobs": nblobs,
                          "seconds": round(dt, 4), "gib_per_s": round(n / dt / 2**30, 3),
                          "vs_raw": round((n / dt / 2**30) / raw, 3),
                          "store_free_s": round(tfree, 4)}), flush=True)
    assert len(roots) == 1


if __name__ == "__main__":
    main()
