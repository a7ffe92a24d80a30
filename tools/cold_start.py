"""Cold-start cost of the streaming Writer: time bsg_open + Write + Close for small streams,
first in the process and then again (python tools/cold_start.py)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bs_amd import bsgpu  # noqa: E402


def one(n, data):
    t0 = time.perf_counter()
    s = bsgpu.StreamingSplitter()
    t1 = time.perf_counter()
    s.write(data[:n])
    t2 = time.perf_counter()
    s.close()
    recs = s.drain() if hasattr(s, "drain") else None
    t3 = time.perf_counter()
    return t1 - t0, t2 - t1, t3 - t2, (len(recs) if recs is not None else -1)


def one_writer(n, data):
    t0 = time.perf_counter()
    st = bsgpu.MemStore()
    w = bsgpu.Writer(st)
    t1 = time.perf_counter()
    w.write(data[:n])
    root = w.close()
    t2 = time.perf_counter()
    return t1 - t0, t2 - t1, len(st)


def main():
    data = np.random.default_rng(1).integers(0, 256, 64 << 20, dtype=np.uint8)
    bsgpu.lib()
    for n in (1 << 20, 10 << 20, 64 << 20):
        for rep in range(3):
            o, w, c, k = one(n, data)
            print(f"{n >> 20:3d} MiB rep {rep}: open {o * 1e3:7.1f} ms  write {w * 1e3:7.1f} ms  "
                  f"close+drain {c * 1e3:7.1f} ms  chunks {k}", flush=True)
    for n in (1 << 20, 10 << 20, 64 << 20):
        for rep in range(3):
            o, t, k = one_writer(n, data)
            print(f"Writer {n >> 20:3d} MiB rep {rep}: new {o * 1e3:7.1f} ms  write+close "
                  f"{t * 1e3:7.1f} ms  blobs {k}", flush=True)


if __name__ == "__main__":
    main()
