"""Latency of one small bsg_hasher_sum batch, the shape split::Writer.Close hashes (≈ 252 tree
nodes of ≈ 10.7 KB for a 4 GiB stream): one packed host buffer, k_sha_blobs path. Prints the
per-call time of 20 calls on a warm hasher (ms)."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from bs_amd import bsgpu  # noqa: E402


def main():
    n, size = int(os.environ.get("HS_N", "252")), int(os.environ.get("HS_SIZE", "10700"))
    rng = np.random.default_rng(5)
    base = rng.integers(0, 256, n * size, dtype=np.uint8)
    off = np.arange(n, dtype=np.uint64) * size
    lens = np.full(n, size, dtype=np.uint64)
    refs = np.zeros(32 * n, dtype=np.uint8)
    bsgpu.init(0)
    h = bsgpu.Hasher()
    L = bsgpu.lib()
    u64p = ctypes.POINTER(ctypes.c_uint64)
    times = []
    for _ in range(20):
        t0 = time.perf_counter()
        rc = L.bsg_hasher_sum(h.h, base.ctypes.data, off.ctypes.data_as(u64p),
                              lens.ctypes.data_as(u64p), n, refs.ctypes.data)
        times.append(round((time.perf_counter() - t0) * 1e3, 3))
        assert rc == 0
    h.free()
    print(json.dumps({"blobs": n, "bytes_each": size, "ms": times}))


if __name__ == "__main__":
    main()
