"""Latency of one small bsg_hasher_sum batch, the shape split::Writer.Close hashes (≈ 252 tree
nodes of ≈ 10.7 KB for a 4 GiB stream): one packed host buffer, k_sha_blobs path. Prints the
per-call time of 20 calls on a warm hasher (ms). HS_LONG=<bytes> makes the first blob that long
(a Writer's geometric node sizes: 1 GiB's 63 nodes of ~11 KB hold one of ~50 KB)."""
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
    lens = np.full(n, size, dtype=np.uint64)
    lens[0] = int(os.environ.get("HS_LONG", str(size)))
    off = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    base = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8)
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
    import hashlib
    ok = all(bytes(refs[32 * i:32 * i + 32]) == hashlib.sha256(base[int(off[i]):int(off[i] + lens[i])].tobytes()).digest()
             for i in range(n))
    print(json.dumps({"blobs": n, "bytes_each": size, "first": int(lens[0]), "ok": ok, "ms": times}))


if __name__ == "__main__":
    main()
