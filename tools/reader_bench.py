"""The read side: split.Reader over a store/mem tree, with and without the
batched GPU verification of every fetched chunk (BSG_READER_VERIFY), and the stream's chunks
hashed as a batch of blobs, from host memory (bsg_hasher_sum_ptrs) and device-resident
(bsg_engine_hash). One SplitMix64 stream (default 1 GiB, READER_MIB) written by the C++
split.Writer with default params; reads of 1 MiB until EOF. Prints one JSON line per case.
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bs_amd import bsgpu  # noqa: E402
from bs_amd.synth import splitmix_array  # noqa: E402


def read_all(r, piece):
    n = 0
    while True:
        b = r.read(piece)
        if not b:
            return n
        n += len(b)


def main():
    n = int(os.environ.get("READER_MIB", "1024")) << 20
    data = splitmix_array(0xB5B52026, n)
    st = bsgpu.MemStore()
    w = bsgpu.Writer(st)
    mv = memoryview(data)
    for i in range(0, n, 32 << 20):
        w.write(mv[i:i + (32 << 20)])
    w.close()
    root = w.root
    w.free()
    print(json.dumps({"bytes": n, "blobs": len(st)}), flush=True)
    for verify in (False, True, False, True):
        r = bsgpu.Reader(st, root, verify=verify)
        t0 = time.perf_counter()
        got = read_all(r, 1 << 20)
        dt = time.perf_counter() - t0
        assert got == n, (got, n)
        print(json.dumps({"case": "split.Reader read_all", "verify": verify,
                          "seconds": round(dt, 4), "gib_per_s": round(n / dt / 2**30, 3)}),
              flush=True)
    st.free()
    # the stream's chunks as a batch of blobs (Blob.Ref of many blobs, bs.go:24-26)
    ch, _ = bsgpu.split_hash_batch([data])
    offs = ch["offset"].astype(np.uint64)
    lens = ch["len"].astype(np.uint64)
    want = [bytes(r) for r in ch["ref"]]
    # (1) from host memory, scattered blobs (bsg_hasher_sum_ptrs: packed into pinned staging,
    #     one H2D, bsg_engine_hash mode), pointers straight into the stream buffer
    h = bsgpu.Hasher()
    ptrs = (ctypes.c_void_p * len(ch))(*[data.ctypes.data + int(o) for o in offs])
    refs = np.zeros(32 * len(ch), dtype=np.uint8)
    for rep in range(3):
        t0 = time.perf_counter()
        rc = bsgpu.lib().bsg_hasher_sum_ptrs(h.h, ptrs, lens.ctypes.data_as(
            ctypes.POINTER(ctypes.c_uint64)), len(ch), refs.ctypes.data)
        dt = time.perf_counter() - t0
        assert rc == 0 and refs[:32].tobytes() == want[0] and refs[-32:].tobytes() == want[-1]
        print(json.dumps({"case": "bsg_hasher_sum_ptrs (host blobs, H2D included)",
                          "blobs": len(ch), "run": rep, "seconds": round(dt, 4),
                          "gib_per_s": round(n / dt / 2**30, 3)}), flush=True)
    h.free()
    # (2) device-resident: the blobs at 16-byte offsets in HBM, bsg_engine_hash + finish
    aoff = np.zeros(len(ch), dtype=np.uint64)
    o = 0
    for i, ln in enumerate(lens):
        aoff[i] = o
        o = (o + int(ln) + 15) & ~15
    host = np.zeros(o, dtype=np.uint8)
    for i in range(len(ch)):
        host[int(aoff[i]):int(aoff[i]) + int(lens[i])] = data[int(offs[i]):int(offs[i]) + int(lens[i])]
    buf = bsgpu.DeviceBuffer(host.size)
    buf.from_host(host)
    eng = bsgpu.Engine()
    for rep in range(4):
        bsgpu.synchronize(0)
        t0 = time.perf_counter()
        eng.hash(buf.ptr, aoff, lens)
        eng.finish()
        dt = time.perf_counter() - t0
        if rep:
            got = eng.chunks()
            assert bytes(got["ref"][0]) == want[0] and bytes(got["ref"][-1]) == want[-1]
            print(json.dumps({"case": "bsg_engine_hash (device-resident blobs)", "blobs": len(ch),
                              "seconds": round(dt, 4), "gib_per_s": round(n / dt / 2**30, 3),
                              "sha_path": eng.diag().get("long")}), flush=True)
    eng.close()
    # (3) the same device-resident blobs, one blob per lane (k_sha_blobs: bsg_hasher_sum's path
    #     for device memory and small batches; the Reader's only path before round 2's end)
    h = bsgpu.Hasher()
    for rep in range(3):
        t0 = time.perf_counter()
        rc = bsgpu.lib().bsg_hasher_sum(h.h, buf.ptr, aoff.ctypes.data_as(
            ctypes.POINTER(ctypes.c_uint64)), lens.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
            len(ch), refs.ctypes.data)
        dt = time.perf_counter() - t0
        assert rc == 0 and refs[:32].tobytes() == want[0] and refs[-32:].tobytes() == want[-1]
        if rep:
            print(json.dumps({"case": "k_sha_blobs (device-resident blobs, one per lane)",
                              "blobs": len(ch), "seconds": round(dt, 4),
                              "gib_per_s": round(n / dt / 2**30, 3)}), flush=True)
    h.free()
    buf.free()


if __name__ == "__main__":
    main()
