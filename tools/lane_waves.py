"""Per-wave view of k_sha's per-lane mode on configs[2] (experiment; needs a BSG_LANE_DIAG build
via BSG_LIB_PATH): when each wave entered and left per-lane mode, how often it moved region,
how many block iterations it ran. Prints exit-time percentiles and the latest waves."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bs_amd import bsgpu  # noqa: E402

REGIONS_BYTES = 8 * (8 + 256 + 257 + 7) + 4 * 256 * 256 + 8 * 8192


def main():
    ns, mib = int(os.environ.get("STREAMS", "256")), int(os.environ.get("MIB", "64"))
    n = mib << 20
    stride = (n + 15) & ~15
    buf = bsgpu.DeviceBuffer(stride * ns + 4096)
    eng = bsgpu.Engine()
    offs = [i * stride for i in range(ns)]
    for i in range(ns):
        bsgpu.fill_splitmix(buf.ptr + offs[i], n, 0xB5B52026 + i, stream=eng.stream)
    for _ in range(2):
        eng.run(buf.ptr, offs, [n] * ns, bits=16, min_size=1024)
        eng.finish()
    L = bsgpu.lib()
    L.bsg_engine_regions_debug.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
    raw = np.zeros(REGIONS_BYTES // 8, dtype=np.uint64)
    rc = L.bsg_engine_regions_debug(eng.h, raw.ctypes.data, REGIONS_BYTES)
    assert rc == 0, rc
    t = np.zeros(4, dtype=np.uint64)
    L.bsg_engine_timeline(eng.h, t.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)))
    t0 = int(t[0])
    R = int(raw[0])
    off = raw[8 + 256: 8 + 256 + 257]
    w = raw[-8192:].reshape(1024, 8).astype(np.int64)
    ent = (w[:, 0] - t0) * 0.01  # us (100 MHz realtime)
    ext = (w[:, 1] - t0) * 0.01
    mv, it = w[:, 2], w[:, 3]
    print(f"R={R} jobs/region min {np.diff(off[:R + 1]).min()} max {np.diff(off[:R + 1]).max()}")
    print(f"timeline us: long_end {(int(t[2]) - t0) * 0.01:.0f} lane_end {(int(t[3]) - t0) * 0.01:.0f}")
    for name, v in (("entry", ent), ("exit", ext), ("moves", mv), ("iters", it)):
        q = np.percentile(v, [0, 10, 50, 90, 99, 100])
        print(f"{name:6s} " + " ".join(f"{x:9.1f}" for x in q))
    late = np.argsort(ext)[-12:]
    print("latest waves: id entry exit moves iters")
    for i in late:
        print(f"  {i:5d} {ent[i]:9.1f} {ext[i]:9.1f} {mv[i]:4d} {it[i]:6d}")
    tk = w[:, 4] > 0
    tend = (w[:, 6] - t0) * 0.01
    tstart = (w[:, 5] - t0) * 0.01
    kind = w[:, 7] >> 32
    nb = w[:, 7] & 0xffffffff
    print(f"ticket waves {tk.sum()}: latest ticket ends (wave, ticket, kind 0 solo 1 group 2 pair,"
          " start us, end us, longest job blocks, us per block)")
    for i in np.argsort(np.where(tk, tend, -1))[-16:]:
        print(f"  {i:5d} {w[i, 4] - 1:5d} {kind[i]} {tstart[i]:8.1f} {tend[i]:9.1f} {nb[i]:6d} "
              f"{(tend[i] - tstart[i]) / max(nb[i], 1):.3f}")
    for k, name in ((0, "solo"), (1, "group"), (2, "pair")):
        m = tk & (kind == k)
        if m.any():
            print(f"{name}: {m.sum()} tickets, end max {tend[m].max():.0f} us, us/block "
                  f"median {np.median((tend[m] - tstart[m]) / np.maximum(nb[m], 1)):.3f}")
    hist, edges = np.histogram(ext, bins=20)
    print("exit histogram (us):", " ".join(f"{int(e)}:{h}" for e, h in zip(edges[:-1], hist)))
    eng.close()
    buf.free()


if __name__ == "__main__":
    main()
