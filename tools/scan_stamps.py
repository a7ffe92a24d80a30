"""Where k_scan's time goes, per phase (experiment; needs a BSG_SCAN_DIAG build via BSG_LIB_PATH,
tools/build_variants.sh "diag:-DBSG_SCAN_DIAG"). Every wave stamps s_memtime around its strip
set-up (the next strip's job), the history load and warm-up, the line loop, and the counts
store + refine-list append; the sums over all waves land in the Regions debug words after the run.
Prints cycles per strip iteration for each phase and its share, the workgroups' clock, and the
event-timed k_scan stage for configs[1] (1 x 1 GiB) and configs[2] (256 x 64 MiB)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bs_amd import bsgpu  # noqa: E402

REGIONS_BYTES = 8 * (8 + 256 + 257 + 7) + 4 * 256 * 256 + 8 * 8192
PHASES = ["prologue", "job", "history+warm-up", "line loop", "append"]


def run(ns: int, mib: int, reps: int = 4) -> None:
    n = mib << 20
    stride = (n + 15) & ~15
    buf = bsgpu.DeviceBuffer(stride * ns + 4096)
    eng = bsgpu.Engine()
    offs = [i * stride for i in range(ns)]
    for i in range(ns):
        bsgpu.fill_splitmix(buf.ptr + offs[i], n, 0xB5B52026 + i, stream=eng.stream)
    eng.profile(1)
    L = bsgpu.lib()
    L.bsg_engine_regions_debug.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
    acc = []
    for r in range(reps):
        eng.run(buf.ptr, offs, [n] * ns, bits=16, min_size=1024)
        eng.finish()
        ms = eng.stage_ms()
        raw = np.zeros(REGIONS_BYTES // 8, dtype=np.uint64)
        assert L.bsg_engine_regions_debug(eng.h, raw.ctypes.data, REGIONS_BYTES) == 0
        d = raw[-8192:].astype(np.float64)
        if r == 0:
            continue  # first run: cold clock
        waves, iters = d[7], d[6]
        wg = raw[-8192 + 16:-8192 + 16 + 4 * 2000].reshape(2000, 4).astype(np.int64)
        wg = wg[wg[:, 1] > 0]
        clk = np.median((wg[:, 1] - wg[:, 0]) / ((wg[:, 3] - wg[:, 2]) * 10.0))  # GHz
        per = d[:6] / iters
        per[0] = d[0] / waves  # the prologue: once per wave
        acc.append((ms[0], per, d[5] / waves, d[8], clk, iters / waves))
        if r == reps - 1:  # the workgroups' spans on the 100 MHz clock, from the first start
            t0 = wg[:, 2].min()
            st, en = (wg[:, 2] - t0) / 100.0, (wg[:, 3] - t0) / 100.0
            q = [0, 10, 50, 90, 99, 100]
            print(f"  last run, {len(wg)} workgroups: start us p{q} = "
                  f"{np.round(np.percentile(st, q), 1).tolist()}, end us = "
                  f"{np.round(np.percentile(en, q), 1).tolist()}")
            late = np.argsort(en)[-6:]
            print("  latest-ending workgroups (index, start, end us): " +
                  ", ".join(f"({i}, {st[i]:.1f}, {en[i]:.1f})" for i in late))
    print(f"== {ns} x {mib} MiB: k_scan+k_refine stage {np.mean([a[0] for a in acc]):.3f} ms "
          f"(event-timed), workgroup clock {np.mean([a[4] for a in acc]):.3f} GHz, "
          f"{np.mean([a[5] for a in acc]):.1f} strips per wave")
    per = np.mean([a[1] for a in acc], axis=0)
    tot = per[1:5].sum()
    for k, name in enumerate(PHASES):
        print(f"  {name:16s} {per[k]:9.0f} cycles " + ("per wave" if k == 0 else "per strip iteration")
              + (f"  {100 * per[k] / tot:5.1f} % of the strip" if k else ""))
    print(f"  wave life        {np.mean([a[2] for a in acc]):9.0f} cycles (max "
          f"{np.mean([a[3] for a in acc]):.0f})")
    eng.close()
    buf.free()


if __name__ == "__main__":
    run(1, 1024)
    run(256, 64)
