"""One streaming configuration of the e2e path, repeated, for a rocprofv3 kernel + memory-copy
trace read by tools/e2e_timeline.py (tools/gpu_e2e_trace.sh). Prints each rep's wall time and
write-phase time, so the trace's rep can be matched to its host-side numbers.
  E2E_MIB (1024), E2E_TILE_MIB (256), E2E_REPS (5)"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bs_amd import bsgpu  # noqa: E402
from bs_amd.synth import splitmix_array  # noqa: E402


def main():
    n = int(os.environ.get("E2E_MIB", "1024")) << 20
    tile = int(os.environ.get("E2E_TILE_MIB", "256")) << 20
    piece = 32 << 20
    data = splitmix_array(0xB5B52026, n)
    mv = memoryview(data)
    bsgpu.init(0)
    w = bsgpu.StreamingSplitter(tile=tile)
    clk = time.CLOCK_BOOTTIME if os.environ.get("E2E_CLOCK", "boot") == "boot" else time.CLOCK_MONOTONIC
    now = lambda: time.clock_gettime_ns(clk)  # noqa: E731  (the tracer's clock: host stamps line up)
    for rep in range(int(os.environ.get("E2E_REPS", "5"))):
        w.reset()
        t0 = time.perf_counter()
        stamps = [("start", now())]
        nch = 0
        for i in range(0, n, piece):
            w.write(mv[i:i + piece])
            stamps.append(("write", now()))
            nch += len(w.drain())
            stamps.append(("drain", now()))
        tw = time.perf_counter() - t0
        w.close()
        stamps.append(("close", now()))
        nch += len(w.drain())
        stamps.append(("end", now()))
        dt = time.perf_counter() - t0
        print(json.dumps({"rep": rep, "seconds": round(dt, 4), "write_phase_s": round(tw, 4),
                          "chunks": nch, "gib_per_s": round(n / dt / 2**30, 3),
                          "host_ns": stamps}), flush=True)
    w.free()


if __name__ == "__main__":
    main()
