"""Where a split::Writer's time goes: 5 Writers of 4 GiB (32 MiB Writes) into store/mem with
BSG_DEBUG_WRITER=1 (each Writer prints copy / drain / node-hash / close times to stderr when it is
freed), with each rep's GiB/s on stdout.   python tools/writer_timing.py [MiB]"""
import json
import os
import sys
import time

os.environ.setdefault("BSG_DEBUG_WRITER", "1")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bs_amd import bsgpu  # noqa: E402
from bs_amd.synth import splitmix_array  # noqa: E402


def main():
    n = (int(sys.argv[1]) if len(sys.argv) > 1 else 4096) << 20
    data = splitmix_array(2, n)
    mv = memoryview(data)
    bsgpu.init(0)
    for rep in range(5):
        st = bsgpu.MemStore()
        t0 = time.perf_counter()
        w = bsgpu.Writer(st)
        for i in range(0, n, 32 << 20):
            w.write(mv[i:i + (32 << 20)])
        w.close()
        dt = time.perf_counter() - t0
        print(json.dumps({"rep": rep, "gib_per_s": round(n / dt / 2**30, 2), "ms": round(dt * 1e3, 1)}),
              flush=True)
        w.free()  # prints the breakdown
        sys.stderr.flush()
        st.free()


if __name__ == "__main__":
    main()
