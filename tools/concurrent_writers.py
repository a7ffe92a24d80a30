"""N split.Writers at once (the fs.Dir.AddDir pattern, fs/dir.go:157-174; one goroutine per file
in a concurrent ingest): aggregate GiB/s of N host threads, each writing its own stream in 32 MiB
Writes into one shared store/mem. After bsg_init; each N three times.

  python tools/concurrent_writers.py [MiB per writer, default 512]
"""
import json
import os
import sys
import threading
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bs_amd import bsgpu  # noqa: E402
from bs_amd.synth import splitmix_array  # noqa: E402


def main():
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    n = mib << 20
    bsgpu.init(0)
    streams = [splitmix_array(100 + i, n) for i in range(8)]
    piece = 32 << 20
    for nw in (1, 2, 4, 8):
        runs = []
        for rep in range(3):
            st = bsgpu.MemStore()
            start = threading.Barrier(nw + 1)

            def one(i):
                w = bsgpu.Writer(st)
                mv = memoryview(streams[i])
                start.wait()
                for o in range(0, n, piece):
                    w.write(mv[o:o + piece])
                w.close()
                w.free()

            with ThreadPoolExecutor(nw) as ex:
                futs = [ex.submit(one, i) for i in range(nw)]
                start.wait()
                t0 = time.perf_counter()
                for f in futs:
                    f.result()
                dt = time.perf_counter() - t0
            runs.append(round(nw * n / dt / 2**30, 2))
            st.free()
        print(json.dumps({"writers": nw, "bytes_each": n, "aggregate_gibs": runs,
                          "best": max(runs)}), flush=True)


if __name__ == "__main__":
    main()
