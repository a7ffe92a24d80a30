"""First-use cost of the drop-in split.Writer: each case in a fresh process
(so nothing is pooled yet), the library loaded and the device counted before the clock starts.

  cold1m   split::Writer New + Write(1 MiB) + Close, the first Writer of the process
  first4g  the first Writer of the process on a 4 GiB stream in 32 MiB Writes, then a second
           one (pooled context and staging)
  breakdown  the same first-use path step by step, without bsg_init

Except in "breakdown", the process first calls bsg_init (HIP context, kernel code object, copy
threads: the once-per-process cost a server pays at start-up), timed separately as init_ms.

  python tools/first_writer.py            -> one JSON line per case
"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def case(name: str) -> dict:
    sys.path.insert(0, ROOT)
    from bs_amd import bsgpu
    from bs_amd.synth import splitmix_array
    assert bsgpu.device_count() >= 1
    if name == "breakdown":  # where the first Writer's time goes, step by step
        import numpy as np
        out, t = {"case": name}, time.perf_counter()

        def lap(k):
            nonlocal t
            t1 = time.perf_counter()
            out[k] = round((t1 - t) * 1e3, 2)
            t = t1
        L = bsgpu.lib()
        lap("after_device_count")
        L.bsg_device_synchronize(0)
        lap("device_context")
        eng = bsgpu.Engine()
        lap("engine_create")
        buf = bsgpu.DeviceBuffer(1 << 20)
        bsgpu.fill_splitmix(buf.ptr, 1 << 20, 3)
        bsgpu.synchronize()
        lap("first_kernel")
        eng.run(buf.ptr, [0], [1 << 20])
        eng.finish()
        lap("first_engine_run")
        eng.run(buf.ptr, [0], [1 << 20])
        eng.finish()
        lap("second_engine_run")
        sp = bsgpu.StreamingSplitter()
        lap("bsg_open")
        data = splitmix_array(1, 1 << 20)
        sp.write(data)
        lap("bsg_write_1m")
        sp.close()
        sp.drain()
        lap("bsg_close_1m")
        sp.reset()
        sp.write(data)
        sp.close()
        sp.drain()
        lap("pooled_ctx_1m")
        st = bsgpu.MemStore()
        w = bsgpu.Writer(st)
        lap("writer_new")
        w.write(data)
        w.close()
        lap("writer_1m")
        return out
    if name == "breakdown_init":  # after bsg_init: what a server's first Writer pays
        t = time.perf_counter()
        bsgpu.init(0)
        out = {"case": name, "init_ms": round((time.perf_counter() - t) * 1e3, 2)}
        data = splitmix_array(1, 1 << 20)
        st = bsgpu.MemStore()
        for rep in range(3):
            t = time.perf_counter()
            w = bsgpu.Writer(st, bits=16 + rep)  # a new parameter key: a fresh context each time
            t1 = time.perf_counter()
            w.write(data)
            t2 = time.perf_counter()
            w.close()
            t3 = time.perf_counter()
            out[f"rep{rep}"] = {"new": round((t1 - t) * 1e3, 2), "write": round((t2 - t1) * 1e3, 2),
                                "close": round((t3 - t2) * 1e3, 2)}
            w.free()
        return out
    t_init = time.perf_counter()
    bsgpu.init(0)
    init_ms = round((time.perf_counter() - t_init) * 1e3, 2)
    if name == "cold1m":
        data = splitmix_array(1, 1 << 20)
        st = bsgpu.MemStore()
        t0 = time.perf_counter()
        w = bsgpu.Writer(st)
        w.write(data)
        w.close()
        t1 = time.perf_counter()
        out = {"case": name, "init_ms": init_ms, "ms": round((t1 - t0) * 1e3, 2),
               "blobs": len(st)}
        w2 = bsgpu.Writer(st)
        t2 = time.perf_counter()
        w2.write(data)
        w2.close()
        out["second_ms"] = round((time.perf_counter() - t2) * 1e3, 2)
        return out
    n = 4 << 30
    data = splitmix_array(2, n)
    mv = memoryview(data)
    out = {"case": name, "init_ms": init_ms, "bytes": n}
    for rep in ("first", "second"):
        st = bsgpu.MemStore()
        t0 = time.perf_counter()
        w = bsgpu.Writer(st)
        for i in range(0, n, 32 << 20):
            w.write(mv[i:i + (32 << 20)])
        w.close()
        dt = time.perf_counter() - t0
        out[rep + "_gibs"] = round(n / dt / 2**30, 2)
        w.free()
        st.free()
    return out


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--case":
        print(json.dumps(case(sys.argv[2])), flush=True)
        return
    names = sys.argv[1:] or ["breakdown", "cold1m", "cold1m", "first4g"]
    for name in names:
        r = subprocess.run([sys.executable, __file__, "--case", name], capture_output=True,
                           text=True, timeout=600)
        sys.stdout.write(r.stdout if r.returncode == 0 else f"{name} failed: {r.stderr[-1500:]}\n")
        sys.stdout.flush()
        if r.returncode:
            sys.exit(r.returncode)


if __name__ == "__main__":
    main()
