"""A/B of library builds on the host-memory paths: for each library (BSG_LIB_PATH), in a fresh
process, 5 repetitions of (a) the C++ split.Writer -> store/mem on a 4 GiB stream in 32 MiB
Writes and (b) the raw bsg_write/bsg_drain streaming of the same bytes; libraries alternate
twice (AB_ROUNDS) so box drift shows.   python tools/writer_ab.py lib_a.so lib_b.so ..."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child():
    sys.path.insert(0, ROOT)
    from bs_amd import bsgpu
    from bs_amd.synth import splitmix_array
    if hasattr(bsgpu.lib(), "bsg_init"):
        bsgpu.init(0)
    else:  # an older build: the same one-time work, by one tiny engine run
        e = bsgpu.Engine()
        e.close()
    n = int(os.environ.get("AB_MIB", "4096")) << 20
    data = splitmix_array(2, n)
    mv = memoryview(data)
    out = {"lib": os.environ["BSG_LIB_PATH"], "writer": [], "raw": []}
    for rep in range(5):
        st = bsgpu.MemStore()
        t0 = time.perf_counter()
        w = bsgpu.Writer(st)
        for i in range(0, n, 32 << 20):
            w.write(mv[i:i + (32 << 20)])
        w.close()
        out["writer"].append(round(n / (time.perf_counter() - t0) / 2**30, 2))
        w.free()
        st.free()
    sp = bsgpu.StreamingSplitter()
    for rep in range(5):
        sp.reset()
        t0 = time.perf_counter()
        for i in range(0, n, 32 << 20):
            sp.write(mv[i:i + (32 << 20)])
            sp.drain()
        sp.close()
        sp.drain()
        out["raw"].append(round(n / (time.perf_counter() - t0) / 2**30, 2))
    sp.free()
    print(json.dumps(out), flush=True)


def main():
    if os.environ.get("AB_CHILD") == "1":
        child()
        return
    libs = [os.path.abspath(x) for x in sys.argv[1:]]
    for rnd in range(int(os.environ.get("AB_ROUNDS", "2"))):
        for lib in libs:
            env = dict(os.environ, AB_CHILD="1", BSG_LIB_PATH=lib, BSG_LIB_PARTIAL="1")
            r = subprocess.run([sys.executable, __file__], env=env, capture_output=True, text=True,
                               timeout=600)
            sys.stdout.write(r.stdout if r.returncode == 0 else f"{lib} failed: {r.stderr[-1500:]}\n")
            sys.stdout.flush()
            if r.returncode:
                sys.exit(r.returncode)


if __name__ == "__main__":
    main()
