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


def node_cpus(node: int):
    cpus = set()
    for part in open(f"/sys/devices/system/node/node{node}/cpulist").read().strip().split(","):
        a, _, b = part.partition("-")
        cpus.update(range(int(a), int(b or a) + 1))
    return cpus


def cpu_now() -> int:
    return int(open("/proc/self/stat").read().rsplit(")", 1)[1].split()[36])


def child():
    if os.environ.get("AB_NODE"):  # bind the process (and so its first-touch memory) to a node
        os.sched_setaffinity(0, node_cpus(int(os.environ["AB_NODE"])) & os.sched_getaffinity(0))
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
    out = {"lib": os.path.basename(os.environ["BSG_LIB_PATH"]), "writer": [], "raw": [],
           "cpus": sorted(os.sched_getaffinity(0))[:1] + [len(os.sched_getaffinity(0))],
           "numa_nodes": len([d for d in os.listdir("/sys/devices/system/node")
                              if d.startswith("node")]) if os.path.isdir("/sys/devices/system/node") else None}
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
    out["cpu_end"] = cpu_now()
    out["node"] = os.environ.get("AB_NODE")
    out["env"] = {k: v for k, v in os.environ.items() if k.startswith("BSG_") and k not in
                  ("BSG_LIB_PATH", "BSG_LIB_PARTIAL")}
    print(json.dumps(out), flush=True)


def main():
    if os.environ.get("AB_CHILD") == "1":
        child()
        return
    # each argument: a library, optionally with environment settings for it: lib.so:K=V,K2=V2
    specs = []
    for x in sys.argv[1:]:
        lib, _, kv = x.partition(":")
        specs.append((os.path.abspath(lib), dict(p.split("=", 1) for p in kv.split(",") if p)))
    for rnd in range(int(os.environ.get("AB_ROUNDS", "2"))):
        for lib, extra in specs:
            env = dict(os.environ, AB_CHILD="1", BSG_LIB_PATH=lib, BSG_LIB_PARTIAL="1", **extra)
            r = subprocess.run([sys.executable, __file__], env=env, capture_output=True, text=True,
                               timeout=600)
            sys.stdout.write(r.stdout if r.returncode == 0 else f"{lib} failed: {r.stderr[-1500:]}\n")
            if r.returncode == 0 and "bsgpu:" in r.stderr:
                sys.stdout.write("".join(l + "\n" for l in r.stderr.splitlines() if "bsgpu:" in l))
            sys.stdout.flush()
            if r.returncode:
                sys.exit(r.returncode)


if __name__ == "__main__":
    main()
