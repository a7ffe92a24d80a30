"""store/file as the sink and source of the path: the C++ split.Writer into a
FileStore (one file per blob, blobs/hh/hhhh/<hex>, O_CREAT|O_EXCL; refs from the split kernels,
PutWithRef), then split.Reader over it with and without verification. One SplitMix64 stream
(default 1 GiB, FILESTORE_MIB) in a fresh directory under FILESTORE_DIR (default: the system
temp dir). Prints one JSON line per case, with the filesystem type.
"""
import json
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bs_amd import bsgpu  # noqa: E402
from bs_amd.synth import splitmix_array  # noqa: E402


def fs_type(path: str) -> str:
    best, kind = "", "?"
    try:
        for line in open("/proc/mounts"):
            f = line.split()
            if len(f) > 2 and path.startswith(f[1]) and len(f[1]) > len(best):
                best, kind = f[1], f[2]
    except OSError:
        pass
    return kind


def main():
    n = int(os.environ.get("FILESTORE_MIB", "1024")) << 20
    base = os.environ.get("FILESTORE_DIR") or tempfile.gettempdir()
    data = splitmix_array(0xB5B52026, n)
    mv = memoryview(data)
    for run in range(2):
        d = tempfile.mkdtemp(prefix="bsfs_", dir=base)
        try:
            fs = bsgpu.FileStore(d)
            t0 = time.perf_counter()
            w = bsgpu.Writer(fs)
            for i in range(0, n, 32 << 20):
                w.write(mv[i:i + (32 << 20)])
            w.close()
            dt = time.perf_counter() - t0
            root = w.root
            w.free()
            print(json.dumps({"case": "split.Writer -> store/file", "run": run, "bytes": n,
                              "blobs": len(fs), "fs": fs_type(d), "seconds": round(dt, 4),
                              "gib_per_s": round(n / dt / 2**30, 3)}), flush=True)
            for verify in (False, True):
                r = bsgpu.Reader(fs, root, verify=verify)
                t0 = time.perf_counter()
                got = 0
                while True:
                    b = r.read(1 << 20)
                    if not b:
                        break
                    got += len(b)
                dt = time.perf_counter() - t0
                assert got == n
                print(json.dumps({"case": "store/file -> split.Reader", "run": run,
                                  "verify": verify, "seconds": round(dt, 4),
                                  "gib_per_s": round(n / dt / 2**30, 3)}), flush=True)
            fs.free()
        finally:
            shutil.rmtree(d, ignore_errors=True)


if __name__ == "__main__":
    main()
