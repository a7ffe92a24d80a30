"""Build libbsgpu.so in-tree for gfx950 (hipcc, no JIT cache): `python -m bs_amd.build`."""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libbsgpu.so")
SOURCES = ["bsgpu_kernels.hip", "bsgpu_host.cpp", "bs_split.cpp", "bs_filestore.cpp"]
HEADERS = ["bsgpu_internal.h", "host_pool.h", "bsgpu_launch.h", "buzhash32_table.inc", "sha256_device.h",
           "sha256_skew_block.inc", "sha256_skew_loop.inc", "sha256_oct_loop.inc",
           "sha256_lane_asm.inc"]
ARCH = os.environ.get("BSG_OFFLOAD_ARCH", "gfx950")


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS]
    deps.append(os.path.join(os.path.dirname(HERE), "include", "bsgpu.h"))
    deps.append(os.path.join(os.path.dirname(HERE), "include", "bs_split.hpp"))
    return any(os.path.getmtime(d) > t for d in deps)


def build_debug(extra=(), name="libbsgpu_dbg.so") -> str:
    """Device-printf build (libbsgpu_dbg.so) for chasing hangs; never loaded by default."""
    out = os.path.join(HERE, name)
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wno-unused-value", "-Wno-unused-result", *extra, "-o", out]
    cmd += [os.path.join(CSRC, f) for f in SOURCES]
    subprocess.run(cmd, check=True)
    return out


def build_locked(out: str, stale, compile_to) -> bool:
    """Runs compile_to(tmp) and renames tmp to `out` if stale() holds, under an exclusive
    flock on out + ".lock", so concurrent builders (bench ranks, test workers) compile once:
    the others wait, re-check stale() and find the fresh library. The temporary file is per
    process and the rename is atomic, so a process loading `out` never sees a partial file.
    Returns True if this call compiled."""
    import fcntl
    with open(out + ".lock", "a") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        try:
            if not stale():
                return False
            tmp = f"{out}.tmp.{os.getpid()}"
            try:
                compile_to(tmp)
                os.replace(tmp, out)
            finally:
                if os.path.exists(tmp):
                    os.unlink(tmp)
            return True
        finally:
            fcntl.flock(lk, fcntl.LOCK_UN)


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return LIB
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

    def compile_to(tmp):
        cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
               "-Wall", "-Wno-unused-function", "-Wno-unused-value", "-Wno-unused-result",
               "-o", tmp]
        cmd += [os.path.join(CSRC, f) for f in SOURCES]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)

    forced = [force]

    def stale():
        if forced[0]:
            forced[0] = False
            return True
        return _stale()

    build_locked(LIB, stale, compile_to)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
