"""Build libbsgpu.so in-tree for gfx950 (hipcc, no JIT cache): `python -m bs_amd.build`."""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libbsgpu.so")
SOURCES = ["bsgpu_kernels.hip", "bsgpu_host.cpp", "bs_split.cpp", "bs_filestore.cpp"]
HEADERS = ["bsgpu_internal.h", "bsgpu_launch.h", "buzhash32_table.inc", "sha256_device.h",
           "sha256_skew_block.inc", "sha256_skew_loop.inc"]
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


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return LIB
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wall", "-Wno-unused-function", "-Wno-unused-value", "-Wno-unused-result", "-o", LIB + ".tmp"]
    cmd += [os.path.join(CSRC, f) for f in SOURCES]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
