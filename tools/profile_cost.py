"""What the engine's stage-timing events (bsg_engine_profile) cost per step: configs[1] and
configs[2] timed with all four events, with the SHA-256 stage's two, and with none, alternating.
python tools/profile_cost.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bs_amd import bsgpu  # noqa: E402


def leg(ns, nbytes, steps=20, warmup=5, rounds=3):
    stride = (nbytes + 15) & ~15
    buf = bsgpu.DeviceBuffer(stride * ns + 4096)
    eng = bsgpu.Engine()
    offs = [i * stride for i in range(ns)]
    for i in range(ns):
        bsgpu.fill_splitmix(buf.ptr + offs[i], nbytes, 0xB5B52026 + i, stream=eng.stream)
    out = {1: [], 2: [], 0: []}
    for _ in range(rounds):
        for prof in (1, 2, 0):
            eng.profile(prof)
            for _ in range(warmup):
                eng.run(buf.ptr, offs, [nbytes] * ns)
                eng.finish()
            bsgpu.synchronize(0)
            t0 = time.perf_counter()
            for _ in range(steps):
                eng.run(buf.ptr, offs, [nbytes] * ns)
                eng.finish()
                if prof:
                    eng.stage_ms()
            bsgpu.synchronize(0)
            out[prof].append((time.perf_counter() - t0) / steps * 1e3)
    eng.close()
    buf.free()
    return out


for name, ns, n in (("configs[1]", 1, 1 << 30), ("configs[2]", 256, 64 << 20)):
    r = leg(ns, n)
    print(f"{name}: ms per step with the four stage events {[round(x, 3) for x in r[1]]}, "
          f"the SHA stage's two {[round(x, 3) for x in r[2]]}, none {[round(x, 3) for x in r[0]]}",
          flush=True)
