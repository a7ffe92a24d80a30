"""A/B of the host copy form on the streaming path (round 6): BSG_KNOB_COPY_NT 1 (non-temporal
stores; the Writer's one read into piece + stage) against 0 (memcpy), interleaved in one process
so box-to-box spread cancels. Each round runs bench.py's end_to_end leg (raw bsg_write, 1 GiB)
and writer_e2e leg (split::Writer -> store/mem) once per form and prints one JSON line per leg
with the per-rep breakdown.   python tools/host_copy_ab.py [rounds] [MiB]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from bs_amd import bsgpu  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    mib = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    bsgpu.init(0)
    print(json.dumps({"host": bench.host_placement()}), flush=True)
    for r in range(rounds):
        for nt in (1, 0) if r % 2 == 0 else (0, 1):
            with bsgpu.debug_knob(bsgpu.KNOB_COPY_NT, nt):
                e = bench.end_to_end(mib, 16, 1024, 0)
                e.pop("records")
                print(json.dumps({"round": r, "nt": nt, "leg": "end_to_end", "value": e["value"],
                                  "reps_ms": e["reps_ms"],
                                  "last": e["reps_breakdown"][-1]}), flush=True)
                w = bench.writer_e2e(mib, 16, 1024, 0)
                w.pop("data")
                print(json.dumps({"round": r, "nt": nt, "leg": "writer_e2e", "value": w["value"],
                                  "reps": w["reps"]}), flush=True)


if __name__ == "__main__":
    main()
