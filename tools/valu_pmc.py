"""Summarise rocprofv3 SQ / GRBM counter passes into profiles/<round>_<tag>_valu_pmc.json
(the VALU work of the SHA-256 stage, the serial chain's cycles).

Usage: python tools/valu_pmc.py --round r05 --tag configs2 --workload "configs[2]: ..." \
           --src gpurun_out/pmc_c2 [--src ...]
Reads every <src>/**/run_counter_collection.csv (one rocprofv3 --pmc pass each) and writes, per
kernel, the launches seen and each counter's mean per launch. SQ_WAVE_CYCLES, SQ_BUSY_CYCLES,
SQ_WAIT_* and SQ_ACTIVE_INST_* count quad-cycles on gfx950 (MI355X_MICROARCH.md, s_memtime row);
SQ_INSTS_* count wave-instructions. bench.py's work_roofline reads SQ_INSTS_VALU from here."""
import argparse
import collections
import csv
import glob
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--round", required=True)
    ap.add_argument("--tag", required=True)
    ap.add_argument("--workload", required=True)
    ap.add_argument("--src", action="append", required=True)
    ap.add_argument("--note", default="")
    a = ap.parse_args()
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    files = []
    for src in a.src:
        for path in sorted(glob.glob(os.path.join(src, "**", "*counter_collection.csv"),
                                     recursive=True)):
            files.append(os.path.relpath(path, ROOT))
            with open(path) as f:
                for r in csv.DictReader(f):
                    vals[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    kernels = {}
    for k, cs in sorted(vals.items()):
        if k.startswith("__amd") or "fill_splitmix" in k:
            continue
        kernels[k] = {"launches": max(len(v) for v in cs.values())}
        for c, v in sorted(cs.items()):
            kernels[k][c] = sum(v) / len(v)
    doc = {"workload": a.workload, "round": a.round, "note": a.note, "sources": files,
           "units": "per launch; SQ_*_CYCLES / SQ_WAIT_* / SQ_ACTIVE_* in quad-cycles summed "
                    "over waves, SQ_INSTS_* in wave-instructions",
           "kernels": kernels}
    out = os.path.join(ROOT, "profiles", f"{a.round}_{a.tag}_valu_pmc.json")
    with open(out, "w") as f:
        json.dump(doc, f, indent=1)
    print(out)
    for k, v in kernels.items():
        print(k[:60], {c: round(x) for c, x in v.items()})


if __name__ == "__main__":
    main()
