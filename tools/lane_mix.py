"""k_sha per-lane mode's instruction mix per SHA-256 block (tools/gpu_r05_call22.sh: configs[2]
with every job in per-lane mode, BSG_LONG_MODE=off, two SQ counter passes).

Usage: python tools/lane_mix.py gpurun_out/lanemix1 gpurun_out/lanemix2 gpurun_out/lanemix1.log
Per k_sha<false> launch: wave-instructions by type per block-lane-step (one block of one lane is
1/64 of a wave's block), and active / wait quad-cycles as shares of the waves' cycles."""
import collections
import csv
import json
import os
import sys


def counters(run_dir):
    agg = collections.defaultdict(collections.Counter)
    with open(os.path.join(run_dir, "run_counter_collection.csv")) as f:
        for r in csv.DictReader(f):
            if "k_sha<false>" in r["Kernel_Name"]:
                agg[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    # the launch that did the work (the other instantiation returns at once)
    return max(agg.values(), key=lambda c: c.get("SQ_INSTS_VALU", 0) + c.get("SQ_ACTIVE_INST_ANY", 0))


def main():
    c1, c2 = counters(sys.argv[1]), counters(sys.argv[2])
    blocks = None
    for line in open(sys.argv[3]):
        if line.startswith("{"):
            blocks = json.loads(line)["sha_path"]["total_blocks"]
    wave_blocks = blocks / 64.0
    out = {"total_blocks": blocks}
    for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_BRANCH", "SQ_INSTS_LDS",
              "SQ_INSTS_VMEM"):
        out[k + "_per_block"] = round(c1[k] / wave_blocks, 1)
    cyc = c1["SQ_WAVE_CYCLES"]
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
              "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_MISC", "SQ_ACTIVE_INST_VMEM",
              "SQ_ACTIVE_INST_FLAT"):
        out[k + "_share"] = round(c2[k] / cyc, 4) if cyc else None
    out["wave_cycles_per_block"] = round(4 * cyc / wave_blocks, 1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
