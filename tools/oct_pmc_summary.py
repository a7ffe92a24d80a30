"""Per-block SQ counters of the octet chain ubench (tools/ubench/oct_pmc: one lone wave, 4,000
blocks x 3 launches per loop form) from a rocprofv3 --pmc csv, as profiles/rNN_oct_pmc.json.
   python tools/oct_pmc_summary.py gpurun_out/<dir>/run_counter_collection.csv out.json"""
import collections
import csv
import json
import sys

BLOCKS = 4000
NAMES = {"void kb<2>(unsigned long*, unsigned int*, int)": "general loop (sha256_blocks_oct)",
         "void kb<3>(unsigned long*, unsigned int*, int)": "solo loop (sha256_blocks_oct_solo)"}


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    by = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in rows:
        if r["Kernel_Name"] in NAMES:
            by[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {"workload": "tools/ubench/oct_pmc: one lone wave, octet chain, 4000 blocks x 3 launches",
           "units": "per block; *_CYCLES / SQ_WAIT_* / SQ_ACTIVE_* converted from quad-cycles "
                    "to cycles (x4), SQ_INSTS_* in wave-instructions",
           "source": sys.argv[1], "loops": {}}
    for k, d in by.items():
        m = {c: sum(v) / len(v) / BLOCKS for c, v in d.items()}
        per = {c: round(v * (4 if "CYCLES" in c or "WAIT" in c or "ACTIVE" in c else 1), 2)
               for c, v in m.items()}
        counted = sum(m[c] for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU",
                                    "SQ_INSTS_BRANCH") if c in m)
        per["counted_instructions"] = round(counted, 2)
        per["active_cycles_per_counted_instruction"] = round(4 * m["SQ_ACTIVE_INST_ANY"] / counted, 3)
        out["loops"][NAMES[k]] = per
    json.dump(out, open(sys.argv[2], "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
