"""HBM read bytes per kernel from one rocprofv3 pass of TCC_EA0_RDREQ split by request size
(tools/gpu_r05_call13.sh): bytes = 32 x RDREQ_32B + 64 x RDREQ_64B + 128 x RDREQ_128B. Unlike
FETCH_SIZE (which tallies gfx950's 128-B requests at 64 B, MI355X_MICROARCH.md HBM section),
this needs no per-pattern correction.
Usage: python tools/rdreq_summary.py <run dir> <algorithmic bytes> [--json out.json]"""
import collections
import csv
import json
import os
import sys


def summarise(run_dir, alg):
    rows = csv.DictReader(open(os.path.join(run_dir, "run_counter_collection.csv")))
    agg = collections.defaultdict(collections.Counter)
    disp = collections.defaultdict(set)
    for r in rows:
        agg[r["Kernel_Name"]][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[r["Kernel_Name"]].add(r["Dispatch_Id"])
    out = {}
    for k, c in agg.items():
        n = max(1, len(disp[k]))
        b = (32 * c["TCC_EA0_RDREQ_32B_sum"] + 64 * c["TCC_EA0_RDREQ_64B_sum"]
             + 128 * c["TCC_EA0_RDREQ_128B_sum"]) / n
        out[k] = {"launches": n, "read_bytes_per_launch": b,
                  "read_over_algorithmic": b / alg if alg else None,
                  "requests_128b_share": c["TCC_EA0_RDREQ_128B_sum"] / max(1.0, c["TCC_EA0_RDREQ_sum"])}
    return out


def main():
    run_dir, alg = sys.argv[1], float(sys.argv[2])
    out = summarise(run_dir, alg)
    for k, v in sorted(out.items(), key=lambda kv: -kv[1]["read_bytes_per_launch"]):
        if v["read_bytes_per_launch"] > 1e6:
            print(f"{k[:50]:50s} {v['read_bytes_per_launch'] / 2**30:8.4f} GiB/launch  "
                  f"x{v['read_over_algorithmic']:.4f}  128-B share {v['requests_128b_share']:.4f}")
    if "--json" in sys.argv:
        with open(sys.argv[sys.argv.index("--json") + 1], "w") as f:
            json.dump({"source": run_dir, "algorithmic_bytes": alg, "kernels": out}, f, indent=1)


if __name__ == "__main__":
    main()
