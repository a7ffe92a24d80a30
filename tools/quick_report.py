"""Prints the bench lines and k_scan / k_refine / k_sha stats of a tools/gpu_quick*.sh run."""
import csv
import json
import os

O = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
for f in ("bench_c1", "bench_c2"):
    try:
        d = json.loads(open(os.path.join(O, f + ".log")).read().strip().splitlines()[-1])
        print(f, d["value"], d["ms_per_step"], d["stage_ms"])
    except Exception as e:  # noqa: BLE001
        print(f, "missing", e)
for q, nbytes in (("c1", 1 << 30), ("c2", 16 << 30)):
    p = os.path.join(O, f"q_{q}", "run_kernel_stats.csv")
    if os.path.exists(p):
        for r in csv.DictReader(open(p)):
            if any(k in r["Name"] for k in ("k_scan", "k_refine", "k_sha", "k_compact")):
                print(q, r["Name"][:40], round(float(r["AverageNs"]) / 1e3, 1), "us")
    p = os.path.join(O, f"qf_{q}", "run_counter_collection.csv")
    if os.path.exists(p):
        for r in csv.DictReader(open(p)):
            if "k_scan" in r["Kernel_Name"]:
                print(q, "k_scan FETCH x2 / input:", round(2 * float(r["Counter_Value"]) * 1024 / nbytes, 4))
