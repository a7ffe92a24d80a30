"""Per-rep timeline of tools/e2e_trace_run.py under rocprofv3 --kernel-trace --memory-copy-trace
(tools/gpu_e2e_trace.sh): k_start (k_init before round 4) / k_scan / k_sha / k_copy_out per queue
and every H2D copy, relative to the rep's first H2D. Reps are told apart by their k_start count
(TILES per rep, after SKIP k_starts of bsg_init's warm-up runs).
  python tools/e2e_rep_timeline.py gpurun_out/e2e_trace REP [TILES=4] [SKIP=3]"""
import csv
import os
import sys


def main(d, rep, tiles=4, skip=3):
    ks = sorted(csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))),
                key=lambda r: int(r["Start_Timestamp"]))
    cp = sorted(csv.DictReader(open(os.path.join(d, "run_memory_copy_trace.csv"))),
                key=lambda r: int(r["Start_Timestamp"]))
    inits = [r for r in ks if "k_init" in r["Kernel_Name"] or "k_start" in r["Kernel_Name"]]
    first = skip + rep * tiles
    # the rep's window: after the previous rep's last kernel, up to the next rep's first k_init
    lo = max(int(r["End_Timestamp"]) for r in ks if int(r["Start_Timestamp"]) < int(inits[first]["Start_Timestamp"])
             and "k_copy_out" in r["Kernel_Name"]) if first else 0
    nxt = first + tiles
    hi = int(inits[nxt]["Start_Timestamp"]) if nxt < len(inits) else 1 << 62
    copies = [r for r in cp if lo < int(r["Start_Timestamp"]) < hi]
    t0 = int(copies[0]["Start_Timestamp"])
    ev = []
    for r in ks:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        n = r["Kernel_Name"].replace("bsg::", "").split("(")[0].replace("void ", "")
        if t0 <= s < hi and any(k in n for k in ("k_init", "k_start", "k_scan", "k_sha", "k_copy_out")):
            ev.append((s, e, f"q{r['Queue_Id']} {n}"))
    for r in copies:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        ev.append((s, e, "H2D" if "HOST_TO_DEVICE" in r["Direction"] else r["Direction"]))
    ev.sort()
    end = max(e for _, e, n in ev if "k_copy_out" in n)  # the rep's last records
    for s, e, n in ev:
        print(f"{(s - t0) / 1e6:8.3f} {(e - t0) / 1e6:8.3f} {(e - s) / 1e6:7.3f}  {n}")
    print(f"first H2D to last records: {(end - t0) / 1e6:.3f} ms (later H2Ds: the next rep)")


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0], int(a[1]), *(int(x) for x in a[2:]))
