"""Timeline of one streaming rep from a rocprofv3 kernel + memory-copy trace
(tools/gpu_e2e_trace.sh): per tile, when its H2D, scan..select and k_sha ran, and on which
queue. Usage: python tools/e2e_timeline.py gpurun_out/e2e_trace [rep] [tiles_per_rep]"""
import csv
import os
import sys


def main(d, rep=3, per=16):
    ks = sorted(csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))),
                key=lambda r: int(r["Start_Timestamp"]))
    cp = sorted(csv.DictReader(open(os.path.join(d, "run_memory_copy_trace.csv"))),
                key=lambda r: int(r["Start_Timestamp"]))
    inits = [r for r in ks if "k_init" in r["Kernel_Name"] or "k_start" in r["Kernel_Name"]]
    first = inits[rep * per]
    t0 = int(first["Start_Timestamp"])
    t_end = int(inits[(rep + 1) * per]["Start_Timestamp"]) if len(inits) > (rep + 1) * per else None
    ev = []
    for r in ks:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s < t0 - 50_000_000 or (t_end and s > t_end):
            continue
        name = r["Kernel_Name"].replace("bsg::", "").split("(")[0].replace("void ", "")
        if name in ("k_init", "k_start", "k_scan", "k_sha") or name.startswith("__amd"):
            ev.append((s, e, f"q{r['Queue_Id']} {name}"))
    for r in cp:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s < t0 - 50_000_000 or (t_end and s > t_end):
            continue
        ev.append((s, e, f"s{r['Stream_Id']} {r['Direction'].replace('MEMORY_COPY_', '')}"))
    ev.sort()
    for s, e, n in ev:
        print(f"{(s - t0) / 1e6:9.3f} ms  {(e - s) / 1e6:8.3f} ms  {n}")


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0], int(a[1]) if len(a) > 1 else 3, int(a[2]) if len(a) > 2 else 16)
