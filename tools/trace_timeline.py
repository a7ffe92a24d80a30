"""Per-step timeline from a rocprofv3 kernel trace (run_kernel_trace.csv): for every engine run
(delimited by k_init), each kernel's start offset and duration, and the run's total span.
Usage: python tools/trace_timeline.py gpurun_out/prof_trace/run_kernel_trace.csv"""
import csv
import sys


def main(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    runs, cur = [], None
    for r in rows:
        name = r["Kernel_Name"].replace("bsg::", "").split("(")[0]
        if name.startswith(("k_init", "k_start")):
            cur = []
            runs.append(cur)
        if cur is not None and not name.startswith("__amd"):
            cur.append((name, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    for i, run in enumerate(runs):
        t0 = run[0][1]
        busy = sum(e - s for _, s, e in run)
        span = run[-1][2] - t0
        print(f"run {i}: span {span / 1e6:.3f} ms, kernels busy {busy / 1e6:.3f} ms, "
              f"gaps {(span - busy) / 1e3:.1f} us")
        if i == len(runs) - 1:
            for name, s, e in run:
                print(f"   +{(s - t0) / 1e3:9.1f} us  {(e - s) / 1e3:9.1f} us  {name}")


if __name__ == "__main__":
    main(sys.argv[1])
