"""Per-step timeline of a traced bench run (tools/gpu_r05_call33.sh): for each engine run, the
GPU work from k_start to the last kernel, the D2H copy of the counters, and the host calls
between one run's end and the next run's first kernel (rocprofv3 kernel / memory-copy / HIP API
trace CSVs).

Usage: python tools/step_gaps.py gpurun_out/gaps33"""
import csv
import os
import sys


def rows(d, name):
    with open(os.path.join(d, name)) as f:
        return list(csv.DictReader(f))


def main():
    d = sys.argv[1]
    ks = sorted(rows(d, "run_kernel_trace.csv"), key=lambda r: int(r["Start_Timestamp"]))
    cps = sorted(rows(d, "run_memory_copy_trace.csv"), key=lambda r: int(r["Start_Timestamp"]))
    api = sorted(rows(d, "run_hip_api_trace.csv"), key=lambda r: int(r["Start_Timestamp"]))
    runs = []
    for i, k in enumerate(ks):
        if k["Kernel_Name"].startswith("bsg::k_start"):
            runs.append(i)
    runs.append(len(ks))
    prev_end = None
    for a, b in zip(runs, runs[1:]):
        kk = ks[a:b]
        t0 = int(kk[0]["Start_Timestamp"])
        end = max(int(k["End_Timestamp"]) for k in kk)
        last = max(kk, key=lambda k: int(k["End_Timestamp"]))
        early = [k for k in kk if "k_early(" in k["Kernel_Name"]]
        line = f"run at {t0}: span {(end - t0) / 1e3:8.1f} us, last {last['Kernel_Name'][:24]}"
        if early:
            e = early[0]
            line += (f", k_early {(int(e['Start_Timestamp']) - t0) / 1e3:.1f} .. "
                     f"{(int(e['End_Timestamp']) - t0) / 1e3:.1f} us")
        if prev_end is not None:
            line += f", gap before {(t0 - prev_end) / 1e3:.1f} us"
            cp = [c for c in cps if prev_end <= int(c["Start_Timestamp"]) < t0]
            for c in cp:
                line += (f"\n    copy {c['Direction'][12:]} {(int(c['Start_Timestamp']) - prev_end) / 1e3:.1f}"
                         f" .. {(int(c['End_Timestamp']) - prev_end) / 1e3:.1f} us after the last kernel")
            calls = [r for r in api if prev_end - 30000 <= int(r["End_Timestamp"]) and int(r["Start_Timestamp"]) < t0]
            for r in calls:
                s = (int(r["Start_Timestamp"]) - prev_end) / 1e3
                e = (int(r["End_Timestamp"]) - prev_end) / 1e3
                if e - s > 2 or r["Function"] in ("hipStreamSynchronize", "hipMemcpyAsync", "hipModuleLaunchKernel", "hipLaunchKernel", "hipExtModuleLaunchKernel"):
                    line += f"\n    {r['Function']:28s} {s:9.1f} .. {e:9.1f} us"
        print(line)
        prev_end = end


if __name__ == "__main__":
    main()
