"""One e2e rep (tools/e2e_trace_run.py under rocprofv3 --hip-trace --kernel-trace
--memory-copy-trace, tools/gpu_e2e_trace.sh with HIP_TRACE=1) with its host stamps: where the
rep's wall time goes outside [first H2D, last records].
  python tools/e2e_host_timeline.py gpurun_out/<OUT> REP
Reads <OUT>/run_kernel_trace.csv, run_memory_copy_trace.csv, run_hip_api_trace.csv (optional) and
<OUT>.log (the runner's JSON lines: host_ns stamps in the tracer's clock, CLOCK_BOOTTIME)."""
import csv
import json
import os
import sys


def rows(path):
    if not os.path.exists(path):
        return []
    with open(path) as f:
        return list(csv.DictReader(f))


def main(d, rep):
    reps = [json.loads(ln) for ln in open(d + ".log") if ln.startswith("{")]
    r = [x for x in reps if x["rep"] == rep][0]
    st = r["host_ns"]
    t0, t_end = st[0][1], st[-1][1]
    ev = []
    for k in rows(os.path.join(d, "run_kernel_trace.csv")):
        s, e = int(k["Start_Timestamp"]), int(k["End_Timestamp"])
        if t0 <= s <= t_end:
            n = k["Kernel_Name"].replace("bsg::", "").split("(")[0].replace("void ", "")
            ev.append((s, e, f"K q{k['Queue_Id']} {n}"))
    for c in rows(os.path.join(d, "run_memory_copy_trace.csv")):
        s, e = int(c["Start_Timestamp"]), int(c["End_Timestamp"])
        if t0 <= s <= t_end:
            ev.append((s, e, "C " + c["Direction"].replace("MEMORY_COPY_", "")))
    api_busy = {}
    for a in rows(os.path.join(d, "run_hip_api_trace.csv")):
        s, e = int(a["Start_Timestamp"]), int(a["End_Timestamp"])
        if t0 <= s <= t_end:
            fn = a["Function"]
            api_busy[fn] = api_busy.get(fn, 0) + (e - s)
            if e - s > 200_000:  # API calls over 0.2 ms: listed
                ev.append((s, e, f"A t{a['Thread_Id']} {fn}"))
    for name, t in st:
        ev.append((t, t, f"H {name}"))
    ev.sort()
    for s, e, n in ev:
        if n.startswith("C") or n.startswith("H drain") or n.startswith("H write"):
            if n.startswith("C") and (e - s) < 1_000_000:
                continue
        print(f"{(s - t0) / 1e6:8.3f} {(e - t0) / 1e6:8.3f} {(e - s) / 1e6:7.3f}  {n}")
    h2d = [(s, e) for s, e, n in ev if n.startswith("C HOST_TO_DEVICE")]
    recs = [e for s, e, n in ev if "k_copy_out" in n]
    print(f"rep {rep}: wall {(t_end - t0) / 1e6:.3f} ms")
    if h2d:
        print(f"  start -> first H2D start   {(h2d[0][0] - t0) / 1e6:8.3f} ms")
        print(f"  first H2D -> last H2D end  {(h2d[-1][1] - h2d[0][0]) / 1e6:8.3f} ms "
              f"({len(h2d)} copies, busy {sum(e - s for s, e in h2d) / 1e6:.3f} ms)")
    if recs:
        print(f"  last H2D end -> last records {(max(recs) - h2d[-1][1]) / 1e6:8.3f} ms")
        print(f"  last records -> end         {(t_end - max(recs)) / 1e6:8.3f} ms")
    for fn, t in sorted(api_busy.items(), key=lambda x: -x[1])[:12]:
        print(f"  API {fn:32s} {t / 1e6:8.3f} ms (summed over threads)")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]))
