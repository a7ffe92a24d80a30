"""Summarises gpurun_out/sweep/*_c{1,2}.log (tools/gpu_variant_sweep.sh)."""
import glob
import json
import os

O = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out", "sweep")
for f in sorted(glob.glob(os.path.join(O, "*_c*.log"))):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception:  # noqa: BLE001
        print(os.path.basename(f), "no line")
        continue
    t = d["sha_path"].get("timeline_us", {})
    print(f"{os.path.basename(f):28s} {d['value']:9.2f} GiB/s {d['ms_per_step']:7.2f} ms  "
          f"long_end {t.get('long_end')} lane_end {t.get('lane_end')} tickets {d['sha_path'].get('wave_tickets')}")
