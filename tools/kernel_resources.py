#!/usr/bin/env python3
"""Per-kernel register / scratch / spill summary of bsgpu_kernels.hip for gfx950 (hipcc
-Rpass-analysis=kernel-resource-usage), to check that a change did not push a kernel into
spills (k_sha sits at the SGPR limit). CPU only: python tools/kernel_resources.py"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "bs_amd", "csrc", "bsgpu_kernels.hip")
out = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-c",
                      "--cuda-device-only", "-Rpass-analysis=kernel-resource-usage", SRC,
                      "-o", "/tmp/kernel_resources.o"] + sys.argv[1:],
                     capture_output=True, text=True, cwd="/tmp").stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m:
        continue
    txt = m.group(1).strip()
    if txt.startswith("Function Name:"):
        cur = {"name": txt.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in txt:
        k, v = txt.split(":", 1)
        cur[k.strip()] = v.strip()
print(f"{'kernel':44s} {'SGPR':>5s} {'VGPR':>5s} {'AGPR':>5s} {'scratch':>7s} {'sspill':>6s} {'vspill':>6s} {'LDS':>7s}")
for r in rows:
    n = subprocess.run(["c++filt", r["name"]], capture_output=True, text=True).stdout.strip()
    print(f"{n[:44]:44s} {r.get('TotalSGPRs', '?'):>5s} {r.get('VGPRs', '?'):>5s} "
          f"{r.get('AGPRs', '?'):>5s} {r.get('ScratchSize [bytes/lane]', '?'):>7s} "
          f"{r.get('SGPRs Spill', '?'):>6s} {r.get('VGPRs Spill', '?'):>6s} "
          f"{r.get('LDS Size [bytes/block]', '?'):>7s}")
