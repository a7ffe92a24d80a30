"""bench.py's one-line JSON contract, on a small workload (the driver runs the full default).

Checks the keys and types the round-end driver and the judge read: the metric and unit of
BASELINE.json, the whole-job value, the roofline object (bound, achieved, peak, unit, frac,
traffic) and the cpu_baseline object (value, unit, cores, kind, sample).
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_bench_json_line():
    cmd = [sys.executable, "bench.py", "--steps", "2", "--warmup", "1", "--streams", "2",
           "--stream-mib", "64", "--cpu-sample-mib", "8", "--e2e-mib", "64"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        base = json.load(f)
    assert d["metric"] == base["metric"]
    assert d["unit"] == "GiB/s" and d["higher_is_better"] is True
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["warmup"] == 1
    assert d["value"] > 0 and d["ms_per_step"] > 0
    assert d["scaling"] == "weak" and d["vs_baseline"] is None
    assert d["dtype"] == "u8" and "synthetic" in d["data"]
    assert d["config"]["workload"] and d["config"]["streams_per_gpu"] == 2
    rf = d["roofline"]
    # the bound that binds; the graded fraction stays the HBM roof's
    assert rf["bound"] and rf["roof"] in ("hbm", "mfma") and rf["unit"] == "GB/s"
    assert rf["peak"] > 0 and rf["achieved"] > 0
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-3
    assert "traffic" in rf
    cb = d["cpu_baseline"]
    assert cb["value"] > 0 and cb["unit"] == "GiB/s" and cb["cores"] >= 1
    assert cb["kind"] in ("port", "reference") and cb["sample"]
    assert d["end_to_end"]["value"] > 0
    assert d["chain_roofline"]["frac"] > 0
    assert d["oracle_check"] is True and d["oracle_checked"]  # parity on the bench's own bytes


@pytest.mark.gpu
def test_bench_default_carries_configs2():
    """The default workload (configs[1]) also carries the nested configs[2] record."""
    cmd = [sys.executable, "bench.py", "--steps", "2", "--warmup", "1", "--configs2-steps", "1",
           "--cpu-sample-mib", "64", "--e2e-mib", "0"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["config"]["workload"].startswith("configs[1]")
    c2 = d["configs2"]
    assert c2["workload"].startswith("configs[2]") and c2["steps"] == 1
    assert c2["value"] > d["value"] and c2["ms_per_step"] > 0
    assert c2["roofline"]["kernel"].startswith("k_sha") and c2["roofline"]["frac"] > 0
    assert c2["roofline"]["k_scan"]["frac"] > 0
    assert c2["cpu_baseline"]["cores"] >= 1 and c2["cpu_baseline"]["full_writer"]["value"] > 0
    assert set(c2["stage_ms"]) == set(d["stage_ms"])
    assert d["oracle_check"] is True and c2["oracle_check"] is True
