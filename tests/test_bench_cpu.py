"""bench.py's host-side helpers on CPU: the committed profiles it reads for the roofline
(FETCH/WRITE summaries for traffic, SQ summaries for the work roofline) parse, and a summary
of one kind is never taken for the other (a round-5 SQ summary once broke the traffic lookup)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_traffic_lookup_reads_byte_summaries_only():
    for kernel in ("k_sha", "k_scan"):
        for wl in (bench.CONFIGS1, bench.CONFIGS2):
            t, src = bench.pmc_traffic(kernel, wl)
            if t is not None:
                assert isinstance(t, int) and t > 0
                assert not src.endswith("_valu_pmc.json")


def test_work_roofline_from_committed_counters():
    r = bench.work_roofline(bench.CONFIGS2, 13.5, {"lane": {"clock_ghz": 2.34}})
    if r is None:  # no SQ summary committed for configs[2]
        return
    assert r["valu_wave_insts_per_run"] > 0 and 0 < r["frac"] < 1
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    assert r["src"].endswith("_valu_pmc.json")
    assert bench.work_roofline(bench.CONFIGS2, 0.0, {}) is None


def test_roofline_names_the_binding_bound():
    rf = bench.roofline(bench.CONFIGS1, 1 << 30, [0.27, 0.1, 10.0],
                        "serial SHA-256 chain (HBM frac reported)")
    assert rf["roof"] == "hbm" and rf["bound"].startswith("serial")
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-4
