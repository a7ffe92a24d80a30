"""Summarise rocprofv3 kernel-trace stats and FETCH_SIZE / WRITE_SIZE passes into profiles/.

Usage: python tools/pmc_summary.py --round r01 [--src gpurun_out]

Reads  <src>/prof_trace/run_kernel_stats.csv            (rocprofv3 --kernel-trace --stats)
       <src>/prof_fetch/run_counter_collection.csv      (rocprofv3 --pmc FETCH_SIZE)
       <src>/prof_write/run_counter_collection.csv      (rocprofv3 --pmc WRITE_SIZE)
Writes profiles/<round>_kernel_stats.csv (verbatim copy) and profiles/<round>_pmc.json:
  per kernel: launches, FETCH_SIZE / WRITE_SIZE per launch (KiB, raw) and corrected HBM bytes.

Correction (/opt/skills/guides/MI355X_MICROARCH.md, HBM section): on gfx950 FETCH_SIZE counts
exactly half the bytes of a wide coalesced streaming read (128-byte requests tallied at 64), so
FETCH bytes are doubled for the kernels whose loads are 16 B per lane (k_sha, k_sha_blobs,
k_scan, k_refine). k_scan's pattern (each lane streams its own 2 KiB strip, 64 B per block) is
also calibrated on its own: tools/ubench/scan_calib reads a known byte count with exactly that
pattern (k_strips) and with the guide's coalesced pattern (k_coalesced); --calib <dir> reads
that run's FETCH_SIZE pass and reports, per kernel of the strip pattern, its FETCH per
algorithmic byte relative to k_strips'. WRITE_SIZE is exact for 16-B streaming stores.

--rdreq <dir> (round 5): a pass of TCC_EA0_RDREQ split by request size (32/64/128-B,
tools/rdreq_summary.py) gives the read bytes directly (32 x n32 + 64 x n64 + 128 x n128; the
coalesced calibration kernel reads exactly its 1 GiB this way); when given, it replaces the
FETCH_SIZE read bytes of every kernel it saw, and FETCH_SIZE stays in the file as a cross-check.
"""
import argparse
import collections
import csv
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FETCH_X2 = {"bsg::k_sha(bsg::ShaArgs)", "void bsg::k_sha<true>(bsg::ShaArgs)",
            "void bsg::k_sha<false>(bsg::ShaArgs)", "bsg::k_sha_blobs(bsg::BlobShaArgs)",
            "bsg::k_early(bsg::ShaArgs, unsigned int)",
            "void bsg::k_scan<true>(bsg::ScanArgs)", "void bsg::k_scan<false>(bsg::ScanArgs)",
            "bsg::k_refine(bsg::ScanArgs)"}
STRIP_PATTERN = {"void bsg::k_scan<true>(bsg::ScanArgs)", "void bsg::k_scan<false>(bsg::ScanArgs)"}


def _counters(path):
    d = collections.defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            d[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--round", required=True)
    ap.add_argument("--src", default=os.path.join(ROOT, "gpurun_out"))
    ap.add_argument("--workload", default="configs[1]: 1 GiB random stream per GPU")
    ap.add_argument("--bytes", type=float, default=float(1 << 30),
                    help="algorithmic input bytes per launch (stream bytes of the batch)")
    ap.add_argument("--calib", default=None, help="scan_calib FETCH_SIZE run directory")
    ap.add_argument("--rdreq", default=None, help="TCC_EA0_RDREQ-by-size run directory")
    a = ap.parse_args()
    rdreq = None
    if a.rdreq:
        import sys
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        from rdreq_summary import summarise
        rdreq = summarise(a.rdreq, a.bytes)
    calib = None
    if a.calib:
        cf = _counters(os.path.join(a.calib, "run_counter_collection.csv"))
        strips = [v for k, v in cf.items() if k.startswith("k_strips")][0][0]
        coal = [v for k, v in cf.items() if k.startswith("k_coalesced")][0][0]
        alg = float(1 << 30) + ((1 << 30) // 2048 - 1) * 64.0  # strips + warm-up blocks
        calib = {"k_strips_fetch_kib": strips, "k_coalesced_fetch_kib": coal,
                 "k_strips_fetch_per_byte": strips * 1024 / alg,
                 "k_coalesced_fetch_per_byte": coal * 1024 / float(1 << 30)}
    out = os.path.join(ROOT, "profiles")
    os.makedirs(out, exist_ok=True)
    stats = os.path.join(a.src, "prof_trace", "run_kernel_stats.csv")
    shutil.copyfile(stats, os.path.join(out, f"{a.round}_kernel_stats.csv"))
    avg_ns = {}
    with open(stats) as f:
        for r in csv.DictReader(f):
            avg_ns[r["Name"]] = float(r["AverageNs"])
    fetch = _counters(os.path.join(a.src, "prof_fetch", "run_counter_collection.csv"))
    write = _counters(os.path.join(a.src, "prof_write", "run_counter_collection.csv"))
    kernels = {}
    for name in sorted(set(fetch) | set(write)):
        fk = sum(fetch.get(name, [0])) / max(1, len(fetch.get(name, [])))
        wk = sum(write.get(name, [0])) / max(1, len(write.get(name, [])))
        x2 = name in FETCH_X2
        fb = fk * 1024 * (2 if x2 else 1)
        wb = wk * 1024
        corr = "x2 (16 B/lane reads, gfx950)" if x2 else "uncalibrated (raw)"
        if rdreq and name in rdreq:
            fb_fetch = fb
            fb = rdreq[name]["read_bytes_per_launch"]
            corr = f"TCC_EA0_RDREQ by request size (FETCH_SIZE-based: {fb_fetch:.0f} B)"
        kernels[name] = {
            "launches": len(fetch.get(name, [])),
            "fetch_kib_raw": fk, "write_kib_raw": wk,
            "fetch_correction": corr,
            "hbm_bytes_per_launch": fb + wb,
            "read_over_algorithmic": fb / a.bytes,
            "write_bytes_per_launch": wb,
            "avg_ns": avg_ns.get(name),
        }
        if calib and name in STRIP_PATTERN:
            kernels[name]["fetch_vs_strip_calibration"] = (fk * 1024 / a.bytes) / \
                calib["k_strips_fetch_per_byte"]
    doc = {"round": a.round, "workload": a.workload, "algorithmic_bytes_per_launch": a.bytes,
           "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, bench.py "
                     "--steps 1 --warmup 0" + ("; reads from a TCC_EA0_RDREQ_{32B,64B,128B} pass"
                                               if rdreq else ""),
           "strip_pattern_calibration": calib,
           "kernels": kernels}
    with open(os.path.join(out, f"{a.round}_pmc.json"), "w") as f:
        json.dump(doc, f, indent=1)
    for n, k in kernels.items():
        if k["hbm_bytes_per_launch"] > 1e6:
            print(f"{n[:40]:40s} {k['hbm_bytes_per_launch'] / 2**30:8.4f} GiB/launch  avg {k['avg_ns']} ns")


if __name__ == "__main__":
    main()
