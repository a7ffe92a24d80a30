#!/usr/bin/env python3
"""How much could configs[2] gain by starting the long SHA-256 chains before the batch's scan
ends? CPU only.

Splits the bench's 256 x 64 MiB streams (SplitMix64, seeds 0xB5B52026 + s, default params) with
the C oracle (checker code, used here only to get the chunk lengths), then computes the time at
which the last chain would end under several schedules, from measured stage costs:

  one batch (today)      every chain starts after the whole scan + selection
  G stream groups        group g is scanned g-th; its chains start after its own scan
  P position phases      phase p scans every stream's p-th 1/P; the chains of the chunks that
                         closed in it start after its selection
  position-major         all streams scanned front to back together; a chunk's chain starts
                         once the scan front has passed its end (its length is known)

The chain bound of each schedule is printed, then the work bound: the scan and the per-lane
SHA-256 blocks share the chip, at the per-lane throughput measured by tools/ubench/lanes_occ.hip.

  python tools/sim_early_chain.py [--scan-ms 3.73] [--sel-ms 0.27] [--us-per-block 1.16]
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

BASE_SEED = 0xB5B52026
CACHE = "/tmp/bs_amd_configs2_chunks.npy"


def chunk_table(streams: int, stream_mib: int, threads: int) -> np.ndarray:
    """(stream, offset, len) of every chunk of the bench's configs[2] batch."""
    if os.path.exists(CACHE):
        return np.load(CACHE)
    from oracle import oracle as O  # checker library, used for the chunk lengths only
    from bs_amd.synth import splitmix_array
    table = O.buzhash32_table(1)
    n = stream_mib << 20
    rows = []
    t0 = time.time()
    for g in range(0, streams, 16):
        ids = list(range(g, min(streams, g + 16)))
        base = np.concatenate([splitmix_array(BASE_SEED + i, n) for i in ids])
        off = np.arange(len(ids), dtype=np.uint64) * n
        ch, counts = O.split_streams(table, base, off, [n] * len(ids), threads=threads)
        k = 0
        for j, s in enumerate(ids):
            c = int(counts[j])
            for o, ln in zip(ch["offset"][k:k + c], ch["len"][k:k + c]):
                rows.append((s, int(o), int(ln)))
            k += c
        print(f"  streams {ids[0]}..{ids[-1]} split ({time.time() - t0:.0f} s)", file=sys.stderr)
    a = np.array(rows, dtype=np.int64)
    np.save(CACHE, a)
    return a


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=256)
    ap.add_argument("--stream-mib", type=int, default=64)
    ap.add_argument("--scan-ms", type=float, default=3.76, help="k_scan + k_refine, whole batch")
    ap.add_argument("--sel-ms", type=float, default=0.27, help="selection kernels")
    ap.add_argument("--us-per-block", type=float, default=1.157, help="solo-chain block time")
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--lane-rate1", type=float, default=23.8, help="k blocks/us, 1 wave/SIMD")
    ap.add_argument("--lane-rate3", type=float, default=27.8, help="k blocks/us, 3 waves/SIMD")
    ap.add_argument("--wave-min-blocks", type=int, default=4065,
                    help="jobs this long go to wave tickets (bench sha_path.long_thresh)")
    ap.add_argument("--tickets", type=int, default=240, help="wave tickets (sha_path)")
    ap.add_argument("--simds", type=int, default=1024)
    ap.add_argument("--clock-ghz", type=float, default=2.31, help="k_sha's loaded clock")
    args = ap.parse_args()

    a = chunk_table(args.streams, args.stream_mib, args.threads)
    s, o, ln = a[:, 0], a[:, 1], a[:, 2]
    nb = (ln + 8) // 64 + 1  # SHA-256 compressions per chunk
    top = np.argsort(-nb)[:8]
    L = args.stream_mib << 20
    blk = args.us_per_block * 1e-3
    print(f"{len(a)} chunks; longest (blocks, stream, offset MiB): " +
          ", ".join(f"({nb[i]}, {s[i]}, {o[i] / 2**20:.1f})" for i in top))
    print(f"stage costs: scan {args.scan_ms} ms, selection {args.sel_ms} ms, "
          f"{args.us_per_block} us per chain block")
    print("schedule                                  last chain ends (ms)")
    one = args.scan_ms + args.sel_ms + nb.max() * blk
    print(f"  one batch (today)                        {one:.3f}")
    for G in (2, 4, 8, 16, 32, 64, args.streams):
        grp = s * G // args.streams
        end = (grp + 1) / G * args.scan_ms + args.sel_ms + nb * blk
        print(f"  {G:3d} stream groups scanned in turn         {end.max():.3f}")
    for P in (2, 3, 4, 6, 8, 16):
        ph = np.minimum(((o + ln - 1) * P) // L, P - 1)  # the phase in which the chunk closes
        end = (ph + 1) / P * args.scan_ms + args.sel_ms + nb * blk
        print(f"  {P:3d} position phases                      {end.max():.3f}")
    fr = (o + ln) / L * args.scan_ms + args.sel_ms + nb * blk
    print(f"  position-major, chain at its chunk's end {fr.max():.3f}")
    # a chain needs its chunk's START, not its end. With a position-major
    # scan the front passes a chunk in len / (L / scan_ms), so starting at the start can gain
    # at most that (a 766 KB chunk: 0.04 ms).
    fs = o / L * args.scan_ms + args.sel_ms + nb * blk
    print(f"  position-major, chain at its chunk's start {fs.max():.3f}")

    # The work bound: the chip must also do the scan and every per-lane SHA-256 block, and the
    # two share it (both VALU-bound). Per-lane throughput from tools/ubench/lanes_occ.hip
    # (profiles/r03_lanes_occ.log): 23.8 k blocks/us chip-wide at one wave per SIMD (k_sha's
    # occupancy), 27.8 k at three; a SIMD running a wave-mode chain does ~1/28 of a per-lane
    # SIMD's blocks, so the tickets' SIMDs are (nearly) lost to the per-lane work while they run.
    blocks = int(nb.sum())
    lane_blocks = blocks - int(nb[nb >= args.wave_min_blocks].sum())
    print(f"work bound: {blocks / 1e6:.1f} M blocks in all, {lane_blocks / 1e6:.1f} M per-lane "
          f"(jobs under {args.wave_min_blocks} blocks)")
    for occ, rate in (("1 wave/SIMD", args.lane_rate1), ("3 waves/SIMD", args.lane_rate3)):
        lane_ms = lane_blocks / (rate * 1e6)
        busy = args.tickets / args.simds  # share of the chip the wave tickets hold
        t_sha = lane_ms / (1 - busy)
        print(f"  {occ:13s}: per-lane work {lane_ms:.2f} ms of full chip, {t_sha:.2f} ms with "
              f"{args.tickets} SIMDs on wave tickets; scan + selection + SHA-256 = "
              f"{args.scan_ms + args.sel_ms + t_sha:.2f} ms")
    print("  a step can end no earlier than the larger of the chain bound of its schedule and "
          "the work bound")

    # Round 4: the hash work with k_sha's actual tiers and their measured costs (wave-cycles per
    # block, DESIGN §4.4: per-lane 6,870 cycles per 64 blocks under full load; pair tickets ~133;
    # group (octet) tickets ~380; a solo chain holds its wave for 2,702 cycles per block), at the
    # loaded clock. It is what k_sha's whole chip has to do while the longest chain runs.
    mx = int(nb.max())
    order = np.argsort(-nb)
    solo = np.zeros(len(nb), dtype=bool)
    solo[order[:16]] = True
    grp = (nb >= mx * 0.50) & ~solo
    pair = (nb >= mx * 0.34) & (nb < mx * 0.50)
    lane = nb < mx * 0.34
    ghz = args.clock_ghz
    tiers = (("per-lane", lane, 6870 / 64), ("pair tickets", pair, 133.0),
             ("group tickets", grp, 380.0), ("solo chains", solo, 2702.0))
    total = 0.0
    print(f"tiered hash work at {ghz} GHz on {args.simds} SIMDs (full-chip ms):")
    for name, m, cyc in tiers:
        ms = float(nb[m].sum()) * cyc / args.simds / (ghz * 1e6)
        total += ms
        print(f"  {name:14s} {int(m.sum()):7d} jobs {nb[m].sum() / 1e6:7.2f} M blocks "
              f"x {cyc:6.0f} cycles = {ms:6.2f} ms")
    chain = mx * 2702 / (ghz * 1e6)
    print(f"  hash work {total:.2f} ms against the longest chain {chain:.2f} ms: the two bounds "
          f"of k_sha coincide (measured k_sha 14.03 ms, driver round 3)")
    q = (nb >= mx * 0.50) & (nb < mx * 0.74) & ~solo
    saved = float(nb[q].sum()) * (380.0 - 190.0) / args.simds / (ghz * 1e6)
    print(f"  a quad tier (16 chains per wave, ~190 cycles per block) for the jobs between 0.50 and "
          f"0.74 x the longest would save {saved:.2f} ms of it")


if __name__ == "__main__":
    main()
