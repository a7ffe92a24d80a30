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

Only the chain bound is modelled: it ignores that per-lane SHA-256 work (which keeps the chip
busy until the chain ends today) would have to shrink as well.

  python tools/sim_early_chain.py [--scan-ms 3.76] [--sel-ms 0.27] [--us-per-block 1.157]
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


if __name__ == "__main__":
    main()
