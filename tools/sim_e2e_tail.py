#!/usr/bin/env python3
"""How much could the end-to-end (host memory -> records) streaming rate gain by starting each
chunk's SHA-256 chain earlier? CPU only.

Splits the bench's e2e stream (SplitMix64, seed 0xB5B52026, default params) with the C oracle
(used here only for the chunk lengths) and computes when the last chain ends if every chunk's
chain starts once the granule holding the chunk's START has landed on the device (H2D at the
measured 57 GB/s, in stream order) plus the scan/selection latency, and runs at the solo chain's
measured 1.115 us per 64-byte block; a chain can never end before its chunk's end has landed.

  tile256   today: a chunk's chain starts after its whole 256 MiB tile has landed and been scanned
  stage64   per 64 MiB staging buffer
  stage16   per 16 MiB
  start     the ideal: as soon as the chunk's first byte has landed

Then the tile-size sweep of today's pipeline: tile t runs on engine t mod 3 (three tiles in
flight) once it has landed and that engine's previous tile has finished; a chunk's chain starts
after the scan of the tile it closes in (an open chunk is carried into the next tile) and the
tile ends with its longest chain.

  python tools/sim_e2e_tail.py [--gib 1 4] [--h2d-gbs 57] [--us-per-block 1.115]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=int, nargs="+", default=[1, 4])
    ap.add_argument("--h2d-gbs", type=float, default=57.0)
    ap.add_argument("--us-per-block", type=float, default=1.115)
    ap.add_argument("--scan-ms", type=float, default=0.15, help="scan + selection of a granule")
    args = ap.parse_args()
    from oracle import oracle as O  # checker library: chunk lengths only
    from bs_amd.synth import splitmix_array
    table = O.buzhash32_table(1)
    h2d = args.h2d_gbs * 1e9
    for gib in args.gib:
        n = gib << 30
        ch = O.split(table, splitmix_array(0xB5B52026, n), with_refs=False)
        off = ch["offset"].astype(np.float64)
        ln = ch["len"].astype(np.float64)
        chain = (np.floor((ln + 8) / 64) + 1) * args.us_per_block * 1e-6
        print(f"{gib} GiB: {len(ch)} chunks, H2D alone {n / h2d * 1e3:.2f} ms")
        for name, gran in (("tile256", 256 << 20), ("stage64", 64 << 20),
                           ("stage16", 16 << 20), ("start", 1)):
            landed = np.minimum((np.floor(off / gran) + 1) * gran, n) / h2d
            t0 = landed + (args.scan_ms * 1e-3 if gran > 1 else 0.05e-3)
            end = np.maximum(t0 + chain, (off + ln) / h2d + args.scan_ms * 1e-3)
            i = int(np.argmax(end))
            print(f"  {name:8s} last chain ends {end.max() * 1e3:7.2f} ms = "
                  f"{n / end.max() / 2**30:5.1f} GiB/s (chunk of {ln[i] / 1e3:.0f} KB at "
                  f"{off[i] / 2**20:.0f} MiB)")
        cend = (off + ln).astype(np.int64)
        for tile_mib in (64, 128, 192, 256, 320, 512):
            tile = tile_mib << 20
            ntiles = -(-n // tile)
            t_of = (cend - 1) // tile
            tend = np.zeros(ntiles)
            for t in range(ntiles):
                st = max(min((t + 1) * tile, n) / h2d, tend[t - 3] if t >= 3 else 0.0)
                sel = t_of == t
                tend[t] = st + args.scan_ms * 1e-3 + (chain[sel].max() if sel.any() else 0.0)
            print(f"  today's pipeline, tile {tile_mib:3d} MiB: {tend.max() * 1e3:7.2f} ms = "
                  f"{n / tend.max() / 2**30:5.1f} GiB/s")


if __name__ == "__main__":
    main()
