"""Randomized parity over batches large enough for k_sha's per-lane address regions (span over
1 GiB, R >= 2; not part of pytest): seeded draws of stream count / lengths / Bits / MinSize,
every record compared with the oracle (threaded C restatement).
python tools/stress_regions.py [N] [seed_base] -- prints one line per draw."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bs_amd import bsgpu  # noqa: E402
from bs_amd.synth import splitmix_array  # noqa: E402
from oracle import oracle as O  # noqa: E402


def main():
    n_draws = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    seed_base = int(sys.argv[2]) if len(sys.argv) > 2 else 90_000
    table = O.buzhash32_table(1)
    threads = max(1, min(int(os.environ.get("OMP_NUM_THREADS", "16")), os.cpu_count() or 1))
    t0 = time.time()
    for d in range(n_draws):
        rng = np.random.default_rng(seed_base + d)
        bits = int(rng.choice([12, 14, 16, 16, 18]))
        mn = int(rng.choice([64, 1024, 4096]))
        ns = int(rng.integers(3, 48))
        total = int(rng.integers(1200, 2600)) << 20          # 1.2 - 2.5 GiB per batch
        cuts = np.sort(rng.integers(0, total, size=ns - 1))
        lens = np.diff(np.concatenate([[0], cuts, [total]])).astype(np.int64)
        base = np.empty(total, dtype=np.uint8)
        off = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
        for i, n in enumerate(lens):
            base[int(off[i]):int(off[i]) + int(n)] = splitmix_array(3_000_000 + 131 * d + i, int(n))
        arrs = [base[int(off[i]):int(off[i]) + int(lens[i])] for i in range(ns)]
        ch, counts = bsgpu.split_hash_batch(arrs, bits=bits, min_size=mn)
        want, wcounts = O.split_streams(table, base, off, lens, bits=bits, min_size=mn,
                                        threads=threads)
        assert (np.asarray(counts, dtype=np.uint64) == wcounts).all(), ("counts", d)
        for f in ("offset", "len", "level", "stream", "ref"):
            assert (ch[f] == want[f]).all(), ("field", f, d, bits, mn, ns, total)
        print(f"draw {d}: {ns} streams, {total >> 20} MiB, bits {bits}, min {mn}, "
              f"{len(ch)} chunks ok ({time.time() - t0:.0f} s)", flush=True)
    print(f"all {n_draws} region draws bit-identical to the oracle", flush=True)


if __name__ == "__main__":
    main()
