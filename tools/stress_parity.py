"""Long randomized parity run (not part of pytest): many seeded draws of batch splits, streaming
splits and (round 3) C++ split.Writer runs with small and large Writes mixed, against the
oracle. python tools/stress_parity.py [N] [seed_base] -- prints a line per 20 draws.
STRESS_WRITER=0 restores the round-1/2 mix (batch and streaming draws only). Round 4: a third of
the streaming and Writer draws start their stream at a random offset past 2^40
(bsg_set_stream_base): streaming records must be the oracle's shifted by it, Writer Roots equal;
every 10th draw is instead a device-resident engine run of 256-320 MiB over 1-6 streams, the
size at which the early chains (BSG_KNOB_EARLY) take the longest sure chunks to a second stream
(STRESS_ENGINE=0 leaves them out)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bs_amd import bsgpu  # noqa: E402
from bs_amd.synth import splitmix_array, splitmix_bytes  # noqa: E402
from oracle import oracle as O  # noqa: E402


def tuples(ch):
    return [(int(c["offset"]), int(c["len"]), int(c["level"]), bytes(c["ref"])) for c in ch]


def main():
    n_draws = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    seed_base = int(sys.argv[2]) if len(sys.argv) > 2 else 70_000  # new draws: another base
    table = O.buzhash32_table(1)
    t0 = time.time()
    for d in range(n_draws):
        rng = np.random.default_rng(seed_base + d)
        bits = int(rng.integers(10, 23))
        mn = int(rng.choice([64, 512, 1024, 4096]))
        if rng.random() < 0.1:   # the full ranges split.Bits / split.MinSize accept
            bits = int(rng.choice([4, 6, 8, 12, 33, 40]))
            mn = int(rng.choice([1, 17, 63, 64]))
        kind = d % 3 if os.environ.get("STRESS_WRITER", "1") == "1" else d % 2
        if d % 10 == 9 and os.environ.get("STRESS_ENGINE", "1") == "1":
            kind = 3
        if kind == 3:  # device-resident engine run >= 256 MiB: early chains beside selection
            bits = int(rng.integers(10, 23))  # (records the Python comparison can hold)
            mn = int(rng.choice([64, 512, 1024, 4096, 65536]))
            ns = int(rng.integers(1, 7))
            total = int(rng.integers(256 << 20, 320 << 20))
            cuts = np.sort(rng.integers(0, total, size=ns - 1))
            lens = [int(x) for x in np.diff(np.concatenate([[0], cuts, [total]]))]
            offs, span = [], 0
            for n in lens:
                offs.append(span)
                span += (n + 15) & ~15
            buf = bsgpu.DeviceBuffer(span + 4096)
            eng = bsgpu.Engine()
            seed0 = 4_000_000 + 97 * d
            for i, (o, n) in enumerate(zip(offs, lens)):
                bsgpu.fill_splitmix(buf.ptr + o, n, seed0 + i, stream=eng.stream)
            eng.run(buf.ptr, offs, lens, bits=bits, min_size=mn)
            eng.finish()
            ch, counts = eng.chunks(), eng.counts()
            k = 0
            for i, n in enumerate(lens):
                want = tuples(O.split(table, splitmix_array(seed0 + i, n), bits=bits, min_size=mn))
                got = tuples(ch[k:k + int(counts[i])])
                assert got == want, ("engine", d, i, bits, mn, lens)
                k += int(counts[i])
            eng.close()
            buf.free()
        elif kind == 2:  # the C++ split.Writer: Writes of 1 KB to 9 MiB mixed, tiles 64 KiB-256 MiB
            n = int(rng.integers(0, 40_000_000))
            data = splitmix_array(3_000_000 + d, n)
            tile = int(rng.choice([65536, 1 << 20, 5 << 20, 16 << 20, 256 << 20]))
            fo = int(rng.choice([2, 4, 8]))
            st = bsgpu.MemStore()
            w = bsgpu.Writer(st, bits=bits, min_size=mn, fanout=fo, tile=tile)
            if rng.random() < 1 / 3:
                w.set_stream_base(int(rng.integers(1 << 40, 1 << 50)))
            mv = memoryview(data)
            pos = 0
            while pos < n:
                k = int(rng.choice([1000, 65536, 1 << 20, 4 << 20, 9 << 20]))
                w.write(mv[pos:pos + k])
                pos += k
            w.close()
            want, _ = O.writer_root(table, data, bits=bits, min_size=mn, fanout=fo)
            assert w.root == want, ("writer", d, bits, mn, fo, n, tile)
            w.free()
            st.free()
        elif kind == 0:  # batch of streams, lengths up to 8 MB
            ns = int(rng.integers(1, 40))
            lens = [int(x) for x in rng.integers(0, 8_000_000, size=ns)]
            arrs = [splitmix_array(1_000_000 + 97 * d + i, n) for i, n in enumerate(lens)]
            ch, counts = bsgpu.split_hash_batch(arrs, bits=bits, min_size=mn)
            k = 0
            for i, a in enumerate(arrs):
                want = tuples(O.split(table, a, bits=bits, min_size=mn))
                got = tuples(ch[k:k + int(counts[i])])
                assert got == want, ("batch", d, i, bits, mn, len(a))
                k += int(counts[i])
        else:  # one stream through the streaming Writer
            n = int(rng.integers(0, 24_000_000))
            data = splitmix_bytes(2_000_000 + d, n)
            tile = int(rng.choice([65536, 1 << 20, 16 << 20]))
            w = bsgpu.StreamingSplitter(bits=bits, min_size=mn, tile=tile)
            base = int(rng.integers(1 << 40, 1 << 50)) if rng.random() < 1 / 3 else 0
            if base:
                w.set_stream_base(base)
            pos, got = 0, []
            while pos < n:
                k = int(rng.choice([4096, 100_000, 4 << 20]))
                w.write(data[pos:pos + k])
                pos += k
                got.append(w.drain())
            w.close()
            got.append(w.drain())
            w.free()
            want = [(o + base, ln, lv, r) for o, ln, lv, r in
                    tuples(O.split(table, np.frombuffer(data, dtype=np.uint8), bits=bits, min_size=mn))]
            assert tuples(np.concatenate(got)) == want, ("stream", d, bits, mn, n, tile, base)
        if d % 20 == 19:
            print(f"{d + 1} draws ok ({time.time() - t0:.0f} s)", flush=True)
    print(f"all {n_draws} draws bit-identical to the oracle", flush=True)


if __name__ == "__main__":
    main()
