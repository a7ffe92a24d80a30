"""Candidates planted at every offset 0..63 of a strip's start, against the oracle.

k_scan gives each lane a 2 KiB strip (kStrip). A strip's first 63 positions hash windows that
start in the strip before it, and round 5's chained strips (BSG_SCAN_CHAIN) check those
positions on the previous lane, which runs its hash on past its own end, while the strip's own
lane checks only position 63 after warming up on its block 0. These tests plant 64-byte windows
whose buzhash32 has its low `low` bits zero so that they END at offset k = j mod 64 of strip j,
over streams whose strips start at every lane of a wave (the streams' lengths shift the strip
grid), and compare the HIP records with the oracle's. A window's hash does not depend on where
it sits (closed form, oracle.py:_window_hash: h(p) = XOR_k rotl(T[x[p-k]], k mod 32)), so the
planted position is a candidate whatever precedes it; the test checks that the oracle agrees
(most planted positions end a chunk) before it compares.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

STRIP = 2048


def _rotl(x, r):
    r %= 32
    if r == 0:
        return x
    return ((x << np.uint32(r)) | (x >> np.uint32(32 - r))).astype(np.uint32)


def zero_windows(table, count, low, seed):
    """`count` 64-byte windows whose window hash has its `low` low bits zero: 62 random bytes,
    then the two last bytes searched over all 65,536 pairs."""
    T = np.asarray(table, dtype=np.uint32)
    mask = np.uint32((1 << low) - 1)
    rng = np.random.default_rng(seed)
    a62 = _rotl(T, 1)          # byte 62 (one step before the newest): rotl 1
    out = []
    while len(out) < count:
        pre = rng.integers(0, 256, 62, dtype=np.uint8)
        h = np.uint32(0)
        for i, b in enumerate(pre):
            h ^= _rotl(np.array([T[b]], dtype=np.uint32), 63 - i)[0]
        hh = (h ^ a62[:, None] ^ T[None, :]) & mask   # [b62, b63]
        hit = np.argwhere(hh == 0)
        if len(hit):
            b62, b63 = hit[rng.integers(0, len(hit))]
            out.append(np.concatenate([pre, np.array([b62, b63], dtype=np.uint8)]))
    return out


def planted_stream(table, n, low, seed):
    """n random bytes with a zero window ending at offset (j mod 64) of every strip j >= 1 that
    holds it; returns (bytes, planted end positions)."""
    rng = np.random.default_rng(seed + 7)
    data = rng.integers(0, 256, n, dtype=np.uint8)
    ends = [STRIP * j + (j % 64) for j in range(1, n // STRIP + 1) if STRIP * j + (j % 64) < n]
    wins = zero_windows(table, len(ends), low, seed)
    for p, w in zip(ends, wins):
        data[p - 63:p + 1] = w
    return data, ends


def _tuples(ch):
    return [(int(c["offset"]), int(c["len"]), int(c["level"]), bytes(c["ref"]).hex()) for c in ch]


@pytest.mark.parametrize("bits,min_size,low", [(16, 1024, 16), (16, 64, 16), (12, 256, 12),
                                               (20, 1024, 16)])
def test_strip_start_candidates(gpu, oracle, table, bits, min_size, low):
    # stream lengths chosen so that consecutive streams start their strips at different lanes
    # of a wave (a stream of 2048 * k + r bytes takes k or k + 1 strips)
    lens = [STRIP * 70 + 5, STRIP * 37, STRIP * 64 + 64, STRIP * 3 + 127, STRIP * 101 + 1,
            STRIP * 1 + 200, STRIP * 130 + 2047, STRIP * 9 + 63, STRIP * 66 + 128]
    arrs, planted = [], []
    for i, n in enumerate(lens):
        d, ends = planted_stream(table, n, low, 1000 * bits + i)
        arrs.append(d)
        planted.append(ends)
    ch, counts = gpu.split_hash_batch(arrs, bits=bits, min_size=min_size)
    k = 0
    hit_ends = 0
    n_ends = 0
    for i, a in enumerate(arrs):
        want = oracle.split(table, a, bits=bits, min_size=min_size)
        got = ch[k:k + int(counts[i])]
        k += int(counts[i])
        assert _tuples(got) == _tuples(want), (bits, min_size, lens[i])
        if low >= bits:
            chunk_ends = {int(c["offset"]) + int(c["len"]) - 1 for c in want}
            hit_ends += sum(p in chunk_ends for p in planted[i])
            n_ends += len(planted[i])
    assert k == len(ch)
    if n_ends:  # the planting works: most planted positions end a chunk
        assert hit_ends >= 0.9 * n_ends, (hit_ends, n_ends)


def test_strip_start_candidates_streaming(gpu, oracle, table):
    """The same planted stream through the streaming Writer path (tiles, carries)."""
    data, _ = planted_stream(table, STRIP * 700 + 333, 16, 4242)
    want = _tuples(oracle.split(table, data, bits=16, min_size=1024))
    w = gpu.StreamingSplitter(bits=16, min_size=1024, tile=1 << 20, carry_cap=1 << 16)
    got = []
    for i in range(0, len(data), 300_001):
        w.write(data[i:i + 300_001])
        got.append(w.drain())
    w.close()
    got.append(w.drain())
    w.free()
    assert _tuples(np.concatenate(got)) == want
