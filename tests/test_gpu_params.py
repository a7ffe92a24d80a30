"""The full parameter ranges split.Bits / split.MinSize accept, on the HIP path vs the oracle.

split/split.go:137-152 store Bits(n) and MinSize(n) in the Splitter unchecked ("The value must
be 64 or higher" is advice, not a check), and hashsplit's Splitter turns 0 into its own
defaults (SplitBits 13, MinSize 64). So the drop-in must produce the reference's chunks for:
  * MinSize 1..63: the 64-byte window spans chunk boundaries; the hash is still a function of
    the last 64 stream bytes (no reset between chunks), only the greedy rule changes;
  * Bits 33 and up (uint in Go, clamped to 2^32-1 by a cgo caller): TrailingZeros32 is at most
    32, so nothing ever splits and the stream is one final chunk of level 0;
  * zeros: the hashsplit defaults.
Every case goes through the batch API, the streaming Writer path (tiles, carries) and the C++
split.Writer (Root vs the oracle's TreeBuilder restatement).
"""
import numpy as np
import pytest

from test_oracle import EDGE_PARAMS, edge_stream

pytestmark = pytest.mark.gpu


def as_tuples(ch):
    return [(int(c["offset"]), int(c["len"]), int(c["level"]), bytes(c["ref"]).hex()) for c in ch]


@pytest.mark.parametrize("bits,mn", EDGE_PARAMS)
def test_batch_edge_params(gpu, oracle, table, bits, mn):
    lens = [0, 1, 2, 63, 64, 65, 130, 1000, 5000, 70_001, 300_000]
    arrs = [np.frombuffer(edge_stream(900 + i, n), dtype=np.uint8) for i, n in enumerate(lens)]
    ch, counts = gpu.split_hash_batch(arrs, bits=bits, min_size=mn)
    k = 0
    for i, a in enumerate(arrs):
        one = oracle.split(table, a, bits=bits, min_size=mn)
        got = ch[k:k + int(counts[i])]
        assert as_tuples(got) == as_tuples(one), (bits, mn, lens[i])
        k += int(counts[i])
    assert k == len(ch)


@pytest.mark.parametrize("bits,mn", EDGE_PARAMS)
def test_streaming_edge_params(gpu, oracle, table, bits, mn):
    data = edge_stream(1234 + mn, 400_003)
    want = as_tuples(oracle.split(table, data, bits=bits, min_size=mn))
    rng = np.random.default_rng(bits % 1000 + mn)
    for tile, carry_cap in ((4096, None), (65536 + 3, 0), (1 << 20, 5000)):
        w = gpu.StreamingSplitter(bits=bits, min_size=mn, tile=tile, carry_cap=carry_cap)
        pos, got = 0, []
        while pos < len(data):
            k = int(rng.choice([1, 63, 64, 1000, 4096, 70_000]))
            w.write(data[pos:pos + k])
            pos += k
            got.append(w.drain())
        w.close()
        got.append(w.drain())
        w.free()
        assert as_tuples(np.concatenate(got)) == want, (bits, mn, tile, carry_cap)


@pytest.mark.parametrize("bits,mn,fanout", [(4, 1, 2), (6, 17, 1), (33, 64, 8), (0, 0, 8),
                                            (10, 63, 3)])
def test_writer_edge_params(gpu, oracle, table, bits, mn, fanout):
    data = edge_stream(55 + mn, 120_000)
    st = gpu.MemStore()
    w = gpu.Writer(st, bits=bits, min_size=mn, fanout=fanout)
    for i in range(0, len(data), 32 * 1024):
        w.write(data[i:i + 32 * 1024])
    w.close()
    ch = oracle.split(table, data, bits=bits, min_size=mn)
    store = {}
    want = oracle.py_tree_root(
        [(data[int(c["offset"]):int(c["offset"] + c["len"])], int(c["level"])) for c in ch],
        fanout, store)
    assert w.root == want
    assert sorted(st.refs()) == sorted(store)
    assert gpu.Reader(st, w.root, verify=True).read_all() == data
