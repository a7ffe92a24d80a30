"""Buffer ownership at the C ABI (SURVEY §8b "Ownership").

io.Writer lets the caller reuse its slice as soon as Write returns, and cgo forbids C from
keeping Go pointers, so bsg_write / bsg_writer_write must copy what they need before returning.
Here the caller overwrites its one reusable buffer right after every call (the way io.Copy
reuses its 32 KiB buffer, and the way the round-1 cgo stub wrongly reused its backing array);
chunk records, refs, stored blobs and Root must still equal the oracle's for the original bytes.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def as_tuples(ch):
    return [(int(c["offset"]), int(c["len"]), int(c["level"]), bytes(c["ref"]).hex()) for c in ch]


def _pieces(data: bytes, rng):
    pos = 0
    while pos < len(data):
        k = int(rng.choice([1, 100, 4096, 32 * 1024, 250_000]))
        yield data[pos:pos + k]
        pos += k


@pytest.mark.parametrize("tile", [4096, 65536 + 3, 1 << 20])
def test_bsg_write_copies_before_return(gpu, oracle, table, tile):
    from bs_amd.synth import splitmix_bytes
    data = splitmix_bytes(606, 2_500_000)
    rng = np.random.default_rng(tile)
    scratch = np.empty(250_000, dtype=np.uint8)  # the caller's one reusable buffer
    w = gpu.StreamingSplitter(bits=12, min_size=256, tile=tile)
    got = []
    for piece in _pieces(data, rng):
        view = scratch[:len(piece)]
        view[:] = np.frombuffer(piece, dtype=np.uint8)
        w.write(view)
        view[:] = 0xA5  # reused at once
        got.append(w.drain())
    w.close()
    got.append(w.drain())
    w.free()
    assert as_tuples(np.concatenate(got)) == as_tuples(
        oracle.split(table, data, bits=12, min_size=256))


def test_writer_copies_before_return(gpu, oracle, table):
    """The C++ split.Writer over store/mem: stored blobs (kept by the store, like mem.go:71)
    must be the original bytes, not whatever the caller's buffer holds later."""
    from bs_amd.synth import splitmix_bytes
    data = splitmix_bytes(707, 1_800_000)
    rng = np.random.default_rng(7)
    scratch = np.empty(250_000, dtype=np.uint8)
    st = gpu.MemStore()
    w = gpu.Writer(st, bits=11, min_size=128, fanout=4)
    for piece in _pieces(data, rng):
        view = scratch[:len(piece)]
        view[:] = np.frombuffer(piece, dtype=np.uint8)
        w.write(view)
        view[:] = 0x5A
    w.close()
    ch = oracle.split(table, data, bits=11, min_size=128)
    store = {}
    want = oracle.py_tree_root(
        [(data[int(c["offset"]):int(c["offset"] + c["len"])], int(c["level"])) for c in ch],
        4, store)
    assert w.root == want
    for c in ch:
        o, n = int(c["offset"]), int(c["len"])
        assert st.get(bytes(c["ref"])) == data[o:o + n]
    assert gpu.Reader(st, w.root, verify=True).read_all() == data
