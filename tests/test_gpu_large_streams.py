"""Streams longer than 4 GiB: every stream offset, length and candidate position past 2^32.

The C ABI carries offsets as uint64; the kernels keep candidate positions segment-relative in
40-bit fields (bsgpu_internal.h: a segment lies whole in device memory) and add the segment's
u64 stream offset when boundaries are formed, so a stream has no length limit, as
split.Writer.Write has none (split/split.go:99-101). A 4.5 GiB + ragged stream is split
  * device-resident in one engine run (the bench path),
  * streamed from host memory through bsg_write in 64 MiB Writes (the cgo boundary),
  * through the C++ split.Writer into store/mem (Root),
and each result is compared bit-exactly with the C oracle on the same bytes (one oracle pass,
about 10 s on one host core).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 0x4D1C
N = (9 << 29) + 77_777  # 4.5 GiB + a ragged end


@pytest.fixture(scope="module")
def big(oracle, table):
    from bs_amd.synth import splitmix_array
    d = splitmix_array(SEED, N)
    want = oracle.split(table, d, bits=16, min_size=1024)
    return d, want


def _same(ch, want):
    assert len(ch) == len(want)
    for f in ("offset", "len", "level", "ref"):
        assert (ch[f] == want[f]).all(), f
    assert int(ch["offset"][-1]) > (1 << 32)  # chunks really sit past 4 GiB
    assert int(ch["len"].sum()) == N


def test_engine_stream_over_4gib(gpu, big):
    d, want = big
    buf = gpu.DeviceBuffer(N)
    eng = gpu.Engine()
    gpu.fill_splitmix(buf.ptr, N, SEED, stream=eng.stream)
    eng.run(buf.ptr, [0], [N])
    eng.finish()
    ch, counts = eng.chunks(), eng.counts()
    eng.close()
    tail = buf.to_host()[N - (1 << 20):]
    buf.free()
    assert np.array_equal(tail, d[N - (1 << 20):])  # the device bytes are the oracle's bytes
    assert int(counts[0]) == len(ch)
    _same(ch, want)


def test_streaming_write_over_4gib(gpu, big):
    d, want = big
    w = gpu.StreamingSplitter(bits=16, min_size=1024)
    got = []
    mv = memoryview(d)
    for i in range(0, N, 64 << 20):
        w.write(mv[i:i + (64 << 20)])
        got.append(w.drain())
    w.close()
    got.append(w.drain())
    w.free()
    _same(np.concatenate(got), want)


def test_writer_root_over_4gib(gpu, oracle, table, big):
    d, want = big
    st = gpu.MemStore()
    w = gpu.Writer(st)
    mv = memoryview(d)
    for i in range(0, N, 32 << 20):
        w.write(mv[i:i + (32 << 20)])
    w.close()
    root = w.root
    nblobs = len(st)
    w.free()
    st.free()
    want_root, _ = oracle.writer_root(table, d, bits=16, min_size=1024, fanout=8)
    assert root == want_root
    assert nblobs > len(want)  # every chunk (random bytes: no duplicates) and the tree nodes


BASE40 = (1 << 40) - (32 << 20)  # 32 MiB before 2^40: the stream crosses 1 TiB in its middle


@pytest.fixture(scope="module")
def past_tib(oracle, table):
    from bs_amd.synth import splitmix_array
    d = splitmix_array(0x7E40, (64 << 20) + 4_321)
    return d, oracle.split(table, d, bits=16, min_size=1024)


@pytest.mark.parametrize("base,tile,carry_cap", [
    (BASE40, None, None),             # one 256 MiB tile: records formed across 2^40
    (BASE40, 8 << 20, None),          # 8 MiB tiles: open chunks carried as device bytes
    (BASE40, 8 << 20, 0),             #   ... and as SHA-256 midstates
    ((3 << 40) + 7, 4 << 20, None),   # an unaligned base far past 2^40
])
def test_streaming_past_2_40(gpu, past_tib, base, tile, carry_cap):
    """a stream at offsets past 2^40 (bsg_set_stream_base) splits into the
    oracle's chunks, each offset shifted by the base (the split depends only on the bytes).
    Before round 4 the library refused any stream reaching 1 TiB with BSG_EINVAL."""
    d, want = past_tib
    w = gpu.StreamingSplitter(bits=16, min_size=1024, tile=tile, carry_cap=carry_cap)
    w.set_stream_base(base)
    got = []
    mv = memoryview(d)
    for i in range(0, len(d), 5 << 20):
        w.write(mv[i:i + (5 << 20)])
        got.append(w.drain())
    w.close()
    got.append(w.drain())
    w.free()
    ch = np.concatenate(got)
    assert len(ch) == len(want)
    assert (ch["offset"] == want["offset"] + np.uint64(base)).all()
    for f in ("len", "level", "ref"):
        assert (ch[f] == want[f]).all(), f
    if base == BASE40:
        assert int(ch["offset"][0]) < (1 << 40) < int(ch["offset"][-1])


@pytest.mark.parametrize("base", [BASE40, (5 << 40) + 12_345])
def test_writer_past_2_40(gpu, oracle, table, past_tib, base):
    """split::Writer with its context's stream at offsets past 2^40: every chunk is stored and
    the Root equals the oracle's (the tree's offsets start at 0, as split.Writer's)."""
    d, want = past_tib
    st = gpu.MemStore()
    w = gpu.Writer(st, tile=8 << 20)
    w.set_stream_base(base)
    mv = memoryview(d)
    for i in range(0, len(d), 3 << 20):
        w.write(mv[i:i + (3 << 20)])
    w.close()
    root = w.root
    nblobs = len(st)
    w.free()
    st.free()
    want_root, _ = oracle.writer_root(table, d, bits=16, min_size=1024, fanout=8)
    assert root == want_root
    assert nblobs > len(want)
