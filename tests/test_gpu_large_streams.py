"""Streams longer than 4 GiB: every stream offset, length and candidate position past 2^32.

The C ABI carries offsets as uint64 and the kernels keep candidate positions in 40-bit fields
(bsgpu_internal.h, 1 TiB per stream). A 4.5 GiB + ragged stream is split
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
