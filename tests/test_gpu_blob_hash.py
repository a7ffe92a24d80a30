"""Batched Blob.Ref (bs.go:24-26) of many blobs through the engine's hash mode (bsg_engine_hash,
bsg_hasher_sum / _ptrs, bsg_sha256_batch), and the verifying split.Reader that uses it a window
of leaf nodes at a time. Every ref is compared with hashlib (FIPS 180-4)."""
import hashlib
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _blobs(seed: int, n: int, mean: int):
    rng = np.random.default_rng(seed)
    lens = rng.exponential(mean, n).astype(np.int64)
    # SHA-256 padding edges, empty blobs and a few long ones
    edge = [0, 0, 1, 55, 56, 63, 64, 65, 119, 120, 127, 128, 4095, 4096, 1 << 20, 3 << 20]
    k = min(n, len(edge))
    lens[:k] = edge[:k]
    rng.shuffle(lens)
    data = rng.integers(0, 256, int(lens.sum()) + 1, dtype=np.uint8).tobytes()
    out, o = [], 0
    for ln in lens:
        out.append(data[o:o + int(ln)])
        o += int(ln)
    return out


def test_sha256_batch_engine_path(gpu):
    blobs = _blobs(5, 2000, 50_000)  # >= 16 blobs and 4 MiB: packed, bsg_engine_hash mode
    assert sum(map(len, blobs)) > 64 << 20
    got = gpu.sha256_batch(blobs)
    assert got == [hashlib.sha256(b).digest() for b in blobs]


def test_hasher_sum_ptrs_engine_and_small(gpu):
    h = gpu.Hasher()
    try:
        big = _blobs(6, 600, 40_000)
        assert h.sum_ptrs(big) == [hashlib.sha256(b).digest() for b in big]
        small = _blobs(7, 9, 100)  # below the engine threshold: one blob per lane
        small[0] = b""
        assert h.sum_ptrs(small) == [hashlib.sha256(b).digest() for b in small]
        assert h.sum_ptrs(big[:300]) == [hashlib.sha256(b).digest() for b in big[:300]]  # reuse
    finally:
        h.free()


@pytest.fixture(scope="module")
def shared_hasher(gpu):
    h = gpu.Hasher()
    yield h
    h.free()


@pytest.mark.parametrize("total_mib,big_mib", [(262, 0), (700, 0), (180, 330)])
def test_hasher_runs_around_256mib(gpu, shared_hasher, total_mib, big_mib):
    """The engine path splits a host batch into runs of 256 MiB, but takes everything left in
    one run when it is at most a quarter more (a Reader window just over 256 MiB), and a blob
    longer than a run alone; the staging is sized once for the largest run. 262 MiB: one run;
    700 MiB: 256 + 444 -> 256 + 256 + 188; a 330 MiB blob among 180 MiB of others. Every ref
    equals hashlib's, on one persistent hasher reused across the three shapes."""
    rng = np.random.default_rng(total_mib)
    n = (total_mib << 20) // 65_000
    lens = rng.integers(1_000, 129_000, n)
    data = np.frombuffer(rng.bytes(int(lens.sum()) + (big_mib << 20)), dtype=np.uint8)
    blobs, o = [], 0
    for ln in lens:
        blobs.append(data[o:o + int(ln)].tobytes())
        o += int(ln)
    if big_mib:
        blobs.insert(len(blobs) // 2, data[o:o + (big_mib << 20)].tobytes())
    assert shared_hasher.sum_ptrs(blobs) == [hashlib.sha256(b).digest() for b in blobs]


def test_hasher_large_blob_small_path_pins_nothing_big(gpu):
    """the small-batch path is chosen by blob count, so one large blob
    (a single Put, a Reader window with a few long chunks) lands there. Its bytes must be
    copied from pageable memory, not through a blob-sized pinned buffer that the pooled hasher
    would then hold for the life of the process. A 256 MiB + 1 blob, through bsg_hasher_sum and
    bsg_hasher_sum_ptrs (one blob, and three blobs), against hashlib; the hasher's pinned
    memory stays under 8 MiB."""
    rng = np.random.default_rng(11)
    big = rng.bytes((256 << 20) + 1)
    small = [b"", rng.bytes(1000)]
    h = gpu.Hasher()
    try:
        want = hashlib.sha256(big).digest()
        assert h.sum([big]) == [want]
        assert h.sum_ptrs([big]) == [want]
        assert h.sum_ptrs([small[0], big, small[1]]) == [hashlib.sha256(b).digest()
                                                         for b in (small[0], big, small[1])]
        assert h.pinned_bytes() < 8 << 20, h.pinned_bytes()
        # the small path still goes through pinned memory for small blobs, and stays correct
        assert h.sum(small) == [hashlib.sha256(b).digest() for b in small]
    finally:
        h.free()


@pytest.mark.parametrize("long_kib", [15, 16, 50, 900])
def test_hasher_small_batch_with_a_long_blob(gpu, long_kib):
    """Round 6: a batch under the engine's byte threshold that holds a blob of 16 KiB or more
    (a split::Writer's tree nodes: geometric leaf counts) goes to the engine's wave-mode chains
    instead of one blob per lane; at 15 KiB it stays on the per-lane path. Both forms, through
    bsg_hasher_sum and _sum_ptrs, against hashlib; the hasher pins only the batch's size."""
    rng = np.random.default_rng(long_kib)
    blobs = [rng.bytes(int(n)) for n in rng.integers(0, 12_000, 62)]
    blobs.insert(17, rng.bytes(long_kib << 10))
    blobs.insert(3, b"")
    want = [hashlib.sha256(b).digest() for b in blobs]
    h = gpu.Hasher()
    try:
        assert h.sum(blobs) == want
        assert h.sum_ptrs(blobs) == want
        assert h.sum(blobs[:2]) == want[:2]
        assert h.pinned_bytes() < 8 << 20, h.pinned_bytes()
    finally:
        h.free()


def test_sha256_batch_over_65535_blobs(gpu):
    rng = np.random.default_rng(8)
    lens = rng.integers(0, 160, 70_000)
    lens[::997] = 40_000  # 4 MiB in all, so the engine path splits into two runs
    data = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8).tobytes()
    blobs, o = [], 0
    for ln in lens:
        blobs.append(data[o:o + int(ln)])
        o += int(ln)
    assert sum(map(len, blobs)) >= 4 << 20
    assert gpu.sha256_batch(blobs) == [hashlib.sha256(b).digest() for b in blobs]


def test_engine_hash_device_resident(gpu):
    blobs = _blobs(9, 300, 30_000)
    off, o = [], 0
    for b in blobs:
        off.append(o)
        o = (o + len(b) + 15) & ~15
    host = np.zeros(o + gpu.READ_SLACK, dtype=np.uint8)
    for b, x in zip(blobs, off):
        host[x:x + len(b)] = np.frombuffer(b, dtype=np.uint8)
    buf = gpu.DeviceBuffer(host.size)
    eng = gpu.Engine()
    try:
        buf.from_host(host)
        eng.hash(buf.ptr, off, [len(b) for b in blobs])
        assert eng.finish() == len(blobs)
        ch = eng.chunks()
        assert [bytes(r) for r in ch["ref"]] == [hashlib.sha256(b).digest() for b in blobs]
        assert list(ch["len"]) == [len(b) for b in blobs]
        assert list(ch["stream"]) == list(range(len(blobs)))
    finally:
        eng.close()
        buf.free()


@pytest.fixture
def small_windows(gpu):
    with gpu.debug_knob(gpu.KNOB_VERIFY_WINDOW, 65536):
        yield


def test_reader_verify_windows(gpu, small_windows, tmp_path):
    """Windows of 64 KiB over a tree with many small leaf nodes on several levels (Bits 10,
    Fanout 2): every read and seek returns the stream's bytes; a corrupted chunk far from the
    read position is caught when its window is verified."""
    from bs_amd.synth import splitmix_bytes
    data = splitmix_bytes(41, 6_000_000)
    fs = gpu.FileStore(str(tmp_path))
    w = gpu.Writer(fs, bits=10, min_size=64, fanout=2)
    for i in range(0, len(data), 1 << 20):
        w.write(data[i:i + (1 << 20)])
    w.close()
    root = w.root
    w.free()
    assert gpu.Reader(fs, root, verify=True).read_all() == data
    r = gpu.Reader(fs, root, verify=True)
    rng = np.random.default_rng(3)
    for _ in range(40):
        pos = int(rng.integers(0, len(data)))
        n = int(rng.integers(1, 300_000))
        assert r.seek(pos, 0) == pos
        assert r.read(n) == data[pos:pos + n]
    # corrupt one chunk in the last quarter of the stream
    victim = None
    for ref in fs.refs():
        b = fs.get(ref)
        k = data.find(b)
        if len(b) > 200 and k > len(data) * 3 // 4:
            victim = ref
            break
    assert victim is not None
    p = os.path.join(str(tmp_path), "blobs", victim.hex()[:2], victim.hex()[:4], victim.hex())
    with open(p, "r+b") as f:
        c = f.read(1)
        f.seek(0)
        f.write(bytes([c[0] ^ 0x5A]))
    r = gpu.Reader(fs, root, verify=True)
    assert r.read(1 << 20) == data[: 1 << 20]  # the first windows are intact
    with pytest.raises(gpu.BsgError) as ei:
        r.read_all()
    assert ei.value.code == gpu.CORRUPT


def test_reader_seek_drops_stale_read_ahead(gpu, small_windows):
    """a window read ahead before a seek belongs to the old position. The
    first sequential read after the seek must not take it (that started yet another full window
    from the old cursor and verified a third on the reading thread): it is dropped, and exactly
    one window is verified at the new position."""
    from bs_amd.synth import splitmix_bytes
    data = splitmix_bytes(43, 3_000_000)
    st = gpu.MemStore()
    w = gpu.Writer(st, bits=10, min_size=64, fanout=2)
    w.write(data)
    w.close()
    root = w.root
    w.free()
    r = gpu.Reader(st, root, verify=True)
    assert r.read(200_000) == data[:200_000]  # sequential: windows ahead are started and taken
    before = r.stats()
    assert before["ahead_windows"] >= 1 and before["dropped"] == 0
    pos = 2_000_000
    assert r.seek(pos, 0) == pos
    assert r.read(10) == data[pos:pos + 10]   # the seeked leaf node alone
    assert r.read(8192) == data[pos + 10:pos + 8202]  # sequential again: one new window
    after = r.stats()
    assert after["dropped"] == 1, (before, after)
    assert after["ahead_windows"] == before["ahead_windows"], (before, after)
    assert after["sync_windows"] == before["sync_windows"] + 2, (before, after)
    assert r.read(500_000) == data[pos + 8202:pos + 508_202]  # and reads ahead from there
    assert r.stats()["ahead_windows"] > after["ahead_windows"]
    r.free()
