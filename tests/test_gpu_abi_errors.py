"""C-ABI error behaviour on the device (mirrors the reference's error conventions: Write after
Close fails, a missing root fails NewReader with bs.ErrNotFound) and the persistent hasher."""
import ctypes
import hashlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _check_chunks(data: bytes, ch) -> None:
    assert b"".join(data[int(c["offset"]):int(c["offset"] + c["len"])] for c in ch) == data
    for c in ch:
        blob = data[int(c["offset"]):int(c["offset"] + c["len"])]
        assert bytes(c["ref"]) == hashlib.sha256(blob).digest()


def test_write_after_close_and_late_knobs(gpu):
    from bs_amd.synth import splitmix_bytes
    L = gpu.lib()
    a, b = splitmix_bytes(1, 300_000), splitmix_bytes(2, 200_000)
    w = gpu.StreamingSplitter()
    w.write(a)
    assert L.bsg_set_tile(w.h, 1 << 20) == -22        # tile fixed once bytes arrived
    assert L.bsg_set_carry_cap(w.h, 0) == -22
    w.close()
    assert L.bsg_write(w.h, b"y", 1) == -71           # BSG_ESTATE: Write after Close
    assert L.bsg_close(w.h) == 0                      # Close is idempotent
    _check_chunks(a, w.drain())
    w.reset()                                         # a reset context takes a new stream
    w.write(b)
    w.close()
    _check_chunks(b, w.drain())
    w.free()


def test_reader_missing_root(gpu):
    st = gpu.MemStore()
    with pytest.raises(gpu.BsgError) as ei:
        gpu.Reader(st, bytes(32))
    assert ei.value.code == gpu.NOT_FOUND


def test_persistent_hasher_batches(gpu):
    L = gpu.lib()
    L.bsg_hasher_new.restype = ctypes.c_void_p
    L.bsg_hasher_new.argtypes = [ctypes.c_int]
    L.bsg_hasher_sum.restype = ctypes.c_int
    L.bsg_hasher_sum.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                 ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]
    L.bsg_hasher_free.argtypes = [ctypes.c_void_p]
    h = L.bsg_hasher_new(0)
    assert h
    rng = np.random.default_rng(11)
    try:
        for n in (1, 7, 300):  # the buffers grow and are reused across calls
            blobs = [rng.integers(0, 256, int(rng.integers(0, 5000)), dtype=np.uint8).tobytes()
                     for _ in range(n)]
            packed = b"".join(blobs)
            off = np.cumsum([0] + [len(b) for b in blobs[:-1]]).astype(np.uint64)
            ln = np.array([len(b) for b in blobs], dtype=np.uint64)
            out = ctypes.create_string_buffer(32 * n)
            assert L.bsg_hasher_sum(h, packed or b"\0", off.ctypes.data, ln.ctypes.data, n,
                                    out) == 0
            assert [out.raw[32 * i:32 * i + 32] for i in range(n)] == \
                [hashlib.sha256(b).digest() for b in blobs]
    finally:
        L.bsg_hasher_free(h)


def test_close_in_steps(gpu, oracle, table):
    """bsg_close_begin + bsg_close_step: the tiles still on the device finish one per step, and
    the chunks of all steps are exactly those of bsg_close (the oracle's); a step before begin is
    BSG_ESTATE, a step after the last returns 0 tiles left."""
    import ctypes
    from bs_amd.synth import splitmix_array
    L = gpu.lib()
    d = splitmix_array(77, (9 << 20) + 4321)
    w = gpu.StreamingSplitter(bits=13, min_size=256, tile=1 << 20)
    left = ctypes.c_size_t(5)
    assert L.bsg_close_step(w.h, ctypes.byref(left)) == -71 and left.value == 0
    got = []
    for i in range(0, len(d), 3 << 20):
        w.write(memoryview(d)[i:i + (3 << 20)])
        got.append(w.drain())
    steps = list(w.close_steps())
    assert len(steps) >= 2                           # several tiles were still on the device
    got += steps
    assert L.bsg_close_step(w.h, ctypes.byref(left)) == 0 and left.value == 0
    assert L.bsg_write(w.h, b"y", 1) == -71
    w.free()
    want = oracle.split(table, d, bits=13, min_size=256)
    ch = np.concatenate(got)
    assert len(ch) == len(want)
    for f in ("offset", "len", "level", "ref"):
        assert (ch[f] == want[f]).all(), f
    e = gpu.StreamingSplitter()                      # an empty stream: nothing on the device
    assert all(len(x) == 0 for x in e.close_steps())
    e.free()


def test_engine_profile_modes(gpu):
    """bsg_engine_profile: 1 times every stage, 2 only the SHA-256 stage (the scan and selection
    stages read -1), 0 off (stage_ms refused); other modes are refused."""
    from bs_amd.synth import splitmix_array
    L = gpu.lib()
    data = splitmix_array(5, 3 << 20)
    buf = gpu.DeviceBuffer(len(data) + 4096)
    buf.from_host(data)
    eng = gpu.Engine()
    assert L.bsg_engine_profile(eng.h, 3) == -22 and L.bsg_engine_profile(eng.h, -1) == -22
    for mode in (1, 2):
        eng.profile(mode)
        eng.run(buf.ptr, [0], [len(data)])
        eng.finish()
        ms = eng.stage_ms()
        assert ms[2] > 0
        assert (ms[0] > 0 and ms[1] > 0) if mode == 1 else (ms[0] == -1 and ms[1] == -1)
    eng.profile(0)
    st = (ctypes.c_float * 3)()
    assert L.bsg_engine_stage_ms(eng.h, st) == -22
    eng.close()
    buf.free()
