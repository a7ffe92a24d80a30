"""HIP path (through the C ABI) vs the CPU oracle and the golden fixtures — bit-exact.

Mirrors the reference's own split tests (split/split_test.go:15-108: empty input, Bits(4)
round trip over yubnub.opus) and the store harness (testutil/readwrite.go:18-54), but compares
chunk boundaries, levels and refs exactly instead of only round-tripping.
"""
import hashlib

import numpy as np
import pytest

from conftest import load_json, read_golden

pytestmark = pytest.mark.gpu


def as_tuples(ch):
    return [(int(c["offset"]), int(c["len"]), int(c["level"]), bytes(c["ref"]).hex()) for c in ch]


def golden_tuples(v):
    return list(zip(v["offset"], v["len"], v["level"], v["ref"]))


def _vector_input(key):
    from bs_amd.synth import splitmix_bytes
    if key.startswith("splitmix:"):
        _, seed, n = key.split(":")
        return splitmix_bytes(0xB5B52026 + int(seed), int(n))
    return read_golden(key)


# --------------------------------------------------------------------------------------------
# SHA-256
# --------------------------------------------------------------------------------------------
def test_sha256_batch_kats(gpu):
    kat = load_json("sha256_kat.json")
    from bs_amd.synth import splitmix_bytes
    pat = splitmix_bytes(kat["pattern_seed"], 1100)
    blobs = [pat[:n] for n in range(1101)]
    got = gpu.sha256_batch(blobs)
    assert [g.hex() for g in got] == kat["pattern_digests"]
    fips = list(kat["fips"].items())
    got = gpu.sha256_batch([m.encode() for m, _ in fips] + [b"a" * 1000000])
    assert [g.hex() for g in got] == [d for _, d in fips] + [kat["million_a"]]
    names = list(kat["files"])
    got = gpu.sha256_batch([read_golden(n) for n in names])
    assert [g.hex() for g in got] == [kat["files"][n] for n in names]


# --------------------------------------------------------------------------------------------
# Split + ref, batch API
# --------------------------------------------------------------------------------------------
def test_split_empty(gpu):
    """split_test.go:15-25 TestSplitEmpty: no input, no chunks."""
    ch, counts = gpu.split_hash_batch([b""])
    assert len(ch) == 0 and counts.tolist() == [0]


def test_chunker_kats_table_independent(gpu, table):
    kat = load_json("chunker_kat.json")
    unit = bytes.fromhex(kat["period32_unit"])
    rng = np.random.default_rng(1)
    rnd_table = rng.integers(0, 2**32, size=256, dtype=np.uint64).astype(np.uint32)
    for c in kat["cases"]:
        n = c["n"]
        data = bytes(n) if c["name"].startswith("zeros") else (unit * (n // 32 + 1))[:n]
        for t in (table, rnd_table):
            ch, _ = gpu.split_hash_batch([data], bits=c["bits"], min_size=c["min_size"], table=t)
            assert as_tuples(ch) == golden_tuples(c), (c["name"], c["bits"], c["min_size"])


def test_split_vectors_golden(gpu):
    for v in load_json("split_vectors.json")["vectors"]:
        data = _vector_input(v["input"])
        ch, _ = gpu.split_hash_batch([data], bits=v["bits"], min_size=v["min_size"])
        assert as_tuples(ch) == golden_tuples(v), (v["input"], v["bits"], v["min_size"])


def test_testsplit_bits4_yubnub(gpu, oracle, table):
    """split_test.go:27-31 configuration (Bits(4), default MinSize) + byte round trip."""
    data = read_golden("yubnub.opus")
    ch, _ = gpu.split_hash_batch([data], bits=4)
    ref = oracle.split(table, data, bits=4, min_size=1024)
    assert as_tuples(ch) == as_tuples(ref)
    rebuilt = b"".join(data[int(c["offset"]):int(c["offset"] + c["len"])] for c in ch)
    assert rebuilt == data
    for c in ch[:50]:
        o, n = int(c["offset"]), int(c["len"])
        assert bytes(c["ref"]) == hashlib.sha256(data[o:o + n]).digest()


EDGE_LENS = [0, 1, 2, 63, 64, 65, 127, 128, 1023, 1024, 1025, 2047, 2048, 2049, 4095, 4096,
             4097, 65535, 65536, 65537, 131072 + 7]


@pytest.mark.parametrize("bits,min_size", [(16, 1024), (13, 64), (8, 64), (4, 1024), (20, 4096),
                                           (1, 64), (32, 64)])
def test_multistream_random_vs_oracle(gpu, oracle, table, bits, min_size):
    from bs_amd.synth import splitmix_array
    rng = np.random.default_rng(bits * 1000 + min_size)
    lens = EDGE_LENS + [int(x) for x in rng.integers(0, 300_000, size=12)]
    arrs = [splitmix_array(1000 + i, n) for i, n in enumerate(lens)]
    ch, counts = gpu.split_hash_batch(arrs, bits=bits, min_size=min_size)
    k = 0
    for i, a in enumerate(arrs):
        one = oracle.split(table, a, bits=bits, min_size=min_size)
        got = ch[k:k + int(counts[i])]
        assert int(counts[i]) == len(one), (i, len(a))
        assert as_tuples(got) == as_tuples(one), (i, len(a))
        assert (got["stream"] == i).all()
        k += int(counts[i])
    assert k == len(ch)


def test_many_streams_past_lds_cache(gpu, oracle, table):
    """3,000 streams: more than the 2,047 whose first strips k_scan / k_compact cache in LDS, so
    the stream of a strip is searched in global memory; short, empty and multi-strip streams."""
    from bs_amd.synth import splitmix_array
    rng = np.random.default_rng(3000)
    lens = [int(x) for x in rng.integers(0, 9000, size=3000)]
    lens[5] = 0
    lens[2500] = 70_000
    arrs = [splitmix_array(5000 + i, n) for i, n in enumerate(lens)]
    ch, counts = gpu.split_hash_batch(arrs, bits=12, min_size=64)
    k = 0
    for i, a in enumerate(arrs):
        one = oracle.split(table, a, bits=12, min_size=64)
        got = ch[k:k + int(counts[i])]
        assert as_tuples(got) == as_tuples(one), (i, len(a))
        k += int(counts[i])
    assert k == len(ch)


def test_batch_past_engine_stream_limit(gpu, oracle, table):
    """140,000 host streams in one bsg_split_hash_batch call: more than an engine run takes
    (65,535), so the batch runs in three groups; records keep their batch stream index and
    every stream's chunks equal the oracle's."""
    rng = np.random.default_rng(140_000)
    lens = rng.integers(0, 2_500, size=140_000).astype(np.uint64)
    lens[[0, 65_534, 65_535, 131_070, 139_999]] = [0, 5_000, 0, 1, 70_000]
    base = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8)
    off = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    arrs = [base[int(o):int(o) + int(n)] for o, n in zip(off, lens)]
    ch, counts = gpu.split_hash_batch(arrs, bits=10, min_size=64)
    want, wcounts = oracle.split_streams(table, base, off, [int(x) for x in lens], bits=10,
                                         min_size=64, threads=8)
    assert (counts == np.asarray(wcounts, dtype=np.uint64)).all()
    assert len(ch) == len(want)
    for f in ("offset", "len", "level", "ref"):
        assert (ch[f] == want[f]).all(), f
    assert (ch["stream"] == np.repeat(np.arange(len(lens)), counts.astype(np.int64))).all()


def test_dense_candidates_zero_runs(gpu, oracle, table):
    """Long zero runs inside random data: every position in the run is a candidate."""
    from bs_amd.synth import splitmix_array
    a = splitmix_array(77, 500_000)
    a[100_000:300_000] = 0
    a[400_000:400_100] = 0
    for bits, mn in ((16, 1024), (12, 64)):
        ch, _ = gpu.split_hash_batch([a], bits=bits, min_size=mn)
        assert as_tuples(ch) == as_tuples(oracle.split(table, a, bits=bits, min_size=mn))


# --------------------------------------------------------------------------------------------
# Streaming split.Writer path: arbitrary Write sizes, tiles carried across segments
# --------------------------------------------------------------------------------------------
@pytest.mark.parametrize("tile,carry_cap", [(4096, None), (5000, None), (65536 + 3, None),
                                            (1 << 20, None), (4096, 0), (65536 + 3, 0),
                                            (5000, 3000), (1 << 20, 40_000)])
def test_streaming_writer_vs_oracle(gpu, oracle, table, tile, carry_cap):
    """carry_cap None: open chunks carried as device bytes (default 8 MiB cap); 0: always as a
    SHA-256 midstate; small caps mix both (the mode changes from tile to tile)."""
    from bs_amd.synth import splitmix_bytes
    data = splitmix_bytes(4242, 3_000_017)
    data = data[:1_500_000] + bytes(70_000) + data[1_500_000:]  # a dense stretch
    rng = np.random.default_rng(tile)
    for bits, mn in ((16, 1024), (10, 64)):
        w = gpu.StreamingSplitter(bits=bits, min_size=mn, tile=tile, carry_cap=carry_cap)
        pos, got = 0, []
        while pos < len(data):
            k = int(rng.choice([1, 7, 100, 4096, 32768, 300_000]))
            w.write(data[pos:pos + k])
            pos += k
            got.append(w.drain())
        w.close()
        got.append(w.drain())
        w.free()
        ch = np.concatenate(got)
        assert as_tuples(ch) == as_tuples(oracle.split(table, data, bits=bits, min_size=mn))


@pytest.mark.parametrize("carry_cap", [None, 0])
def test_streaming_tile_multiples(gpu, oracle, table, carry_cap):
    """Streams that end exactly on a tile boundary (the final segment is empty) and chunks far
    longer than a tile (bits=20: mean chunk 1 MiB over 64 KiB tiles)."""
    from bs_amd.synth import splitmix_bytes
    tile = 65536
    for n, bits in ((4 * tile, 16), (tile, 16), (40 * tile, 20), (40 * tile + 1, 20)):
        d = splitmix_bytes(n + bits, n)
        w = gpu.StreamingSplitter(bits=bits, min_size=1024, tile=tile, carry_cap=carry_cap)
        w.write(d[: n // 3])
        w.write(d[n // 3:])
        w.close()
        ch = w.drain()
        w.free()
        assert as_tuples(ch) == as_tuples(oracle.split(table, d, bits=bits, min_size=1024)), n


def test_streaming_candidate_overflow(gpu, oracle, table):
    """Every byte a candidate (zeros, bits=1): the first run of each tile overflows the
    candidate buffer and is re-run at its exact size inside the pipeline."""
    from bs_amd.synth import splitmix_bytes
    d = bytes(600_000) + splitmix_bytes(5, 300_000) + bytes(500_000)
    w = gpu.StreamingSplitter(bits=1, min_size=64, tile=1 << 19)
    for i in range(0, len(d), 100_000):
        w.write(d[i:i + 100_000])
    w.close()
    ch = w.drain()
    w.free()
    assert as_tuples(ch) == as_tuples(oracle.split(table, d, bits=1, min_size=64))


def test_streaming_zero_copy_window(gpu, oracle, table, tmp_path):
    """bsg_write_window/commit: a file read straight into pinned staging (io.Reader form)."""
    from bs_amd.synth import splitmix_bytes
    d = splitmix_bytes(77, 1_500_000)
    f = tmp_path / "stream.bin"
    f.write_bytes(d)
    want = as_tuples(oracle.split(table, d, bits=12, min_size=256))
    w = gpu.StreamingSplitter(bits=12, min_size=256, tile=1 << 18)
    with open(f, "rb") as fh:
        assert w.read_from(fh, piece=100_000) == len(d)
    w.close()
    assert as_tuples(w.drain()) == want
    # a stream whose length is an exact multiple of the tile, read to EOF through the window
    e = d[: 5 * (1 << 18)]
    f.write_bytes(e)
    w.reset()
    with open(f, "rb") as fh:
        assert w.read_from(fh, piece=1 << 18) == len(e)
    w.close()
    assert as_tuples(w.drain()) == as_tuples(oracle.split(table, e, bits=12, min_size=256))
    w.free()


def test_streaming_small_and_empty(gpu, oracle, table):
    for n in (0, 1, 63, 64, 1023, 1024, 1025, 4095, 4096, 4097):
        from bs_amd.synth import splitmix_bytes
        d = splitmix_bytes(n, n)
        w = gpu.StreamingSplitter(bits=8, min_size=64, tile=4096)
        w.write(d)
        w.close()
        ch = w.drain()
        w.free()
        assert as_tuples(ch) == as_tuples(oracle.split(table, d, bits=8, min_size=64)), n


# --------------------------------------------------------------------------------------------
# Device-resident engine (the bench path) at full size
# --------------------------------------------------------------------------------------------
def _device_stream_run(gpu, nbytes_list, seed0, bits=16, min_size=1024):
    offs, total = [], 0
    for n in nbytes_list:
        offs.append(total)
        total += (n + 15) & ~15
    buf = gpu.DeviceBuffer(max(total, 16))
    eng = gpu.Engine()
    for i, (o, n) in enumerate(zip(offs, nbytes_list)):
        gpu.fill_splitmix(buf.ptr + o, n, seed0 + i, stream=eng.stream)
    eng.run(buf.ptr, offs, nbytes_list, bits=bits, min_size=min_size)
    eng.finish()
    return eng, buf, offs


def test_engine_device_resident_vs_oracle(gpu, oracle, table):
    from bs_amd.synth import splitmix_array
    lens = [64 << 20, 3_000_001, 0, 17]
    eng, buf, offs = _device_stream_run(gpu, lens, 0xB5B52026)
    ch = eng.chunks()
    counts = eng.counts()
    k = 0
    for i, n in enumerate(lens):
        host = splitmix_array(0xB5B52026 + i, n)
        dev = buf.to_host(offs[i], n)
        assert np.array_equal(host, dev)  # device generator == host generator
        one = oracle.split(table, host)
        assert as_tuples(ch[k:k + int(counts[i])]) == as_tuples(one)
        k += int(counts[i])
    eng.close()


def test_engine_finish_polling(gpu, oracle, table):
    """bsg_engine_finish with BSG_KNOB_POLL (the bench's wait: stream queries instead of a
    blocking synchronize), over a run with early chains (>= 256 MiB) and repeated runs of one
    engine: same records as the oracle, and the same as the blocking wait's."""
    from bs_amd.synth import splitmix_array
    lens = [300 << 20, 5_000_003]
    got = {}
    for poll in (1, 0, 1):
        with gpu.debug_knob(gpu.KNOB_POLL, poll):
            eng, buf, offs = _device_stream_run(gpu, lens, 0x5EED)
            for _ in range(2):  # a second run of the same engine, waited the same way
                eng.run(buf.ptr, offs, lens)
                assert eng.finish() == len(eng.chunks())
            got.setdefault(poll, []).append(as_tuples(eng.chunks()))
            counts = eng.counts()
            eng.close()
            buf.free()
    assert got[1][0] == got[0][0] == got[1][1]
    k = 0
    for i, n in enumerate(lens):
        one = oracle.split(table, splitmix_array(0x5EED + i, n))
        assert got[1][0][k:k + int(counts[i])] == as_tuples(one)
        k += int(counts[i])


@pytest.mark.slow
def test_engine_1gib_full_parity(gpu, oracle, table):
    """BASELINE config 2 (1 GiB random stream, default params): full oracle comparison."""
    from bs_amd.synth import splitmix_array
    n = 1 << 30
    eng, buf, offs = _device_stream_run(gpu, [n], 0xB5B52026)
    ch = eng.chunks()
    host = splitmix_array(0xB5B52026, n)
    one = oracle.split(table, host)
    assert len(ch) == len(one)
    assert (ch["offset"] == one["offset"]).all() and (ch["len"] == one["len"]).all()
    assert (ch["level"] == one["level"]).all() and (ch["ref"] == one["ref"]).all()
    # size-independent properties
    assert int(ch["len"].sum()) == n
    assert (ch["len"][:-1] >= 1024).all()
    eng.close()


def test_early_chains_on_off(gpu, oracle, table):
    """Early chains (KNOB_EARLY): the two longest chunks whose ends are sure
    boundaries are hashed on a second stream from right after k_compact. Stream 0 is cut one
    byte before the end of its longest chunk, so its final (forced) chunk is the run's longest
    and early slot 0 takes it; slot 1 takes an ordinary chunk. Records with the knob on and off
    and the oracle's are identical, and the longest chain's stamps come from the early chain
    (it starts before k_sha does: a negative long_start)."""
    from bs_amd.synth import splitmix_array
    seed = 0xE4C2  # its longest chunk (658,353 B) ends at 263 MiB: the run is >= 256 MiB
    full = splitmix_array(seed, 270 << 20)
    one = oracle.split(table, full)
    k = int(np.argmax(one["len"][:-1]))
    n0 = int(one["offset"][k] + one["len"][k]) - 1
    lens = [n0, 40 << 20]
    assert sum(lens) >= 256 << 20  # engine runs below that take no early chains
    want = [oracle.split(table, full[:n0]), oracle.split(table, splitmix_array(seed + 1, lens[1]))]
    assert int(want[0]["len"][-1]) == int(one["len"][k]) - 1
    got = {}
    for on in (1, 0):
        with gpu.debug_knob(gpu.KNOB_EARLY, on):
            eng, buf, offs = _device_stream_run(gpu, lens, seed)
            got[on] = (as_tuples(eng.chunks()), [int(c) for c in eng.counts()], eng.diag())
            eng.close()
            buf.free()
    assert got[1][:2] == got[0][:2]
    ch, counts = got[1][0], got[1][1]
    assert counts == [len(w) for w in want]
    assert ch == as_tuples(want[0]) + as_tuples(want[1])
    tl = got[1][2].get("timeline_us")
    assert tl and tl["long_start"] < 0, got[1][2]
    assert got[1][2]["long"]["blocks"] == (int(one["len"][k]) - 1 + 8) // 64 + 1
    tl0 = got[0][2].get("timeline_us")
    assert tl0 and tl0["long_start"] >= 0, got[0][2]


def test_early_chains_light_and_loaded_schedules(gpu, oracle, table):
    """every test input is at most the 4 GiB light-run threshold, so the loaded
    schedule (selection and k_sha on the engine stream, k_pick on the second one, k_lens waiting
    for the pick) ran only in the bench's configs[2] leg. BSG_KNOB_LIGHT_BYTES moves the
    threshold: the same 300 MiB batch with the early chains runs both ways, and both give the
    oracle's records."""
    from bs_amd.synth import splitmix_array
    lens = [190 << 20, (110 << 20) + 12345]
    seeds = [0x5EED1, 0x5EED2]
    want = [oracle.split(table, splitmix_array(s, n)) for s, n in zip(seeds, lens)]
    stride = [(n + 15) & ~15 for n in lens]
    buf = gpu.DeviceBuffer(sum(stride) + 4096)
    offs = [0, stride[0]]
    for o, n, s in zip(offs, lens, seeds):
        gpu.fill_splitmix(buf.ptr + o, n, s)
    gpu.synchronize()
    got = {}
    for light in (4 << 30, 0):
        with gpu.debug_knob(gpu.KNOB_LIGHT_BYTES, light), gpu.debug_knob(gpu.KNOB_EARLY, 1):
            eng = gpu.Engine()
            eng.run(buf.ptr, offs, lens)
            eng.finish()
            got[light] = (as_tuples(eng.chunks()), [int(c) for c in eng.counts()], eng.diag())
            eng.close()
    buf.free()
    for light, (ch, counts, diag) in got.items():
        assert counts == [len(w) for w in want], light
        assert ch == as_tuples(want[0]) + as_tuples(want[1]), light
    tl = got[4 << 30][2].get("timeline_us")
    assert tl and tl["long_start"] < 0, got[4 << 30][2]  # light: the longest chain ran early


@pytest.mark.parametrize("bits,min_size", [(13, 8192), (20, 64), (16, 65536), (14, 1)])
def test_early_chains_params(gpu, oracle, table, bits, min_size):
    """The sure-boundary rule behind the early picks (E_i - E_i-1 >= MinSize) under other
    params: a large MinSize (few sync points, long forced walks), tiny MinSize, 1 MiB chunks.
    A 260 MiB stream plus a short one; records with the early chains on and off and the
    oracle's identical."""
    from bs_amd.synth import splitmix_array
    lens = [260 << 20, 3 << 20]
    seed = 0xEA00 + bits
    got, tl = {}, {}
    for on in (1, 0):
        with gpu.debug_knob(gpu.KNOB_EARLY, on):
            eng, buf, offs = _device_stream_run(gpu, lens, seed, bits=bits, min_size=min_size)
            got[on] = (as_tuples(eng.chunks()), [int(c) for c in eng.counts()])
            tl[on] = eng.diag().get("timeline_us", {})
            eng.close()
            buf.free()
    assert got[1] == got[0]
    assert tl[1]["long_start"] < 0 <= tl[0]["long_start"], tl  # the longest ran early
    want = []
    for i, n in enumerate(lens):
        want += as_tuples(oracle.split(table, splitmix_array(seed + i, n), bits=bits,
                                       min_size=min_size))
    assert got[1][0] == want


def test_early_chains_candidate_overflow(gpu, oracle, table):
    """A 264 MiB run whose first 96 MiB are zeros: a candidate at every position there, far past
    the candidate estimate, so the first run overflows (its early chains stand down) and
    bsg_engine_finish re-runs at the exact size with the early chains on; records equal the
    oracle's."""
    from bs_amd.synth import splitmix_array
    n = 264 << 20
    host = splitmix_array(0xE0F0, n)
    host[: 96 << 20] = 0
    buf = gpu.DeviceBuffer(n + 4096)
    buf.from_host(host)
    with gpu.debug_knob(gpu.KNOB_EARLY, 1):
        eng = gpu.Engine()
        eng.run(buf.ptr, [0], [n])
        eng.finish()
        got = eng.chunks()
        tl = eng.diag().get("timeline_us", {})
        eng.close()
    buf.free()
    want = oracle.split(table, host)
    assert len(got) == len(want)
    for f in ("offset", "len", "level", "ref"):
        assert (got[f] == want[f]).all(), f
    assert tl.get("long_start", 0) < 0, tl  # the re-run's longest chunk ran early


def test_early_chains_concurrent_engines(gpu, oracle, table):
    """Three engines on three host threads, each running a >= 256 MiB batch with early chains at
    the same time (six HIP streams over the process's hardware queues, cross-stream waits in
    both directions), twice: every run's records equal that engine's run alone with the early
    chains off, and stream 0 of the first engine equals the oracle."""
    from concurrent.futures import ThreadPoolExecutor
    from bs_amd.synth import splitmix_array
    lens = [[200 << 20, 60 << 20 | 12345], [270 << 20], [130 << 20, 130 << 20, 1 << 20]]
    seeds = [0xC0C0, 0xC1C1, 0xC2C2]

    def prepare(k):
        offs, total = [], 0
        for n in lens[k]:
            offs.append(total)
            total += (n + 15) & ~15
        buf = gpu.DeviceBuffer(total + 4096)
        eng = gpu.Engine()
        for i, (o, n) in enumerate(zip(offs, lens[k])):
            gpu.fill_splitmix(buf.ptr + o, n, seeds[k] + i, stream=eng.stream)
        return eng, buf, offs

    def run(k, eng, buf, offs):
        eng.run(buf.ptr, offs, lens[k], bits=16, min_size=1024)
        eng.finish()
        return as_tuples(eng.chunks()), [int(c) for c in eng.counts()]

    setups = [prepare(k) for k in range(3)]
    with gpu.debug_knob(gpu.KNOB_EARLY, 0):
        alone = [run(k, *setups[k]) for k in range(3)]
    with gpu.debug_knob(gpu.KNOB_EARLY, 1):
        with ThreadPoolExecutor(3) as ex:
            for _ in range(2):
                got = list(ex.map(lambda k: run(k, *setups[k]), range(3)))
                assert got == alone
    want0 = as_tuples(oracle.split(table, splitmix_array(seeds[0], lens[0][0])))
    assert alone[0][0][:alone[0][1][0]] == want0
    for eng, buf, _ in setups:
        eng.close()
        buf.free()


def test_dedup_edited_streams(gpu, oracle, table):
    """BASELINE config 5 (dedup), scaled to 2 x 64 MiB: stream B = stream A with 1 % seeded
    edits (64 sites x 10486 B). Both streams split in one batch must equal the oracle, and the
    content-defined boundaries must resynchronise after every edit, so most chunks are shared."""
    from bs_amd.synth import edit_stream, splitmix_array
    a = splitmix_array(0xB5B52026, 64 << 20)
    b = edit_stream(a, 0xB5B52026 + 5, sites=64)
    ch, counts = gpu.split_hash_batch([a, b])
    na = int(counts[0])
    for part, data in ((ch[:na], a), (ch[na:], b)):
        one = oracle.split(table, data)
        assert as_tuples(part) == as_tuples(one)
    refs_a = {bytes(r) for r in ch[:na]["ref"]}
    refs_b = [bytes(r) for r in ch[na:]["ref"]]
    shared = sum(r in refs_a for r in refs_b) / len(refs_b)
    assert shared > 0.75, shared


# --------------------------------------------------------------------------------------------
# Seeded fuzz: random params, stream shapes, tiles, carry caps and Write sizes
# --------------------------------------------------------------------------------------------
@pytest.mark.parametrize("seed", range(24))
def test_streaming_fuzz_vs_oracle(gpu, oracle, table, seed):
    """Each seed draws split params (bits 8..22, MinSize 64..8192), a stream of 0..2.5 MB with
    optional zero / period-32 stretches (dense candidates, h = 0 windows), a tile size, a carry
    cap (device bytes, midstate, or a mix) and a Write-size pattern, and compares every chunk
    with the oracle; the batch API (split_hash_batch) must agree with the streaming one."""
    from bs_amd.synth import splitmix_bytes
    rng = np.random.default_rng(9000 + seed)
    bits = int(rng.integers(8, 23))
    mn = int(rng.choice([64, 100, 1024, 4096, 8192]))
    n = (int(rng.choice([0, 1, 63, 64, 65, 1023, 1024, 1025])) if rng.random() < 0.2
         else int(rng.integers(10_000, 2_500_000)))
    data = bytearray(splitmix_bytes(777 + seed, n))
    if n > 10_000 and rng.random() < 0.5:  # a zero stretch: a candidate at every position
        s = int(rng.integers(0, n - 5000))
        z = int(rng.integers(100, 5000))
        data[s:s + z] = bytes(z)
    if n > 10_000 and rng.random() < 0.5:  # a period-32 stretch: h = 0 once the window is in it
        s = int(rng.integers(0, n - 4096))
        unit = bytes(rng.integers(0, 256, 32, dtype=np.uint8))
        data[s:s + 4096] = unit * 128
    data = bytes(data)
    tile = int(rng.choice([4096, 10_000, 65536, 1 << 20, 3 << 20]))
    carry_cap = [None, 0, int(rng.integers(1, 200_000))][int(rng.integers(0, 3))]
    want = as_tuples(oracle.split(table, data, bits=bits, min_size=mn))
    w = gpu.StreamingSplitter(bits=bits, min_size=mn, tile=tile, carry_cap=carry_cap)
    pos, got = 0, []
    sizes = [1, 3, 64, 1000, 4096, 65536, 250_000]
    while pos < len(data):
        k = int(rng.choice(sizes))
        w.write(data[pos:pos + k])
        pos += k
        if rng.random() < 0.5:
            got.append(w.drain())
    w.close()
    got.append(w.drain())
    w.free()
    ch = np.concatenate(got) if got else got
    assert as_tuples(ch) == want, (seed, bits, mn, n, tile, carry_cap)
    bch, _ = gpu.split_hash_batch([np.frombuffer(data, dtype=np.uint8)], bits=bits, min_size=mn)
    assert as_tuples(bch) == want, (seed, "batch")


@pytest.mark.parametrize("mode", ["off", "all"])
def test_sha_path_forced(gpu, oracle, table, mode):
    """Every job through one SHA-256 path: per-lane only (BSG_LONG_MODE=off) or wave mode only
    (all: solo and group tickets for every eligible job), over streams whose chunks span short
    to very long; both must give the oracle's refs."""
    from bs_amd.synth import splitmix_array
    arrs = [splitmix_array(31 + i, n) for i, n in enumerate([0, 5_000, 700_000, 3_000_001])]
    with gpu.debug_knob(gpu.KNOB_LONG_MODE, {"off": 1, "all": 2}[mode]):
        for bits, mn in ((16, 1024), (13, 64), (18, 4096)):
            ch, counts = gpu.split_hash_batch(arrs, bits=bits, min_size=mn)
            k = 0
            for i, a in enumerate(arrs):
                one = oracle.split(table, a, bits=bits, min_size=mn)
                assert as_tuples(ch[k:k + int(counts[i])]) == as_tuples(one), (mode, bits, i)
                k += int(counts[i])


@pytest.mark.parametrize("carry_cap", [None, 0])
def test_streaming_big_tiles_regions(gpu, oracle, table, carry_cap):
    """Tiles over 1 GiB, so k_sha's per-lane jobs split into two address regions while the
    open chunk of each tile is continued in the next (carry_cap 0: from a SHA-256 midstate, a
    per-lane job on the synchronous setup path inside the region queues)."""
    from bs_amd.synth import splitmix_array
    n = (9 << 28) + 12345                 # 2.25 GiB + a ragged end
    tile = (9 << 27) + 3                  # 1.125 GiB tiles
    d = splitmix_array(0xB16, n)
    want = oracle.split(table, d, bits=16, min_size=1024)
    w = gpu.StreamingSplitter(bits=16, min_size=1024, tile=tile, carry_cap=carry_cap)
    got = []
    mv = memoryview(d)
    for i in range(0, n, 256 << 20):
        w.write(mv[i:i + (256 << 20)])
        got.append(w.drain())
    w.close()
    got.append(w.drain())
    w.free()
    ch = np.concatenate(got)
    assert len(ch) == len(want)
    assert (ch["offset"] == want["offset"]).all() and (ch["len"] == want["len"]).all()
    assert (ch["ref"] == want["ref"]).all() and (ch["level"] == want["level"]).all()


@pytest.mark.parametrize("tile,pieces", [
    (1 << 20, [3 << 20, 1 << 20, 777, (2 << 20) + 5]),   # pinned segments across tiles
    (4096, [4096, 1, 4095, 10_000]),                       # tile-sized and tiny segments
    (256 << 20, [7 << 20, 9 << 20]),                       # the default tile, one partial tile
])
def test_write_pinned_matches_oracle(gpu, oracle, table, tile, pieces):
    """bsg_write_pinned from registered host memory (no staging copy), mixed with staged
    bsg_write calls, against the oracle; the caller's bytes stay registered until close."""
    import mmap
    from bs_amd.synth import splitmix_array
    n = sum(pieces)
    data = splitmix_array(0xD1CE + tile, n)
    m = mmap.mmap(-1, max(n, 1))  # page-aligned, like the C++ Writer's pieces
    buf = np.frombuffer(m, dtype=np.uint8)
    buf[:n] = data
    ptr = buf.ctypes.data
    gpu.host_register(ptr, len(m))
    sp = gpu.StreamingSplitter(bits=13, min_size=256, tile=tile)
    try:
        o, got = 0, []
        for i, k in enumerate(pieces):
            if i % 2 == 0:
                sp.write_pinned(ptr + o, k)
            else:
                sp.write(data[o:o + k])
            o += k
            got.append(sp.drain())
        sp.close()
        got.append(sp.drain())
    finally:
        sp.free()
        gpu.host_unregister(ptr)
        del buf
        m.close()
    got = np.concatenate(got)
    ref = oracle.split(table, data, bits=13, min_size=256)
    assert len(got) == len(ref)
    assert (got["offset"] == ref["offset"]).all() and (got["ref"] == ref["ref"]).all()
    assert (got["level"] == ref["level"]).all()


def test_split_hash_batch_tables_interleaved_and_threads(gpu, oracle, table):
    """bsg_split_hash_batch re-uses pooled engines: a call with another buzhash32 table (bsg_open's
    and split_hash_batch's `table` argument) must not see the previous call's, whether calls
    alternate on one thread or run on several at once. Random data, so every boundary depends on
    the table; each result equals the oracle's under the same table."""
    from concurrent.futures import ThreadPoolExecutor
    from bs_amd.synth import splitmix_array
    rng = np.random.default_rng(7)
    tables = [table] + [rng.integers(0, 2**32, size=256, dtype=np.uint64).astype(np.uint32)
                        for _ in range(2)]
    streams = [splitmix_array(900 + i, (3 << 20) + 77 * i) for i in range(3)]
    want = {(t, s): as_tuples(oracle.split(tables[t], streams[s], bits=13, min_size=256))
            for t in range(3) for s in range(3)}
    assert want[(0, 0)] != want[(1, 0)]                # the tables do change the boundaries
    order = [(t, s) for s in range(3) for t in (0, 1, 0, 2, 1)]
    for t, s in order:
        ch, _ = gpu.split_hash_batch([streams[s]], bits=13, min_size=256, table=tables[t])
        assert as_tuples(ch) == want[(t, s)], (t, s)

    def run(job):
        t, s = job
        ch, _ = gpu.split_hash_batch([streams[s]], bits=13, min_size=256, table=tables[t])
        return as_tuples(ch) == want[(t, s)]
    with ThreadPoolExecutor(max_workers=6) as ex:
        assert all(ex.map(run, order * 2))
