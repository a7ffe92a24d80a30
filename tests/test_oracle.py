"""CPU oracle pinned against the committed golden fixtures (no GPU)."""
import hashlib
import os

import numpy as np
import pytest

from conftest import load_json, read_golden


def test_go_rand_known_answers(oracle):
    kat = load_json("go_rand_kat.json")
    assert oracle.gorand_int63(kat["seed"], len(kat["int63"])) == kat["int63"]


def test_default_table_is_generatehashes_1(oracle, table):
    t = oracle.buzhash32_table(1)
    assert t.tolist() == table.tolist()
    assert len(set(t.tolist())) == 256


def test_sha256_kats(oracle):
    kat = load_json("sha256_kat.json")
    for msg, dig in kat["fips"].items():
        assert oracle.sha256(msg.encode()).hex() == dig
    assert oracle.sha256(b"a" * 1000000).hex() == kat["million_a"]
    from bs_amd.synth import splitmix_bytes
    pat = splitmix_bytes(kat["pattern_seed"], 1100)
    for n, d in enumerate(kat["pattern_digests"]):
        assert oracle.sha256(pat[:n]).hex() == d, n
    for name, d in kat["files"].items():
        assert oracle.sha256(read_golden(name)).hex() == d


def test_rolling_closed_form_matches_roll(oracle, table):
    from bs_amd.synth import splitmix_bytes
    d = splitmix_bytes(7, 3000)
    sums = oracle.rolling_sums(table, d)
    for p in [0, 1, 31, 62, 63, 64, 65, 127, 128, 1000, 2999]:
        assert oracle.py_window_hash(table, d, p) == int(sums[p])


def test_period32_windows_hash_to_zero(oracle):
    rng = np.random.default_rng(5)
    for _ in range(3):
        t = rng.integers(0, 2**32, size=256, dtype=np.uint64).astype(np.uint32)
        unit = rng.integers(0, 256, size=32, dtype=np.uint8).tobytes()
        sums = oracle.rolling_sums(t, unit * 10)
        assert (sums[63:] == 0).all()
        assert (oracle.rolling_sums(t, bytes(500)) == 0).all()


@pytest.mark.parametrize("case", range(8))
def test_chunker_kats_table_independent(oracle, table, case):
    kat = load_json("chunker_kat.json")
    c = kat["cases"][case]
    unit = bytes.fromhex(kat["period32_unit"])
    n = c["n"]
    data = bytes(n) if c["name"].startswith("zeros") else (unit * (n // 32 + 1))[:n]
    rng = np.random.default_rng(case)
    for t in (table, rng.integers(0, 2**32, size=256, dtype=np.uint64).astype(np.uint32)):
        ch = oracle.split(t, data, bits=c["bits"], min_size=c["min_size"])
        assert ch["offset"].tolist() == c["offset"]
        assert ch["len"].tolist() == c["len"]
        assert ch["level"].tolist() == c["level"]
        assert [bytes(r).hex() for r in ch["ref"]] == c["ref"]


def _vector_input(key):
    from bs_amd.synth import splitmix_bytes
    if key.startswith("splitmix:"):
        _, seed, n = key.split(":")
        return splitmix_bytes(0xB5B52026 + int(seed), int(n))
    return read_golden(key)


def test_split_vectors(oracle, table):
    for v in load_json("split_vectors.json")["vectors"]:
        data = _vector_input(v["input"])
        ch = oracle.split(table, data, bits=v["bits"], min_size=v["min_size"])
        assert ch["offset"].tolist() == v["offset"], v["input"]
        assert ch["len"].tolist() == v["len"]
        assert ch["level"].tolist() == v["level"]
        assert [bytes(r).hex() for r in ch["ref"]] == v["ref"]


def test_python_and_c_restatements_agree(oracle, table):
    from bs_amd.synth import splitmix_bytes
    for seed, n, bits, mn in [(11, 70_000, 8, 64), (12, 5000, 4, 64), (13, 200, 4, 64),
                              (14, 64, 2, 64), (15, 0, 16, 1024), (16, 1, 16, 1024)]:
        d = splitmix_bytes(seed, n)
        a = oracle.split(table, d, bits=bits, min_size=mn)
        b = oracle.py_split(table, d, bits=bits, min_size=mn)
        assert [(int(x["offset"]), int(x["len"]), int(x["level"]), bytes(x["ref"])) for x in a] \
            == [(y.offset, y.len, y.level, y.ref) for y in b]


# The full ranges split.Bits / split.MinSize accept (split/split.go:137-152 store them
# unchecked): MinSize 1..63 (a window may span a boundary), Bits 0 (hashsplit default 13) and
# Bits > 32 (TrailingZeros32 <= 32: never splits, one final chunk of level 0).
EDGE_PARAMS = [(4, 1), (8, 2), (6, 17), (10, 63), (1, 1), (0, 0), (0, 100), (33, 64), (40, 1),
               (2**32 - 1, 1024), (32, 1), (31, 5)]


def edge_stream(seed: int, n: int) -> bytes:
    """Random bytes with zero runs and a period-32 stretch (dense candidates: h = 0)."""
    from bs_amd.synth import splitmix_bytes
    d = bytearray(splitmix_bytes(seed, n))
    if n > 3000:
        d[1000:1700] = bytes(700)
        pat = splitmix_bytes(seed + 1, 32)
        d[2000:2900] = (pat * 30)[:900]
    return bytes(d)


@pytest.mark.parametrize("bits,mn", EDGE_PARAMS)
def test_restatements_agree_on_edge_params(oracle, table, bits, mn):
    for seed, n in [(21, 5000), (22, 130), (23, 64), (24, 1), (25, 0)]:
        d = edge_stream(seed + bits % 97 + mn, n)
        a = oracle.split(table, d, bits=bits, min_size=mn)
        b = oracle.py_split(table, d, bits=bits, min_size=mn)
        assert [(int(x["offset"]), int(x["len"]), int(x["level"]), bytes(x["ref"])) for x in a] \
            == [(y.offset, y.len, y.level, y.ref) for y in b], (bits, mn, n)
        if n:
            assert sum(int(x["len"]) for x in a) == n
        eff_min = mn if mn > 0 else 64
        assert all(int(x["len"]) >= eff_min for x in a[:-1])
        if bits > 32:  # never splits: the stream is its final chunk, level 0
            assert len(a) == (1 if n else 0)
            assert all(int(x["level"]) == 0 for x in a)


def test_multistream_oracle_equals_single(oracle, table):
    from bs_amd.synth import splitmix_array
    arrs = [splitmix_array(100 + i, n) for i, n in enumerate([0, 1, 5000, 70000, 200_000])]
    base = np.concatenate(arrs)
    lens = [len(a) for a in arrs]
    off = np.concatenate([[0], np.cumsum(lens)[:-1]])
    ch, counts = oracle.split_streams(table, base, off, lens, bits=10, min_size=256, threads=3)
    k = 0
    for i, a in enumerate(arrs):
        one = oracle.split(table, a, bits=10, min_size=256)
        assert counts[i] == len(one)
        got = ch[k:k + len(one)]
        assert (got["offset"] == one["offset"]).all() and (got["ref"] == one["ref"]).all()
        assert (got["stream"] == i).all()
        k += len(one)


def test_edit_stream_boundaries_resynchronise(oracle, table):
    """Config 5's premise on the oracle (8 MiB, 8 edits): content-defined boundaries realign
    after each edit, so the chunks of the edited stream are mostly chunks of the original."""
    from bs_amd.synth import edit_stream, splitmix_array
    a = splitmix_array(0xB5B52026, 8 << 20)
    b = edit_stream(a, 0xB5B52026 + 5, sites=8)
    assert len(b) != len(a) or not np.array_equal(a, b)
    assert np.array_equal(b, edit_stream(a, 0xB5B52026 + 5, sites=8))  # deterministic
    ca, cb = oracle.split(table, a), oracle.split(table, b)
    refs_a = {bytes(r) for r in ca["ref"]}
    shared = sum(bytes(r) in refs_a for r in cb["ref"]) / len(cb)
    assert 0.75 < shared < 1.0, shared


def test_sha256_implementations_agree(oracle):
    """The C oracle's SHA-256 with the x86 SHA extensions (the CPU baseline's, as Go's amd64
    crypto/sha256) and its scalar FIPS 180-4 compression give hashlib's digests."""
    rng = np.random.default_rng(5)
    msgs = [rng.integers(0, 256, n, dtype=np.uint8).tobytes()
            for n in list(range(0, 300)) + [1000, 4096, 100_000]]
    try:
        for ni in (True, False):
            impl = oracle.sha256_use(ni)
            assert impl == ("scalar" if not ni else impl)
            for m in msgs:
                assert oracle.sha256(m) == hashlib.sha256(m).digest(), (impl, len(m))
    finally:
        oracle.sha256_use(True)


@pytest.mark.parametrize("name,bits,min_size,fanout", [
    ("commonsense.txt", 16, 1024, 8), ("commonsense.txt", 8, 64, 2), ("commonsense.txt", 4, 0, 1),
    ("yubnub.opus", 4, 1024, 2), ("yubnub.opus", 12, 1024, 4), ("yubnub.opus", 16, 1024, 8)])
def test_c_writer_root_matches_python_tree(oracle, table, name, bits, min_size, fanout):
    """bso_writer_root (C, the full-Writer CPU baseline) == py_tree_root over the same chunks."""
    data = read_golden(name)
    ch = oracle.split(table, data, bits=bits, min_size=min_size)
    store = {}
    want = oracle.py_tree_root(
        [(data[int(c["offset"]):int(c["offset"] + c["len"])], int(c["level"])) for c in ch],
        fanout, store)
    root, puts = oracle.writer_root(table, data, bits=bits, min_size=min_size, fanout=fanout,
                                    keep_copies=True)
    assert root == want
    assert puts >= len(store)  # every chunk and node Put (duplicates included)
    assert oracle.writer_root(table, data, bits=bits, min_size=min_size, fanout=fanout)[0] == want


def test_c_writer_root_empty_and_synthetic(oracle, table):
    assert oracle.writer_root(table, b"")[0] == bytes(32)  # Root stays bs.Zero
    from bs_amd.synth import splitmix_bytes
    data = splitmix_bytes(7, 3_000_000)
    for bits, fanout in ((10, 2), (13, 8), (16, 4)):
        ch = oracle.split(table, data, bits=bits, min_size=64)
        want = oracle.py_tree_root(
            [(data[int(c["offset"]):int(c["offset"] + c["len"])], int(c["level"])) for c in ch],
            fanout)
        assert oracle.writer_root(table, data, bits=bits, min_size=64, fanout=fanout)[0] == want


def test_tree_root_variant_fixture(oracle, table):
    """tests/golden/tree_root_variants.json (make_tree_fixture.py): the Roots of both
    TreeBuilder.Root fold variants, regenerated by the C oracle and the Python tree restatement;
    the variants differ exactly on the cases marked so (the stream's last chunk closes a level
    below a taller tree)."""
    from bs_amd.synth import splitmix_array
    from conftest import load_json
    doc = load_json("tree_root_variants.json")
    assert doc["library_variant"] == "nonempty"
    assert any(c["variants_differ"] for c in doc["cases"])
    assert any(not c["variants_differ"] for c in doc["cases"])
    for c in doc["cases"]:
        data = splitmix_array(c["seed"], c["length"])
        kw = dict(bits=c["bits"], min_size=c["min_size"], fanout=c["fanout"])
        ch = oracle.split(table, data, bits=c["bits"], min_size=c["min_size"])
        assert len(ch) == c["chunks"] and int(ch["level"][-1]) == c["last_chunk_level"]
        assert int(ch["offset"][-1] + ch["len"][-1]) == len(data)
        for fold in ("nonempty", "leaf_gated"):
            want = c["root_" + fold]
            assert oracle.writer_root(table, data, fold=fold, **kw)[0].hex() == want
            if len(ch) < 500:
                pieces = [(data[int(x["offset"]):int(x["offset"] + x["len"])], int(x["level"]))
                          for x in ch]
                assert oracle.py_tree_root(pieces, c["fanout"], fold=fold).hex() == want
        assert (c["root_nonempty"] != c["root_leaf_gated"]) == c["variants_differ"]
