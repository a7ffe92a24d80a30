"""store/file mirror (bs::FileStore) and the split.Reader's batched GPU verification.

Mirrors store/file/file_test.go TestStore (testutil.ReadWrite of yubnub.opus into a file store
in a temp dir) and testutil.AllRefs (random blobs, ListRefs returns exactly the added set in
lexicographic order). The on-disk layout is store/file/file.go:33-40
(<root>/blobs/<hex[:2]>/<hex[:4]>/<hex>); Put's O_EXCL semantics are file.go:59-66.
"""
import hashlib
import os

import numpy as np
import pytest

from conftest import read_golden

pytestmark = pytest.mark.gpu


def write_all(gpu, st, data: bytes, piece: int = 32 * 1024, **kw):
    w = gpu.Writer(st, **kw)
    for i in range(0, len(data), piece):
        w.write(data[i:i + piece])
    w.close()
    return w.root


def blob_path(root: str, ref: bytes) -> str:
    h = ref.hex()
    return os.path.join(root, "blobs", h[:2], h[:4], h)


def test_filestore_readwrite_yubnub(gpu, tmp_path, oracle, table):
    """file_test.go TestStore: ReadWrite(yubnub.opus); the tree equals the mem store's."""
    data = read_golden("yubnub.opus")
    fs = gpu.FileStore(str(tmp_path))
    root = write_all(gpu, fs, data)
    mem = gpu.MemStore()
    assert write_all(gpu, mem, data) == root
    assert sorted(fs.refs()) == sorted(mem.refs())
    assert gpu.Reader(fs, root).read_all() == data
    # every chunk the oracle finds is a file whose name is its SHA-256 and whose bytes are it
    for c in oracle.split(table, data):
        ref = bytes(c["ref"])
        with open(blob_path(str(tmp_path), ref), "rb") as f:
            blob = f.read()
        assert blob == data[int(c["offset"]):int(c["offset"] + c["len"])]
        assert hashlib.sha256(blob).digest() == ref


def test_filestore_put_get_exclusive(gpu, tmp_path):
    fs = gpu.FileStore(str(tmp_path))
    ref, added = fs.put(b"hello")
    assert ref == hashlib.sha256(b"hello").digest() and added
    assert os.path.isfile(blob_path(str(tmp_path), ref))
    assert fs.put(b"hello") == (ref, False)  # O_EXCL: already present
    assert fs.get(ref) == b"hello"
    with pytest.raises(KeyError):
        fs.get(bytes(32))
    e, added = fs.put(b"")                    # the empty blob is a valid blob
    assert e == hashlib.sha256(b"").digest() and added and fs.get(e) == b""


def test_filestore_allrefs(gpu, tmp_path):
    """testutil.AllRefs: ListRefs yields exactly the added refs, lexicographically."""
    rng = np.random.default_rng(5)
    fs = gpu.FileStore(str(tmp_path))
    want = set()
    for _ in range(200):
        n = int(rng.integers(0, 300))
        blob = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        ref, added = fs.put(blob)
        if added:
            want.add(ref)
    got = fs.refs()
    assert got == sorted(want)
    assert len(fs) == len(want)
    # stray entries the reference skips: non-hex dirs, wrong-length names, files at dir levels
    os.makedirs(os.path.join(str(tmp_path), "blobs", "zz", "zzzz"))
    os.makedirs(os.path.join(str(tmp_path), "blobs", "abc"))
    open(os.path.join(str(tmp_path), "blobs", "xy"), "w").close()
    assert fs.refs() == sorted(want)


def test_reader_verify_detects_corruption(gpu, tmp_path):
    from bs_amd.synth import splitmix_bytes
    data = splitmix_bytes(31, 3_000_000)
    fs = gpu.FileStore(str(tmp_path))
    root = write_all(gpu, fs, data, piece=1 << 20)
    assert gpu.Reader(fs, root, verify=True).read_all() == data
    r = gpu.Reader(fs, root, verify=True)
    r.seek(1_234_567, 0)
    assert r.read(100_000) == data[1_234_567:1_334_567]
    # flip one byte of one chunk file (not a tree node: pick a file holding stream bytes)
    victim = None
    for ref in fs.refs():
        b = fs.get(ref)
        if len(b) > 1000 and data.find(b) >= 0:
            victim = ref
            break
    assert victim is not None
    p = blob_path(str(tmp_path), victim)
    with open(p, "r+b") as f:
        f.seek(500)
        c = f.read(1)
        f.seek(500)
        f.write(bytes([c[0] ^ 0xFF]))
    assert gpu.Reader(fs, root).read_all() != data  # the reference trusts its store
    with pytest.raises(gpu.BsgError) as ei:
        gpu.Reader(fs, root, verify=True).read_all()
    assert ei.value.code == gpu.CORRUPT


@pytest.mark.parametrize("write_behind", [1 << 30, 1])
def test_writer_put_failure_surfaces(gpu, tmp_path, oracle, table, write_behind):
    """A chunk that store/file cannot write (its blobs/<hh> directory is a regular file) makes a
    later Write or the Close fail, as a Put error inside split.Writer's F propagates out of
    Write / Close in the reference (split/split.go:71-77, :104-126), and the Writer stays failed.
    The chunks are Put on the Writer's background
    thread while the next Write copies, so the error arrives one Write late or at Close."""
    from bs_amd.synth import splitmix_array
    data = splitmix_array(4242, 24 << 20).tobytes()
    chunks = oracle.split(table, data)
    bad = bytes(chunks[len(chunks) // 2]["ref"]).hex()
    root = str(tmp_path)
    os.makedirs(os.path.join(root, "blobs"), exist_ok=True)
    with open(os.path.join(root, "blobs", bad[:2]), "wb") as f:
        f.write(b"not a directory")
    fs = gpu.FileStore(root)
    fs.set_write_behind(write_behind)
    w = gpu.Writer(fs, tile=1 << 20)
    failed = None
    for i in range(0, len(data), 1 << 20):
        try:
            w.write(data[i:i + (1 << 20)])
        except gpu.BsgError as e:
            failed = e
            break
    if failed is None:
        with pytest.raises(gpu.BsgError):
            w.close()
    with pytest.raises(gpu.BsgError):    # sticky
        w.write(b"x")
    with pytest.raises(gpu.BsgError):
        w.close()
    w.free()
    fs.free()  # waits for the write-behind queue
    # every blob that did reach the disk is whole and named by its hash
    n = 0
    for dirpath, _, files in os.walk(os.path.join(root, "blobs")):
        for name in files:
            if len(name) != 64:
                continue  # the blocking file
            with open(os.path.join(dirpath, name), "rb") as f:
                assert hashlib.sha256(f.read()).hexdigest() == name
            n += 1
    assert n > 0
