"""Host-side store logic through the C ABI, no GPU: store/mem and store/file semantics.

PutWithRef takes the ref from the caller (as the Writer does with chunk records), so nothing
here launches a kernel. Semantics follow the reference:
  - Put / added flag: store/mem/mem.go:62-77, store/file/file.go:53-80 (O_EXCL create);
  - Get of an absent ref is bs.ErrNotFound: store/mem/mem.go:29-36, store/file/file.go:43-51;
  - ListRefs(start) yields refs > start in lexicographic order: store.go:13-24,
    store/mem/mem.go:39-59, store/file/file.go:83-160 (non-hex / wrong-length entries skipped);
  - on-disk layout root/blobs/hh/hhhh/<64 hex>: store/file/file.go:33-41.
"""
import hashlib
import os

import numpy as np
import pytest


def _blobs(n, seed=7):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        b = rng.integers(0, 256, int(rng.integers(0, 300)), dtype=np.uint8).tobytes()
        out.append((hashlib.sha256(b).digest(), b))
    return out


@pytest.fixture(params=["mem", "file"])
def store(request, tmp_path):
    from bs_amd import bsgpu
    if request.param == "mem":
        return bsgpu.MemStore()
    return bsgpu.FileStore(str(tmp_path / "fs"))


def test_put_get_added(store):
    items = _blobs(40)
    for r, b in items:
        assert store.put_ref(r, b) is True
    for r, b in items:
        assert store.put_ref(r, b) is False
    assert len(store) == len({r for r, _ in items})
    for r, b in items:
        assert store.get(r) == b
    with pytest.raises(KeyError):
        store.get(hashlib.sha256(b"absent").digest())


def test_list_refs_order_and_start(store):
    items = _blobs(60, seed=3)
    for r, b in items:
        store.put_ref(r, b)
    want = sorted({r for r, _ in items})
    assert store.refs() == want
    assert store.refs_after(bytes(32)) == want
    for k in (0, 1, 17, len(want) - 1):
        assert store.refs_after(want[k]) == want[k + 1:]
    # a start that is not itself a stored ref
    mid = bytes(want[30][:5]) + b"\xff" * 27
    assert store.refs_after(mid) == [r for r in want if r > mid]
    assert store.refs_after(b"\xff" * 32) == []


def test_empty_blob(store):
    r = hashlib.sha256(b"").digest()
    assert store.put_ref(r, b"") is True
    assert store.get(r) == b""
    assert store.refs() == [r]


def test_filestore_layout_and_stray_entries(tmp_path):
    from bs_amd import bsgpu
    root = tmp_path / "fs"
    fs = bsgpu.FileStore(str(root))
    items = _blobs(12, seed=11)
    for r, b in items:
        fs.put_ref(r, b)
    for r, b in items:
        h = r.hex()
        p = root / "blobs" / h[:2] / h[:4] / h
        assert p.read_bytes() == b
    want = sorted({r for r, _ in items})
    # entries ListRefs must skip: non-hex and wrong-length dirs, files at dir levels,
    # a directory where a blob would be, a non-ref file name inside a leaf dir
    blobs = root / "blobs"
    (blobs / "xy").mkdir()
    (blobs / "abc").mkdir()
    (blobs / "README").write_bytes(b"x")
    h0 = want[0].hex()
    (blobs / h0[:2] / "zzzz").mkdir()
    (blobs / h0[:2] / (h0[:2] + "0")).mkdir()
    (blobs / h0[:2] / h0[:4] / "notaref").write_bytes(b"x")
    (blobs / h0[:2] / h0[:4] / ("f" * 64)).mkdir()
    assert fs.refs() == want
    # a second store on the same root sees the same blobs
    fs2 = bsgpu.FileStore(str(root))
    assert fs2.refs() == want
    assert fs2.get(want[-1]) == dict(items)[want[-1]]


def test_filestore_readonly_root_reports_error(tmp_path):
    from bs_amd import bsgpu
    if os.geteuid() == 0:
        pytest.skip("root ignores directory permissions")
    root = tmp_path / "ro"
    root.mkdir()
    fs = bsgpu.FileStore(str(root))
    os.chmod(root, 0o500)
    try:
        r, b = _blobs(1)[0]
        with pytest.raises(bsgpu.BsgError):
            fs.put_ref(r, b)
    finally:
        os.chmod(root, 0o700)
