"""split.Reader over store/mem through the C ABI, no GPU (no verification, so no kernel runs).

The tree is built by the oracle's restatement of split.Writer's TreeBuilder + PutProto
(`py_tree_root`, split/split.go:51-126) and stored with PutWithRef, so nothing here hashes on
the device. Checks:
  - Read / Seek / Size against the bytes the tree was built from (split/split.go:181-303;
    testutil.ReadWrite reads a whole file back);
  - store contents the reference would never produce (a node blob altered under its ref, a
    missing blob): every Read / Seek either returns bytes or an error code — never a crash or an
    out-of-bounds copy. Go's bounds checks turn such trees into a panic (split.go:227-262), the
    C++ Reader into kCorrupt / kNotFound. The fuzz runs in a child process, so a fault there
    fails this test instead of ending the run.
"""
import hashlib
import os
import subprocess
import sys
import textwrap

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _tree(seed, n=200_000, fanout=2):
    from oracle import oracle as O
    rng = np.random.default_rng(seed)
    data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
    chunks, pos = [], 0
    while pos < n:
        ln = int(rng.integers(1, 4000))
        lvl = int(rng.choice([0, 0, 0, 1, 2, 3, 5, 9]))
        chunks.append((data[pos:pos + ln], lvl))
        pos += ln
    store = {}
    root = O.py_tree_root(chunks, fanout=fanout, store=store)
    leaves = {hashlib.sha256(c).digest() for c, _ in chunks}
    return data, root, store, leaves


def _memstore(blobs):
    from bs_amd import bsgpu
    st = bsgpu.MemStore()
    for r, b in blobs.items():
        st.put_ref(r, b)
    return st


@pytest.mark.parametrize("seed,fanout", [(1, 2), (2, 8), (3, 3)])
def test_reader_roundtrip_and_seeks(seed, fanout):
    from bs_amd import bsgpu
    data, root, blobs, _ = _tree(seed, fanout=fanout)
    st = _memstore(blobs)
    r = bsgpu.Reader(st, root)
    assert r.size == len(data)
    assert r.read_all() == data
    rng = np.random.default_rng(seed + 100)
    for _ in range(60):
        off = int(rng.integers(0, len(data) + 1))
        n = int(rng.integers(0, 20_000))
        assert r.seek(off, 0) == off
        assert r.read(n) == data[off:off + n]
    assert r.seek(-10, 2) == len(data) - 10 and r.read(100) == data[-10:]
    assert r.seek(0, 2) == len(data) and r.read(10) == b""
    r.free()
    st.free()


def test_reader_missing_chunk_is_an_error():
    from bs_amd import bsgpu
    data, root, blobs, leaves = _tree(4)
    gone = sorted(leaves)[len(leaves) // 2]
    del blobs[gone]
    st = _memstore(blobs)
    r = bsgpu.Reader(st, root)
    with pytest.raises(bsgpu.BsgError):
        r.read_all()
    r.free()
    st.free()


_FUZZ = textwrap.dedent("""
    import sys
    sys.path.insert(0, {root!r})
    import numpy as np
    from bs_amd import bsgpu
    from oracle import oracle as O
    from tests.test_reader_cpu import _tree, _memstore
    data, root, blobs, leaves = _tree({seed}, n=60_000, fanout=2)
    nodes = sorted(r for r in blobs if r not in leaves)
    leaves_l = sorted(leaves)
    rng = np.random.default_rng({seed})
    outcomes = {{"ok": 0, "err": 0}}
    for trial in range({trials}):
        bad = dict(blobs)
        for _ in range(int(rng.integers(1, 3))):
            ref = nodes[int(rng.integers(0, len(nodes)))]
            b = bytearray(bad[ref])
            kind = int(rng.integers(0, 8))
            if kind == 0 and b:                      # flip bytes
                for _ in range(int(rng.integers(1, 4))):
                    b[int(rng.integers(0, len(b)))] ^= int(rng.integers(1, 256))
            elif kind == 1 and b:                    # truncate
                b = b[:int(rng.integers(0, len(b)))]
            elif kind == 2:                          # append garbage
                b += rng.integers(0, 256, int(rng.integers(1, 40)), dtype=np.uint8).tobytes()
            elif kind == 3:                          # random bytes
                b = bytearray(rng.integers(0, 256, int(rng.integers(0, 200)),
                                           dtype=np.uint8).tobytes())
            else:                                    # well-formed node, wrong numbers
                nd, lv, off, size = O._unwrap(blobs, ref)
                kids = nd if (nd and (not lv or rng.integers(0, 2))) else lv
                if not kids:
                    continue
                k = int(rng.integers(0, len(kids)))
                if kind == 4:                        # a child offset anywhere
                    kids[k] = (kids[k][0], int(rng.integers(0, 2 * size + 2)))
                elif kind == 5:                      # node size / offset off
                    size = int(rng.integers(0, 2 * size + 2))
                    off = int(rng.integers(0, off + 3))
                elif kind == 6:                      # a child that points elsewhere
                    kids[k] = (leaves_l[int(rng.integers(0, len(leaves_l)))], kids[k][1])
                else:                                # a child repeated or dropped
                    if rng.integers(0, 2):
                        kids.insert(k, kids[k])
                    else:
                        kids.pop(k)
                b = bytearray(O.proto_node(nd, lv, off, size))
            bad[ref] = bytes(b)
        st = _memstore(bad)
        try:
            r = bsgpu.Reader(st, root)
        except bsgpu.BsgError:
            outcomes["err"] += 1
            st.free()
            continue
        try:
            size = r.size
            # Go's Read copies whole leaf chunks, so a corrupt tree may yield more or fewer
            # bytes than Size(); only a clean error or data is asserted, not the length.
            r.read_all()
            for _ in range(8):
                off = int(rng.integers(0, max(size, 1) + 1))
                r.seek(off, 0)
                r.read(int(rng.integers(0, 5000)))
            outcomes["ok"] += 1
        except bsgpu.BsgError:
            outcomes["err"] += 1
        r.free()
        st.free()
    print(outcomes)
""")


@pytest.mark.parametrize("seed", [11, 12])
def test_reader_corrupt_trees_never_crash(seed):
    code = _FUZZ.format(root=ROOT, seed=seed, trials=150)
    p = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True,
                       timeout=600)
    assert p.returncode == 0, (p.returncode, p.stdout[-2000:], p.stderr[-4000:])
    assert "'err'" in p.stdout
