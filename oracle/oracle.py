"""CPU ORACLE — test infrastructure only.

ctypes wrapper over oracle/libbsoracle.so (the C restatement in bsoracle.c) plus a pure-Python
restatement (`py_split`, `py_rolling_sums`) used to cross-check the C one on small inputs.
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module,
and only as the checker. The product path (bs_amd/) never imports it.

Reference anchors: split/split.go:85-89 (Splitter wiring + defaults), bs.go:24-26 (ref =
SHA-256). The Splitter / buzhash32 semantics are restated from github.com/bobg/hashsplit v1.1.1
and github.com/chmduquesne/rollinghash v4.0.0 (not in /root/reference; see bsoracle.c).
"""
from __future__ import annotations

import ctypes
import hashlib
import os
import subprocess
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libbsoracle.so")


class Chunk(ctypes.Structure):
    _fields_ = [
        ("offset", ctypes.c_uint64),
        ("len", ctypes.c_uint64),
        ("level", ctypes.c_uint32),
        ("stream", ctypes.c_uint32),
        ("ref", ctypes.c_uint8 * 32),
    ]


CHUNK_DTYPE = np.dtype(
    [("offset", "<u8"), ("len", "<u8"), ("level", "<u4"), ("stream", "<u4"), ("ref", "u1", (32,))]
)
assert CHUNK_DTYPE.itemsize == ctypes.sizeof(Chunk) == 56


def build() -> str:
    """Compile the oracle (gcc) in place; returns the .so path."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        u32p = ctypes.POINTER(ctypes.c_uint32)
        u64p = ctypes.POINTER(ctypes.c_uint64)
        L.bso_gorand_seed.argtypes = [ctypes.c_int64]
        L.bso_gorand_int63.restype = ctypes.c_int64
        L.bso_buzhash32_generate.argtypes = [ctypes.c_int64, u32p]
        L.bso_rolling_sums.argtypes = [u32p, u8p, ctypes.c_size_t, u32p]
        L.bso_sha256.argtypes = [u8p, ctypes.c_size_t, u8p]
        L.bso_sha256_impl.restype = ctypes.c_int
        L.bso_sha256_use.restype = ctypes.c_int
        L.bso_sha256_use.argtypes = [ctypes.c_int]
        L.bso_split.restype = ctypes.c_size_t
        L.bso_split.argtypes = [u32p, u8p, ctypes.c_size_t, ctypes.c_uint, ctypes.c_uint,
                                ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t]
        L.bso_split_streams.restype = ctypes.c_size_t
        L.bso_split_streams.argtypes = [u32p, u8p, u64p, u64p, ctypes.c_uint32, ctypes.c_uint,
                                        ctypes.c_uint, ctypes.c_int, ctypes.c_void_p,
                                        ctypes.c_size_t, u64p]
        L.bso_writer_root.restype = ctypes.c_size_t
        L.bso_writer_root.argtypes = [u32p, u8p, ctypes.c_size_t, ctypes.c_uint, ctypes.c_uint,
                                      ctypes.c_uint, ctypes.c_int, u8p]
        L.bso_writer_root_fold.restype = ctypes.c_size_t
        L.bso_writer_root_fold.argtypes = [u32p, u8p, ctypes.c_size_t, ctypes.c_uint,
                                           ctypes.c_uint, ctypes.c_uint, ctypes.c_int,
                                           ctypes.c_int, u8p]
        _lib = L
    return _lib


def _p(a: np.ndarray, ct):
    return a.ctypes.data_as(ctypes.POINTER(ct))


def gorand_int63(seed: int, n: int) -> list[int]:
    L = lib()
    L.bso_gorand_seed(seed)
    return [L.bso_gorand_int63() for _ in range(n)]


def buzhash32_table(seed: int = 1) -> np.ndarray:
    t = np.zeros(256, dtype=np.uint32)
    lib().bso_buzhash32_generate(seed, _p(t, ctypes.c_uint32))
    return t


def rolling_sums(table: np.ndarray, data: bytes | np.ndarray) -> np.ndarray:
    x = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    x = np.ascontiguousarray(x, dtype=np.uint8)
    out = np.zeros(len(x), dtype=np.uint32)
    t = np.ascontiguousarray(table, dtype=np.uint32)
    lib().bso_rolling_sums(_p(t, ctypes.c_uint32), _p(x, ctypes.c_uint8), len(x),
                           _p(out, ctypes.c_uint32))
    return out


def sha256(data: bytes | np.ndarray) -> bytes:
    x = np.ascontiguousarray(np.frombuffer(bytes(data), dtype=np.uint8))
    out = np.zeros(32, dtype=np.uint8)
    lib().bso_sha256(_p(x, ctypes.c_uint8), len(x), _p(out, ctypes.c_uint8))
    return out.tobytes()


def sha256_impl() -> str:
    """'sha-ni' or 'scalar': the compression the C oracle's SHA-256 uses on this host."""
    return "sha-ni" if lib().bso_sha256_impl() == 1 else "scalar"


def sha256_use(ni: bool) -> str:
    """Select SHA-NI (when the host has it) or the scalar compression; returns the one in use."""
    return "sha-ni" if lib().bso_sha256_use(int(ni)) == 1 else "scalar"


def split(table: np.ndarray, data, bits: int = 16, min_size: int = 1024,
          with_refs: bool = True) -> np.ndarray:
    """Chunks of one stream as a CHUNK_DTYPE array (offset, len, level, stream=0, ref)."""
    x = data if isinstance(data, np.ndarray) else np.frombuffer(bytes(data), dtype=np.uint8)
    x = np.ascontiguousarray(x, dtype=np.uint8)
    t = np.ascontiguousarray(table, dtype=np.uint32)
    L = lib()
    # one pass: every non-final chunk has >= MinSize bytes, so len // MinSize + 1 records fit
    ms = min_size if min_size > 0 else 64
    cap = len(x) // ms + 1
    out = np.empty(max(cap, 1), dtype=CHUNK_DTYPE)
    n = L.bso_split(_p(t, ctypes.c_uint32), _p(x, ctypes.c_uint8), len(x), bits, min_size,
                    int(with_refs), out.ctypes.data, cap)
    assert n <= cap
    return out[:n].copy() if n < cap // 2 else out[:n]


def split_streams(table: np.ndarray, base: np.ndarray, off, lens, bits: int = 16,
                  min_size: int = 1024, threads: int = 1) -> tuple[np.ndarray, np.ndarray]:
    """Multi-stream split+ref (threads = worker threads). Returns (chunks, counts)."""
    t = np.ascontiguousarray(table, dtype=np.uint32)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.uint64)
    base = np.ascontiguousarray(base, dtype=np.uint8)
    counts = np.zeros(len(off), dtype=np.uint64)
    ms = min_size if min_size > 0 else 64  # hashsplit: MinSize 0 means the 64-byte window
    cap = int(sum(int(l) // ms + 1 for l in lens))
    out = np.zeros(max(cap, 1), dtype=CHUNK_DTYPE)
    n = lib().bso_split_streams(_p(t, ctypes.c_uint32), _p(base, ctypes.c_uint8),
                                _p(off, ctypes.c_uint64), _p(lens, ctypes.c_uint64), len(off),
                                bits, min_size, threads, out.ctypes.data, cap,
                                _p(counts, ctypes.c_uint64))
    assert n <= cap
    return out[:n], counts


def writer_root(table: np.ndarray, data, bits: int = 16, min_size: int = 1024, fanout: int = 8,
                keep_copies: bool = False, fold: str = "nonempty") -> tuple[bytes, int]:
    """split.Writer end to end in C (Splitter + TreeBuilder + PutProto + Close): (Root, puts).
    keep_copies also copies every blob as store/mem's Put would (puts counts them). fold: the
    TreeBuilder.Root variant (py_tree_root)."""
    x = data if isinstance(data, np.ndarray) else np.frombuffer(bytes(data), dtype=np.uint8)
    x = np.ascontiguousarray(x, dtype=np.uint8)
    t = np.ascontiguousarray(table, dtype=np.uint32)
    root = np.zeros(32, dtype=np.uint8)
    mode = {"nonempty": 0, "leaf_gated": 1}[fold]
    puts = lib().bso_writer_root_fold(_p(t, ctypes.c_uint32), _p(x, ctypes.c_uint8), len(x),
                                      bits, min_size, fanout, int(keep_copies), mode,
                                      _p(root, ctypes.c_uint8))
    return root.tobytes(), int(puts)


# ---------------------------------------------------------------------------------------------
# Pure-Python restatement (small inputs only): literal Splitter + Buzhash32 loop.
# ---------------------------------------------------------------------------------------------
def _rotl(x: int, r: int) -> int:
    r &= 31
    return ((x << r) | (x >> (32 - r))) & 0xFFFFFFFF if r else x


def py_rolling_sums(table, data: bytes) -> list[int]:
    T = [int(v) for v in table]
    window = [0] * 64          # rs.Write(64 zero bytes)
    s = 0
    for _ in range(64):
        s = _rotl(s, 1) ^ T[0]
    oldest = 0
    out = []
    for c in data:             # Roll(c)
        h0 = T[window[oldest]]
        window[oldest] = c
        oldest = (oldest + 1) % 64
        s = _rotl(s, 1) ^ _rotl(h0, 64 % 32) ^ T[c]
        out.append(s)
    return out


def py_window_hash(table, data: bytes, p: int) -> int:
    """Closed form h(p) = XOR_{k<64} rotl(T[x[p-k]], k mod 32), x[j<0] = 0."""
    T = [int(v) for v in table]
    h = 0
    for k in range(64):
        j = p - k
        h ^= _rotl(T[data[j] if j >= 0 else 0], k % 32)
    return h


@dataclass
class PyChunk:
    offset: int
    len: int
    level: int
    ref: bytes


def py_split(table, data: bytes, bits: int = 16, min_size: int = 1024) -> list[PyChunk]:
    # hashsplit's zero defaults: SplitBits 0 -> 13, MinSize <= 0 -> 64 (the window) [recalled]
    bits = bits or 13
    min_size = min_size if min_size > 0 else 64
    sums = py_rolling_sums(table, data)
    out, start = [], 0
    for p, h in enumerate(sums):
        if p + 1 - start < min_size:
            continue
        tz = (h & -h).bit_length() - 1 if h else 32
        if tz >= bits:
            out.append(PyChunk(start, p + 1 - start, tz - bits,
                               hashlib.sha256(data[start:p + 1]).digest()))
            start = p + 1
    if start < len(data):
        h = sums[-1]
        tz = (h & -h).bit_length() - 1 if h else 32
        out.append(PyChunk(start, len(data) - start, tz - bits if tz >= bits else 0,
                           hashlib.sha256(data[start:]).digest()))
    return out


# ---------------------------------------------------------------------------------------------
# Tree + Root restatement (split.Writer.Close -> Root). Parity vs Go is UNPINNED: hashsplit's
# TreeBuilder (v1.1.1) is restated from its published source as recalled; see DESIGN.md.
#   split/split.go:51-83   F: PutProto child nodes, Put chunks, Node{Offset, Size, Nodes, Leaves}
#   split/split.go:85-87   tb.Add(chunk, level / fanout)
#   split/split.go:104-126 Close: tb.Root(); PutProto(root) -> Root (zero ref if no input)
#   split/split.proto:6-26 Node {nodes=1, leaves=2, offset=3, size=4}; Child {ref=1, offset=2}
# ---------------------------------------------------------------------------------------------
def _varint(v: int) -> bytes:
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def proto_child(ref: bytes, offset: int) -> bytes:
    out = b"\x0a" + _varint(len(ref)) + ref if ref else b""
    if offset:
        out += b"\x10" + _varint(offset)
    return out


def proto_node(nodes, leaves, offset: int, size: int) -> bytes:
    """proto3 wire format as Go's proto.Marshal emits it (field order, zero values omitted)."""
    out = bytearray()
    for ref, off in nodes:
        c = proto_child(ref, off)
        out += b"\x0a" + _varint(len(c)) + c
    for ref, off in leaves:
        c = proto_child(ref, off)
        out += b"\x12" + _varint(len(c)) + c
    if offset:
        out += b"\x18" + _varint(offset)
    if size:
        out += b"\x20" + _varint(size)
    return bytes(out)


class _TBNode:
    def __init__(self, offset=0, size=0):
        self.nodes, self.chunks, self.offset, self.size = [], [], offset, size


class _Wrapped:  # split.nodeWrapper: a finished Node (its children already stored)
    def __init__(self, nodes, leaves, offset, size):
        self.nodes, self.leaves, self.offset, self.size = nodes, leaves, offset, size

    def proto(self) -> bytes:
        return proto_node(self.nodes, self.leaves, self.offset, self.size)


def py_tree_root(chunks, fanout: int = 8, store: dict | None = None,
                 fold: str = "nonempty") -> bytes:
    """chunks: iterable of (chunk_bytes, level) in stream order; returns Writer.Root (32 bytes).
    Chunk refs are SHA-256 of their bytes (bs.go:24-26). If `store` is given (a dict), every
    Put lands in it (ref -> blob), like store/mem.

    fold selects the one recalled detail of hashsplit's TreeBuilder.Root that changes Root
    (DESIGN §2): "nonempty" (the library's choice, and the C oracle's) folds every non-empty
    level below the top into its parent; "leaf_gated" folds the levels only when the leaf level
    holds chunks, i.e. not when the last chunk itself closed a level (then any nodes waiting in
    the levels between are not under the Root). The two differ only when the last chunk closes
    a level while a level between it and the top is non-empty (tests/golden/tree_root_variants.json)."""
    assert fold in ("nonempty", "leaf_gated")
    store = {} if store is None else store

    def put(b: bytes) -> bytes:
        r = hashlib.sha256(b).digest()
        store[r] = b
        return r

    def F(n: _TBNode) -> _Wrapped:  # split/split.go:52-81
        off = n.offset
        nodes, leaves = [], []
        for child in n.nodes:
            nodes.append((put(child.proto()), off))
            off += child.size
        for ref, ln in n.chunks:
            leaves.append((ref, off))
            off += ln
        return _Wrapped(nodes, leaves, n.offset, n.size)

    levels: list[_TBNode] = []
    for data, level in chunks:  # hashsplit TreeBuilder.Add(bytes, level / fanout)
        ln = len(data)
        ref = put(bytes(data))
        level //= fanout
        if not levels:
            levels.append(_TBNode())
        levels[0].chunks.append((ref, ln))
        for n in levels:
            n.size += ln
        for i in range(level):
            if i == len(levels) - 1:
                levels.append(_TBNode(offset=levels[i].offset, size=levels[i].size))
            levels[i + 1].nodes.append(F(levels[i]))
            levels[i] = _TBNode(offset=levels[i + 1].offset + levels[i + 1].size)
    if not levels:
        return bytes(32)  # Root stays bs.Zero (split_test.go:15-25)
    # Root(): fold every non-empty level below the top into its parent
    if fold == "nonempty" or levels[0].chunks:
        for i in range(len(levels) - 1):
            if levels[i].chunks or levels[i].nodes:
                levels[i + 1].nodes.append(F(levels[i]))
    if len(levels) == 1:
        root = F(levels[0])
    else:
        top = levels[-1]
        if len(top.nodes) > 1:
            root = F(top)
        else:
            root = top.nodes[0]  # prune single-child roots (their F already ran)
            while len(root.nodes) == 1:
                root = _Wrapped(*_unwrap(store, root.nodes[0][0]))
    return put(root.proto())


def _unwrap(store, ref):
    """Decode a stored Node proto back into (nodes, leaves, offset, size)."""
    b = store[ref]
    nodes, leaves, offset, size = [], [], 0, 0
    i = 0

    def varint(i):
        v, s = 0, 0
        while True:
            c = b[i]; i += 1
            v |= (c & 0x7F) << s
            s += 7
            if c < 0x80:
                return v, i
    while i < len(b):
        tag, i = varint(i)
        f, wt = tag >> 3, tag & 7
        if wt == 2:
            ln, i = varint(i)
            sub = b[i:i + ln]; i += ln
            r, o, j = b"", 0, 0
            while j < len(sub):
                t2, j2 = sub[j], j + 1
                if t2 == 0x0a:
                    l2 = sub[j2]; r = bytes(sub[j2 + 1:j2 + 1 + l2]); j = j2 + 1 + l2
                else:
                    v, s, j = 0, 0, j2
                    while True:
                        c = sub[j]; j += 1
                        v |= (c & 0x7F) << s; s += 7
                        if c < 0x80:
                            break
                    o = v
            (nodes if f == 1 else leaves).append((r, o))
        else:
            v, i = varint(i)
            if f == 3:
                offset = v
            else:
                size = v
    return nodes, leaves, offset, size
