"""Python binding of libbsgpu (include/bsgpu.h) via ctypes.

This is plumbing for tests and bench.py; it carries no compute of its own. Every function
runs on the HIP path and raises if the shared library is missing or a call fails — there is no
CPU fallback anywhere in bs_amd.

Reference surface mirrored: split.NewWriter / Write / Close / Root options Bits, MinSize,
Fanout (/root/reference/split/split.go:44-165) and bs.Blob.Ref (/root/reference/bs.go:24-26).
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import re

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("BSG_LIB_PATH") or os.path.join(_HERE, "libbsgpu.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "bsgpu.h")

BSG_OK = 0
READ_SLACK = 256  # BSG_READ_SLACK: readable bytes required after the last stream
ERRORS = {-22: "EINVAL", -12: "ENOMEM", -5: "EDEVICE", -71: "ESTATE", -19: "ENODEV",
          -2: "ENOTFOUND", -74: "ECORRUPT", -1001: "EIO"}


class BsgError(RuntimeError):
    def __init__(self, code: int, what: str = ""):
        self.code = code
        super().__init__(f"{what}: bsgpu error {code} ({ERRORS.get(code, '?')})")


class Params(ctypes.Structure):
    _fields_ = [("split_bits", ctypes.c_uint32), ("min_size", ctypes.c_uint32),
                ("fanout", ctypes.c_uint32), ("reserved", ctypes.c_uint32)]


class StreamStats(ctypes.Structure):
    """bsg_stream_stats (include/bsgpu.h): where a stream's host-to-device time went."""
    _fields_ = [("host_bytes", ctypes.c_uint64), ("host_copy_ns", ctypes.c_uint64),
                ("stage_wait_ns", ctypes.c_uint64), ("h2d_bytes", ctypes.c_uint64),
                ("h2d_copies", ctypes.c_uint64), ("h2d_busy_ns", ctypes.c_uint64),
                ("h2d_span_ns", ctypes.c_uint64), ("copy_bytes_node", ctypes.c_uint64 * 4),
                ("last_tile_ns", ctypes.c_uint64), ("tail_ns", ctypes.c_uint64),
                ("gpu_node", ctypes.c_int32), ("stage_nodes", ctypes.c_uint32),
                ("src_nodes", ctypes.c_uint32), ("copy_nt", ctypes.c_uint32)]

    def as_dict(self) -> dict:
        def gbs(b, ns):
            return round(b / ns, 2) if ns else None  # bytes per ns = GB/s

        def nodes(mask):
            return [k for k in range(32) if mask >> k & 1]
        return {"host_copy_ms": round(self.host_copy_ns / 1e6, 3),
                "host_copy_gbs": gbs(self.host_bytes, self.host_copy_ns),
                "stage_wait_ms": round(self.stage_wait_ns / 1e6, 3),
                "h2d_busy_ms": round(self.h2d_busy_ns / 1e6, 3),
                "h2d_busy_gbs": gbs(self.h2d_bytes, self.h2d_busy_ns),
                "h2d_span_ms": round(self.h2d_span_ns / 1e6, 3),
                "h2d_span_gbs": gbs(self.h2d_bytes, self.h2d_span_ns),
                "h2d_copies": int(self.h2d_copies),
                "last_tile_ms": round(self.last_tile_ns / 1e6, 3),
                "tail_after_h2d_ms": round(self.tail_ns / 1e6, 3),
                "copy_mib_by_node": [int(b) >> 20 for b in self.copy_bytes_node],
                "gpu_node": int(self.gpu_node), "stage_nodes": nodes(self.stage_nodes),
                "src_nodes": nodes(self.src_nodes), "copy_nt": int(self.copy_nt)}


CHUNK_DTYPE = np.dtype(
    [("offset", "<u8"), ("len", "<u8"), ("level", "<u4"), ("stream", "<u4"), ("ref", "u1", (32,))]
)
assert CHUNK_DTYPE.itemsize == 56

_lib = None


def exported_symbols_from_header(path: str = HEADER_PATH) -> list[str]:
    """Every function name declared in include/bsgpu.h."""
    text = open(path).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(bsg_[a-z0-9_]+)\s*\(", text)))


def lib() -> ctypes.CDLL:
    """Load libbsgpu.so (built by `python -m bs_amd.build`). Raises if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} not built: run `python -m bs_amd.build` "
                           "(the HIP path is the only path; there is no CPU fallback)")
    L = ctypes.CDLL(LIB_PATH)
    vp, u8p, u32p, u64p = (ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint8),
                           ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint64))
    sig = {
        "bsg_errstr": (ctypes.c_char_p, [ctypes.c_int]),
        "bsg_params_default": (Params, []),
        "bsg_default_table": (None, [u32p]),
        "bsg_device_count": (ctypes.c_int, []),
        "bsg_init": (ctypes.c_int, [ctypes.c_int]),
        "bsg_open": (vp, [ctypes.c_int, ctypes.POINTER(Params), u32p, ctypes.POINTER(ctypes.c_int)]),
        "bsg_write": (ctypes.c_int, [vp, vp, ctypes.c_size_t]),
        "bsg_close": (ctypes.c_int, [vp]),
        "bsg_close_begin": (ctypes.c_int, [vp]),
        "bsg_close_step": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_size_t)]),
        "bsg_pending": (ctypes.c_size_t, [vp]),
        "bsg_drain": (ctypes.c_size_t, [vp, vp, ctypes.c_size_t]),
        "bsg_set_tile": (ctypes.c_int, [vp, ctypes.c_size_t]),
        "bsg_set_carry_cap": (ctypes.c_int, [vp, ctypes.c_size_t]),
        "bsg_write_window": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_void_p),
                                            ctypes.POINTER(ctypes.c_size_t)]),
        "bsg_write_commit": (ctypes.c_int, [vp, ctypes.c_size_t]),
        "bsg_host_register": (ctypes.c_int, [vp, ctypes.c_size_t]),
        "bsg_host_unregister": (ctypes.c_int, [vp]),
        "bsg_write_pinned": (ctypes.c_int, [vp, vp, ctypes.c_size_t]),
        "bsg_free": (None, [vp]),
        "bsg_reset": (ctypes.c_int, [vp]),
        "bsg_engine_create": (vp, [ctypes.c_int, u32p, ctypes.POINTER(ctypes.c_int)]),
        "bsg_engine_destroy": (None, [vp]),
        "bsg_engine_run": (ctypes.c_int, [vp, vp, u64p, u64p, ctypes.c_uint32,
                                          ctypes.POINTER(Params)]),
        "bsg_engine_hash": (ctypes.c_int, [vp, vp, u64p, u64p, ctypes.c_uint32]),
        "bsg_engine_finish": (ctypes.c_int, [vp, u64p]),
        "bsg_engine_chunks_device": (vp, [vp]),
        "bsg_engine_copy_chunks": (ctypes.c_int, [vp, vp, ctypes.c_uint64]),
        "bsg_engine_copy_counts": (ctypes.c_int, [vp, u64p, ctypes.c_uint32]),
        "bsg_engine_stream": (vp, [vp]),
        "bsg_engine_candidates": (ctypes.c_uint64, [vp]),
        "bsg_engine_profile": (ctypes.c_int, [vp, ctypes.c_int]),
        "bsg_engine_diag": (ctypes.c_int, [vp, u64p]),
        "bsg_engine_timeline": (ctypes.c_int, [vp, u64p]),
        "bsg_engine_stage_ms": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_float)]),
        "bsg_split_hash_batch": (ctypes.c_int, [ctypes.c_int, vp, u64p, u64p, ctypes.c_uint32,
                                                ctypes.POINTER(Params), u32p, vp,
                                                ctypes.c_uint64, u64p, u64p]),
        "bsg_sha256_batch": (ctypes.c_int, [ctypes.c_int, vp, u64p, u64p, ctypes.c_uint32, vp]),
        "bsg_hasher_new": (vp, [ctypes.c_int]),
        "bsg_hasher_sum": (ctypes.c_int, [vp, vp, u64p, u64p, ctypes.c_uint32, vp]),
        "bsg_hasher_sum_ptrs": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_void_p), u64p,
                                               ctypes.c_uint32, vp]),
        "bsg_hasher_free": (None, [vp]),
        "bsg_hasher_pinned_bytes": (ctypes.c_size_t, [vp]),
        "bsg_fill_splitmix": (ctypes.c_int, [ctypes.c_int, vp, ctypes.c_uint64, ctypes.c_uint64,
                                             vp]),
        "bsg_device_malloc": (vp, [ctypes.c_int, ctypes.c_size_t]),
        "bsg_device_free": (ctypes.c_int, [ctypes.c_int, vp]),
        "bsg_memcpy": (ctypes.c_int, [ctypes.c_int, vp, vp, ctypes.c_size_t, ctypes.c_int]),
        "bsg_device_synchronize": (ctypes.c_int, [ctypes.c_int]),
        "bsg_memstore_new": (vp, [ctypes.c_int]),
        "bsg_filestore_new": (vp, [ctypes.c_char_p, ctypes.c_int]),
        "bsg_store_free": (None, [vp]),
        "bsg_store_count": (ctypes.c_size_t, [vp]),
        "bsg_filestore_set_write_behind": (ctypes.c_int, [vp, ctypes.c_uint64]),
        "bsg_store_held_bytes": (ctypes.c_size_t, [vp]),
        "bsg_store_get": (ctypes.c_int, [vp, vp, vp, ctypes.c_size_t,
                                         ctypes.POINTER(ctypes.c_size_t)]),
        "bsg_store_put": (ctypes.c_int, [vp, vp, ctypes.c_size_t, vp,
                                         ctypes.POINTER(ctypes.c_int)]),
        "bsg_store_list": (ctypes.c_size_t, [vp, vp, ctypes.c_size_t]),
        "bsg_store_put_ref": (ctypes.c_int, [vp, vp, vp, ctypes.c_size_t,
                                             ctypes.POINTER(ctypes.c_int)]),
        "bsg_store_list_from": (ctypes.c_size_t, [vp, vp, vp, ctypes.c_size_t]),
        "bsg_store_delete": (ctypes.c_int, [vp, vp]),
        "bsg_split_protect": (ctypes.c_int, [vp, vp, vp, vp, ctypes.c_size_t,
                                             ctypes.POINTER(ctypes.c_size_t)]),
        "bsg_writer_new": (vp, [ctypes.c_int, vp, ctypes.POINTER(Params), ctypes.c_size_t,
                                ctypes.POINTER(ctypes.c_int)]),
        "bsg_writer_write": (ctypes.c_int, [vp, vp, ctypes.c_size_t]),
        "bsg_writer_close": (ctypes.c_int, [vp]),
        "bsg_writer_root": (ctypes.c_int, [vp, vp]),
        "bsg_writer_timings": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_double)]),
        "bsg_stream_stats_get": (ctypes.c_int, [vp, ctypes.POINTER(StreamStats)]),
        "bsg_writer_free": (None, [vp]),
        "bsg_reader_new": (vp, [vp, vp, ctypes.POINTER(ctypes.c_int)]),
        "bsg_reader_open": (vp, [vp, vp, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]),
        "bsg_reader_read": (ctypes.c_int64, [vp, vp, ctypes.c_size_t]),
        "bsg_reader_seek": (ctypes.c_int64, [vp, ctypes.c_int64, ctypes.c_int]),
        "bsg_reader_size": (ctypes.c_uint64, [vp]),
        "bsg_reader_stats": (ctypes.c_int, [vp, u64p]),
        "bsg_debug_set": (ctypes.c_int, [ctypes.c_int, ctypes.c_int64]),
        "bsg_debug_get": (ctypes.c_int64, [ctypes.c_int]),
        "bsg_set_stream_base": (ctypes.c_int, [vp, ctypes.c_uint64]),
        "bsg_writer_set_stream_base": (ctypes.c_int, [vp, ctypes.c_uint64]),
        "bsg_reader_free": (None, [vp]),
    }
    partial = os.environ.get("BSG_LIB_PARTIAL") == "1"  # A/B of older builds (tools/)
    for name, (res, args) in sig.items():
        if partial and not hasattr(L, name):
            continue
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def _check(rc: int, what: str) -> None:
    if rc != BSG_OK:
        raise BsgError(rc, what)


def _as_u8(data) -> np.ndarray:
    """Zero-copy uint8 view of bytes / bytearray / memoryview / ndarray."""
    if isinstance(data, np.ndarray):
        return np.ascontiguousarray(data.reshape(-1).view(np.uint8))
    return np.frombuffer(data, dtype=np.uint8)


def _u64(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.uint64))


def _p(a: np.ndarray, ct):
    return a.ctypes.data_as(ctypes.POINTER(ct))


# bsg_debug_set
(KNOB_SEQ_WAIT, KNOB_LONG_MODE, KNOB_VERIFY_WINDOW, KNOB_EARLY, KNOB_POLL, KNOB_COPY_NT,
 KNOB_LIGHT_BYTES) = range(1, 8)


def debug_get(knob: int) -> int:
    return int(lib().bsg_debug_get(knob))


def debug_set(knob: int, value: int) -> None:
    """bsg_debug_set: a process-wide test knob (no environment changes at run time)."""
    _check(lib().bsg_debug_set(knob, value), "bsg_debug_set")


@contextlib.contextmanager
def debug_knob(knob: int, value: int):
    old = debug_get(knob)
    debug_set(knob, value)
    try:
        yield
    finally:
        debug_set(knob, old)


def device_count() -> int:
    return lib().bsg_device_count()


def init(device: int = 0) -> None:
    """bsg_init: the process's one-time device / kernel / thread start-up, done up front."""
    _check(lib().bsg_init(device), "bsg_init")


def default_table() -> np.ndarray:
    t = np.zeros(256, dtype=np.uint32)
    lib().bsg_default_table(_p(t, ctypes.c_uint32))
    return t


def params(bits: int = 16, min_size: int = 1024, fanout: int = 8) -> Params:
    """split.NewWriter defaults (split/split.go:48,88-89); pass Bits/MinSize/Fanout overrides."""
    return Params(bits, min_size, fanout, 0)


def _table_arg(table):
    if table is None:
        return None, None
    t = np.ascontiguousarray(np.asarray(table, dtype=np.uint32))
    assert t.shape == (256,)
    return t, _p(t, ctypes.c_uint32)


def split_hash_batch(streams: list[bytes] | list[np.ndarray], bits: int = 16,
                     min_size: int = 1024, table=None, device: int = 0):
    """Split + hash host-resident streams on the GPU. Returns (chunks, counts)."""
    arrs = [np.frombuffer(bytes(s), dtype=np.uint8) if not isinstance(s, np.ndarray)
            else np.ascontiguousarray(s, dtype=np.uint8) for s in streams]
    lens = _u64([len(a) for a in arrs])
    off = _u64(np.concatenate([[0], np.cumsum(lens)[:-1]]) if len(arrs) else [])
    base = np.concatenate(arrs) if arrs else np.zeros(1, np.uint8)
    if base.size == 0:
        base = np.zeros(1, np.uint8)
    cap = int(sum(int(l) // (min_size or 64) + 2 for l in lens)) + 1
    out = np.zeros(cap, dtype=CHUNK_DTYPE)
    counts = np.zeros(max(len(arrs), 1), dtype=np.uint64)
    n = ctypes.c_uint64(0)
    p = params(bits, min_size)
    _t, tp = _table_arg(table)
    rc = lib().bsg_split_hash_batch(device, base.ctypes.data, _p(off, ctypes.c_uint64),
                                    _p(lens, ctypes.c_uint64), len(arrs), ctypes.byref(p), tp,
                                    out.ctypes.data, cap, _p(counts, ctypes.c_uint64),
                                    ctypes.byref(n))
    _check(rc, "bsg_split_hash_batch")
    return out[: n.value], counts[: len(arrs)]


def sha256_batch(blobs: list[bytes], device: int = 0) -> list[bytes]:
    arrs = [np.frombuffer(bytes(b), dtype=np.uint8) for b in blobs]
    lens = _u64([len(a) for a in arrs])
    off = _u64(np.concatenate([[0], np.cumsum(lens)[:-1]]) if arrs else [])
    base = np.concatenate(arrs) if arrs else np.zeros(1, np.uint8)
    if base.size == 0:
        base = np.zeros(1, np.uint8)
    refs = np.zeros(32 * max(len(arrs), 1), dtype=np.uint8)
    rc = lib().bsg_sha256_batch(device, base.ctypes.data, _p(off, ctypes.c_uint64),
                                _p(lens, ctypes.c_uint64), len(arrs), refs.ctypes.data)
    _check(rc, "bsg_sha256_batch")
    return [refs[32 * i:32 * i + 32].tobytes() for i in range(len(arrs))]


class Hasher:
    """bsg_hasher: persistent batched SHA-256 (Blob.Ref of many blobs)."""

    def __init__(self, device: int = 0):
        self.h = lib().bsg_hasher_new(device)
        if not self.h:
            raise BsgError(-19, "bsg_hasher_new")

    def sum_ptrs(self, blobs: list) -> list[bytes]:
        """Scattered host blobs (bsg_hasher_sum_ptrs): one GPU call, no packing by the caller."""
        keep = [np.frombuffer(bytes(b), dtype=np.uint8) if len(b) else np.zeros(1, np.uint8)
                for b in blobs]
        ptrs = (ctypes.c_void_p * max(len(keep), 1))(*[a.ctypes.data for a in keep])
        lens = _u64([len(b) for b in blobs])
        refs = np.zeros(32 * max(len(blobs), 1), dtype=np.uint8)
        _check(lib().bsg_hasher_sum_ptrs(self.h, ptrs, _p(lens, ctypes.c_uint64), len(blobs),
                                         refs.ctypes.data), "bsg_hasher_sum_ptrs")
        return [refs[32 * i:32 * i + 32].tobytes() for i in range(len(blobs))]

    def sum(self, blobs: list) -> list[bytes]:
        """Blobs packed into one host buffer (bsg_hasher_sum)."""
        arrs = [np.frombuffer(bytes(b), dtype=np.uint8) for b in blobs]
        lens = _u64([len(a) for a in arrs])
        off = _u64(np.concatenate([[0], np.cumsum(lens)[:-1]]) if arrs else [])
        base = np.concatenate(arrs) if arrs and sum(len(a) for a in arrs) else np.zeros(1, np.uint8)
        refs = np.zeros(32 * max(len(arrs), 1), dtype=np.uint8)
        _check(lib().bsg_hasher_sum(self.h, base.ctypes.data, _p(off, ctypes.c_uint64),
                                    _p(lens, ctypes.c_uint64), len(arrs), refs.ctypes.data),
               "bsg_hasher_sum")
        return [refs[32 * i:32 * i + 32].tobytes() for i in range(len(blobs))]

    def pinned_bytes(self) -> int:
        """bsg_hasher_pinned_bytes: pinned host memory the hasher holds (diagnostics)."""
        return int(lib().bsg_hasher_pinned_bytes(self.h))

    def free(self):
        if self.h:
            lib().bsg_hasher_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def host_register(ptr: int, n: int) -> None:
    """bsg_host_register: page-lock caller memory for bsg_write_pinned."""
    _check(lib().bsg_host_register(ptr, n), "bsg_host_register")


def host_unregister(ptr: int) -> None:
    _check(lib().bsg_host_unregister(ptr), "bsg_host_unregister")


def fill_splitmix(ptr: int, nbytes: int, seed: int, stream: int | None = None,
                  device: int = 0) -> None:
    _check(lib().bsg_fill_splitmix(device, ptr, nbytes, seed, stream), "bsg_fill_splitmix")


class DeviceBuffer:
    """Raw HIP allocation owned by libbsgpu (torch ships its own HIP runtime, so GPU processes
    here never initialise torch's CUDA/HIP side)."""

    def __init__(self, nbytes: int, device: int = 0):
        self.device, self.nbytes = device, nbytes
        self.ptr = lib().bsg_device_malloc(device, nbytes + READ_SLACK)
        if not self.ptr:
            raise BsgError(-12, "bsg_device_malloc")

    def to_host(self, offset: int = 0, n: int | None = None) -> np.ndarray:
        n = self.nbytes - offset if n is None else n
        out = np.empty(max(n, 1), dtype=np.uint8)
        _check(lib().bsg_memcpy(self.device, out.ctypes.data, self.ptr + offset, n, 1),
               "bsg_memcpy")
        return out[:n]

    def from_host(self, a: np.ndarray, offset: int = 0) -> None:
        a = np.ascontiguousarray(a, dtype=np.uint8)
        _check(lib().bsg_memcpy(self.device, self.ptr + offset, a.ctypes.data, a.nbytes, 0),
               "bsg_memcpy")

    def free(self) -> None:
        if self.ptr:
            lib().bsg_device_free(self.device, self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def synchronize(device: int = 0) -> None:
    _check(lib().bsg_device_synchronize(device), "bsg_device_synchronize")


class Engine:
    """Device-resident batch of independent streams (bsg_engine_*)."""

    def __init__(self, device: int = 0, table=None):
        err = ctypes.c_int(0)
        self._t, tp = _table_arg(table)
        self.h = lib().bsg_engine_create(device, tp, ctypes.byref(err))
        if not self.h:
            raise BsgError(err.value, "bsg_engine_create")
        self.nstreams = 0

    def run(self, d_ptr: int, off, lens, bits: int = 16, min_size: int = 1024) -> None:
        self._off, self._len = _u64(off), _u64(lens)
        self._p = params(bits, min_size)
        self.nstreams = len(self._off)
        _check(lib().bsg_engine_run(self.h, d_ptr, _p(self._off, ctypes.c_uint64),
                                    _p(self._len, ctypes.c_uint64), self.nstreams,
                                    ctypes.byref(self._p)), "bsg_engine_run")

    def hash(self, d_ptr: int, off, lens) -> None:
        """bsg_engine_hash: SHA-256 of whole blobs (record i: blob i's ref), no splitting."""
        self._off, self._len = _u64(off), _u64(lens)
        self.nstreams = len(self._off)
        _check(lib().bsg_engine_hash(self.h, d_ptr, _p(self._off, ctypes.c_uint64),
                                     _p(self._len, ctypes.c_uint64), self.nstreams),
               "bsg_engine_hash")

    def finish(self) -> int:
        n = ctypes.c_uint64(0)
        _check(lib().bsg_engine_finish(self.h, ctypes.byref(n)), "bsg_engine_finish")
        self.nchunks = n.value
        return n.value

    def chunks(self) -> np.ndarray:
        out = np.zeros(max(self.nchunks, 1), dtype=CHUNK_DTYPE)
        _check(lib().bsg_engine_copy_chunks(self.h, out.ctypes.data, self.nchunks),
               "bsg_engine_copy_chunks")
        return out[: self.nchunks]

    def counts(self) -> np.ndarray:
        c = np.zeros(max(self.nstreams, 1), dtype=np.uint64)
        _check(lib().bsg_engine_copy_counts(self.h, _p(c, ctypes.c_uint64), self.nstreams),
               "bsg_engine_copy_counts")
        return c[: self.nstreams]

    @property
    def stream(self) -> int:
        return lib().bsg_engine_stream(self.h) or 0

    def profile(self, enable: int = 1) -> None:
        """bsg_engine_profile: 0 off, 1 (or True) every stage, 2 the SHA-256 stage only."""
        _check(lib().bsg_engine_profile(self.h, int(enable)), "bsg_engine_profile")

    def stage_ms(self) -> list[float]:
        out = (ctypes.c_float * 3)()
        _check(lib().bsg_engine_stage_ms(self.h, out), "bsg_engine_stage_ms")
        return [float(x) for x in out]

    def diag(self) -> dict:
        d = np.zeros(16, dtype=np.uint64)
        _check(lib().bsg_engine_diag(self.h, _p(d, ctypes.c_uint64)), "bsg_engine_diag")
        out = {"nlong": int(d[0]), "long_thresh": int(d[1]), "max_nblocks": int(d[2]),
               "nshort": int(d[13]), "wave_tickets": int(d[14]), "total_blocks": int(d[15])}
        t = np.zeros(4, dtype=np.uint64)
        _check(lib().bsg_engine_timeline(self.h, _p(t, ctypes.c_uint64)), "bsg_engine_timeline")
        if t[0] and t[1] and t[3]:  # microseconds after the first k_sha wave started (an
            t0 = int(t[0])           # early chain, KNOB_EARLY, starts before it: negative)
            out["timeline_us"] = {"long_start": round((int(t[1]) - t0) * 0.01, 1),
                                  "long_end": round((int(t[2]) - t0) * 0.01, 1),
                                  "lane_end": round((int(t[3]) - t0) * 0.01, 1)}
        if os.environ.get("BSG_DIAG_RAW") == "1":  # experiment builds (BSG_LANE_DIAG)
            out["diag2_raw"] = [int(x) for x in d[8:13]]
        for tag, o in (("long", 3), ("lane", 8)):
            cyc, rt, nb = int(d[o + 1] - d[o]), int(d[o + 3] - d[o + 2]), int(d[o + 4])
            if nb and rt:
                out[tag] = {"blocks": nb, "cycles_per_block": round(cyc / nb, 1),
                            "clock_ghz": round(cyc / (rt * 10.0), 3),
                            "us_per_block": round(rt * 0.01 / nb, 4)}
        return out

    @property
    def candidates(self) -> int:
        return lib().bsg_engine_candidates(self.h)

    def close(self) -> None:
        if self.h:
            lib().bsg_engine_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class StreamingSplitter:
    """bsg_open/bsg_write/bsg_close/bsg_drain: the C-ABI form of split.Writer's chunking."""

    def __init__(self, bits: int = 16, min_size: int = 1024, fanout: int = 8, table=None,
                 device: int = 0, tile: int | None = None, carry_cap: int | None = None):
        err = ctypes.c_int(0)
        self._p = params(bits, min_size, fanout)
        self._t, tp = _table_arg(table)
        self.h = lib().bsg_open(device, ctypes.byref(self._p), tp, ctypes.byref(err))
        if not self.h:
            raise BsgError(err.value, "bsg_open")
        if tile is not None:
            _check(lib().bsg_set_tile(self.h, tile), "bsg_set_tile")
        if carry_cap is not None:
            _check(lib().bsg_set_carry_cap(self.h, carry_cap), "bsg_set_carry_cap")

    def set_stream_base(self, base: int) -> None:
        """bsg_set_stream_base (tests): the stream's first byte has offset `base`."""
        _check(lib().bsg_set_stream_base(self.h, base), "bsg_set_stream_base")

    def write(self, data) -> int:
        a = _as_u8(data)
        _check(lib().bsg_write(self.h, a.ctypes.data, a.nbytes), "bsg_write")
        return a.nbytes

    def write_pinned(self, ptr: int, n: int) -> None:
        """bsg_write_pinned: n bytes at ptr, host memory registered with host_register; the
        caller keeps them unchanged until close()."""
        _check(lib().bsg_write_pinned(self.h, ptr, n), "bsg_write_pinned")

    def close(self) -> None:
        _check(lib().bsg_close(self.h), "bsg_close")

    def close_steps(self):
        """bsg_close_begin, then one bsg_close_step per tile still on the device; yields the
        chunks each step made drainable (their concatenation is what close() + drain() give)."""
        _check(lib().bsg_close_begin(self.h), "bsg_close_begin")
        left = ctypes.c_size_t(1)
        while left.value:
            _check(lib().bsg_close_step(self.h, ctypes.byref(left)), "bsg_close_step")
            yield self.drain()

    def reset(self) -> None:
        _check(lib().bsg_reset(self.h), "bsg_reset")

    def window(self) -> memoryview:
        """bsg_write_window: writable memoryview of pinned staging; fill, then commit(n)."""
        p, cap = ctypes.c_void_p(), ctypes.c_size_t()
        _check(lib().bsg_write_window(self.h, ctypes.byref(p), ctypes.byref(cap)),
               "bsg_write_window")
        return memoryview((ctypes.c_uint8 * cap.value).from_address(p.value)).cast("B")

    def commit(self, n: int) -> None:
        _check(lib().bsg_write_commit(self.h, n), "bsg_write_commit")

    def pread_file(self, path: str, threads: int = 8, piece: int = 16 << 20) -> int:
        """Reads a whole file straight into pinned staging with `threads` parallel preads per
        staging window (the form a Go caller gets with io.ReaderAt and goroutines)."""
        from concurrent.futures import ThreadPoolExecutor
        fd = os.open(path, os.O_RDONLY)
        try:
            size = os.fstat(fd).st_size
            pos = 0
            with ThreadPoolExecutor(threads) as ex:
                while pos < size:
                    win = self.window()
                    n = min(len(win), size - pos)
                    parts = [(o, min(piece, n - o)) for o in range(0, n, piece)]
                    got = list(ex.map(lambda p: os.preadv(fd, [win[p[0]:p[0] + p[1]]], pos + p[0]),
                                      parts))
                    if sum(got) != n:
                        raise OSError("short read")
                    self.commit(n)
                    pos += n
            return pos
        finally:
            os.close(fd)

    def read_from(self, f, piece: int = 32 << 20) -> int:
        """Reads a file object to EOF straight into pinned staging (readinto); returns bytes."""
        total = 0
        while True:
            win = self.window()
            k = f.readinto(win[:piece])
            if not k:
                return total
            self.commit(k)
            total += k

    def stats(self) -> dict:
        """bsg_stream_stats_get: host copy / H2D times and NUMA placement since open / reset."""
        st = StreamStats()
        _check(lib().bsg_stream_stats_get(self.h, ctypes.byref(st)), "bsg_stream_stats_get")
        return st.as_dict()

    def drain(self) -> np.ndarray:
        n = lib().bsg_pending(self.h)
        out = np.zeros(max(n, 1), dtype=CHUNK_DTYPE)
        got = lib().bsg_drain(self.h, out.ctypes.data, n)
        return out[:got]

    def free(self) -> None:
        if self.h:
            lib().bsg_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


# ---------------------------------------------------------------------------------------------
# C++ host mirror (include/bs_split.hpp) through its C ABI: store/mem, split.Writer/Reader.
# ---------------------------------------------------------------------------------------------
NOT_FOUND = -2    # BSG_ENOTFOUND = bs.ErrNotFound
CORRUPT = -74     # BSG_ECORRUPT: a fetched chunk does not hash to its ref (Reader verify)
READER_VERIFY = 1


class MemStore:
    """store/mem (store/mem/mem.go): refs are computed on the GPU."""

    def __init__(self, device: int = 0):
        self.h = lib().bsg_memstore_new(device)
        if not self.h:
            raise BsgError(-12, "bsg_memstore_new")

    def put(self, blob: bytes) -> tuple[bytes, bool]:
        ref = ctypes.create_string_buffer(32)
        added = ctypes.c_int(0)
        b = bytes(blob)
        _check(lib().bsg_store_put(self.h, b, len(b), ref, ctypes.byref(added)), "put")
        return ref.raw, bool(added.value)

    def put_ref(self, ref: bytes, blob: bytes) -> bool:
        """PutWithRef: store blob under a ref the caller computed (no hashing)."""
        added = ctypes.c_int(0)
        b = bytes(blob)
        _check(lib().bsg_store_put_ref(self.h, bytes(ref), b, len(b), ctypes.byref(added)),
               "put_ref")
        return bool(added.value)

    def refs_after(self, start: bytes) -> list[bytes]:
        """ListRefs(start, ...): refs > start, lexicographic."""
        n = lib().bsg_store_list_from(self.h, bytes(start), None, 0)
        buf = ctypes.create_string_buffer(32 * max(n, 1))
        lib().bsg_store_list_from(self.h, bytes(start), buf, n)
        return [buf.raw[32 * i:32 * i + 32] for i in range(n)]

    def get(self, ref: bytes) -> bytes:
        n = ctypes.c_size_t(0)
        rc = lib().bsg_store_get(self.h, bytes(ref), None, 0, ctypes.byref(n))
        if rc == NOT_FOUND:
            raise KeyError(bytes(ref).hex())
        _check(rc, "get")
        buf = ctypes.create_string_buffer(max(n.value, 1))
        _check(lib().bsg_store_get(self.h, bytes(ref), buf, n.value, ctypes.byref(n)), "get")
        return buf.raw[: n.value]

    def refs(self) -> list[bytes]:
        n = lib().bsg_store_list(self.h, None, 0)
        buf = ctypes.create_string_buffer(32 * max(n, 1))
        lib().bsg_store_list(self.h, buf, n)
        return [buf.raw[32 * i:32 * i + 32] for i in range(n)]

    def __len__(self) -> int:
        return lib().bsg_store_count(self.h)

    def held_bytes(self) -> int:
        """Host bytes the store keeps alive (store/mem: copies + aliased Write pieces)."""
        return lib().bsg_store_held_bytes(self.h)

    def delete(self, ref: bytes) -> None:
        """bs.DeleterStore.Delete (store/mem only)."""
        _check(lib().bsg_store_delete(self.h, bytes(ref)), "Delete")

    def protect_children(self, ref: bytes) -> list[tuple[bytes, bool]]:
        """split.Protect (split/split.go:306-322): [(child ref, traverse?)] of the Node at ref,
        child nodes (traverse=True) first, then leaves."""
        n = ctypes.c_size_t(0)
        _check(lib().bsg_split_protect(self.h, bytes(ref), None, None, 0, ctypes.byref(n)),
               "Protect")
        refs = ctypes.create_string_buffer(32 * max(n.value, 1))
        trav = ctypes.create_string_buffer(max(n.value, 1))
        _check(lib().bsg_split_protect(self.h, bytes(ref), refs, trav, n.value, ctypes.byref(n)),
               "Protect")
        return [(refs.raw[32 * i:32 * i + 32], trav.raw[i] == 1) for i in range(n.value)]

    def free(self):
        if self.h:
            lib().bsg_store_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class FileStore(MemStore):
    """store/file (store/file/file.go): one file per blob at root/blobs/hh/hhhh/<hex>; refs are
    computed on the GPU (or taken from the split kernels' chunk records by the Writer)."""

    def __init__(self, root: str, device: int = 0):  # noqa: D107 (no MemStore.__init__)
        self.root = root
        self.h = lib().bsg_filestore_new(os.fsencode(root), device)
        if not self.h:
            raise BsgError(-22, "bsg_filestore_new")

    def set_write_behind(self, nbytes: int) -> None:
        _check(lib().bsg_filestore_set_write_behind(self.h, nbytes), "set_write_behind")


class Writer:
    """split.NewWriter(ctx, st, Bits(..), MinSize(..), Fanout(..)) -> Write / Close / Root."""

    def __init__(self, store: MemStore, bits: int = 16, min_size: int = 1024, fanout: int = 8,
                 device: int = 0, tile: int = 0):
        err = ctypes.c_int(0)
        self._p = params(bits, min_size, fanout)
        self.h = lib().bsg_writer_new(device, store.h, ctypes.byref(self._p), tile,
                                      ctypes.byref(err))
        if not self.h:
            raise BsgError(err.value, "bsg_writer_new")
        self.store = store

    def set_stream_base(self, base: int) -> None:
        """bsg_writer_set_stream_base (tests), before the first write."""
        _check(lib().bsg_writer_set_stream_base(self.h, base), "bsg_writer_set_stream_base")

    def write(self, data) -> int:
        a = _as_u8(data)
        _check(lib().bsg_writer_write(self.h, a.ctypes.data, a.nbytes), "Write")
        return a.nbytes

    def close(self) -> None:
        _check(lib().bsg_writer_close(self.h), "Close")

    @property
    def root(self) -> bytes:
        out = ctypes.create_string_buffer(32)
        _check(lib().bsg_writer_root(self.h, out), "Root")
        return out.raw

    def timings(self) -> dict:
        """bsg_writer_timings, in ms: Write copies, background Put + tree, waits for it, node
        hashes, Close, Close's wait for the device, node-hash calls."""
        t = (ctypes.c_double * 7)()
        _check(lib().bsg_writer_timings(self.h, t), "bsg_writer_timings")
        keys = ("copy_ms", "put_tree_ms", "join_ms", "node_hash_ms", "close_ms", "close_dev_ms")
        out = {k: round(t[i] * 1e3, 3) for i, k in enumerate(keys)}
        out["node_hash_calls"] = int(t[6])
        return out

    def free(self):
        if self.h:
            lib().bsg_writer_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Reader:
    """split.NewReader(ctx, g, ref) -> Read / Seek / Size. verify=True checks each leaf node's
    chunks against their refs with one batched GPU SHA-256 call (BSG_READER_VERIFY)."""

    def __init__(self, store: MemStore, root: bytes, verify: bool = False, device: int = 0):
        err = ctypes.c_int(0)
        self.h = lib().bsg_reader_open(store.h, bytes(root), READER_VERIFY if verify else 0,
                                       device, ctypes.byref(err))
        if not self.h:
            raise BsgError(err.value, "bsg_reader_open")
        self.store = store

    def read(self, n: int) -> bytes:
        buf = ctypes.create_string_buffer(max(n, 1))
        got = lib().bsg_reader_read(self.h, buf, n)
        if got < 0:
            raise BsgError(int(got), "Read")
        return buf.raw[:got]

    def read_all(self) -> bytes:
        parts = []
        while True:
            b = self.read(1 << 20)
            if not b:
                return b"".join(parts)
            parts.append(b)

    def seek(self, off: int, whence: int = 0) -> int:
        return lib().bsg_reader_seek(self.h, off, whence)

    @property
    def size(self) -> int:
        return lib().bsg_reader_size(self.h)

    def stats(self) -> dict:
        """bsg_reader_stats (verify mode): windows verified on the reading thread / taken from
        the read-ahead, bytes verified, read-ahead windows dropped after a seek."""
        out = np.zeros(4, dtype=np.uint64)
        _check(lib().bsg_reader_stats(self.h, _p(out, ctypes.c_uint64)), "bsg_reader_stats")
        return {"sync_windows": int(out[0]), "ahead_windows": int(out[1]),
                "bytes": int(out[2]), "dropped": int(out[3])}

    def free(self):
        if self.h:
            lib().bsg_reader_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass
