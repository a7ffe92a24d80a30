"""C-ABI library: builds, loads, exports every symbol include/bsgpu.h declares (no GPU needed)."""
import ctypes
import os
import subprocess

import numpy as np

from conftest import GOLD


def test_library_builds_and_exports_header_symbols():
    from bs_amd import build, bsgpu
    path = build.build()
    declared = bsgpu.exported_symbols_from_header()
    assert len(declared) >= 20
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True,
                         check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = [s for s in declared if s not in exported]
    assert not missing, missing
    L = bsgpu.lib()
    for s in declared:
        assert hasattr(L, s)


def test_struct_layout_and_defaults():
    from bs_amd import bsgpu
    from oracle.oracle import CHUNK_DTYPE as ORACLE_DTYPE
    assert bsgpu.CHUNK_DTYPE == ORACLE_DTYPE
    p = bsgpu.lib().bsg_params_default()
    assert (p.split_bits, p.min_size, p.fanout) == (16, 1024, 8)  # split/split.go:48,88-89
    assert ctypes.sizeof(bsgpu.Params) == 16
    # bsg_stream_stats (include/bsgpu.h): 13 u64 words (9 counters and copy_bytes_node[4]), then
    # gpu_node (i32) and three u32 masks/flags
    assert ctypes.sizeof(bsgpu.StreamStats) == 13 * 8 + 4 * 4
    assert bsgpu.StreamStats.gpu_node.offset == 13 * 8


def test_default_table_matches_golden():
    from bs_amd import bsgpu
    golden = np.fromfile(f"{GOLD}/buzhash32_table.bin", dtype="<u4")
    assert bsgpu.default_table().tolist() == golden.tolist()


def test_missing_library_fails_loudly(tmp_path):
    """No CPU fallback: with libbsgpu.so absent, every entry of the binding raises."""
    import os
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("from bs_amd import bsgpu\n"
            "try:\n    bsgpu.split_hash_batch([b'x' * 5000])\n"
            "except RuntimeError as e:\n    print('RAISED', e)\n")
    env = dict(os.environ, BSG_LIB_PATH=str(tmp_path / "absent.so"))
    out = subprocess.run([sys.executable, "-c", code], cwd=root, env=env, capture_output=True,
                         text=True, timeout=120)
    assert "RAISED" in out.stdout and "no CPU fallback" in out.stdout, out.stdout + out.stderr


def test_errstr_and_bad_device():
    from bs_amd import bsgpu
    L = bsgpu.lib()
    assert L.bsg_errstr(0) == b"ok"
    assert L.bsg_errstr(-22) == b"invalid argument"
    err = ctypes.c_int(0)
    n = L.bsg_device_count()
    h = L.bsg_open(n + 3, None, None, ctypes.byref(err))  # no such device
    assert not h and err.value == -19
    for code, text in ((-2, b"not found"), (-74, b"blob does not match its ref"),
                       (-1001, b"filesystem error"), (-12, b"out of memory")):
        assert L.bsg_errstr(code) == text
    # MinSize below the window and Bits above 32 are valid (split.go:137-152 accept any value):
    # never EINVAL; without a GPU the open fails only for want of a device
    for bits, mn in ((16, 32), (16, 1), (33, 64), (2**32 - 1, 1)):
        p = bsgpu.Params(bits, mn, 8, 0)
        h = L.bsg_open(0, ctypes.byref(p), None, ctypes.byref(err))
        if n == 0:
            assert not h and err.value == -19
        else:
            assert h and err.value == 0
            L.bsg_free(h)


def test_debug_knobs_and_null_handles():
    """bsg_debug_set / bsg_debug_get (the test knobs that replaced run-time getenv)
    and the round-4 entry points on null handles: no GPU needed."""
    from bs_amd import bsgpu
    L = bsgpu.lib()
    for knob in (bsgpu.KNOB_SEQ_WAIT, bsgpu.KNOB_LONG_MODE, bsgpu.KNOB_VERIFY_WINDOW,
                 bsgpu.KNOB_EARLY, bsgpu.KNOB_POLL, bsgpu.KNOB_COPY_NT, bsgpu.KNOB_LIGHT_BYTES):
        old = bsgpu.debug_get(knob)
        assert old >= 0
        with bsgpu.debug_knob(knob, 1):
            assert bsgpu.debug_get(knob) == 1
        assert bsgpu.debug_get(knob) == old
    assert L.bsg_debug_set(bsgpu.KNOB_LONG_MODE, 3) == -22   # 0 auto, 1 off, 2 all
    assert L.bsg_debug_set(bsgpu.KNOB_SEQ_WAIT, -1) == -22
    assert L.bsg_debug_set(bsgpu.KNOB_EARLY, 2) == -22       # 0 off, 1 on
    assert L.bsg_debug_set(bsgpu.KNOB_POLL, 2) == -22        # 0 block, 1 poll
    assert L.bsg_debug_set(bsgpu.KNOB_COPY_NT, 2) == -22     # 0 memcpy, 1 non-temporal
    if "BSG_POLL" not in os.environ:
        assert bsgpu.debug_get(bsgpu.KNOB_POLL) == 1         # the bounded poll is the default
    if "BSG_COPY_NT" not in os.environ:
        assert bsgpu.debug_get(bsgpu.KNOB_COPY_NT) == 1
    assert bsgpu.debug_get(bsgpu.KNOB_LIGHT_BYTES) == 4 << 30
    assert L.bsg_debug_set(99, 0) == -22 and L.bsg_debug_get(99) == -1
    out = np.zeros(4, dtype=np.uint64)
    assert L.bsg_reader_stats(None, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))) == -22
    assert L.bsg_set_stream_base(None, 1 << 40) == -22
    assert L.bsg_writer_set_stream_base(None, 1 << 40) == -22
    assert L.bsg_hasher_pinned_bytes(None) == 0
    assert L.bsg_engine_profile(None, 2) == -22          # modes 0, 1, 2 on a real engine
    st = (ctypes.c_float * 3)()
    assert L.bsg_engine_stage_ms(None, st) == -22
