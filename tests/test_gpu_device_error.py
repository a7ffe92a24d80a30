"""The device-error path: a k_sha sanity check that fails must surface as BSG_EDEVICE from the
call that finishes the run, never as a hang or as wrong records, and the context must be
usable again afterwards (bsgpu.h documents both).

The reference has no device, but its error convention is the one kept here: no
panics; a failure inside the chunker or a Put propagates out of Write / Close as an error
(split/split.go:99-126), and the caller may start over.

The test knob BSG_KNOB_SEQ_WAIT = 0 (bsg_debug_set; BSG_DEBUG_SEQ_WAIT in the environment is only
its starting value) makes every helper-wave handshake of k_sha (lds_seq_wait: the helped solo
chains of a lightly loaded launch) give up at once, which sets Counters::error exactly as a real
~1 s handshake timeout would.
"""

import pytest

pytestmark = pytest.mark.gpu

MiB = 1 << 20
EDEVICE = -5


def failing_handshakes():
    # a process-wide knob, not the environment: a setenv while library threads run races their
    # getenv
    from bs_amd import bsgpu
    return bsgpu.debug_knob(bsgpu.KNOB_SEQ_WAIT, 0)


def test_errstr_names_edevice(gpu):
    assert gpu.lib().bsg_errstr(EDEVICE) == b"HIP device error"


def test_engine_run_reports_and_recovers(gpu, oracle, table):
    from bs_amd.synth import splitmix_array
    n = 64 * MiB
    buf = gpu.DeviceBuffer(n)
    gpu.fill_splitmix(buf.ptr, n, 4242)
    eng = gpu.Engine()
    with failing_handshakes():
        eng.run(buf.ptr, [0], [n])
        with pytest.raises(gpu.BsgError) as e:
            eng.finish()
    assert e.value.code == EDEVICE
    # the same engine, next run: correct records
    eng.run(buf.ptr, [0], [n])
    eng.finish()
    got = eng.chunks()
    ref = oracle.split(table, splitmix_array(4242, n))
    assert len(got) == len(ref) and (got["ref"] == ref["ref"]).all()
    assert (got["offset"] == ref["offset"]).all() and (got["level"] == ref["level"]).all()
    eng.close()
    buf.free()


def test_streaming_context_sticky_then_reset(gpu, oracle, table):
    from bs_amd.synth import splitmix_array
    data = splitmix_array(4243, 48 * MiB)
    sp = gpu.StreamingSplitter()
    with failing_handshakes():
        sp.write(data)
        with pytest.raises(gpu.BsgError) as e:
            sp.close()
    assert e.value.code == EDEVICE
    # sticky: the failed stream keeps reporting its error
    assert gpu.lib().bsg_close(sp.h) == EDEVICE
    assert gpu.lib().bsg_write(sp.h, data.ctypes.data, 16) in (EDEVICE, -71)
    # bsg_reset starts a clean stream on the same context
    sp.reset()
    for i in range(0, len(data), 5 * MiB):
        sp.write(data[i:i + 5 * MiB])
    sp.close()
    got = sp.drain()
    ref = oracle.split(table, data)
    assert len(got) == len(ref) and (got["ref"] == ref["ref"]).all()
    sp.free()


def test_writer_close_returns_device_error(gpu, oracle, table):
    from bs_amd.synth import splitmix_array
    data = splitmix_array(4244, 40 * MiB)
    st = gpu.MemStore()
    w = gpu.Writer(st)
    with failing_handshakes():
        w.write(data)
        with pytest.raises(gpu.BsgError) as e:
            w.close()
    assert e.value.code == EDEVICE
    with pytest.raises(gpu.BsgError):  # the Writer is sticky-failed (Close is idempotent)
        w.close()
    w.free()  # its context goes back to the pool through bsg_reset
    # the next Writer (the pooled context) is correct
    w2 = gpu.Writer(st)
    w2.write(data)
    w2.close()
    want, _ = oracle.writer_root(table, data)
    assert w2.root == want
    w2.free()
    st.free()
