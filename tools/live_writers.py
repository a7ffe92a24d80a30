"""Latency of the library's short calls after bsg_init (one JSON line): six 1 MiB split::Writers
each opened while the earlier ones are still alive (each needs its own context, hasher and
streams), three pooled ones, bsg_split_hash_batch of 64 x 256 KiB streams and bsg_sha256_batch of
256 x 64 KiB blobs, six calls each (ms). BSG_INIT_STREAMS sets the warm stream pool.

  python tools/live_writers.py
"""
import os, sys, time, json
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from bs_amd import bsgpu
from bs_amd.synth import splitmix_array
bsgpu.init(0)
tag = os.environ.get("BSG_LIB_PATH", "default") + " init_streams=" + os.environ.get("BSG_INIT_STREAMS", "16")
data = splitmix_array(1, 1 << 20)
st = bsgpu.MemStore()
ws, out = [], []
for rep in range(6):  # each further Writer opened while the earlier ones are alive
    t0 = time.perf_counter(); w = bsgpu.Writer(st); w.write(data); w.close()
    out.append(round((time.perf_counter() - t0) * 1e3, 2)); ws.append(w)
for w in ws: w.free()
pooled = []
for rep in range(3):
    t0 = time.perf_counter(); w = bsgpu.Writer(st); w.write(data); w.close(); w.free()
    pooled.append(round((time.perf_counter() - t0) * 1e3, 2))
small = [splitmix_array(50 + i, 256 << 10) for i in range(64)]
bt = []
for rep in range(6):
    t0 = time.perf_counter(); ch, cnt = bsgpu.split_hash_batch(small)
    bt.append(round((time.perf_counter() - t0) * 1e3, 2))
sh = []
blobs = [bytes(splitmix_array(90 + i, 64 << 10)) for i in range(256)]
for rep in range(6):
    t0 = time.perf_counter(); r = bsgpu.sha256_batch(blobs)
    sh.append(round((time.perf_counter() - t0) * 1e3, 2))
print(json.dumps({"lib": tag, "live_writers_1m_ms": out, "pooled_writer_1m_ms": pooled,
                  "split_hash_batch_64x256k_ms": bt, "sha256_batch_256x64k_ms": sh}), flush=True)
