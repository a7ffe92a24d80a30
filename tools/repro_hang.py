"""Quick GPU sanity run of the SHA paths (BSG_LONG_MODE=off|all|auto) with the oracle check."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bs_amd import bsgpu
from bs_amd.synth import splitmix_bytes
from oracle import oracle as O
g = os.path.join(os.path.dirname(__file__), "..", "tests", "golden")
t = O.buzhash32_table(1)
for name, data, bits in [("yubnub", open(os.path.join(g, "yubnub.opus"), "rb").read(), 16),
                         ("rand200k", splitmix_bytes(3, 200_000), 20),
                         ("rand5M", splitmix_bytes(4, 5_000_000), 16)]:
    ch, _ = bsgpu.split_hash_batch([data], bits=bits, min_size=1024)
    ref = O.split(t, data, bits=bits, min_size=1024)
    ok = len(ch) == len(ref) and (ch["ref"] == ref["ref"]).all() and (ch["len"] == ref["len"]).all()
    print(os.environ.get("BSG_LONG_MODE", "auto"), name, len(ch), "OK" if ok else "MISMATCH", flush=True)
    assert ok
