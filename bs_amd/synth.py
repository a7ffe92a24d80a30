"""Synthetic, regenerable byte streams: SplitMix64 of a counter.

Word i (little-endian 8 bytes) of the stream with seed S is splitmix64(S + (i + 1) * GAMMA).
The same generator runs on the device (bsg_fill_splitmix in libbsgpu) so benchmarks can build
multi-GiB inputs directly in HBM; the host version here builds identical bytes for checks.
"""
from __future__ import annotations

import numpy as np

GAMMA = np.uint64(0x9E3779B97F4A7C15)
BASE_SEED = 0xB5B52026


def splitmix_words(seed: int, nwords: int, first: int = 0) -> np.ndarray:
    with np.errstate(over="ignore"):
        i = np.arange(first + 1, first + nwords + 1, dtype=np.uint64)
        z = np.uint64(seed) + i * GAMMA
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def splitmix_array(seed: int, n: int) -> np.ndarray:
    """n bytes as a uint8 numpy array."""
    w = splitmix_words(seed, (n + 7) // 8)
    return w.astype("<u8").view(np.uint8)[:n].copy()


def splitmix_bytes(seed: int, n: int) -> bytes:
    return splitmix_array(seed, n).tobytes()


def edit_stream(a: np.ndarray, seed: int, sites: int = 1024, span: int = 10486) -> np.ndarray:
    """Config 5 (dedup): stream B = stream A with `sites` seeded edits of `span` bytes each
    (overwrite / insert / delete, chosen uniformly) at uniform positions of A. Sites are applied
    in ascending position order; a site that falls inside the previous edit starts right after
    it. Built with one concatenate (linear in len(a))."""
    rng = np.random.default_rng(seed)
    pos = np.sort(rng.integers(0, max(len(a) - span, 1), size=sites))
    kinds = rng.integers(0, 3, size=sites)
    fills = rng.integers(0, 256, size=(sites, span), dtype=np.uint8)
    parts = []
    cur = 0
    for p, k, fill in zip(pos, kinds, fills):
        p = max(int(p), cur)
        parts.append(a[cur:p])
        if k == 0:    # overwrite
            parts.append(fill)
            cur = min(p + span, len(a))
        elif k == 1:  # insert
            parts.append(fill)
            cur = p
        else:         # delete
            cur = min(p + span, len(a))
    parts.append(a[cur:])
    return np.concatenate(parts)
