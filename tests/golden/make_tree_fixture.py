#!/usr/bin/env python3
"""Generates tests/golden/tree_root_variants.json: streams on which the one recalled detail of
hashsplit v1.1.1's TreeBuilder.Root decides Writer.Root.

The detail: when Root() is called, are the levels below the top folded into their parents
  "nonempty"   — every non-empty level, always (this library, oracle/bsoracle.c), or
  "leaf_gated" — only when the leaf level holds chunks, i.e. not when the last chunk itself
                 closed a level (nodes waiting in the levels between would then not be under
                 the Root)?
The two give different Roots exactly when the stream's last chunk has level/fanout = L >= 1
while the tree is already taller than L + 1 (an earlier chunk had a larger level): after the
last Add, level L holds the node just closed and sits below the top.

Each case is a SplitMix64 stream (bs_amd/synth.py: 8-byte little-endian word i is
splitmix64(seed + (i + 1) * 0x9E3779B97F4A7C15)), truncated right after such a chunk, with the
Root under both variants (computed by the C oracle and, independently, by the pure-Python tree
restatement over the C oracle's chunks). One Go run of split.NewWriter(ctx, mem.New(),
Bits(b), MinSize(m), Fanout(f)) over these bytes — or `bs put -split -bits 4` for the fanout-8,
MinSize-1024 case — tells which variant hashsplit implements. Control cases (both variants
equal) are included. This script is test infrastructure: the oracle is only the checker.

  python tests/golden/make_tree_fixture.py
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "tests", "golden", "tree_root_variants.json")


def tree_heights(levels, fanout):
    """After each Add: (L of that chunk, number of tree levels)."""
    nlv, out = 0, []
    for lv in levels:
        L = int(lv) // fanout
        nlv = max(nlv, 1, L + 1)
        out.append((L, nlv))
    return out


def find_cut(ch, fanout, want_differ: bool, min_chunks: int):
    """Index of the chunk to end the stream with: L >= 1 and a taller tree (differ), or L >= 1
    with the tree exactly L + 1 high (control: the folds agree)."""
    hs = tree_heights(ch["level"], fanout)
    for k in range(min_chunks, len(ch)):
        L, nlv = hs[k]
        if L < 1:
            continue
        if want_differ and nlv > L + 1:
            return k
        if not want_differ and nlv == L + 1:
            return k
    return None


def main() -> None:
    from oracle import oracle as O
    from bs_amd.synth import splitmix_array
    table = O.buzhash32_table(1)
    specs = [  # (name, bits, min_size, fanout, stream bytes to search, differ?)
        ("bits4_min64_fanout2_differ", 4, 64, 2, 1 << 20, True),
        ("bits4_min64_fanout2_control", 4, 64, 2, 1 << 20, False),
        ("bits6_min64_fanout3_differ", 6, 64, 3, 4 << 20, True),
        ("bits4_min1024_fanout8_cli_differ", 4, 1024, 8, 160 << 20, True),
        ("bits4_min1024_fanout8_cli_control", 4, 1024, 8, 160 << 20, False),
    ]
    cases = []
    for name, bits, ms, fo, n, differ in specs:
        for seed in range(1, 200):
            data = splitmix_array(seed, n)
            ch = O.split(table, data, bits=bits, min_size=ms)
            k = find_cut(ch, fo, differ, min_chunks=8)
            if k is None:
                continue
            end = int(ch["offset"][k] + ch["len"][k])
            cut = data[:end]
            roots = {}
            for fold in ("nonempty", "leaf_gated"):
                r_c, _ = O.writer_root(table, cut, bits=bits, min_size=ms, fanout=fo, fold=fold)
                cc = ch[: k + 1]
                r_py = O.py_tree_root([(cut[int(c["offset"]):int(c["offset"] + c["len"])],
                                        int(c["level"])) for c in cc], fo, fold=fold)
                assert r_c == r_py, (name, fold)
                roots[fold] = r_c.hex()
            assert (roots["nonempty"] != roots["leaf_gated"]) == differ, name
            L, nlv = tree_heights(ch["level"][: k + 1], fo)[-1]
            cases.append({"name": name, "generator": "splitmix64", "seed": seed, "length": end,
                          "bits": bits, "min_size": ms, "fanout": fo, "chunks": k + 1,
                          "last_chunk_level": int(ch["level"][k]), "last_chunk_L": L,
                          "tree_levels": nlv,
                          "root_nonempty": roots["nonempty"],
                          "root_leaf_gated": roots["leaf_gated"],
                          "variants_differ": differ})
            print(f"{name}: seed {seed}, {end} bytes, {k + 1} chunks, L {L}, "
                  f"{nlv} levels", file=sys.stderr)
            break
        else:
            raise SystemExit(f"no stream found for {name}")
    doc = {"about": __doc__.split("\n\n")[0] + " (see make_tree_fixture.py)",
           "library_variant": "nonempty",
           "cases": cases}
    with open(OUT, "w") as f:
        json.dump(doc, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main()
