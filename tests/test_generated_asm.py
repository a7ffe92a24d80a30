"""The generated inline-asm loops in bs_amd/csrc/*.inc are reproduced by their generators in
tools/ (so a reader can trust the generators' docstrings for what the kernels run): the k_scan
fast pass (gen_scan_loop.py), the octet / pair SHA-256 chains (gen_skew_asm.py) and the per-lane
compression (gen_lane_asm.py). CPU only; gen_scan_loop.py sizes instructions with llvm-mc."""
import contextlib
import importlib.util
import io
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "bs_amd", "csrc")
MC = "/opt/rocm/lib/llvm/bin/llvm-mc"


def load(name):
    spec = importlib.util.spec_from_file_location(name, os.path.join(ROOT, "tools", f"{name}.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def same(tmp_path, name):
    with open(tmp_path / name, "rb") as a, open(os.path.join(CSRC, name), "rb") as b:
        return a.read() == b.read()


@pytest.mark.skipif(not os.path.exists(MC), reason="llvm-mc (ROCm) not installed")
def test_scan_loop_matches_generator(tmp_path):
    g = load("gen_scan_loop")
    g.OUT = str(tmp_path / "scan_block_loop.inc")
    with contextlib.redirect_stdout(io.StringIO()):
        g.main()
    assert same(tmp_path, "scan_block_loop.inc")


def test_chain_loops_match_generator(tmp_path):
    g = load("gen_skew_asm")
    with contextlib.redirect_stdout(io.StringIO()):
        g.main_loop_oct_solo(out_path=str(tmp_path / "sha256_oct_solo_loop.inc"))
        g.main_loop_oct(out_path=str(tmp_path / "sha256_oct_loop.inc"))
        g.main_loop(out_path=str(tmp_path / "sha256_skew_loop.inc"))
        g.main(out_path=str(tmp_path / "sha256_skew_block.inc"))
    for name in ("sha256_oct_solo_loop.inc", "sha256_oct_loop.inc", "sha256_skew_loop.inc",
                 "sha256_skew_block.inc"):
        assert same(tmp_path, name), name


def test_lane_compression_matches_generator(tmp_path):
    g = load("gen_lane_asm")
    g.OUT = str(tmp_path / "sha256_lane_asm.inc")
    g.ROOT = str(tmp_path)  # its ubench variants file goes under tmp_path too
    os.makedirs(tmp_path / "tools" / "ubench", exist_ok=True)
    with contextlib.redirect_stdout(io.StringIO()):
        g.gen()
    assert same(tmp_path, "sha256_lane_asm.inc")
