"""Probe: does `import torch` (no CUDA init) coexist with libbsgpu in one process?"""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa
import torch.distributed  # noqa
import __graft_entry__ as g
g.smoke()
print("torch imported first: ok")
