"""Shared test setup: import paths and the `gpu` marker.

`-m "not gpu"` tests run here (no GPU): the oracle against the reference's
golden vectors, host logic, and that the C-ABI library loads/exports.
`-m gpu` tests run on an MI355X and call the HIP path through the C-ABI.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "ffmpeg-ffv1-p-frames_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

# torch first: the tests that stage frames in HBM use torch, whose bundled
# HIP runtime must be the process's one before libffv1hip.so loads (loaded
# the other way round, torch finds no GPU)
try:
    import torch  # noqa: F401
except ImportError:
    pass


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    config.addinivalue_line("markers", "slow: long-running CPU oracle test")
