"""The debug build's device bounds checks (build.py --check,
lib/libffv1hip_check.so, ffv1_internal.h Bounds).

The walk's recorded states, the carried states and the coder's digits and
bytes are written only inside the extents the layout gave them: a walk
chain its own chain and pad, a coder stream its slice slot.  The debug build
checks every such write and an encode whose batch wrote outside fails with
-EFAULT naming the kernel.  CPU: the library is built and says it is the
debug build.  GPU (a child process, since the library is chosen at load):
the checked build encodes bit-exactly and reports nothing, and with the
bounds_shrink hook (a decision buffer declared smaller than it is) the
checks fire.
"""
import ctypes
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "ffmpeg-ffv1-p-frames_amd", "lib")
CHECK_LIB = os.path.join(LIB, "libffv1hip_check.so")

CHILD = r"""
import os, sys
sys.path[:0] = [{root!r}, os.path.join({root!r}, "ffmpeg-ffv1-p-frames_amd"), os.path.join({root!r}, "tests")]
from ffv1hip import HipEncoder, load_library
from ffv1hip.encoder import FFV1Error
from oracle import oracle
from helpers import Stream
assert load_library().ffv1hip_debug_checks() == 1
from test_gpu_parity import hip_params
for s in [Stream("c420", 352, 288, "yuv420p10", 6, slices=4, level=3, coder=1, gop_size=3, source="random"),
          Stream("c444", 176, 144, "yuv444p", 5, slices=6, level=3, coder=1, gop_size=5, chroma444=True)]:
    frames = list(s.frames())
    try:
        enc = HipEncoder(hip_params(s), 0, len(frames))
        got = enc.encode(frames)
    except FFV1Error as e:
        print("FAULT", s.name, e)
        sys.exit(3)
    ref = oracle.Encoder(s.oracle_config())
    for i, f in enumerate(frames):
        assert got[i] == ref.encode(f), (s.name, i)
    enc.close()
print("CLEAN")
"""


def _run_child(debug):
    env = dict(os.environ, FFV1HIP_LIB=CHECK_LIB, FFV1HIP_DEBUG=debug)
    return subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT)], env=env, capture_output=True,
                          text=True, timeout=240)


def test_check_library_is_the_debug_build():
    if not os.path.exists(CHECK_LIB):
        pytest.skip("lib/libffv1hip_check.so not built (build.py --no-check)")
    chk = ctypes.CDLL(CHECK_LIB)
    assert chk.ffv1hip_debug_checks() == 1
    from ffv1hip import load_library
    assert load_library().ffv1hip_debug_checks() == 0


@pytest.mark.gpu
def test_checked_build_is_bit_exact_and_clean():
    r = _run_child("")
    assert r.returncode == 0 and "CLEAN" in r.stdout, r.stdout + r.stderr


@pytest.mark.gpu
def test_checked_build_reports_writes_outside_their_extent():
    r = _run_child("bounds_shrink=40")  # the decision buffer declared empty: every chain's writes fail
    assert r.returncode == 3, r.stdout + r.stderr
    assert "device bounds check" in r.stdout and "ffv1_walk" in r.stdout, r.stdout
